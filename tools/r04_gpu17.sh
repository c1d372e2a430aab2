#!/bin/bash
# Round-4 GPU check 17: the scatter backward (kernel tests, P = 8 trainer tests), its timing (probe, phase skips),
# the per-rank middle-trainer step and a kernel trace of rank 0.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_mid_scatter.py > gpurun_out/r04_t20.log 2>&1 || { tail -40 gpurun_out/r04_t20.log; exit 1; }
tail -1 gpurun_out/r04_t20.log
timeout -k 10 300 python -u tools/scatter_probe.py > gpurun_out/r04_sp5.json 2> gpurun_out/r04_sp5.err || { tail -5 gpurun_out/r04_sp5.err; exit 1; }
cat gpurun_out/r04_sp5.json
timeout -k 10 300 python -u tools/scatter_probe.py --fp32 --cpw 0 > gpurun_out/r04_sp5f.json 2>> gpurun_out/r04_sp5.err || exit 1
cat gpurun_out/r04_sp5f.json
timeout -k 10 200 python -u tools/scatter_exp.py > gpurun_out/r04_sexp3.json 2> gpurun_out/r04_sexp3.err || { tail -8 gpurun_out/r04_sexp3.err; exit 1; }
cat gpurun_out/r04_sexp3.json
timeout -k 10 900 python -u -m pytest -x -v --timeout 850 --timeout-method thread tests/test_gpu_middle_train.py > gpurun_out/r04_t20b.log 2>&1 || { tail -60 gpurun_out/r04_t20b.log; exit 1; }
grep -E "passed|failed" gpurun_out/r04_t20b.log
timeout -k 10 300 python -u tools/middle_train_probe.py > gpurun_out/r04_mtp17.json 2> gpurun_out/r04_mtp17.err || { tail -30 gpurun_out/r04_mtp17.err; exit 1; }
cat gpurun_out/r04_mtp17.json
rm -rf gpurun_out/prof_mtp17
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_mtp17 -o k --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/middle_train_probe.py --ranks 0 --reps 10 > $GRAFT_REPO_ROOT/gpurun_out/r04_mtp17b.json 2> $GRAFT_REPO_ROOT/gpurun_out/r04_mtp17b.err || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/r04_mtp17b.err; exit 1; }
cd $GRAFT_REPO_ROOT && find gpurun_out/prof_mtp17 -name "*kernel_stats.csv" -exec cp {} gpurun_out/r04_mtp17_kernel_stats.csv \; && find gpurun_out/prof_mtp17 -name "*kernel_trace.csv" -exec cp {} gpurun_out/r04_mtp17_kernel_trace.csv \;
rm -rf gpurun_out/prof_mtp17
