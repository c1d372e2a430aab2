#!/bin/bash
# Round-4 GPU check 15: the scatter-form middle-partition backward (kernel tests, the P = 8 config-5 trainer test,
# the HIP-graph test), the per-rank probe, and a kernel trace of rank 0.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_mid_scatter.py > gpurun_out/r04_t15a.log 2>&1 || { tail -60 gpurun_out/r04_t15a.log; exit 1; }
tail -2 gpurun_out/r04_t15a.log
timeout -k 10 900 python -u -m pytest -x -v --timeout 850 --timeout-method thread tests/test_gpu_middle_train.py > gpurun_out/r04_t15b.log 2>&1 || { tail -60 gpurun_out/r04_t15b.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" gpurun_out/r04_t15b.log
timeout -k 10 300 python -u tools/middle_train_probe.py > gpurun_out/r04_mtp15.json 2> gpurun_out/r04_mtp15.err || { tail -30 gpurun_out/r04_mtp15.err; exit 1; }
cat gpurun_out/r04_mtp15.json
rm -rf gpurun_out/prof_mtp15
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_mtp15 -o k --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/middle_train_probe.py --ranks 0 --reps 10 > $GRAFT_REPO_ROOT/gpurun_out/r04_mtp15b.json 2> $GRAFT_REPO_ROOT/gpurun_out/r04_mtp15b.err || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/r04_mtp15b.err; exit 1; }
cd $GRAFT_REPO_ROOT && find gpurun_out/prof_mtp15 -name "*kernel_stats.csv" -exec cp {} gpurun_out/r04_mtp15_kernel_stats.csv \; && find gpurun_out/prof_mtp15 -name "*kernel_trace.csv" -exec cp {} gpurun_out/r04_mtp15_kernel_trace.csv \;
rm -rf gpurun_out/prof_mtp15
head -25 gpurun_out/r04_mtp15_kernel_stats.csv | cut -c1-160
