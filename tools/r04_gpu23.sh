#!/bin/bash
# Round-4 GPU check 21: 16K-element chunks of the multi-tensor kernels (Adam, L2 sums) (P = 8 tests, HIP-graph test), the
# per-rank probe and a kernel trace of rank 0 (breakdown of the graph-mode steps).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_middle_train.py -k "train or adam or l2 or sqsum or hip_graph" > gpurun_out/r04_t27.log 2>&1 || { grep -E "PASSED|FAILED|Error|error" gpurun_out/r04_t27.log | tail -30; exit 1; }
grep -E "PASSED|passed" gpurun_out/r04_t27.log
timeout -k 10 300 python -u tools/middle_train_probe.py > gpurun_out/r04_mtp22.json 2> gpurun_out/r04_mtp22.err || { tail -30 gpurun_out/r04_mtp22.err; exit 1; }
cat gpurun_out/r04_mtp22.json
rm -rf gpurun_out/prof_mtp22
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_mtp22 -o k --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/middle_train_probe.py --ranks 0 --reps 10 > $GRAFT_REPO_ROOT/gpurun_out/r04_mtp22b.json 2> $GRAFT_REPO_ROOT/gpurun_out/r04_mtp22b.err || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/r04_mtp22b.err; exit 1; }
cd $GRAFT_REPO_ROOT && find gpurun_out/prof_mtp22 -name "*kernel_trace.csv" -exec cp {} gpurun_out/r04_mtp22_kernel_trace.csv \;
rm -rf gpurun_out/prof_mtp22
python tools/trace_breakdown.py gpurun_out/r04_mtp22_kernel_trace.csv 10 40 2 > gpurun_out/r04_mtp22_breakdown.txt
head -12 gpurun_out/r04_mtp22_breakdown.txt | cut -c1-150
