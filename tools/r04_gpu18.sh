#!/bin/bash
# Round-4 GPU check 18: the per-rank middle-trainer step with the scatter backward (probe) and a kernel trace of rank 0.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/middle_train_probe.py > gpurun_out/r04_mtp18.json 2> gpurun_out/r04_mtp18.err || { tail -30 gpurun_out/r04_mtp18.err; exit 1; }
cat gpurun_out/r04_mtp18.json
rm -rf gpurun_out/prof_mtp18
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_mtp18 -o k --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/middle_train_probe.py --ranks 0 --reps 10 > $GRAFT_REPO_ROOT/gpurun_out/r04_mtp18b.json 2> $GRAFT_REPO_ROOT/gpurun_out/r04_mtp18b.err || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/r04_mtp18b.err; exit 1; }
cd $GRAFT_REPO_ROOT && find gpurun_out/prof_mtp18 -name "*kernel_stats.csv" -exec cp {} gpurun_out/r04_mtp18_kernel_stats.csv \; && find gpurun_out/prof_mtp18 -name "*kernel_trace.csv" -exec cp {} gpurun_out/r04_mtp18_kernel_trace.csv \;
rm -rf gpurun_out/prof_mtp18
ls -la gpurun_out/r04_mtp18_kernel_trace.csv
