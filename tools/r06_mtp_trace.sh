#!/bin/bash
# round 6: kernel trace of config 5's rank step (MiddleTrainer, P = 8, rank 0, no-op collectives, replayed graphs)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/r06_mtp_tr
timeout -s KILL 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06_mtp_tr -o run -- python3 tools/middle_train_probe.py --ranks 0 --reps 20 > gpurun_out/r06_mtp_tr.json 2> gpurun_out/r06_mtp_tr.err || { tail -20 gpurun_out/r06_mtp_tr.err; exit 1; }
cut -c1-600 gpurun_out/r06_mtp_tr.json
f=$(find gpurun_out/r06_mtp_tr -name "*kernel_trace.csv" | head -1)
cp $f gpurun_out/r06_mtp_kernel_trace.csv
rm -rf gpurun_out/r06_mtp_tr
