#!/bin/bash
# round 6: kernel trace of config 5's single-GPU step (train_step + train.Adam, bf16, dims [128,256,256,256])
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06_c5_tr -o run -- python3 tools/train_probe.py 30 --fused --our-adam --bf16 --dims=128,256,256,256 > gpurun_out/r06_c5_tr.txt 2>&1 || { tail -20 gpurun_out/r06_c5_tr.txt; exit 1; }
grep "train step" gpurun_out/r06_c5_tr.txt
python3 tools/r05_gaps.py gpurun_out/r06_c5_tr/run_kernel_trace.csv 20 adam_kernel > gpurun_out/r06_c5_timeline.txt 2>&1 || true
head -70 gpurun_out/r06_c5_timeline.txt
