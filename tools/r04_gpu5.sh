#!/bin/bash
# Round-4 GPU check 5: the dense kernel's per-iteration stamps and phase-skip table (diagnostics build).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/dense_exp.py --stamps > gpurun_out/r04_dense_stamps.txt 2>&1 || { tail -20 gpurun_out/r04_dense_stamps.txt; exit 1; }
grep stamps gpurun_out/r04_dense_stamps.txt
timeout -k 10 300 python -u tools/dense_exp.py 4 20 > gpurun_out/r04_dense_exp.txt 2>&1 || { tail -20 gpurun_out/r04_dense_exp.txt; exit 1; }
tail -3 gpurun_out/r04_dense_exp.txt
