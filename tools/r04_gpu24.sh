#!/bin/bash
# Round-4 GPU check 24: host call sites of the config-5 rank step's GPU time (glue copies / fills / casts).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/middle_train_attr.py > gpurun_out/r04_attr.txt 2> gpurun_out/r04_attr.err || { tail -30 gpurun_out/r04_attr.err; exit 1; }
head -50 gpurun_out/r04_attr.txt | cut -c1-300
