#!/bin/bash
# Round-4 GPU check 7: the IL dense variant (bit-exactness, stamps, A/B), then the whole -m gpu suite.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/r04_gpu6.sh || exit 1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_gpu_suite.log 2>&1 || { tail -60 gpurun_out/r04_gpu_suite.log; exit 1; }
tail -3 gpurun_out/r04_gpu_suite.log
