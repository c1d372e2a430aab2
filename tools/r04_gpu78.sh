#!/bin/bash
set -o pipefail
bash tools/r04_gpu6.sh && bash tools/r04_gpu8.sh && bash -c 'timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_gpu_suite.log 2>&1 || { tail -60 gpurun_out/r04_gpu_suite.log; exit 1; }; tail -3 gpurun_out/r04_gpu_suite.log'
