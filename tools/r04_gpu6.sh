#!/bin/bash
# Round-4 GPU check 6: dense kernel stamps (pointer hoisted), direct-epilogue variant bit-exactness + A/B timing.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread \
  "tests/test_gpu_parity.py::test_dense_dma_interleave_bitexact" > gpurun_out/r04_t6.log 2>&1 || { tail -40 gpurun_out/r04_t6.log; exit 1; }
tail -2 gpurun_out/r04_t6.log
timeout -k 10 200 python -u tools/dense_exp.py --stamps --il > gpurun_out/r04_dense_stamps_il.txt 2>&1 || { tail -20 gpurun_out/r04_dense_stamps_il.txt; exit 1; }
grep stamps gpurun_out/r04_dense_stamps_il.txt
timeout -k 10 300 python -u tools/dense_ab.py 4 20 20 > gpurun_out/r04_dense_ab.json 2> gpurun_out/r04_dense_ab.err || { tail -20 gpurun_out/r04_dense_ab.err; exit 1; }
cat gpurun_out/r04_dense_ab.json
