#!/bin/bash
# Round-4 GPU check 14: the fused-split dense variant: bit-exactness, then the A/B against the default.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  "tests/test_gpu_parity.py::test_dense_dma_interleave_bitexact" > gpurun_out/r04_t14.log 2>&1 || { tail -40 gpurun_out/r04_t14.log; exit 1; }
grep -cE "PASSED" gpurun_out/r04_t14.log
timeout -k 10 300 python -u tools/dense_ab.py 4 20 20 > gpurun_out/r04_dense_ab2.json 2> gpurun_out/r04_dense_ab2.err || { tail -20 gpurun_out/r04_dense_ab2.err; exit 1; }
cat gpurun_out/r04_dense_ab2.json
