#!/bin/bash
# Round-4 GPU check 1: bf16 determinism probe, the bench contract, the shard tests, then the default bench line.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/r04_bf16det.py > gpurun_out/r04_det.log 2>&1; echo "det rc=$?"; grep -v amdgpu.ids gpurun_out/r04_det.log | tail -30
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread \
  tests/test_gpu_bench.py tests/test_gpu_shard.py \
  "tests/test_gpu_parity.py::test_rows_gather_scatter" > gpurun_out/r04_t1.log 2>&1 || { tail -40 gpurun_out/r04_t1.log; exit 1; }
tail -5 gpurun_out/r04_t1.log
timeout -k 10 300 python -u bench.py > gpurun_out/r04_b1.json 2> gpurun_out/r04_b1.err || { tail -30 gpurun_out/r04_b1.err; exit 1; }
cat gpurun_out/r04_b1.json
tail -5 gpurun_out/r04_b1.err
