#!/bin/bash
# Round-5 GPU check 3: RCCL test with teardown diagnostics, then the bf16 determinism probe (progress on stderr).
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 280 --timeout-method thread tests/test_gpu_rccl.py 2>&1 | tee gpurun_out/r05_rccl2.log | grep -E "PASSED|FAILED|Error|Thread|File"
timeout -k 10 400 python -u tools/r05_bf16det.py 5 > gpurun_out/r05_bf16det.json 2> >(tee gpurun_out/r05_bf16det.err >&2)
echo "probe rc=$?"
