#!/bin/bash
# round 6: config-5 single-GPU step with / without the bf16 PropagateDense backward, plus the bf16 tests
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/train_probe.py 20 --fused --our-adam --bf16 --dims=128,256,256,256 2>&1 | grep -v amdgpu.ids > gpurun_out/r06_c5.txt || exit 1
timeout -k 10 300 python -u tools/train_probe.py 20 --fused --our-adam --bf16 --dims=128,256,256,256 --no-span 2>&1 | grep -v amdgpu.ids >> gpurun_out/r06_c5.txt || exit 1
cat gpurun_out/r06_c5.txt
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread tests/test_gpu_parity.py -k "propagate_dense or bf16" > gpurun_out/r06_t4.log 2>&1
rc=$?
grep -E "^E |passed|failed" gpurun_out/r06_t4.log | cut -c1-300 | head -20
exit $rc
