#!/bin/bash
# round 6: the bf16 F = 256 head-train kernel: parity tests, head timing, config-5 step
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "head_train" > gpurun_out/r06_t5.log 2>&1
rc=$?
grep -E "^E |passed|failed|head_train_bf16 M" gpurun_out/r06_t5.log | cut -c1-300 | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/r06_head5_probe.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r06_head5_probe.json || exit 1
timeout -k 10 300 python -u tools/train_probe.py 20 --fused --our-adam --bf16 --dims=128,256,256,256 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r06_c5b.txt || exit 1
