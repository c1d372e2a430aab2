#!/bin/bash
# round 6: MiddleTrainer with the fused bf16 head -- its GPU tests and the per-rank step (RCCL at world 1)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/middle_train_probe.py --comm rccl > gpurun_out/r06_mtp_rccl.json 2> gpurun_out/r06_mtp_rccl.err || { tail -20 gpurun_out/r06_mtp_rccl.err; exit 1; }
cat gpurun_out/r06_mtp_rccl.json | cut -c1-1500
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread tests/test_gpu_middle_train.py tests/test_gpu_rccl.py > gpurun_out/r06_t7.log 2>&1
rc=$?
grep -E "^E |passed|failed|PASS|FAIL" gpurun_out/r06_t7.log | cut -c1-300 | head -30
exit $rc
