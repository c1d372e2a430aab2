#!/bin/bash
# Round-5 GPU check 2: RCCL test (MiddleTrainer over TorchComm, eager + captured), bf16 determinism bisection probe,
# the P = 8 middle-trainer tests with per-rank phase timings.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 280 --timeout-method thread tests/test_gpu_rccl.py > gpurun_out/r05_rccl.log 2>&1; echo "rccl rc=$?"; grep -E "PASSED|FAILED|Error" gpurun_out/r05_rccl.log | tail -5
timeout -k 10 300 python -u tools/r05_bf16det.py 5 > gpurun_out/r05_bf16det.json 2> gpurun_out/r05_bf16det.err || { echo "probe rc=$?"; tail -20 gpurun_out/r05_bf16det.err; exit 1; }
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 880 --timeout-method thread tests/test_gpu_middle_train.py -k p8 --durations=0 > gpurun_out/r05_p8.log 2>&1; echo "p8 rc=$?"; grep -E "PASSED|FAILED|passed|failed" gpurun_out/r05_p8.log | tail -4
