#!/bin/bash
# Round-5 GPU check 8: bf16 dense backward determinism (new test + whole-step probe), RCCL test (bitwise bf16 again),
# then the P = 8 middle-trainer tests with per-rank phase timings (progress streamed to gpurun_out/).
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_rccl.py > gpurun_out/r05_det.log 2>&1; rc=$?; tail -4 gpurun_out/r05_det.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/r05_bf16det.py 5 > gpurun_out/r05_bf16det2.json 2> gpurun_out/r05_bf16det2.err || exit 1
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 880 --timeout-method thread tests/test_gpu_middle_train.py -k p8 --durations=0 > gpurun_out/r05_p8.log 2>&1; echo "p8 rc=$?"; grep -E "PASSED|FAILED|passed|failed" gpurun_out/r05_p8.log | tail -4
