#!/bin/bash
# Round-4 GPU check 22: the P = 8 middle-trainer tests three times (an intermittent stall of the bf16 case: the
# workers dump their stacks after 150 s and exit), then the multi-tensor chunk-size change's tests.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2 3; do
  timeout -k 10 420 python -u -m pytest -x -v -s --timeout 400 --timeout-method thread tests/test_gpu_middle_train.py -k p8 > gpurun_out/r04_t26_$i.log 2>&1
  rc=$?
  echo "run $i rc=$rc"; grep -E "PASSED|FAILED|passed|failed" gpurun_out/r04_t26_$i.log | tail -3
  if [ $rc -ne 0 ]; then grep -B2 -A30 "Thread 0x\|Current thread\|Timeout (0" gpurun_out/r04_t26_$i.log | head -120; exit 1; fi
done
