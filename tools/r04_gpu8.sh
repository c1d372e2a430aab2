#!/bin/bash
# Round-4 GPU check 8: MiddleTrainer HIP-graph capture (test + probe).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread \
  "tests/test_gpu_middle_train.py::test_middle_trainer_hip_graph_matches_eager" > gpurun_out/r04_t8.log 2>&1 || { tail -40 gpurun_out/r04_t8.log; exit 1; }
grep -E "PASSED|FAILED" gpurun_out/r04_t8.log
timeout -k 10 300 python -u tools/middle_train_probe.py > gpurun_out/r04_mtp3.json 2> gpurun_out/r04_mtp3.err || { tail -30 gpurun_out/r04_mtp3.err; exit 1; }
cat gpurun_out/r04_mtp3.json
