#!/bin/bash
# Round-4 GPU check 9: MiddleTrainer HIP-graph capture (test + per-rank probe), the dense default flip (IL), the full
# -m gpu suite, then a default bench line.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread \
  "tests/test_gpu_middle_train.py::test_middle_trainer_hip_graph_matches_eager" \
  "tests/test_gpu_parity.py::test_dense_dma_interleave_bitexact" > gpurun_out/r04_t9.log 2>&1 || { tail -40 gpurun_out/r04_t9.log; exit 1; }
grep -cE "PASSED" gpurun_out/r04_t9.log
timeout -k 10 300 python -u tools/middle_train_probe.py > gpurun_out/r04_mtp3.json 2> gpurun_out/r04_mtp3.err || { tail -30 gpurun_out/r04_mtp3.err; exit 1; }
cat gpurun_out/r04_mtp3.json
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_gpu_suite.log 2>&1 || { tail -60 gpurun_out/r04_gpu_suite.log; exit 1; }
tail -3 gpurun_out/r04_gpu_suite.log
timeout -k 10 300 python -u bench.py > gpurun_out/r04_bench9.json 2> gpurun_out/r04_bench9.err || { tail -30 gpurun_out/r04_bench9.err; exit 1; }
cat gpurun_out/r04_bench9.json
