#!/bin/bash
# Round-4 GPU check 11: HBM traffic and kernel stats of the transposed kernels (rocprofv3), the config-3 training
# step, the MiddleTrainer HIP-graph capture (test + per-rank probe), then the full -m gpu suite and a bench line.
set -o pipefail
mkdir -p gpurun_out/tpmc
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --pmc $c --kernel-trace -d gpurun_out/tpmc/$c -o k -- python3 tools/tprobe.py 10 > gpurun_out/tpmc/$c.log 2>&1 || { tail -20 gpurun_out/tpmc/$c.log; exit 1; }
done
python tools/pmc_traffic.py gpurun_out/tpmc/FETCH_SIZE gpurun_out/tpmc/WRITE_SIZE gpurun_out/r04_transposed_traffic.json transposed_B20_4_F128 || exit 1
timeout -s KILL 150 rocprofv3 --kernel-trace --stats -d gpurun_out/tstats -o k -- python3 tools/tprobe.py 20 > gpurun_out/tstats.log 2>&1 || { tail -20 gpurun_out/tstats.log; exit 1; }
find gpurun_out/tstats -name "*kernel_stats.csv" -exec cp {} gpurun_out/r04_transposed_kernel_stats.csv \;
timeout -k 10 300 python -u tools/train_probe.py 20 --fused --our-adam > gpurun_out/r04_train_c3.txt 2>&1 || { tail -20 gpurun_out/r04_train_c3.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r04_train_c3.txt | tail -3
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread \
  "tests/test_gpu_middle_train.py::test_middle_trainer_hip_graph_matches_eager" > gpurun_out/r04_t11.log 2>&1 || { tail -40 gpurun_out/r04_t11.log; exit 1; }
grep -cE "PASSED" gpurun_out/r04_t11.log
timeout -k 10 300 python -u tools/middle_train_probe.py > gpurun_out/r04_mtp3.json 2> gpurun_out/r04_mtp3.err || { tail -30 gpurun_out/r04_mtp3.err; exit 1; }
cat gpurun_out/r04_mtp3.json
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_gpu_suite.log 2>&1 || { tail -60 gpurun_out/r04_gpu_suite.log; exit 1; }
tail -3 gpurun_out/r04_gpu_suite.log
