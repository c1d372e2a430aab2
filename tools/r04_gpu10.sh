#!/bin/bash
# Round-4 GPU check 10: the off-diagonal transposed middle-tile kernel (parity vs CSR, accumulate, determinism),
# then its timing against the 4x4-block and CSR transposed kernels at B(20,4), F = 128 and 256.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  "tests/test_gpu_ngram.py::test_ngram_spmm3t_vs_csr" > gpurun_out/r04_t10.log 2>&1 || { tail -40 gpurun_out/r04_t10.log; exit 1; }
grep -cE "PASSED" gpurun_out/r04_t10.log
timeout -k 10 200 python -u tools/ngram_probe_k.py 4 128 20 > gpurun_out/r04_probe_t128.txt 2>&1 || { tail -20 gpurun_out/r04_probe_t128.txt; exit 1; }
cat gpurun_out/r04_probe_t128.txt | grep -v amdgpu.ids
timeout -k 10 200 python -u tools/ngram_probe_k.py 4 256 10 > gpurun_out/r04_probe_t256.txt 2>&1 || { tail -20 gpurun_out/r04_probe_t256.txt; exit 1; }
cat gpurun_out/r04_probe_t256.txt | grep -v amdgpu.ids
timeout -k 10 300 python -u tools/map_probe.py > gpurun_out/r04_mapprobe2.json 2> gpurun_out/r04_mapprobe2.err || { tail -20 gpurun_out/r04_mapprobe2.err; exit 1; }
cat gpurun_out/r04_mapprobe2.json
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_builder_graph.py "tests/test_gpu_ngram.py" > gpurun_out/r04_t10b.log 2>&1 || { tail -40 gpurun_out/r04_t10b.log; exit 1; }
tail -2 gpurun_out/r04_t10b.log
