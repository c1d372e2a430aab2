#!/bin/bash
# Round-4 GPU check 13: the bf16 transposed middle-tile kernel (diagonal in-kernel): parity, then timing vs the 4x4
# bf16 kernel at F = 128 / 256, then the bf16 training step (config 5 single GPU) and the n-gram / builder GPU tests.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  "tests/test_gpu_ngram.py::test_ngram_transposed_bf16" > gpurun_out/r04_t13.log 2>&1 || { tail -40 gpurun_out/r04_t13.log; exit 1; }
grep -cE "PASSED" gpurun_out/r04_t13.log
timeout -k 10 200 python -u tools/ngram_probe_k.py 4 128 20 > gpurun_out/r04_probe13_f128.txt 2>&1 || { tail -20 gpurun_out/r04_probe13_f128.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r04_probe13_f128.txt | tail -3
timeout -k 10 200 python -u tools/ngram_probe_k.py 4 256 10 > gpurun_out/r04_probe13_f256.txt 2>&1 || { tail -20 gpurun_out/r04_probe13_f256.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r04_probe13_f256.txt | tail -3
timeout -k 10 300 python -u tools/train_probe.py 20 --fused --our-adam --bf16 --dims=128,256,256,256 > gpurun_out/r04_train_c5.txt 2>&1 || { tail -20 gpurun_out/r04_train_c5.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r04_train_c5.txt | tail -2
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ngram.py tests/test_gpu_configs.py > gpurun_out/r04_t13b.log 2>&1 || { tail -40 gpurun_out/r04_t13b.log; exit 1; }
tail -2 gpurun_out/r04_t13b.log
