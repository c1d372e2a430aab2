#!/bin/bash
# Round-4 GPU check 25: LayerDense backward hands autograd contiguous, unshared weight/bias gradients (no AccumulateGrad
# copies), MiddleTrainer caches the bf16 input and skips the unused embeddings: the training tests, the attribution
# and the per-rank probe.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_middle_train.py tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_rccl.py tests/test_gpu_shard.py -k "train or backward or dense or hip_graph or rccl or grad" > gpurun_out/r04_t28.log 2>&1 || { grep -E "PASSED|FAILED|Error|error" gpurun_out/r04_t28.log | tail -30; exit 1; }
grep -cE "PASSED" gpurun_out/r04_t28.log; tail -1 gpurun_out/r04_t28.log
timeout -k 10 400 python -u tools/middle_train_attr.py > gpurun_out/r04_attr2.txt 2> gpurun_out/r04_attr2.err || { tail -30 gpurun_out/r04_attr2.err; exit 1; }
head -30 gpurun_out/r04_attr2.txt | cut -c1-250
timeout -k 10 300 python -u tools/middle_train_probe.py > gpurun_out/r04_mtp25.json 2> gpurun_out/r04_mtp25.err || { tail -30 gpurun_out/r04_mtp25.err; exit 1; }
cat gpurun_out/r04_mtp25.json
