set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "fused_dropout or dense_backward or graphed or train_step or head_train or span" > gpurun_out/fd_tests.log 2>&1 || { tail -40 gpurun_out/fd_tests.log; exit 1; }
tail -3 gpurun_out/fd_tests.log
for a in "--fused --our-adam" "--fused --our-adam --no-fdrop" "--fused --our-adam --bf16 --dims=128,256,256,256" "--fused --our-adam --bf16 --dims=128,256,256,256 --no-fdrop"; do
  timeout -k 10 200 python -u tools/train_probe.py 20 $a >> gpurun_out/fd_train.txt 2>&1 || { tail -20 gpurun_out/fd_train.txt; exit 1; }
done
grep "train step" gpurun_out/fd_train.txt
