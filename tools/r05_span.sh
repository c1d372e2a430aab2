set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "span or fused_dropout or propagate_dense or model_fused" > gpurun_out/span_tests.log 2>&1 || { tail -40 gpurun_out/span_tests.log; exit 1; }
tail -2 gpurun_out/span_tests.log
timeout -k 10 200 python -u tools/train_probe.py 20 --fused --our-adam > gpurun_out/span_train.txt 2>&1 || { tail -20 gpurun_out/span_train.txt; exit 1; }
grep "train step" gpurun_out/span_train.txt
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/span_tr -o run -- python3 tools/train_probe.py 30 --fused --our-adam > gpurun_out/span_tr.txt 2>&1 || { tail -20 gpurun_out/span_tr.txt; exit 1; }
f=$(find gpurun_out/span_tr -name "*kernel_stats.csv" | head -1); head -12 "$f" | cut -c1-200
