#!/bin/bash
# Round-4 final tree (training glue removed: contiguous unshared dense gradients, cached bf16 input, no unused
# embeddings in the trainer step, forward-packed weights reused by the backward): smoke(), the full -m gpu suite, the
# per-rank probe and attribution, the default bench line and the driver-argument bench line.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04f5_smoke.log 2>&1 || { tail -30 gpurun_out/r04f5_smoke.log; exit 1; }
tail -1 gpurun_out/r04f5_smoke.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/r04f5_suite.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/r04f5_suite.log | tail -20; tail -30 gpurun_out/r04f5_suite.log; exit 1; }
tail -1 gpurun_out/r04f5_suite.log
timeout -k 10 300 python -u tools/middle_train_probe.py > gpurun_out/r04_mtp26.json 2> gpurun_out/r04_mtp26.err || { tail -30 gpurun_out/r04_mtp26.err; exit 1; }
cat gpurun_out/r04_mtp26.json
timeout -k 10 400 python -u tools/middle_train_attr.py > gpurun_out/r04_attr3.txt 2> gpurun_out/r04_attr3.err || { tail -30 gpurun_out/r04_attr3.err; exit 1; }
head -3 gpurun_out/r04_attr3.txt | cut -c1-200
timeout -k 10 400 python -u bench.py > gpurun_out/r04f5_bench.json 2> gpurun_out/r04f5_bench.err || { tail -30 gpurun_out/r04f5_bench.err; exit 1; }
cut -c1-400 gpurun_out/r04f5_bench.json
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-pmc --no-cpu-baseline > gpurun_out/r04f5_bench_driverargs.json 2> gpurun_out/r04f5_bench_driverargs.err || { tail -30 gpurun_out/r04f5_bench_driverargs.err; exit 1; }
cut -c1-300 gpurun_out/r04f5_bench_driverargs.json
