#!/bin/bash
# Round-4 final tree (after the multi-tensor Adam kernels): smoke(), the full -m gpu suite, the default
# bench line and the driver-argument bench line.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04f4_smoke.log 2>&1 || { tail -30 gpurun_out/r04f4_smoke.log; exit 1; }
tail -1 gpurun_out/r04f4_smoke.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/r04f4_suite.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/r04f4_suite.log | tail -20; tail -30 gpurun_out/r04f4_suite.log; exit 1; }
tail -2 gpurun_out/r04f4_suite.log
timeout -k 10 400 python -u bench.py > gpurun_out/r04f4_bench.json 2> gpurun_out/r04f4_bench.err || { tail -30 gpurun_out/r04f4_bench.err; exit 1; }
cat gpurun_out/r04f4_bench.json
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-pmc --no-cpu-baseline > gpurun_out/r04f4_bench_driverargs.json 2> gpurun_out/r04f4_bench_driverargs.err || { tail -30 gpurun_out/r04f4_bench_driverargs.err; exit 1; }
cat gpurun_out/r04f4_bench_driverargs.json
