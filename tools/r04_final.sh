#!/bin/bash
# Round-4 final tree on one MI355X: smoke(), the full -m gpu suite, the default bench line (live PMC passes + CPU
# baseline), its rocprofv3 kernel stats, the driver-argument bench line, and the fasta / bf16 lines.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04f_smoke.log 2>&1 || { tail -30 gpurun_out/r04f_smoke.log; exit 1; }
tail -1 gpurun_out/r04f_smoke.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/r04f_suite.log 2>&1 || { tail -60 gpurun_out/r04f_suite.log; exit 1; }
tail -2 gpurun_out/r04f_suite.log
timeout -k 10 400 python -u bench.py > gpurun_out/r04f_bench.json 2> gpurun_out/r04f_bench.err || { tail -30 gpurun_out/r04f_bench.err; exit 1; }
cat gpurun_out/r04f_bench.json
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-pmc --no-cpu-baseline > gpurun_out/r04f_bench_driverargs.json 2> gpurun_out/r04f_bench_driverargs.err || { tail -30 gpurun_out/r04f_bench_driverargs.err; exit 1; }
cat gpurun_out/r04f_bench_driverargs.json
rm -rf gpurun_out/r04f_prof
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04f_prof -o run -- python3 bench.py --no-pmc --no-cpu-baseline > gpurun_out/r04f_prof.json 2> gpurun_out/r04f_prof.err || { tail -30 gpurun_out/r04f_prof.err; exit 1; }
find gpurun_out/r04f_prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/r04f_bench_kernel_stats.csv \;
rm -rf gpurun_out/r04f_prof
head -6 gpurun_out/r04f_bench_kernel_stats.csv | cut -c1-160
timeout -k 10 400 python -u bench.py --graph fasta --no-cpu-baseline > gpurun_out/r04f_fasta.json 2> gpurun_out/r04f_fasta.err || { tail -30 gpurun_out/r04f_fasta.err; exit 1; }
cat gpurun_out/r04f_fasta.json
timeout -k 10 300 python -u bench.py --bf16 --no-pmc --no-cpu-baseline > gpurun_out/r04f_bf16.json 2> gpurun_out/r04f_bf16.err || { tail -30 gpurun_out/r04f_bf16.err; exit 1; }
cat gpurun_out/r04f_bf16.json
