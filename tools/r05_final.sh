#!/bin/bash
# Round-5 final tree: smoke(), the full -m gpu suite, the
# default bench line (live PMC traffic + CPU baseline), the driver-argument line, its rocprofv3 kernel stats and the
# builder-produced (fasta) level's line.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r05f1_smoke.log 2>&1 || { tail -30 gpurun_out/r05f1_smoke.log; exit 1; }
tail -1 gpurun_out/r05f1_smoke.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/r05f1_suite.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/r05f1_suite.log | tail -20; tail -30 gpurun_out/r05f1_suite.log; exit 1; }
tail -1 gpurun_out/r05f1_suite.log
timeout -k 10 400 python -u bench.py > gpurun_out/r05f1_bench.json 2> gpurun_out/r05f1_bench.err || { tail -30 gpurun_out/r05f1_bench.err; exit 1; }
cut -c1-300 gpurun_out/r05f1_bench.json
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-pmc --no-cpu-baseline > gpurun_out/r05f1_bench_driverargs.json 2> gpurun_out/r05f1_bench_driverargs.err || { tail -30 gpurun_out/r05f1_bench_driverargs.err; exit 1; }
cut -c1-300 gpurun_out/r05f1_bench_driverargs.json
rm -rf gpurun_out/r05f1_prof
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05f1_prof -o run -- python3 bench.py --no-pmc --no-cpu-baseline > gpurun_out/r05f1_prof.json 2> gpurun_out/r05f1_prof.err || { tail -30 gpurun_out/r05f1_prof.err; exit 1; }
find gpurun_out/r05f1_prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/r05f1_bench_kernel_stats.csv \;
rm -rf gpurun_out/r05f1_prof
head -5 gpurun_out/r05f1_bench_kernel_stats.csv | cut -c1-160
timeout -k 10 300 python -u bench.py --graph fasta --no-pmc --no-cpu-baseline > gpurun_out/r05f1_fasta.json 2> gpurun_out/r05f1_fasta.err || { tail -30 gpurun_out/r05f1_fasta.err; exit 1; }
cut -c1-300 gpurun_out/r05f1_fasta.json
timeout -k 10 200 python -u tools/train_probe.py 10 --fused --our-adam > gpurun_out/r05f1_train3.txt 2>&1 || { tail -20 gpurun_out/r05f1_train3.txt; exit 1; }
tail -1 gpurun_out/r05f1_train3.txt
timeout -k 10 400 python -u tools/middle_train_probe.py --comm rccl > gpurun_out/r05f1_mtp_rccl.json 2> gpurun_out/r05f1_mtp_rccl.err || { tail -20 gpurun_out/r05f1_mtp_rccl.err; exit 1; }
cut -c1-400 gpurun_out/r05f1_mtp_rccl.json
