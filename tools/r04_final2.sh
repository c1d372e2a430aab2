#!/bin/bash
# Round-4 final tree, after restoring the plain middle-tile kernel's register form: the n-gram GPU tests, the forward
# kernel probe, the default bench line (live PMC + CPU baseline), the driver-argument line and its rocprofv3 kernel
# stats, and the fasta line.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ngram.py tests/test_gpu_builder_graph.py tests/test_gpu_bench.py > gpurun_out/r04f2_t.log 2>&1 || { tail -40 gpurun_out/r04f2_t.log; exit 1; }
tail -1 gpurun_out/r04f2_t.log
timeout -k 10 200 python -u tools/ngram_probe_k.py 4 128 20 > gpurun_out/r04f2_probe.txt 2>&1 || { tail -20 gpurun_out/r04f2_probe.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r04f2_probe.txt | tail -3
timeout -k 10 400 python -u bench.py > gpurun_out/r04f2_bench.json 2> gpurun_out/r04f2_bench.err || { tail -30 gpurun_out/r04f2_bench.err; exit 1; }
cat gpurun_out/r04f2_bench.json | cut -c1-400
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-pmc --no-cpu-baseline > gpurun_out/r04f2_bench_driverargs.json 2> gpurun_out/r04f2_bench_driverargs.err || { tail -30 gpurun_out/r04f2_bench_driverargs.err; exit 1; }
cut -c1-300 gpurun_out/r04f2_bench_driverargs.json
rm -rf gpurun_out/r04f2_prof
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04f2_prof -o run -- python3 bench.py --no-pmc --no-cpu-baseline > gpurun_out/r04f2_prof.json 2> gpurun_out/r04f2_prof.err || { tail -30 gpurun_out/r04f2_prof.err; exit 1; }
find gpurun_out/r04f2_prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/r04f2_bench_kernel_stats.csv \;
rm -rf gpurun_out/r04f2_prof
head -4 gpurun_out/r04f2_bench_kernel_stats.csv | cut -c1-160
timeout -k 10 400 python -u bench.py --graph fasta --no-cpu-baseline > gpurun_out/r04f2_fasta.json 2> gpurun_out/r04f2_fasta.err || { tail -30 gpurun_out/r04f2_fasta.err; exit 1; }
cut -c1-300 gpurun_out/r04f2_fasta.json
