#!/bin/bash
# Round-4 GPU check 4: builder-graph tests with the one-launch residual pass, bench --graph fasta (kernel trace),
# kernel trace of one middle-trainer rank (P = 8).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_builder_graph.py > gpurun_out/r04_t4.log 2>&1 || { tail -60 gpurun_out/r04_t4.log; exit 1; }
grep -cE "PASSED" gpurun_out/r04_t4.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_fasta2 -o k --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --graph fasta --no-pmc --no-cpu-baseline --steps 20 --warmup 5 > $GRAFT_REPO_ROOT/gpurun_out/r04_fasta2.json 2> $GRAFT_REPO_ROOT/gpurun_out/r04_fasta2.err || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/r04_fasta2.err; exit 1; }
head -6 $(find $GRAFT_REPO_ROOT/gpurun_out/prof_fasta2 -name "*kernel_stats.csv" | head -1) | cut -c1-200
cd $GRAFT_REPO_ROOT && timeout -k 10 300 python -u bench.py --graph fasta --no-cpu-baseline > gpurun_out/r04_fasta3.json 2> gpurun_out/r04_fasta3.err || { tail -30 gpurun_out/r04_fasta3.err; exit 1; }
cut -c1-300 gpurun_out/r04_fasta3.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_mtp -o k --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/middle_train_probe.py --ranks 0 --reps 10 > $GRAFT_REPO_ROOT/gpurun_out/r04_mtp2.json 2> $GRAFT_REPO_ROOT/gpurun_out/r04_mtp2.err || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/r04_mtp2.err; exit 1; }
head -25 $(find $GRAFT_REPO_ROOT/gpurun_out/prof_mtp -name "*kernel_stats.csv" | head -1) | cut -c1-160
cd $GRAFT_REPO_ROOT && timeout -k 10 300 python -u tools/map_probe.py > gpurun_out/r04_mapprobe.json 2> gpurun_out/r04_mapprobe.err || { tail -20 gpurun_out/r04_mapprobe.err; exit 1; }
cat gpurun_out/r04_mapprobe.json
