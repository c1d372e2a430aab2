#!/bin/bash
# Round-4 GPU check 3: config 5's middle-partition trainer (8 ranks on this GPU) and its per-rank probe; kernel trace
# of bench --graph fasta.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 880 --timeout-method thread \
  tests/test_gpu_middle_train.py > gpurun_out/r04_t3.log 2>&1 || { grep -E "Error|assert" gpurun_out/r04_t3.log | tail -20; exit 1; }
grep -E "PASSED|FAILED|ranks \(" gpurun_out/r04_t3.log
timeout -k 10 300 python -u tools/middle_train_probe.py > gpurun_out/r04_mtp.json 2> gpurun_out/r04_mtp.err || { tail -30 gpurun_out/r04_mtp.err; exit 1; }
cat gpurun_out/r04_mtp.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_fasta -o k --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --graph fasta --no-pmc --no-cpu-baseline --steps 20 --warmup 5 > $GRAFT_REPO_ROOT/gpurun_out/r04_fasta_prof.json 2> $GRAFT_REPO_ROOT/gpurun_out/r04_fasta_prof.err || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/r04_fasta_prof.err; exit 1; }
find $GRAFT_REPO_ROOT/gpurun_out/prof_fasta -name "*kernel_stats.csv" | head -3
head -12 $(find $GRAFT_REPO_ROOT/gpurun_out/prof_fasta -name "*kernel_stats.csv" | head -1)
