#!/bin/bash
# round 6: A/B of library builds abtmp/<name>.so on bench.py --graph fasta (no PMC, no CPU baseline), interleaved,
# three rounds: ms per step and the dense / propagation / head per-launch HIP-event times
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
: > gpurun_out/r06_ab_fasta.txt
for i in 1 2 3; do
  for lib in "$@"; do
    PG_DIRECTGCN_LIB=$PWD/abtmp/$lib.so timeout -k 10 300 python -u bench.py --graph fasta --no-pmc --no-cpu-baseline --steps 100 --warmup 30 2>/dev/null \
      | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); k=d['roofline']['kernels']; print('$lib', d['ms_per_step'], k['dense']['avg_launch_ms'], k['propagation']['avg_launch_ms'], k['head']['avg_launch_ms'])" >> gpurun_out/r06_ab_fasta.txt || exit 1
  done
done
cat gpurun_out/r06_ab_fasta.txt
