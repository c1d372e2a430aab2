#!/bin/bash
# round 6: A/B of two library builds on the default bench step (interleaved runs): abtmp/lib_slp.so vs the in-tree one
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
: > gpurun_out/r06_ab.txt
for i in 1 2 3; do
  for lib in abtmp/lib_slp.so protgram-directgcn_amd/libpgdgcn.so; do
    PG_DIRECTGCN_LIB=$PWD/$lib timeout -k 10 200 python -u bench.py --no-pmc --no-cpu-baseline --steps 100 --warmup 30 2>/dev/null \
      | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); k=d['roofline']['kernels']; print('$lib', d['ms_per_step'], k['dense']['avg_launch_ms'], k['propagation']['avg_launch_ms'], k['head']['avg_launch_ms'])" >> gpurun_out/r06_ab.txt || exit 1
  done
done
cat gpurun_out/r06_ab.txt
