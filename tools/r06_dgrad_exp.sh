#!/bin/bash
# round 6: the layer backward with each diagnostics build of the dgrad kernel (abtmp/libdx_<mask>.so), two rounds
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
: > gpurun_out/r06_dgrad_exp.txt
for r in 1 2; do
  for m in "$@"; do
    PG_DIRECTGCN_LIB=$PWD/abtmp/libdx_$m.so timeout -k 10 120 python -u tools/r06_dgrad_exp.py 2>/dev/null >> gpurun_out/r06_dgrad_exp.txt || exit 1
  done
done
cat gpurun_out/r06_dgrad_exp.txt
