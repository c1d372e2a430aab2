#!/bin/bash
# round 6: A/B of library builds abtmp/<name>.so on a probe script, interleaved, three rounds:
#   tools/r06_ab_lib2.sh <probe.py> <name> [<name> ...]
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
probe=$1; shift
out=gpurun_out/r06_ab_$(basename $probe .py).txt
: > $out
for i in 1 2 3; do
  for lib in "$@"; do
    PG_DIRECTGCN_LIB=$PWD/abtmp/$lib.so timeout -k 10 200 python -u $probe 2>/dev/null >> $out || exit 1
  done
done
cat $out
