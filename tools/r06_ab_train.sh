#!/bin/bash
# round 6: A/B of two library builds (abtmp/lib_head.so vs abtmp/lib_new.so) on the config-3 and config-5 training
# steps, interleaved, three rounds
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
: > gpurun_out/r06_ab_train.txt
for i in 1 2 3; do
  for lib in ${LIBS:-lib_head lib_new}; do
    for a in "--fused --our-adam" "--fused --our-adam --bf16 --dims=128,256,256,256"; do
      echo -n "$lib " >> gpurun_out/r06_ab_train.txt
      PG_DIRECTGCN_LIB=$PWD/abtmp/$lib.so timeout -k 10 200 python -u tools/train_probe.py 20 $a 2>&1 | grep "train step" >> gpurun_out/r06_ab_train.txt || exit 1
    done
  done
done
cat gpurun_out/r06_ab_train.txt | sed 's/(amp.*opts=\[\])//'
