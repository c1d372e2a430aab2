#!/bin/bash
# Round-5 GPU check 5: the bf16 dgrad determinism probe against the default library and four diagnostic builds
mkdir -p gpurun_out
export PROBE_MODES=poison_random,poison_big
: > gpurun_out/r05_dgrad_exp.json
for e in ${EXPS:-"" 1 2 3 4}; do
  if [ -n "$e" ]; then export PG_DIRECTGCN_LIB=$PWD/protgram-directgcn_amd/libpgdgcn_exp$e.so; fi
  timeout -k 10 120 python -u tools/r05_dgrad_bf16_probe.py 20 >> gpurun_out/r05_dgrad_exp.json || exit 1
done
