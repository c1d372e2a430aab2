#!/bin/bash
# round 6: diagnostics builds of dgrad_bf16r_kernel with phases skipped (-DPG_DGRAD_EXP=mask; results are garbage),
# each a whole library abtmp/libdx_<mask>.so for tools/r06_dgrad_exp.sh. Bits: 0 epilogue global loads/stores,
# 1 B k-tile loads, 2 prologue dpre / dpre32 stores, 3 MFMAs, 4 the whole epilogue, 5 prologue dY / Y loads,
# 6 the epilogue's Z loads, 7 its gate-partial (dsp) stores; bit 0 is then the dZ / dres stores only.
set -e
cd "$(dirname "$0")/../protgram-directgcn_amd/csrc"
OBJS=$(ls ../build/*.o | grep -v pg_dense_bwd.o)
for m in "$@"; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I../../include -I. -fno-slp-vectorize \
    -DPG_DGRAD_EXP=$m -c pg_dense_bwd.hip -o ../../abtmp/dx_$m.o &
done
wait
for m in "$@"; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../abtmp/libdx_$m.so $OBJS ../../abtmp/dx_$m.o
done
ls -la ../../abtmp/
