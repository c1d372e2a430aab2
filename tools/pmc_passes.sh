#!/bin/bash
# Counter passes for tools/kprobe.py (one rocprofv3 run per pass; counters only with --kernel-trace).
# usage: tools/pmc_passes.sh OUTDIR [PASSFILE]   (PASSFILE: one space-separated counter group per line)
# KPROBE_ARGS: arguments for tools/kprobe.py (default "3": every hot-path kernel)
set -e
export TMPDIR=/tmp
OUT=${1:-$GRAFT_REPO_ROOT/gpurun_out/pmc}
PASSES=${2:-}
mkdir -p $OUT
if [ -z "$PASSES" ]; then
  PASSES=$OUT/passes.txt
  cat > $PASSES <<'P'
SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_LEVEL_WAVES
TCC_HIT TCC_MISS TCC_REQ TCC_BUSY
TCP_TOTAL_CACHE_ACCESSES TCP_TCC_READ_REQ TCP_PENDING_STALL_CYCLES TCP_TCR_TCP_STALL_CYCLES
TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES TD_TD_BUSY
TA_DATA_STALLED_BY_TC_CYCLES
SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT
P
fi
i=0
while read -r line; do
  [ -z "$line" ] && continue
  i=$((i+1))
  timeout -k 10 150 rocprofv3 --pmc $line --kernel-trace -d $OUT/p$i -o k --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/kprobe.py ${KPROBE_ARGS:-3} > $OUT/p$i.log 2>&1
done < $PASSES
echo done
