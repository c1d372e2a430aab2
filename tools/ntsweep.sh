# Cache-policy A/B of the bench step: each entry "flags:head" runs bench.py (200 steps, no PMC / CPU baseline) with
# PG_SPMM_FLAGS=flags and PG_HEAD_NT=head, twice over, appending "rep flags head ms_per_step avg_launch_ms" lines to
# gpurun_out/ntsweep.txt. usage: CASES="0:0 0x400:0 0:1" bash tools/ntsweep.sh
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
for c in ${CASES:-0:0 0x400:0 0:1}; do
  f=${c%%:*}; h=${c##*:}
  PG_SPMM_FLAGS=$f PG_HEAD_NT=$h timeout -k 10 120 python bench.py --no-pmc --no-cpu-baseline --steps 200 --warmup 50 > gpurun_out/b_$f_$h.json 2>/dev/null || exit 1
  echo "$rep $f $h $(python -c "import json;d=json.loads(open('gpurun_out/b_$f_$h.json').read().strip().splitlines()[-1]);print(d['ms_per_step'], d['roofline']['avg_launch_ms'])")" >> gpurun_out/ntsweep.txt
done
done
