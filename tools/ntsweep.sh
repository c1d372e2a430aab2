set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
for f in ${FLAGS:-0 0x400 0x800 0xc00}; do
  PG_SPMM_FLAGS=$f timeout -k 10 120 python bench.py --no-pmc --no-cpu-baseline --steps 200 --warmup 50 > gpurun_out/b_$f.json 2>/dev/null || exit 1
  echo "$rep $f $(python -c "import json;d=json.loads(open('gpurun_out/b_$f.json').read().strip().splitlines()[-1]);print(d['ms_per_step'], d['roofline']['avg_launch_ms'])")" >> gpurun_out/ntsweep.txt
done
done
