set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python tools/dense_exp.py 4 20 > gpurun_out/dense_exp.log 2>&1 || exit 1
for rep in 1 2; do
for f in 0 0x800 0x1000 0x2000 0x1800 0x3800; do
  PG_SPMM_FLAGS=$f timeout -k 10 120 python bench.py --no-pmc --no-cpu-baseline --steps 200 --warmup 50 > gpurun_out/b_$f.json 2>/dev/null || exit 1
  echo "$rep $f $(python -c "import json;d=json.loads(open('gpurun_out/b_$f.json').read().strip().splitlines()[-1]);print(d['ms_per_step'], d['roofline']['avg_launch_ms'])")" >> gpurun_out/ntsweep.txt
done
done
