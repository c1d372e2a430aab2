#!/bin/bash
# Round-4 GPU check 16: HBM traffic of the scatter kernel and the gather-sums (rocprofv3 --pmc FETCH_SIZE /
# WRITE_SIZE passes) at config 5's rank-0 shapes.
set -o pipefail
rm -rf gpurun_out/spmc
mkdir -p gpurun_out/spmc
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --pmc $c --kernel-trace -d gpurun_out/spmc/$c -o k --output-format csv -- python3 tools/scatter_probe.py --cpw 0 --reps 5 --no-csr > gpurun_out/spmc/$c.log 2>&1 || { tail -20 gpurun_out/spmc/$c.log; exit 1; }
done
python tools/pmc_traffic.py gpurun_out/spmc/FETCH_SIZE gpurun_out/spmc/WRITE_SIZE gpurun_out/r04_scatter_traffic.json scatter_cfg5_rank0 || exit 1
cat gpurun_out/r04_scatter_traffic.json
rm -rf gpurun_out/spmc
