#!/bin/bash
# Round-4 GPU check 12: HBM traffic (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, csv) and kernel stats of the transposed
# kernels at B(20,4), F = 128; raw rocprofv3 output removed, summaries kept.
set -o pipefail
rm -rf gpurun_out/tpmc gpurun_out/tstats
mkdir -p gpurun_out/tpmc
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --pmc $c --kernel-trace -d gpurun_out/tpmc/$c -o k --output-format csv -- python3 tools/tprobe.py 10 > gpurun_out/tpmc/$c.log 2>&1 || { tail -20 gpurun_out/tpmc/$c.log; exit 1; }
done
python tools/pmc_traffic.py gpurun_out/tpmc/FETCH_SIZE gpurun_out/tpmc/WRITE_SIZE gpurun_out/r04_transposed_traffic.json transposed_B20_4_F128 || exit 1
timeout -s KILL 150 rocprofv3 --kernel-trace --stats -d gpurun_out/tstats -o k --output-format csv -- python3 tools/tprobe.py 20 > gpurun_out/tstats.log 2>&1 || { tail -20 gpurun_out/tstats.log; exit 1; }
find gpurun_out/tstats -name "*kernel_stats.csv" -exec cp {} gpurun_out/r04_transposed_kernel_stats.csv \;
grep -E "spmm3t|midt2" gpurun_out/r04_transposed_kernel_stats.csv | cut -c1-200
rm -rf gpurun_out/tpmc gpurun_out/tstats
