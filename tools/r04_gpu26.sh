#!/bin/bash
# Round-4 GPU check 26b: head kernel, W1 loads first and their split pinned before the h rows land (112 VGPRs, occupancy 4)
# two bench lines (per-kernel head time from HIP events).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "head" > gpurun_out/r04_t29.log 2>&1 || { tail -30 gpurun_out/r04_t29.log; exit 1; }
tail -1 gpurun_out/r04_t29.log
timeout -k 10 120 python -u tools/head_probe.py > gpurun_out/r04_head_probe.txt 2>&1 || { tail -20 gpurun_out/r04_head_probe.txt; exit 1; }
cat gpurun_out/r04_head_probe.txt
for i in 1 2; do
timeout -k 10 300 python -u bench.py --no-pmc --no-cpu-baseline > gpurun_out/r04_b26_$i.json 2> gpurun_out/r04_b26_$i.err || { tail -30 gpurun_out/r04_b26_$i.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r04_b26_$i.json'));print(d['ms_per_step'], d['roofline']['dominant_by'])"
done
