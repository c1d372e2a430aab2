#!/bin/bash
# One GPU call's worth of profiles for the committed evidence (run from the repo root on the GPU box):
#  1. rocprofv3 --kernel-trace --stats of the default bench command -> per-kernel durations
#  2. FETCH_SIZE and WRITE_SIZE passes over tools/kprobe.py -> per-launch HBM bytes (tools/pmc_traffic.py)
#  3. the counter passes of tools/pmc_passes.sh -> tools/pmc_summary.py
#  4. the same counter passes over bench.py's forward alone; bench.py --extra (kernel variants, training step);
#     the 5-gram bench under the kernel trace
# Each GPU step has its own time limit; the script stops at the first failure.
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/round
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/bench -o b --output-format csv -- python3 $R/bench.py --no-cpu-baseline > $O/bench.log 2>&1
echo "bench trace done"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/fetch -o k --output-format csv -- python3 $R/tools/kprobe.py 3 > $O/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/write -o k --output-format csv -- python3 $R/tools/kprobe.py 3 > $O/write.log 2>&1
python3 $R/tools/pmc_traffic.py $O/fetch $O/write $O/traffic.json "B(20,4)/F128" > $O/traffic.txt
echo "traffic done"
bash $R/tools/pmc_passes.sh $O/pmc
python3 $R/tools/pmc_summary.py $O/pmc > $O/pmc_summary.txt 2>&1 || true
echo "pmc done"
KPROBE_ARGS="--forward 5" bash $R/tools/pmc_passes.sh $O/pmcf
python3 $R/tools/pmc_summary.py $O/pmcf > $O/pmcf_summary.txt 2>&1 || true
echo "forward pmc done"
timeout -k 10 300 python3 $R/bench.py --no-cpu-baseline --no-pmc --extra > $O/extra.log 2>&1
echo "extra done"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/bench5 -o b --output-format csv -- python3 $R/bench.py --ngram 5 --steps 20 --warmup 5 --no-cpu-baseline --no-pmc > $O/bench5.log 2>&1
echo "5-gram trace done"
