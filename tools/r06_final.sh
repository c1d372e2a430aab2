#!/bin/bash
# Round-6 final tree: smoke(), the full -m gpu suite (the driver's command), the default bench line (live PMC traffic
# + CPU baseline), the driver-argument line, its rocprofv3 kernel stats, the builder-produced (fasta) level's line,
# the training probes (config 3 eager / graphed, config 5), the dense backward's kernels, the config-5 rank step under
# RCCL calls, and a kernel trace + counter pass of the config-3 training step. Argument 1 / 2: the first / second half
# (each fits one gpurun call).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out/${R06_TAG:-r06f1}
PART=${1:-all}
if [ "$PART" != "2" ]; then
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > ${O}_smoke.log 2>&1 || { tail -30 ${O}_smoke.log; exit 1; }
tail -1 ${O}_smoke.log
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread -p no:cacheprovider > ${O}_suite.log 2>&1 || { grep -E "FAILED|Error" ${O}_suite.log | tail -20; tail -30 ${O}_suite.log; exit 1; }
tail -1 ${O}_suite.log
timeout -k 10 400 python -u bench.py > ${O}_bench.json 2> ${O}_bench.err || { tail -30 ${O}_bench.err; exit 1; }
cut -c1-300 ${O}_bench.json
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-pmc --no-cpu-baseline > ${O}_bench_driverargs.json 2> ${O}_bench_driverargs.err || { tail -30 ${O}_bench_driverargs.err; exit 1; }
cut -c1-300 ${O}_bench_driverargs.json
rm -rf ${O}_prof
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d ${O}_prof -o run -- python3 bench.py --no-pmc --no-cpu-baseline > ${O}_prof.json 2> ${O}_prof.err || { tail -30 ${O}_prof.err; exit 1; }
find ${O}_prof -name "*kernel_stats.csv" -exec cp {} ${O}_bench_kernel_stats.csv \;
rm -rf ${O}_prof
head -5 ${O}_bench_kernel_stats.csv | cut -c1-160
timeout -k 10 300 python -u bench.py --graph fasta --no-pmc --no-cpu-baseline > ${O}_fasta.json 2> ${O}_fasta.err || { tail -30 ${O}_fasta.err; exit 1; }
cut -c1-300 ${O}_fasta.json
fi
if [ "$PART" != "1" ]; then
for a in "--fused --our-adam" "--graph --our-adam" "--fused --our-adam --no-head" "--fused --our-adam --no-span" "--fused --our-adam --bf16 --dims=128,256,256,256"; do
  timeout -k 10 200 python -u tools/train_probe.py 20 $a >> ${O}_train.txt 2>&1 || { tail -20 ${O}_train.txt; exit 1; }
done
grep "train step" ${O}_train.txt
timeout -k 10 200 python -u tools/r05_dgrad_time.py > ${O}_dense_bwd_times.json 2>&1 || { tail -20 ${O}_dense_bwd_times.json; exit 1; }
tail -1 ${O}_dense_bwd_times.json
timeout -k 10 400 python -u tools/middle_train_probe.py --comm rccl > ${O}_mtp_rccl.json 2> ${O}_mtp_rccl.err || { tail -20 ${O}_mtp_rccl.err; exit 1; }
cut -c1-400 ${O}_mtp_rccl.json
rm -rf ${O}_trtr
timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d ${O}_trtr -o run -- python3 tools/train_probe.py 30 --fused --our-adam > ${O}_trtr.txt 2>&1 || { tail -20 ${O}_trtr.txt; exit 1; }
f=$(find ${O}_trtr -name "*kernel_trace.csv" | head -1)
python3 tools/r05_gaps.py $f 20 adam_kernel > ${O}_train_timeline.txt
rm -rf ${O}_trtr
head -3 ${O}_train_timeline.txt
rm -rf ${O}_fpmc
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d ${O}_fpmc -o run -- python3 tools/kprobe.py --forward > ${O}_fpmc.txt 2>&1 || { tail -20 ${O}_fpmc.txt; exit 1; }
python3 tools/r05_pmc_sum.py ${O}_fpmc dense_x3p ngram_mid_kernel head_x3 > ${O}_forward_pmc.txt
rm -rf ${O}_fpmc
cut -c1-300 ${O}_forward_pmc.txt
for a in "--fused --our-adam --bf16 --dims=128,256,256,256" "--graph --our-adam --bf16 --dims=128,256,256,256"; do
  timeout -k 10 200 python -u tools/train_probe.py 20 $a >> ${O}_train.txt 2>&1 || { tail -20 ${O}_train.txt; exit 1; }
done
rm -rf ${O}_pmc
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d ${O}_pmc -o run -- python3 tools/train_probe.py 5 --fused --our-adam > ${O}_pmc.txt 2>&1 || { tail -20 ${O}_pmc.txt; exit 1; }
python3 tools/r05_pmc_sum.py ${O}_pmc head_train_kernel wgrad_x3 dgrad_span dgrad_x3 ngram_midt2 > ${O}_train_pmc.txt
rm -rf ${O}_pmc
cut -c1-300 ${O}_train_pmc.txt
fi
echo final-ok
