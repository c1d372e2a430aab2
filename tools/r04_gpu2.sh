#!/bin/bash
# Round-4 GPU check 2: builder-produced graphs on the mapped middle-tile kernel (tests), bench --graph fasta, the
# default bench line, then config 5's middle-partition trainer (8 ranks on this GPU) and its per-rank probe.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_builder_graph.py > gpurun_out/r04_t2.log 2>&1 || { tail -60 gpurun_out/r04_t2.log; exit 1; }
tail -12 gpurun_out/r04_t2.log
timeout -k 10 300 python -u bench.py --graph fasta --no-cpu-baseline > gpurun_out/r04_fasta.json 2> gpurun_out/r04_fasta.err || { tail -30 gpurun_out/r04_fasta.err; exit 1; }
cat gpurun_out/r04_fasta.json
grep "\[bench\]" gpurun_out/r04_fasta.err
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-pmc > gpurun_out/r04_b2.json 2> gpurun_out/r04_b2.err || { tail -30 gpurun_out/r04_b2.err; exit 1; }
cat gpurun_out/r04_b2.json
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 880 --timeout-method thread \
  tests/test_gpu_middle_train.py > gpurun_out/r04_t3.log 2>&1 || { tail -60 gpurun_out/r04_t3.log; exit 1; }
grep -E "PASSED|FAILED|ranks \(" gpurun_out/r04_t3.log
timeout -k 10 300 python -u tools/middle_train_probe.py > gpurun_out/r04_mtp.json 2> gpurun_out/r04_mtp.err || { tail -30 gpurun_out/r04_mtp.err; exit 1; }
cat gpurun_out/r04_mtp.json
