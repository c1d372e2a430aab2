# Round-end check on one MI355X: the GPU suite, the default bench line (live PMC traffic, CPU baseline), and a
# rocprofv3 kernel trace of the bench. Every GPU step has its own time limit; the first failure ends the script.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gputests.log 2>&1 || exit 11
timeout -k 10 240 python bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err || exit 12
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --no-pmc --no-cpu-baseline > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err || exit 13
timeout -k 10 240 python bench.py --ngram 5 --steps 20 --warmup 5 --no-pmc --no-cpu-baseline > gpurun_out/bench5.json 2> gpurun_out/bench5.err || exit 14
