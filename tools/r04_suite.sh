#!/bin/bash
# Round-4 tree on one MI355X: smoke() and the full -m gpu suite.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04s_smoke.log 2>&1 || { tail -30 gpurun_out/r04s_smoke.log; exit 1; }
tail -1 gpurun_out/r04s_smoke.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/r04s_suite.log 2>&1 || { tail -60 gpurun_out/r04s_suite.log; exit 1; }
tail -2 gpurun_out/r04s_suite.log
