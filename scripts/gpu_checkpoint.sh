#!/bin/bash
# Round 4 checkpoint: the whole GPU suite, smoke, then the default bench line
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
run() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; [ $rc = 0 ] || { echo "rc=$rc: $*"; exit $rc; }; }
run 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/r9_gpu_tests.log 2>&1
run 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r9_smoke.log 2>&1
run 900 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r9_bench.log 2>&1
