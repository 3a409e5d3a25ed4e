#!/bin/bash
# Round 4: nested walker with LDS cursors: parity, A/B timing, kernel stats
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
run() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; [ $rc = 0 ] || { echo "rc=$rc: $*"; exit $rc; }; }
run 400 python -u -m pytest tests/test_gpu_nested.py tests/test_gpu_pbn.py -x -q --timeout 120 --timeout-method thread > gpurun_out/nested_tests.log 2>&1
for v in 0 1; do run 200 env KX_NESTED_LDS=$v python -u scripts/nested_time.py; done > gpurun_out/nested_ab.log 2>&1
run 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_nested -o run --output-format csv -- python3 scripts/nested_time.py > gpurun_out/prof_nested.log 2>&1
