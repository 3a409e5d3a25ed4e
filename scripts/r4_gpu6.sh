#!/bin/bash
# Round 4: gather diagnostics, nested A/B, then the default bench line
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
run() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; [ $rc = 0 ] || { echo "rc=$rc: $*"; exit $rc; }; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_thrift.py -q --timeout 120 --timeout-method thread -k "length_gather" > gpurun_out/r6_gather.log 2>&1
rc=$?; [ $rc = 0 ] || [ $rc = 1 ] || exit $rc
for v in 0 1; do run 200 env KX_NESTED_LDS=$v python -u scripts/nested_time.py; done > gpurun_out/nested_ab.log 2>&1
run 900 python -u bench.py --steps 10 --warmup 3 --no-host > gpurun_out/r6_bench.log 2>&1
