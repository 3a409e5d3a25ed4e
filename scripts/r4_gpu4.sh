#!/bin/bash
# Round 4: GPU parity of the round's changes (split points, 16 var slots, nested, frames), the small c5
# run, then the full default bench line (headline + extras incl. the nested entry).
set -u
cd "$(dirname "$0")/.."
run() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; [ $rc = 0 ] || { echo "rc=$rc: $*"; exit $rc; }; }
run 600 python -u -m pytest tests/test_gpu_thrift.py tests/test_gpu_adversarial.py tests/test_gpu_nested.py tests/test_gpu_frames.py tests/test_gpu_pbn.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4_tests.log 2>&1
run 300 python -u bench.py --config c5 --c5-scale 0.25 --steps 3 --warmup 1 --no-cpu > gpurun_out/c5_small.log 2>&1
run 600 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r4_bench.log 2>&1
