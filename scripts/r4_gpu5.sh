#!/bin/bash
# Round 4: fused CRC32Check + LDS-cursor nested walker: GPU parity, nested A/B, then the default bench line
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
run() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; [ $rc = 0 ] || { echo "rc=$rc: $*"; exit $rc; }; }
run 600 python -u -m pytest tests/test_gpu_frames.py tests/test_gpu_crc.py tests/test_gpu_nested.py tests/test_gpu_pbn.py tests/test_gpu_messages.py tests/test_gpu_thrift.py tests/test_gpu_adversarial.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5_tests.log 2>&1
for v in 0 1; do run 200 env KX_NESTED_LDS=$v python -u scripts/nested_time.py; done > gpurun_out/nested_ab.log 2>&1
run 900 python -u bench.py --steps 10 --warmup 3 --no-host > gpurun_out/r5_bench.log 2>&1
