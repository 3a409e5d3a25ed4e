#!/bin/bash
# Round 4: message-path scan fix: parity of the message / frame suites, frames timing + kernel stats
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
run() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; [ $rc = 0 ] || { echo "rc=$rc: $*"; exit $rc; }; }
run 400 python -u -m pytest tests/test_gpu_messages.py tests/test_gpu_frames.py tests/test_gpu_crc.py tests/test_gpu_grpc.py tests/test_gpu_generic.py tests/test_gpu_ttstream.py tests/test_gpu_thrift.py -q -x --timeout 120 --timeout-method thread > gpurun_out/r8_tests.log 2>&1
run 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_frames2 -o run --output-format csv -- python3 scripts/frames_time.py > gpurun_out/prof_frames2.log 2>&1
