#!/bin/bash
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
run() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; [ $rc = 0 ] || { echo "rc=$rc: $*"; exit $rc; }; }
run 400 python -u -m pytest tests/test_gpu_thrift.py tests/test_gpu_adversarial.py tests/test_gpu_messages.py tests/test_gpu_frames.py -q -x --timeout 120 --timeout-method thread > gpurun_out/r11_tests.log 2>&1
run 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_off -o run --output-format csv -- python3 bench.py --mode offsets --steps 5 --warmup 2 --no-cpu --no-host --no-extra > gpurun_out/prof_off.log 2>&1
