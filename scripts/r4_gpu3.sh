#!/bin/bash
# Round 4: split points (tests + c5 bench at reduced scale), then the fast-plan variant's parity and A/B.
set -u
cd "$(dirname "$0")/.."
run() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; [ $rc = 0 ] || { echo "rc=$rc: $*"; exit $rc; }; }
run 400 python -u -m pytest tests/test_gpu_thrift.py tests/test_gpu_adversarial.py -x -q --timeout 120 --timeout-method thread > gpurun_out/split_tests.log 2>&1
run 300 python -u bench.py --config c5 --c5-scale 0.25 --steps 3 --warmup 1 --no-cpu > gpurun_out/c5_small.log 2>&1
run 300 env KXCODEC_LIB=kitex_amd/lib/fp/libkxcodec.so python -u -m pytest tests/test_gpu_thrift.py -x -q --timeout 120 --timeout-method thread -k "not split and not 2gib" > gpurun_out/fp_tests.log 2>&1
VARIANT=fp bash scripts/r4_ab.sh > gpurun_out/ab_fp.log 2>&1
