#!/bin/bash
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
run() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; [ $rc = 0 ] || { echo "rc=$rc: $*"; exit $rc; }; }
run 400 python -u -m pytest tests/test_gpu_nested.py tests/test_gpu_pbn.py tests/test_gpu_list_struct.py tests/test_gpu_generic.py -q -x --timeout 120 --timeout-method thread > gpurun_out/r12_tests.log 2>&1
run 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_nested -o run --output-format csv -- python3 scripts/nested_time.py > gpurun_out/prof_nested.log 2>&1
