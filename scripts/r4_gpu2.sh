#!/bin/bash
# Round 4: nested proto3 GPU parity + nested thrift regression, then the index-pass diagnostics.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_pbn.py tests/test_gpu_nested.py -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/r4_gpu2_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -5 gpurun_out/r4_gpu2_tests.log
[ $rc = 0 ] || [ $rc = 1 ] || exit $rc
bash scripts/r4_diag1.sh > gpurun_out/r4_diag1.log 2>&1; rc=$?
echo "diag rc=$rc"; grep -v amdgpu.ids gpurun_out/r4_diag1.log | tail -30
