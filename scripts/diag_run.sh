#!/bin/bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for a in "$@"; do
  echo "== $a"
  timeout -k 10 120 python3 -u scripts/fast_diag.py $a > gpurun_out/diag.log 2>&1; rc=$?
  cat gpurun_out/diag.log | grep -v amdgpu.ids
  [ $rc = 0 ] || exit $rc
done
