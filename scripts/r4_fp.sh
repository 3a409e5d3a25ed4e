#!/bin/bash
# Round 4: the segment-plan walk (KX_FASTPLAN) A/B, index-only and whole decode, concat and offsets; parity.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
run() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; [ $rc = 0 ] || { echo "rc=$rc: $*"; exit $rc; }; }
run 400 python -u -m pytest tests/test_gpu_thrift.py tests/test_gpu_adversarial.py -x -q --timeout 120 --timeout-method thread
for fp in 0 1; do for d in 256 0; do
  echo "KX_FASTPLAN=$fp"; run 120 env KX_FASTPLAN=$fp KX_DIAG=$d python -u scripts/index_diag.py r2
  run 120 env KX_FASTPLAN=$fp KX_DIAG=$d python -u scripts/index_diag.py r2 16777216 offsets
done; done
for fp in 0 1; do echo "r3 KX_FASTPLAN=$fp"; run 120 env KX_FASTPLAN=$fp python -u scripts/index_diag.py r3 4194304; done
