#!/bin/bash
# Round 4: chunked two-stream decode pipeline (chain on the aux stream) sweep, combo schedule, CRC A/B,
# chunked-path parity tests. Each step has its own time limit; stops at the first failure.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; [ $rc = 0 ] || { echo "rc=$rc: $*"; exit $rc; }; }
run 300 python -u -m pytest tests/test_gpu_chunked.py -x -q --timeout 120 --timeout-method thread
run 120 env KX_DIAG=0 python -u scripts/index_diag.py r2
for mb in 32 64 128 256; do for a in 1 2; do
  echo "chunk ${mb}MB ahead $a"; run 120 env KX_CHUNK_MB=$mb KX_CHUNK_AHEAD=$a python -u scripts/index_diag.py r2
done; done
for mb in 64 128; do echo "combo ${mb}MB"; run 120 env KX_COMBO_MB=$mb python -u scripts/index_diag.py r2; done
run 120 python -u scripts/run_crc.py r2 16777216 10
run 120 env KXCODEC_LIB=kitex_amd/lib/crcstage/libkxcodec.so python -u scripts/run_crc.py r2 16777216 10
echo sweep done
