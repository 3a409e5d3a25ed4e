#!/bin/bash
# Round-4 GPU diagnostics 1: where the R2 index pass spends its time (index-only, DMA-only floor,
# per-phase cycles of the fast path), full decode for reference, CRC32C staging A/B.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; [ $rc = 0 ] || { echo "rc=$rc: $*"; exit $rc; }; }
run 150 env KX_DIAG=0 python -u scripts/index_diag.py r2
run 150 env KX_DIAG=256 python -u scripts/index_diag.py r2
run 150 env KX_DIAG=257 python -u scripts/index_diag.py r2
run 150 env KX_DIAG=320 python -u scripts/index_diag.py r2
run 150 env KX_DIAG=0 python -u scripts/index_diag.py r2 16777216 offsets
run 150 env KX_DIAG=256 python -u scripts/index_diag.py r2 16777216 offsets
run 150 python -u scripts/run_crc.py r2 16777216 10
run 150 env KXCODEC_LIB=kitex_amd/lib/crcstage/libkxcodec.so python -u scripts/run_crc.py r2 16777216 10
echo diag1 done
