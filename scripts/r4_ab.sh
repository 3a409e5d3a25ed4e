#!/bin/bash
# Round 4: A/B of two library builds (default vs $VARIANT), alternating, on index-only and whole decode.
set -u
cd "$(dirname "$0")/.."
V=${VARIANT:-dsigold}
run() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; [ $rc = 0 ] || { echo "rc=$rc: $*"; exit $rc; }; }
for rep in 1 2; do
  for lib in kitex_amd/lib/libkxcodec.so kitex_amd/lib/$V/libkxcodec.so; do
    echo "== $lib"
    for d in 256 0; do run 120 env KXCODEC_LIB=$lib KX_DIAG=$d python -u scripts/index_diag.py ${CFG:-r2} ${N:-16777216} ${MODE:-concat}; done
  done
done
