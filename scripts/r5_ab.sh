#!/bin/bash
# Round 5: A/B of library builds, alternating, whole decode of one config (scripts/index_diag.py, KX_DIAG=0)
#   LIBS="default nt ef:KX_EMIT_FAST=0" CFG=r2 N=16777216 MODE=concat bash scripts/r5_ab.sh
# "default" is kitex_amd/lib/libkxcodec.so, any other name kitex_amd/lib/<name>/libkxcodec.so; ":VAR=VAL"
# adds an environment setting for that entry.
set -u
cd "$(dirname "$0")/.."
run() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; [ $rc = 0 ] || { echo "rc=$rc: $*"; exit $rc; }; }
for rep in ${REPS:-1 2}; do
  for ent in ${LIBS:-default}; do
    v=${ent%%:*}
    extra=""
    [ "$ent" != "$v" ] && extra=${ent#*:}
    lib=kitex_amd/lib/libkxcodec.so
    [ "$v" != default ] && lib=kitex_amd/lib/$v/libkxcodec.so
    echo "== $ent (rep $rep)"
    run 120 env KXCODEC_LIB=$lib KX_DIAG=${DIAG:-0} $extra python -u scripts/index_diag.py ${CFG:-r2} ${N:-16777216} ${MODE:-concat}
  done
done
