#!/bin/bash
# Round 4: A/B of an environment knob ($KNOB = A vs B), alternating, on index-only and whole decode
# (or on the command in $CMD); parity of the GPU suites named in $TESTS first.
set -u
cd "$(dirname "$0")/.."
run() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; [ $rc = 0 ] || { echo "rc=$rc: $*"; exit $rc; }; }
[ -n "${TESTS:-}" ] && run 600 python -u -m pytest $TESTS -x -q --timeout 120 --timeout-method thread
for rep in 1 2; do for v in ${VALS:-${A:-0} ${B:-1}}; do
  echo "== $KNOB=$v"
  if [ -n "${CMD:-}" ]; then run 120 env $KNOB=$v $CMD; continue; fi
  for d in ${DIAGS:-256 0}; do run 120 env $KNOB=$v KX_DIAG=$d python -u scripts/index_diag.py ${CFG:-r2} ${N:-16777216} ${MODE:-concat}; done
done; done
