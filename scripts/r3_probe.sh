#!/bin/bash
# Round-3 baseline probe: decode ablations (KX_DIAG) and SQ counter passes of the R2 decode kernels.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u scripts/ablate.py r2 16777216 0,256,768,257 > gpurun_out/r3_ablate.log 2>&1; rc=$?
echo "ablate rc=$rc"; cat gpurun_out/r3_ablate.log
[ $rc = 0 ] || exit $rc
timeout -k 10 300 ./scripts/sq_counters.sh r2; rc=$?
echo "sq rc=$rc"
exit $rc
