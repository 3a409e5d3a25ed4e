#!/bin/bash
# Decode ablations (KX_DIAG) + per-kernel times (rocprofv3 kernel trace) + SQ counter passes, R2.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
CFG=${1:-r2}
timeout -k 10 300 python3 -u scripts/ablate.py $CFG 16777216 0,256,257 > gpurun_out/r3_ablate2.log 2>&1; rc=$?
echo "ablate rc=$rc"; cat gpurun_out/r3_ablate2.log
[ $rc = 0 ] || exit $rc
rm -rf gpurun_out/prof_k && mkdir -p gpurun_out/prof_k
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_k -o run --output-format csv -- python3 scripts/run_decode.py $CFG 16777216 5 > gpurun_out/prof_k.log 2>&1; rc=$?
echo "prof rc=$rc"
[ $rc = 0 ] || exit $rc
timeout -k 10 300 ./scripts/sq_counters.sh $CFG; rc=$?
echo "sq rc=$rc"
exit $rc
