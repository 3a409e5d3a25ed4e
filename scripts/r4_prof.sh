#!/bin/bash
# Round 4 profiles: kernel stats + FETCH/WRITE PMC passes of every timed workload (profile_all.sh), SQ
# counters of the R2 decode (split index kernels) and of the R3 encode write pass
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
bash scripts/profile_all.sh r4 r2_concat pf_concat r3_concat r2_encode r3_encode || exit $?
bash scripts/sq_counters.sh r2 || exit $?
RUN=scripts/run_encode.py N=4194304 SUFFIX=_enc bash scripts/sq_counters.sh r3 || exit $?
echo prof done
