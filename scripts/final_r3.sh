#!/bin/bash
# Round-3 evidence in one GPU call, all with the library being committed: smoke, the GPU parity suite,
# the default bench line, the config-5 line, then scripts/profile_all.sh (kernel-trace stats + FETCH_SIZE
# + WRITE_SIZE passes of every timed workload, each pass its own rocprofv3 run). Every GPU step has its
# own time limit; the script stops at the first failure.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r3b}
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/${TAG}_$name.log" 2>&1; local rc=$?
  echo "$name rc=$rc"; grep -v amdgpu.ids "gpurun_out/${TAG}_$name.log" | tail -2 | cut -c1-300
  [ $rc = 0 ] || exit $rc
}
[ "${SMOKE:-1}" = 1 ] && step smoke 300 python -u __graft_entry__.py smoke
[ "${TESTS:-1}" = 1 ] && step tests 700 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread
[ "${BENCH:-1}" = 1 ] && step bench 500 python -u bench.py
[ "${C5:-1}" = 1 ] && step c5 300 python -u bench.py --config c5 --steps 5 --warmup 2 --no-cpu --no-host
[ "${PROF:-1}" = 1 ] && step profile 900 bash scripts/profile_all.sh $TAG
echo final_r3 done
