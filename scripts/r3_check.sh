#!/bin/bash
# Round-3 check: targeted GPU tests, config-5 bench line, per-kernel stats of the bench (with extras).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
  echo "$name rc=$rc"; grep -v amdgpu.ids "gpurun_out/$name.log" | tail -${TAILN:-3} | cut -c1-600
  case $rc in 0|1) return 0;; *) echo "stopping after $name rc=$rc"; exit $rc;; esac
}
[ -n "${TESTS:-}" ] && step tests 600 python -u -m pytest -q -m gpu --timeout 120 --timeout-method thread $TESTS
[ "${C5:-0}" = 1 ] && step c5 300 python -u bench.py --config c5 --steps 5 --warmup 2 --no-cpu --no-host
if [ "${STATS:-1}" = 1 ]; then
  rm -rf gpurun_out/prof_r3 && mkdir -p gpurun_out/prof_r3
  step stats 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r3/stats -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu --no-host ${BENCH_ARGS:-}
  python3 scripts/kstats.py gpurun_out/prof_r3/stats 45 || true
fi
