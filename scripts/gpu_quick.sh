#!/bin/bash
# GPU-box: smoke, GPU parity tests, short benches. Each step time-limited; stop at the first crash-like exit.
set -u
mkdir -p gpurun_out
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -${TAILN:-4} "gpurun_out/$name.log"
  case $rc in 0) return 0;; 1) [ "${STRICT:-0}" = 1 ] && exit 1; return 0;; *) echo "stopping after $name rc=$rc"; exit $rc;; esac
}
[ "${SMOKE:-1}" = 1 ] && step smoke 300 python -u __graft_entry__.py smoke
[ "${TESTS:-1}" = 1 ] && step gpu_tests 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread ${PYTEST_ARGS:-}
for r in ${BENCH_RECORDS:-16777216}; do
  step bench_$r 300 python -u bench.py --steps 10 --warmup 3 --no-cpu --records $r ${BENCH_ARGS:-}
done
