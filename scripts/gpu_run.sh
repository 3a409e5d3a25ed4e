#!/bin/bash
# Generic GPU-box step runner: scripts/gpu_run.sh "<pytest args>" [bench args...]
# pytest step (if non-empty), then bench.py with the given args; each step under its own time limit.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-}; shift || true
if [ -n "$T" ]; then
  timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread $T > gpurun_out/run_tests.log 2>&1; rc=$?
  echo "tests rc=$rc"; tail -15 gpurun_out/run_tests.log
  [ $rc = 0 ] || exit $rc
fi
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u bench.py "$@" > gpurun_out/run_bench.log 2>&1; rc=$?
  echo "bench rc=$rc"; tail -c 3000 gpurun_out/run_bench.log
  exit $rc
fi
