#!/bin/bash
# One GPU-box checkpoint, step by step (each step under its own time limit; the first failure ends the run).
# Usage: scripts/gpu_round.sh TAG STEP...   STEP: tests | smoke | frames | nested | bench | host
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
TAG=$1; shift
run() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; [ $rc = 0 ] || { echo "rc=$rc: $*"; exit $rc; }; }
for step in "$@"; do
  case $step in
    tests) run 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1;;
    smoke) run 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1;;
    frames) run 300 python -u scripts/frames_time.py > gpurun_out/${TAG}_frames.log 2>&1;;
    nested) run 300 python -u scripts/nested_time.py > gpurun_out/${TAG}_nested.log 2>&1;;
    bench) run 900 python -u bench.py --steps 10 --warmup 3 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench_progress.log;;
    host) run 600 python -u bench.py --steps 3 --warmup 1 --no-cpu --no-extra > gpurun_out/${TAG}_host.json 2> gpurun_out/${TAG}_host_progress.log;;
    *) echo "unknown step $step"; exit 2;;
  esac
  echo "$step ok"
done
