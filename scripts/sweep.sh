#!/bin/bash
# scripts/sweep.sh "<env_sweep args>" ["<env_sweep args>" ...]: each sweep under its own time limit
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for a in "$@"; do
  timeout -k 10 400 python3 -u scripts/env_sweep.py $a >> gpurun_out/sweep.log 2>&1; rc=$?
  [ $rc = 0 ] || { echo "sweep rc=$rc"; cat gpurun_out/sweep.log; exit $rc; }
done
cat gpurun_out/sweep.log
