#!/bin/bash
# Round 4: kernel stats of the known-offsets decode with and without the length gather
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
run() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; [ $rc = 0 ] || { echo "rc=$rc: $*"; exit $rc; }; }
run 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_off -o run --output-format csv -- python3 bench.py --mode offsets --steps 5 --warmup 2 --no-cpu --no-host --no-extra > gpurun_out/prof_off.log 2>&1
export KX_GATHER=0
run 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_off0 -o run --output-format csv -- python3 bench.py --mode offsets --steps 5 --warmup 2 --no-cpu --no-host --no-extra > gpurun_out/prof_off0.log 2>&1
