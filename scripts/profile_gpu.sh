#!/bin/bash
# GPU-box profiling recipe (run through gpurun): kernel-trace stats + separate PMC passes
# (FETCH_SIZE, WRITE_SIZE: one TCC counter group per pass) of the default bench workload.
# Usage: scripts/profile_gpu.sh <tag> [bench args...]
set -e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
TAG=${1:-r2}; shift || true
ARGS="--steps 5 --warmup 2 --no-cpu --no-host --no-extra $*"
OUT=gpurun_out/prof_$TAG
rm -rf $OUT && mkdir -p $OUT
sha256sum ${KXCODEC_LIB:-kitex_amd/lib/libkxcodec.so} | cut -d" " -f1 > $OUT/lib.sha256
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- python3 bench.py $ARGS > $OUT/bench.log 2>&1
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 bench.py $ARGS > $OUT/fetch.log 2>&1
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 bench.py $ARGS > $OUT/write.log 2>&1
echo done
