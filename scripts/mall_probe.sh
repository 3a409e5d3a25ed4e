#!/bin/bash
# Per-kernel decode time vs batch size (Infinity-Cache residency probe): kernel-trace stats of
# the default R2 bench at several record counts.
set -e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
for r in ${RECORDS:-1000000 16777216}; do
  OUT=gpurun_out/mall_$r
  rm -rf $OUT && mkdir -p $OUT
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu --no-host --no-extra --records $r ${BENCH_ARGS:-} > $OUT/bench.log 2>&1
  echo "== $r"; find $OUT -name '*kernel_stats.csv' -exec head -8 {} \;
done
