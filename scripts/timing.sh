#!/bin/bash
# GPU-box diagnostics: per-phase timing of the decode kernel (KX_TIMING=1) for each library variant
# named in VARIANTS ("" = the default build), R2 concat at 1M and 16M records.
set -u
mkdir -p gpurun_out
for v in ${VARIANTS:-default}; do
  lib=kitex_amd/lib/libkxcodec.so; [ "$v" != default ] && lib=kitex_amd/lib/$v/libkxcodec.so
  for r in ${RECORDS:-1000000 16777216}; do
    KXCODEC_LIB=$PWD/$lib KX_TIMING=${TIMING:-1} timeout -k 10 120 python -u bench.py --steps ${STEPS:-2} --warmup 1 --no-cpu \
      --records $r ${BENCH_ARGS:-} > gpurun_out/timing_${v}_$r.log 2>&1 || { echo "$v $r rc=$?"; tail -5 gpurun_out/timing_${v}_$r.log; exit 1; }
    echo "== $v $r: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/timing_${v}_$r.log)"
    grep KX_TIMING gpurun_out/timing_${v}_$r.log | tail -1
  done
done
