#!/bin/bash
# Decode pipelining sweep (KX_CHUNK_MB x KX_CHUNK_AHEAD) on the default R2 bench and the PF bench.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/sweep
for cfg in ${CONFIGS:-r2}; do
  for mb in ${MBS:-0 32 64 128}; do
    for ah in ${AHEADS:-1}; do
      f=gpurun_out/sweep/${cfg}_${mb}_${ah}.log
      KX_CHUNK_MB=$mb KX_CHUNK_AHEAD=$ah timeout -k 10 120 python -u bench.py --config $cfg --steps ${STEPS:-20} \
        --warmup 3 --no-cpu --no-host --no-extra > $f 2>&1 || { echo "$cfg $mb $ah rc=$?"; tail -5 $f; exit 1; }
      echo "$cfg chunk=${mb}MiB ahead=$ah $(grep -o '"ms_per_step": [0-9.]*' $f) $(grep -o '"verified": [a-z]*' $f | head -1)"
    done
  done
done
