#!/bin/bash
# Index-pass variants on the default R2 bench (and PF): KX_INDEX_PF=0 (one tile per wave) vs the
# persistent double-buffered kernel with N workgroups per CU.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/pf
for cfg in ${CONFIGS:-r2}; do
  for pf in ${PFS:-0 1 2}; do
    f=gpurun_out/pf/${cfg}_${pf}.log
    KX_INDEX_PF=$pf timeout -k 10 120 python -u bench.py --config $cfg --steps ${STEPS:-20} --warmup 3 --no-cpu \
      --no-host --no-extra > $f 2>&1 || { echo "$cfg $pf rc=$?"; tail -5 $f; exit 1; }
    echo "$cfg pf=$pf $(grep -o '"ms_per_step": [0-9.]*' $f) $(grep -o '"verified": [a-z]*' $f | head -1)"
  done
done
