#!/bin/bash
# Decode variants (lib/<variant>/ builds): headline + extras decode times and bit-exactness from bench.py.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/dec
for v in ${VARIANTS:-default}; do
  lib=kitex_amd/lib/libkxcodec.so; [ "$v" != default ] && lib=kitex_amd/lib/$v/libkxcodec.so
  f=gpurun_out/dec/$v.log
  KXCODEC_LIB=$PWD/$lib timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu --no-host > $f 2>&1 || { echo "$v rc=$?"; tail -3 $f; exit 1; }
  python3 -c "
import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); x=d['extra']
print('$v', 'headline', round(d['ms_per_step'],3), {k:(round(v['ms_per_step'],3), v.get('bit_exact')) for k,v in x.items()})"
done
