#!/bin/bash
# Encoder write-pass variants (lib/<variant>/ builds): R2 / R3 encode times from the bench extras.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/enc
for v in ${VARIANTS:-default}; do
  lib=kitex_amd/lib/libkxcodec.so; [ "$v" != default ] && lib=kitex_amd/lib/$v/libkxcodec.so
  f=gpurun_out/enc/$v.log
  KXCODEC_LIB=$PWD/$lib timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu --no-host > $f 2>&1 || { echo "$v rc=$?"; tail -3 $f; exit 1; }
  python3 -c "
import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); x=d['extra']
print('$v', {k:(round(v['ms_per_step'],3), v.get('bit_exact')) for k,v in x.items() if k.endswith('encode')})"
done
