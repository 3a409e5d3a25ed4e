#!/bin/bash
# Round-3 GPU call: targeted tests, SQ counters of the decode + encode kernels, bench line.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
  echo "$name rc=$rc"; grep -v amdgpu.ids "gpurun_out/$name.log" | tail -${TAILN:-3} | cut -c1-400
  case $rc in 0|1) return 0;; *) echo "stopping after $name rc=$rc"; exit $rc;; esac
}
[ -n "${TESTS:-}" ] && step tests 900 python -u -m pytest -q -m gpu --timeout 120 --timeout-method thread --maxfail=20 $TESTS
if [ "${SQ:-1}" = 1 ]; then
  step sq 300 bash scripts/sq_counters.sh r2
  python3 scripts/sq_summary.py gpurun_out/sq_r2 > gpurun_out/sq_r2_summary.json 2>&1 || true
fi
[ "${BENCH:-1}" = 1 ] && step bench 400 python -u bench.py --steps 10 --warmup 3 --no-cpu --no-host
echo r3_run2 done
if [ "${ENC_AB:-0}" = 1 ]; then
  for c in 0 1; do
    KX_ENC_CANON=$c step enc_canon$c 300 python -u bench.py --steps 10 --warmup 3 --no-cpu --no-host
    python3 -c "
import json; d=json.loads(open('gpurun_out/enc_canon$c.log').read().strip().splitlines()[-1]); x=d['extra']
print('canon=$c', {k:(round(v['ms_per_step'],3), v.get('bit_exact')) for k,v in x.items() if k.endswith('encode')})"
  done
fi
# AB="VAR v1 v2 ...": the bench once per value of environment variable VAR, extras' times side by side
if [ -n "${AB:-}" ]; then
  set -- $AB
  var=$1; shift
  for c in "$@"; do
    env "$var=$c" timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu --no-host > gpurun_out/ab_$c.log 2>&1 || { echo "ab $c failed"; tail -5 gpurun_out/ab_$c.log; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/ab_$c.log').read().strip().splitlines()[-1]); x=d['extra']
print('$var=$c', 'headline', round(d['ms_per_step'],3), {k:(round(v['ms_per_step'],3), v.get('bit_exact', v.get('verified'))) for k,v in x.items()})"
  done
fi
