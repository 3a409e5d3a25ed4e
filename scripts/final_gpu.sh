#!/bin/bash
# Round-end GPU evidence in one call: smoke, the GPU parity suite, the default bench line, then the
# rocprofv3 kernel-trace stats and the FETCH_SIZE / WRITE_SIZE passes of the headline workload (each
# profiler pass a run of its own), and a stats pass over the extras (R3, PF, encode, CRC32C kernels).
# Every GPU step has its own time limit; the script stops at the first failure.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/final_$name.log" 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -2 "gpurun_out/final_$name.log" | cut -c1-300
  [ $rc = 0 ] || exit $rc
}
step smoke 300 python -u __graft_entry__.py smoke
step tests 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread
step bench 500 python -u bench.py
step profile 600 ./scripts/profile_gpu.sh final
rm -rf gpurun_out/prof_final_extra && mkdir -p gpurun_out/prof_final_extra
step extra_stats 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_final_extra/stats -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu --no-host
echo final done
