#!/bin/bash
# GPU-box bench + profile. Each GPU step has its own time limit; stop at the first crash-like exit.
set -u
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -3 "gpurun_out/$name.log"
  case $rc in 0|1) return 0;; *) echo "stopping after $name rc=$rc"; exit $rc;; esac
}
run bench 600 python bench.py ${BENCH_ARGS:-}
if [ "${PROFILE:-1}" = "1" ]; then
  run rocprof_stats 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/stats -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --no-cpu --no-host ${BENCH_ARGS:-}
  run rocprof_fetch 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof/fetch -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu --no-host ${BENCH_ARGS:-}
  run rocprof_sq 600 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VALU -d gpurun_out/prof/sq -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu --no-host ${BENCH_ARGS:-}
  run rocprof_write 600 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof/write -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu --no-host ${BENCH_ARGS:-}
fi
