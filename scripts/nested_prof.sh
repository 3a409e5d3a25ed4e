#!/bin/bash
# Round 5: kernel trace + SQ / TCP counter passes over the nested walker (baseline.thrift Nesting, 1 M
# records, decode concat + offsets + encode: scripts/nested_time.py). Each pass its own rocprofv3 run.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
N=${N:-1048576}
OUT=gpurun_out/prof_r5_nested
rm -rf $OUT && mkdir -p $OUT
sha256sum kitex_amd/lib/libkxcodec.so | cut -d" " -f1 > $OUT/lib.sha256
pass() {
  local name=$1; shift
  timeout -k 10 180 rocprofv3 "$@" -d $OUT/$name -o run --output-format csv -- python3 scripts/nested_time.py $N > $OUT/$name.log 2>&1
  local rc=$?
  echo "nested $name rc=$rc"
  [ $rc = 0 ] || exit $rc
}
pass stats --kernel-trace --stats
pass sq1 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VALU
pass sq2 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT
pass tcp --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCP_PENDING_STALL_CYCLES_sum
pass fetch --pmc FETCH_SIZE
echo nested_prof done
