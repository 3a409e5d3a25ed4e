#!/bin/bash
# GPU-box profiling of every timed workload (run through gpurun): per workload a kernel-trace stats pass
# and the FETCH_SIZE / WRITE_SIZE passes (each pass its own rocprofv3 run, one TCC counter group per pass).
# Usage: scripts/profile_all.sh <tag> [workloads...]   (default: r2_concat pf_concat r3_concat r2_encode r3_encode)
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
TAG=${1:-r3}; shift || true
WL=${*:-r2_concat pf_concat r3_concat r2_encode r3_encode}
LIB=${KXCODEC_LIB:-kitex_amd/lib/libkxcodec.so}
for w in $WL; do
  OUT=gpurun_out/prof_${TAG}_$w
  rm -rf $OUT && mkdir -p $OUT
  sha256sum $LIB | cut -d" " -f1 > $OUT/lib.sha256
  case $w in
    r2_concat) CMD="bench.py --steps 5 --warmup 2 --no-cpu --no-host --no-extra";;
    pf_concat) CMD="bench.py --config pf --steps 5 --warmup 2 --no-cpu --no-host --no-extra";;
    r3_concat) CMD="bench.py --config r3 --records 4194304 --steps 5 --warmup 2 --no-cpu --no-host --no-extra";;
    r2_encode) CMD="scripts/run_encode.py r2 16777216 5";;
    r3_encode) CMD="scripts/run_encode.py r3 4194304 5";;
    r2_crc) CMD="scripts/run_crc.py r2 16777216 5";;
    *) echo "unknown workload $w"; exit 2;;
  esac
  for pass in stats fetch write; do
    case $pass in
      stats) P="--kernel-trace --stats";;
      fetch) P="--pmc FETCH_SIZE";;
      write) P="--pmc WRITE_SIZE";;
    esac
    timeout -k 10 240 rocprofv3 $P -d $OUT/$pass -o run --output-format csv -- python3 $CMD > $OUT/$pass.log 2>&1
    rc=$?
    echo "$w $pass rc=$rc"
    [ $rc = 0 ] || exit $rc
  done
done
echo profile_all done
