#!/bin/bash
# PMC traffic and kernel stats of the bench line's extra workloads (scripts/run_workload.py): per workload the
# inputs are prepared once outside the profiler, then a kernel-trace stats pass and the FETCH_SIZE / WRITE_SIZE
# passes (each its own rocprofv3 run) over 1 warm-up + 3 calls; summaries under gpurun_out/<TAG>_summ.
# Usage: scripts/profile_extras.sh TAG [workloads...]
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
TAG=$1; shift
WL=${*:-frames_off frames_on nested_concat nested_offsets pb_nested r2_views r2_offsets r2_offsets_views}
LIB=kitex_amd/lib/libkxcodec.so
S=gpurun_out/${TAG}_summ
mkdir -p $S
for w in $WL; do
  OUT=gpurun_out/prof_${TAG}_$w
  rm -rf $OUT && mkdir -p $OUT
  sha256sum $LIB | cut -d" " -f1 > $OUT/lib.sha256
  timeout -k 10 300 python3 scripts/run_workload.py prep $w > $OUT/prep.log 2>&1 || { echo "$w prep failed"; exit 1; }
  for pass in stats fetch write; do
    case $pass in
      stats) P="--kernel-trace --stats";;
      fetch) P="--pmc FETCH_SIZE";;
      write) P="--pmc WRITE_SIZE";;
    esac
    timeout -k 10 240 rocprofv3 $P -d $OUT/$pass -o run --output-format csv -- python3 scripts/run_workload.py run $w 3 > $OUT/$pass.log 2>&1
    rc=$?
    echo "$w $pass rc=$rc"
    [ $rc = 0 ] || exit $rc
  done
  M=all; case $w in *_encode) M=nenc;; esac
  PMC_OUT=$S python3 scripts/pmc_summary.py $OUT $w $M 4 > /dev/null || exit 1
  f=$(find $OUT/stats -name "*kernel_stats.csv" | head -1)
  cp "$f" $S/${w}_kernel_stats.csv
  rm -rf $OUT /tmp/kxw_$w.npz
done
echo profile_extras done
