#!/bin/bash
# A round's final profiles, in parts (each part fits one gpurun call): kernel stats + FETCH/WRITE PMC passes
# of every timed workload (profile_all.sh), SQ counters of the R2 decode and the R3 encode write pass, and of
# the nested walker (Nesting with offsets, PN); the extras' PMC is scripts/profile_extras.sh TAG. Summaries
# only are kept under gpurun_out/<TAG>_summ (the raw traces exceed what gpurun copies back).
# Usage: scripts/profile_round.sh TAG PART...   PART: main | sq | nested_sq
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
TAG=$1; shift
S=gpurun_out/${TAG}_summ
mkdir -p $S
for part in "$@"; do
  case $part in
    main)
      bash scripts/profile_all.sh $TAG r2_concat pf_concat r3_concat r2_encode r3_encode r2_crc || exit $?
      for w in r2_concat pf_concat r3_concat; do
        PMC_OUT=$S python3 scripts/pmc_summary.py gpurun_out/prof_${TAG}_$w ${w%_concat} concat > /dev/null || exit $?
      done
      for w in r2 r3; do
        PMC_OUT=$S python3 scripts/pmc_summary.py gpurun_out/prof_${TAG}_${w}_encode $w encode > /dev/null || exit $?
      done
      PMC_OUT=$S python3 scripts/pmc_summary.py gpurun_out/prof_${TAG}_r2_crc r2 crc > /dev/null || exit $?
      for w in r2_concat pf_concat r3_concat r2_encode r3_encode r2_crc; do
        cp gpurun_out/prof_${TAG}_$w/stats/run_kernel_stats.csv $S/${w}_kernel_stats.csv || exit $?
        cp gpurun_out/prof_${TAG}_$w/lib.sha256 $S/lib.sha256
      done
      rm -rf gpurun_out/prof_${TAG}_*;;
    sq)
      bash scripts/sq_counters.sh r2 || exit $?
      RUN=scripts/run_encode.py N=4194304 SUFFIX=_enc bash scripts/sq_counters.sh r3 || exit $?
      python3 scripts/sq_summary.py gpurun_out/sq_r2 > $S/sq_r2_decode.json || exit $?
      python3 scripts/sq_summary.py gpurun_out/sq_r3_enc > $S/sq_r3_encode.json || exit $?
      rm -rf gpurun_out/sq_r2 gpurun_out/sq_r3_enc;;
    nested_sq)
      for w in nested_offsets pb_nested; do
        timeout -k 10 300 python3 scripts/run_workload.py prep $w > /dev/null 2>&1 || { echo "$w prep failed"; exit 1; }
        RUN="scripts/run_workload.py run" N=3 bash scripts/sq_counters.sh $w || exit $?
        python3 scripts/sq_summary.py gpurun_out/sq_$w > $S/sq_$w.json || exit $?
        rm -rf gpurun_out/sq_$w /tmp/kxw_$w.npz
      done;;
    *) echo "unknown part $part"; exit 2;;
  esac
  echo "$part done"
done
