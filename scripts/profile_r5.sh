#!/bin/bash
# Round 5 profiles: kernel stats + FETCH/WRITE PMC passes of every timed workload (profile_all.sh), SQ
# counters of the R2 decode (fast index / fast chain / fast emit kernels), and the nested walker's stats,
# SQ and TCP counters (nested_prof.sh). Summaries only are kept under gpurun_out/r5_summ.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
S=gpurun_out/r5_summ
rm -rf $S && mkdir -p $S
bash scripts/profile_all.sh r5 r2_concat pf_concat r3_concat r2_encode r3_encode || exit $?
bash scripts/sq_counters.sh r2 || exit $?
for w in r2_concat pf_concat r3_concat; do
  PMC_OUT=$S python3 scripts/pmc_summary.py gpurun_out/prof_r5_$w ${w%_concat} concat > /dev/null || exit $?
done
for w in r2 r3; do
  PMC_OUT=$S python3 scripts/pmc_summary.py gpurun_out/prof_r5_${w}_encode $w encode > /dev/null || exit $?
done
python3 scripts/sq_summary.py gpurun_out/sq_r2 > $S/sq_r2_decode.json || exit $?
for w in r2_concat pf_concat r3_concat r2_encode r3_encode; do
  cp gpurun_out/prof_r5_$w/stats/run_kernel_stats.csv $S/${w}_kernel_stats.csv || exit $?
  cp gpurun_out/prof_r5_$w/lib.sha256 $S/lib.sha256
done
rm -rf gpurun_out/prof_r5_r2_concat gpurun_out/prof_r5_pf_concat gpurun_out/prof_r5_r3_concat gpurun_out/prof_r5_r2_encode gpurun_out/prof_r5_r3_encode gpurun_out/sq_r2
bash scripts/nested_prof.sh || exit $?
python3 scripts/nested_summary.py gpurun_out/prof_r5_nested > $S/nested_pmc_sq.json || exit $?
cp gpurun_out/prof_r5_nested/stats/run_kernel_stats.csv $S/nested_kernel_stats.csv || exit $?
echo prof done
