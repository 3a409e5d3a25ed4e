#!/bin/bash
# Round 4 profiles: kernel stats + FETCH/WRITE PMC passes of every timed workload (profile_all.sh), SQ
# counters of the R2 decode (split index kernels) and of the R3 encode write pass. Summaries only are
# kept under gpurun_out/r4_summ (the raw traces exceed what gpurun copies back).
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
S=gpurun_out/r4_summ
rm -rf $S && mkdir -p $S
bash scripts/profile_all.sh r4 r2_concat pf_concat r3_concat r2_encode r3_encode r2_crc || exit $?
bash scripts/sq_counters.sh r2 || exit $?
RUN=scripts/run_encode.py N=4194304 SUFFIX=_enc bash scripts/sq_counters.sh r3 || exit $?
for w in r2_concat pf_concat r3_concat; do
  PMC_OUT=$S python3 scripts/pmc_summary.py gpurun_out/prof_r4_$w ${w%_concat} concat > /dev/null || exit $?
done
for w in r2 r3; do
  PMC_OUT=$S python3 scripts/pmc_summary.py gpurun_out/prof_r4_${w}_encode $w encode > /dev/null || exit $?
done
PMC_OUT=$S python3 scripts/pmc_summary.py gpurun_out/prof_r4_r2_crc r2 crc > /dev/null || exit $?
python3 scripts/sq_summary.py gpurun_out/sq_r2 > $S/sq_r2_decode.json || exit $?
python3 scripts/sq_summary.py gpurun_out/sq_r3_enc > $S/sq_r3_encode.json || exit $?
for w in r2_concat pf_concat r3_concat r2_encode r3_encode r2_crc; do
  cp gpurun_out/prof_r4_$w/stats/run_kernel_stats.csv $S/${w}_kernel_stats.csv || exit $?
  cp gpurun_out/prof_r4_$w/lib.sha256 $S/lib.sha256
done
rm -rf gpurun_out/prof_r4_* gpurun_out/sq_r2 gpurun_out/sq_r3_enc
echo prof done
