set -u
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/r5l_occ.log
for o in 0 20480 40960 81920; do
  KX_NESTED_OCC=$o timeout -k 10 120 python3 scripts/nested_time.py >> gpurun_out/r5l_occ.log 2>&1 || exit 1
  rm -rf gpurun_out/prof_r5l_$o
  KX_NESTED_OCC=$o timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r5l_$o -o run --output-format csv -- python3 scripts/nested_time.py > /dev/null 2>&1 || exit 1
  echo "occ $o done" >> gpurun_out/r5l_occ.log
done
echo ALLOK
