set -u
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; [ $rc = 0 ] || { echo "rc=$rc: $*"; exit $rc; }; }
run 500 python -u -m pytest tests/test_gpu_nested.py tests/test_gpu_pbn.py tests/test_gpu_list_struct.py tests/test_gpu_generic.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5r_tests.log 2>&1
: > gpurun_out/r5r_nested.log
for rpl in 0 1 2 4 8; do
  if [ $rpl = 0 ]; then unset KX_NESTED_RPL; else export KX_NESTED_RPL=$rpl; fi
  echo "rpl=$rpl" >> gpurun_out/r5r_nested.log
  run 200 python3 scripts/nested_time.py 1048576 4096 >> gpurun_out/r5r_nested.log 2>&1
done
unset KX_NESTED_RPL
rm -rf gpurun_out/prof_r5r_nested
run 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r5r_nested -o run --output-format csv -- python3 scripts/nested_time.py > gpurun_out/r5r_nested_prof.log 2>&1
echo ALLOK
