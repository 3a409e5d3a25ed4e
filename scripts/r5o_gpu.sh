set -u
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; [ $rc = 0 ] || { echo "rc=$rc: $*"; exit $rc; }; }
run 200 python3 scripts/nested_time.py > gpurun_out/r5o_nested.log 2>&1
KX_NESTED_WIN=0 run 200 python3 scripts/nested_time.py >> gpurun_out/r5o_nested.log 2>&1
run 500 python -u -m pytest tests/test_gpu_nested.py tests/test_gpu_pbn.py tests/test_gpu_list_struct.py tests/test_gpu_generic.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5o_tests.log 2>&1
rm -rf gpurun_out/prof_r5o_nested
run 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r5o_nested -o run --output-format csv -- python3 scripts/nested_time.py > gpurun_out/r5o_nested_prof.log 2>&1
echo ALLOK
