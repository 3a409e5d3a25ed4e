set -u
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; [ $rc = 0 ] || { echo "rc=$rc: $*"; exit $rc; }; }
run 600 python -u -m pytest tests/test_gpu_thrift.py tests/test_gpu_c5.py tests/test_gpu_chunked.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5f_tests.log 2>&1
run 600 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r5f_bench.log 2>&1
echo ALLOK
