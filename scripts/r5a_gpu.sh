set -u
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; [ $rc = 0 ] || { echo "rc=$rc: $*"; exit $rc; }; }
run 300 python -u -m pytest tests/test_gpu_crc.py tests/test_gpu_pb.py tests/test_gpu_thrift.py -x -q --timeout 120 --timeout-method thread -k "crc32 or split or base" > gpurun_out/r5a_tests.log 2>&1
run 500 python -u -m pytest tests/test_gpu_thrift.py tests/test_gpu_adversarial.py tests/test_gpu_c5.py tests/test_gpu_chunked.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5a_ef_tests.log 2>&1
run 120 scripts/copy_floor > gpurun_out/r5a_floor.log 2>&1
LIBS="default default:KX_EMIT_FAST=0 nt e1:KX_EMIT_FAST=0 e2:KX_EMIT_FAST=0 e4:KX_EMIT_FAST=0" run 900 bash scripts/r5_ab.sh > gpurun_out/r5a_ab.log 2>&1
echo ALLOK
