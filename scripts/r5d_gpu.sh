set -u
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; [ $rc = 0 ] || { echo "rc=$rc: $*"; exit $rc; }; }
run 600 python -u -m pytest tests/test_gpu_chunked.py tests/test_gpu_thrift.py tests/test_gpu_adversarial.py tests/test_gpu_c5.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5d_tests.log 2>&1
LIBS="default default:KX_CHAIN_FAST=0 default:KX_REDO_WG=1 default:KX_REDO_WG=2" REPS="1 2 3" run 600 bash scripts/r5_ab.sh > gpurun_out/r5d_ab.log 2>&1
cd /tmp
run 200 rocprofv3 --kernel-trace --stats -d /root/repo/gpurun_out/r5d_prof -o run --output-format csv -- python3 /root/repo/scripts/run_decode.py r2 16777216 3 > /root/repo/gpurun_out/r5d_prof.log 2>&1
KX_REDO_WG=1 run 200 rocprofv3 --kernel-trace --stats -d /root/repo/gpurun_out/r5d_prof1 -o run --output-format csv -- python3 /root/repo/scripts/run_decode.py r2 16777216 3 > /root/repo/gpurun_out/r5d_prof1.log 2>&1
echo ALLOK
