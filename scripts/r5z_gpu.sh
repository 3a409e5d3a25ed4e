set -u
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; [ $rc = 0 ] || { echo "rc=$rc: $*"; exit $rc; }; }
rm -rf gpurun_out/prof_r5z_idl
run 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r5z_idl -o run --output-format csv -- python3 scripts/idl_order_time.py > gpurun_out/r5z_idl.log 2>&1
: > gpurun_out/r5z_adv.log
for i in 1 2; do run 300 python -u -m pytest tests/test_gpu_adversarial.py -q -s --timeout 120 --timeout-method thread >> gpurun_out/r5z_adv.log 2>&1; done
run 300 python -u -m pytest tests/test_gpu_thrift.py tests/test_gpu_generic.py tests/test_gpu_messages.py -q -x --timeout 120 --timeout-method thread > gpurun_out/r5z_thrift.log 2>&1
echo ALLOK
