set -u
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; [ $rc = 0 ] || { echo "rc=$rc: $*"; exit $rc; }; }
: > gpurun_out/r5y_adv.log
for i in 1 2; do run 300 python -u -m pytest tests/test_gpu_adversarial.py -q -s --timeout 120 --timeout-method thread >> gpurun_out/r5y_adv.log 2>&1; done
run 300 python -u -m pytest tests/test_gpu_thrift.py -q -x --timeout 120 --timeout-method thread > gpurun_out/r5y_thrift.log 2>&1
echo ALLOK
