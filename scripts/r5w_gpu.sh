set -u
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; [ $rc = 0 ] || { echo "rc=$rc: $*"; exit $rc; }; }
run 300 python -u -m pytest tests/test_gpu_adversarial.py tests/test_gpu_thrift.py -q -x --timeout 120 --timeout-method thread > gpurun_out/r5w_tests.log 2>&1
run 200 python -u bench.py --steps 10 --warmup 3 --no-cpu --no-host --no-extra > gpurun_out/r5w_head.json 2>/dev/null
run 1000 bash scripts/profile_r5.sh > gpurun_out/r5w_prof.log 2>&1
echo ALLOK
