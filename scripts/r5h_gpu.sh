set -u
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; [ $rc = 0 ] || { echo "rc=$rc: $*"; exit $rc; }; }
run 300 python -u -m pytest tests/test_gpu_adversarial.py -v -s --timeout 120 --timeout-method thread > gpurun_out/r5g_adv.log 2>&1
run 400 python -u -m pytest tests/test_gpu_thrift.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5g_thrift.log 2>&1
run 600 bash scripts/nested_prof.sh
run 900 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r5g_bench.json 2> gpurun_out/r5g_bench.err
echo ALLOK
