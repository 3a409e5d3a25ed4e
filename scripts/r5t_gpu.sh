set -u
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; [ $rc = 0 ] || { echo "rc=$rc: $*"; exit $rc; }; }
run 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/r5t_gpu_tests.log 2>&1
grep -h "canonical R2" gpurun_out/r5t_gpu_tests.log > /dev/null || true
run 300 python -u -m pytest tests/test_gpu_adversarial.py -q -s --timeout 120 --timeout-method thread > gpurun_out/r5t_adv.log 2>&1
run 900 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r5t_bench.json 2> gpurun_out/r5t_bench.err
rm -rf gpurun_out/prof_r5t_pbn
run 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r5t_pbn -o run --output-format csv -- python3 scripts/pbn_time.py > gpurun_out/r5t_pbn.log 2>&1
echo ALLOK
