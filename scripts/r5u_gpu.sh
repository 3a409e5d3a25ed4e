set -u
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; [ $rc = 0 ] || { echo "rc=$rc: $*"; exit $rc; }; }
run 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/r5u_gpu_tests.log 2>&1
run 200 python3 scripts/pbn_time.py > gpurun_out/r5u_pbn.log 2>&1
run 200 python3 scripts/nested_time.py > gpurun_out/r5u_nested.log 2>&1
rm -rf gpurun_out/prof_r5u_pbn
run 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r5u_pbn -o run --output-format csv -- python3 scripts/pbn_time.py > /dev/null 2>&1
run 300 python -u bench.py --config pf --steps 10 --warmup 3 --no-cpu --no-host --no-extra > gpurun_out/r5u_pf.json 2> gpurun_out/r5u_pf.err
echo ALLOK
