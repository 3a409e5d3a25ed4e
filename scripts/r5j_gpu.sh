set -u
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; [ $rc = 0 ] || { echo "rc=$rc: $*"; exit $rc; }; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_adversarial.py -v -s --timeout 120 --timeout-method thread > gpurun_out/r5j_adv.log 2>&1
rc=$?; [ $rc = 0 ] || [ $rc = 1 ] || { echo "adv rc=$rc"; exit $rc; }
run 120 python3 scripts/bimodal_time.py > gpurun_out/r5j_bimodal.log 2>&1
run 600 bash scripts/nested_prof.sh
run 900 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r5j_bench.json 2> gpurun_out/r5j_bench.err
echo ALLOK
