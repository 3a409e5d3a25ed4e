set -u
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; [ $rc = 0 ] || { echo "rc=$rc: $*"; exit $rc; }; }
run 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r5x_gpu_tests.log 2>&1
run 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5x_smoke.log 2>&1
run 900 python -u bench.py > gpurun_out/r5x_bench.json 2> gpurun_out/r5x_bench.err
echo ALLOK
