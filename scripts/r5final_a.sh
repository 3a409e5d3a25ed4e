set -u
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; [ $rc = 0 ] || { echo "rc=$rc: $*"; exit $rc; }; }
run 120 python3 scripts/run_decode_offsets.py r2 16777216 5 > gpurun_out/r5final_off.log 2>&1
run 1000 bash scripts/profile_r5.sh > gpurun_out/r5final_prof.log 2>&1
run 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r5final_gpu_tests.log 2>&1
run 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5final_smoke.log 2>&1
echo ALLOK
