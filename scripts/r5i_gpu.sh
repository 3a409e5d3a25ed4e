set -u
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; [ $rc = 0 ] || { echo "rc=$rc: $*"; exit $rc; }; }
rm -rf gpurun_out/prof_r5_bimodal
run 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r5_bimodal -o run --output-format csv -- python3 scripts/bimodal_time.py > gpurun_out/r5i_bimodal.log 2>&1
run 400 python -u -m pytest tests/test_gpu_thrift.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5i_thrift.log 2>&1
run 600 bash scripts/nested_prof.sh
echo ALLOK
