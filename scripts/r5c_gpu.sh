set -u
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; [ $rc = 0 ] || { echo "rc=$rc: $*"; exit $rc; }; }
run 120 scripts/launch_cost > gpurun_out/r5c_launch.log 2>&1
for d in 256 257 1280 2304 4352 320; do
  KX_DIAG=$d run 120 python -u scripts/index_diag.py r2 16777216 concat >> gpurun_out/r5c_index.log 2>&1
done
echo ALLOK
