set -u
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; [ $rc = 0 ] || { echo "rc=$rc: $*"; exit $rc; }; }
for n in 1048576 2097152 4194304 8388608 16777216; do
  run 120 python -u scripts/index_diag.py r2 $n concat >> gpurun_out/r5e_scale.log 2>&1
done
echo ALLOK
