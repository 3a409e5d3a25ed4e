set -u
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; [ $rc = 0 ] || { echo "rc=$rc: $*"; exit $rc; }; }
: > gpurun_out/r5p_nested.log
for k in 1 16 4096; do
  KX_NESTED_WIN=0 run 200 python3 scripts/nested_time.py 1048576 $k >> gpurun_out/r5p_nested.log 2>&1
done
echo ALLOK
