set -u
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; [ $rc = 0 ] || { echo "rc=$rc: $*"; exit $rc; }; }
run 500 python -u -m pytest tests/test_gpu_chunked.py tests/test_gpu_thrift.py tests/test_gpu_adversarial.py tests/test_gpu_c5.py tests/test_gpu_pb.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5b_tests.log 2>&1
for mb in 0 32 64 96 128 256; do for ah in 1 2; do
  [ $mb = 0 ] && [ $ah = 2 ] && continue
  echo "== KX_CHUNK_MB=$mb KX_CHUNK_AHEAD=$ah" >> gpurun_out/r5b_sweep.log
  KX_CHUNK_MB=$mb KX_CHUNK_AHEAD=$ah run 120 python -u scripts/index_diag.py r2 16777216 concat >> gpurun_out/r5b_sweep.log 2>&1
done; done
cd /tmp
for mb in 0 64; do
  KX_CHUNK_MB=$mb run 200 rocprofv3 --kernel-trace --stats -d /root/repo/gpurun_out/r5b_prof_$mb -o run --output-format csv -- python3 /root/repo/scripts/run_decode.py r2 16777216 3 > /root/repo/gpurun_out/r5b_prof_$mb.log 2>&1
done
echo ALLOK
