#!/bin/bash
# round 5: nested walks in length order (KX_NESTED_SORT = log2 bucket bytes, -1 off) A/B + the nested GPU tests
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; [ $rc = 0 ] || { echo "rc=$rc: $*"; exit $rc; }; }
run 300 python -u -m pytest tests/test_gpu_nested.py tests/test_gpu_pbn.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5sort_tests.log 2>&1
for s in 0 1 2 3 -1; do   # needs a kx_nested.hip build with the sort (reverted)
  KX_NESTED_SORT=$s run 120 python3 scripts/nested_time.py 1048576 4096 > gpurun_out/r5sort_nt_$s.log 2>&1
  KX_NESTED_SORT=$s NEST_FILE=tmpdata/nest_distinct_262144.bin run 120 python3 scripts/nested_time.py 262144 > gpurun_out/r5sort_nd_$s.log 2>&1
  KX_NESTED_SORT=$s run 120 python3 scripts/pbn_time.py > gpurun_out/r5sort_pbn_$s.log 2>&1
done
echo done
