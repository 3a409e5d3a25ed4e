#!/bin/bash
# encode A/B: the default library against a variant (kitex_amd/lib/$VARIANT), outputs checked against
# the direct path inside each run (scripts/enc_time.py), plus the encode parity suites
set -u
cd "$(dirname "$0")/.."
run() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; [ $rc = 0 ] || { echo "rc=$rc: $*"; exit $rc; }; }
run 400 python -u -m pytest tests/test_gpu_thrift.py tests/test_gpu_list_struct.py tests/test_gpu_messages.py -q -x --timeout 120 --timeout-method thread -k "encode or marshal or Marshal or bit_exact or roundtrip" > gpurun_out/enc_tests.log 2>&1
run 200 python -u scripts/enc_time.py r3 > gpurun_out/enc_ab.log 2>&1
run 200 env KXCODEC_LIB=kitex_amd/lib/${VARIANT:-iq0}/libkxcodec.so python -u scripts/enc_time.py r3 >> gpurun_out/enc_ab.log 2>&1
run 200 python -u scripts/enc_time.py r2 16777216 >> gpurun_out/enc_ab.log 2>&1
