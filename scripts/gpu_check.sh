#!/bin/bash
# GPU-box check: smoke, then the GPU parity tests. Stops at the first crash-like exit.
set -u
mkdir -p gpurun_out
timeout -k 10 400 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -5 gpurun_out/smoke.log
case $rc in 0|1) ;; *) echo "stopping after smoke rc=$rc"; exit $rc;; esac
timeout -k 10 1200 python -m pytest tests -q -m gpu --timeout 180 ${PYTEST_ARGS:-} > gpurun_out/gpu_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -40 gpurun_out/gpu_tests.log
exit $rc
