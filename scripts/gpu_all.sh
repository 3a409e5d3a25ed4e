#!/bin/bash
./scripts/gpu_check.sh; rc=$?; echo "check rc=$rc"
case $rc in 0|1) ;; *) exit $rc;; esac
./scripts/gpu_bench.sh
