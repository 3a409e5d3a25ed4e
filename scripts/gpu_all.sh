./scripts/gpu_check.sh; rc=$?; echo "check rc=$rc"
case $rc in 0|1) ;; *) exit $rc;; esac
PROFILE=0 ./scripts/gpu_bench.sh
