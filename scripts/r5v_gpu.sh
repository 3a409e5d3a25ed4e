set -u
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 bash scripts/profile_r5.sh > gpurun_out/r5v_prof.log 2>&1
rc=$?; echo "profile rc=$rc"; exit $rc
