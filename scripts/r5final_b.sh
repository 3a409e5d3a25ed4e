set -u
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u bench.py > gpurun_out/r5final_bench.json 2> gpurun_out/r5final_bench.err
rc=$?; echo "bench rc=$rc"; exit $rc
