set -u
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/prof_r5off
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r5off -o run --output-format csv -- python3 scripts/run_decode_offsets.py r2 16777216 5 > gpurun_out/r5off.log 2>&1
echo rc=$?
