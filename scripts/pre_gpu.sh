#!/bin/bash
# run before every gpurun: fresh in-tree build + CPU suite must pass
set -e
cd "$(dirname "$0")/.."
python kitex_amd/build.py > /tmp/kx_build.log 2>&1 || { grep -E "error" -A3 /tmp/kx_build.log | head -30; exit 1; }
make -s -C oracle
timeout 900 python -m pytest tests -q -m "not gpu" -x 2>&1 | tail -1
