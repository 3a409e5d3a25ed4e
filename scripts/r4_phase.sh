#!/bin/bash
# Round 4: marginal cost of each fast-index phase (index pass only, KX_DIAG=256 + stop bits)
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for d in 256 257 1280 2304 4352 256; do
  timeout -k 10 120 env KX_DIAG=$d python -u scripts/index_diag.py r2 || exit $?
done
