#!/bin/bash
# SQ counter passes over the decode kernels (each pass its own rocprofv3 run, <= 8 SQ counters).
set -e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
CFG=${1:-r2}
N=${N:-16777216}
RUN=${RUN:-scripts/run_decode.py}   # or scripts/run_crc.py / scripts/run_encode.py
OUT=gpurun_out/sq_$CFG${SUFFIX:-}
rm -rf $OUT && mkdir -p $OUT
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VALU -d $OUT/p1 -o run --output-format csv -- python3 $RUN $CFG $N 2 > $OUT/p1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU -d $OUT/p2 -o run --output-format csv -- python3 $RUN $CFG $N 2 > $OUT/p2.log 2>&1
echo sq done
