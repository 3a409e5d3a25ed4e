#!/bin/bash
# Kernel trace (stats) of the nested walker's timing scripts: Thrift Nesting (decode concatenated / offsets,
# encode) and Kitex-PB PN decode. Usage: scripts/nested_prof.sh TAG
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
TAG=$1
for w in nested pbn; do
  OUT=gpurun_out/prof_${TAG}_$w
  rm -rf $OUT && mkdir -p $OUT
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- python3 scripts/${w}_time.py > $OUT/run.log 2>&1 || exit $?
  f=$(find $OUT -name "*kernel_stats.csv" | head -1)
  cp "$f" gpurun_out/${TAG}_${w}_kernel_stats.csv || exit 1
done
echo nested_prof done
