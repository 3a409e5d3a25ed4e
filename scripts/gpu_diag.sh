#!/bin/bash
# GPU-box diagnostics: phase timing, offsets-mode and r1 benches, HBM copy reference.
set -u
mkdir -p gpurun_out
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
  echo "== $name rc=$rc"; tail -${TAILN:-12} "gpurun_out/$name.log"
  case $rc in 0|1) return 0;; *) echo "stopping after $name rc=$rc"; exit $rc;; esac
}
run copybw 120 python -c "
import torch,time
x=torch.empty(2800*1000*1000,dtype=torch.uint8,device='cuda'); y=torch.empty_like(x)
for _ in range(3): y.copy_(x)
torch.cuda.synchronize(); e0=torch.cuda.Event(enable_timing=True); e1=torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(10): y.copy_(x)
e1.record(); torch.cuda.synchronize(); t=e0.elapsed_time(e1)/10
print('copy 2.8GB: %.3f ms  %.1f GB/s (r+w)'%(t, 2*2.8e9/t/1e6))
"
run phase 300 python scripts/phase_timing.py r2
run bench_off 300 python bench.py --mode offsets --no-cpu --no-host --steps 10
run bench_r1 300 python bench.py --config r1 --no-cpu --no-host --steps 10
