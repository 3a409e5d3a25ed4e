"""Profiler driver and A/B timer: CRC32C Generate (crcPayloadValidator.Generate) over the encoded
records of one config; prints the median event-timed ms per call.
  python scripts/run_crc.py [cfg] [n] [calls]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from kitex_amd import schema as S, synth  # noqa: E402
from kitex_amd.codec import CRC32PayloadValidator, ThriftCodec  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "r2"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 16 << 20
calls = int(sys.argv[3]) if len(sys.argv) > 3 else 3
dev = torch.device("cuda", 0)
cdc = ThriftCodec(S.SCHEMAS[cfg]())
wire, offs = cdc.Marshal(synth.TORCH_GENERATORS[cfg](n, dev))
v = CRC32PayloadValidator(device=0)
crc = v.Generate(wire, offs)
torch.cuda.synchronize()
evs = [torch.cuda.Event(enable_timing=True) for _ in range(calls + 1)]
evs[0].record()
for k in range(calls):
    crc = v.Generate(wire, offs)
    evs[k + 1].record()
torch.cuda.synchronize()
ms = sorted(evs[k].elapsed_time(evs[k + 1]) for k in range(calls))
# spot check against a bytewise CRC-32C of a few records
o = offs.cpu()


def crc32c(data):
    c = 0xFFFFFFFF
    for x in data:
        c ^= x
        for _ in range(8):
            c = (c >> 1) ^ 0x82F63B78 if c & 1 else c >> 1
    return c ^ 0xFFFFFFFF


ok = all(crc32c(bytes(wire[int(o[i]):int(o[i + 1])].cpu().numpy())) == int(crc[i]) for i in (0, 1, n // 2, n - 1))
print(f"crc {cfg} n={n} lib={os.environ.get('KXCODEC_LIB', 'default')}: median {ms[len(ms) // 2]:.4f} ms "
      f"min {ms[0]:.4f} ms sample_ok={ok}", flush=True)
