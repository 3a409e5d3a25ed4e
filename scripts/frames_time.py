"""Round 4: time kx_thrift_decode_frames over n TTHeader frames with "crc32c" (bench.py frames entry), CRC
check off / on: python scripts/frames_time.py [n]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kitex_amd import schema as S  # noqa: E402
from kitex_amd import synth  # noqa: E402
from kitex_amd.codec import CRC32PayloadValidator, ThriftCodec  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 16 << 20
dev = torch.device("cuda", 0)
cdc = ThriftCodec(S.schema_r1())
src = synth.TORCH_GENERATORS["r1"](n, dev)
msgs, moffs = cdc.MarshalMessages(src, "Echo", torch.zeros(n, dtype=torch.int32, device=dev))
M = msgs.numel() // n
crc = CRC32PayloadValidator(0).Generate(msgs, moffs)
info = bytes([0, 0, 1, 0, 1, 0, 6]) + b"crc32c" + bytes([0, 8]) + b"0" * 8
info += bytes(-len(info) % 4)
H = 14 + len(info)
hdr = (H + M - 4).to_bytes(4, "big") + bytes([0x10, 0, 0, 0]) + bytes(4) + (len(info) // 4).to_bytes(2, "big")
fr = torch.empty((n, H + M), dtype=torch.uint8, device=dev)
fr[:, :H] = torch.tensor(list(hdr + info), dtype=torch.uint8, device=dev)
nib = (crc[:, None] >> torch.arange(28, -4, -4, device=dev)) & 0xF
fr[:, H - len(info) + 15:H - len(info) + 23] = torch.where(nib < 10, nib + 48, nib + 87).to(torch.uint8)
fr[:, H:] = msgs.view(n, M)
wire = fr.view(-1)
for chk in (False, True):
    for _ in range(2):
        cdc.UnmarshalFrames(wire, n, raise_on_error=False, crc32_check=chk)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        r = cdc.UnmarshalFrames(wire, n, raise_on_error=False, crc32_check=chk)
    torch.cuda.synchronize()
    s = r.read_status()
    print(f"frames n={n} crc={chk}: {(time.perf_counter() - t0) / 3 * 1e3:.2f} ms code={s.code}", flush=True)
from kitex_amd.codec import frame_scan, read_status  # noqa: E402
for _ in range(2):
    res = frame_scan(wire, n)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(3):
    res = frame_scan(wire, n)
torch.cuda.synchronize()
st = read_status(res[-1])
print(f"frame_scan n={n}: {(time.perf_counter() - t0) / 3 * 1e3:.2f} ms code={st.code} diag={list(st.diag)}", flush=True)
