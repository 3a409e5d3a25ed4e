"""Profiler driver for the bench line's extra workloads (test infrastructure for PMC passes, not product).

  python scripts/run_workload.py prep NAME          -> /tmp/kxw_NAME.npz (inputs built once, outside the profile)
  python scripts/run_workload.py run NAME CALLS     -> 1 warm-up + CALLS calls of exactly that workload

The run step launches no codec kernel besides the workload's own (inputs come from the prep file, output
capacities too), so `scripts/pmc_summary.py DIR NAME all CALLS+1` can sum every codec kernel of the profile.
NAME: frames_off, frames_on (16 M TTHeader frames of R1 messages, CRC32Check off / on: bench.py
frames_crc32c), nested_concat, nested_offsets (1 M baseline.thrift Nesting records, 4096 distinct tiled:
bench.py nested_decode_encode), pb_nested (1 M PN records, Batch-framed: bench.py pb_nested), r2_views
(16 M R2 records, string views: bench.py r2_decode_views), nested_encode / pb_nested_encode (the columns of
one decode, encoded: bench.py nested_decode_encode.encode / pb_nested.encode; summarise with mode "nenc"), r2_offsets / r2_offsets_views (the same records
with their offsets known, copies / views: bench.py r2_decode_offsets / r2_decode_offsets_views)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def path(name):
    return f"/tmp/kxw_{name}.npz"


def prep(name):
    import torch

    from kitex_amd import idl, synth
    from kitex_amd import schema as S
    from kitex_amd.codec import CRC32PayloadValidator, ProtobufCodec, ThriftCodec
    dev = torch.device("cuda", 0)
    if name.startswith("frames"):
        n = 16 << 20
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
        np.savez(path(name), wire=fr.view(-1).cpu().numpy(), n=np.array([n]))
    elif name.startswith("nested") or name.startswith("pb_nested"):
        n, k = 1 << 20, 4096
        if name.startswith("pb_nested"):
            from tests import pbn_cases as PB
            sch = PB.schema_pn()
            cdc = ProtobufCodec(sch)
            _, b, o = PB.batch(k, seed=7, name="PN")
            recs = [b"\x0a" + PB.uvarint(int(o[i + 1] - o[i])) + b[int(o[i]):int(o[i + 1])].tobytes() for i in range(k)]
        else:
            doc = idl.parse_idl(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests",
                                             "golden", "idl", "baseline.thrift"))
            sch = idl.to_schema(doc.struct("Nesting"))
            cdc = ThriftCodec(sch)
            recs = synth.thrift_records(sch, k, seed=7)
        one = np.frombuffer(b"".join(recs), dtype=np.uint8)
        wire = np.tile(one, n // k)
        buf = torch.from_numpy(wire).to(dev)
        units = cdc.DecodeSizes(buf, n)
        offs = cdc.Skip(buf, n).cpu().numpy() if name == "nested_offsets" else np.zeros(1, np.int64)
        np.savez(path(name), wire=wire, n=np.array([n]), units=np.array(units, dtype=np.int64), offs=offs)
    elif name in ("r2_views", "r2_offsets", "r2_offsets_views"):
        n = 16 << 20
        cdc = ThriftCodec(S.schema_r2())
        src = synth.TORCH_GENERATORS["r2"](n, dev)
        wire, offs = cdc.Marshal(src)
        np.savez(path(name), wire=wire.cpu().numpy(), n=np.array([n]), offs=offs.cpu().numpy())
    else:
        raise SystemExit(f"unknown workload {name}")


def run(name, calls):
    import torch

    from kitex_amd import _abi as A
    from kitex_amd import idl
    from kitex_amd import schema as S
    from kitex_amd.codec import ProtobufCodec, ThriftCodec, status_tensor
    from kitex_amd.columns import alloc_device
    dev = torch.device("cuda", 0)
    d = np.load(path(name))
    n = int(d["n"][0])
    wire = torch.from_numpy(d["wire"]).to(dev)
    if name.startswith("frames"):
        cdc = ThriftCodec(S.schema_r1())

        def call():
            cdc.UnmarshalFrames(wire, n, raise_on_error=False, crc32_check=name == "frames_on")
    elif name.startswith("nested") or name.startswith("pb_nested"):
        if name.startswith("pb_nested"):
            from tests import pbn_cases as PB
            cdc = ProtobufCodec(PB.schema_pn())
        else:
            doc = idl.parse_idl(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests",
                                             "golden", "idl", "baseline.thrift"))
            cdc = ThriftCodec(idl.to_schema(doc.struct("Nesting")))
        ds = cdc.dschema
        u = [int(x) for x in d["units"]]
        vc, ec, sc = u[0::3], u[1::3], u[2::3]
        out = alloc_device(ds.infos, n, vc, ds.npresence, dev, elem_caps=ec, sub_caps=sc)
        offs = torch.from_numpy(d["offs"]).to(dev) if name == "nested_offsets" else None
        st = status_tensor(dev)

        def call():
            cdc.Unmarshal(wire, n, offsets=offs, out=out, var_caps=vc, raise_on_error=False, status=st)
        if name.endswith("_encode"):   # the columns of one decode; the first Marshal is the warm-up
            call()
            w2, _ = cdc.Marshal(out)
            buf = torch.empty_like(w2)
            st2 = status_tensor(dev)

            def call():
                cdc.Marshal(out, with_offsets=False, out=buf, status=st2, check_status=False)
            calls -= 1
    elif name in ("r2_views", "r2_offsets", "r2_offsets_views"):
        cdc = ThriftCodec(S.schema_r2())
        ds = cdc.dschema
        caps = [0 if ci.kind == A.COL_FIXED else max(1, wire.numel()) for ci in ds.infos]
        out = alloc_device(ds.infos, n, caps, ds.npresence, dev, views=name != "r2_offsets")
        offs = torch.from_numpy(d["offs"]).to(dev) if name != "r2_views" else None
        st = status_tensor(dev)

        def call():
            cdc.Unmarshal(wire, n, offsets=offs, out=out, var_caps=caps, raise_on_error=False, status=st)
    else:
        raise SystemExit(f"unknown workload {name}")
    for _ in range(calls + 1):
        call()
    torch.cuda.synchronize()
    print("ok", name, calls + 1)


if __name__ == "__main__":
    if sys.argv[1] == "prep":
        prep(sys.argv[2])
    else:
        run(sys.argv[2], int(sys.argv[3]))
