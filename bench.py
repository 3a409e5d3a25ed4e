#!/usr/bin/env python3
"""Benchmark: Thrift-binary batch decode on MI355X (BASELINE.json metric).

A step = one kx_thrift_decode_batch over the whole device-resident batch (config 2: 16,777,216
flat R2 records = 8 x i64 + 2 x string[32], 167 wire bytes each, concatenated as the elements of a
list<R2>; boundaries found on the GPU). Inputs are synthetic, generated in HBM and
encoded by the GPU encoder before the timed region; the decoded columns are checked against the
generator's columns after it.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--records R] [--mode concat|offsets]
                  [--config r2|r1|r3]

N > 1: launched by torch.distributed.run, one rank per GPU, each rank decodes its own 16M-record
shard (weak scaling, no collective in the data path); value = all records / max time.
Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)

# algorithmic bytes per record: wire bytes in + decoded column bytes out
WIRE_BYTES = {"r1": 89, "r2": 167}
OUT_BYTES = {"r1": 64, "r2": 8 * 8 + 2 * (4 + 32)}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--records", type=int, default=16 * 1024 * 1024)
    ap.add_argument("--config", default="r2", choices=["r1", "r2", "r3", "pf"])
    ap.add_argument("--mode", default="concat", choices=["concat", "offsets"])
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-host", action="store_true")
    ap.add_argument("--no-concat", action="store_true", help="N>1: skip the RCCL concatenation into rank 0")
    ap.add_argument("--cpu-records", type=int, default=4 * 1024 * 1024)
    return ap.parse_args()


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    from kitex_amd import _abi as A
    from kitex_amd import schema as S
    from kitex_amd import synth
    from kitex_amd.codec import ProtobufCodec, ThriftCodec, read_status
    from kitex_amd.columns import alloc_device

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    n = args.records
    cfg = args.config
    sch = S.SCHEMAS[cfg]()
    cdc = ProtobufCodec(sch, device=local) if cfg == "pf" else ThriftCodec(sch, device=local)
    infos = cdc.dschema.infos

    # ---- synthetic shard in HBM, encoded by the GPU encoder (untimed) ----
    src = synth.TORCH_GENERATORS[cfg](n, dev, start=rank * n)
    wire, offs = cdc.Marshal(src, with_offsets=True)
    torch.cuda.synchronize()
    in_bytes = wire.numel()
    var_caps = [0 if ci.kind == A.COL_FIXED else synth_cap(src, c) for c, ci in enumerate(infos)]
    out = alloc_device(infos, n, var_caps, cdc.dschema.npresence, dev)
    offsets = offs if args.mode == "offsets" else None

    from kitex_amd.codec import status_tensor
    st_buf = status_tensor(dev)

    def step():
        return cdc.Unmarshal(wire, n, offsets=offsets, out=out, var_caps=var_caps, raise_on_error=False,
                             status=st_buf)

    for _ in range(args.warmup):
        res = step()
    torch.cuda.synchronize()
    st = read_status(res.status)
    assert st.code == 0 and st.n_records == n, f"decode failed: code={st.code} n={st.n_records}"

    # ---- timed region: K decode passes, events on the launch stream ----
    stream = torch.cuda.current_stream()
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    evs[0].record(stream)
    for k in range(args.steps):
        res = step()
        evs[k + 1].record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    wall = time.perf_counter() - t0
    per_launch_ms = [evs[k].elapsed_time(evs[k + 1]) for k in range(args.steps)]
    ev_total_s = sum(per_launch_ms) / 1e3
    t_rank = max(wall, ev_total_s)
    if world > 1:
        tt = torch.tensor([t_rank], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t_rank = float(tt.item())

    # ---- verify (size-independent property: decode(encode(x)) == x) ----
    st = read_status(res.status)
    ok = st.code == 0 and st.n_records == n and (args.mode == "offsets" or st.consumed == in_bytes)
    for c, ci in enumerate(infos):
        if ci.kind == A.COL_FIXED:
            ok &= bool(torch.equal(out.cols[c], src.cols[c]))
        else:
            ok &= bool(torch.equal(out.cols[c][0], src.cols[c][0]))
            tot = int(src.cols[c][0][-1].item()) & 0xFFFFFFFF
            ok &= bool(torch.equal(out.cols[c][1][:tot], src.cols[c][1][:tot]))
    if world > 1:
        okt = torch.tensor([1 if ok else 0], device=dev)
        dist.all_reduce(okt, op=dist.ReduceOp.MIN)
        ok = bool(okt.item())

    # ---- N > 1: concatenation of the decoded shards into rank 0 over RCCL (reported separately) ----
    concat = None
    if world > 1 and not args.no_concat:
        from kitex_amd.shard import concat_to_root
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        full = concat_to_root(out, n, infos)
        torch.cuda.synchronize()
        dist.barrier()
        tc = time.perf_counter() - t0
        shard_bytes = sum((c[0][:n + 1].numel() * 4 + int(src.cols[i][0][-1].item()) * c[1].element_size())
                          if isinstance(c, tuple) else n * c.element_size() for i, c in enumerate(out.cols))
        concat = {"ms": tc * 1e3, "bytes_to_root": shard_bytes * (world - 1),
                  "gb_s": shard_bytes * (world - 1) / tc / 1e9, "ok": full is None or full.n == n * world,
                  "note": "decoded shards -> rank 0, batched isend/irecv over RCCL (xGMI); not in value"}
        del full

    steps = args.steps
    total_records = n * world * steps
    value = total_records / t_rank
    ms_per_step = t_rank / steps * 1e3
    per_rec_in = in_bytes / n
    per_rec_out = sum(
        (ci.width if ci.kind == A.COL_FIXED else 4) for ci in infos) + sum(
        (var_caps[c] * (ci.width if ci.kind == A.COL_LIST else 1)) / n for c, ci in enumerate(infos)
        if ci.kind != A.COL_FIXED) + (8 if cdc.dschema.npresence else 0)
    avg_launch_s = sum(per_launch_ms) / len(per_launch_ms) / 1e3
    alg_bytes = (per_rec_in + per_rec_out) * n
    achieved = alg_bytes / avg_launch_s / 1e9
    gib_s = in_bytes * world * steps / t_rank / 2**30

    result = {
        "metric": ("Kitex-Protobuf decode records/s, device-resident 16M flat records (second codec path)"
                   if cfg == "pf" else "Thrift-binary decode records/s + GiB/s, device-resident 16M×96B batch"),
        "value": value,
        "unit": "records/s",
        "n_gpus": world,
        "steps": steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (splitmix64, SURVEY.md §8d), generated + GPU-encoded in HBM",
        "config": {"workload": f"{cfg}_decode_{args.mode}", "records_per_gpu": n,
                   "wire_bytes_per_record": per_rec_in, "out_bytes_per_record": per_rec_out,
                   "parallelism": f"shard{world}"},
        "gib_s": gib_s,
        "verified": ok,
        "decode_diag": {"tile_rewalks": st.diag[0], "group_rescans": st.diag[1]},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": pmc_traffic(cfg, args.mode),
                     "read_only_frac": per_rec_in * n / avg_launch_s / 1e9 / HBM_PEAK_GBS,
                     "kernel": "decode_kernel", "avg_launch_ms": avg_launch_s * 1e3},
        "cpu_baseline": None,
    }
    if concat is not None:
        result["concat"] = concat

    if rank == 0 and world == 1 and not args.no_host and cfg != "pf":
        result["host_inclusive"] = host_inclusive(cdc, wire, n, offsets, var_caps, infos, dev)
    if rank == 0 and world == 1 and not args.no_cpu:
        result["cpu_baseline"] = cpu_baseline(cfg, args.cpu_records)
        if result["cpu_baseline"].get("value"):
            result["cpu_baseline"]["gpu_speedup"] = value / result["cpu_baseline"]["value"]
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


def synth_cap(src, c):
    return int(src.cols[c][0][-1].item()) & 0xFFFFFFFF


def pmc_traffic(cfg, mode):
    """HBM bytes per launch from the committed rocprofv3 PMC summary, if one exists for this workload."""
    p = os.path.join(ROOT, "profiles", f"pmc_{cfg}_{mode}.json")
    try:
        with open(p) as fh:
            return json.load(fh).get("hbm_bytes_per_launch")
    except Exception:
        return None


def host_inclusive(cdc, wire, n, offsets, var_caps, infos, dev):
    """Pinned host -> HBM copy + decode + columns back to pinned host (the netpoll-buffer path)."""
    import torch

    from kitex_amd import _abi as A
    from kitex_amd.columns import alloc_device
    h_in = torch.empty(wire.numel(), dtype=torch.uint8, pin_memory=True)
    h_in.copy_(wire)
    d_in = torch.empty_like(wire)
    out = alloc_device(infos, n, var_caps, cdc.dschema.npresence, dev)
    h_out = [((torch.empty(c[0].numel(), dtype=c[0].dtype, pin_memory=True),
               torch.empty(c[1].numel(), dtype=c[1].dtype, pin_memory=True)) if isinstance(c, tuple)
              else torch.empty(c.numel(), dtype=c.dtype, pin_memory=True)) for c in out.cols]
    d_off = offsets
    reps = 3
    best = 1e30
    for _ in range(reps + 1):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        d_in.copy_(h_in, non_blocking=True)
        cdc.Unmarshal(d_in, n, offsets=d_off, out=out, var_caps=var_caps, raise_on_error=False)
        for ho, c in zip(h_out, out.cols):
            if isinstance(c, tuple):
                ho[0].copy_(c[0], non_blocking=True)
                ho[1].copy_(c[1], non_blocking=True)
            else:
                ho.copy_(c, non_blocking=True)
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    out_bytes = sum((c[0].numel() * c[0].element_size() + c[1].numel() * c[1].element_size())
                    if isinstance(c, tuple) else c.numel() * c.element_size() for c in out.cols)
    return {"records_per_s": n / best, "ms": best * 1e3, "h2d_bytes": wire.numel(), "d2h_bytes": out_bytes,
            "pcie_gb_s": (wire.numel() + out_bytes) / best / 1e9,
            "note": "pinned H2D + decode + D2H, serial on one stream (PCIe-bound)"}


def cpu_baseline(cfg, nrec):
    """The CPU restatement of the reference FastRead (oracle, 'port'), all host cores, offsets known."""
    try:
        import numpy as np

        from kitex_amd import schema as S
        from kitex_amd import synth
        from oracle import oracle
        oracle.build()
        threads = int(os.environ.get("OMP_NUM_THREADS") or os.cpu_count() or 1)
        threads = max(1, min(threads, 64))
        sch = S.SCHEMAS[cfg]()
        cs = synth.GENERATORS[cfg](nrec)
        pb = cfg == "pf"
        rc, wire, offs = oracle.encode(sch, cs, threads=threads, pb=pb)
        assert rc == 0
        if pb:  # strip the Batch frame headers: bare bodies with known extents (per-message proto.Unmarshal)
            bs = offs[:nrec].astype(np.int64)                       # body starts
            u = np.where(wire[bs - 2] >= 0x80, 2, 1)                 # frame length varint bytes (bodies < 16 KiB)
            fs = bs - 1 - u                                          # frame starts
            keep = np.ones(wire.size, dtype=bool)
            hdr = np.repeat(fs, 1 + u) + (np.arange(int((1 + u).sum())) - np.repeat(np.cumsum(1 + u) - (1 + u), 1 + u))
            keep[hdr] = False
            lens = np.append(fs[1:], wire.size) - bs
            wire = wire[keep]
            offs = np.zeros(nrec + 1, dtype=np.uint64)
            offs[1:] = np.cumsum(lens)
        caps = [None] * 0
        best = 1e30
        for _ in range(3):
            t0 = time.perf_counter()
            rc, out, st, _ = oracle.decode(sch, wire, nrec, offsets=offs, threads=threads, pb=pb)
            best = min(best, time.perf_counter() - t0)
            assert rc == 0
        one = min(nrec, 1 << 19)
        t0 = time.perf_counter()
        oracle.decode(sch, wire[:int(offs[one])], one, offsets=offs[:one + 1], threads=1, pb=pb)
        t1 = time.perf_counter() - t0
        cpu = ""
        try:
            with open("/proc/cpuinfo") as fh:
                cpu = next((l.split(":", 1)[1].strip() for l in fh if l.startswith("model name")), "")
        except Exception:
            pass
        del caps
        return {"value": nrec / best, "unit": "records/s", "cores": threads, "kind": "port",
                "sample": f"{nrec} {cfg} records, FastRead restatement (oracle/kx_oracle.c) with message "
                          f"offsets known, best of 3, {threads} threads",
                "gib_s": wire.size / best / 2**30, "one_thread_records_per_s": one / t1, "cpu_model": cpu}
    except Exception as e:  # the baseline must never break the GPU line
        return {"value": None, "error": repr(e)}


if __name__ == "__main__":
    main()
