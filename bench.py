#!/usr/bin/env python3
"""Benchmark: Thrift-binary batch decode on MI355X (BASELINE.json metric).

A step = one kx_thrift_decode_batch over the whole device-resident batch (config 2: 16,777,216
flat R2 records = 8 x i64 + 2 x string[32], 167 wire bytes each, concatenated as the elements of a
list<R2>; boundaries found on the GPU). Inputs are synthetic, generated in HBM and
encoded by the GPU encoder before the timed region; the decoded columns are checked against the
generator's columns after it.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--records R] [--mode concat|offsets]
                  [--config r2|r1|r3|pf|c5] [--no-extra] [--no-cpu] [--no-host]

N > 1: launched by torch.distributed.run, one rank per GPU, each rank decodes its own 16M-record
shard (weak scaling, no collective in the data path); value = all records / max time.
--config c5 (BASELINE config 5): 112M R2 + 16M R3 records in total, record-range shards over the
ranks (strong scaling); a step decodes both of a rank's batches; the decoded shards are then
concatenated into rank 0 over RCCL (reported as "concat", outside `value`).
At N = 1 the line also carries "extra": R3 decode + encode (config 3), PF decode (config 4) and R2
encode, each timed the same way. Prints ONE JSON line on rank 0.
"""
import argparse
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
C5_R2, C5_R3 = 112 << 20, 16 << 20   # config 5 record totals


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--records", type=int, default=16 * 1024 * 1024)
    ap.add_argument("--config", default="r2", choices=["r1", "r2", "r3", "pf", "c5"])
    ap.add_argument("--mode", default="concat", choices=["concat", "offsets"])
    ap.add_argument("--c5-scale", type=float, default=1.0, help="c5: fraction of the 112M + 16M records")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-host", action="store_true")
    ap.add_argument("--no-extra", action="store_true")
    ap.add_argument("--no-concat", action="store_true", help="N>1: skip the RCCL concatenation into rank 0")
    ap.add_argument("--cpu-records", type=int, default=8 * 1024 * 1024)
    ap.add_argument("--dry-run", action="store_true",
                    help="launch / rendezvous check only: no GPU call, gloo between the ranks")
    return ap.parse_args()


def launch_ranks(args) -> int:
    """--gpus N > 1 without a torch.distributed launcher around us: start N ranks (one process per GPU)
    with torch.distributed.run as a CHILD (this process has not touched the GPU, and never execs) and
    return its exit code. Every rank re-enters main() with WORLD_SIZE set."""
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__), *sys.argv[1:]]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    return subprocess.run(cmd, env=env).returncode


def dry_run(args, world, rank):
    """the launch path without the GPU: ranks meet over gloo, agree on the world size, rank 0 prints"""
    import torch
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group("gloo")
        t = torch.tensor([1], dtype=torch.int64)
        dist.all_reduce(t)
        seen = int(t.item())
        dist.destroy_process_group()
    else:
        seen = 1
    if rank == 0:
        print(json.dumps({"metric": "dry-run", "n_gpus": world, "ranks_seen": seen, "gpus_flag": args.gpus,
                          "dry_run": True}), flush=True)


def last_offset(off) -> int:
    """the last entry of an offset column (4-byte columns hold uint32 values in int32)"""
    import torch
    v = int(off[-1].item())
    return v & 0xFFFFFFFF if off.dtype == torch.int32 else v


def same_offsets(a, b) -> bool:
    import torch
    u = (lambda t: t.to(torch.int64) & 0xFFFFFFFF if t.dtype == torch.int32 else t.to(torch.int64))
    return bool(torch.equal(u(a), u(b)))


class Batch:
    """One same-schema batch resident in HBM: source columns, GPU-encoded wire, decode outputs."""

    def __init__(self, cfg, n, dev, start, mode, local, views=False):
        import torch

        from kitex_amd import _abi as A
        from kitex_amd import schema as S
        from kitex_amd import synth
        from kitex_amd.codec import ProtobufCodec, ThriftCodec, status_tensor
        from kitex_amd.columns import alloc_device
        self.cfg, self.n, self.mode, self.views = cfg, n, mode, views
        sch = S.SCHEMAS[cfg]()
        self.cdc = ProtobufCodec(sch, device=local) if cfg == "pf" else ThriftCodec(sch, device=local)
        self.infos = infos = self.cdc.dschema.infos
        self.src = synth.TORCH_GENERATORS[cfg](n, dev, start=start)
        self.wire, self.offs = self.cdc.Marshal(self.src, with_offsets=True)
        torch.cuda.synchronize()
        self.in_bytes = self.wire.numel()
        self.var_caps = [0 if ci.kind == A.COL_FIXED else last_offset(self.src.cols[c][0])
                         for c, ci in enumerate(infos)]
        wide = any(v >= (1 << 32) for v in self.var_caps)
        self.out = alloc_device(infos, n, self.var_caps, self.cdc.dschema.npresence, dev, wide=wide, views=views)
        self.offsets = self.offs if mode == "offsets" else None
        self.st = status_tensor(dev)

    def step(self, stream=None):
        return self.cdc.Unmarshal(self.wire, self.n, offsets=self.offsets, out=self.out, var_caps=self.var_caps,
                                  raise_on_error=False, status=self.st, stream=stream)

    def status(self):
        from kitex_amd.codec import read_status
        return read_status(self.st)

    def verify(self) -> bool:
        import torch

        from kitex_amd import _abi as A
        st = self.status()
        ok = st.code == 0 and st.n_records == self.n and (self.mode == "offsets" or st.consumed == self.in_bytes)
        for c, ci in enumerate(self.infos):
            if ci.kind == A.COL_FIXED:
                ok &= bool(torch.equal(self.out.cols[c], self.src.cols[c]))
            elif self.views and ci.kind == A.COL_BYTES:
                ok &= self._verify_views(c)
            else:
                ok &= same_offsets(self.out.cols[c][0], self.src.cols[c][0])
                tot = self.var_caps[c]
                ok &= bool(torch.equal(self.out.cols[c][1][:tot], self.src.cols[c][1][:tot]))
        if self.src.presence is not None:
            ok &= bool(torch.equal(self.out.presence[:self.n], self.src.presence[:self.n]))
        return ok

    def _verify_views(self, c, limit=1 << 20) -> bool:
        """view pairs of the first `limit` records name exactly the source strings"""
        import torch
        k = min(self.n, limit)
        pairs = self.out.cols[c].pairs[:k].to(torch.int64) & 0xFFFFFFFF
        so = self.src.cols[c][0][:k + 1].to(torch.int64) & 0xFFFFFFFF
        lens = so[1:] - so[:-1]
        if not torch.equal(pairs[:, 1], lens):
            return False
        idx = torch.repeat_interleave(pairs[:, 0] - so[:-1], lens) + torch.arange(int(so[-1] - so[0]),
                                                                                    device=pairs.device) + so[0]
        return bool(torch.equal(self.wire[idx], self.src.cols[c][1][int(so[0]):int(so[-1])]))

    def out_bytes_per_record(self) -> float:
        from kitex_amd import _abi as A
        n = self.n
        if self.views:   # zero-copy views: (offset, length) per string, no arena (SURVEY.md §8d, 247 B for R2)
            return (sum((ci.width if ci.kind == A.COL_FIXED else 8 if ci.kind == A.COL_BYTES else 4)
                        for ci in self.infos)
                    + sum(self.var_caps[c] * (ci.width if ci.kind == A.COL_LIST else 1) / n
                          for c, ci in enumerate(self.infos) if ci.kind not in (A.COL_FIXED, A.COL_BYTES))
                    + (8 if self.cdc.dschema.npresence else 0))
        return (sum((ci.width if ci.kind == A.COL_FIXED else 4) for ci in self.infos)
                + sum(self.var_caps[c] * (ci.width if ci.kind == A.COL_LIST else 1) / n
                      for c, ci in enumerate(self.infos) if ci.kind != A.COL_FIXED)
                + (8 if self.cdc.dschema.npresence else 0))


def time_steps(fn, steps, warmup, world, dev):
    """W untimed calls, then K calls bracketed by barrier + synchronize; events on the launch stream
    give the per-call durations. Returns (max-over-ranks seconds, per-call ms list)."""
    import torch
    import torch.distributed as dist
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream()
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    evs[0].record(stream)
    for k in range(steps):
        fn()
        evs[k + 1].record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    wall = time.perf_counter() - t0
    per = [evs[k].elapsed_time(evs[k + 1]) for k in range(steps)]
    t = max(wall, sum(per) / 1e3)
    if world > 1:
        tt = torch.tensor([t], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t = float(tt.item())
    return t, per


def lib_sha256() -> str:
    from kitex_amd import _lib
    h = hashlib.sha256()
    with open(_lib.LIB_PATH, "rb") as fh:
        for blk in iter(lambda: fh.read(1 << 20), b""):
            h.update(blk)
    return h.hexdigest()


def pmc_traffic(workload):
    """HBM bytes per call from the committed rocprofv3 PMC summary of this workload, only when that
    profile was taken with the library being timed (same sha256); else None with the reason."""
    p = os.path.join(ROOT, "profiles", f"pmc_{workload}.json")
    try:
        with open(p) as fh:
            prof = json.load(fh)
    except Exception:
        return None, "no profile"
    sha = lib_sha256()
    if prof.get("lib_sha256") != sha:
        return None, f"profiles/pmc_{workload}.json was taken with another build of libkxcodec.so"
    return prof.get("hbm_bytes_per_launch"), f"profiles/pmc_{workload}.json (lib sha256 {sha[:16]})"


def roofline(alg_bytes, avg_launch_s, kernel, traffic=None, note=None):
    achieved = alg_bytes / avg_launch_s / 1e9
    r = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
         "traffic": traffic, "kernel": kernel, "avg_launch_ms": avg_launch_s * 1e3}
    if note:
        r["traffic_source"] = note
    return r


_T0 = time.perf_counter()


def note(msg: str):
    """progress on stderr (the JSON line alone goes to stdout): long runs stay visibly alive"""
    print(f"[bench {time.perf_counter() - _T0:7.1f}s] {msg}", file=sys.stderr, flush=True)


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: launch one rank per GPU")
    if args.dry_run:
        dry_run(args, world, rank)
        return
    import torch
    import torch.distributed as dist
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    if args.config == "c5":
        result = run_c5(args, world, rank, dev, local)
    else:
        result = run_single(args, world, rank, dev, local)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


def run_single(args, world, rank, dev, local):
    import torch
    import torch.distributed as dist
    cfg, n = args.config, args.records
    b = Batch(cfg, n, dev, rank * n, args.mode, local)
    b.step()
    torch.cuda.synchronize()
    st = b.status()
    assert st.code == 0 and st.n_records == n, f"decode failed: code={st.code} n={st.n_records}"

    note(f"{cfg} {args.mode}: {n} records ready, timing")
    t_rank, per = time_steps(b.step, args.steps, args.warmup, world, dev)
    note(f"headline: {t_rank / args.steps * 1e3:.3f} ms per step")
    st = b.status()
    ok = b.verify()
    if world > 1:
        okt = torch.tensor([1 if ok else 0], device=dev)
        dist.all_reduce(okt, op=dist.ReduceOp.MIN)
        ok = bool(okt.item())

    concat = None
    if world > 1 and not args.no_concat:
        concat = concat_shards([b], world, rank, dev)

    steps = args.steps
    value = n * world * steps / t_rank
    per_rec_in = b.in_bytes / n
    per_rec_out = b.out_bytes_per_record()
    avg_launch_s = sum(per) / len(per) / 1e3
    traffic, tnote = pmc_traffic(f"{cfg}_{args.mode}")
    rl = roofline((per_rec_in + per_rec_out) * n, avg_launch_s, "decode (index+group+chain+emit)", traffic, tnote)
    rl["read_only_frac"] = per_rec_in * n / avg_launch_s / 1e9 / HBM_PEAK_GBS
    result = {
        "metric": ("Kitex-Protobuf decode records/s, device-resident 16M flat records (second codec path)"
                   if cfg == "pf" else "Thrift-binary decode records/s + GiB/s, device-resident 16M×96B batch"),
        "value": value,
        "unit": "records/s",
        "n_gpus": world,
        "steps": steps,
        "warmup": args.warmup,
        "ms_per_step": t_rank / steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (splitmix64, SURVEY.md §8d), generated + GPU-encoded in HBM",
        "config": {"workload": f"{cfg}_decode_{args.mode}", "records_per_gpu": n,
                   "wire_bytes_per_record": per_rec_in, "out_bytes_per_record": per_rec_out,
                   "parallelism": f"shard{world}"},
        "gib_s": b.in_bytes * world * steps / t_rank / 2**30,
        "verified": ok,
        "decode_diag": {"tile_rewalks": st.diag[0], "group_rescans": st.diag[1]},
        "roofline": rl,
        "cpu_baseline": None,
        "lib_sha256": lib_sha256()[:16],
    }
    if concat is not None:
        result["concat"] = concat
    if rank == 0 and world == 1 and not args.no_host and cfg != "pf":
        note("host-inclusive paths")
        result["host_inclusive"] = host_inclusive(b, dev)
        for shape, cnt in (("mockreq", 4 << 20), ("nesting", 1 << 20)):
            note(f"host-inclusive {shape}")
            try:
                result["host_inclusive"][shape] = host_inclusive_shape(shape, cnt)
            except Exception as e:   # never break the bench line
                result["host_inclusive"][shape] = {"error": repr(e)}
    if world == 1 and not args.no_extra:
        result["extra"] = extras(args, b if cfg == "r2" else None, dev, local)
    if rank == 0 and world == 1 and not args.no_cpu:
        note("cpu baseline")
        result["cpu_baseline"] = cpu_baseline(cfg, args.cpu_records)
        if result["cpu_baseline"].get("value"):
            result["cpu_baseline"]["gpu_speedup"] = value / result["cpu_baseline"]["value"]
    return result


def run_c5(args, world, rank, dev, local):
    """BASELINE config 5: 112M R2 + 16M R3 records sharded by record range over the ranks."""
    import torch
    import torch.distributed as dist

    from kitex_amd.shard import shard_range
    totals = {"r2": int(C5_R2 * args.c5_scale), "r3": int(C5_R3 * args.c5_scale)}
    batches, split = [], {}
    for cfg, tot in totals.items():
        s0, cnt = shard_range(tot, world, rank)
        b = Batch(cfg, cnt, dev, s0, args.mode, local)
        split[cfg] = split_and_scatter(b, cfg, tot, world, rank, dev)
        batches.append(b)
    torch.cuda.synchronize()

    def step():
        for b in batches:
            b.step()

    t_rank, per = time_steps(step, args.steps, args.warmup, world, dev)
    ok = all(b.verify() for b in batches)
    if world > 1:
        okt = torch.tensor([1 if ok else 0], device=dev)
        dist.all_reduce(okt, op=dist.ReduceOp.MIN)
        ok = bool(okt.item())
    concat = concat_shards(batches, world, rank, dev) if world > 1 and not args.no_concat else None
    steps = args.steps
    total = sum(totals.values())
    value = total * steps / t_rank
    avg_launch_s = sum(per) / len(per) / 1e3
    alg = sum((b.in_bytes + b.out_bytes_per_record() * b.n) for b in batches)
    if world > 1:
        t = torch.tensor([alg], dtype=torch.float64, device=dev)
        dist.all_reduce(t)
        alg = float(t.item()) / world   # per-rank average: the roofline is per GPU
    result = {
        "metric": "Thrift-binary decode records/s, config 5: 112M R2 + 16M R3 sharded over the GPUs",
        "value": value, "unit": "records/s", "n_gpus": world, "steps": steps, "warmup": args.warmup,
        "ms_per_step": t_rank / steps * 1e3, "higher_is_better": True, "scaling": "strong",
        "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (splitmix64, SURVEY.md §8d), generated + GPU-encoded in HBM",
        "config": {"workload": f"c5_decode_{args.mode}", "records_total": totals,
                   "records_per_gpu": {k: shard_range(v, world, rank)[1] for k, v in totals.items()},
                   "parallelism": f"shard{world}"},
        "verified": ok,
        "roofline": roofline(alg, avg_launch_s, "decode R2 shard + decode R3 shard"),
        "cpu_baseline": None,
        "lib_sha256": lib_sha256()[:16],
    }
    result["split"] = split
    if concat is not None:
        result["concat"] = concat
    if rank == 0 and world == 1 and not args.no_cpu:
        result["cpu_baseline"] = cpu_baseline("r2", args.cpu_records)
    return result


def split_and_scatter(b, cfg, tot, world, rank, dev):
    """Config 5's input as it arrives: ONE concatenated batch of `tot` records per schema on rank 0. Rank 0
    finds the world + 1 split points on the device (kx_thrift_split_points: the index and chain passes of a
    decode, no emit; SURVEY.md §8e pass A), then sends shard k's bytes to rank k (RCCL point-to-point). Each
    rank checks the bytes it got against its own encoding of the same record range (the generator is
    per-record) and decodes them in the timed steps. Split-pass time and scatter time are reported, not
    in `value`."""
    import torch
    import torch.distributed as dist

    from kitex_amd import synth
    from kitex_amd.shard import shard_range
    pts = torch.zeros(world + 1, dtype=torch.int64, device=dev)
    info = {}
    full = None
    if rank == 0:
        cdc = b.cdc
        src = synth.TORCH_GENERATORS[cfg](tot, dev, start=0)
        full = cdc.Marshal(src)[0]
        del src
        torch.cuda.synchronize()
        cdc.SplitPoints(full, tot, world)              # warm
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        reps = 5
        ev[0].record()
        for _ in range(reps):
            pts = cdc.SplitPoints(full, tot, world)
        ev[1].record()
        torch.cuda.synchronize()
        info = {"split_points_ms": ev[0].elapsed_time(ev[1]) / reps, "batch_bytes": int(full.numel())}
    if world > 1:
        dist.broadcast(pts, 0)
    p = [int(x) for x in pts.tolist()]
    ok = all(p[k + 1] - p[k] >= 0 for k in range(world)) and p[0] == 0
    s0, cnt = shard_range(tot, world, rank)
    ok &= s0 == (rank * tot) // world and cnt == ((rank + 1) * tot) // world - s0
    t0 = time.perf_counter()
    if world > 1:
        if rank == 0:
            ops = [dist.P2POp(dist.isend, full[p[k]:p[k + 1]].contiguous(), k) for k in range(1, world)]
            mine = full[p[0]:p[1]]
        else:
            mine = torch.empty(p[rank + 1] - p[rank], dtype=torch.uint8, device=dev)
            ops = [dist.P2POp(dist.irecv, mine, 0)]
        for r in dist.batch_isend_irecv(ops):
            r.wait()
        torch.cuda.synchronize()
        dist.barrier()
    else:
        mine = full[p[0]:p[1]]
    ok &= mine.numel() == b.wire.numel() and bool(torch.equal(mine, b.wire))
    if world > 1:
        okt = torch.tensor([1 if ok else 0], device=dev)
        dist.all_reduce(okt, op=dist.ReduceOp.MIN)
        ok = bool(okt.item())
    b.wire = mine.clone() if rank == 0 else mine      # the timed decode reads the shard it was sent
    b.in_bytes = b.wire.numel()
    del full
    info.update({"parts": world, "shard_equals_local_encoding": ok,
                 "scatter_ms": (time.perf_counter() - t0) * 1e3 if world > 1 else 0.0})
    return info


def concat_shards(batches, world, rank, dev):
    """decoded shards -> rank 0 (RCCL point-to-point over xGMI), checked there against the shards'
    generator (same splitmix64 streams); outside `value`"""
    import torch
    import torch.distributed as dist

    from kitex_amd import synth
    from kitex_amd.shard import concat_batches_to_root
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    outs = concat_batches_to_root([(b.out, b.n, b.infos, b.in_bytes) for b in batches])
    torch.cuda.synchronize()
    dist.barrier()
    tc = time.perf_counter() - t0
    moved = sum(sum((c[0][:b.n + 1].numel() * c[0].element_size() + b.var_caps[i] * c[1].element_size())
                    if isinstance(c, tuple) else b.n * c.element_size() for i, c in enumerate(b.out.cols))
                for b in batches)
    t = torch.tensor([moved], dtype=torch.float64, device=dev)
    dist.all_reduce(t)
    to_root = float(t.item()) - moved if rank == 0 else 0.0
    ok = True
    if rank == 0:   # head and tail (or all) of every concatenated batch against the generator
        for b, full in zip(batches, outs):
            N = full.n
            k = min(N, 1 << 20)
            for s0 in sorted({0, N - k}):
                ref = synth.TORCH_GENERATORS[b.cfg](k, dev, start=s0)
                for c in range(len(b.infos)):
                    if isinstance(ref.cols[c], tuple):
                        ro, rd = ref.cols[c]
                        fo, fd = full.cols[c]
                        ro = ro.to(torch.int64) & 0xFFFFFFFF if ro.dtype == torch.int32 else ro
                        base = int(fo[s0].item())
                        ok &= bool(torch.equal(fo[s0:s0 + k + 1] - base, ro))
                        ok &= bool(torch.equal(fd[base:base + int(ro[-1].item())], rd[:int(ro[-1].item())]))
                    else:
                        ok &= bool(torch.equal(full.cols[c][s0:s0 + k], ref.cols[c]))
                del ref
        del outs
    return {"ms": tc * 1e3, "bytes_to_root": to_root, "gb_s": to_root / tc / 1e9 if rank == 0 else None,
            "checked_against_generator": ok,
            "note": "decoded shards -> rank 0, batched isend/irecv over RCCL (xGMI), int64 offsets; not in value"}


def extras(args, r2, dev, local):
    """The other BASELINE configs, timed the same way on this GPU: R3 decode + encode (config 3, 4M),
    PF decode (config 4, 16M), R2 encode (16M)."""
    import torch

    from kitex_amd.codec import status_tensor
    steps, warm = max(3, min(args.steps, 10)), 2
    out = {}

    def encode_entry(b):
        buf = torch.empty_like(b.wire)
        st = status_tensor(dev)

        def enc():  # fastMarshal: BLength (the size pass inside the call) + FastWriteNocopy
            b.cdc.Marshal(b.src, with_offsets=False, out=buf, status=st, check_status=False)
        t, per = time_steps(enc, steps, warm, 1, dev)
        ok = bool(torch.equal(buf, b.wire))
        avg = sum(per) / len(per) / 1e3
        alg = b.out_bytes_per_record() * b.n + b.in_bytes      # columns in + wire out
        traffic, tnote = pmc_traffic(f"{b.cfg}_encode")
        return {"records_per_s": b.n * steps / t, "ms_per_step": t / steps * 1e3, "bit_exact": ok,
                "roofline": roofline(alg, avg, "encode (size pass + scan + write pass)", traffic, tnote)}

    def decode_entry(b):
        t, per = time_steps(b.step, steps, warm, 1, dev)
        avg = sum(per) / len(per) / 1e3
        ok = b.verify()
        st = b.status()
        views = getattr(b, "views", False)
        traffic, tnote = pmc_traffic(f"{b.cfg}_{b.mode}") if not views else \
            pmc_traffic(f"{b.cfg}_views") if b.mode == "concat" else pmc_traffic(f"{b.cfg}_offsets_views")
        return {"records_per_s": b.n * steps / t, "ms_per_step": t / steps * 1e3, "verified": ok,
                "decode_diag": {"tile_rewalks": st.diag[0], "group_rescans": st.diag[1]},
                "roofline": roofline(b.in_bytes + b.out_bytes_per_record() * b.n, avg, "decode", traffic, tnote)}

    def crc_entry(b):
        """CRC32C (crcPayloadValidator.Generate, validate.go:187-217) of every encoded R2 record"""
        from kitex_amd.codec import CRC32PayloadValidator
        v = CRC32PayloadValidator(device=local)
        res = {}
        t, per = time_steps(lambda: res.__setitem__("crc", v.Generate(b.wire, b.offs)), steps, warm, 1, dev)
        avg = sum(per) / len(per) / 1e3
        crc = res["crc"]
        pick = [0, 1, b.n // 3, b.n // 2, b.n - 1]
        offs = b.offs.cpu()
        ok = all(crc32c_py(bytes(b.wire[int(offs[i]):int(offs[i + 1])].cpu().numpy())) == int(crc[i]) for i in pick)
        alg = b.in_bytes + 12 * b.n  # payload bytes + u64 offsets in + u32 CRC out
        traffic, tnote = pmc_traffic("r2_crc")
        return {"ranges": b.n, "ranges_per_s": b.n * steps / t, "ms_per_step": t / steps * 1e3, "sample_ok": ok,
                "roofline": roofline(alg, avg, "crc32c", traffic, tnote)}

    def nested_entry(n=1 << 20, k=4096, pb=False):
        """config-3-style nested records on the nested walker (lane = record), decode + encode; k distinct
        host-written records tiled to n on the device. Thrift: baseline.thrift's Nesting (NestingMethod's
        request: list<Simple>, map<string,Simple>, map<i32,i64>, list<string>, ...; tests/golden/idl/
        baseline.thrift). pb: the nested Kitex-Protobuf test message PN (tests/pbn_cases.py: zig-zag, fixed,
        packed repeated, nested and repeated messages, maps with message values), Batch-framed. Beside it the
        oracle's nested FastRead / proto.Unmarshal on the host's threads (nested_cpu_baseline)."""
        import numpy as np

        from kitex_amd import idl, synth
        from kitex_amd.codec import ProtobufCodec, ThriftCodec, read_status
        from kitex_amd.columns import alloc_device
        if pb:
            from tests import pbn_cases as PB
            sch = PB.schema_pn()
            cdc = ProtobufCodec(sch, device=local)
            _, bodies_np, boffs = PB.batch(k, seed=7, name="PN")
            lens = np.diff(boffs).astype(np.int64)
            framed = [b"\x0a" + PB.uvarint(int(x)) for x in lens]
            recs = [framed[i] + bodies_np[int(boffs[i]):int(boffs[i + 1])].tobytes() for i in range(k)]
            cpu_recs = [bodies_np[int(boffs[i]):int(boffs[i + 1])].tobytes() for i in range(k)]   # bare bodies
        else:
            doc = idl.parse_idl(os.path.join(os.path.dirname(os.path.abspath(__file__)), "tests", "golden", "idl",
                                             "baseline.thrift"))
            sch = idl.to_schema(doc.struct("Nesting"))
            cdc = ThriftCodec(sch, device=local)
            recs = synth.thrift_records(sch, k, seed=7)
            cpu_recs = recs
        ds = cdc.dschema
        note(f"  nested {'pb' if pb else 'thrift'}: {k} records generated")
        one = np.frombuffer(b"".join(recs), dtype=np.uint8).copy()
        wire = torch.from_numpy(one).to(dev).repeat(n // k)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record()
        units = cdc.DecodeSizes(wire, n)
        ev[1].record()
        torch.cuda.synchronize()
        sizes_ms = ev[0].elapsed_time(ev[1])
        vc, ec, sc = units[0::3], units[1::3], units[2::3]
        outc = alloc_device(ds.infos, n, vc, ds.npresence, dev, elem_caps=ec, sub_caps=sc)
        st = status_tensor(dev)

        def dec():
            cdc.Unmarshal(wire, n, out=outc, var_caps=vc, raise_on_error=False, status=st)
        t, per = time_steps(dec, steps, warm, 1, dev)
        note(f"  nested decode timed: {t / steps * 1e3:.2f} ms")
        s = read_status(st)
        ok = s.code == 0 and s.n_records == n and s.consumed == wire.numel()

        def tensors(cs):
            for c in cs.cols:
                yield from (c if isinstance(c, tuple) else (c,))
            if cs.presence is not None:
                yield cs.presence
        out_bytes = sum(x.numel() * x.element_size() for x in tensors(outc))
        avg = sum(per) / len(per) / 1e3
        res = {"records": n, "distinct_records": k, "wire_bytes_per_record": wire.numel() / n,
               "schema": "PN (tests/pbn_cases.py), Batch-framed" if pb else "Nesting (baseline.thrift)",
               "decode": {"records_per_s": n * steps / t, "ms_per_step": t / steps * 1e3, "verified": ok,
                          "mode": "concatenated (skip pass + measure + write)", "sizes_pass_ms": sizes_ms,
                          "roofline": roofline(wire.numel() + out_bytes, avg, "nested decode (measure + write)",
                                               *pmc_traffic("pb_nested" if pb else "nested_concat"))}}
        if not pb:
            # with message lengths known (dataLen, codec_fast.go:60-71): measure + write only, the form the CPU
            # baseline below runs (it is given every record's extent)
            offs = cdc.Skip(wire, n)
            st3 = status_tensor(dev)

            def dec_off():
                cdc.Unmarshal(wire, n, offsets=offs, out=outc, var_caps=vc, raise_on_error=False, status=st3)
            t3, per3 = time_steps(dec_off, steps, warm, 1, dev)
            s3 = read_status(st3)
            res["decode_offsets"] = {"records_per_s": n * steps / t3, "ms_per_step": t3 / steps * 1e3,
                                     "verified": s3.code == 0 and s3.n_records == n,
                                     "roofline": roofline(wire.numel() + out_bytes + 8 * (n + 1),
                                                          sum(per3) / len(per3) / 1e3, "nested decode, offsets known",
                                                          *pmc_traffic("nested_offsets"))}
            note(f"  nested decode with offsets timed: {t3 / steps * 1e3:.2f} ms")
        w2, _ = cdc.Marshal(outc)
        note("  nested encode: first Marshal done")
        buf = torch.empty_like(w2)
        st2 = status_tensor(dev)

        def enc():
            cdc.Marshal(outc, with_offsets=False, out=buf, status=st2, check_status=False)
        t, per = time_steps(enc, steps, warm, 1, dev)
        note(f"  nested encode timed: {t / steps * 1e3:.2f} ms")
        avg = sum(per) / len(per) / 1e3
        back = cdc.Unmarshal(buf, n, raise_on_error=False)
        torch.cuda.synchronize()
        note("  nested encode: round-trip decode done")
        eq = all(bool(torch.equal(a, b)) for a, b in zip(tensors(outc), tensors(back.columns)))
        res["encode"] = {"records_per_s": n * steps / t, "ms_per_step": t / steps * 1e3,
                         "round_trip_equal": eq and bool(torch.equal(buf, w2)),
                         "roofline": roofline(out_bytes + buf.numel(), avg, "nested encode (size + write)",
                                              *pmc_traffic("pb_nested_encode" if pb else "nested_encode"))}
        note("  nested round trip compared; cpu baseline")
        if not args.no_cpu:
            cb = nested_cpu_baseline(sch, cpu_recs, n, pb)
            note("  nested cpu baseline done")
            if cb.get("value"):
                cb["gpu_speedup"] = res["decode"]["records_per_s"] / cb["value"]
                if "decode_offsets" in res:   # like for like: both given every record's extent
                    cb["gpu_speedup_offsets"] = res["decode_offsets"]["records_per_s"] / cb["value"]
            res["cpu_baseline"] = cb
        return res

    def frames_entry(n=16 << 20):
        """kx_thrift_decode_frames over a socket buffer of n TTHeader frames (R1 request messages) whose
        str-info carries "crc32c" (default_codec.go:205-209, validate.go:183-217), CRC32Check off and on.
        With the check fused into the frame scan's emit pass the payloads are not read a second time."""
        from kitex_amd import schema as S
        from kitex_amd import synth
        from kitex_amd.codec import CRC32PayloadValidator, ThriftCodec
        cdc = ThriftCodec(S.schema_r1(), device=local)
        src = synth.TORCH_GENERATORS["r1"](n, dev)
        msgs, moffs = cdc.MarshalMessages(src, "Echo", torch.zeros(n, dtype=torch.int32, device=dev))
        M = msgs.numel() // n
        assert M * n == msgs.numel()
        crc = CRC32PayloadValidator(local).Generate(msgs, moffs)
        # TTHeader: length, magic 0x1000 + flags, seqid, header size / 4; protocol 0 (binary), no transforms,
        # one string KV "crc32c" -> 8 lowercase hex digits, zero padding to a multiple of 4
        info = bytes([0, 0, 1, 0, 1, 0, 6]) + b"crc32c" + bytes([0, 8]) + b"0" * 8
        info += bytes(-len(info) % 4)
        H = 14 + len(info)
        hdr = (H + M - 4).to_bytes(4, "big") + bytes([0x10, 0, 0, 0]) + bytes(4) + (len(info) // 4).to_bytes(2, "big")
        tmpl = torch.tensor(list(hdr + info), dtype=torch.uint8, device=dev)
        fr = torch.empty((n, H + M), dtype=torch.uint8, device=dev)
        fr[:, :H] = tmpl
        nib = (crc[:, None] >> torch.arange(28, -4, -4, device=dev)) & 0xF
        fr[:, H - len(info) + 15:H - len(info) + 23] = torch.where(nib < 10, nib + 48, nib + 87).to(torch.uint8)
        fr[:, H:] = msgs.view(n, M)
        wire = fr.view(-1)
        del fr, msgs, nib
        res = {"frames": n, "frame_bytes": H + M}
        for chk in (False, True):
            last = {}

            def dec():
                last["r"] = cdc.UnmarshalFrames(wire, n, raise_on_error=False, crc32_check=chk)
            t, per = time_steps(dec, steps, warm, 1, dev)
            r = last["r"]
            s = r.read_status()
            ok = s.code == 0 and s.n_records == n and bool(torch.equal(r.columns.cols[0], src.cols[0]))
            res["crc32_check_on" if chk else "crc32_check_off"] = {
                "ms_per_step": t / steps * 1e3, "frames_per_s": n * steps / t, "verified": ok,
                "roofline": roofline(wire.numel() + 8 * 8 * n, sum(per) / len(per) / 1e3,
                                     "frame scan + message decode" + (" + fused CRC32C check" if chk else ""),
                                     *pmc_traffic("frames_on" if chk else "frames_off"))}
        res["check_overhead"] = res["crc32_check_on"]["ms_per_step"] / res["crc32_check_off"]["ms_per_step"] - 1
        bad = wire.clone()
        bad[(n // 2) * (H + M) + H + M - 3] ^= 1   # one payload byte of frame n/2
        rb = cdc.UnmarshalFrames(bad, n, raise_on_error=False, crc32_check=True)
        sb = rb.read_status()
        res["tamper_detected"] = sb.code == 11 and sb.record == n // 2
        return res

    try:
        note("extra: frames")
        out["frames_crc32c"] = frames_entry()
        torch.cuda.empty_cache()
    except Exception as e:
        out["frames_crc32c"] = {"error": repr(e)}
    try:
        note("extra: nested")
        out["nested_decode_encode"] = nested_entry()
        torch.cuda.empty_cache()
    except Exception as e:
        out["nested_decode_encode"] = {"error": repr(e)}
    try:
        note("extra: nested Kitex-Protobuf")
        out["pb_nested"] = nested_entry(pb=True)
        torch.cuda.empty_cache()
    except Exception as e:
        out["pb_nested"] = {"error": repr(e)}
    try:
        if r2 is not None:
            note("extra: r2 encode, crc, views, offsets")
            out["r2_encode"] = {"records": r2.n, **encode_entry(r2)}
            out["crc32c_generate"] = crc_entry(r2)
            bv = Batch("r2", r2.n, dev, 0, "concat", local, views=True)
            e = decode_entry(bv)
            e["roofline"]["read_only_frac"] = bv.in_bytes / (e["roofline"]["avg_launch_ms"] / 1e3) / 1e9 / HBM_PEAK_GBS
            out["r2_decode_views"] = {"records": bv.n, "out_bytes_per_record": bv.out_bytes_per_record(), **e}
            del bv
            torch.cuda.empty_cache()
            # known message lengths (fastUnmarshal with dataLen, codec_fast.go:60-71): the u64 offsets array
            # is read too, so it counts in the algorithmic bytes (8 B / record)
            bo = Batch("r2", r2.n, dev, 0, "offsets", local)
            e = decode_entry(bo)
            avg = e["roofline"]["avg_launch_ms"] / 1e3
            e["roofline"] = roofline(bo.in_bytes + 8 * (bo.n + 1) + bo.out_bytes_per_record() * bo.n, avg,
                                     "decode (known offsets)", *pmc_traffic("r2_offsets"))
            out["r2_decode_offsets"] = {"records": bo.n, **e}
            del bo
            torch.cuda.empty_cache()
            # known offsets + string views: no arena to lay out, the emit pass runs alone
            bov = Batch("r2", r2.n, dev, 0, "offsets", local, views=True)
            e = decode_entry(bov)
            avg = e["roofline"]["avg_launch_ms"] / 1e3
            e["roofline"] = roofline(bov.in_bytes + 8 * (bov.n + 1) + bov.out_bytes_per_record() * bov.n, avg,
                                     "decode (known offsets, views: emit pass alone)", *pmc_traffic("r2_offsets_views"))
            e["roofline"]["read_only_frac"] = bov.in_bytes / avg / 1e9 / HBM_PEAK_GBS
            out["r2_decode_offsets_views"] = {"records": bov.n, "out_bytes_per_record": bov.out_bytes_per_record(),
                                              **e}
            del bov
            torch.cuda.empty_cache()
        note("extra: r3, pf")
        b3 = Batch("r3", 4 << 20, dev, 0, "concat", local)
        out["r3_decode"] = {"records": b3.n, "wire_bytes_per_record": b3.in_bytes / b3.n, **decode_entry(b3)}
        out["r3_encode"] = {"records": b3.n, **encode_entry(b3)}
        del b3
        torch.cuda.empty_cache()
        bp = Batch("pf", 16 << 20, dev, 0, "concat", local)
        out["pf_decode"] = {"records": bp.n, "wire_bytes_per_record": bp.in_bytes / bp.n, **decode_entry(bp)}
        del bp
        torch.cuda.empty_cache()
    except Exception as e:  # the extras must never break the headline line
        out["error"] = repr(e)
    return out


def cpu_decode_pool(sch, wire, offs, n, pb, threads, runs=5):
    """The oracle's FastRead / proto.Unmarshal restatement (oracle/kx_oracle.c, kx_oracle_nested.c) over n
    records with message offsets known, on a persistent pool of `threads` host threads: one record range
    per thread, each decoded by the single-threaded restatement into its own columns, allocated once, sized
    exactly from the range's wire bytes and pre-faulted (written once) before any timed run, so a run
    times decode alone (no thread start, no first-touch page faults). One untimed warm-up run, then `runs`
    timed runs. Returns (per-run seconds, all records decoded without error)."""
    import ctypes as C
    from concurrent.futures import ThreadPoolExecutor

    import numpy as np

    from kitex_amd import _abi as A
    from kitex_amd.columns import alloc_host, to_kx_columns
    from oracle import oracle
    oracle.build()
    L = oracle.lib()
    rc, infos, npres = oracle.flatten(sch)
    tab, ns = sch.struct_table()
    fn = L.kxo_pb_decode if pb else L.kxo_thrift_decode
    jobs = []
    for t in range(threads):
        a, b = n * t // threads, n * (t + 1) // threads
        if a == b:
            continue
        base = int(offs[a])
        so = (offs[a:b + 1] - offs[a]).astype(np.uint64)
        nb = int(offs[b]) - base
        caps = [0 if ci.kind == A.COL_FIXED else max(1, nb) for ci in infos]
        out = alloc_host(infos, b - a, caps, npres, elem_caps=caps, sub_caps=caps)
        for c in out.cols:   # pre-fault every page the decode may write
            for x in (c if isinstance(c, tuple) else (c,)):
                x.fill(1)
        if out.presence is not None:
            out.presence.fill(1)
        kc = to_kx_columns(out, infos, caps)
        jobs.append((wire.ctypes.data + base, nb, so, b - a, kc, A.Status(), np.ones(b - a, dtype=np.uint8), out))

    def run(j):
        d, nb, so, m, kc, st, rs, _ = j
        return fn(tab, ns, d, nb, so.ctypes.data, m, C.byref(kc), rs.ctypes.data, C.byref(st)), st.code
    ts = []
    ok = True
    with ThreadPoolExecutor(max_workers=threads) as ex:
        list(ex.map(run, jobs))   # warm-up (pool threads started, caches and TLBs warm)
        for _ in range(runs):
            t0 = time.perf_counter()
            got = list(ex.map(run, jobs))
            ts.append(time.perf_counter() - t0)
            ok &= all(r == 0 and c == 0 for r, c in got)
    return ts, ok


def spread(n, ts):
    """records/s statistics of per-run times"""
    rates = sorted(n / t for t in ts)
    return {"median": rates[len(rates) // 2], "min": rates[0], "max": rates[-1], "runs": len(rates),
            "spread": (rates[-1] - rates[0]) / rates[len(rates) // 2]}


def nested_cpu_baseline(sch, recs, n, pb):
    """The oracle's nested decode (oracle/kx_oracle_nested.c: FastRead / proto.Unmarshal into a value tree,
    then flattened) over n records (the k distinct ones tiled) with message offsets known, on the persistent
    pre-faulted pool of cpu_decode_pool; the concatenation of the ranges is not timed, as the GPU's is not."""
    try:
        import numpy as np
        threads = max(1, min(len(os.sched_getaffinity(0)), 256))
        k = len(recs)
        lens = np.array([len(r) for r in recs], dtype=np.uint64)
        one = np.frombuffer(b"".join(recs), dtype=np.uint8)
        reps = n // k
        wire = np.tile(one, reps)
        offs = np.zeros(n + 1, dtype=np.uint64)
        offs[1:] = np.cumsum(np.tile(lens, reps))
        ts, ok = cpu_decode_pool(sch, wire, offs, n, pb, threads)
        st = spread(n, ts)
        return {"value": st["median"], "unit": "records/s", "cores": threads, "kind": "port", "verified": ok,
                "spread": st,
                "sample": f"{n} records ({k} distinct, tiled), nested {'proto.Unmarshal' if pb else 'FastRead'} "
                          f"restatement (oracle/kx_oracle_nested.c) with message offsets known, one record range "
                          f"per thread of a persistent pool, pre-faulted outputs, median of {st['runs']} runs, "
                          f"{threads} threads"}
    except Exception as e:  # never break the bench line
        return {"error": repr(e)}


def crc32c_py(data: bytes) -> int:
    """CRC-32C by definition (bench-side spot check of the device values)"""
    c = 0xFFFFFFFF
    for x in data:
        c ^= x
        for _ in range(8):
            c = (c >> 1) ^ 0x82F63B78 if c & 1 else c >> 1
    return c ^ 0xFFFFFFFF


def host_inclusive(b, dev):
    """The netpoll-buffer path: records start and end in host memory. Measured through the library's
    kx_host_decode_batch from pinned buffers with message offsets known (the RPC case: framing gives
    every message's length), which pipelines 8 record-range chunks so H2D, decode and D2H overlap;
    plus the serial H2D -> decode -> D2H of the concatenated batch for comparison."""
    import numpy as np
    import torch

    from kitex_amd import _abi as A
    from kitex_amd.columns import alloc_device

    def pinned(n, dtype):
        return torch.empty(max(1, n), dtype=dtype, pin_memory=True)

    h_in = pinned(b.wire.numel(), torch.uint8)
    h_in.copy_(b.wire)
    h_off = pinned(b.n + 1, torch.int64)
    h_off.copy_(b.offs)
    infos, n = b.infos, b.n
    cols = []
    for c, ci in enumerate(infos):
        if ci.kind == A.COL_FIXED:
            cols.append(pinned(n * ci.width, torch.uint8).numpy().view(np.dtype(f"<u{ci.width}")
                                                                         if ci.width > 1 else np.uint8))
        else:
            w = 1 if ci.kind == A.COL_BYTES else ci.width
            cols.append((pinned(n + 1, torch.int32).numpy().view(np.uint32),
                         pinned(b.var_caps[c] * w, torch.uint8).numpy()))
    from kitex_amd.synth import ColumnSet
    pres = pinned(n, torch.int64).numpy().view(np.uint64) if b.cdc.dschema.npresence else None
    hout = ColumnSet(cols, pres, n)
    wire_np, off_np = h_in.numpy(), h_off.numpy().view(np.uint64)
    best = 1e30
    for _ in range(4):
        t0 = time.perf_counter()
        _, st = b.cdc.UnmarshalHost(wire_np, n, offsets=off_np, var_caps=b.var_caps, out=hout, raise_on_error=False)
        best = min(best, time.perf_counter() - t0)
    ok = st.code == 0 and st.n_records == n
    ok &= bool(np.array_equal(cols[0][:n].view(np.int64), b.src.cols[0][:n].cpu().numpy()))
    out_bytes = sum((c[0].nbytes + c[1].nbytes) if isinstance(c, tuple) else c.nbytes for c in cols)
    res = {"records_per_s": n / best, "ms": best * 1e3, "h2d_bytes": b.wire.numel() + (n + 1) * 8,
           "d2h_bytes": out_bytes, "pcie_gb_s": (b.wire.numel() + out_bytes) / best / 1e9, "verified": ok,
           "note": "kx_host_decode_batch from pinned host buffers, message offsets known: 16-chunk pipeline, "
                   "H2D / decode / D2H of different chunks overlap"}
    # serial reference: the concatenated batch, H2D -> decode -> D2H on one stream
    d_in = torch.empty_like(b.wire)
    out = alloc_device(infos, n, b.var_caps, b.cdc.dschema.npresence, dev)
    h_out = [((torch.empty(c[0].numel(), dtype=c[0].dtype, pin_memory=True),
               torch.empty(c[1].numel(), dtype=c[1].dtype, pin_memory=True)) if isinstance(c, tuple)
              else torch.empty(c.numel(), dtype=c.dtype, pin_memory=True)) for c in out.cols]
    sbest = 1e30
    for _ in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        d_in.copy_(h_in[:b.wire.numel()], non_blocking=True)
        b.cdc.Unmarshal(d_in, n, out=out, var_caps=b.var_caps, raise_on_error=False)
        for ho, c in zip(h_out, out.cols):
            if isinstance(c, tuple):
                ho[0].copy_(c[0], non_blocking=True)
                ho[1].copy_(c[1], non_blocking=True)
            else:
                ho.copy_(c, non_blocking=True)
        torch.cuda.synchronize()
        sbest = min(sbest, time.perf_counter() - t0)
    res["serial_concat"] = {"records_per_s": n / sbest, "ms": sbest * 1e3,
                            "note": "concatenated batch (no offsets): pinned H2D, decode, D2H serial on one stream"}
    # latency of a 64 Ki-record batch (16 chunks of 4096 records, decode k + 1 queued before the host reads
    # chunk k's status) and of a 4 Ki-record batch (one chunk)
    lat = {}
    for kk in (1 << 16, 1 << 12):
        k64 = min(n, kk)
        sub_off = np.ascontiguousarray(off_np[:k64 + 1])
        sub_in = wire_np[:int(sub_off[k64])]
        ts = []
        for _ in range(30):
            t0 = time.perf_counter()
            b.cdc.UnmarshalHost(sub_in, k64, offsets=sub_off, var_caps=b.var_caps, out=hout, raise_on_error=False)
            ts.append(time.perf_counter() - t0)
        lat[str(k64)] = {"median_ms": sorted(ts)[len(ts) // 2] * 1e3, "min_ms": min(ts) * 1e3}
    res["latency"] = lat
    # the reply path: kx_host_encode_batch from the pinned host columns just decoded back to a pinned wire
    h_wire = pinned(b.wire.numel(), torch.uint8).numpy()
    h_eoff = pinned(n + 1, torch.int64).numpy().view(np.uint64)
    ebest = 1e30
    for _ in range(4):
        t0 = time.perf_counter()
        w, _, est = b.cdc.MarshalHost(hout, out=h_wire, with_offsets=False, raise_on_error=False)
        ebest = min(ebest, time.perf_counter() - t0)
    eok = est.code == 0 and est.consumed == b.wire.numel()
    eok &= bool(np.array_equal(h_wire, wire_np[:b.wire.numel()]))
    del h_eoff
    res["encode"] = {"records_per_s": n / ebest, "ms": ebest * 1e3, "h2d_bytes": out_bytes,
                     "d2h_bytes": b.wire.numel(), "pcie_gb_s": (b.wire.numel() + out_bytes) / ebest / 1e9,
                     "verified": eok,
                     "note": "kx_host_encode_batch: pinned host columns -> pinned host wire, 16-chunk pipeline "
                             "(H2D of the columns / encode / D2H of the wire overlap; each chunk's output placed "
                             "by the previous chunk's device status)"}
    return res


def host_inclusive_shape(name, n, k=4096):
    """The host path on the reference's own request shapes (ABI 7): kx_host_decode_batch with message offsets
    known and kx_host_encode_batch, pinned buffers, k distinct records tiled to n. mockreq: MockReq{Msg,
    map<string,string>, list<string>} (internal/mocks/thrift/mock.thrift:3-6, flat LIST_BYTES columns);
    nesting: baseline.thrift's Nesting (the nested record walker). Arenas sized exactly (the distinct
    records' units times the tiling); verified against a decode of the distinct records and the wire."""
    import numpy as np
    import torch

    from kitex_amd import _abi as A
    from kitex_amd import idl, synth
    from kitex_amd import schema as S
    from kitex_amd.codec import ThriftCodec
    from kitex_amd.synth import ColumnSet
    if name == "mockreq":
        sch = S.schema_mockreq()
    else:
        doc = idl.parse_idl(os.path.join(ROOT, "tests", "golden", "idl", "baseline.thrift"))
        sch = idl.to_schema(doc.struct("Nesting"))
    cdc = ThriftCodec(sch)
    ds = cdc.dschema
    recs = synth.thrift_records(sch, k, seed=11)
    one = np.frombuffer(b"".join(recs), dtype=np.uint8)
    lens = np.array([len(r) for r in recs], dtype=np.uint64)
    reps = n // k
    n = reps * k

    def pinned(cnt, dtype):
        return torch.empty(max(1, cnt), dtype=dtype, pin_memory=True).numpy()
    wire = pinned(one.size * reps, torch.uint8)
    wire[:] = np.tile(one, reps)
    offs = pinned(n + 1, torch.int64).view(np.uint64)
    offs[0] = 0
    offs[1:] = np.cumsum(np.tile(lens, reps))
    ooffs = np.zeros(k + 1, dtype=np.uint64)
    ooffs[1:] = np.cumsum(lens)
    ref, st0 = cdc.UnmarshalHost(one.copy(), k, offsets=ooffs)   # the distinct records' columns and units
    var, elem, sub = [], [], []
    for c, ci in enumerate(ds.infos):
        if ci.kind == A.COL_FIXED:
            var.append(0), elem.append(0), sub.append(0)
            continue
        hi, lv = k, []
        for arr in ref.cols[c][:-1]:
            hi = int(arr[hi])
            lv.append(hi * reps)
        var.append(max(1, lv[-1]))
        elem.append(lv[0] if len(lv) >= 2 else 0)
        sub.append(lv[1] if len(lv) >= 3 else 0)
    fixed = {1: np.uint8, 2: np.int16, 4: np.int32, 8: np.int64}
    cols = []
    for c, ci in enumerate(ds.infos):
        if ci.kind == A.COL_FIXED:
            cols.append(pinned(n * ci.width, torch.uint8).view(fixed[ci.width]))
            continue
        arrs = [pinned(n + 1, torch.int32).view(np.uint32)]
        if ci.kind in (A.COL_LIST_BYTES, A.COL_LIST2, A.COL_LIST2_BYTES):
            arrs.append(pinned(elem[c] + 1, torch.int32).view(np.uint32))
        if ci.kind == A.COL_LIST2_BYTES:
            arrs.append(pinned(sub[c] + 1, torch.int32).view(np.uint32))
        w = 1 if ci.kind in (A.COL_BYTES, A.COL_LIST_BYTES, A.COL_LIST2_BYTES) else ci.width
        arrs.append(pinned(var[c] * w, torch.uint8).view(fixed[w]))
        cols.append(tuple(arrs))
    pres = pinned(n * 8, torch.uint8).view(np.uint64) if ds.npresence else None
    hout = ColumnSet(cols, pres, n)
    best = 1e30
    for _ in range(4):
        t0 = time.perf_counter()
        _, st, rs = cdc.UnmarshalHost(wire, n, offsets=offs, var_caps=var, elem_caps=elem, sub_caps=sub, out=hout,
                                      raise_on_error=False, record_status=True)
        best = min(best, time.perf_counter() - t0)
    ok = st.code == 0 and st.n_records == n and not rs.any()
    try:   # the first k records equal the distinct records' decode
        from tests.helpers import assert_columns_equal
        assert_columns_equal(hout, ref, ds.infos, k)
    except Exception:
        ok = False
    out_bytes = sum(sum(x.nbytes for x in c) if isinstance(c, tuple) else c.nbytes for c in cols) + \
        (pres.nbytes if pres is not None else 0)
    res = {"schema": "MockReq (mock.thrift:3-6)" if name == "mockreq" else "Nesting (baseline.thrift)",
           "records": n, "wire_bytes_per_record": wire.size / n,
           "decode": {"records_per_s": n / best, "ms": best * 1e3, "pcie_gb_s": (wire.size + out_bytes) / best / 1e9,
                      "verified": ok},
           "note": "kx_host_decode_batch / kx_host_encode_batch (ABI 7) from pinned buffers, offsets known, "
                   "16-chunk pipelines; arenas sized exactly"}
    # the reply bytes: the encoder's bytes of the distinct records, tiled (the generator may write fields in
    # another order than FastWriteNocopy's, so the input is not the reference)
    one_enc, _, st1 = cdc.MarshalHost(ref)
    h_wire = pinned(max(wire.size, one_enc.size * reps), torch.uint8)
    ebest = 1e30
    for _ in range(4):
        t0 = time.perf_counter()
        w, _, est = cdc.MarshalHost(hout, out=h_wire, with_offsets=False, raise_on_error=False)
        ebest = min(ebest, time.perf_counter() - t0)
    exact = est.code == 0 and st1.code == 0 and est.consumed == one_enc.size * reps and \
        bool(np.array_equal(h_wire[:est.consumed].reshape(reps, -1), np.broadcast_to(one_enc, (reps, one_enc.size))))
    res["encode"] = {"records_per_s": n / ebest, "ms": ebest * 1e3,
                     "pcie_gb_s": (est.consumed + out_bytes) / ebest / 1e9,
                     "bit_exact": bool(exact)}
    return res


def physical_cores():
    """distinct physical cores (package id, core id) among the CPUs this process may run on"""
    try:
        seen = set()
        for cpu in os.sched_getaffinity(0):
            base = f"/sys/devices/system/cpu/cpu{cpu}/topology/"
            with open(base + "physical_package_id") as a, open(base + "core_id") as b:
                seen.add((a.read().strip(), b.read().strip()))
        return len(seen) or None
    except Exception:
        return None


def cpu_baseline(cfg, nrec):
    """The CPU restatement of the reference FastRead (oracle, 'port') on every core this process may
    run on (sched_getaffinity): offsets known (per-message fastUnmarshal, parallel over records),
    plus the concatenated list<R> figure (one sequential walk: the GPU headline's mode)."""
    try:
        import numpy as np

        from kitex_amd import schema as S
        from kitex_amd import synth
        from oracle import oracle
        oracle.build()
        threads = max(1, min(len(os.sched_getaffinity(0)), 256))
        phys = physical_cores()
        sch = S.SCHEMAS[cfg]()
        cs = synth.GENERATORS[cfg](nrec)
        pb = cfg == "pf"
        rc, wire, offs = oracle.encode(sch, cs, threads=threads, pb=pb)
        assert rc == 0
        concat_wire = wire
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
        ts, ok = cpu_decode_pool(sch, wire, offs, nrec, pb, threads)
        st = spread(nrec, ts)
        best = nrec / st["median"]
        one = min(nrec, 1 << 20)
        t0 = time.perf_counter()
        oracle.decode(sch, wire[:int(offs[one])], one, offsets=offs[:one + 1], threads=1, pb=pb)
        t1 = time.perf_counter() - t0
        # concatenated mode (record boundaries found by walking, as the GPU headline decodes)
        cend = int(offs[one]) if not pb else None
        t0 = time.perf_counter()
        if not pb:
            rc, _, cst, _ = oracle.decode(sch, concat_wire[:cend], one, offsets=None)
            assert rc == 0 and cst.code == 0
        tc = time.perf_counter() - t0
        cpu = ""
        try:
            with open("/proc/cpuinfo") as fh:
                cpu = next((l.split(":", 1)[1].strip() for l in fh if l.startswith("model name")), "")
        except Exception:
            pass
        return {"value": st["median"], "unit": "records/s", "cores": threads, "kind": "port", "verified": ok,
                "spread": st,
                "sample": f"{nrec} {cfg} records, FastRead restatement (oracle/kx_oracle.c) with message "
                          f"offsets known, one record range per thread of a persistent pool with pre-faulted "
                          f"outputs, median of {st['runs']} runs after a warm-up, {threads} threads "
                          f"(len(sched_getaffinity))",
                "threads": threads, "physical_cores": phys,
                "cores_note": "cores = worker threads used (one per logical CPU of the affinity mask); "
                              "physical_cores = distinct (package, core) pairs among them",
                "gib_s": wire.size / best / 2**30, "one_thread_records_per_s": one / t1,
                "concat_one_thread_records_per_s": (one / tc) if not pb else None,
                "concat_note": f"{one} records as one concatenated list<{cfg}> body, walked sequentially "
                               "(the mode of the GPU headline; inherently one thread on the CPU)",
                "cpu_model": cpu}
    except Exception as e:  # the baseline must never break the GPU line
        return {"value": None, "error": repr(e)}


if __name__ == "__main__":
    main()
