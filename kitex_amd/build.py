"""Build libkxcodec.so (HIP kernels for gfx950 + the C-ABI) in-tree with hipcc.

The .so is written to kitex_amd/lib/ so it travels with the repo snapshot to the GPU box.
"""
from __future__ import annotations

import glob
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIBDIR = os.path.join(HERE, "lib")
LIB = os.path.join(LIBDIR, "libkxcodec.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"


def sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.cpp")))


def _stale() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = sources() + glob.glob(os.path.join(CSRC, "*.h")) + [os.path.join(HERE, "..", "include", "kxcodec.h")]
    return any(os.path.getmtime(d) > t for d in deps)


DECODE_PARTS = 8   # kx_decode.hip is compiled once per part (-DKX_DEC_PART=k): its kernels in parallel


def _units(libdir=LIBDIR):
    """(source, object, extra flags) per translation unit."""
    out = []
    for src in sources():
        base = os.path.join(libdir, os.path.basename(src))
        if os.path.basename(src) == "kx_decode.hip":
            out += [(src, f"{base}.{k}.o", [f"-DKX_DEC_PART={k}"]) for k in range(DECODE_PARTS)]
        else:
            out.append((src, base + ".o", []))
    return out


def build(force: bool = False, verbose: bool = False, extra=(), variant: str = "") -> str:
    """variant: build into lib/<variant>/ (with `extra` flags) for kernel-tuning experiments."""
    libdir = os.path.join(LIBDIR, variant) if variant else LIBDIR
    lib = os.path.join(libdir, "libkxcodec.so")
    if not force and not variant and not _stale():
        return LIB
    os.makedirs(libdir, exist_ok=True)
    hdrs = glob.glob(os.path.join(CSRC, "*.h")) + [os.path.join(HERE, "..", "include", "kxcodec.h")]
    newest_hdr = max(os.path.getmtime(h) for h in hdrs)
    jobs = []
    # KX_VARIANT_PARTS=1,3: a variant recompiles only these decode parts with its flags and links the default
    # build's other objects (a kernel-tuning experiment that touches one instantiation builds in one unit)
    only = os.environ.get("KX_VARIANT_PARTS") if variant else None
    only_objs = {f"kx_decode.hip.{k}.o" for k in only.split(",")} if only else None
    for src, obj, flags in _units(libdir):
        if only_objs is not None and os.path.basename(obj) not in only_objs:
            import shutil
            dflt = os.path.join(LIBDIR, os.path.basename(obj))
            if not os.path.exists(dflt) or os.path.getmtime(dflt) < max(os.path.getmtime(src), newest_hdr):
                raise RuntimeError(f"KX_VARIANT_PARTS: the default build's {os.path.basename(obj)} is missing or "
                                   "older than its sources; run `python -m kitex_amd.build` first")
            shutil.copy2(dflt, obj)
            continue
        fresh = (not force and not extra and not variant and os.path.exists(obj)
                 and os.path.getmtime(obj) > max(os.path.getmtime(src), newest_hdr))
        if fresh:
            continue
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17", "-Wall",
               "-Wno-unused-function", "-munsafe-fp-atomics", *flags, "-c", src, "-o", obj, *extra]
        jobs.append(cmd)

    def run(cmd):
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        return subprocess.run(cmd).returncode

    workers = max(1, min(len(jobs), len(os.sched_getaffinity(0)), 8))
    with ThreadPoolExecutor(max_workers=workers) as ex:
        rcs = list(ex.map(run, jobs))
    if any(rcs):
        raise RuntimeError("hipcc failed")
    objs = [obj for _, obj, _ in _units(libdir)]
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", lib + ".tmp", *objs]
    subprocess.run(cmd, check=True)
    os.replace(lib + ".tmp", lib)
    return lib


if __name__ == "__main__":
    args = [a for a in sys.argv[1:] if a != "--force"]
    # python -m kitex_amd.build [--force] [VARIANT -DFLAG ...]
    print(build(force="--force" in sys.argv, verbose=True, variant=args[0] if args else "", extra=tuple(args[1:])))
