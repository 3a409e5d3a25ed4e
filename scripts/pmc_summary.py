"""Summarise a scripts/profile_all.sh run into profiles/: per-kernel average duration (kernel trace)
and HBM bytes per decode call from the PMC passes (MI355X_MICROARCH.md HBM section: FETCH_SIZE and
WRITE_SIZE are in KiB; gfx950 FETCH_SIZE counts half of a wide streaming read -> x2).

  python scripts/pmc_summary.py <gpurun_out/prof_TAG> <cfg> <mode>  -> profiles/pmc_<cfg>_<mode>.json
  mode "encode": the encode kernels (size pass, scan, write pass) of scripts/run_encode.py instead
  mode "crc": the CRC32C Generate kernels of scripts/run_crc.py
  python scripts/pmc_summary.py <dir> <name> all <calls>  -> profiles/pmc_<name>.json: every codec kernel of a
  scripts/run_workload.py run (it launches no other), per call of `calls`
  mode "nenc" (same arguments): the nested encoder's kernels only (its run decodes the columns once first)
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

DECODE = ("index_kernel", "index_fast_kernel", "redo_kernel", "group_kernel", "chain_kernel", "chain_fast_kernel", "emit_kernel",
          "emit_fast_kernel", "emit_redo_kernel", "finalize_kernel")
ENCODE = ("size_kernel", "scan_kernel", "write_kernel")
CRC = ("crc_kernel", "crc_final_kernel")
NENC = ("esize_kernel", "escan_kernel", "ewrite_kernel")   # the nested encoder
KERNELS = DECODE


def short(name):
    if KERNELS is None:   # mode "all": every codec kernel (they all live in anonymous namespaces)
        if "(anonymous namespace)::" not in name:
            return None
        k = name.split("(anonymous namespace)::", 1)[1]
        return k.split("(", 1)[0]
    for k in KERNELS:
        if "namespace)::" + k in name:
            return k
    return None


def counter_sums(path, counter):
    per = defaultdict(list)
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = short(row["Kernel_Name"])
                if k and row["Counter_Name"] == counter:
                    per[k].append(float(row["Counter_Value"]))
    return per


def main():
    global KERNELS
    d, cfg, mode = sys.argv[1], sys.argv[2], sys.argv[3]
    KERNELS = None if mode == "all" else NENC if mode == "nenc" else ENCODE if mode == "encode" else CRC if mode == "crc" \
        else DECODE
    last = "write_kernel" if mode == "encode" else "crc_kernel" if mode == "crc" else "emit_kernel"
    fetch = counter_sums(os.path.join(d, "fetch"), "FETCH_SIZE")
    write = counter_sums(os.path.join(d, "write"), "WRITE_SIZE")
    if mode in ("all", "nenc"):
        calls = int(sys.argv[4])
    else:
        # one launch of every kernel of the pipeline per call: the most-launched one counts the calls (the
        # fast-path kernels replace emit_kernel / chain_kernel on the headline)
        calls = max([len(fetch.get(last, []))] + [len(v) for v in fetch.values()]) or 1
    kib = 1024.0
    fetch_b = sum(sum(v) for v in fetch.values()) * kib * 2 / calls
    write_b = sum(sum(v) for v in write.values()) * kib / calls
    names = sorted(set(fetch) | set(write)) if KERNELS is None else KERNELS
    per_kernel = {k: {"fetch_bytes": sum(fetch.get(k, [])) * kib * 2 / calls,
                      "write_bytes": sum(write.get(k, [])) * kib / calls} for k in names}
    dur = defaultdict(list)
    for f in glob.glob(os.path.join(d, "stats", "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = short(row["Kernel_Name"])
                if k:
                    dur[k].append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e6)
    sha = None
    try:
        with open(os.path.join(d, "lib.sha256")) as fh:
            sha = fh.read().strip()
    except OSError:
        pass
    res = {"workload": cfg if mode in ("all", "nenc") else f"{cfg}_{mode}" if mode in ("encode", "crc") else f"{cfg}_decode_{mode}",
           "calls": calls, "lib_sha256": sha,
           "hbm_bytes_per_launch": fetch_b + write_b, "fetch_bytes_per_call": fetch_b,
           "write_bytes_per_call": write_b, "per_kernel": per_kernel,
           "avg_ms": {k: sum(v) / len(v) for k, v in dur.items() if v},
           "note": "FETCH_SIZE x2 (gfx950 wide-read correction) + WRITE_SIZE, KiB -> bytes, summed over the "
                   "kernels of one call; Infinity-Cache hits are counted by these counters; bench.py "
                   "uses it only when lib_sha256 matches the library it times"}
    odir = os.environ.get("PMC_OUT") or os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                     "profiles")
    out = os.path.join(odir, f"pmc_{cfg}.json" if mode in ("all", "nenc") else f"pmc_{cfg}_{mode}.json")
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
