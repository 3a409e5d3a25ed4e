"""Per-tile SQ counters of the decode kernels from scripts/sq_counters.sh output (exact kernel-name
match, averaged over the matching dispatches).  python scripts/sq_summary.py gpurun_out/sq_r2 [tiles]"""
import csv
import glob
import json
import sys
from collections import defaultdict

d = sys.argv[1]
KS = ("index_kernel<", "index_fast_kernel<", "redo_kernel<", "group_kernel<", "chain_kernel<", "chain_fast_kernel<",
      "emit_kernel<", "emit_fast_kernel<", "emit_redo_kernel<", "combo_kernel<", "write_kernel<", "size_kernel<",
      "crc_kernel(", "measure_kernel<", "esize_kernel<", "ewrite_kernel<")
agg = defaultdict(lambda: defaultdict(list))
for p in ("p1", "p2"):
    for f in glob.glob(f"{d}/{p}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            for k in KS:
                if "(anonymous namespace)::" + k in name:
                    agg[k.rstrip("<(")][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {}
for k, cs in agg.items():
    waves = sum(cs["SQ_WAVES"]) / max(1, len(cs["SQ_WAVES"])) if "SQ_WAVES" in cs else None
    out[k] = {c: sum(v) / len(v) for c, v in cs.items()}
    if waves:
        out[k]["per_wave"] = {c: sum(v) / len(v) / waves for c, v in cs.items() if c != "SQ_WAVES"}
print(json.dumps(out, indent=1))
