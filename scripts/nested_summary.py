"""Round 5: per-kernel PMC / SQ counters of the nested walker runs (scripts/nested_prof.sh output), averaged
over dispatches, plus per-wave values.  python scripts/nested_summary.py gpurun_out/prof_r5_nested"""
import csv
import glob
import json
import re
import sys
from collections import defaultdict

d = sys.argv[1]
agg = defaultdict(lambda: defaultdict(list))
for p in ("sq1", "sq2", "tcp", "fetch"):
    for f in glob.glob(f"{d}/{p}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            name = re.sub(r"\(anonymous namespace\)::", "", r["Kernel_Name"]).split("(")[0].replace("void ", "")
            agg[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {"lib_sha256": open(f"{d}/lib.sha256").read().strip() if glob.glob(f"{d}/lib.sha256") else None,
       "note": "FETCH_SIZE in KB as rocprofv3 reports it (gfx950: see MI355X_MICROARCH.md for the correction)"}
keep = ("measure_kernel", "write_kernel", "esize_kernel", "ewrite_kernel", "index_kernel<0, 1>", "emit_kernel<0, 1, false>")
for k, cs in agg.items():
    if not any(k.startswith(x) for x in keep):
        continue
    waves = sum(cs["SQ_WAVES"]) / max(1, len(cs["SQ_WAVES"])) if "SQ_WAVES" in cs else None
    e = {c: sum(v) / len(v) for c, v in cs.items()}
    if waves:
        e["per_wave"] = {c: sum(v) / len(v) / waves for c, v in cs.items() if c != "SQ_WAVES"}
    out[k] = e
print(json.dumps(out, indent=1))
