"""Print a rocprofv3 --stats kernel summary compactly: calls, average us, total ms, short name.
python scripts/kstats.py <dir with *kernel_stats.csv>"""
import csv
import glob
import re
import sys

for f in glob.glob(f"{sys.argv[1]}/**/*kernel_stats.csv", recursive=True):
    rows = list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
    for r in rows[:int(sys.argv[2]) if len(sys.argv) > 2 else 40]:
        name = re.sub(r"\(anonymous namespace\)::", "", r["Name"])[:110]
        print(f'{int(r["Calls"]):6d} {float(r["AverageNs"]) / 1e3:10.1f} us {float(r["TotalDurationNs"]) / 1e6:9.2f} ms  {name}')
