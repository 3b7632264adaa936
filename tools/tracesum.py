"""Per-kernel-family time per forward from a rocprofv3 kernel trace (development
tool): tracesum.py trace.csv forwards [topN]"""
import collections
import csv
import re
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
fw = float(sys.argv[2])
top = int(sys.argv[3]) if len(sys.argv) > 3 else 25
per = collections.defaultdict(list)
for r in rows:
    n = re.sub(r"\(.*", "", r["Kernel_Name"])
    per[n].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
tot = sum(sum(v) for v in per.values())
span = (int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])) / 1e3
print(f"kernels {len(rows)} ({len(rows) / fw:.1f}/fwd)  busy {tot / fw:.1f} us/fwd  span {span / fw:.1f} us/fwd")
for k, v in sorted(per.items(), key=lambda kv: -sum(kv[1]))[:top]:
    print(f"{sum(v) / fw:8.1f} us/fwd  n={len(v) / fw:5.1f}  avg={sum(v) / len(v):7.1f}  {k[:110]}")
