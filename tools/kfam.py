"""Per-forward kernel time by family from a rocprofv3 kernel_stats.csv (development):
python tools/kfam.py <run_kernel_stats.csv> <forwards>"""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
nf = float(sys.argv[2])
tot = 0.0
out = []
for r in rows:
    name = r["Name"]
    if any(s in name for s in ("rocclr", "at::native", "distribution")):
        continue
    name = re.sub(r"^void |cfd::|\(.*$", "", name)
    name = re.sub(r"_ZN3cfd\d+(\w+?)E.*", r"\1", name)
    ms = float(r["TotalDurationNs"]) / 1e6 / nf
    n = int(r["Calls"]) / nf
    tot += ms
    out.append((ms, n, name[:70]))
for ms, n, name in sorted(out, reverse=True):
    print("%-72s %6.1f  %7.3f ms  %6.1f us" % (name, n, ms, ms / n * 1e3 if n else 0))
print("total kernel time per forward %.3f ms, launches %.0f" % (tot, sum(o[1] for o in out)))
