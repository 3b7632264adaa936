"""Per-(kernel, grid) time from a rocprofv3 kernel_trace.csv (development tool):
total microseconds per forward (divided by --per), calls, and share, largest first."""
import argparse
import collections
import csv
import glob

ap = argparse.ArgumentParser()
ap.add_argument("dir")
ap.add_argument("--per", type=float, default=1.0, help="divide totals by this (e.g. the forward count)")
ap.add_argument("--top", type=int, default=40)
args = ap.parse_args()
tot = collections.Counter()
cnt = collections.Counter()
for f in glob.glob(f"{args.dir}/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].replace("void ", "").replace("cfd::", "")
        name = name[:name.find("(")] if "(" in name else name
        g = int(r.get("Grid_Size_X", r.get("Grid_Size", 0)) or 0) * int(r.get("Grid_Size_Y", 1) or 1) * int(r.get("Grid_Size_Z", 1) or 1)
        wg = int(r.get("Workgroup_Size_X", r.get("Workgroup_Size", 1)) or 1) * int(r.get("Workgroup_Size_Y", 1) or 1) * int(r.get("Workgroup_Size_Z", 1) or 1)
        key = (name[:60], g // max(wg, 1))
        tot[key] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        cnt[key] += 1
T = sum(tot.values())
print(f"total {T / 1e3 / args.per:.1f} us per unit")
fam = collections.Counter()
for k, v in tot.items():
    fam[k[0].split("<")[0]] += v
for k, v in fam.most_common():
    print(f"  family {k:40s} {v / 1e3 / args.per:9.1f} us {100 * v / T:5.1f}%")
for k, v in tot.most_common(args.top):
    print(f"{v / 1e3 / args.per:9.1f} us {100 * v / T:5.1f}% n={cnt[k] / args.per:6.1f} WGs={k[1]:6d} {k[0]}")
