"""Join the CFD_CONV_LOG GroupNorm lines with a rocprofv3 kernel trace (development
tool): per GroupNorm shape, time per forward and the achieved HBM-level bandwidth
over its algorithmic bytes (reads: ksplits slabs or the input, + residual; writes:
the normalised output, + the raw sum when kx)."""
import collections
import csv
import sys

trace, log, fw = sys.argv[1], sys.argv[2], float(sys.argv[3])
rows = sorted(csv.DictReader(open(trace)), key=lambda r: int(r["Start_Timestamp"]))
gnk = [r for r in rows if "gn_" in r["Kernel_Name"]]
logs = [l.split()[1:] for l in open(log) if l.startswith("GN ")]
B = 8
per = collections.defaultdict(list)
i = 0
for l in logs:
    hw = l[1]
    c1, c2 = map(int, l[2][2:].split("+"))
    ks, kres, kx = int(l[3].split("=")[1]), int(l[4].split("=")[1]), int(l[5].split("=")[1])
    # a three-kernel GroupNorm launches partial/finalize/apply
    r = gnk[i]
    n = 3 if "partial" in r["Kernel_Name"] else 1
    t = sum(int(x["End_Timestamp"]) - int(x["Start_Timestamp"]) for x in gnk[i:i + n]) / 1e3
    i += n
    H, W = map(int, hw.split("x"))
    el = B * H * W * (c1 + c2)
    rd = el * 4 * (ks if ks else 1) + (B * H * W * c1 * 4 if kres else 0)
    wr = el * 4 + (B * H * W * c1 * 4 if kx else 0)
    per[" ".join(l[1:])].append((t, rd + wr))
tot = 0
for k, v in sorted(per.items(), key=lambda kv: -sum(x[0] for x in kv[1])):
    t = sum(x[0] for x in v) / fw
    byt = v[0][1]
    tot += t
    print(f"{t:8.1f} us/fwd n={len(v) / fw:4.1f} avg={t / (len(v) / fw):6.1f} us  {byt / 1e6:6.1f} MB  {byt / (t / (len(v) / fw)) / 1e6:6.2f} TB/s  {k}")
print("total GN us/fwd", tot)
