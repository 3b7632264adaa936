"""Join the CFD_CONV_LOG convolution lines with a rocprofv3 kernel trace
(development tool): per convolution shape and plan, time per forward and its
TFLOP/s fp32-equivalent (2 M Cout K).  Usage: convjoin.py trace.csv stderr.log forwards"""
import collections
import csv
import sys

trace, log, fw = sys.argv[1], sys.argv[2], float(sys.argv[3])
rows = sorted(csv.DictReader(open(trace)), key=lambda r: int(r["Start_Timestamp"]))
convk = [r for r in rows if any(k in r["Kernel_Name"] for k in ("conv_h_kernel", "conv_x_kernel", "conv_gemm_kernel"))]
logs = [l.split(None, 1)[1].strip() for l in open(log) if l.startswith("CONV ")]
per = collections.defaultdict(list)
for l, r in zip(logs, convk):
    per[" ".join(l.split()[1:])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
tot = 0.0
for k, v in sorted(per.items(), key=lambda kv: -sum(kv[1])):
    f = dict(x.split("=") for x in k.split() if "=" in x)
    cin = sum(map(int, f["C"].split("->")[0].split("+")))
    cout = int(f["C"].split("->")[1])
    flop = 2.0 * int(f["M"]) * cout * int(f["ks"]) ** 2 * cin
    t = sum(v) / fw
    tot += t
    print(f"{t:8.1f} us/fwd n={len(v) / fw:4.1f} avg={sum(v) / len(v):7.1f} us {flop / (sum(v) / len(v)) / 1e6:6.1f} TF  {k}")
print("total conv us/fwd", tot)
