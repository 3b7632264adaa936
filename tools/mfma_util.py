"""MFMA utilisation per kernel from a rocprofv3 --pmc pass (development tool,
tools/gpujob_mfma_util.sh).

GRBM_GUI_ACTIVE is summed over the 8 XCDs: kernel cycles = GRBM_GUI_ACTIVE / 8,
effective clock = kernel cycles / duration (MI355X_MICROARCH.md, DVFS give-back).
SQ_VALU_MFMA_BUSY_CYCLES counts matrix-pipe busy cycles summed over all SIMDs
(32 per v_mfma_*_32x32x16_f16, 16 per 16x16x32), so
    util = MFMA_BUSY / (kernel cycles x 1024 SIMDs)
is the fraction of the chip's matrix-pipe cycles in use at the clock it held --
the dense-MFMA peak at that clock is util = 1."""
import collections
import csv
import sys

SIMDS = 256 * 4
acc = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.defaultdict(collections.Counter)
dur = collections.defaultdict(dict)
args = [a for a in sys.argv[1:] if not a.startswith("--json=")]
jout = [a[7:] for a in sys.argv[1:] if a.startswith("--json=")]
for f in args:
    for x in csv.DictReader(open(f)):
        kn = x["Kernel_Name"]
        if not kn.startswith(("cfd::", "void cfd::", "_ZN3cfd")):
            continue
        key = kn.replace("void ", "")[:48]
        acc[key][x["Counter_Name"]] += float(x["Counter_Value"])
        n[key][x["Counter_Name"]] += 1
        dur[key][(f, x["Dispatch_Id"])] = int(x["End_Timestamp"]) - int(x["Start_Timestamp"])
rows = []
for k, d in acc.items():
    g = lambda c: d[c] / max(n[k][c], 1)
    t_ns = sum(dur[k].values()) / len(dur[k])
    cyc = g("GRBM_GUI_ACTIVE") / 8
    util = g("SQ_VALU_MFMA_BUSY_CYCLES") / max(cyc * SIMDS, 1)
    clk = cyc / t_ns if t_ns else 0.0
    rows.append((t_ns * len(dur[k]), k, len(dur[k]), t_ns / 1e3, clk, util, g("SQ_INSTS_MFMA")))
print("%-48s %6s %10s %8s %8s %12s" % ("kernel", "calls", "avg_us", "clk_GHz", "mfma_util", "mfma_insts"))
for r in sorted(rows, reverse=True)[:14]:
    print("%-48s %6d %10.1f %8.3f %8.3f %12.0f" % r[1:])
if jout:
    import json
    rec = {r[1]: {"calls": r[2], "avg_us": round(r[3], 1), "held_clock_ghz": round(r[4], 3),
                  "mfma_busy_frac": round(r[5], 4), "mfma_insts_per_call": r[6]} for r in rows}
    rec["_note"] = ("rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_BUSY_CYCLES "
                    "(tools/gpujob_mfma_util.sh); mfma_busy_frac = busy matrix-pipe cycles / (GRBM_GUI_ACTIVE/8 x 1024 "
                    "SIMDs); held_clock from GRBM_GUI_ACTIVE/8 / duration reads high below ~0.3 ms dispatches")
    json.dump(rec, open(jout[0], "w"), indent=1)
