"""U-Net forward PMC summary per kernel family (development tool,
tools/gpujob_unet_pmc.sh): rocprofv3 --pmc passes over `tools/kbench.py unet`
(B = 8, 64x64, split_f16).  Per family, averaged over its dispatches: duration,
wave-state fractions of SQ_WAVE_CYCLES (SQ_WAIT_ANY = parked on s_waitcnt /
barrier, SQ_WAIT_INST_ANY = issue stall, SQ_ACTIVE_INST_ANY = issuing), matrix
pipe busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs), LDS
bank-conflict cycles / LDS array cycles, VALU and LDS instructions per MFMA, L2
hit rate, and FETCH (x2, gfx950 16-B reads) / WRITE bytes per dispatch."""
import collections
import csv
import glob
import json
import sys

acc = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.defaultdict(collections.Counter)
dur = collections.defaultdict(list)
for d in sys.argv[1:]:
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for x in csv.DictReader(open(f)):
            kn = x["Kernel_Name"].replace("void ", "").replace("cfd::", "")
            kn = kn[:kn.find("(")] if "(" in kn else kn
            if not any(p in kn for p in ("conv", "gn_", "gn2_", "attention", "attn", "splitk", "linear")):
                continue
            key = kn[:44]
            acc[key][x["Counter_Name"]] += float(x["Counter_Value"])
            n[key][x["Counter_Name"]] += 1
            if x["Counter_Name"] in ("SQ_WAVE_CYCLES",):
                dur[key].append(int(x["End_Timestamp"]) - int(x["Start_Timestamp"]))
rows = {}
for k, d in acc.items():
    g = lambda c: d[c] / max(n[k][c], 1)
    t = sum(dur[k]) / max(len(dur[k]), 1)
    wc = max(g("SQ_WAVE_CYCLES"), 1)
    cyc = g("GRBM_GUI_ACTIVE") / 8
    m = max(g("SQ_INSTS_MFMA"), 1)
    rows[k] = dict(dispatches=len(dur[k]), avg_us=round(t / 1e3, 2),
                   wait=round(g("SQ_WAIT_ANY") / wc, 3), issue_stall=round(g("SQ_WAIT_INST_ANY") / wc, 3),
                   active=round(g("SQ_ACTIVE_INST_ANY") / wc, 3),
                   mfma_busy=round(g("SQ_VALU_MFMA_BUSY_CYCLES") / max(cyc * 1024, 1), 3) if cyc else None,
                   lds_conflict=round(g("SQ_LDS_BANK_CONFLICT") / max(g("SQ_LDS_IDX_ACTIVE"), 1), 3),
                   valu_per_mfma=round(g("SQ_INSTS_VALU") / m, 2) if g("SQ_INSTS_MFMA") else None,
                   lds_per_mfma=round(g("SQ_INSTS_LDS") / m, 2) if g("SQ_INSTS_MFMA") else None,
                   l2_hit=round(g("TCC_HIT_sum") / max(g("TCC_HIT_sum") + g("TCC_MISS_sum"), 1), 3),
                   fetch_MB=round(2 * g("FETCH_SIZE") / 1e3, 2), write_MB=round(g("WRITE_SIZE") / 1e3, 2))
out = sys.stdout
cols = ["dispatches", "avg_us", "wait", "issue_stall", "active", "mfma_busy", "lds_conflict", "valu_per_mfma",
        "lds_per_mfma", "l2_hit", "fetch_MB", "write_MB"]
print("%-44s " % "kernel" + " ".join("%10s" % c[:10] for c in cols))
for k in sorted(rows, key=lambda k: -rows[k]["avg_us"] * rows[k]["dispatches"]):
    print("%-44s " % k + " ".join("%10s" % rows[k][c] for c in cols))
json.dump(rows, open("gpurun_out/unet_pmc.json", "w"), indent=1)
