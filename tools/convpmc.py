"""Per-(kernel, grid) averages of rocprofv3 --pmc passes over tools/convbench.bin
(development tool, tools/gpujob_convpmc.sh).  Derived: wave-state fractions of
SQ_WAVE_CYCLES, matrix-pipe busy fraction (SQ_VALU_MFMA_BUSY_CYCLES over the
chip's SIMD cycles at the held clock, GRBM_GUI_ACTIVE / 8), L2 hit rate, fetch
bytes (FETCH_SIZE kB x 2 for gfx950 16-B reads, MI355X_MICROARCH.md)."""
import collections
import csv
import glob
import os
import sys

acc = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.defaultdict(collections.Counter)
dur = collections.defaultdict(list)
for d in sys.argv[1:]:
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for x in csv.DictReader(open(f)):
            kn = x["Kernel_Name"]
            if not os.environ.get("PMC_ALL") and "conv" not in kn and "splitk" not in kn:
                continue
            name = kn.replace("void ", "").replace("cfd::", "")
            name = name[:name.find("(")] if "(" in name else name
            key = (name[:40], int(x["Grid_Size"]) // int(x["Workgroup_Size"]))
            acc[key][x["Counter_Name"]] += float(x["Counter_Value"])
            n[key][x["Counter_Name"]] += 1
            if x["Counter_Name"] in ("SQ_WAVE_CYCLES", "GRBM_GUI_ACTIVE", "TCC_HIT_sum", "FETCH_SIZE"):
                dur[key].append(int(x["End_Timestamp"]) - int(x["Start_Timestamp"]))
print("%-40s %6s %8s %5s %5s %5s %6s %6s %6s %6s %7s %6s" % ("kernel", "WGs", "us", "wait", "inst", "act", "mfma",
                                                            "GHz", "v/mf", "l/mf", "L2hit", "MBfet") + "  ldsW  bankc")
for k in sorted(acc, key=lambda k: (k[0], k[1])):
    d = acc[k]
    g = lambda c: d[c] / max(n[k][c], 1)
    t = sum(dur[k]) / max(len(dur[k]), 1)
    wc = max(g("SQ_WAVE_CYCLES"), 1)
    cyc = g("GRBM_GUI_ACTIVE") / 8
    util = g("SQ_VALU_MFMA_BUSY_CYCLES") / max(cyc * 1024, 1) if cyc else float("nan")
    m = max(g("SQ_INSTS_MFMA"), 1)
    hit = g("TCC_HIT_sum") / max(g("TCC_HIT_sum") + g("TCC_MISS_sum"), 1)
    print("%-40s %6d %8.1f %5.2f %5.2f %5.2f %6.3f %6.2f %6.2f %6.2f %7.3f %6.1f" % (
        k[0], k[1], t / 1e3, g("SQ_WAIT_ANY") / wc, g("SQ_WAIT_INST_ANY") / wc, g("SQ_ACTIVE_INST_ANY") / wc, util,
        cyc / t if t else 0, g("SQ_INSTS_VALU") / m, g("SQ_INSTS_LDS") / m, hit, 2 * g("FETCH_SIZE") / 1e3) +
        "  %5.2f %5.2f" % (g("SQ_WAIT_INST_LDS") / wc, g("SQ_LDS_BANK_CONFLICT") / max(g("SQ_LDS_IDX_ACTIVE"), 1)))
