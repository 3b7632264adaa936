"""HEAD PMC record of the headline configuration (bench.py config B, pipelined):
merges three rocprofv3 --pmc passes of ``bench.py --steps 4 --warmup 0`` into one
JSON (profiles/r06c_pipe_pmc.json), which the bench line's roofline cites.

    python tools/pipe_pmc.py SQ.csv FETCH.csv WRITE.csv OUT.json

Per kernel (name up to its template arguments) and, for the decoder
(siren_split32), per dispatch in launch order -- PipelineB decodes batches
1..K-1 on the upper CU half and the last one on the whole chip:
  * mfma_busy_frac = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x SIMDs of
    the CUs it ran on): the matrix pipes' busy share at the clock the chip held;
  * clock_ghz_grbm = GRBM_GUI_ACTIVE / 8 / duration (reads high below ~0.3 ms);
  * traffic = 2 x FETCH_SIZE + WRITE_SIZE bytes (MI355X_MICROARCH.md HBM section:
    FETCH_SIZE counts half the bytes of 16-B-per-lane reads on gfx950; both count
    Infinity-Cache hits, so this bounds HBM bytes from above);
  * valu_per_mfma, lds_per_mfma instruction ratios.
Under --pmc the dispatches are serialised: the side-by-side decodes ran on their
CU half but without the sampler beside them (their clock is the half-chip-alone
clock; tools/dev/siren_clock.py measures the pipelined one)."""
import collections
import csv
import json
import sys


def load(path):
    rows = collections.defaultdict(dict)   # dispatch id -> {counter: value, meta}
    for r in csv.DictReader(open(path)):
        d = rows[int(r["Dispatch_Id"])]
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        d["_name"] = r["Kernel_Name"].replace("void ", "")
        d["_ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        d["_grid"] = int(r["Grid_Size"])
    return rows


def family(name):
    return name.split("(")[0]


def main():
    sq, fe, wr, out = sys.argv[1:5]
    passes = [load(sq), load(fe), load(wr)]
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    dec = [[] for _ in passes]
    for i, p in enumerate(passes):
        for did in sorted(p):
            d = p[did]
            fam = family(d["_name"])
            for k, v in d.items():
                if not k.startswith("_"):
                    per[fam][k].append(v)
            per[fam]["_ns" + str(i)].append(d["_ns"])
            if "siren_split32" in fam:
                dec[i].append(d)
    rec = {"command": "rocprofv3 --pmc <pass> -- python3 bench.py --steps 4 --warmup 0 --no-cpu-baseline",
           "kernels": {}, "decoder_dispatches": []}
    for fam, c in per.items():
        mean = lambda k: sum(c[k]) / len(c[k]) if c.get(k) else None  # noqa: E731
        ns = mean("_ns0")
        e = {"calls": len(c.get("_ns0", [])), "avg_us": ns / 1e3 if ns else None}
        for k in ("SQ_INSTS_VALU", "SQ_INSTS_MFMA", "SQ_INSTS_LDS", "SQ_VALU_MFMA_BUSY_CYCLES", "GRBM_GUI_ACTIVE"):
            e[k] = mean(k)
        if e["SQ_INSTS_MFMA"]:
            e["valu_per_mfma"] = e["SQ_INSTS_VALU"] / e["SQ_INSTS_MFMA"]
            e["lds_per_mfma"] = e["SQ_INSTS_LDS"] / e["SQ_INSTS_MFMA"]
        f, w = mean("FETCH_SIZE"), mean("WRITE_SIZE")
        if f is not None and w is not None:
            e["traffic_bytes"] = 2 * f * 1024 + w * 1024
        rec["kernels"][fam] = e
    n = min(len(x) for x in dec)
    for j in range(n):
        s, f, w = dec[0][j], dec[1][j], dec[2][j]
        whole = j == n - 1
        simds = 256 * 4 if whole else 128 * 4
        cyc = s["GRBM_GUI_ACTIVE"] / 8
        rec["decoder_dispatches"].append({
            "cus": 256 if whole else 128, "ms": s["_ns"] / 1e6, "clock_ghz_grbm": cyc / s["_ns"],
            "mfma_busy_frac": s["SQ_VALU_MFMA_BUSY_CYCLES"] / (cyc * simds),
            "valu_per_mfma": s["SQ_INSTS_VALU"] / s["SQ_INSTS_MFMA"],
            "lds_per_mfma": s["SQ_INSTS_LDS"] / s["SQ_INSTS_MFMA"],
            "fetch_bytes_corrected": 2 * f["FETCH_SIZE"] * 1024, "write_bytes": w["WRITE_SIZE"] * 1024,
            "traffic_bytes": 2 * f["FETCH_SIZE"] * 1024 + w["WRITE_SIZE"] * 1024})
    rec["note"] = __doc__.split("\n\n", 2)[2].strip()
    json.dump(rec, open(out, "w"), indent=1)
    print(json.dumps(rec["decoder_dispatches"], indent=1))
    top = sorted(rec["kernels"].items(), key=lambda kv: -(kv[1]["avg_us"] or 0) * kv[1]["calls"])[:12]
    for k, e in top:
        print(f"{k[:60]:60s} calls {e['calls']:7d} avg {e['avg_us'] or 0:9.1f} us  valu/mfma "
              f"{e.get('valu_per_mfma', 0):6.2f}")


if __name__ == "__main__":
    main()
