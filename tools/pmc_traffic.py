"""Per-launch HBM-side traffic of one kernel from two rocprofv3 --pmc passes.

    python tools/pmc_traffic.py FETCH.csv WRITE.csv KERNEL_SUBSTR OUT.json [algorithmic_bytes [launch_json]]

FETCH_SIZE / WRITE_SIZE are in KB (x1024).  Per MI355X_MICROARCH.md (HBM /
rocprofv3 section) FETCH_SIZE reports half the bytes of 16-B-per-lane streaming
reads on gfx950 (global_load_lds_dwordx4 included), so it is doubled; WRITE_SIZE
is exact for 16-B stores.  Both count L2 misses served by the Infinity Cache
(MALL), so the figure is an upper bound on HBM bytes.
"""
import csv
import json
import sys


def mean_counter(path, substr, name):
    vals, kname, grid, wg = [], None, None, None
    for r in csv.DictReader(open(path)):
        if substr in r["Kernel_Name"] and r["Counter_Name"] == name:
            vals.append(float(r["Counter_Value"]))
            kname, grid, wg = r["Kernel_Name"], int(r["Grid_Size"]), int(r["Workgroup_Size"])
    if not vals:
        raise SystemExit(f"no {name} rows for {substr!r} in {path}")
    return sum(vals) / len(vals), len(vals), kname, grid, wg


def main():
    fpath, wpath, substr, out = sys.argv[1:5]
    alg = float(sys.argv[5]) if len(sys.argv) > 5 else None
    launch = json.loads(sys.argv[6]) if len(sys.argv) > 6 else {}
    f_kb, nf, kname, grid, wg = mean_counter(fpath, substr, "FETCH_SIZE")
    w_kb, nw, _, _, _ = mean_counter(wpath, substr, "WRITE_SIZE")
    fetch = 2.0 * f_kb * 1024.0
    write = w_kb * 1024.0
    rec = {"kernel": kname, "launch": launch, "grid_size": grid, "workgroup_size": wg, "dispatches": [nf, nw],
           "fetch_size_kb_raw_mean": f_kb, "write_size_kb_mean": w_kb, "fetch_bytes_corrected": fetch,
           "write_bytes": write, "traffic_bytes_per_launch": fetch + write, "algorithmic_bytes_per_launch": alg,
           "note": "separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes; FETCH doubled (gfx950 16B/lane "
                   "reads count half); both include Infinity-Cache (MALL) hits, so this bounds HBM traffic "
                   "from above"}
    json.dump(rec, open(out, "w"), indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
