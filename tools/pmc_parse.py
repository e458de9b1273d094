"""Parse rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into per-launch HBM bytes (profiles/pmc_traffic.json).

gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE reports exactly half of the bytes of a wide
coalesced streaming read (16 B/lane dwordx4) -> x2; WRITE_SIZE is exact for 16 B/lane stores.  Both
counters are in KiB.  usage: python tools/pmc_parse.py <fetch_dir> <write_dir> <workload_key> <alg_bytes> [kernel | "k1*n1+k2*n2"] [launches]
"""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_dispatch(d, counter, kernel_substr):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    vals = {}
    for f in files:
        for row in csv.DictReader(open(f)):
            if row.get("Counter_Name") != counter or kernel_substr not in row.get("Kernel_Name", ""):
                continue
            did = row.get("Dispatch_Id")
            vals[did] = vals.get(did, 0.0) + float(row["Counter_Value"])
    return list(vals.values())


def main():
    fetch_dir, write_dir, key, alg = sys.argv[1], sys.argv[2], sys.argv[3], float(sys.argv[4])
    kern = sys.argv[5] if len(sys.argv) > 5 else "k_reduce"
    launches = int(sys.argv[6]) if len(sys.argv) > 6 else 1
    alg = alg / launches
    # kern "a*4+b*1": a step of several kernels (4 launches of a, 1 of b); per launch = the step's bytes / launches
    terms = [(t.split("*")[0], int(t.split("*")[1]) if "*" in t else 1) for t in kern.split("+")]
    fkb = wkb = 0.0
    ndisp = 0
    for name, count in terms:
        f = per_dispatch(fetch_dir, "FETCH_SIZE", name)
        w = per_dispatch(write_dir, "WRITE_SIZE", name)
        if not f or not w:
            raise SystemExit(f"no {name} dispatches found (fetch {len(f)}, write {len(w)})")
        scale = count / launches if len(terms) > 1 else 1.0
        fkb += scale * sum(f) / len(f)
        wkb += scale * sum(w) / len(w)
        ndisp += len(f)
    f = [None] * ndisp
    hbm = (2 * fkb + wkb) * 1024
    out_path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    db = json.load(open(out_path)) if os.path.exists(out_path) else {}
    db[key] = {"kernel": kern, "dispatches": len(f), "FETCH_SIZE_KiB": fkb, "WRITE_SIZE_KiB": wkb,
               "hbm_bytes_per_launch": hbm, "alg_bytes_per_launch": alg, "traffic_over_alg": hbm / alg,
               "launches_per_step": launches,
               "correction": "bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE counts half of "
                             "16B/lane streaming reads, MI355X_MICROARCH.md HBM section)"}
    json.dump(db, open(out_path, "w"), indent=1, sort_keys=True)
    print(json.dumps(db[key]))


if __name__ == "__main__":
    main()
