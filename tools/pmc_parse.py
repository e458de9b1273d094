"""Parse rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into per-launch HBM bytes (profiles/pmc_traffic.json).

gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE reports exactly half of the bytes of a wide
coalesced streaming read (16 B/lane dwordx4) -> x2; WRITE_SIZE is exact for 16 B/lane stores.  Both
counters are in KiB.

An entry belongs to ONE run: it is keyed by (workload, resident clients per pass, launches per round, build id of
the library that ran), all read from the bench line printed by the same rocprofv3 command, so bench.py attaches it
only to a run of the same library over the same shape (``roofline.traffic``; null otherwise).

    python tools/pmc_parse.py --bench B.json --fetch F --write W [--kernel "k1*n1+k2*n2"]
        F / W: a rocprofv3 output directory or a counter_collection.csv file of each pass
    python tools/pmc_parse.py --fix-profile P_under_rocprof.json --fetch F --write W [--kernel ...]
        rewrite an under-rocprof bench record's roofline.traffic from ITS OWN PMC files (no table entry)
"""
import argparse
import csv
import glob
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TABLE = os.path.join(ROOT, "profiles", "pmc_traffic.json")
CORRECTION = ("bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE counts half of 16B/lane streaming reads, "
              "MI355X_MICROARCH.md HBM section)")


def per_dispatch(path, counter, kernel_substr):
    files = [path] if os.path.isfile(path) else glob.glob(os.path.join(path, "**", "*counter_collection.csv"),
                                                           recursive=True)
    vals = {}
    for f in files:
        for row in csv.DictReader(open(f)):
            if row.get("Counter_Name") != counter or kernel_substr not in row.get("Kernel_Name", ""):
                continue
            did = row.get("Dispatch_Id")
            vals[did] = vals.get(did, 0.0) + float(row["Counter_Value"])
    return list(vals.values())


def traffic_per_launch(fetch, write, kern: str, launches: int):
    """HBM bytes per launch of the step's kernels: kern "a*4+b*1" = a step of 4 launches of a and 1 of b."""
    terms = [(t.split("*")[0], int(t.split("*")[1]) if "*" in t else 1) for t in kern.split("+")]
    fkb = wkb = 0.0
    ndisp = 0
    for name, count in terms:
        f = per_dispatch(fetch, "FETCH_SIZE", name)
        w = per_dispatch(write, "WRITE_SIZE", name)
        if not f or not w:
            raise SystemExit(f"no {name} dispatches found (fetch {len(f)}, write {len(w)})")
        scale = count / launches if len(terms) > 1 else 1.0
        fkb += scale * sum(f) / len(f)
        wkb += scale * sum(w) / len(w)
        ndisp += len(f)
    return (2 * fkb + wkb) * 1024, fkb, wkb, ndisp


def key_of(workload, resident, launches, build_id) -> str:
    return f"{workload}|C{resident}|L{launches}|{build_id}"


def bench_key(line: dict) -> tuple:
    """(key, fields) of a bench.py JSON line: its workload, resident clients per pass, launches per round, build."""
    r = line["roofline"]
    f = {"workload": line["config"]["workload"], "resident_clients": r["resident_clients"],
         "launches_per_step": r["launches_per_step"], "build_id": line["build_id"]}
    return key_of(f["workload"], f["resident_clients"], f["launches_per_step"], f["build_id"]), f


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bench", help="the bench.py JSON line of the profiled command (a file)")
    ap.add_argument("--fix-profile", help="an under-rocprof bench record to correct in place")
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--kernel", default=None)
    a = ap.parse_args()
    src = a.bench or a.fix_profile
    line = json.loads([ln for ln in open(src).read().splitlines() if ln.startswith("{")][-1])
    r = line["roofline"]
    launches = int(r["launches_per_step"])
    kern = a.kernel or ("k_qfed_accum" if line["config"].get("policy") == "qfedavg" else
                        "k_reduce*%d+k_yogi_step*1" % (launches - 1) if line["config"].get("policy") == "fedyogi"
                        else "k_reduce")
    hbm, fkb, wkb, nd = traffic_per_launch(a.fetch, a.write, kern, launches)
    alg = float(r["alg_bytes_per_launch"])
    if a.fix_profile:
        r["traffic"] = hbm
        r["traffic_source"] = {"fetch": os.path.relpath(a.fetch, ROOT), "write": os.path.relpath(a.write, ROOT),
                               "kernel": kern, "traffic_over_alg": hbm / alg, "correction": CORRECTION}
        with open(a.fix_profile, "w") as f:
            f.write(json.dumps(line) + "\n")
        print(a.fix_profile, "traffic", hbm, "ratio", hbm / alg)
        return
    key, fields = bench_key(line)
    db = json.load(open(TABLE)) if os.path.exists(TABLE) else {}
    entries = db.setdefault("entries", {})
    entries[key] = dict(fields, kernel=kern, dispatches=nd, FETCH_SIZE_KiB=fkb, WRITE_SIZE_KiB=wkb,
                        hbm_bytes_per_launch=hbm, alg_bytes_per_launch=alg, traffic_over_alg=hbm / alg,
                        fetch=os.path.relpath(a.fetch, ROOT), write=os.path.relpath(a.write, ROOT),
                        correction=CORRECTION)
    json.dump(db, open(TABLE, "w"), indent=1, sort_keys=True)
    print(key, json.dumps(entries[key]))


if __name__ == "__main__":
    main()
