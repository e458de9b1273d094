"""Per (kernel, grid) averages from a rocprofv3 --kernel-trace CSV: one bench.py run times several configs whose
launches differ in grid size, so the rocprof figures of each config are the rows of its own shape.
usage: python tools/trace_by_shape.py trace.csv [min_dispatches]"""
import collections
import csv
import json
import sys


def main(path, min_n=2):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        grid = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
        wg = int(r["Workgroup_Size_X"]) * int(r["Workgroup_Size_Y"]) * int(r["Workgroup_Size_Z"])
        key = (r["Kernel_Name"].split("(")[0][:90], grid, wg)
        acc[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    rows = []
    for (name, grid, wg), d in acc.items():
        if len(d) < min_n:
            continue
        d.sort()
        rows.append({"kernel": name, "grid": grid, "workgroup": wg, "dispatches": len(d),
                     "mean_us": sum(d) / len(d), "median_us": d[len(d) // 2], "min_us": d[0], "max_us": d[-1],
                     "total_ms": sum(d) / 1e3})
    rows.sort(key=lambda x: -x["total_ms"])
    for x in rows:
        print(json.dumps(x))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 2)
