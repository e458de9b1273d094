"""VALU issue figures of one kernel from a rocprofv3 --pmc pass of SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES
SQ_BUSY_CYCLES GRBM_GUI_ACTIVE (tools/pmc_qfed_r02.sh).  Capacity: each SIMD issues one wave64 VALU instruction
per 2 cycles (MI355X_MICROARCH.md), 256 CUs x 4 SIMDs; GRBM_GUI_ACTIVE / 8 XCDs = the kernel's cycles.
usage: python tools/pmc_valu_parse.py <pmc_dir> <kernel_substr> <fp32_elements_per_launch>"""
import csv
import glob
import json
import os
import sys

CTRS = ("SQ_INSTS_VALU", "SQ_ACTIVE_INST_VALU", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "GRBM_GUI_ACTIVE")


def main():
    d, kern, elems = sys.argv[1], sys.argv[2], float(sys.argv[3])
    per = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if kern not in row.get("Kernel_Name", "") or row.get("Counter_Name") not in CTRS:
                continue
            dd = per.setdefault(row["Dispatch_Id"], {})
            dd[row["Counter_Name"]] = dd.get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
    if not per:
        raise SystemExit(f"no {kern} dispatches in {d}")
    avg = {c: sum(p.get(c, 0.0) for p in per.values()) / len(per) for c in CTRS}
    cyc = avg["GRBM_GUI_ACTIVE"] / 8
    cap = cyc * 256 * 4 / 2
    print(json.dumps({"kernel": kern, "dispatches": len(per), "per_dispatch": avg, "kernel_cycles_per_xcd": cyc,
                      "valu_wave_instr_capacity": cap, "valu_issue_utilization": avg["SQ_INSTS_VALU"] / cap,
                      "valu_active_over_wave_cycles": avg["SQ_ACTIVE_INST_VALU"] / avg["SQ_WAVE_CYCLES"],
                      "valu_lane_ops_per_fp32_element": avg["SQ_INSTS_VALU"] * 64 / elems}, indent=1))


if __name__ == "__main__":
    main()
