"""Per-launch durations and launch-to-launch gaps of one kernel in rocprofv3 kernel traces (--kernel-trace,
--output-format csv), and its busy time over the last ``steps`` of ``steps + warmup`` rounds.
usage: python tools/trace_gaps.py KERNEL_SUBSTRING STEPS WARMUP trace.csv [trace.csv ...]"""
import csv
import json
import statistics as st
import sys


def summary(path, name, steps, warmup):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    ks = [r for r in rows if name in r["Kernel_Name"]]
    dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in ks]
    gaps = [(int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3
            for a, b in zip(rows, rows[1:]) if name in a["Kernel_Name"] and name in b["Kernel_Name"]]
    per = len(ks) // (steps + warmup)
    timed = ks[-steps * per:]
    q = sorted(dur)
    return {"trace": path, "kernel": ks[0]["Kernel_Name"], "launches": len(ks), "launches_per_round": per,
            "dur_us": {"mean": st.mean(dur), "median": st.median(dur), "p10": q[len(q) // 10],
                       "p90": q[9 * len(q) // 10], "max": q[-1]},
            "gap_us": {"mean": st.mean(gaps), "median": st.median(gaps), "max": max(gaps)},
            "timed_rounds_busy_ms": sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in timed) / 1e6,
            "timed_rounds_span_ms": (int(timed[-1]["End_Timestamp"]) - int(timed[0]["Start_Timestamp"])) / 1e6}


if __name__ == "__main__":
    name, steps, warmup = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    for p in sys.argv[4:]:
        print(json.dumps(summary(p, name, steps, warmup)))
