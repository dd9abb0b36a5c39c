#!/usr/bin/env python3
"""Per-kernel statistics of a rocprofv3 kernel trace restricted to bench.py's timed window.

rocprofv3 --stats covers the whole process: engine setup, the warm-up steps and (Paxos C3) the
t = 0 START window of every gnode, which can dominate the file without being part of what the
bench times.  This restricts the trace to the dispatches from the first to the last k_link-class
launch of the timed window (the bench line's roofline.first_timed_launch / .launches; the class
and its grouping into launches as tools/pmc_summary.py defines them) and writes the usual
columns (Name, Calls, TotalDurationNs, AverageNs, Percentage, MinNs, MaxNs) plus the window.

  python tools/window_stats.py <trace dir>/run_kernel_trace.csv <bench line .log/.json> out.csv
"""
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import link_groups  # noqa: E402


def bench_window(path):
    for line in open(path):
        if line.startswith("{"):
            r = json.loads(line)["roofline"]
            return int(r["first_timed_launch"]), int(r["launches"])
    raise SystemExit(f"no bench line in {path}")


def main(trace, line, out):
    first, n = bench_window(line)
    rows = list(csv.DictReader(open(trace)))
    names = {int(r["Dispatch_Id"]): r["Kernel_Name"].split("(")[0].replace("void ", "") for r in rows}
    groups = link_groups(names)[first:first + n]
    if not groups:
        raise SystemExit("timed window not in the trace")
    lo, hi = groups[0][0], groups[-1][-1]
    # the window runs to the k_next that closes its last launch's window
    after = sorted(d for d in names if d > hi and names[d].startswith("bcsim::k_next"))
    if after:
        hi = after[0]
    stats = {}
    for r in rows:
        d = int(r["Dispatch_Id"])
        if not lo <= d <= hi:
            continue
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        dur = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        s = stats.setdefault(k, [0, 0, 1 << 62, 0])
        s[0] += 1
        s[1] += dur
        s[2] = min(s[2], dur)
        s[3] = max(s[3], dur)
    tot = sum(v[1] for v in stats.values()) or 1
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs",
                    "Window"])
        for k, v in sorted(stats.items(), key=lambda kv: -kv[1][1]):
            w.writerow([k, v[0], v[1], v[1] / v[0], 100.0 * v[1] / tot, v[2], v[3],
                        f"dispatches [{lo}, {hi}] = link launches [{first}, +{n})"])
    print(f"timed window: dispatches [{lo}, {hi}], {sum(v[0] for v in stats.values())} dispatches, "
          f"{tot / 1e6:.2f} ms of kernel time")


if __name__ == "__main__":
    main(*sys.argv[1:4])
