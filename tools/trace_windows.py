#!/usr/bin/env python3
"""Per-step / per-window breakdown of a rocprofv3 kernel trace of bench.py (tests/gpu_trace.sh).

A window ends with its k_next dispatch; a PBFT step (one 50 ms block interval) holds one
k_pbft_tick.  For the steps after the first `--skip` ticks this prints, per step, the wall span
from its first dispatch to the last, the GPU-busy time (union of dispatch intervals), the idle
gaps between dispatches (host round trips: read-backs, launch latency) and the kernel time by
kernel name.
  python3 tools/trace_windows.py gpurun_out/trace/.../kt_kernel_trace.csv [--skip 6] [--windows]
"""
import argparse
import csv
import collections
import re


def short(name):
    n = re.sub(r"\(.*$", "", name).replace("bcsim::", "").replace("void ", "")
    return n.strip()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--skip", type=int, default=6, help="ticks (steps) to skip: warm-up")
    ap.add_argument("--windows", action="store_true", help="print every window of the analysed steps")
    a = ap.parse_args()
    rows = []
    with open(a.csv) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    rows.sort()
    ticks = [k for k, r in enumerate(rows) if r[2] == "k_pbft_tick"]
    if len(ticks) <= a.skip:
        start = 0
    else:
        start = ticks[a.skip - 1] + 1 if a.skip else 0
    sel = rows[start:]
    # split into steps at the ticks
    steps, cur = [], []
    for r in sel:
        cur.append(r)
        if r[2] == "k_pbft_tick":
            steps.append(cur)
            cur = []
    if cur:
        steps.append(cur)
    tot = collections.Counter()
    tot_busy = tot_span = tot_gap = 0
    nwin = 0
    for si, st in enumerate(steps):
        span = st[-1][1] - st[0][0]
        busy, gaps, last_end = 0, 0, st[0][0]
        by = collections.Counter()
        for s, e, n in st:
            if s > last_end:
                gaps += s - last_end
            busy += max(0, e - max(s, last_end))
            last_end = max(last_end, e)
            by[n] += e - s
        w = sum(1 for r in st if r[2] == "k_next")
        nwin += w
        tot.update(by)
        tot_busy += busy
        tot_span += span
        tot_gap += gaps
        print(f"step {si}: span {span / 1e3:.1f} us, busy {busy / 1e3:.1f}, gaps {gaps / 1e3:.1f}, windows {w}, "
              f"dispatches {len(st)}")
        if a.windows:
            wk = []
            for s, e, n in st:
                wk.append(f"{n}:{(e - s) / 1e3:.0f}")
                if n == "k_next":
                    print("   ", " ".join(wk))
                    wk = []
            if wk:
                print("   ", " ".join(wk))
    ns = max(1, len(steps))
    print(f"\nper step (mean of {len(steps)}): span {tot_span / ns / 1e3:.1f} us, busy {tot_busy / ns / 1e3:.1f}, "
          f"gaps {tot_gap / ns / 1e3:.1f}, windows {nwin / ns:.1f}")
    for n, v in tot.most_common():
        print(f"  {n:45s} {v / ns / 1e3:9.1f} us/step")


if __name__ == "__main__":
    main()
