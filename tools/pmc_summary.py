"""Summarise rocprofv3 PMC passes (tests/gpu_prof.sh) into per-kernel HBM traffic.

FETCH_SIZE / WRITE_SIZE are rocprofv3 derived counters in KiB per dispatch
(TCC_EA0_RDREQ / _WRREQ based).  Per MI355X_MICROARCH.md §HBM, on gfx950
FETCH_SIZE reports half the bytes of wide coalesced streaming reads, so the
read side is doubled; WRITE_SIZE is exact for 16-B-per-lane stores.

  python tools/pmc_summary.py gpurun_out/prof_r01 profiles/r01_pmc.json

The bench line of the profiled run (trace.log) names the timed window of its k_link
launches (roofline.first_timed_launch, roofline.launches); every k_link instantiation's
dispatches in that window get a "timed_window" entry: the rocprofv3 average duration (to
compare with the bench's HIP-event avg_launch_us) and the HBM bytes per launch.
"""
import csv
import json
import sys
from collections import defaultdict


def per_dispatch(path):
    out = defaultdict(dict)
    names = {}
    for r in csv.DictReader(open(path)):
        d = int(r["Dispatch_Id"])
        out[d][r["Counter_Name"]] = out[d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        names[d] = r["Kernel_Name"].split("(")[0].replace("void ", "")
    return out, names


def timed_window(src):
    """(first, count) of the bench's timed k_link launches, from the profiled bench line."""
    try:
        for line in open(f"{src}/trace.log"):
            if line.startswith("{"):
                r = json.loads(line)["roofline"]
                return int(r["first_timed_launch"]), int(r["launches"])
    except (OSError, KeyError, ValueError):
        pass
    return None


def kernel_durations(path, prefix):
    """Durations (ns) of the dispatches of kernels whose name starts with prefix, in order."""
    rows = [r for r in csv.DictReader(open(path)) if r["Kernel_Name"].replace("void ", "").startswith(prefix)]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    return [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows]


def main(src, dst):
    fetch, names = per_dispatch(f"{src}/fetch/run_counter_collection.csv")
    write, names_w = per_dispatch(f"{src}/write/run_counter_collection.csv")
    win = timed_window(src)
    res = {}
    for kern in sorted(set(names.values())):
        f = [v["FETCH_SIZE"] for d, v in fetch.items() if names[d] == kern and "FETCH_SIZE" in v]
        w = [v["WRITE_SIZE"] for d, v in write.items() if names_w[d] == kern and "WRITE_SIZE" in v]
        hit = [v.get("TCC_HIT_sum", 0.0) for d, v in write.items() if names_w[d] == kern]
        miss = [v.get("TCC_MISS_sum", 0.0) for d, v in write.items() if names_w[d] == kern]
        if not f or not w:
            continue
        fb = 2 * 1024 * sum(f) / len(f)       # gfx950 FETCH_SIZE correction (x2), KiB -> B
        wb = 1024 * sum(w) / len(w)
        res[kern] = dict(dispatches=len(f), fetch_bytes_per_launch=fb, write_bytes_per_launch=wb,
                         hbm_bytes_per_launch=fb + wb,
                         l2_hit_rate=(sum(hit) / max(1.0, sum(hit) + sum(miss))))
        if win and kern.startswith("bcsim::k_link"):
            a, n = win
            fd = [v["FETCH_SIZE"] for d, v in sorted(fetch.items()) if names[d] == kern and "FETCH_SIZE" in v][a:a + n]
            wd = [v["WRITE_SIZE"] for d, v in sorted(write.items()) if names_w[d] == kern and "WRITE_SIZE" in v][a:a + n]
            dur = kernel_durations(f"{src}/trace/run_kernel_trace.csv", kern)[a:a + n]
            if fd and wd:
                res[kern]["timed_window"] = dict(
                    first=a, launches=len(fd),
                    hbm_bytes_per_launch=2 * 1024 * sum(fd) / len(fd) + 1024 * sum(wd) / len(wd),
                    rocprof_avg_us=(sum(dur) / len(dur) / 1000.0) if dur else None)
    json.dump(dict(source=src, correction="FETCH_SIZE x2 (gfx950), KiB->bytes", kernels=res),
              open(dst, "w"), indent=1)
    for k, v in res.items():
        print(f"{k:28s} {v['dispatches']:4d} disp  HBM/launch {v['hbm_bytes_per_launch'] / 1e6:10.2f} MB  "
              f"L2 hit {v['l2_hit_rate']:.2f}")
        if "timed_window" in v:
            t = v["timed_window"]
            print(f"  timed window: dispatches [{t['first']}, +{t['launches']}) HBM/launch "
                  f"{t['hbm_bytes_per_launch'] / 1e6:.2f} MB, rocprof avg {t['rocprof_avg_us']} us")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
