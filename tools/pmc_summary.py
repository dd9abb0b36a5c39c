"""Summarise rocprofv3 PMC passes (tests/gpu_prof.sh) into per-kernel HBM traffic.

FETCH_SIZE / WRITE_SIZE are rocprofv3 derived counters in KiB per dispatch
(TCC_EA0_RDREQ / _WRREQ based).  Per MI355X_MICROARCH.md §HBM, on gfx950
FETCH_SIZE reports half the bytes of wide coalesced streaming reads, so the
read side is doubled; WRITE_SIZE is exact for 16-B-per-lane stores.

  python tools/pmc_summary.py gpurun_out/prof_r01 profiles/r01_pmc.json
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


def main(src, dst):
    fetch, names = per_dispatch(f"{src}/fetch/run_counter_collection.csv")
    write, names_w = per_dispatch(f"{src}/write/run_counter_collection.csv")
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
    json.dump(dict(source=src, correction="FETCH_SIZE x2 (gfx950), KiB->bytes", kernels=res),
              open(dst, "w"), indent=1)
    for k, v in res.items():
        print(f"{k:28s} {v['dispatches']:4d} disp  HBM/launch {v['hbm_bytes_per_launch'] / 1e6:10.2f} MB  "
              f"L2 hit {v['l2_hit_rate']:.2f}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
