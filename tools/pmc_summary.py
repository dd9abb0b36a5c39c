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

A timed "launch" of the k_link class is every link-stage dispatch of one window (fast-path
kernels -- k_link_mesh or k_mesh_prep + k_mesh_tile, k_gossip_cell, k_paxos_link -- and the
looped generic kernels over the nodes they hand on, both streams).  The "link_class" entry
groups them by window (k_next delimits windows) and reports the timed window over the groups
(bytes and durations summed over a group's dispatches): the figure bench.py compares with its
HIP-event time (which, with the second stream, is the span of the two streams, not the sum).
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


# the kernels of the k_link class as bench.py times it: the fast-path link kernels (full-mesh
# k_link_mesh, or the tiled k_mesh_prep + k_mesh_tile (summary mode: + k_mesh_row); dense gossip's fused kernel and its
# frontier pass; sparse Paxos) and the looped generic k_link / k_link_sparse over the nodes they
# hand on -- including the second stream's list-2 link stage
LINK_CLASS = {"bcsim::k_link", "bcsim::k_link_mesh", "bcsim::k_link_sparse", "bcsim::k_mesh_prep", "bcsim::k_mesh_row",
              "bcsim::k_mesh_tile", "bcsim::k_gossip_link", "bcsim::k_gossip_cell", "bcsim::k_gossip_active",
              "bcsim::k_paxos_link"}


def link_groups(names):
    """Dispatch ids of the k_link class grouped into bench launches: one launch per window,
    windows delimited by their k_next dispatch (see the module doc)."""
    groups, cur = [], []
    for d in sorted(names):
        n = names[d].split("<")[0]
        if n == "bcsim::k_next":
            if cur:
                groups.append(cur)
            cur = []
        elif n in LINK_CLASS:
            cur.append(d)
    if cur:
        groups.append(cur)
    return groups


def trace_durations(path):
    """Dispatch id -> duration (ns) from a rocprofv3 kernel trace."""
    return {int(r["Dispatch_Id"]): int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in csv.DictReader(open(path))}


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
    if win:  # the k_link class as the bench times it (fast path + looped generic kernel)
        a, n = win
        gf, gw = link_groups(names)[a:a + n], link_groups(names_w)[a:a + n]
        try:
            dur = trace_durations(f"{src}/trace/run_kernel_trace.csv")
            gt = link_groups({d: nm.split("(")[0].replace("void ", "") for d, nm in (
                (int(r["Dispatch_Id"]), r["Kernel_Name"]) for r in csv.DictReader(open(f"{src}/trace/run_kernel_trace.csv")))})[a:a + n]
        except OSError:
            dur, gt = {}, []
        if gf and gw:
            fb = 2 * 1024 * sum(fetch[d].get("FETCH_SIZE", 0.0) for g in gf for d in g) / len(gf)
            wb = 1024 * sum(write[d].get("WRITE_SIZE", 0.0) for g in gw for d in g) / len(gw)
            kinds = sorted({names[d] for g in gf for d in g})
            res["link_class"] = dict(kernels=kinds, timed_window=dict(
                first=a, launches=len(gf), hbm_bytes_per_launch=fb + wb,
                fetch_bytes_per_launch=fb, write_bytes_per_launch=wb,
                rocprof_avg_us=(sum(dur[d] for g in gt for d in g) / len(gt) / 1000.0) if gt else None))
    # SQ pass (when present): per kernel, the counters summed over its dispatches and the
    # stall / issue shares of the wave cycles
    try:
        sq, names_s = per_dispatch(f"{src}/sq/run_counter_collection.csv")
    except OSError:
        sq, names_s = {}, {}
    for kern in sorted(set(names_s.values())):
        tot = defaultdict(float)
        nd = 0
        for d, v in sq.items():
            if names_s[d] != kern:
                continue
            nd += 1
            for c, x in v.items():
                tot[c] += x
        cyc = tot.get("SQ_WAVE_CYCLES", 0.0)
        if kern in res and cyc > 0:
            res[kern]["sq"] = dict(dispatches=nd, counters_per_launch={c: x / nd for c, x in sorted(tot.items())},
                                   wait_any_frac=tot.get("SQ_WAIT_ANY", 0.0) / cyc,
                                   wait_inst_any_frac=tot.get("SQ_WAIT_INST_ANY", 0.0) / cyc,
                                   active_inst_any_frac=tot.get("SQ_ACTIVE_INST_ANY", 0.0) / cyc)
    json.dump(dict(source=src, correction="FETCH_SIZE x2 (gfx950), KiB->bytes", kernels=res),
              open(dst, "w"), indent=1)
    for k, v in res.items():
        if k == "link_class":
            t = v["timed_window"]
            print(f"link class {v['kernels']}: timed window [{t['first']}, +{t['launches']}) HBM/launch "
                  f"{t['hbm_bytes_per_launch'] / 1e6:.2f} MB, rocprof avg {t['rocprof_avg_us']} us")
            continue
        q = v.get("sq")
        sqs = (f"  wait {q['wait_any_frac']:.2f} issue {q['active_inst_any_frac']:.2f}" if q else "")
        print(f"{k:28s} {v['dispatches']:4d} disp  HBM/launch {v['hbm_bytes_per_launch'] / 1e6:10.2f} MB  "
              f"L2 hit {v['l2_hit_rate']:.2f}{sqs}")
        if "timed_window" in v:
            t = v["timed_window"]
            print(f"  timed window: dispatches [{t['first']}, +{t['launches']}) HBM/launch "
                  f"{t['hbm_bytes_per_launch'] / 1e6:.2f} MB, rocprof avg {t['rocprof_avg_us']} us")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
