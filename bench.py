#!/usr/bin/env python3
"""bench.py — delivered consensus msgs/sec, PBFT n=4096 (BASELINE.json metric).

Workload (BASELINE.json configs[3], the config the metric names): PBFT on an
N=4096 full mesh (16.8 M directed 3 Mbps / 3 ms links), reference block size
(50 KB) and fixed 3 ms app delay, synthetic (no dataset exists).  One "step"
is one PBFT block interval: 50 ms (Seconds(0.05f)) of simulated time in which
the leader ticks once and every node runs its prepare/commit traffic.

Multi-GPU (BASELINE configs[3]: "1/2/4/8 MI355X node-partitioned PDES"): one
process per GPU; by default the SAME n=4096 network is node-partitioned over
the ranks (contiguous node ranges, cross-rank records exchanged
by RCCL all-to-all over xGMI once per lookahead cell), so total work is fixed
("scaling": "strong") and `value` = msgs delivered on all ranks / max wall time
over ranks.  `--mode replicas` runs one independent replica per rank instead
("scaling": "weak"); it is also the fallback if the RCCL partition cannot be
set up (reported in config.parallelism).

Prints ONE JSON line on rank 0 with metric/value/roofline/cpu_baseline.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [REPO, os.path.join(REPO, "blockchain-simulator_amd")]

METRIC = "delivered consensus msgs/sec (whole node), PBFT n=4096; committed rounds/sec"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


def make_cfg(n_nodes, rounds, device, workload="pbft", replicas=1):
    import bcsim
    c = bcsim.preset({"pbft": "c4_pbft4096", "gossip": "c5_gossip65536", "paxos": "c3_paxos"}[workload])
    c.n_nodes = n_nodes
    c.n_replicas = replicas
    c.pbft_rounds = rounds
    c.device = device
    c.stop_ns = -1
    return c


def make_topology(n_nodes, workload):
    """None = the reference's full mesh; gossip: random 8-regular graph, seed 1."""
    if workload != "gossip":
        return None
    import bcsim
    return bcsim.random_regular(n_nodes, 8, 1)


PMC_ROUNDS = ("r06", "r05")  # newest first: the committed PMC summaries this line reads


def pmc_name(n_nodes, workload="pbft", replicas=1, queue="infinite", jitter=False):
    """profiles/<round>_pmc_<name>.json: the workload's PMC summary (tests/gpu_prof.sh with the
    same bench arguments, tools/pmc_summary.py)."""
    name = f"{workload}{n_nodes}"
    if replicas > 1:
        name += f"_r{replicas}"
    if queue != "infinite":
        name += f"_{queue}"
    if jitter:
        name += "_jitter"
    return name


def pmc_traffic(n_nodes, kernel="bcsim::k_link", workload="pbft", replicas=1, queue="infinite", jitter=False):
    """(HBM bytes per launch of `kernel`, source file) from the newest committed rocprofv3 PMC
    summary of this workload (tools/pmc_summary.py over tests/gpu_prof.sh: FETCH_SIZE x2 gfx950
    correction + WRITE_SIZE, separate passes), over the bench's own timed window of dispatches
    when the summary has it; (None, None) if absent."""
    name = pmc_name(n_nodes, workload, replicas, queue, jitter)
    for rnd in PMC_ROUNDS:
        path = os.path.join(REPO, "profiles", f"{rnd}_pmc_{name}.json")
        try:
            with open(path) as f:
                ks = json.load(f)["kernels"]
        except (OSError, KeyError, ValueError):
            continue
        v = _pmc_kernel(ks, kernel)
        if v is not None:
            return v, os.path.relpath(path, REPO)
    return None, None


def _pmc_kernel(ks, kernel):
    # the k_link class as the bench times it (fast path + looped generic kernel)
    if "link_class" in ks and kernel == "bcsim::k_link":
        return ks["link_class"]["timed_window"]["hbm_bytes_per_launch"]
    # templated kernels (k_link<QM, XR>): the instantiation with the most dispatches
    cands = [v for k, v in ks.items() if k == kernel or k.startswith(kernel + "<")]
    if not cands:
        return None
    best = max(cands, key=lambda v: v.get("dispatches", 0))
    return best.get("timed_window", {}).get("hbm_bytes_per_launch", best["hbm_bytes_per_launch"])


def host_cpu():
    """CPU model and logical core count of this host (for the cpu_baseline line)."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return model, os.cpu_count()


def commit_records(sim, workload):
    """Commit-kind trace records so far (PBFT commit lines, gossip first receipts)."""
    import bcsim
    kind = {"pbft": bcsim.TR["PBFT_COMMIT"], "gossip": bcsim.TR["GOSSIP_DELIVER"], "paxos": bcsim.TR["PAXOS_COMMIT"]}[workload]
    return sum(1 for r in sim.trace() if r[6] == kind)


def cpu_baseline(n_nodes, budget_s, workload="pbft", tweak=None):
    """Serial oracle DES (same semantics) on the host: a bounded time slice of
    the same workload, run from t=0 in 1 ms slices until budget_s of CPU."""
    import oracle
    cfg = make_cfg(n_nodes, 100, 0, workload)  # one replica (the oracle runs replicas serially)
    if tweak:
        tweak(cfg)
    o = oracle.OracleSim(cfg)
    topo = make_topology(n_nodes, workload)
    if topo is not None:
        o.set_topology(*topo)
    t0 = time.process_time()
    w0 = time.time()
    t = 0
    while time.process_time() - t0 < budget_s:
        t += 1_000_000
        o.run(t)
        if o.status()["quiescent"]:
            break
    cpu = time.process_time() - t0
    wall = time.time() - w0
    cnt = o.counters()
    o.close()
    model, nproc = host_cpu()
    return dict(value=cnt["delivered_total"] / max(cpu, 1e-9), unit="msgs/s", cores=1, kind="port",
                cpu_model=model, nproc=nproc,
                sample=f"oracle DES (serial, one core of {nproc}: {model}), {workload} n={n_nodes}, "
                       f"first {t / 1e6:.0f} ms simulated ({cnt['delivered_total']} msgs, {cpu:.1f} s CPU, "
                       f"{wall:.1f} s wall)")


def _oracle_slice(cfg_fields, budget_s):
    """One worker of the all-cores baseline: a single-replica oracle run of budget_s CPU."""
    sys.path[:0] = [REPO, os.path.join(REPO, "blockchain-simulator_amd")]
    import oracle
    from bcsim import _abi
    cfg = _abi.Config()
    for k, v in cfg_fields.items():
        if k == "reserved":
            for i, x in enumerate(v):
                cfg.reserved[i] = x
        else:
            setattr(cfg, k, v)
    o = oracle.OracleSim(cfg)
    t0 = time.process_time()
    t = 0
    while time.process_time() - t0 < budget_s:
        t += 1_000_000
        o.run(t)
        if o.status()["quiescent"]:
            break
    n = o.counters()["delivered_total"]
    o.close()
    return n, time.process_time() - t0


def cpu_baseline_all_cores(n_nodes, budget_s, workload, tweak, cores):
    """Monte Carlo replicas are independent (all-cores figure for the replica
    config): `cores` oracle processes, one replica each (different seeds), run side by side;
    value = their summed deliveries / the wall time."""
    import multiprocessing as mp
    from bcsim import _abi
    cfg = make_cfg(n_nodes, 100, 0, workload)
    if tweak:
        tweak(cfg)
    jobs = []
    for k in range(cores):
        d = _abi.config_dict(cfg)
        d["seed"] = cfg.seed + k
        jobs.append(d)
    w0 = time.time()
    with mp.get_context("spawn").Pool(cores) as pool:
        res = pool.starmap(_oracle_slice, [(d, budget_s) for d in jobs])
    wall = time.time() - w0
    msgs = sum(r[0] for r in res)
    cpu = sum(r[1] for r in res)
    model, nproc = host_cpu()
    return dict(value=msgs / wall, unit="msgs/s", cores=cores, kind="port", cpu_model=model, nproc=nproc,
                sample=f"{cores} oracle processes side by side, one {workload} n={n_nodes} replica each (seeds "
                       f"differ), each until {budget_s:.0f} s CPU or the end of its run ({msgs} msgs, {cpu:.1f} s CPU "
                       f"in total, {wall:.1f} s wall incl. process start)")


def aggregate(dist, device, dt, msgs, trace_delta):
    """Whole-job numbers over ranks: max wall time, summed work (the per-rank
    deliveries of a partitioned run, or of independent replicas)."""
    if dist is None:
        return dt, msgs, trace_delta
    import torch
    t = torch.tensor([dt], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    m = torch.tensor([float(msgs), float(trace_delta)], dtype=torch.float64, device=device)
    dist.all_reduce(m, op=dist.ReduceOp.SUM)
    return float(t.item()), int(m[0].item()), int(m[1].item())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--warmup", type=int, default=6)
    ap.add_argument("--workload", choices=("pbft", "gossip", "paxos"), default="pbft",
                    help="pbft: BASELINE configs[3] (the metric); gossip: configs[4], random 8-regular graph; "
                         "paxos: configs[2] shape (jittered links, batched Monte Carlo replicas)")
    ap.add_argument("--nodes", type=int, default=0, help="default 4096 (pbft, paxos) / 65536 (gossip)")
    ap.add_argument("--replicas", type=int, default=0,
                    help="paxos: replicas in one engine (default 10000 = configs[2], sparse layout)")
    ap.add_argument("--decrees", type=int, default=2, help="paxos: decrees per proposer (multi-decree extension)")
    ap.add_argument("--cpu-budget", type=float, default=20.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--engine", choices=("auto", "dense", "sparse"), default="auto",
                    help="engine layout (DESIGN.md §4): per-edge inbox slots or sparse bucket lists")
    ap.add_argument("--jitter", action="store_true",
                    help="pbft: the reference's default getRandomDelay() app delay (3-5 ms per send, "
                         "pbft-node.cc:66-69) with the counter RNG, instead of the fixed 3 ms")
    ap.add_argument("--mode", choices=("pdes", "replicas"), default="pdes",
                    help="multi-GPU mode (N>1): node-partitioned PDES or independent replicas")
    ap.add_argument("--queue", choices=("infinite", "droptail", "fqcodel"), default="infinite",
                    help="link queue model: the reference's unbounded FIFO reading (default), or the "
                         "device queue + pfifo_fast / FqCoDel root queue disc (DESIGN.md §2.2, §2.2b)")
    ap.add_argument("--pdes1", action="store_true",
                    help="one GPU with the partition machinery on (a world-1 RCCL group, the per-window "
                         "control exchange): its cost against the plain single-GPU run")
    args = ap.parse_args()
    if args.nodes <= 0:
        args.nodes = 65536 if args.workload == "gossip" else 4096
    if args.replicas <= 0:  # configs[2]: 10k batched Monte Carlo replicas
        args.replicas = 10000 if args.workload == "paxos" else 1

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    dist = None
    if world > 1 or args.pdes1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        if world == 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29561")
            dist.init_process_group("nccl", rank=0, world_size=1)
        else:
            dist.init_process_group("nccl")

    # HIP-event timing around the k_link class only inside the timed region (an event pair
    # costs a few us of dispatch per launch); the other classes are timed in an extra
    # untimed breakdown pass after it
    os.environ.setdefault("BCSIM_KSTATS", "2")  # (a diagnostic run may time more classes)
    import bcsim
    period = 50_000_001  # Seconds(0.05f) in ns (round mode)
    cfg = make_cfg(args.nodes, args.warmup + 2 * args.steps + 4, local, args.workload, args.replicas)
    if args.workload == "paxos":
        cfg.paxos_decrees = args.decrees
    cfg.engine_mode = {"auto": bcsim.ENGINE_AUTO, "dense": bcsim.ENGINE_DENSE, "sparse": bcsim.ENGINE_SPARSE}[args.engine]
    if args.jitter and args.workload == "pbft":
        cfg.delay_mode = bcsim.DELAY_RANDOM
        cfg.rng_mode = bcsim.RNG_COUNTER
        cfg.app_delay_ns = 0
    cfg.queue_model = {"infinite": bcsim.QUEUE_INFINITE, "droptail": bcsim.QUEUE_DROPTAIL,
                       "fqcodel": bcsim.QUEUE_FQCODEL}[args.queue]
    topo = make_topology(args.nodes, args.workload)

    def new_sim():
        sm = bcsim.Simulator(cfg)
        if topo is not None:
            sm.set_topology(*topo)
        return sm
    sim = new_sim()
    mode = "single"
    if dist is not None:
        mode = args.mode
        if mode == "pdes":
            err = ""
            try:
                sim.set_partition(dist, transport="rccl")
            except Exception as e:  # every rank must agree before the first collective run
                err = repr(e)
            ok = torch.tensor([0 if err else 1], dtype=torch.int64, device=f"cuda:{local}")
            dist.all_reduce(ok, op=dist.ReduceOp.MIN)
            if not int(ok.item()):
                print(f"[bench] rank {rank}: RCCL partition unavailable ({err or 'peer failed'}); "
                      f"falling back to replicas", file=sys.stderr, flush=True)
                sim.close()
                sim = new_sim()
                mode = "replicas"

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize(local)

    # warmup: fill the pipeline (first block needs ~135 ms to serialize)
    t_sim = 0
    for k in range(args.warmup):
        t_sim += period
        w = time.perf_counter()
        sim.run(t_sim)
        if rank == 0:
            print(f"[bench] warmup {k}: {time.perf_counter() - w:.2f}s msgs={sim.counters()['delivered_total']}",
                  file=sys.stderr, flush=True)
    c0 = sim.counters()
    cm0 = commit_records(sim, args.workload)
    link_before = sim.kernel_stats()["link"]["launches"]  # k_link launches before the timed region
    ls0 = sim.loop_stats()
    hs0 = sim.host_stats()
    sim.reset_kernel_stats()
    barrier()
    w0 = time.perf_counter()
    for _ in range(args.steps):
        t_sim += period
        sim.run(t_sim)
    barrier()
    dt = time.perf_counter() - w0
    c1 = sim.counters()
    ks = sim.kernel_stats()
    ls1 = sim.loop_stats()
    loop = {k: ls1[k] - ls0[k] for k in ls1}
    hs1 = sim.host_stats()
    host = {k: hs1[k] - hs0[k] for k in hs1}
    msgs = c1["delivered_total"] - c0["delivered_total"]
    commits = commit_records(sim, args.workload) - cm0
    dt, msgs, commits = aggregate(dist, f"cuda:{local}", dt, msgs, commits)
    # breakdown pass (untimed): every kernel class timed.  One process: a fresh engine replays
    # the warm-up and then the timed window's steps (the same simulated interval -- a run can
    # go quiet after it, e.g. PBFT under FQCODEL); node-partitioned: as many steps after it
    os.environ["BCSIM_KSTATS"] = "15"
    if dist is None:
        sim.close()
        sim = new_sim()
        t_sim = 0
        for _ in range(args.warmup):
            t_sim += period
            sim.run(t_sim)
    sim.reset_kernel_stats()
    for _ in range(args.steps):
        t_sim += period
        sim.run(t_sim)
    ks_all = sim.kernel_stats()
    sim.close()

    if rank == 0:
        # committed rounds: commit-kind records / N (every node commits each block;
        # block / stop / view records are not counted)
        rounds = commits / args.nodes
        dom = max(("scan", "link", "group", "aux"), key=lambda k: ks_all[k]["us"])
        lk = ks["link"]
        # roofline of the scatter (k_link): SURVEY.md §8(d) algorithmic bytes = 48 B per record
        # emitted by the timed k_link launches, over their HIP-event time on the engine stream
        ach = (lk["bytes"] / 1e9) / (lk["us"] / 1e6) if lk["us"] > 0 else 0.0
        # PMC traffic of this workload's committed profile (same bench arguments)
        traffic, traffic_src = pmc_traffic(args.nodes, workload=args.workload, replicas=args.replicas,
                                           queue=args.queue, jitter=args.jitter)
        avg_us = lk["us"] / max(1, lk["launches"])
        all_us = sum(v["us"] for v in ks_all.values())
        if args.workload == "pbft":
            data = "synthetic (PBFT n=%d full mesh, 3Mbps/3ms links, 50KB blocks, %s)" % (
                args.nodes, "app delay U{3,4,5} ms per send, counter RNG" if args.jitter else "fixed 3 ms app delay")
            wl = f"PBFT n={args.nodes} full O(n^2) prepare/commit (BASELINE configs[3])"
            if args.queue != "infinite":
                data = data[:-1] + f", {args.queue} link queues)"
                wl += f", {args.queue} link queues"
        elif args.workload == "paxos":
            data = ("synthetic (Paxos n=%d full mesh, 3Mbps/3ms links, app delay U{0..49} ms, counter RNG, "
                    "%d replicas, %d decrees, seeds by replica, sparse layout)" % (args.nodes, args.replicas, args.decrees))
            wl = (f"Paxos n={args.nodes} multi-decree ({args.decrees}), jittered links, {args.replicas} batched "
                  f"Monte Carlo replicas (BASELINE configs[2])")
        else:
            data = ("synthetic (PBFT-style gossip, n=%d random 8-regular graph seed 1, 3Mbps/3ms links, "
                    "1000 B blocks, fixed 3 ms app delay)" % args.nodes)
            wl = f"PBFT-style gossip n={args.nodes} random 8-regular (BASELINE configs[4])"
        lk_launch_bytes = lk["bytes"] / max(1, lk["launches"])
        # the whole scan -> link pipeline priced the same way: 48 B per record over the time of
        # both classes (untimed breakdown pass, every class timed)
        sl_us = ks_all["scan"]["us"] + ks_all["link"]["us"]
        pipe_ach = (ks_all["link"]["bytes"] / 1e9) / (sl_us / 1e6) if sl_us > 0 else 0.0
        impl_launch_bytes = ks["aux"]["bytes"] / max(1, lk["launches"])
        out = {
            "metric": METRIC,
            "value": msgs / dt,
            "unit": "msgs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1000.0 * dt / args.steps,
            "higher_is_better": True,
            "scaling": "strong" if mode == "pdes" else "weak",
            "vs_baseline": None,
            "dtype": "int64",
            "data": data,
            "config": {"workload": wl,
                       "nodes": args.nodes, "step": "one 50 ms block interval",
                       "engine": args.engine,
                       "link_queue": {"infinite": "unbounded FIFO per link (no queue disc)",
                                      "droptail": "100-packet device queue + pfifo_fast",
                                      "fqcodel": "100-packet device queue + FqCoDel"}[args.queue],
                       "parallelism": f"{mode}{world}" if world > 1 or args.pdes1 else "single"},
            "committed_rounds_per_s": rounds / dt,
            "roofline": {"kernel": "k_link (inbox scatter)", "bound": "hbm", "achieved": ach,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": ach / HBM_PEAK_GBS,
                         "traffic": traffic, "algorithmic_bytes_per_launch": lk_launch_bytes,
                         "bytes_per_record": 48, "records": lk["bytes"] / 48.0,
                         "implementation_bytes_per_launch": impl_launch_bytes,
                         # the measured HBM bytes per launch (PMC) over the same time, and their
                         # ratio to the algorithmic bytes: < 1 where the heavy waves' records travel
                         # as summaries, > 1 where bytes are re-read
                         "traffic_GBs": (traffic / 1e9) / (avg_us / 1e6) if traffic and avg_us > 0 else None,
                         # what the hardware moved: the PMC bytes per launch over this line's average
                         # launch time, against the peak (frac prices the algorithmic bytes)
                         "hw_frac": (traffic / 1e9) / (avg_us / 1e6) / HBM_PEAK_GBS if traffic and avg_us > 0 else None,
                         "traffic_source": traffic_src,
                         "traffic_over_algorithmic": traffic / lk_launch_bytes if traffic and lk_launch_bytes else None,
                         "avg_launch_us": lk["us"] / max(1, lk["launches"]),
                         "launches": lk["launches"],
                         # the timed launches are k_link dispatches [first, first + launches) of the
                         # process: tools/pmc_summary.py restricts rocprofv3 traces to them
                         "first_timed_launch": link_before,
                         "dominant_kernel_class": dom,
                         "pipeline": {"kernels": "k_scan + k_link classes", "achieved": pipe_ach,
                                      "frac": pipe_ach / HBM_PEAK_GBS, "us": sl_us,
                                      "records": ks_all["link"]["bytes"] / 48.0}},
            # the cell loop over the timed steps (rank 0): windows, host syncs (spins, stream syncs,
            # blocking collectives), windows run as device-chained windows
            "loop": {"windows_per_step": loop["windows"] / args.steps,
                     "host_syncs_per_window": loop["host_syncs"] / max(1, loop["windows"]),
                     "chain_windows": loop["chain_windows"], "spec_hits": loop["spec_hits"],
                     "idle_parts": loop["idle_parts"], "collectives": loop["collectives"],
                     # host time per step inside kernel launches / waiting on the mirror words
                     "host_launch_us_per_step": host["launch_us"] / args.steps,
                     "host_wait_us_per_step": host["wait_us"] / args.steps,
                     "launches_per_step": host["launches"] / args.steps,
                     "chained_frontier_hits": host["frontier_hits"]},
            "kernel_us": {k: v["us"] for k, v in ks.items()},
            "kernel_launches": {k: v["launches"] for k, v in ks.items()},
            # untimed pass of as many steps with every kernel class timed (the timed region
            # times k_link only)
            "breakdown": {"kernel_us": {k: v["us"] for k, v in ks_all.items()},
                                 "kernel_launches": {k: v["launches"] for k, v in ks_all.items()},
                                 "records": ks_all["link"]["bytes"] / 48.0,
                                 "pipeline_frac": ((ks_all["link"]["bytes"] / 1e9) / (all_us / 1e6) / HBM_PEAK_GBS
                                                   if all_us else 0.0)},
        }
        if not args.no_cpu_baseline and world == 1:
            try:
                def tweak(c):
                    c.delay_mode, c.rng_mode, c.app_delay_ns = cfg.delay_mode, cfg.rng_mode, cfg.app_delay_ns
                    c.queue_model = cfg.queue_model
                    if args.workload == "paxos":
                        c.paxos_decrees = args.decrees
                out["cpu_baseline"] = cpu_baseline(args.nodes, args.cpu_budget, args.workload, tweak)
                if args.workload == "paxos":  # replicas: the all-cores figure too (16 = the box's CPU share)
                    out["cpu_baseline_all_cores"] = cpu_baseline_all_cores(
                        args.nodes, args.cpu_budget, args.workload, tweak, min(16, os.cpu_count() or 1))
            except Exception as e:  # never let the baseline leg kill the GPU number
                out["cpu_baseline"] = {"error": str(e)}
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
