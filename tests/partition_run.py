"""Node-partitioned parity driver: run a parity case on `world` ranks
(torch.distributed gloo, host-callback transport, all ranks on one GPU or on
the host emulator), merge the per-rank traces / counters and compare with the
oracle.  Used by tests/test_partition.py (GPU) and for emulator debugging:

    python tests/partition_run.py WORLD CASE [CASE...]
"""
import os
import socket
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tests"), os.path.join(REPO, "blockchain-simulator_amd")]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, names, transport, q):
    sys.path[:0] = [REPO, os.path.join(REPO, "tests"), os.path.join(REPO, "blockchain-simulator_amd")]
    import torch.distributed as dist
    import bcsim
    from parity_cases import any_case, topology
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        for name in names:
            cfg = any_case(name)
            try:
                with bcsim.Simulator(cfg) as s:
                    topo = topology(name)
                    if topo is not None:
                        s.set_topology(*topo)
                    s.set_partition(dist, transport=transport)
                    s.run()
                    cnt = s.counters()
                    if transport == "host":  # exchange volume (bytes this rank sent to the others)
                        cnt["xfer_bytes"] = s._transport.bytes
                    ls = s.loop_stats()  # per-rank cell-loop collectives (summed over ranks by merge)
                    cnt["windows"], cnt["collectives"] = ls["windows"], ls["collectives"]
                    q.put((name, rank, s.trace(), cnt, None))
            except Exception as e:  # report, keep the other ranks' collectives aligned
                q.put((name, rank, None, None, repr(e)))
                raise
    finally:
        dist.destroy_process_group()


def run(world, names, transport="host", timeout=600):
    """-> {case: (merged (trace, counters) or None, error string or None)}"""
    import torch.multiprocessing as mp
    from bcsim import partition
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, list(names), transport, q)) for r in range(world)]
    for p in ps:
        p.start()
    import queue
    import time
    got = {}
    deadline = time.time() + timeout
    try:
        n = 0
        while n < world * len(names) and time.time() < deadline:
            try:
                name, rank, tr, cnt, err = q.get(timeout=2)
            except queue.Empty:
                dead = [r for r, p in enumerate(ps) if p.exitcode not in (None, 0)]
                if dead:
                    got.setdefault("_", {})[-1] = (None, None, f"ranks {dead} exited "
                                                   f"{[ps[r].exitcode for r in dead]}")
                    break
                continue
            n += 1
            got.setdefault(name, {})[rank] = (tr, cnt, err)
            if err:
                break
    finally:
        for p in ps:
            p.join(timeout=30)
            if p.exitcode is None:
                p.kill()
    out = {}
    for name in names:
        parts = got.get(name, {})
        errs = [v[2] for v in list(parts.values()) + list(got.get("_", {}).values()) if v[2]]
        if errs or len(parts) != world:
            out[name] = (None, "; ".join(errs) or f"{len(parts)}/{world} ranks reported")
        else:
            out[name] = (partition.merge([(parts[r][0], parts[r][1]) for r in range(world)]), None)
    return out


if __name__ == "__main__":
    import oracle
    from parity_cases import cases, compare
    world = int(sys.argv[1])
    names = sys.argv[2:]
    res = run(world, names)
    bad = 0
    for name in names:
        merged, err = res[name]
        if err:
            print(f"{name:24s} EXC {err}", flush=True)
            bad += 1
            continue
        ref = oracle.run(cases()[name], topology=topology(name))
        d = compare(ref, merged)
        print(f"{name:24s} {'OK ' if d is None else 'BAD'} world={world} deliv={ref[1]['delivered_total']}/"
              f"{merged[1]['delivered_total']} {d or ''}", flush=True)
        bad += d is not None
    sys.exit(1 if bad else 0)
