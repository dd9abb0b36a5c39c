"""world_size-2 gloo test of the multi-GPU aggregation path of bench.py
(replica sharding: max wall time over ranks, summed work), on CPU."""
import os
import socket

import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, repo)
    import torch.distributed as dist
    import bench
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dt, msgs, tr = bench.aggregate(dist, "cpu", 1.0 + rank, 100 * (rank + 1), 7)
    q.put((rank, dt, msgs, tr))
    dist.destroy_process_group()


def test_bench_aggregate_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, dt, msgs, tr in res:
        assert dt == 2.0 and msgs == 300 and tr == 14
