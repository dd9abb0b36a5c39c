"""Node-partitioned multi-GPU runs.

Each rank owns a contiguous node range of every replica; the engine
exchanges the records that cross ranks once per lookahead cell.  Two
transports sit behind ``bcsim_set_partition*`` (include/bcsim.h):

* RCCL over xGMI, device buffers on the engine stream (production):
  :func:`partition_rccl`;
* host callbacks over an initialised ``torch.distributed`` process group
  (gloo in the tests, several ranks may share one GPU):
  :class:`TorchTransport` / :func:`partition_torch`.

Counters and traces stay per rank: :func:`merge` combines them into the
single-process result (the oracle's shape).
"""
import ctypes as C

from . import _abi

PEER_ERR = 1 << 62  # send count of a failed rank (include/bcsim.h bcsim_transport)
ALLREDUCE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_int64), C.c_uint32, C.c_int32)
ALLTOALLV_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.POINTER(C.c_uint64), C.c_void_p,
                           C.c_uint64, C.POINTER(C.c_uint64))


class Transport(C.Structure):
    _fields_ = [("ctx", C.c_void_p), ("allreduce_i64", ALLREDUCE_FN), ("alltoallv", ALLTOALLV_FN)]


def declare(lib):
    lib.bcsim_set_partition.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.POINTER(Transport)]
    lib.bcsim_set_partition.restype = C.c_int
    lib.bcsim_rccl_unique_id.argtypes = [C.c_void_p, C.c_uint64, C.POINTER(C.c_uint64)]
    lib.bcsim_rccl_unique_id.restype = C.c_int
    lib.bcsim_set_partition_rccl.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_void_p, C.c_uint64]
    lib.bcsim_set_partition_rccl.restype = C.c_int


class TorchTransport:
    """bcsim_transport callbacks over a torch.distributed process group
    (host tensors; any backend with all_reduce / all_gather, e.g. gloo)."""

    def __init__(self, dist, group=None):
        self.dist, self.group = dist, group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.error = None
        self.bytes = 0  # payload bytes this rank sent through alltoallv (exchange volume)
        # keep the ctypes thunks alive as long as the transport
        self._ar = ALLREDUCE_FN(self._allreduce)
        self._a2a = ALLTOALLV_FN(self._alltoallv)
        self.struct = Transport(None, self._ar, self._a2a)

    def _allreduce(self, _ctx, v, n, op):
        try:
            import torch
            t = torch.tensor([v[k] for k in range(n)], dtype=torch.int64)
            red = self.dist.ReduceOp.MIN if op == 0 else self.dist.ReduceOp.SUM
            self.dist.all_reduce(t, op=red, group=self.group)
            for k in range(n):
                v[k] = int(t[k])
            return 0
        except Exception as e:  # surfaced by the caller through EngineError
            self.error = e
            return 1

    def _alltoallv(self, _ctx, send, send_bytes, recv, recv_cap, recv_bytes):
        try:
            import torch
            P = self.world
            sb = [int(send_bytes[r]) for r in range(P)]
            self.bytes += sum(b for r, b in enumerate(sb) if b < PEER_ERR and r != self.rank)
            # sizes: row r of the gathered matrix = what rank r sends to each rank
            sz = torch.tensor(sb, dtype=torch.int64)
            rows = [torch.empty(P, dtype=torch.int64) for _ in range(P)]
            self.dist.all_gather(rows, sz, group=self.group)
            mat = torch.stack(rows)
            if bool((mat >= PEER_ERR).any()):  # a rank failed: counts only, no payload
                for r in range(P):
                    recv_bytes[r] = int(mat[r, self.rank])
                return 0
            width = max(1, int(mat.sum(dim=1).max()))
            buf = torch.zeros(width, dtype=torch.uint8)
            tot = sum(sb)
            if tot:
                C.memmove(buf.data_ptr(), send, tot)
            bufs = [torch.empty(width, dtype=torch.uint8) for _ in range(P)]
            self.dist.all_gather(bufs, buf, group=self.group)
            off_out = 0
            for r in range(P):
                n = int(mat[r, self.rank])
                off_in = int(mat[r, :self.rank].sum())
                if off_out + n > recv_cap:
                    raise RuntimeError("alltoallv: receive buffer too small")
                if n:
                    C.memmove(recv + off_out, bufs[r].data_ptr() + off_in, n)
                recv_bytes[r] = n
                off_out += n
            return 0
        except Exception as e:
            self.error = e
            return 1


def partition_torch(sim, dist, group=None):
    """Partition `sim` (a bcsim.Simulator, before its first run) over the
    ranks of an initialised torch.distributed group with host callbacks."""
    tr = TorchTransport(dist, group)
    sim._transport = tr  # lifetime: the engine calls back during run()
    sim._call("set_partition", sim.h, tr.rank, tr.world, C.byref(tr.struct))
    return tr


def rccl_unique_id(lib):
    buf = (C.c_uint8 * 512)()
    n = C.c_uint64(0)
    rc = lib.bcsim_rccl_unique_id(buf, 512, C.byref(n))
    if rc:
        raise _abi.EngineError(rc, "bcsim_rccl_unique_id")
    return bytes(buf[:n.value])


def partition_rccl(sim, dist, group=None):
    """Partition `sim` over RCCL: rank 0 makes the ncclUniqueId, the
    torch.distributed group broadcasts it, every rank joins the clique."""
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    obj = [rccl_unique_id(sim.lib) if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0, group=group)
    uid = obj[0]
    b = (C.c_uint8 * len(uid)).from_buffer_copy(uid)
    sim._call("set_partition_rccl", sim.h, rank, world, b, len(uid))


def merge(parts):
    """Per-rank (trace, counters[, status]) -> the single-process result:
    traces merged in the engine's canonical order, counters summed."""
    trace = sorted(t for p in parts for t in p[0])
    cnt = dict(parts[0][1])
    for key in cnt:
        if key == "t_last_ns":
            cnt[key] = max(p[1][key] for p in parts)
        elif key == "delivered":
            cnt[key] = [sum(v) for v in zip(*(p[1][key] for p in parts))]
        else:
            cnt[key] = sum(p[1][key] for p in parts)
    return (trace, cnt) + tuple(parts[0][2:])
