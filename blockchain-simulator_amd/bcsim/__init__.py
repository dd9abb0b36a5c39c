"""bcsim — Python binding of the MI355X consensus-propagation engine.

Thin ctypes layer over the in-tree C ABI library ``libbcsim.so`` (built by
``make -C blockchain-simulator_amd``; include/bcsim.h).  There is no CPU
fallback: if the library or a HIP device is missing, calls fail loudly with
``EngineError``.
"""
import ctypes as C
import os
import subprocess

from . import _abi, partition
from ._abi import (  # noqa: F401
    PBFT, RAFT, PAXOS, GOSSIP, DELAY_FIXED, DELAY_RANDOM, RNG_GLIBC, RNG_COUNTER,
    TIME_ROUND, TIME_TRUNC, ENC_EXTENDED, ENC_COMPAT, TR, INT64_MAX,
    QUEUE_INFINITE, QUEUE_DROPTAIL, QUEUE_FQCODEL, ENGINE_AUTO, ENGINE_DENSE, ENGINE_SPARSE,
    Config, TraceRec, Counters, Status, EngineError, default_config,
)

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("BCSIM_LIB") or os.path.join(PKG_DIR, "libbcsim.so")
_LIB = None


def build(jobs=8):
    """Compile libbcsim.so / bcsim_cli for gfx950 in-tree (make)."""
    subprocess.check_call(["make", "-s", "-C", PKG_DIR, f"-j{jobs}", "all"])
    return LIB_PATH


def lib():
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise EngineError(-8, "bcsim", f"{LIB_PATH} not built (run make -C {PKG_DIR})")
        _LIB = C.CDLL(LIB_PATH)
        _abi.declare(_LIB, "bcsim_")
        _LIB.bcsim_config_default.argtypes = [C.POINTER(Config), C.c_uint32, C.c_uint32]
        _LIB.bcsim_config_default.restype = C.c_int
        _LIB.bcsim_strerror.argtypes = [C.c_int]
        _LIB.bcsim_strerror.restype = C.c_char_p
        _LIB.bcsim_last_error_detail.argtypes = []
        _LIB.bcsim_last_error_detail.restype = C.c_char_p
        _LIB.bcsim_read_kernel_stats.argtypes = [C.c_void_p, C.POINTER(C.c_double),
                                                 C.POINTER(C.c_double), C.POINTER(C.c_uint64)]
        _LIB.bcsim_read_kernel_stats.restype = C.c_int
        _LIB.bcsim_read_engine_counters.argtypes = [C.c_void_p, C.POINTER(C.c_uint64)]
        _LIB.bcsim_read_engine_counters.restype = C.c_int
        _LIB.bcsim_read_loop_stats.argtypes = [C.c_void_p, C.POINTER(C.c_uint64)]
        _LIB.bcsim_read_loop_stats.restype = C.c_int
        _LIB.bcsim_reset_kernel_stats.argtypes = [C.c_void_p]
        _LIB.bcsim_reset_kernel_stats.restype = C.c_int
        _LIB.bcsim_topology_random_regular.argtypes = [C.c_uint32, C.c_uint32, C.c_uint64,
                                                       C.c_void_p, C.c_void_p]
        _LIB.bcsim_topology_random_regular.restype = C.c_int
        _LIB.bcsim_format_trace_line.argtypes = [C.POINTER(TraceRec), C.c_void_p, C.c_char_p, C.c_uint64,
                                                 C.POINTER(C.c_uint64)]
        _LIB.bcsim_format_trace_line.restype = C.c_int
        partition.declare(_LIB)
    return _LIB


def format_trace_line(rec, cfg=None):
    """The reference's NS_LOG_INFO text of one trace record (tuple as returned by
    trace()), byte for byte -- bcsim_format_trace_line (host code, no GPU)."""
    r = TraceRec(t_ns=rec[1], key_ts=rec[2], key_origin=rec[3], key_sub=rec[4], replica=rec[0],
                 node=rec[5], kind=rec[6], a=rec[7], b=rec[8], c=rec[9])
    n = C.c_uint64(0)
    cp = C.byref(cfg) if cfg is not None else None
    lib().bcsim_format_trace_line(C.byref(r), cp, None, 0, C.byref(n))
    buf = C.create_string_buffer(n.value + 1)
    rc = lib().bcsim_format_trace_line(C.byref(r), cp, buf, n.value + 1, C.byref(n))
    if rc:
        raise EngineError(rc, "bcsim_format_trace_line")
    return buf.raw[:n.value].decode("utf-8", errors="surrogateescape")


def c_default_config(protocol=PBFT, n_nodes=8):
    c = Config()
    rc = lib().bcsim_config_default(C.byref(c), protocol, n_nodes)
    if rc:
        raise EngineError(rc, "bcsim_config_default")
    return c


def _detail():
    d = lib().bcsim_last_error_detail()
    return d.decode() if d else ""


class Simulator(_abi.Handle):
    """One engine instance (all replicas) on one HIP device."""

    def __init__(self, cfg):
        super().__init__(lib(), "bcsim_", cfg, detail_fn=_detail)

    def kernel_stats(self):
        us = (C.c_double * 4)()
        by = (C.c_double * 4)()
        ln = (C.c_uint64 * 4)()
        self._call("read_kernel_stats", self.h, us, by, ln)
        names = ("scan", "link", "group", "aux")
        return {n: dict(us=us[k], bytes=by[k], launches=ln[k]) for k, n in enumerate(names)}

    def engine_counters(self):
        """Raw work counters (include/bcsim.h bcsim_read_engine_counters)."""
        out = (C.c_uint64 * 8)()
        self._call("read_engine_counters", self.h, out)
        names = ("records", "due_ops", "edges", "kept_ops", "delivered", "scan_ops", "echoes", "split_windows")
        return dict(zip(names, out))

    def loop_stats(self):
        """Cell-loop statistics (include/bcsim.h bcsim_read_loop_stats)."""
        out = (C.c_uint64 * 8)()
        self._call("read_loop_stats_ex", self.h, out)
        return dict(windows=out[0], collectives=out[1], tag_zeroes=out[2], spec_hits=out[3], idle_parts=out[4],
                    host_syncs=out[5], idle_checked=out[6], chain_windows=out[7])

    def host_stats(self):
        """Host time of the cell loop (include/bcsim.h bcsim_read_host_stats)."""
        out = (C.c_double * 4)()
        self._call("read_host_stats", self.h, out)
        return dict(launch_us=out[0], wait_us=out[1], launches=int(out[2]), frontier_hits=int(out[3]))

    def reset_kernel_stats(self):
        self._call("reset_kernel_stats", self.h)

    def set_partition(self, dist, group=None, transport="rccl"):
        """Own this rank's node range of a node-partitioned multi-GPU run
        (DESIGN.md §5): transport "rccl" (device, xGMI) or "host" (callbacks
        over the torch.distributed group, e.g. gloo)."""
        if transport == "rccl":
            partition.partition_rccl(self, dist, group)
        elif transport == "host":
            partition.partition_torch(self, dist, group)
        else:
            raise ValueError(transport)


def run(cfg, t_until=INT64_MAX, topology=None):
    """One-shot engine run -> (trace tuples, counters dict, status dict)."""
    with Simulator(cfg) as s:
        if topology is not None:
            s.set_topology(*topology)
        s.run(t_until)
        return s.trace(), s.counters(), s.status()


def full_mesh(n):
    """CSR of blockchain-simulator.cc:34-51 (peers ascending, self excluded)."""
    import numpy as np
    row = np.arange(n + 1, dtype=np.uint32) * (n - 1)
    col = np.array([j for i in range(n) for j in range(n) if j != i], dtype=np.uint32)
    return row, col


def random_regular(n, d=8, seed=1):
    """CSR (row_ptr, col_idx) of a simple random d-regular graph, rows ascending
    (bcsim_topology_random_regular, host-only)."""
    import numpy as np
    row = np.zeros(n + 1, dtype=np.uint32)
    col = np.zeros(n * d, dtype=np.uint32)
    rc = lib().bcsim_topology_random_regular(n, d, seed, row.ctypes.data, col.ctypes.data)
    if rc:
        raise EngineError(rc, "bcsim_topology_random_regular")
    return row, col


def preset(name):
    """Named configs from BASELINE.json (synthetic inputs of SURVEY.md §8d)."""
    if name == "c1_pbft16":       # PBFT n=16, fixed 3 ms links, 100 client requests
        c = default_config(PBFT, 16)
        c.delay_mode = DELAY_FIXED
        c.app_delay_ns = 3_000_000
        c.pbft_rounds = 100
        return c
    if name == "c2_raft1024":     # Raft n=1024, fixed-delay mesh, glibc seed 1
        c = default_config(RAFT, 1024)
        c.delay_mode = DELAY_FIXED
        c.app_delay_ns = 1_000_000
        c.t_end_ns = 4_000_000_000
        c.cap_ops_per_node = 16384  # the leader holds ~2 waves of N-1 pending reply/echo ops
        return c
    if name == "c3_paxos":        # Paxos, jittered app delay U{0..49} ms, replicas
        c = default_config(PAXOS, 4096)
        c.delay_mode = DELAY_RANDOM
        c.rng_mode = RNG_COUNTER
        return c
    if name == "c4_pbft4096":     # PBFT n=4096 full O(n^2) prepare/commit
        c = default_config(PBFT, 4096)
        c.delay_mode = DELAY_FIXED
        c.app_delay_ns = 3_000_000
        c.pbft_rounds = 100
        return c
    if name == "c5_gossip65536":  # PBFT-style gossip, random 8-regular graph (random_regular(n, 8, 1))
        c = default_config(GOSSIP, 65536)
        c.delay_mode = DELAY_FIXED
        c.app_delay_ns = 3_000_000
        c.pbft_rounds = 100
        c.pbft_block_bytes = 1000
        c.stop_ns = -1
        return c
    raise KeyError(name)
