"""ctypes mirror of include/bcsim.h (the C ABI of the engine).

Struct layouts must match the header byte for byte; tests/test_abi.py checks
the sizes against the compiled library.
"""
import ctypes as C

ABI_VERSION = 2

PBFT, RAFT, PAXOS, GOSSIP = 0, 1, 2, 3
DELAY_FIXED, DELAY_RANDOM = 0, 1
RNG_GLIBC, RNG_COUNTER = 0, 1
TIME_ROUND, TIME_TRUNC = 0, 1
ENC_EXTENDED, ENC_COMPAT = 0, 1
QUEUE_INFINITE, QUEUE_DROPTAIL, QUEUE_FQCODEL = 0, 1, 2
ENGINE_AUTO, ENGINE_DENSE, ENGINE_SPARSE = 0, 1, 2

OK = 0
ERRORS = {
    -1: "E_INVAL", -2: "E_NOMEM", -3: "E_HIP", -4: "E_OVERFLOW",
    -5: "E_UNSUPPORTED", -6: "E_ENCODING", -7: "E_TIE", -8: "E_NODEVICE",
    -9: "E_STATE", -10: "E_INDEX", -11: "E_PEER",
}

TR = dict(
    PBFT_COMMIT=1, PBFT_BLOCK=2, PBFT_STOP=3, PBFT_VIEW=4,
    RAFT_ELECTION=10, RAFT_LEADER=11, RAFT_BLOCK=12, RAFT_DONE=13,
    RAFT_PROPOSAL=14, RAFT_STOP=15, PAXOS_COMMIT=20, PAXOS_TICKET=21,
    GOSSIP_BLOCK=30, GOSSIP_DELIVER=31,
)

MSG_TYPES = 16
INT64_MAX = (1 << 63) - 1


class Config(C.Structure):
    _fields_ = [
        ("abi_version", C.c_uint32),
        ("protocol", C.c_uint32),
        ("n_nodes", C.c_uint32),
        ("n_replicas", C.c_uint32),
        ("link_rate_bps", C.c_uint64),
        ("link_delay_ns", C.c_int64),
        ("mtu", C.c_uint32),
        ("delay_mode", C.c_uint32),
        ("app_delay_ns", C.c_int64),
        ("rng_mode", C.c_uint32),
        ("time_round", C.c_uint32),
        ("seed", C.c_uint64),
        ("encoding", C.c_uint32),
        ("echo", C.c_uint32),
        ("t_end_ns", C.c_int64),
        ("stop_ns", C.c_int64),
        ("pbft_rounds", C.c_uint32),
        ("pbft_block_bytes", C.c_uint32),
        ("pbft_timeout_s", C.c_float),
        ("pbft_view_change", C.c_uint32),
        ("pbft_seq_cap", C.c_uint32),
        ("raft_blocks", C.c_uint32),
        ("raft_proposal_bytes", C.c_uint32),
        ("raft_heartbeat_s", C.c_float),
        ("raft_proposal_rounds", C.c_uint32),
        ("raft_proposal_delay_ns", C.c_int64),
        ("paxos_proposers", C.c_uint32),
        ("device", C.c_uint32),
        ("cap_ops_per_node", C.c_uint32),
        ("cap_bucket_records", C.c_uint32),
        ("n_buckets", C.c_uint32),
        ("cap_timers_per_node", C.c_uint32),
        ("max_events", C.c_uint64),
        ("queue_model", C.c_uint32),
        ("queue_dev_pkts", C.c_uint32),
        ("queue_disc_pkts", C.c_uint32),
        ("cap_queue_msgs", C.c_uint32),
        ("paxos_decrees", C.c_uint32),
        ("engine_mode", C.c_uint32),
        ("fq_limit_pkts", C.c_uint32),
        ("fq_flows", C.c_uint32),
        ("fq_quantum", C.c_uint32),
        ("fq_drop_batch", C.c_uint32),
        ("fq_target_ns", C.c_int64),
        ("fq_interval_ns", C.c_int64),
        ("fq_min_bytes", C.c_uint32),
        ("fq_perturbation", C.c_uint32),
        ("reserved", C.c_uint32 * 2),
    ]


class TraceRec(C.Structure):
    _fields_ = [
        ("t_ns", C.c_int64),
        ("key_ts", C.c_int64),
        ("key_origin", C.c_uint32),
        ("key_sub", C.c_uint32),
        ("replica", C.c_uint32),
        ("node", C.c_uint32),
        ("kind", C.c_uint32),
        ("a", C.c_int32),
        ("b", C.c_int32),
        ("c", C.c_int32),
    ]


class Counters(C.Structure):
    _fields_ = [
        ("delivered", C.c_uint64 * MSG_TYPES),
        ("delivered_total", C.c_uint64),
        ("echoes", C.c_uint64),
        ("sends", C.c_uint64),
        ("dropped", C.c_uint64),
        ("wrong_msgs", C.c_uint64),
        ("events", C.c_uint64),
        ("t_last_ns", C.c_int64),
        ("trace_records", C.c_uint64),
        ("frames_dropped", C.c_uint64),
        ("msgs_lost", C.c_uint64),
        ("reserved", C.c_uint64 * 5),
    ]


class Status(C.Structure):
    _fields_ = [
        ("now_ns", C.c_int64),
        ("next_ns", C.c_int64),
        ("cells", C.c_uint64),
        ("quiescent", C.c_uint32),
        ("error", C.c_int32),
        ("lookahead_ns", C.c_int64),
    ]


def default_config(protocol=PBFT, n_nodes=8):
    """Reference defaults (blockchain-simulator.cc:23-24,55,67 and each
    protocol's StartApplication).  Mirrors bcsim_config_default()."""
    c = Config()
    c.abi_version = ABI_VERSION
    c.protocol = protocol
    c.n_nodes = n_nodes
    c.n_replicas = 1
    c.link_rate_bps = 3_000_000          # "3Mbps"
    c.link_delay_ns = 3_000_000          # "3ms"
    c.mtu = 1500
    c.delay_mode = DELAY_RANDOM
    c.app_delay_ns = 0
    c.rng_mode = RNG_GLIBC
    c.time_round = TIME_ROUND
    c.seed = 1
    c.encoding = ENC_EXTENDED
    c.echo = 1
    c.t_end_ns = 0
    c.stop_ns = 10_000_000_000           # Stop(Seconds(10.0))
    c.pbft_rounds = 40
    c.pbft_block_bytes = 0
    c.pbft_timeout_s = 0.05
    c.pbft_view_change = 1
    c.pbft_seq_cap = 1000
    c.raft_blocks = 50
    c.raft_proposal_bytes = 0
    c.raft_heartbeat_s = 0.05
    c.raft_proposal_rounds = 50
    c.raft_proposal_delay_ns = 1_000_000_000
    c.paxos_proposers = 3
    c.queue_model = QUEUE_INFINITE
    c.queue_dev_pkts = 100               # DropTailQueue "100p" (PointToPointNetDevice)
    c.queue_disc_pkts = 1000             # pfifo_fast "1000p"
    return c


def config_dict(c):
    return {name: (list(getattr(c, name)) if name == "reserved" else getattr(c, name))
            for name, _ in c._fields_}


def trace_to_tuples(buf, n):
    return [(r.replica, r.t_ns, r.key_ts, r.key_origin, r.key_sub, r.node, r.kind,
             r.a, r.b, r.c) for r in buf[:n]]


def counters_dict(c):
    d = {name: getattr(c, name) for name, _ in c._fields_ if name not in ("delivered", "reserved")}
    d["delivered"] = list(c.delivered)
    return d


def declare(lib, prefix, handle_t=C.c_void_p):
    """Declare the bcsim-shaped entry points of `lib` under `prefix`
    (bcsim_ for the product, bcsim_oracle_ for the oracle)."""
    f = getattr(lib, prefix + "create")
    f.argtypes = [C.POINTER(Config), C.POINTER(handle_t)]
    f.restype = C.c_int
    f = getattr(lib, prefix + "set_topology_csr")
    f.argtypes = [handle_t, C.c_uint32, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32),
                  C.POINTER(C.c_int64)]
    f.restype = C.c_int
    f = getattr(lib, prefix + "run")
    f.argtypes = [handle_t, C.c_int64]
    f.restype = C.c_int
    f = getattr(lib, prefix + "read_trace")
    f.argtypes = [handle_t, C.POINTER(TraceRec), C.c_uint64, C.POINTER(C.c_uint64)]
    f.restype = C.c_int
    f = getattr(lib, prefix + "read_counters")
    f.argtypes = [handle_t, C.POINTER(Counters)]
    f.restype = C.c_int
    f = getattr(lib, prefix + "read_status")
    f.argtypes = [handle_t, C.POINTER(Status)]
    f.restype = C.c_int
    f = getattr(lib, prefix + "destroy")
    f.argtypes = [handle_t]
    f.restype = C.c_int


class EngineError(RuntimeError):
    def __init__(self, code, where, detail=""):
        self.code = code
        super().__init__(f"{where}: {ERRORS.get(code, code)} ({code}) {detail}".strip())


class Handle:
    """Generic driver over a bcsim-shaped C API (product or oracle)."""

    def __init__(self, lib, prefix, cfg, detail_fn=None):
        self.lib, self.prefix, self.cfg = lib, prefix, cfg
        self._detail = detail_fn
        self.h = C.c_void_p()
        self._call("create", C.byref(cfg), C.byref(self.h))

    def _call(self, name, *args):
        rc = getattr(self.lib, self.prefix + name)(*args)
        if rc != OK:
            raise EngineError(rc, self.prefix + name, self._detail() if self._detail else "")
        return rc

    def set_topology(self, row_ptr, col_idx, prop_ns=None):
        import numpy as np
        n = len(row_ptr) - 1
        rp = np.ascontiguousarray(row_ptr, dtype=np.uint32)
        ci = np.ascontiguousarray(col_idx, dtype=np.uint32)
        pp = None if prop_ns is None else np.ascontiguousarray(prop_ns, dtype=np.int64)
        self._call("set_topology_csr", self.h, n,
                   rp.ctypes.data_as(C.POINTER(C.c_uint32)),
                   ci.ctypes.data_as(C.POINTER(C.c_uint32)),
                   None if pp is None else pp.ctypes.data_as(C.POINTER(C.c_int64)))

    def run(self, t_until=INT64_MAX):
        self._call("run", self.h, t_until)

    def trace(self):
        n = C.c_uint64(0)
        self._call("read_trace", self.h, None, 0, C.byref(n))
        buf = (TraceRec * max(1, n.value))()
        self._call("read_trace", self.h, buf, n.value, C.byref(n))
        return trace_to_tuples(buf, n.value)

    def counters(self):
        c = Counters()
        self._call("read_counters", self.h, C.byref(c))
        return counters_dict(c)

    def status(self):
        s = Status()
        self._call("read_status", self.h, C.byref(s))
        return {name: getattr(s, name) for name, _ in s._fields_}

    def close(self):
        if self.h:
            getattr(self.lib, self.prefix + "destroy")(self.h)
            self.h = C.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
