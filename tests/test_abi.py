"""The C-ABI library loads and exports every symbol include/bcsim.h declares;
struct layouts match; the product fails loudly without a GPU (no fallback)."""
import ctypes
import os
import re

import pytest

import bcsim
from bcsim import _abi

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    txt = open(os.path.join(REPO, "include", "bcsim.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(bcsim_\w+)\s*\(", txt, re.M)))


def test_every_declared_symbol_is_exported(engine_lib):
    syms = header_symbols()
    assert len(syms) >= 12
    for s in syms:
        assert hasattr(engine_lib, s), s


def test_struct_sizes():
    assert ctypes.sizeof(_abi.TraceRec) == 48
    assert ctypes.sizeof(_abi.Counters) == 8 * (16 + 15)
    assert ctypes.sizeof(_abi.Config) % 8 == 0


def test_config_default_matches_python_mirror(engine_lib):
    for proto in (_abi.PBFT, _abi.RAFT, _abi.PAXOS):
        assert _abi.config_dict(bcsim.c_default_config(proto, 8)) == _abi.config_dict(_abi.default_config(proto, 8))


def test_create_validates_config(engine_lib):
    c = _abi.default_config(_abi.PBFT, 1)
    with pytest.raises(_abi.EngineError):
        bcsim.Simulator(c)
    c = _abi.default_config(_abi.PBFT, 8)  # random delays + glibc stream: oracle only
    with pytest.raises(_abi.EngineError) as e:
        bcsim.Simulator(c)
    assert e.value.code == -5


def test_topology_validation(engine_lib):
    import numpy as np
    c = _abi.default_config(_abi.PBFT, 4)
    c.delay_mode = _abi.DELAY_FIXED
    s = bcsim.Simulator(c)
    with pytest.raises(_abi.EngineError):   # asymmetric: 0->1 without 1->0
        s.set_topology(np.array([0, 1, 1, 1, 1]), np.array([1]))
    row, col = bcsim.full_mesh(4)
    s.set_topology(row, col)
    s.close()


def test_no_cpu_fallback_without_gpu(engine_lib):
    from conftest import gpu_available
    if gpu_available():
        pytest.skip("GPU present")
    c = _abi.default_config(_abi.PBFT, 8)
    c.delay_mode = _abi.DELAY_FIXED
    with bcsim.Simulator(c) as s:
        with pytest.raises(_abi.EngineError) as e:
            s.run()
        assert e.value.code == -8  # E_NODEVICE: the product never runs on the CPU


def test_strerror(engine_lib):
    engine_lib.bcsim_strerror.restype = ctypes.c_char_p
    assert engine_lib.bcsim_strerror(-4) == b"engine buffer capacity exceeded"
