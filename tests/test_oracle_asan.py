"""The CPU oracle under AddressSanitizer + UndefinedBehaviorSanitizer (`make -C oracle asan`):
a child process with the sanitizer runtime preloaded runs the oracle over parity
configurations of every protocol, queue model and delay mode, and must finish clean and
give the same traces and counters as the plain build.  Host code only (the oracle is test
infrastructure: it checks the engine, it is never the product path)."""
import json
import os
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
NAMES = ["pbft8_fixed_40", "pbft12_jitter_b2", "raft64_fixed", "paxos32_jitter_ctr", "paxos32_jitter_k4",
         "gossip64_d4_fixed", "gossip64_d4_droptail", "pbft16_fq_100", "gossip64_d4_fq"]

CHILD = r"""
import json, sys
sys.path.insert(0, {repo!r}); sys.path.insert(0, {tests!r})
import oracle
from parity_cases import cases, fq_cases, topology
c = dict(cases(), **fq_cases())
out = {{}}
for n in {names!r}:
    tr, cnt, st = oracle.run(c[n], topology=topology(n))
    out[n] = [len(tr), hash(tuple(map(tuple, tr))) & 0xFFFFFFFF, cnt["delivered_total"], cnt["dropped"], st["error"]]
print(json.dumps(out))
"""


def _run(env):
    code = CHILD.format(repo=REPO, tests=HERE, names=NAMES)
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-3000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_oracle_clean_under_asan_ubsan():
    pc = __import__("parity_cases")
    names = set(pc.cases()) | set(pc.fq_cases())
    assert set(NAMES) <= names
    rc = subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle"), "asan"], capture_output=True, text=True)
    if rc.returncode != 0:
        pytest.skip("sanitizer build unavailable: " + rc.stderr[-300:])
    libasan = subprocess.run(["gcc", "-print-file-name=libasan.so"], capture_output=True, text=True).stdout.strip()
    if not os.path.isabs(libasan):
        pytest.skip("libasan runtime not found")
    plain = _run(dict(os.environ, PYTHONHASHSEED="0"))
    env = dict(os.environ, PYTHONHASHSEED="0", LD_PRELOAD=libasan, ASAN_OPTIONS="detect_leaks=0",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1",
               BCSIM_ORACLE_LIB=os.path.join(REPO, "oracle", "liboracle_asan.so"))
    san = _run(env)
    assert san == plain
