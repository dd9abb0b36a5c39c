"""CPU checks of the measurement plumbing (VERDICT r5 "next" #5): bench.py finds the committed
PMC summary of each workload by the name tests/gpu_prof_all.sh + tools/collect_profiles.sh give
it, and tools/window_stats.py restricts a kernel trace to the bench's timed window."""
import csv
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO]


def test_pmc_names_match_the_profile_collector():
    import bench
    assert bench.pmc_name(4096) == "pbft4096"
    assert bench.pmc_name(65536, "gossip") == "gossip65536"
    assert bench.pmc_name(4096, "paxos", replicas=10000) == "paxos4096_r10000"
    assert bench.pmc_name(4096, queue="fqcodel") == "pbft4096_fqcodel"
    assert bench.pmc_name(4096, jitter=True) == "pbft4096_jitter"
    text = open(os.path.join(REPO, "tools", "collect_profiles.sh")).read()
    for name in ("pbft4096", "gossip65536", "paxos4096_r10000"):
        assert name in text


def test_pmc_traffic_reads_the_newest_committed_summary():
    import bench
    for args in ((4096,), (65536, "bcsim::k_link", "gossip"), (4096, "bcsim::k_link", "paxos", 10000)):
        v, src = bench.pmc_traffic(*args)
        assert v is not None and v > 0, args
        assert src.startswith("profiles/") and os.path.exists(os.path.join(REPO, src)), src
    assert bench.pmc_traffic(4096, jitter=True) == (None, None)  # no such profile: no traffic claimed


def test_window_stats_restricts_to_the_timed_window(tmp_path):
    # dispatches: setup kernels, two warm-up windows, two timed windows, one after
    rows, d, t = [], 0, 0
    def k(name, dur):
        nonlocal d, t
        d += 1
        rows.append({"Dispatch_Id": d, "Kernel_Name": name + "(bcsim::KP const*)", "Start_Timestamp": t,
                     "End_Timestamp": t + dur})
        t += dur + 10
    k("bcsim::k_scan<2, true, true>", 688_000)        # the t = 0 START window
    for w, dur in enumerate((100, 100, 200, 300, 999)):
        k("bcsim::k_mesh_prep", dur)
        k("bcsim::k_link<0, false, true>", dur)
        k("bcsim::k_next", 5)
    trace = tmp_path / "kt.csv"
    with open(trace, "w", newline="") as f:
        wr = csv.DictWriter(f, fieldnames=list(rows[0]))
        wr.writeheader()
        wr.writerows(rows)
    line = tmp_path / "bench.log"
    line.write_text("noise\n" + json.dumps({"roofline": {"first_timed_launch": 2, "launches": 2}}) + "\n")
    out = tmp_path / "ws.csv"
    subprocess.check_call([sys.executable, os.path.join(REPO, "tools", "window_stats.py"), str(trace), str(line),
                           str(out)])
    got = {r["Name"]: r for r in csv.DictReader(open(out))}
    assert "bcsim::k_scan<2, true, true>" not in got          # setup / START window excluded
    assert int(got["bcsim::k_mesh_prep"]["Calls"]) == 2
    assert int(got["bcsim::k_mesh_prep"]["TotalDurationNs"]) == 200 + 300
    assert int(got["bcsim::k_next"]["Calls"]) == 2            # the k_next closing each timed window
