"""Measurement tooling on the CPU: the rocprofv3 PMC summary restricted to the bench's timed
k_link window (tools/pmc_summary.py), and the bench's CPU baselines (oracle only)."""
import csv
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "tools"), REPO]


def _write_pass(d, rows, counters):
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "run_counter_collection.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"])
        for disp, name, vals in rows:
            for c, v in zip(counters, vals):
                w.writerow([disp, name, c, v])


def test_pmc_summary_timed_window(tmp_path):
    import pmc_summary
    src = tmp_path / "prof"
    link = "void bcsim::k_link<false, false, false>(bcsim::KP const*, long long, long long, long long, int)"
    scan = "void bcsim::k_scan<0, false, false>(bcsim::KP const*)"
    # dispatches: scan, link, scan, link, ... ; link k has FETCH = k KiB, WRITE = 10 KiB
    rows_f, rows_w, trace = [], [], []
    t = 0
    for k in range(6):
        rows_f += [(2 * k, scan, [1.0]), (2 * k + 1, link, [float(k)])]
        rows_w += [(2 * k, scan, [1.0, 0, 0]), (2 * k + 1, link, [10.0, 0, 0])]
        trace += [(2 * k, scan, t, t + 5), (2 * k + 1, link, t + 10, t + 10 + 1000 * (k + 1))]
        t += 10000
    _write_pass(str(src / "fetch"), rows_f, ["FETCH_SIZE"])
    _write_pass(str(src / "write"), rows_w, ["WRITE_SIZE", "TCC_HIT_sum", "TCC_MISS_sum"])
    os.makedirs(src / "trace")
    with open(src / "trace" / "run_kernel_trace.csv", "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Dispatch_Id", "Kernel_Name", "Start_Timestamp", "End_Timestamp"])
        for row in trace:
            w.writerow(row)
    with open(src / "trace.log", "w") as f:
        f.write("[bench] warmup\n" + json.dumps({"roofline": {"first_timed_launch": 2, "launches": 3}}) + "\n")
    dst = tmp_path / "out.json"
    pmc_summary.main(str(src), str(dst))
    res = json.load(open(dst))["kernels"]["bcsim::k_link<false, false, false>"]
    tw = res["timed_window"]
    assert tw["first"] == 2 and tw["launches"] == 3
    # links 2,3,4: FETCH 2,3,4 KiB (x2 gfx950 correction) + WRITE 10 KiB each
    assert abs(tw["hbm_bytes_per_launch"] - (2 * 1024 * 3.0 + 10 * 1024)) < 1e-6
    assert abs(tw["rocprof_avg_us"] - 4.0) < 1e-9  # durations 3, 4, 5 us


def test_cpu_baselines_small():
    import bench
    one = bench.cpu_baseline(16, 0.3, "pbft")
    assert one["value"] > 0 and one["cores"] == 1 and one["kind"] == "port" and one["nproc"] >= 1

    def tweak(c):
        c.paxos_decrees = 2
    allc = bench.cpu_baseline_all_cores(16, 0.3, "paxos", tweak, 2)
    assert allc["value"] > 0 and allc["cores"] == 2


def test_pmc_summary_link_class_groups(tmp_path):
    """A timed k_link-class launch = the link-stage dispatches of one window (fast path +
    looped generic kernel; windows end at their k_next): the link_class entry sums them over
    the bench's timed window."""
    import pmc_summary
    src = tmp_path / "prof"
    mesh = "bcsim::k_link_mesh(bcsim::KP const*, long long, long long, long long, int)"
    loop = "void bcsim::k_link<false, false, true>(bcsim::KP const*, long long, long long, long long, int)"
    scan = "void bcsim::k_scan<0, false, false>(bcsim::KP const*)"
    nxt = "bcsim::k_next(bcsim::KP const*, unsigned int)"
    rows_f, rows_w, trace = [], [], []
    t, d = 0, 0
    for k in range(5):
        for name, fv, wv, us in ((scan, 1.0, 1.0, 1), (mesh, float(k), 10.0, 10 * (k + 1)), (loop, 1.0, 2.0, 2),
                                 (nxt, 0.5, 0.5, 1)):
            rows_f.append((d, name, [fv]))
            rows_w.append((d, name, [wv, 0, 0]))
            trace.append((d, name, t, t + 1000 * us))
            t += 100000
            d += 1
    _write_pass(str(src / "fetch"), rows_f, ["FETCH_SIZE"])
    _write_pass(str(src / "write"), rows_w, ["WRITE_SIZE", "TCC_HIT_sum", "TCC_MISS_sum"])
    os.makedirs(src / "trace")
    with open(src / "trace" / "run_kernel_trace.csv", "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Dispatch_Id", "Kernel_Name", "Start_Timestamp", "End_Timestamp"])
        for row in trace:
            w.writerow(row)
    with open(src / "trace.log", "w") as f:
        f.write(json.dumps({"roofline": {"first_timed_launch": 1, "launches": 3}}) + "\n")
    dst = tmp_path / "out.json"
    pmc_summary.main(str(src), str(dst))
    tw = json.load(open(dst))["kernels"]["link_class"]["timed_window"]
    assert tw["first"] == 1 and tw["launches"] == 3
    # groups 1..3: mesh FETCH 1,2,3 + loop FETCH 1 (x2), WRITE 10 + 2
    assert abs(tw["hbm_bytes_per_launch"] - (2 * 1024 * (2.0 + 1.0) + 12 * 1024)) < 1e-6
    assert abs(tw["rocprof_avg_us"] - (30.0 + 2.0)) < 1e-9  # mesh 20, 30, 40 us + loop 2 us
