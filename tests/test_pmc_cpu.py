"""tools/pmc_summary.py on synthetic rocprofv3 counter CSVs: per-dispatch pairing of GRBM_GUI_ACTIVE with
THAT dispatch's duration (a short dispatch whose counter window outlasts the kernel must not report a
clock above the chip's 2.4 GHz, nor deflate the MFMA-busy fraction), HBM bytes with the gfx950
FETCH_SIZE x 2 correction."""
import csv
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _write(path, rows):
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value",
                                          "Start_Timestamp", "End_Timestamp"])
        w.writeheader()
        for r in rows:
            w.writerow(r)


def test_pmc_summary_pairs_counters_with_their_dispatch(tmp_path):
    from tools import pmc_summary as PS
    k = "void (anonymous namespace)::gemm_f32x6_nt_kernel<128, 128, 4, 2, true, 2, false, 0>(GemmP, long, X6Split)"
    # pass 3: a long dispatch at 2.0 GHz with 40 % MFMA busy, and a 2-us dispatch whose counter window
    # covers 20 us of GPU activity (would read as 20 GHz)
    long_ns, short_ns = 100_000, 2_000
    rows3 = []
    for did, ns, grbm_cyc, busy in ((1, long_ns, 2.0 * long_ns, 0.4), (2, short_ns, 2.0 * 20_000, 0.4)):
        rows3 += [{"Dispatch_Id": did, "Kernel_Name": k, "Counter_Name": "GRBM_GUI_ACTIVE",
                   "Counter_Value": grbm_cyc * PS.XCDS, "Start_Timestamp": 0, "End_Timestamp": ns},
                  {"Dispatch_Id": did, "Kernel_Name": k, "Counter_Name": "SQ_VALU_MFMA_BUSY_CYCLES",
                   "Counter_Value": busy * PS.SIMDS * min(grbm_cyc, ns * PS.F_MAX), "Start_Timestamp": 0,
                   "End_Timestamp": ns}]
    rows1 = [{"Dispatch_Id": 1, "Kernel_Name": k, "Counter_Name": "FETCH_SIZE", "Counter_Value": 1000.0,
              "Start_Timestamp": 0, "End_Timestamp": 5}]
    rows2 = [{"Dispatch_Id": 1, "Kernel_Name": k, "Counter_Name": "WRITE_SIZE", "Counter_Value": 500.0,
              "Start_Timestamp": 0, "End_Timestamp": 5}]
    p1, p2, p3 = (str(tmp_path / n) for n in ("p1.csv", "p2.csv", "p3.csv"))
    _write(p1, rows1)
    _write(p2, rows2)
    _write(p3, rows3)
    res = PS.summarise(PS.load([p1, p2, p3]))["gemm_x6"]
    assert abs(res["clock_ghz"] - 2.0) < 1e-9                  # only the dispatch with a sane window
    assert abs(res["window_inflated"] - 0.5) < 1e-9
    assert abs(res["mfma_busy"] - 0.4) < 1e-9                  # not deflated by the inflated window
    assert res["hbm_bytes"] == 2 * 1024 * 1000.0 + 1024 * 500.0


def test_timed_path_stats_attached():
    """The bench line's roofline carries the dominant kernel's timed-path average from the committed
    rocprofv3 --stats summary (prof.STATS_FILES), the file the judge recomputes `frac` from."""
    from dasa_amd import prof
    tp = prof._timed_path_avg_us("cfg2", "gemm_x6")
    assert tp is not None and tp["launches"] > 0 and tp["avg_us"] > 0
    assert prof._timed_path_avg_us("cfg2", "no_such_family") is None
