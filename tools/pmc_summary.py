"""Summarise rocprofv3 --pmc counter-collection CSVs per kernel family (tools/prof_compare.family).

One CSV per pass (gfx950 cannot collect FETCH_SIZE and WRITE_SIZE, or many SQ counters, in one pass).
Per family it reports the dispatch count, the mean of every counter per dispatch, and derived values:
  * hbm_read_bytes  = 2 x FETCH_SIZE x 1024 (MI355X_MICROARCH.md "HBM": FETCH_SIZE reads exactly half
                      the bytes of a wide coalesced stream on gfx950, in KB), hbm_write_bytes = WRITE_SIZE x 1024;
  * per dispatch, from the counters and the duration of THAT dispatch in the same pass: kernel cycles
    = GRBM_GUI_ACTIVE / XCDs (rocprofv3 sums it over the 8 XCDs) and clock = kernel cycles / duration.
    For short dispatches the counter window outlasts the kernel (clock > F_MAX = 2.4 GHz, impossible on
    MI355X): there the kernel's cycles are taken as duration x F_MAX, and the dispatch is left out of
    the clock estimate (`window_inflated` = the fraction of such dispatches);
  * mfma_busy       = sum SQ_VALU_MFMA_BUSY_CYCLES / (SIMDs x sum kernel cycles), SIMDs = 4 x 256 CUs;
  * clock_ghz       = the duration-weighted mean clock of the dispatches whose window is not inflated.

    python tools/pmc_summary.py out.json pass1_counter_collection.csv [pass2 ...]
"""
import csv
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.prof_compare import family  # noqa: E402

XCDS, SIMDS = 8, 1024
F_MAX = 2.4   # GHz: MI355X peak engine clock (MI355X_MICROARCH.md)


def _f(r, *names):
    for n in names:
        if n in r and r[n] not in (None, ""):
            return r[n]
    return None


def load(paths):
    # (dispatch id, family) -> {counter: value}, plus durations
    disp = {}
    for path in paths:
        for r in csv.DictReader(open(path)):
            name = _f(r, "Kernel_Name", "Kernel-Name", "KernelName") or ""
            did = _f(r, "Dispatch_Id", "Dispatch-Id", "DispatchId") or str(len(disp))
            key = (path, did)
            e = disp.setdefault(key, {"family": family(name), "counters": {}, "ns": None})
            cname = _f(r, "Counter_Name", "Counter-Name")
            val = float(_f(r, "Counter_Value", "Counter-Value") or 0.0)
            e["counters"][cname] = e["counters"].get(cname, 0.0) + val
            t0, t1 = _f(r, "Start_Timestamp", "Start-Timestamp"), _f(r, "End_Timestamp", "End-Timestamp")
            if t0 and t1:
                e["ns"] = float(t1) - float(t0)
    return disp


def summarise(disp):
    fam = defaultdict(lambda: {"dispatches": defaultdict(int), "sums": defaultdict(float), "ns": [],
                               "busy": 0.0, "cyc": 0.0, "clk_w": 0.0, "clk_ns": 0.0, "clk_n": 0, "inflated": 0})
    for e in disp.values():
        f = fam[e["family"]]
        c = e["counters"]
        for k, v in c.items():
            f["sums"][k] += v
            f["dispatches"][k] += 1
        if e["ns"]:
            f["ns"].append(e["ns"])
        if "GRBM_GUI_ACTIVE" in c and e["ns"]:
            cyc = c["GRBM_GUI_ACTIVE"] / XCDS
            clk = cyc / e["ns"]
            f["clk_n"] += 1
            if clk > F_MAX:                     # the counter window outlasts the dispatch
                f["inflated"] += 1
                cyc = e["ns"] * F_MAX
            else:
                f["clk_w"] += clk * e["ns"]
                f["clk_ns"] += e["ns"]
            if "SQ_VALU_MFMA_BUSY_CYCLES" in c:
                f["busy"] += c["SQ_VALU_MFMA_BUSY_CYCLES"]
                f["cyc"] += cyc
    out = {}
    for name, f in fam.items():
        mean = {c: f["sums"][c] / f["dispatches"][c] for c in f["sums"]}
        ent = {"dispatches": max(f["dispatches"].values()), "counters_mean": mean}
        if "FETCH_SIZE" in mean:
            ent["hbm_read_bytes"] = 2.0 * 1024.0 * mean["FETCH_SIZE"]
        if "WRITE_SIZE" in mean:
            ent["hbm_write_bytes"] = 1024.0 * mean["WRITE_SIZE"]
        if "hbm_read_bytes" in ent and "hbm_write_bytes" in ent:
            ent["hbm_bytes"] = ent["hbm_read_bytes"] + ent["hbm_write_bytes"]
        if f["cyc"]:
            ent["mfma_busy"] = f["busy"] / (SIMDS * f["cyc"])
        if f["clk_ns"]:
            ent["clock_ghz"] = f["clk_w"] / f["clk_ns"]
        if f["clk_n"]:
            ent["window_inflated"] = f["inflated"] / f["clk_n"]
        out[name] = ent
    return out


def main(out, *paths):
    res = summarise(load(paths))
    json.dump({"source": "rocprofv3 --pmc passes: " + ", ".join(os.path.basename(p) for p in paths),
               "families": res}, open(out, "w"), indent=1, sort_keys=True)
    for k, v in sorted(res.items(), key=lambda kv: -kv[1]["dispatches"])[:20]:
        extra = " ".join(f"{x}={v[x]:.4g}" for x in ("hbm_bytes", "mfma_busy", "clock_ghz", "window_inflated")
                         if v.get(x) is not None)
        print(f"{k:<40}{v['dispatches']:>8}  {extra}")


if __name__ == "__main__":
    main(*sys.argv[1:])
