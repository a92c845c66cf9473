"""Per-launch HBM traffic of each kernel family from two rocprofv3 --pmc passes (FETCH_SIZE and
WRITE_SIZE cannot share a pass on gfx950), corrected as MI355X_MICROARCH.md "HBM" prescribes:
FETCH_SIZE counts 64 B per 128-B request of a wide (16 B/lane) coalesced read, so it is doubled;
WRITE_SIZE is exact for 16-B/lane stores. Units: both counters are KB.

    python tools/pmc_traffic.py fetch_counter_collection.csv write_counter_collection.csv out.json
"""
import csv
import json
import sys
from collections import defaultdict

sys.path.insert(0, __file__.rsplit("/", 2)[0])
from tools.prof_compare import family  # noqa: E402


def load(path, counter):
    vals = defaultdict(list)
    for r in csv.DictReader(open(path)):
        name = r.get("Kernel_Name") or r.get("Kernel-Name") or r.get("KernelName") or ""
        cname = r.get("Counter_Name") or r.get("Counter-Name") or ""
        if cname and cname != counter:
            continue
        v = float(r.get("Counter_Value") or r.get("Counter-Value") or r.get(counter) or 0.0)
        vals[family(name)].append(v)
    return vals


def main(fetch_csv, write_csv, out):
    f = load(fetch_csv, "FETCH_SIZE")
    w = load(write_csv, "WRITE_SIZE")
    res = {}
    for fam in sorted(set(f) | set(w)):
        fr, wr = f.get(fam, []), w.get(fam, [])
        if not fr or not wr:
            continue
        rd = 2.0 * 1024.0 * sum(fr) / len(fr)
        wb = 1024.0 * sum(wr) / len(wr)
        res[fam] = {"launches": len(fr), "read_bytes_per_launch": rd, "write_bytes_per_launch": wb,
                    "hbm_bytes_per_launch": rd + wb}
    json.dump({"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, FETCH_SIZE x2 (gfx950 correction)",
               "families": res}, open(out, "w"), indent=1)
    for k, v in sorted(res.items(), key=lambda kv: -kv[1]["hbm_bytes_per_launch"] * kv[1]["launches"])[:12]:
        print(f"{k:<40}{v['launches']:>8}{v['hbm_bytes_per_launch'] / 1e6:>12.3f} MB/launch")


if __name__ == "__main__":
    main(*sys.argv[1:])
