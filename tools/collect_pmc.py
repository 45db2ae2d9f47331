"""Summarise rocprofv3 outputs for pianosim_kernel into profiles/.

usage: python tools/collect_pmc.py <trace_dir> <fetch_dir> <write_dir> <envs> <out_prefix>

* <trace_dir>: `rocprofv3 --kernel-trace --stats --output-format csv` of bench.py
* <fetch_dir>/<write_dir>: separate `--pmc FETCH_SIZE` / `--pmc WRITE_SIZE` passes
HBM bytes per launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 (MI355X_MICROARCH.md, HBM:
FETCH_SIZE reports half the bytes of wide coalesced reads on gfx950; units KB).
"""
import csv
import json
import sys
from collections import defaultdict
from pathlib import Path


def rows(d, pattern):
    out = []
    for f in Path(d).rglob(pattern):
        with open(f) as fh:
            out += list(csv.DictReader(fh))
    return out


def counter(d, name):
    per_dispatch = defaultdict(float)
    for r in rows(d, "*counter_collection.csv"):
        if "pianosim_kernel" not in r.get("Kernel_Name", ""):
            continue
        if r.get("Counter_Name") != name:
            continue
        per_dispatch[r.get("Dispatch_Id")] += float(r["Counter_Value"])
    vals = list(per_dispatch.values())
    return sum(vals) / len(vals) if vals else None


def main():
    tdir, fdir, wdir, envs, prefix = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4]), sys.argv[5]
    stats = [r for r in rows(tdir, "*kernel_stats.csv") if "pianosim_kernel" in r.get("Name", "")]
    fetch_kb = counter(fdir, "FETCH_SIZE")
    write_kb = counter(wdir, "WRITE_SIZE")
    out = {"envs": envs, "kernel": "pianosim_kernel"}
    if stats:
        s = stats[0]
        out["rocprof_avg_ns"] = float(s.get("AverageNs", 0))
        out["rocprof_calls"] = int(s.get("Calls", 0))
    if fetch_kb is not None and write_kb is not None:
        out["fetch_kb_per_launch"] = fetch_kb
        out["write_kb_per_launch"] = write_kb
        out["hbm_bytes_per_launch"] = (2.0 * fetch_kb + write_kb) * 1024.0
    Path("profiles").mkdir(exist_ok=True)
    Path(f"profiles/{prefix}_pmc.json").write_text(json.dumps(out, indent=1))
    Path("profiles/pmc_latest.json").write_text(json.dumps(out, indent=1))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
