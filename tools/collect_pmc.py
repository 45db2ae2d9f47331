"""Summarise rocprofv3 outputs for pianosim_kernel into profiles/.

usage: python tools/collect_pmc.py <trace_dir> <fetch_dir> <write_dir> <envs> <song> <out_prefix> [warmup] [sq_dir]

* <trace_dir>: `rocprofv3 --kernel-trace --stats --output-format csv` of bench.py
* <fetch_dir>/<write_dir>: separate `--pmc FETCH_SIZE` / `--pmc WRITE_SIZE` passes
* [sq_dir]: a `--pmc` pass of the SQ wave-state counters (SQ_COUNTERS below): how much of
  the waves' lifetime issues an instruction vs waits on a counter (s_waitcnt / barrier) vs
  is stalled at issue (dependency or pipe busy: SQ_WAIT_INST_ANY, MI355X_MICROARCH.md)
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


# the profiled collider set (bench.py --hand; PIANOSIM_HAND, default the bench's default "hull") and
# its kernel instantiation: pianosim_kernel<true> (box / hull colliders) or <false> (all-capsule
# hand); bench.py's line also times the other sets (its legs), which must not mix in
HAND = __import__("os").environ.get("PIANOSIM_HAND", "hull")
KNAME = "pianosim_kernel<false" if HAND == "authored" else "pianosim_kernel<true"  # <XG, waves per SIMD>


def counter(d, name):
    per_dispatch = defaultdict(float)
    for r in rows(d, "*counter_collection.csv"):
        if KNAME not in r.get("Kernel_Name", ""):
            continue
        if r.get("Counter_Name") != name:
            continue
        per_dispatch[r.get("Dispatch_Id")] += float(r["Counter_Value"])
    vals = list(per_dispatch.values())
    return sum(vals) / len(vals) if vals else None


SQ_COUNTERS = ("SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_WAIT_ANY",
               "SQ_WAIT_INST_ANY", "SQ_INSTS_VALU", "SQ_INSTS_LDS")


def main():
    tdir, fdir, wdir, envs, song, prefix = sys.argv[1:4] + [int(sys.argv[4])] + sys.argv[5:7]
    warmup = int(sys.argv[7]) if len(sys.argv) > 7 else 5
    sqdir = sys.argv[8] if len(sys.argv) > 8 else None
    stats = [r for r in rows(tdir, "*kernel_stats.csv") if KNAME in r.get("Name", "")]
    fetch_kb = counter(fdir, "FETCH_SIZE")
    write_kb = counter(wdir, "WRITE_SIZE")
    sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
    from bench import lib_sha  # the profiled binary (bench.py quotes only profiles of its own build)
    hand = HAND
    out = {"envs": envs, "song": song, "hand": hand, "kernel": KNAME, "lib_sha": lib_sha()}
    if stats:
        s = stats[0]
        out["rocprof_avg_ns_all_launches"] = float(s.get("AverageNs", 0))
        out["rocprof_calls"] = int(s.get("Calls", 0))
    # the timed steps only: bench.py launches reset (1) + warmup (5) before the timed region
    tr = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows(tdir, "*kernel_trace.csv")
                if KNAME in r.get("Kernel_Name", ""))
    timed = [e - b for b, e in tr[1 + warmup:]]
    if timed:
        out["rocprof_avg_ns"] = sum(timed) / len(timed)
        out["rocprof_timed_launches"] = len(timed)
    if fetch_kb is not None and write_kb is not None:
        out["fetch_kb_per_launch"] = fetch_kb
        out["write_kb_per_launch"] = write_kb
        out["hbm_bytes_per_launch"] = (2.0 * fetch_kb + write_kb) * 1024.0
    if sqdir:
        sq = {c: counter(sqdir, c) for c in SQ_COUNTERS}
        if all(v is not None for v in sq.values()):
            out["sq_per_launch"] = sq
            wc = sq["SQ_WAVE_CYCLES"]
            out["wave_issue_frac"] = sq["SQ_ACTIVE_INST_ANY"] / wc  # lifetime issuing
            out["wave_wait_frac"] = sq["SQ_WAIT_ANY"] / wc  # waiting on s_waitcnt
            out["wave_issue_stall_frac"] = sq["SQ_WAIT_INST_ANY"] / wc  # issue stalls (RAW dependency / pipe)
            out["valu_insts_per_env_step"] = sq["SQ_INSTS_VALU"] / envs
    Path("profiles").mkdir(exist_ok=True)
    if stats:
        with open(f"profiles/{prefix}_kernel_stats.csv", "w", newline="") as fh:
            w = csv.DictWriter(fh, fieldnames=list(stats[0].keys()))
            w.writeheader()
            w.writerows(rows(tdir, "*kernel_stats.csv"))
    Path(f"profiles/{prefix}_pmc.json").write_text(json.dumps(out, indent=1))
    if hand == "hull":  # the bench's default workload; the other sets' summaries stay under their prefix
        Path("profiles/pmc_latest.json").write_text(json.dumps(out, indent=1))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
