#!/usr/bin/env python3
"""Summarise rocprofv3 outputs into profiles/ (measurement infrastructure).

  tools/pmc_summary.py --trace DIR --fetch DIR --write DIR --sq DIR --out profiles/pmc_sumvec.json

HBM bytes per launch follow MI355X_MICROARCH.md §HBM: FETCH_SIZE (KiB) reads exactly half of a wide
coalesced stream's bytes on gfx950, so read bytes = 2 x FETCH_SIZE x 1024; WRITE_SIZE x 1024 for
writes.  (Other access widths are uncalibrated; the per-kernel `note` says which applies.)
"""
import argparse
import collections
import csv
import glob
import json
import os


def short(name):
    n = name.split("(")[0]
    n = n.replace("void ", "").replace("p3g::", "")
    return n.split("<")[0]


def load_counters(d):
    """Per-kernel counter values averaged over the FULL-SIZE dispatches (those with the kernel's
    largest grid: the bench's timed batches, not its small parity-gate batch)."""
    if not d:
        return {}
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    rows = collections.defaultdict(lambda: collections.defaultdict(dict))  # k -> disp -> {..}
    grid = {}
    for f in files:
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            dsp = r["Dispatch_Id"]
            rows[k][dsp][r["Counter_Name"]] = rows[k][dsp].get(r["Counter_Name"], 0.0) + \
                float(r["Counter_Value"])
            grid[(k, dsp)] = int(r["Grid_Size"])
    out = {}
    for k, disp in rows.items():
        gmax = max(grid[(k, dsp)] for dsp in disp)
        full = [c for dsp, c in disp.items() if grid[(k, dsp)] == gmax]
        names = set().union(*full)
        out[k] = {c: sum(x.get(c, 0.0) for x in full) / len(full) for c in names}
        out[k]["dispatches_full"] = len(full)
    return out


def load_trace(d):
    """Per-kernel durations: all dispatches (kernel_stats.csv) and the full-size ones (largest
    grid, from kernel_trace.csv) -- `avg_ms` is the full-size average, the number the bench's HIP
    events time."""
    out = {}
    for f in glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            out[short(r["Name"])] = {"calls_all": int(r["Calls"]),
                                      "avg_ms_all": float(r["AverageNs"]) / 1e6,
                                      "total_ms": float(r["TotalDurationNs"]) / 1e6,
                                      "pct": float(r["Percentage"])}
    disp = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            g = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
            disp[short(r["Kernel_Name"])].append(
                (g, (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6))
    for k, v in disp.items():
        gmax = max(g for g, _ in v)
        full = [t for g, t in v if g == gmax]
        e = out.setdefault(k, {})
        e.update({"calls": len(full), "avg_ms": sum(full) / len(full), "grid": gmax})
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trace")
    ap.add_argument("--fetch")
    ap.add_argument("--write")
    ap.add_argument("--sq")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    tr = load_trace(a.trace) if a.trace else {}
    fe, wr, sq = load_counters(a.fetch), load_counters(a.write), load_counters(a.sq)
    res = {}
    for k in sorted(set(tr) | set(fe) | set(wr) | set(sq)):
        if not k.startswith("k_"):
            continue
        e = {}
        if k in tr:
            e.update(tr[k])
        rd = fe.get(k, {}).get("FETCH_SIZE")
        wb = wr.get(k, {}).get("WRITE_SIZE")
        if rd is not None:
            e["hbm_read_bytes_per_launch"] = 2 * rd * 1024
        if wb is not None:
            e["hbm_write_bytes_per_launch"] = wb * 1024
        if rd is not None and wb is not None:
            e["hbm_bytes_per_launch"] = 2 * rd * 1024 + wb * 1024
        for c, v in sq.get(k, {}).items():
            e[c] = v
        if "SQ_INSTS_VALU" in e and "SQ_WAVES" in e:
            e["valu_insts_per_wave"] = e["SQ_INSTS_VALU"] / max(1.0, e["SQ_WAVES"])
        res[k] = e
    json.dump(res, open(a.out, "w"), indent=1)
    for k, e in res.items():
        print(k, {x: (round(y, 4) if isinstance(y, float) else y) for x, y in e.items()})


if __name__ == "__main__":
    main()
