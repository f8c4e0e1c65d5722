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
    if not d:
        return {}
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for f in files:
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k].add(r["Dispatch_Id"])
    return {k: {c: v / len(disp[k]) for c, v in cs.items()} for k, cs in agg.items()}


def load_trace(d):
    files = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)
    out = {}
    for f in files:
        for r in csv.DictReader(open(f)):
            out[short(r["Name"])] = {"calls": int(r["Calls"]),
                                      "avg_ms": float(r["AverageNs"]) / 1e6,
                                      "total_ms": float(r["TotalDurationNs"]) / 1e6,
                                      "pct": float(r["Percentage"])}
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
