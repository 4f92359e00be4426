#!/usr/bin/env python3
"""Per-launch HBM traffic of each kernel from rocprofv3 PMC passes -> profiles/traffic.json.

Usage: tools/traffic.py <prof_dir> <bench_log> <tag>
  prof_dir  : tools/profile.sh output (pmc*/ passes with FETCH_SIZE and WRITE_SIZE)
  bench_log : the bench.py JSON line of the same workload (its config.workload keys the entry)

Correction (MI355X_MICROARCH.md, HBM section): on gfx950 FETCH_SIZE reports half the
bytes of a 16-B-per-lane streaming read; the pixel kernel's dominant reads are
global_load_dwordx4 BGR chunks, so traffic = 2 * FETCH_SIZE + WRITE_SIZE (KiB -> bytes).
bench.py reports this as roofline.traffic when its workload matches.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

SHORT = {"k_pix": "pix", "k_pix5": "pix", "k_pixw": "pix", "k_tile_ccl": "tile_ccl", "k_merge": "merge", "k_fold_emit": "fold_emit", "k_fold": "fold", "k_emit": "emit",
         "k_regions": "regions", "k_resize_area": "resize_area", "k_resize_area_nt": "resize_area",
         "k_small_blur": "small_blur", "k_small_scan": "small_scan", "k_frame_contours": "frame_contours", "k_pixel": "pixel"}


def short(name):
    base = name.split("(")[0]
    for k, v in SHORT.items():
        if base.split("<")[0].endswith(k):
            return v
    return None


def main(prof, bench_log, tag):
    acc = defaultdict(lambda: defaultdict(list))
    for f in sorted(glob.glob(os.path.join(prof, "**", "*counter_collection.csv"), recursive=True)):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = row["Kernel_Name"]
                if "k_pix<" in k and ", true>" in k:  # the init-frame variant is a one-off
                    continue
                s = short(k)
                if s:
                    acc[s][row["Counter_Name"]].append(float(row["Counter_Value"]))
    line = [l for l in open(bench_log).read().splitlines() if l.startswith("{")][-1]
    workload = json.loads(line)["config"]["workload"]
    out = {"tag": tag, "workload": workload, "source": f"profiles/{tag}_pmc.txt", "kernels": {}}
    for k, cs in acc.items():
        if "FETCH_SIZE" not in cs or "WRITE_SIZE" not in cs:
            continue
        fetch = sum(cs["FETCH_SIZE"]) / len(cs["FETCH_SIZE"]) * 1024
        write = sum(cs["WRITE_SIZE"]) / len(cs["WRITE_SIZE"]) * 1024
        out["kernels"][k] = {"fetch_size_bytes": round(fetch), "write_size_bytes": round(write),
                             "traffic_bytes": round(2 * fetch + write), "dispatches": len(cs["FETCH_SIZE"])}
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        if m.get("SQ_WAVE_CYCLES"):
            # what bounds the kernel, from the SQ counters of the same passes (per dispatch means):
            # WAIT_ANY (parked on s_waitcnt / barrier) + WAIT_INST_ANY (issue stalls) + ACTIVE_INST_ANY
            # = WAVE_CYCLES (MI355X_MICROARCH.md, rocprofv3 PMC slots)
            wc = m["SQ_WAVE_CYCLES"]
            out["kernels"][k]["sq"] = {
                "wait_any_frac": round(m.get("SQ_WAIT_ANY", 0) / wc, 3),
                "wait_inst_any_frac": round(m.get("SQ_WAIT_INST_ANY", 0) / wc, 3),
                "active_inst_any_frac": round(m.get("SQ_ACTIVE_INST_ANY", 0) / wc, 3),
                "valu_insts": round(m.get("SQ_INSTS_VALU", 0)), "salu_insts": round(m.get("SQ_INSTS_SALU", 0)),
                "lds_insts": round(m.get("SQ_INSTS_LDS", 0)),
                "lds_bank_conflict_per_active": round(m.get("SQ_LDS_BANK_CONFLICT", 0) / max(m.get("SQ_ACTIVE_INST_LDS", 1), 1), 3),
                "waves": round(m.get("SQ_WAVES", 0))}
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "profiles", "traffic.json")
    entries = []
    try:  # one entry per workload: replace this workload's, keep the others
        with open(path) as fh:
            old = json.load(fh)
        entries = [e for e in old.get("entries", [old]) if e.get("workload") != workload]
    except (OSError, ValueError):
        pass
    with open(path, "w") as fh:
        json.dump({"entries": entries + [out]}, fh, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:4])
