"""Aggregate rocprofv3 --pmc CSVs: per kernel, mean counter value per dispatch.

FETCH_SIZE/WRITE_SIZE are KB (rocprofv3 derived counters).  On gfx950
FETCH_SIZE reads half the bytes of wide streaming loads
(MI355X_MICROARCH.md §HBM), so hbm_bytes_per_launch = (2*FETCH_SIZE +
WRITE_SIZE) * 1024 — an upper estimate for narrower gathers.
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def short(name):
    m = re.search(r"tile_kernel<\w+, (\d)", name)   # dense tiles: one entry per mode
    if m:
        return "tile_kernel_m" + m.group(1)
    m = re.search(r"(\w+_kernel)\b", name)
    if m:
        return m.group(1)
    if "rocprim" in name:
        for k in ("radix_sort", "scan", "select", "partition"):
            if k in name:
                return "rocprim_" + k
    return name[:60]


REPS = int(os.environ.get("PROF_REPS", "2"))   # trains per profiled run (tools/prof_one.py)


def main(dirs):
    acc = defaultdict(lambda: defaultdict(list))
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for row in csv.DictReader(open(f)):
                k = short(row.get("Kernel_Name", ""))
                c = row.get("Counter_Name")
                try:
                    v = float(row.get("Counter_Value", "nan"))
                except ValueError:
                    continue
                disp = row.get("Dispatch_Id") or row.get("Correlation_Id") or ""
                acc[k][c].append((disp, v))
    out = {}
    for k, cs in acc.items():
        o = {}
        for c, vals in cs.items():
            per = defaultdict(float)
            for disp, v in vals:
                per[disp] += v        # sum over dimensions (XCD/SE instances)
            o[c] = sum(per.values()) / max(1, len(per))
        if "FETCH_SIZE" in o or "WRITE_SIZE" in o:
            o["hbm_bytes_per_launch"] = (2 * o.get("FETCH_SIZE", 0.0) + o.get("WRITE_SIZE", 0.0)) * 1024
        # dispatches of this kernel name per profiled train (the FETCH_SIZE
        # pass: every counter pass runs the same trains)
        disp = {dd for dd, _ in cs.get("FETCH_SIZE", next(iter(cs.values())))}
        o["dispatches_per_train"] = len(disp) / REPS
        out[k] = o
    out["_meta"] = {"trains": REPS, "note": "counter values: mean per dispatch; "
                    "dispatches_per_train: launches of this kernel name in one train"}
    json.dump(out, sys.stdout, indent=1, sort_keys=True)


if __name__ == "__main__":
    main(sys.argv[1:])
