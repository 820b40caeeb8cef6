"""Summarise rocprofv3 PMC csv files per kernel (average per dispatch).

python scripts/pmc_summary.py <dir-with-*/run_counter_collection.csv> [kernel-substring]
Applies the gfx950 FETCH_SIZE correction of MI355X_MICROARCH.md (HBM
section): FETCH_SIZE (KiB) reads half the bytes of a wide coalesced stream,
so HBM read bytes = 2 * FETCH_SIZE * 1024; WRITE_SIZE * 1024 as is.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(root):
    acc = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            k = row["Kernel_Name"]
            acc[k][row["Counter_Name"]] += float(row["Counter_Value"])
            disp[(k, row["Counter_Name"])].add(row["Dispatch_Id"])
    out = {}
    for k, cs in acc.items():
        out[k] = {c: v / max(1, len(disp[(k, c)])) for c, v in cs.items()}
    return out


if __name__ == "__main__":
    root = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 else ""
    for k, cs in load(root).items():
        if sub and sub not in k:
            continue
        short = k.split("(")[0]
        d = dict(cs)
        if "FETCH_SIZE" in d:
            d["hbm_read_bytes_corrected"] = 2 * d["FETCH_SIZE"] * 1024
        if "WRITE_SIZE" in d:
            d["hbm_write_bytes"] = d["WRITE_SIZE"] * 1024
        print(short, json.dumps({a: round(b, 1) for a, b in d.items()}))
