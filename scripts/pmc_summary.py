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


def load(root, how="mean"):
    """Per kernel and counter: the mean over its dispatches, or (how="max")
    the largest dispatch's value (config 3's bench also runs the MD5 kernel
    on its largest file alone for the chain floor; those one-file dispatches
    would halve a mean)."""
    per = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            per[row["Kernel_Name"]][row["Counter_Name"]][row["Dispatch_Id"]] += float(row["Counter_Value"])
    out = {}
    for k, cs in per.items():
        if how == "max":
            out[k] = {c: max(d.values()) for c, d in cs.items()}
        else:
            out[k] = {c: sum(d.values()) / max(1, len(d)) for c, d in cs.items()}
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
