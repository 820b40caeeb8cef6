"""Per-call kernel breakdown from a rocprofv3 --kernel-trace run of a script
that made `calls` identical calls after `skip` warm-up calls: each fdfs
kernel's dispatches and mean duration per call (the first `skip` calls'
dispatches dropped by timestamp order), plus the summed kernel time.

python3 scripts/kernel_share.py <trace dir> <calls> [skip]
"""
import csv
import glob
import sys
from collections import OrderedDict


def main(d, calls, skip=0):
    tr = sorted(glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True))[0]
    rows = [r for r in csv.DictReader(open(tr)) if "fdfs::" in (r.get("Kernel_Name") or "")]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    per = OrderedDict()
    for r in rows:
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("fdfs::", "")
        per.setdefault(k, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    total = 0.0
    print(f"# per call of {calls} timed calls ({skip} warm-up calls dropped): kernel, dispatches/call, ms/call, mean ms")
    for k, v in per.items():
        per_call = len(v) // (calls + skip)
        v = v[per_call * skip:]
        ms = sum(v) / calls
        total += ms
        print(f"{k:60s} {per_call:3d} {ms:8.4f} {sum(v) / max(len(v), 1):8.4f}")
    print(f"{'sum of kernel time per call':60s}     {total:8.4f}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), int(sys.argv[3]) if len(sys.argv) > 3 else 0)
