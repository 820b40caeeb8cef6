"""Static report on a built libfdfs_gpu (CPU only; tests/isa_check.py):
per kernel the register and scratch metadata, the counted `vmcnt(N > 0)`
waits, and every instruction that names a register a vector-memory load is
still writing (vm_hazards), plus the MFMA/DPP wait-state hazards.

usage: python scripts/isa_report.py [LIB] [--kernel SUBSTRING]

DESIGN.md 4.1 uses it on the round-5 forced-four-wave crc_lane_kernel
(rebuilt on the CPU box: amdgpu_waves_per_eu(4) on the kernel) to name the
cause of that build's wrong CRCs (profiles/r06/isa_w4_variant.txt)."""
import argparse
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import isa_check as I  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib", nargs="?", default=os.path.join(ROOT, "fastdfs_amd", "lib", "libfdfs_gpu.so"))
    ap.add_argument("--kernel", default="")
    ap.add_argument("--show", type=int, default=12, help="hazards listed per kernel")
    a = ap.parse_args()
    r = I.check_library(a.lib)
    print(f"# {a.lib}: {r['functions']} functions")
    per = collections.defaultdict(list)
    for h in r["vm_hazards"]:
        fn, what = h.split(": ", 1)
        per[fn].append(what)
    for fn, m in sorted(r["meta"].items()):
        if a.kernel not in fn:
            continue
        waits = r["counted_waits"].get(fn, 0)
        hz = per.get(fn, [])
        if not (waits or hz or m.get("private_segment_fixed_size")):
            continue
        print(f"{fn}\n  vgpr {m.get('vgpr_count')} agpr {m.get('agpr_count')} "
              f"scratch {m.get('private_segment_fixed_size')} B (vgpr spills {m.get('vgpr_spill_count')}, "
              f"sgpr spills {m.get('sgpr_spill_count')}); counted vmcnt waits {waits}; "
              f"in-flight-load hazards {len(hz)}")
        for w in hz[:a.show]:
            print("    " + w)
    other = [h for h in r["hazards"] if a.kernel in h]
    print(f"# MFMA/DPP wait-state hazards: {len(other)}; in-flight-load hazards: "
          f"{sum(len(v) for k, v in per.items() if a.kernel in k)}")


if __name__ == "__main__":
    main()
