"""Clock and issue picture of one kernel from rocprofv3 --pmc passes.

For each pass directory (run_counter_collection.csv) the dispatches of the
kernel whose name contains PATTERN are read; per dispatch it prints the
duration, the clock the chip held (GRBM_GUI_ACTIVE is summed over the 8 XCDs:
clock = GRBM_GUI_ACTIVE / 8 / duration, MI355X_MICROARCH.md 'DVFS
give-back') and, when the pass holds them, the SQ counters per wave and as
fractions of the wave cycles (SQ_*_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_*
count quad-cycles).  The last dispatch of each pass is the steady one.

usage: python3 scripts/pmc_clock.py PATTERN DIR[+DIR2...] ...
  DIR+DIR2: passes of the same command, merged by dispatch id; with
  SQ_ACTIVE_INST_ANY and GRBM_GUI_ACTIVE merged it also prints the SIMDs'
  issue occupancy = 4 x sum(SQ_ACTIVE_INST_ANY) / (SIMDs x GUI cycles per
  XCD): near 1.0 when every SIMD issues an instruction every quad-cycle.
"""
import collections
import csv
import sys

SIMDS = 256 * 4  # MI355X: 256 CUs x 4 SIMDs

def dispatches(d, pat):
    r = collections.OrderedDict()
    for row in csv.DictReader(open(d + "/run_counter_collection.csv")):
        if pat not in row["Kernel_Name"]:
            continue
        k = int(row["Dispatch_Id"])
        e = r.setdefault(k, {"t0": int(row["Start_Timestamp"]), "t1": int(row["End_Timestamp"]),
                             "name": row["Kernel_Name"], "c": collections.defaultdict(float)})
        e["c"][row["Counter_Name"]] += float(row["Counter_Value"])
    return r


def main():
    pat, dirs = sys.argv[1], sys.argv[2:]
    for d in dirs:
        merged = collections.OrderedDict()
        for part in d.split("+"):
            for k, e in dispatches(part, pat).items():
                m = merged.setdefault(k, e)
                if m is not e:
                    for n, v in e["c"].items():
                        m["c"][n] = v
        for k, e in merged.items():
            c, dur = e["c"], (e["t1"] - e["t0"]) * 1e-9
            line = [f"{d} dispatch {k} {dur * 1e3:.3f} ms"]
            if "GRBM_GUI_ACTIVE" in c:
                line.append(f"clock {c['GRBM_GUI_ACTIVE'] / 8 / dur / 1e9:.2f} GHz")
            if "SQ_WAVES" in c and c["SQ_WAVES"]:
                w = c["SQ_WAVES"]
                for n in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU"):
                    if n in c:
                        line.append(f"{n[9:].lower()}/wave {c[n] / w:.0f}")
            if "SQ_WAVE_CYCLES" in c and c["SQ_WAVE_CYCLES"]:
                wc = c["SQ_WAVE_CYCLES"]
                for n in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY"):
                    if n in c:
                        line.append(f"{n[3:].lower()} {c[n] / wc:.3f}")
            if "SQ_ACTIVE_INST_ANY" in c and "GRBM_GUI_ACTIVE" in c:
                line.append(f"simd_issue {4 * c['SQ_ACTIVE_INST_ANY'] / (SIMDS * c['GRBM_GUI_ACTIVE'] / 8):.2f}")
            print("  ".join(line))


if __name__ == "__main__":
    main()
