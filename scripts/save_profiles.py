"""Copy a gpu_round.sh run's evidence into profiles/<round>/ (short kernel
names, fdfs kernels only) and refresh profiles/pmc_<config>.json, the HBM
traffic per launch that bench.py reports as roofline.traffic.

python scripts/save_profiles.py gpurun_out/round_r01b profiles/r01
"""
import csv
import glob
import json
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import load  # noqa: E402

BENCH_KERNEL = {"c2": ("sig_hash_kernel<true, false>", "sig_hash_kernel<SAR>"),
                "c3": ("md5_pair_kernel<true", "md5_pair_kernel<SAR>"),
                "c4": ("crc_seg_kernel<true>", "crc_seg_kernel<SAR>")}


BENCH_C5_KERNEL = "dedup_group (dp_tile + scan + chunks + dp_split + dp_group)"


def short(name):
    return name.split("(")[0].replace("void ", "").replace("fdfs::", "")


def steady(trace, out_path):
    """Per fdfs kernel from a kernel trace: dispatches, mean over all, mean
    without the first dispatch (cold: first touch of the batch's pages, the
    tables' upload), min and max, in ms."""
    per = {}
    for r in csv.DictReader(open(trace)):
        name = r.get("Kernel_Name") or r.get("Name") or ""
        if "fdfs::" not in name:
            continue
        t = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        per.setdefault(short(name), []).append(t)
    with open(out_path, "w") as out:
        out.write("# kernel dispatches mean_ms mean_without_first_ms min_ms max_ms (rocprofv3 --kernel-trace)\n")
        for k, v in sorted(per.items(), key=lambda kv: -sum(kv[1])):
            rest = v[1:] if len(v) > 1 else v
            out.write(f"{k} {len(v)} {sum(v) / len(v):.4f} {sum(rest) / len(rest):.4f} {min(v):.4f} {max(v):.4f}\n")


def main(src, dst):
    os.makedirs(dst, exist_ok=True)
    for c in ("c1", "c2", "c3", "c4", "c5", "c4_hash", "c4_md5", "c2_crc"):
        log = os.path.join(src, f"bench_{c}.log")
        if os.path.exists(log):
            line = open(log).read().strip().split("\n")[-1]
            json.loads(line)
            open(os.path.join(dst, f"bench_{c}.json"), "w").write(line + "\n")
    for c in ("c1", "c2", "c3", "c4", "c5"):
        for f in glob.glob(os.path.join(src, f"stats_{c}", "**", "*kernel_stats.csv"), recursive=True):
            rows = list(csv.DictReader(open(f)))
            with open(os.path.join(dst, f"kernel_stats_{c}.csv"), "w", newline="") as out:
                w = csv.DictWriter(out, fieldnames=list(rows[0].keys()))
                w.writeheader()
                for r in rows:
                    if "fdfs::" in r["Name"] or "rocclr" in r["Name"]:
                        r["Name"] = short(r["Name"])
                        w.writerow(r)
        for f in glob.glob(os.path.join(src, f"stats_{c}", "**", "*kernel_trace.csv"), recursive=True):
            steady(f, os.path.join(dst, f"kernel_steady_{c}.txt"))
        if c == "c5":  # the dedup group is five kernels: traffic summed over them
            tot = {}
            for kind in ("fetch", "write"):
                if not os.path.isdir(os.path.join(src, f"{kind}_{c}")):
                    continue
                d = load(os.path.join(src, f"{kind}_{c}"))
                with open(os.path.join(dst, f"pmc_{kind}_{c}.txt"), "w") as out:
                    for k, v in d.items():
                        if "fdfs::" in k:
                            out.write(f"{short(k)} {json.dumps(v)}\n")
                for k, v in d.items():
                    if any(x in k for x in ("dp_tile", "dp_chunk", "dp_split", "dp_group",
                                            "scan_reduce", "scan_sums", "scan_apply")):
                        for m, val in v.items():
                            tot[m] = tot.get(m, 0.0) + val
            if "FETCH_SIZE" in tot and "WRITE_SIZE" in tot:
                rd, wr = 2 * tot["FETCH_SIZE"] * 1024, tot["WRITE_SIZE"] * 1024
                rel = os.path.relpath(dst, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
                json.dump({"kernel": BENCH_C5_KERNEL, "hbm_bytes_per_launch": round(rd + wr),
                           "read_bytes": round(rd), "write_bytes": round(wr),
                           "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes, summed over the "
                                     "dedup_group kernels; read = 2 x FETCH_SIZE x 1024 (gfx950 "
                                     "correction), write = WRITE_SIZE x 1024",
                           "files": [f"{rel}/pmc_fetch_{c}.txt", f"{rel}/pmc_write_{c}.txt"]},
                          open(os.path.join(os.path.dirname(dst), f"pmc_{c}.json"), "w"), indent=1)
            continue
        if c not in BENCH_KERNEL:
            continue
        pm = {}
        for kind in ("fetch", "write"):
            if not os.path.isdir(os.path.join(src, f"{kind}_{c}")):
                continue  # no PMC pass for this config in this run: keep the committed one
            d = load(os.path.join(src, f"{kind}_{c}"), "max" if c == "c3" else "mean")
            with open(os.path.join(dst, f"pmc_{kind}_{c}.txt"), "w") as out:
                for k, v in d.items():
                    if "fdfs::" in k:
                        out.write(f"{short(k)} {json.dumps(v)}\n")
            for k, v in d.items():
                if BENCH_KERNEL[c][0] in k:
                    pm.update(v)
        if "FETCH_SIZE" in pm and "WRITE_SIZE" in pm:
            rd, wr = 2 * pm["FETCH_SIZE"] * 1024, pm["WRITE_SIZE"] * 1024
            rel = os.path.relpath(dst, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
            json.dump({"kernel": BENCH_KERNEL[c][1], "hbm_bytes_per_launch": round(rd + wr),
                       "read_bytes": round(rd), "write_bytes": round(wr),
                       "source": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE (separate passes); "
                                 "read = 2 x FETCH_SIZE x 1024 (gfx950 correction, MI355X_MICROARCH.md "
                                 "HBM section), write = WRITE_SIZE x 1024",
                       "files": [f"{rel}/pmc_fetch_{c}.txt", f"{rel}/pmc_write_{c}.txt"]},
                      open(os.path.join(os.path.dirname(dst), f"pmc_{c}.json"), "w"), indent=1)
    for c in ("c2", "c3", "c4"):
        if not os.path.isdir(os.path.join(src, f"sq_{c}")):
            continue
        # clock and SIMD issue occupancy of the dominant kernel, per dispatch
        pat = {"c2": "sig_hash_kernel", "c3": "md5_pair_kernel", "c4": "crc_seg_kernel"}[c]
        with open(os.path.join(dst, f"issue_clock_{c}.txt"), "w") as out:
            out.write(f"# python3 scripts/pmc_clock.py {pat} sq_{c} (one pass)\n")
            out.write(subprocess.run([sys.executable, os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                                                   "pmc_clock.py"), pat, os.path.join(src, f"sq_{c}")],
                                     capture_output=True, text=True, check=True).stdout.replace(src + "/", ""))
        sq = load(os.path.join(src, f"sq_{c}"), "max" if c == "c3" else "mean")  # c3: skip the chain-floor dispatches
        with open(os.path.join(dst, f"pmc_sq_{c}.txt"), "w") as out:
            for k, v in sq.items():
                if "fdfs::" in k:
                    out.write(f"{short(k)} {json.dumps(v)}\n")

if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
