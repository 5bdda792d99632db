"""Summarise a tools/profile.sh run (merged back under gpurun_out/prof_<tag>) into
profiles/<tag>/ (kernel stats + HBM traffic) and profiles/hbm_traffic.json (bench.py's
roofline.traffic source).  Run locally after the gpurun call:
    python tools/prof_summary.py gpurun_out/prof_r01 r01"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

out, tag = sys.argv[1], sys.argv[2]
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
dst = os.path.join(root, "profiles", tag)
os.makedirs(dst, exist_ok=True)


def find(pattern):
    hits = glob.glob(os.path.join(out, "**", pattern), recursive=True)
    return sorted(hits)


def short(name):
    for k in ("k_commit_step", "k_grad_reduce", "k_adam_tf", "k_prep_sort", "k_prep_counts"):
        if k in name:
            return k
    return name[:60]


lines = []
stats = find("*kernel_stats.csv")
if stats:
    with open(stats[0]) as f:
        rows = list(csv.DictReader(f))
    lines.append("# rocprofv3 --kernel-trace --stats: bench.py --steps 50 --warmup 10 (glide B=100)")
    lines.append("%-16s %8s %12s %12s %8s" % ("kernel", "calls", "avg_us", "total_us", "pct"))
    for r in rows:
        lines.append("%-16s %8s %12.2f %12.1f %8s" % (short(r["Name"]), r["Calls"],
                                                     float(r["AverageNs"]) / 1e3,
                                                     float(r["TotalDurationNs"]) / 1e3,
                                                     r.get("Percentage", "")))
    with open(os.path.join(dst, "kernel_stats.csv"), "w") as f:
        f.write(open(stats[0]).read())


def pmc(kind):
    files = find("*counter_collection.csv")
    files = [p for p in files if ("pmc_" + kind) in p]
    acc = defaultdict(list)
    if not files:
        return acc
    with open(files[0]) as f:
        for r in csv.DictReader(f):
            acc[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return acc


fetch, write = pmc("fetch"), pmc("write")
traffic = {}
if fetch or write:
    lines.append("")
    lines.append("# HBM traffic per launch (separate --pmc passes; FETCH_SIZE/WRITE_SIZE in KiB,")
    lines.append("# gfx950 correction: FETCH_SIZE counts half of wide streaming reads -> x2)")
    lines.append("%-16s %14s %14s %16s" % ("kernel", "FETCH_KiB", "WRITE_KiB", "bytes(2F+W)"))
    for k in sorted(set(fetch) | set(write)):
        fv = sorted(fetch.get(k, [0]))[len(fetch.get(k, [0])) // 2]
        wv = sorted(write.get(k, [0]))[len(write.get(k, [0])) // 2]
        b = (2 * fv + wv) * 1024
        traffic[k] = b
        lines.append("%-16s %14.1f %14.1f %16.0f" % (k, fv, wv, b))
txt = "\n".join(lines) + "\n"
with open(os.path.join(dst, "summary.txt"), "w") as f:
    f.write(txt)
print(txt)
if traffic:
    with open(os.path.join(dst, "hbm_traffic_all.json"), "w") as f:
        json.dump({"batch": 100, "ne": 200, "nc": 74, "bytes_per_launch": traffic}, f, indent=1)
    if "k_commit_step" in traffic:
        with open(os.path.join(root, "profiles", "hbm_traffic.json"), "w") as f:
            json.dump({"kernel": "k_commit_step", "batch": 100, "ne": 200, "nc": 74,
                       "bytes_per_launch": traffic["k_commit_step"],
                       "source": "profiles/%s/summary.txt (2*FETCH_SIZE + WRITE_SIZE)" % tag},
                      f, indent=1)
