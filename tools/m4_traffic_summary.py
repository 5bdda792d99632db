"""Per-kernel HBM traffic + SQ summary of model_4 hybrid at glide from tools/pmc_m4_traffic.sh
(merged under gpurun_out/pmc_m4).  FETCH_SIZE / WRITE_SIZE in KiB per dispatch, averaged
per kernel; bytes = 2 FETCH + WRITE (the gfx950 correction of profiles/r03/summary.txt).
    python tools/m4_traffic_summary.py gpurun_out/pmc_m4 profiles/r03/m4_traffic.txt"""
import csv
import glob
import os
import sys
from collections import defaultdict


def per_kernel(path):
    acc = defaultdict(list)
    for f in glob.glob(os.path.join(path, "**", "run_counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            acc[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def short(n):
    n = n.replace("hdg::", "").replace("(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0][:28]


def main(src, dst):
    fe, wr = per_kernel(os.path.join(src, "FETCH_SIZE")), per_kernel(os.path.join(src, "WRITE_SIZE"))
    rows = []
    for k in fe:
        if k in wr and ("kw_" in k or "k_commit_step" in k):
            rows.append((short(k), fe[k], wr[k], (2 * fe[k] + wr[k]) * 1024))
    rows.sort(key=lambda r: -r[3])
    out = ["# model_4 hybrid, glide B=100: HBM traffic per launch (rocprofv3 --pmc FETCH_SIZE / "
           "WRITE_SIZE, separate passes; KiB; bytes = 2 FETCH + WRITE)",
           "%-30s %12s %12s %14s" % ("kernel", "FETCH_KiB", "WRITE_KiB", "bytes")]
    out += ["%-30s %12.1f %12.1f %14.0f" % r for r in rows]
    sq = os.path.join(src, "sq.txt")
    if os.path.exists(sq):
        out += ["", "# SQ counters (tools/pmc_sq_m4.sh, eager launches)"] + open(sq).read().splitlines()
    open(dst, "w").write("\n".join(out) + "\n")
    print("\n".join(out[:14]))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
