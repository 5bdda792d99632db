"""Median per-dispatch counter values per kernel from rocprofv3 --pmc CSV output.
    python tools/pmc_table.py <dir> [--json out.json]"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def short(n):
    n = re.sub(r"^void ", "", n)
    n = re.sub(r"\(anonymous namespace\)::", "", n)
    n = n.split("(")[0]
    return n.split("<")[0] if not n.startswith("k_commit_step") else n.split("(")[0]


def table(out):
    vals = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(out, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            vals[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: {c: sorted(v)[len(v) // 2] for c, v in d.items()} for k, d in vals.items()}


if __name__ == "__main__":
    res = table(sys.argv[1])
    for k, med in sorted(res.items()):
        waves = med.get("SQ_WAVES", 0)
        print("==", k)
        for c in sorted(med):
            per = "   per-wave %12.1f" % (med[c] / waves) if waves else ""
            print("  %-30s %16.0f%s" % (c, med[c], per))
    if "--json" in sys.argv:
        with open(sys.argv[sys.argv.index("--json") + 1], "w") as f:
            json.dump(res, f, indent=1, sort_keys=True)
