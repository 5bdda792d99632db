import csv, glob, os, sys
from collections import defaultdict
out = sys.argv[1]
def short(n):
    for k in ("k_commit_step", "k_grad_reduce", "k_adam_tf", "k_prep_sort", "k_prep_counts"):
        if k in n:
            return k
    return None
vals = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(out, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k = short(r["Kernel_Name"])
        if k:
            vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in vals.items():
    med = {c: sorted(v)[len(v) // 2] for c, v in d.items()}
    waves = med.get("SQ_WAVES", 1)
    print("==", k)
    for c in sorted(med):
        per = med[c] / waves if waves else 0
        print("  %-24s %16.0f   per-wave %12.1f" % (c, med[c], per))
