"""VALU issue view of k_commit_step (the engine's executed-instruction roofline): from a
tools/pmc_sq.sh run (SQ_INSTS_VALU, SQ_WAVES per launch) and the rocprofv3 kernel-trace
average duration, write profiles/<tag>/valu_issue.json:
  issue_frac = VALU wave-instructions per launch / (duration * clock * SIMDs / 4)
(a wave64 VALU instruction occupies a 16-lane SIMD for 4 cycles; 4 SIMDs per CU; gfx950
peak engine clock 2.4 GHz, MI355X_MICROARCH.md).  Reported for the whole chip (256 CUs)
and for the CUs the grid occupies (one 1024-thread block per CU).
    python tools/valu_issue.py gpurun_out/pmc_sq gpurun_out/prof_r01 r01 200"""
import csv
import glob
import json
import os
import sys

sq, prof, tag, blocks = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4])
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLOCK, CUS, SIMDS = 2.4e9, 256, 4

vals = {}
for f in glob.glob(os.path.join(sq, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_commit_step" in r["Kernel_Name"]:
            vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
med = {k: sorted(v)[len(v) // 2] for k, v in vals.items()}
dur = None
for f in glob.glob(os.path.join(prof, "**", "*kernel_stats.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_commit_step" in r["Name"]:
            dur = float(r["AverageNs"]) * 1e-9
valu = med.get("SQ_INSTS_VALU")
out = {"kernel": "k_commit_step", "avg_duration_us": dur * 1e6 if dur else None,
       "sq_insts_valu_per_launch": valu, "sq_insts_lds_per_launch": med.get("SQ_INSTS_LDS"),
       "sq_waves_per_launch": med.get("SQ_WAVES"), "clock_hz": CLOCK, "blocks": blocks}
if valu and dur:
    cap = dur * CLOCK / 4
    out["issue_frac_chip"] = valu / (cap * CUS * SIMDS)
    out["issue_frac_busy_cus"] = valu / (cap * min(blocks, CUS) * SIMDS)
dst = os.path.join(root, "profiles", tag)
os.makedirs(dst, exist_ok=True)
with open(os.path.join(dst, "valu_issue.json"), "w") as f:
    json.dump(out, f, indent=1)
print(json.dumps(out, indent=1))
