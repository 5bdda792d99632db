"""Summarise tools/lds_phases.sh: per HDG_STOP_AFTER build, k_commit_step's counters and
trace duration, and the per-phase differences (phase n = build n minus build n-1).
    python tools/lds_phases_sum.py gpurun_out/lds [out.txt]"""
import glob
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from roofline_profile import pmc, stats  # noqa: E402

d = sys.argv[1]
K = "k_commit_step"
rows = {}
for p in glob.glob(os.path.join(d, "pmc_*")):
    if not os.path.isdir(p):
        continue
    tag = os.path.basename(p)[4:]
    c = pmc(p).get(K)
    s = stats(os.path.join(d, "tr_" + tag)).get(K)
    if c and s:
        rows[tag] = (c, s["avg_us"])
order = sorted((t for t in rows if t != "full"), key=int) + (["full"] if "full" in rows else [])
cols = ["SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE", "SQ_INSTS_LDS", "SQ_INSTS_VALU", "SQ_INSTS_SALU",
        "SQ_WAIT_ANY", "SQ_WAVE_CYCLES"]
out = ["# k_commit_step per HDG_STOP_AFTER build (cumulative to the phase boundary), then "
       "per-phase differences; counters are per-launch totals (medians over launches)",
       "%-5s %8s %10s %10s %10s %11s %10s %10s %8s" % ("stop", "us", "ldsconf", "ldsactive",
                                                     "insts_lds", "insts_valu", "salu",
                                                     "wait_any", "conf/act")]
prev = None
for t in order:
    c, us = rows[t]
    v = [c.get(k, 0.0) for k in cols]
    out.append("%-5s %8.2f %10.0f %10.0f %10.0f %11.0f %10.0f %10.0f %8.3f" % (
        t, us, v[0], v[1], v[2], v[3], v[4], v[5], v[0] / max(v[1], 1)))
out.append("# per phase (build n - build n-1)")
for t in order:
    c, us = rows[t]
    v = [c.get(k, 0.0) for k in cols]
    if prev is not None:
        dv = [a - b for a, b in zip(v, prev[1])]
        out.append("%-5s %8.2f %10.0f %10.0f %10.0f %11.0f %10.0f %10.0f %8.3f" % (
            "%s-%s" % (prev[0], t), us - prev[2], dv[0], dv[1], dv[2], dv[3], dv[4], dv[5],
            dv[0] / dv[1] if dv[1] > 0 else 0.0))
    prev = (t, v, us)
txt = "\n".join(out)
print(txt)
if len(sys.argv) > 2:
    open(sys.argv[2], "w").write(txt + "\n")
