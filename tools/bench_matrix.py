"""Summarise a tools/bench_matrix.sh run: one row per workload with the bench line's value,
ms/step, dominant kernel and its roofline (from the committed profile of that workload).
    python tools/bench_matrix.py gpurun_out/matrix profiles/r04/bench_matrix
writes <dst>.json (the bench lines, whole) and <dst>.txt (the table)."""
import glob
import json
import os
import sys


def main(src, dst):
    lines = {}
    for f in sorted(glob.glob(os.path.join(src, "*.log"))):
        for ln in open(f):
            if ln.startswith("{"):
                lines[os.path.basename(f)[:-4]] = json.loads(ln)
    with open(dst + ".json", "w") as fh:
        json.dump(lines, fh, indent=1)
    rows = ["%-18s %12s %9s %12s %9s %-16s %9s %8s %8s %9s %s" % (
        "workload", "commits/s", "ms/step", "steady/s", "steady_ms", "dominant", "kern_us",
        "frac", "issue", "hbm_MB", "profile")]
    for tag, d in lines.items():
        r = d.get("roofline") or {}
        ex = r.get("executed") or {}
        st = d.get("steady_state") or {}
        rows.append("%-18s %12.1f %9.4f %12s %9s %-16s %9.2f %8s %8s %9s %s" % (
            tag, d["value"], d["ms_per_step"], st.get("value"), st.get("ms_per_step"),
            (r.get("kernel") or "-")[:16],
            (r.get("avg_launch_ms") or 0) * 1e3, r.get("frac"), ex.get("issue_frac_chip"),
            "%.2f" % (r["traffic"] / 1e6) if r.get("traffic") else None, r.get("profile")))
    txt = "\n".join(rows) + "\n"
    with open(dst + ".txt", "w") as fh:
        fh.write(txt)
    print(txt)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
