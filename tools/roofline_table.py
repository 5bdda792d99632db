"""One row per workload profile under profiles/<round>/*/roofline.json: the bench line under
the kernel trace, the dominant kernel (longest total time per step) and its roofline terms.
    python tools/roofline_table.py profiles/r04 > profiles/r04/roofline_table.txt"""
import glob
import json
import os
import sys

ORDER = ["glide", "m2_general_glide", "m1_glide", "m3_glide", "m4_glide", "m4_general_glide",
         "s3", "s5", "m4_s5", "m4_general_s5", "stress", "m4_stress"]


def main(d):
    found = {os.path.basename(os.path.dirname(f)): f
             for f in glob.glob(os.path.join(d, "*", "roofline.json"))}
    tags = [t for t in ORDER if t in found] + sorted(t for t in found if t not in ORDER)
    print("%-17s %-24s %10s %9s %-15s %8s %8s %6s %8s %7s %6s" % (
        "workload", "config", "commits/s", "ms/step", "dominant", "avg_us", "TFLOP/s", "issue",
        "HBM_MB", "TB/s", "ldsc"))
    for t in tags:
        pj = json.load(open(found[t]))
        ks = {k: v for k, v in pj["kernels"].items() if v.get("calls", 0) >= 20}
        dom = max(ks, key=lambda k: ks[k]["total_us"])
        e = ks[dom]
        c = pj["config"]
        cfg = "v%d %s %dx%d B%d%s" % (c["variant"], (c["path"] or "auto")[:3], c["ne"], c["nc"],
                                      c["batch"], "" if c.get("hunk", "auto") == "auto"
                                      else " " + c["hunk"])
        bl = pj.get("bench_line") or {}
        print("%-17s %-24s %10.0f %9.4f %-15s %8.2f %8.2f %6.3f %8.2f %7.3f %6.3f" % (
            t, cfg, bl.get("value") or 0, bl.get("ms_per_step") or 0, dom[:15], e["avg_us"],
            e.get("tflops", 0), e.get("issue_frac_chip", 0), e.get("hbm_bytes", 0) / 1e6,
            e.get("hbm_tbs", 0), e.get("lds_bank_conflict_frac", 0)))
    print("# bench line under the kernel trace (rocprofv3 adds overhead: the bench matrix has "
          "the unprofiled numbers); TFLOP/s = executed FP32 (calibrated PMC) / trace avg; issue = "
          "VALU wave-instructions / chip issue slots; HBM = 2 FETCH_SIZE + WRITE_SIZE "
          "(calibrated); ldsc = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE")


if __name__ == "__main__":
    main(sys.argv[1])
