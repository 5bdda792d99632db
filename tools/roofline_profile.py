"""Summarise a tools/profile_config.sh run into profiles/<round>/<tag>/roofline.json (the
file bench.py's roofline reads for the same workload) and a readable summary.txt.

    python tools/roofline_profile.py gpurun_out/r04/glide profiles/r04/glide [bench args]
    python tools/roofline_profile.py --cal gpurun_out/r04/cal profiles/r04/calibration.json

Per kernel (names as the live per-kernel events report them, template arguments dropped):
  avg_us            rocprofv3 --kernel-trace --stats average (HIP-graph replay, as bench runs)
  fetch_kib/write_kib  FETCH_SIZE / WRITE_SIZE medians per launch (separate --pmc passes)
  hbm_bytes_lower/upper  F*min / F*max of the calibrated read factors + W*write factor
  hbm_bytes         the estimate bench.py reports (see traffic_note)
  valu_wave_insts, lds/salu insts, waves, wait_any_frac   SQ pass
  executed_flops    64 SQ_INSTS_VALU_FLOPS_FP32 + 512 SQ_INSTS_VALU_MFMA_MOPS_F32 (calibrated
                    on tools/probe/flops_cal.hip: every lane counted, MFMA padding included)
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLOCK = 2.4e9


def base(name):
    n = re.sub(r"^void ", "", name)
    n = re.sub(r"\(anonymous namespace\)::", "", n)
    n = re.sub(r"hdg::", "", n)
    n = n.split("(")[0]
    return n.split("<")[0].strip()


def pmc(d):
    vals = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            vals[base(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: {c: sorted(v)[len(v) // 2] for c, v in dd.items()} for k, dd in vals.items()}


def stats(d):
    out = {}
    for f in glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = base(r["Name"])
            if k in out:       # several instantiations of one kernel: keep the longest
                if float(r["TotalDurationNs"]) <= out[k]["total_us"] * 1e3:
                    continue
            out[k] = {"calls": int(r["Calls"]), "avg_us": float(r["AverageNs"]) / 1e3,
                      "total_us": float(r["TotalDurationNs"]) / 1e3}
    return out


def calibration(src, dst):
    """fetch_cal: every kernel moves 64 MiB (strided ones: 64 MiB of whole lines)."""
    nbytes = 64 << 20
    f, w = pmc(os.path.join(src, "fetch")), pmc(os.path.join(src, "write"))
    cal = {"bytes_per_kernel": nbytes, "read": {}, "write": {},
           "note": "factor = known bytes / (counter KiB * 1024): multiply a counter by the "
                   "factor of the access pattern to get bytes"}
    for k, v in sorted(f.items()):
        if k.startswith("rd_") and v.get("FETCH_SIZE"):
            useful = nbytes // {"rd_x1_s64": 16, "rd_x1_s128": 32}.get(k, 1)
            cal["read"][k] = {"fetch_kib": v["FETCH_SIZE"],
                              "factor_line_bytes": nbytes / (v["FETCH_SIZE"] * 1024),
                              "factor_useful_bytes": useful / (v["FETCH_SIZE"] * 1024)}
    for k, v in sorted(w.items()):
        if k.startswith("wr_") and v.get("WRITE_SIZE"):
            useful = nbytes // {"wr_x1_s64": 16}.get(k, 1)
            cal["write"][k] = {"write_kib": v["WRITE_SIZE"],
                               "factor_line_bytes": nbytes / (v["WRITE_SIZE"] * 1024),
                               "factor_useful_bytes": useful / (v["WRITE_SIZE"] * 1024)}
    fl = pmc(os.path.join(src, "flops"))
    cal["flops_counters"] = {k: v for k, v in sorted(fl.items()) if k.startswith("cal_")}
    with open(dst, "w") as fh:
        json.dump(cal, fh, indent=1)
    print(json.dumps(cal, indent=1))


def parse_args(argv):
    cfg = {"variant": 2, "ne": 200, "nc": 74, "batch": 100, "path": None, "hunk": "auto"}
    it = iter(argv)
    for a in it:
        if a in ("--variant", "--ne", "--nc", "--batch"):
            cfg[a[2:]] = int(next(it))
        elif a == "--hunk":
            cfg["hunk"] = next(it)
        elif a == "--path":
            cfg["path"] = {"0": None, "1": "fused", "2": "general"}[next(it)]
    return cfg


def bench_line(d):
    for f in ("bench_trace.log",):
        p = os.path.join(d, f)
        if os.path.exists(p):
            for ln in open(p):
                if ln.startswith("{"):
                    return json.loads(ln)
    return None


def main(src, dst, argv):
    cfg = parse_args(argv or open(os.path.join(src, "args.txt")).read().split())
    line = bench_line(src)
    if line:                                        # the path AUTO resolved to
        cfg["path"] = line["config"]["engine_path"].split()[0]
    calf = os.path.join(os.path.dirname(dst), "calibration.json")
    cal = json.load(open(calf)) if os.path.exists(calf) else None
    if cal:
        rf = [v["factor_line_bytes"] for v in cal["read"].values()]
        wf = cal["write"].get("wr_x1", {}).get("factor_line_bytes", 1.0)
        rlo, rhi = min(rf), max(rf)
        rmid = cal["read"].get("rd_x1", {}).get("factor_line_bytes", rhi)
        note = ("2 x FETCH_SIZE + WRITE_SIZE: FETCH_SIZE x %.4g..%.4g over every read "
                "pattern calibrated (dword / dwordx2 / dwordx4, device and system scope, one "
                "dword per 64 B or 128 B line: tools/probe/fetch_cal.hip, %s) -- the x2 is the "
                "128 B line count, independent of access width, so the figure is the lines "
                "moved, not an upper bound; WRITE_SIZE x %.3g (dword and dwordx4 stores; "
                "partial-line stores count 32 B granules)" % (rlo, rhi, os.path.relpath(calf, ROOT), wf))
    else:
        rlo, rhi, rmid, wf = 1.0, 2.0, 2.0, 1.0
        note = ("no calibration: FETCH_SIZE x1..x2 (MI355X_MICROARCH.md: x2 for 16 B/lane "
                "streaming reads), the estimate is the upper bound")
    tr, fe, wr = stats(os.path.join(src, "trace")), pmc(os.path.join(src, "fetch")), \
        pmc(os.path.join(src, "write"))
    sq, fl = pmc(os.path.join(src, "sq")), pmc(os.path.join(src, "flops"))
    ld = pmc(os.path.join(src, "lds"))
    kernels = {}
    for k in sorted(set(tr) | set(fe) | set(sq)):
        if k.startswith("__amd") or "at::native" in k or k.startswith("at::"):
            continue
        e = dict(tr.get(k, {}))
        F, W = fe.get(k, {}).get("FETCH_SIZE"), wr.get(k, {}).get("WRITE_SIZE")
        if F is not None and W is not None:
            e["fetch_kib"], e["write_kib"] = F, W
            e["hbm_bytes_lower"] = round((F * rlo + W * wf) * 1024)
            e["hbm_bytes_upper"] = round((F * rhi + W * wf) * 1024)
            e["hbm_bytes"] = round((F * rmid + W * wf) * 1024)
        s = sq.get(k, {})
        if s:
            e["valu_wave_insts"] = s.get("SQ_INSTS_VALU")
            e["lds_wave_insts"] = s.get("SQ_INSTS_LDS")
            e["salu_wave_insts"] = s.get("SQ_INSTS_SALU")
            e["waves"] = s.get("SQ_WAVES")
            if s.get("SQ_WAVE_CYCLES"):
                e["wait_any_frac"] = round(s.get("SQ_WAIT_ANY", 0) / s["SQ_WAVE_CYCLES"], 4)
                e["active_inst_frac"] = round(s.get("SQ_ACTIVE_INST_ANY", 0) / s["SQ_WAVE_CYCLES"], 4)
        lq = ld.get(k, {})
        if lq.get("SQ_LDS_IDX_ACTIVE"):
            e["lds_bank_conflict_frac"] = round(lq.get("SQ_LDS_BANK_CONFLICT", 0)
                                                / lq["SQ_LDS_IDX_ACTIVE"], 4)
            e["vmem_rd_wave_insts"] = lq.get("SQ_INSTS_VMEM_RD")
        f = fl.get(k, {})
        if f:
            e["executed_flops"] = (64 * f.get("SQ_INSTS_VALU_FLOPS_FP32", 0)
                                   + 512 * f.get("SQ_INSTS_VALU_MFMA_MOPS_F32", 0))
            e["mfma_flops"] = 512 * f.get("SQ_INSTS_VALU_MFMA_MOPS_F32", 0)
        if e.get("avg_us") and e.get("valu_wave_insts"):
            t = e["avg_us"] * 1e-6
            e["issue_frac_chip"] = round(e["valu_wave_insts"] / (t * CLOCK / 4 * 256 * 4), 4)
            if e.get("executed_flops"):
                e["tflops"] = round(e["executed_flops"] / t / 1e12, 3)
            if e.get("hbm_bytes"):
                e["hbm_tbs"] = round(e["hbm_bytes"] / t / 1e12, 4)
        kernels[k] = e
    out = {"config": cfg, "args": argv or None, "kernels": kernels, "traffic_note": note,
           "bench_line": {k: line.get(k) for k in ("value", "ms_per_step", "kernels_ms")}
           if line else None,
           "source": "tools/profile_config.sh -> %s" % os.path.relpath(src, ROOT)}
    os.makedirs(dst, exist_ok=True)
    for f in glob.glob(os.path.join(src, "trace", "**", "*kernel_stats.csv"), recursive=True):
        with open(f) as a, open(os.path.join(dst, "kernel_stats.csv"), "w") as b:
            b.write(a.read())
    with open(os.path.join(dst, "pmc_medians.json"), "w") as fh:
        json.dump({"fetch": fe, "write": wr, "sq": sq, "flops": fl, "lds": ld}, fh, indent=1,
                  sort_keys=True)
    with open(os.path.join(dst, "roofline.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    rows = ["# %s  config %s" % (os.path.relpath(dst, ROOT), json.dumps(cfg)),
            "# avg_us: rocprofv3 kernel-trace (graph replay); HBM MB per launch: " + note,
            "# issue: VALU wave-instructions / chip issue slots; wait: SQ_WAIT_ANY / wave cycles; "
            "ldsc: SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE",
            "%-16s %6s %9s %9s %9s %9s %8s %8s %8s %7s %6s" % (
                "kernel", "calls", "avg_us", "hbm_MB", "lo_MB", "hi_MB", "TB/s", "TFLOP/s",
                "issue", "wait", "ldsc")]
    tot = sum(e.get("total_us", 0) for e in kernels.values())
    for k, e in sorted(kernels.items(), key=lambda kv: -kv[1].get("total_us", 0)):
        rows.append("%-16s %6s %9.2f %9.2f %9.2f %9.2f %8.3f %8.2f %8.3f %7.3f %6.3f" % (
            k[:16], e.get("calls", "-"), e.get("avg_us", 0), e.get("hbm_bytes", 0) / 1e6,
            e.get("hbm_bytes_lower", 0) / 1e6, e.get("hbm_bytes_upper", 0) / 1e6,
            e.get("hbm_tbs", 0), e.get("tflops", 0), e.get("issue_frac_chip", 0),
            e.get("wait_any_frac", 0), e.get("lds_bank_conflict_frac", 0)))
    rows.append("# total kernel time in the trace %.1f us" % tot)
    if line:
        rows.append("# bench line: %s commits/s, %s ms/step" % (line["value"], line["ms_per_step"]))
    txt = "\n".join(rows) + "\n"
    with open(os.path.join(dst, "summary.txt"), "w") as fh:
        fh.write(txt)
    print(txt)


if __name__ == "__main__":
    if sys.argv[1] == "--cal":
        calibration(sys.argv[2], sys.argv[3])
    else:
        main(sys.argv[1], sys.argv[2], sys.argv[3:])
