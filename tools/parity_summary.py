"""Condense a parity report (tests/_errlog.py, HDG_PARITY_REPORT=...) into the worst case
per test file and quantity: max error / scale and max error / enforced tolerance, with the
test that produced it.  Writes <dst>.json and prints the table DESIGN.md 6 quotes.
    python tools/parity_summary.py gpurun_out/parity_report.json profiles/r03/parity_summary
"""
import collections
import json
import sys


def main(src, dst):
    rows = json.load(open(src))
    worst = collections.OrderedDict()
    for r in rows:
        f = r["test"].split("::")[0].split("/")[-1]
        q = r["quantity"]
        q = q.split(":")[0] + ":*" if ":" in q else q    # per-variable records: one row
        k = (f, q)
        w = worst.get(k)
        if w is None:
            w = worst[k] = {"file": f, "quantity": q, "n": 0, "err_over_scale": 0.0,
                            "err_over_tol": 0.0, "worst_test": None}
        w["n"] += 1
        if r["err_over_scale"] >= w["err_over_scale"]:
            w["err_over_scale"] = r["err_over_scale"]
            w["worst_test"] = r["test"].split("::")[-1] + " " + r["quantity"]
        w["err_over_tol"] = max(w["err_over_tol"], r["err_over_tol"])
    out = list(worst.values())
    with open(dst + ".json", "w") as fh:
        json.dump(out, fh, indent=1)
    for w in out:
        print("%-26s %-22s n=%-4d err/scale %.2e  err/tol %.3f  (%s)" % (
            w["file"], w["quantity"], w["n"], w["err_over_scale"], w["err_over_tol"],
            w["worst_test"]))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
