"""Achieved-error log of the parity tests (test infrastructure).

The parity helpers call record() with the largest error they saw next to the tolerance
they enforced; with HDG_PARITY_REPORT=<path> set, conftest writes every record of the
session there as JSON (tools/gpu_full.sh copies it to profiles/, DESIGN §6 quotes it).
"""
import os

RECORDS = []


def record(quantity, err_over_scale, err_over_tol, **extra):
    """quantity: "logits", "grad:<var>", "weights@50", ...;  err_over_scale: max error
    relative to the quantity's scale (per-commit max|logit|, per-variable max|ref|);
    err_over_tol: max error / enforced tolerance (<= 1 passes)."""
    test = os.environ.get("PYTEST_CURRENT_TEST", "?").split(" ")[0]
    row = {"test": test, "quantity": quantity, "err_over_scale": float(err_over_scale),
           "err_over_tol": float(err_over_tol)}
    row.update(extra)
    RECORDS.append(row)
