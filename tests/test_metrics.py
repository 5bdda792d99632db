"""hdgnn.metrics reproduces the reference's EvaluationFuncs numbers (quirks included) on
the committed golden inputs (tools/gen_metric_golden.py ran the reference here)."""
import json
import os

import numpy as np
import pytest

from hdgnn import metrics


def _golden(golden_dir):
    z = np.load(os.path.join(golden_dir, "metrics_tiny.npz"))
    with open(os.path.join(golden_dir, "metrics_tiny.json")) as f:
        return z, json.load(f)["values"]


@pytest.mark.parametrize("name", ["top_ACC", "prec", "recall", "f1", "AUC"])
def test_metric_matches_reference(golden_dir, name):
    z, vals = _golden(golden_dir)
    got = getattr(metrics, name)(z["label"].copy(), z["probs"].copy())
    np.testing.assert_allclose(got, vals[name], rtol=1e-12, atol=0)


def test_top_acc_count_is_additive_over_shards(golden_dir):
    z, vals = _golden(golden_dir)
    lab, pr = z["label"], z["probs"]
    c = metrics.top_acc_count(lab[:2], pr[:2]) + metrics.top_acc_count(lab[2:], pr[2:])
    assert c / (lab.shape[0] * lab.shape[2]) == pytest.approx(vals["top_ACC"], abs=0)
