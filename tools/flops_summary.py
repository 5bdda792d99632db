"""Executed FP32 FLOPs per kernel launch from the PMC pass of tools/pmc_flops.sh.

Calibration (tools/probe/flops_cal.hip, 1024 waves x 1000 instructions per kernel, same
pass): SQ_INSTS_VALU_FLOPS_FP32 counts per wave-instruction 1 for v_add / v_mul / v_exp
(transcendentals included), 2 for v_fma and v_pk_add, 4 for v_pk_fma, 0 for v_max;
SQ_INSTS_VALU_MFMA_MOPS_F32 counts 4 per v_mfma_f32_16x16x4_f32 (= its 2048 flops / 512).
So executed FLOPs = 64 x SQ_INSTS_VALU_FLOPS_FP32 + 512 x SQ_INSTS_VALU_MFMA_MOPS_F32
(every lane counted: an upper bound for exec-masked instructions; MFMA zero padding
counted as executed).
    python tools/flops_summary.py gpurun_out/pmc_flops profiles/r02/flops_pmc.json
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_table import table  # noqa: E402


def executed(med):
    return (64 * med.get("SQ_INSTS_VALU_FLOPS_FP32", 0)
            + 512 * med.get("SQ_INSTS_VALU_MFMA_MOPS_F32", 0))


def main(src, dst, ne=200, nc=74, batch=100):
    cal = table(os.path.join(src, "cal"))
    bench = table(os.path.join(src, "bench"))
    out = {"calibration": {k: {"counters": v, "executed_flops": executed(v)}
                           for k, v in sorted(cal.items())},
           "kernels": {k: {"counters": v, "executed_flops_per_launch": executed(v)}
                       for k, v in sorted(bench.items())},
           "config": {"ne": ne, "nc": nc, "batch": batch},
           "formula": "64 * SQ_INSTS_VALU_FLOPS_FP32 + 512 * SQ_INSTS_VALU_MFMA_MOPS_F32",
           "source": "rocprofv3 --pmc (tools/pmc_flops.sh), median over dispatches"}
    with open(dst, "w") as f:
        json.dump(out, f, indent=1)
    for k, v in out["kernels"].items():
        print("%-40s %14.0f executed FLOP / launch" % (k, v["executed_flops_per_launch"]))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
