#!/usr/bin/env python3
"""Issue cost of each VALU instruction class in SIMD-cycles, from a rocprofv3
pass over tools/valu_rate (GRBM_GUI_ACTIVE + SQ_INSTS_VALU per form kernel):
cycles per wave-instruction per SIMD = SIMDs x (GRBM_GUI_ACTIVE / 8 XCDs) /
SQ_INSTS_VALU, the same normalisation tools/pmc_traffic.py applies to k_icp.
Each form kernel keeps 8 independent chains of one form in each of 4 waves
per SIMD, so its rate is that form's issue cost.  The SQ_INSTS_VALU_* type
counters of the same pass say which class each form is counted under
(cmp / cndmask / floor / mov / and / div_scale: no class = "other").

usage: tools/valu_costs.py <prof_valu root> <out.json>"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import summarize  # noqa: E402

SIMDS = 1024
# class -> the microbenchmark forms that represent it (distinct operands,
# as the compiler allocates them in the pixel loop)
CLASSES = {
    "ADD_F32": ["k_add"], "MUL_F32": ["k_mul2", "k_mul"], "FMA_F32": ["k_fmac3", "k_fma3"],
    "TRANS_F32": ["k_rcp"], "FMA_F64": ["k_fmac64d", "k_fma64"], "ADD_F64": ["k_add64"],
    "MUL_F64": ["k_fma64"], "CVT": ["k_cvt64d", "k_cvtif2", "k_cvtfi"],
    "INT32": ["k_addu", "k_mu24"], "INT64": ["k_u64"],
    "other": ["k_cmp64", "k_cnd64d", "k_floor2"], "other_2cycle": ["k_mov", "k_andb"],
}


def main():
    r = summarize(sys.argv[1])
    per_form = {}
    for k, v in r.items():
        if "GRBM_GUI_ACTIVE" in v and v.get("SQ_INSTS_VALU", 0) > 0 and k.startswith("k_"):
            per_form[k] = SIMDS * v["GRBM_GUI_ACTIVE"] / 8 / v["SQ_INSTS_VALU"]
    costs = {}
    for cls, forms in CLASSES.items():
        vals = [per_form[f] for f in forms if f in per_form]
        costs[cls] = {"cycles": sum(vals) / len(vals), "min": min(vals), "max": max(vals),
                      "forms": forms}
    json.dump({"simd_cycles_per_wave_instruction": costs, "per_form": per_form,
               "source": sys.argv[1]}, open(sys.argv[2], "w"), indent=1)
    for cls, c in costs.items():
        print(f"{cls:14s} {c['cycles']:6.3f}  ({c['min']:.3f}-{c['max']:.3f})")


if __name__ == "__main__":
    main()
