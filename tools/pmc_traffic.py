#!/usr/bin/env python3
"""Per-launch HBM traffic of k_reduce from rocprofv3 PMC passes -> JSON.

traffic = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 bytes, averaged over the
k_reduce dispatches.  The factor 2 on FETCH_SIZE is MI355X_MICROARCH.md §HBM's
gfx950 correction, re-calibrated here: tools/kbench's k_stream_read of a known
550.5 MB reports FETCH_SIZE = 275.3 MB for both dwordx4 and dword loads
(profiles/r01/pmc_calibration.txt).

VALU issue: when the SQ pass holds SQ_INSTS_VALU and GRBM_GUI_ACTIVE, also
  effective clock = GRBM_GUI_ACTIVE / n_XCD / kernel duration (MI355X_MICROARCH.md
                    "DVFS give-back": rocprofv3 sums GRBM over the 8 XCDs),
  VALU cycles per instruction = SIMDs x (GRBM_GUI_ACTIVE / n_XCD) / SQ_INSTS_VALU,
i.e. how many SIMD cycles the kernel spends per issued VALU wave-instruction;
compare with the per-form issue costs of tools/valu_rate (about 2.4 cycles
for 2-operand fp32/int ops, 4 for fp64 FMA, converts, compares, selects and
packed ops): a value near the mix's cost means the kernel is issue-bound.
SIMD count from the pass's agent_info.csv.

usage: tools/pmc_traffic.py <profile_root> <out.json> <pairs> <width> <height> [iters]
(iters: ICP iterations each k_icp launch covers; 1 for per-iteration k_reduce)
"""
import csv
import glob
import hashlib
import json
import os
import sys

N_XCD = 8

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import summarize  # noqa: E402


def valu_account(r, simds, costs_path, root_dir):
    """VALU issue account of one kernel's PMC row: instruction
    classes from the SQ_INSTS_VALU_* counters x their measured issue cost in
    SIMD-cycles (tools/valu_costs.py over tools/valu_rate, the same GRBM
    normalisation), against the SIMD-cycles of the launch.  "other" =
    SQ_INSTS_VALU minus the classified ones (v_cmp, v_cndmask, v_mov,
    permlane / readlane / DPP); its cost is bracketed by the 4.3-cycle
    compare/select forms and the 2.4-cycle moves.  None without the counters."""
    cls = ["ADD_F32", "MUL_F32", "FMA_F32", "TRANS_F32", "FMA_F64", "ADD_F64", "MUL_F64", "CVT",
           "INT32", "INT64"]
    if not (os.path.exists(costs_path) and all(f"SQ_INSTS_VALU_{c}" in r for c in cls) and
            "GRBM_GUI_ACTIVE" in r and "SQ_INSTS_VALU" in r):
        return None
    cost = json.load(open(costs_path))["simd_cycles_per_wave_instruction"]
    avail = simds * r["GRBM_GUI_ACTIVE"] / N_XCD
    counts = {c: r[f"SQ_INSTS_VALU_{c}"] for c in cls}
    counts["other"] = max(0.0, r["SQ_INSTS_VALU"] - sum(counts.values()))
    cyc = {c: counts[c] * cost[c]["cycles"] for c in counts}
    lo = sum(cyc.values()) - cyc["other"] + counts["other"] * cost["other_2cycle"]["cycles"]
    return {
        "simd_cycles_available": avail,
        "instructions_by_class": counts,
        "issue_cycles_by_class": cyc,
        "issue_cycles": sum(cyc.values()),
        "busy_frac": sum(cyc.values()) / avail,
        "busy_frac_other_at_2_4_cycles": lo / avail,
        "cost_source": os.path.relpath(costs_path, root_dir),
    }


def main():
    root, out, pairs, W, H = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), \
        int(sys.argv[5])
    iters = int(sys.argv[6]) if len(sys.argv) > 6 else 1
    res = summarize(root)
    key = next(k for k in res if k.startswith("k_icp") or k.startswith("k_reduce"))
    r = res[key]
    fetch = r["FETCH_SIZE"] * 1024.0
    write = r.get("WRITE_SIZE", 0.0) * 1024.0
    px = pairs * W * H
    doc = {
        "kernel": key, "pairs": pairs, "width": W, "height": H,
        "fetch_size_bytes": fetch, "write_size_bytes": write,
        "iterations_per_launch": iters,
        "hbm_bytes_per_launch": 2.0 * fetch + write,
        "hbm_bytes_per_iteration": (2.0 * fetch + write) / iters,
        "bytes_per_px": (2.0 * fetch + write) / iters / px,
        "correction": "2 x FETCH_SIZE (gfx950 tallies 128-B requests as 64 B)",
        # bench.py uses these figures only for the kernel source they were taken on
        "kernel_sha16": hashlib.sha256(open(os.path.join(
            os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "slam-rgbd_amd", "csrc",
            "icp_kernels.hip"), "rb").read()).hexdigest()[:16],
        "profile_root": root,
    }
    if "SQ_INSTS_VALU" in r and "GRBM_GUI_ACTIVE" in r:
        simds = 1024
        for f in glob.glob(os.path.join(root, "**", "*agent_info.csv"), recursive=True):
            for a in csv.DictReader(open(f)):
                if a.get("Name", "").startswith("gfx") and a.get("Simd_Count"):
                    simds = int(a["Simd_Count"])
        cyc = r["GRBM_GUI_ACTIVE"] / N_XCD
        doc["valu_wave_instructions_per_launch"] = r["SQ_INSTS_VALU"]
        doc["valu_lane_ops_per_px_iteration"] = r["SQ_INSTS_VALU"] * 64 / (px * iters)
        doc["valu_cycles_per_instruction"] = simds * cyc / r["SQ_INSTS_VALU"]
        doc["gpu_cycles_per_launch"] = cyc
        doc["simds"] = simds
        if "SQ_ACTIVE_INST_VALU" in r:
            # rocprof's derived VALUBusy: 4 x SQ_ACTIVE_INST_VALU (quad-cycles) /
            # SIMDs / GRBM_GUI_ACTIVE (per XCD); ~1 = a VALU instruction in
            # execution on every SIMD in every cycle of the kernel
            # rocprof's derived VALUBusy (4 x SQ_ACTIVE_INST_VALU / SIMDs /
            # cycles): SQ_ACTIVE_INST_VALU counts, per wave, the quad-cycles
            # its VALU instruction is in execution, and the 4 waves of a SIMD
            # overlap there, so it can exceed 1; not an issue fraction
            doc["rocprof_valubusy"] = 4.0 * r["SQ_ACTIVE_INST_VALU"] / simds / cyc
        durs = []
        for f in glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True):
            if "pmc_sq" not in f:
                continue
            for row in csv.DictReader(open(f)):
                if key in row.get("Kernel_Name", ""):
                    durs.append(int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
        if durs:
            avg_ns = sum(durs) / len(durs)
            doc["effective_clock_ghz"] = cyc / avg_ns
    root_dir = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    costs_path = os.path.join(root_dir, "profiles", "r03", "valu_costs.json")
    acc = valu_account(r, doc.get("simds", 1024), costs_path, root_dir)
    if acc:
        doc["valu_account"] = acc
        doc["valu_busy_frac"] = acc["busy_frac"]
        doc["valu_busy_definition"] = ("sum over VALU classes of SQ_INSTS_VALU_<class> x its "
                                       "measured issue cost (SIMD-cycles, tools/valu_rate) / "
                                       "(SIMDs x GRBM_GUI_ACTIVE / 8 XCDs)")
    if all(k in r for k in ("SQ_WAVE_CYCLES", "SQ_WAIT_INST_ANY")) and "SQ_ACTIVE_INST_ANY" in r:
        w = r["SQ_WAVE_CYCLES"]
        doc["wave_state_frac"] = {"active": r["SQ_ACTIVE_INST_ANY"] / w,
                                  "issue_stalled": r["SQ_WAIT_INST_ANY"] / w,
                                  "parked": r.get("SQ_WAIT_ANY", float("nan")) / w}
    for k in ("k_prep", "k_solve"):
        m = next((x for x in res if x.startswith(k)), None)
        if m and "FETCH_SIZE" in res[m]:
            doc[k + "_hbm_bytes"] = 2.0 * res[m]["FETCH_SIZE"] * 1024 + \
                res[m].get("WRITE_SIZE", 0.0) * 1024
    # k_prep (one target frame per pair): bytes per target pixel and its VALU issue
    m = next((x for x in res if x.startswith("k_prep")), None)
    if m:
        if "k_prep_hbm_bytes" in doc:
            doc["k_prep_bytes_per_px"] = doc["k_prep_hbm_bytes"] / (pairs * W * H)
        pacc = valu_account(res[m], doc.get("simds", 1024), costs_path, root_dir)
        if pacc:
            doc["k_prep_valu_account"] = pacc
            doc["k_prep_valu_busy_frac"] = pacc["busy_frac"]
    json.dump(doc, open(out, "w"), indent=1)
    print(json.dumps(doc, indent=1))


if __name__ == "__main__":
    main()
