"""Per-kernel hardware-counter table from the passes of scripts/prof.sh pmc (a-d; e adds the
instruction-issue table).

    python scripts/pmc_table.py gpurun_out/TAG_CONFIG [--batch 8192] > profiles/<tag>/pmc_table.md
    (passes written by: scripts/prof.sh pmc TAG CONFIG)

Columns: mean duration (counter runs, kernel-trace timestamps), VGPR/AGPR/LDS per workgroup,
waves per SIMD the resources allow, MFMA-busy share of the kernel's SIMD-cycles, LDS bank-conflict
share of LDS-active cycles, LDS-active share of the kernel's CU-cycles, wave cycles spent parked
(s_waitcnt / barrier), achieved TFLOP/s (analytic FLOP per image, survey §2.6), and HBM-side
GB/s from FETCH_SIZE (x2: gfx950 tallies 128-B requests at 64 B, MI355X_MICROARCH.md §HBM) and
WRITE_SIZE.  Counter values are summed over the dispatch's instances and averaged over dispatches.
"""
from __future__ import annotations

import argparse
import collections
import csv
import os

N_CU, SIMD, N_XCD = 256, 4, 8
# GRBM_GUI_ACTIVE comes back summed over the 8 XCDs (x8 the kernel's cycles: 1.544e6 for a 78 us
# conv_bwd at ~2.4 GHz); SQ_VALU_MFMA_BUSY_CYCLES is summed over all 1024 SIMDs (it equals the
# kernel's MFMA count x 16 cycles of v_mfma_f32_16x16x32_bf16) and SQ_LDS_* over the 256 CUs.
# analytic FLOP per image of each LeNet-5 kernel (2 x MACs), batch 8192 in the bench
FLOP_PER_IMG = {
    "conv_fwd": 2 * (6 * 784 * 25 + 16 * 100 * 150),
    "head": 2 * 2 * (400 * 120 + 120 * 84 + 84 * 10),
    "wgrad": 2 * (400 * 120 + 120 * 84 + 84 * 10),
    "conv_bwd": 2 * (16 * 100 * 150 * 2 + 6 * 784 * 25),
    "head16": 2 * 2 * (400 * 120 + 120 * 84 + 84 * 10),
}
FLOP_PER_IMG["fwd_head"] = FLOP_PER_IMG["conv_fwd"] + FLOP_PER_IMG["head"]  # fused forward + FC head
FLOP_PER_IMG_MLP = {  # reference MLP: head = forward + dgrad of layers 3, 2 (no input grad); wgrad = all three layers
    "head": 2 * (784 * 128 + 128 * 128 + 128 * 10) + 2 * (10 * 128 + 128 * 128),
    "wgrad": 2 * (784 * 128 + 128 * 128 + 128 * 10),
}


def short(name: str) -> str:
    for k in ("fwd_head", "head16", "conv_fwd", "conv_bwd", "head_kernel", "wgrad", "reduce_sgd", "reduce_slabs", "sgd_pack"):
        if k in name:
            return k.replace("_kernel", "")
    return name[:24]


def load(path):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    meta, dur = {}, collections.defaultdict(dict)
    for r in csv.DictReader(open(path)):
        k = short(r["Kernel_Name"])
        if k.startswith("void at::") or "rocclr" in k:
            continue
        did = r["Dispatch_Id"]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(did)
        meta[k] = (int(r["VGPR_Count"]), int(r["Accum_VGPR_Count"]), int(r["LDS_Block_Size"]),
                   int(r["Workgroup_Size"]), int(r["Grid_Size"]))
        dur[k][did] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    out = {}
    for k in agg:
        n = len(disp[k])
        out[k] = ({c: v / n for c, v in agg[k].items()}, meta[k], sum(dur[k].values()) / len(dur[k]), n)
    return out


def waves_per_simd(vgpr, agpr, lds, wg):
    regs = -(-(vgpr + agpr) // 8) * 8
    by_reg = min(8, 512 // max(regs, 1))
    waves_per_wg = max(1, wg // 64)
    by_lds = (160 * 1024 // lds) * waves_per_wg / SIMD if lds else 8
    return min(by_reg, by_lds)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("prefix", help="e.g. gpurun_out/pmcf (expects _a.._d run dirs)")
    ap.add_argument("--batch", type=int, default=8192)
    ap.add_argument("--model", default="lenet5", choices=["lenet5", "mlp"])
    a = ap.parse_args()
    P = {s: load(os.path.join(f"{a.prefix}_{s}", "run_counter_collection.csv")) for s in "abcd"}
    pe = os.path.join(f"{a.prefix}_e", "run_counter_collection.csv")
    if os.path.exists(pe):
        P["e"] = load(pe)
    print("| kernel | calls | us | VGPR/AGPR | LDS B/WG | waves/SIMD (res.) | MFMA busy % | LDS bank-conflict % "
          "| LDS active % | WAIT_ANY % | TFLOP/s | HBM read GB/s | HBM write GB/s |")
    print("|---|---|---|---|---|---|---|---|---|---|---|---|---|")
    for k in sorted(P["b"], key=lambda x: -P["b"][x][2]):
        cb, (vg, ag, lds, wg, grid), t, n = P["b"][k]
        ca = P["a"].get(k, ({}, None, t, 0))[0]
        cc, _, tc, _ = P["c"].get(k, ({}, None, t, 0))
        cd, _, td, _ = P["d"].get(k, ({}, None, t, 0))
        cyc = cb.get("GRBM_GUI_ACTIVE", 0.0) / N_XCD
        mfma = 100.0 * cb.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / max(1.0, cyc * N_CU * SIMD) if cyc else float("nan")
        lds_act = 100.0 * cb.get("SQ_LDS_IDX_ACTIVE", 0.0) / max(1.0, cyc * N_CU) if cyc else float("nan")
        lds_c = 100.0 * cb.get("SQ_LDS_BANK_CONFLICT", 0.0) / max(1.0, cb.get("SQ_LDS_IDX_ACTIVE", 0.0))
        wait = 100.0 * ca.get("SQ_WAIT_ANY", 0.0) / max(1.0, ca.get("SQ_WAVE_CYCLES", 0.0))
        fl = (FLOP_PER_IMG_MLP if a.model == "mlp" else FLOP_PER_IMG).get(k)
        tf = fl * a.batch / t / 1e12 if fl else float("nan")
        rd = 2 * cc.get("FETCH_SIZE", 0.0) * 1024 / tc / 1e9 if tc else float("nan")
        wr = cd.get("WRITE_SIZE", 0.0) * 1024 / td / 1e9 if td else float("nan")
        occ = waves_per_simd(vg, ag, lds, wg)
        print(f"| {k} | {n} | {t * 1e6:.1f} | {vg}/{ag} | {lds} | {occ:g} | {mfma:.1f} | {lds_c:.1f} | {lds_act:.0f} | {wait:.0f} | "
              f"{tf:.1f} | {rd:.0f} | {wr:.0f} |")
    if "e" in P:
        issue_table(P)


def issue_table(P):
    """Instruction issue mix (pass e + a + b): instructions per wave by class and how full the issue
    slots were.  SQ_INSTS_VALU includes the MFMAs; a wave64 VALU instruction occupies its SIMD's vector
    issue for 2 cycles and a v_mfma_f32_16x16x32_bf16 for 8 of its 16 (MI355X_MICROARCH.md, 'vector-
    instruction ISSUE cost'); SQ_ACTIVE_INST_* and SQ_WAVE_CYCLES count quad-cycles."""
    print()
    print("| kernel | waves | VALU/wave | MFMA/wave | LDS/wave | SALU/wave | SMEM/wave | VMEM/wave | branch/wave "
          "| vector-issue busy % of SIMD cycles | MFMA pipe busy % | VALU-active % of wave time | LDS-active % of wave time "
          "| any-inst % of wave time |")
    print("|---|---|---|---|---|---|---|---|---|---|---|---|---|---|")
    for k in sorted(P["e"], key=lambda x: -P["e"][x][2]):
        ce, _, t, n = P["e"][k]
        ca = P["a"].get(k, ({},))[0]
        cb = P["b"].get(k, ({},))[0]
        waves = ce.get("SQ_WAVES", 0.0) or 1.0
        cyc = ce.get("GRBM_GUI_ACTIVE", 0.0) / N_XCD
        valu, mfma = ca.get("SQ_INSTS_VALU", 0.0), ce.get("SQ_INSTS_MFMA", 0.0)
        simd_cyc = max(1.0, cyc * N_CU * SIMD)
        vec_issue = 100.0 * ((valu - mfma) * 2 + mfma * 8) / simd_cyc
        mfma_busy = 100.0 * cb.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / simd_cyc
        wc = max(1.0, ce.get("SQ_WAVE_CYCLES", 0.0))
        pw = lambda v: v / waves
        print(f"| {k} | {waves:.0f} | {pw(valu - mfma):.0f} | {pw(mfma):.0f} | {pw(ca.get('SQ_INSTS_LDS', 0.0)):.0f} | "
              f"{pw(cb.get('SQ_INSTS_SALU', 0.0)):.0f} | {pw(ce.get('SQ_INSTS_SMEM', 0.0)):.0f} | "
              f"{pw(cb.get('SQ_INSTS_VMEM', 0.0)):.0f} | {pw(ce.get('SQ_INSTS_BRANCH', 0.0)):.0f} | {vec_issue:.1f} | "
              f"{mfma_busy:.1f} | {100.0 * ce.get('SQ_ACTIVE_INST_VALU', 0.0) / wc:.0f} | "
              f"{100.0 * ce.get('SQ_ACTIVE_INST_LDS', 0.0) / wc:.0f} | {100.0 * ca.get('SQ_ACTIVE_INST_ANY', 0.0) / max(1.0, ca.get('SQ_WAVE_CYCLES', 0.0)):.0f} |")


if __name__ == "__main__":
    main()
