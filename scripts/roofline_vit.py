#!/usr/bin/env python
"""ViT-B/16 (batch 256, 224 px: 197 tokens, width 768, MLP 3072, 12 heads) per-op roofline from a
rocprofv3 kernel trace: achieved TFLOP/s and HBM TB/s per kernel class over the last N steps,
against MI355X's dense bf16 peak (2.5 PF/s) and HBM3E (8 TB/s).

FLOPs are the model's useful work (2 M N K per GEMM; attention on the unpadded 197 x 197 score
matrix: the forward does QK^T and PV, the dq kernel recomputes S then dP and dQ, the dkv kernel
recomputes S and dP then dV and dK). Bytes are the minimum HBM traffic of the op (each operand
read once, each output written once), so TB/s is a lower bound on what the kernel moved.

Which kernel does which op (the model's dispatch, models/vit.py + ops/): the forward GEMMs run on
hipBLASLt (`Custom_Cijk…MT256x256x64`: 11 blocks x {qkv, proj, fc1, fc2} + the last block's qkv
+ the patch embedding = 46 calls), the input-gradient GEMMs on hipBLASLt (`Cijk_Ailk_Bljk…MT256x256`:
11 x {qkv, proj, fc1} + last qkv = 34) except fc2's (gemm_nt EPI 2 with the GELU backward, 11), every
weight gradient on wgrad256 (46). The last block's proj / fc1 / fc2 act on the [CLS] token only.

usage: python scripts/roofline_vit.py <kernel_trace.csv> [N] > profiles/<name>.md
"""
import csv
import re
import sys

B, T, D, F, H, DH = 256, 197, 768, 3072, 12, 64
M = B * T              # token rows
MP = B * 196           # patch rows (embedding GEMM)
BLK = 11               # full blocks (the 12th is CLS-only after attention)
G = 1e9


def lin(m, k, n):
    return 2.0 * m * k * n


FWD_FULL = lin(M, D, 3 * D) + lin(M, D, D) + lin(M, D, F) + lin(M, F, D)
QKV = lin(M, D, 3 * D)
PATCH = lin(MP, D, D)
ATT_OP = 2.0 * B * H * T * T * DH          # one T x T x 64 GEMM over all heads
TOK = M * D * 2                            # one [M, 768] bf16 tensor
HID = M * F * 2                            # one [M, 3072] bf16 tensor
PARAMS = 86.6e6

# (label, kernel-name regex, FLOPs per step, min HBM bytes per step)
CLASSES = [
    ("Linear forward (hipBLASLt)", r"^Custom_Cijk_Alik_Bljk.*MT256x256x64",
     BLK * FWD_FULL + QKV + PATCH,
     BLK * (4 * TOK + TOK + TOK + HID + TOK + HID + TOK) + (TOK + 3 * TOK) + 2 * TOK),
    ("Linear input gradient (hipBLASLt: qkv, proj, fc1)", r"^Cijk_Ailk_Bljk.*MT256x256x64",
     BLK * (QKV + lin(M, D, D) + lin(M, D, F)) + QKV,
     BLK * ((3 * TOK + TOK) + (TOK + TOK) + (HID + TOK)) + 4 * TOK),
    ("fc2 input gradient + GELU backward + fc1 bias grad (gemm_nt EPI 2)", r"gemm_nt_kernel<2,",
     BLK * lin(M, D, F), BLK * (TOK + HID + HID)),
    ("Linear weight gradients (wgrad256, split-K)", r"wgrad256",
     BLK * FWD_FULL + QKV + PATCH,
     BLK * ((TOK + 3 * TOK) + 2 * TOK + (TOK + HID) + (HID + TOK)) + 4 * TOK + 2 * TOK),
    ("attention forward", r"attn_fwd_res_kernel", 12 * 2 * ATT_OP, 12 * (3 * TOK + TOK)),
    ("attention backward dQ", r"attn_bwd_dq_res_kernel", 12 * 3 * ATT_OP, 12 * (4 * TOK + TOK)),
    ("attention backward dK dV", r"attn_bwd_dkv_res_kernel", 12 * 4 * ATT_OP, 12 * (4 * TOK + 2 * TOK)),
    ("GELU forward (PyTorch elementwise)", r"GeluCUDAKernelImpl", 0.0, BLK * 2 * HID),
    ("LayerNorm forward (+ residual add)", r"ln_fwd_kernel", 0.0, 23 * 4 * TOK),
    ("LayerNorm backward (+ residual grad)", r"ln_bwd_kernel", 0.0, 23 * 4 * TOK),
    ("fused Adam (bf16 params, fp32 master / moments)", r"mt_adam_kernel", 0.0, 30 * PARAMS),
]


def main():
    path = sys.argv[1]
    nsteps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    ends = [i for i, r in enumerate(rows) if "adam_advance" in r["Kernel_Name"]]
    if len(ends) < nsteps + 1:
        ends = [i for i, r in enumerate(rows) if "mt_adam" in r["Kernel_Name"]]
    win = rows[ends[-nsteps - 1] + 1:ends[-1] + 1]
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in win) / nsteps
    print("# ViT-B/16 roofline per op (batch 256, bf16; MI355X dense peaks 2.5 PF/s, 8 TB/s)\n")
    print(f"Source: `{path.split('gpurun_out/')[-1]}`, last {nsteps} steps; kernel busy "
          f"{busy * 1e-6:.2f} ms/step. FLOPs = useful model work; bytes = minimum HBM traffic "
          "(see scripts/roofline_vit.py).\n")
    print("| op | calls/step | ms/step | GFLOP/step | TFLOP/s | % bf16 peak | min GB/step | TB/s | % HBM peak |")
    print("|---|---|---|---|---|---|---|---|---|")
    covered = 0.0
    tot_flops = 0.0
    for label, pat, flops, nbytes in CLASSES:
        rx = re.compile(pat)
        ks = [r for r in win if rx.search(r["Kernel_Name"])]
        t = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in ks) / nsteps  # ns
        covered += t
        if not ks:
            print(f"| {label} | 0 | - | | | | | | |")
            continue
        tf = flops / (t * 1e-9) / 1e12 if flops else 0.0
        tb = nbytes / (t * 1e-9) / 1e12
        tot_flops += flops
        fl = f"{flops / G:.0f} | {tf:.0f} | {100 * tf / 2500:.0f} %" if flops else "- | - | -"
        print(f"| {label} | {len(ks) / nsteps:g} | {t * 1e-6:.3f} | {fl} | {nbytes / G:.1f} | {tb:.2f} | "
              f"{100 * tb / 8:.0f} % |")
    print(f"| (other kernels) | | {(busy - covered) * 1e-6:.3f} | | | | | | |")
    print(f"\nWhole step: {tot_flops / G:.0f} GFLOP of model work in {busy * 1e-6:.2f} ms of kernel time = "
          f"{tot_flops / (busy * 1e-9) / 1e12:.0f} TFLOP/s ({100 * tot_flops / (busy * 1e-9) / 2.5e15:.0f} % of "
          "the dense bf16 peak).")


if __name__ == "__main__":
    main()
