#!/usr/bin/env python3
"""CPU emulation of split-precision matrix-core arithmetic on the golden cases.

    python tools/numerics_study.py [--modes f32,x6,h3] [--cases n512,n1024]

Runs the oracle's forward (oracle/lightglue_ref.py) with every dense contraction (Linear layers,
QK^T, PV, the assignment similarity) replaced by an emulation of one arithmetic scheme, and reports
how far the outputs land from the reference's golden vectors (tests/golden).  Used to choose the
MFMA operand format of the HIP kernels; it is test tooling, not product code.

Schemes (products exact, 16-term partial sums in fp64 then accumulated in fp32, like one
v_mfma_*_32x32x16 step per 16-deep k slice):
  f64  plain float64 contraction (reference point: fp32 CPU vs exact)
  f32  fp32 FMA chain (what v_mfma_f32_32x32x2_f32 computes)
  x6   bf16x6: x = h + m + l (three bf16), the six terms of weight >= 2^-16
  x3   bf16x3: x = h + l (two bf16), terms hh + hl + lh
  h3   fp16x3: x = h + l * 2^-11 (two fp16, lo pre-scaled by 2^11), terms hh + (hl + lh) * 2^-11,
       two fp32 accumulators combined at the end
  h4   h3 + the ll term
"""
import argparse
import os
import sys
import time

import numpy as np
import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import lgamd  # noqa: E402,F401
import oracle  # noqa: E402
from oracle import lightglue_ref as R  # noqa: E402
from golden_util import case_inputs, load  # noqa: E402

MODE = "f32"
KCH = 16


def _bf16(x):
    return x.to(torch.bfloat16).to(torch.float64)


def _f16(x):
    return x.to(torch.float16).to(torch.float64)


def pieces(x):
    """Split x (fp32 values held in fp64) into (list of pieces, list of scales)."""
    x = x.to(torch.float32).to(torch.float64)
    if MODE == "x6":
        h = _bf16(x); r = x - h; m = _bf16(r); lo = _bf16(r - m)
        return [h, m, lo]
    if MODE == "x3":
        h = _bf16(x); lo = _bf16(x - h)
        return [h, lo]
    if MODE in ("h3", "h4"):
        assert x.abs().max() < 65000, "fp16 overflow"
        h = _f16(x); lo = _f16((x - h) * 2048.0) / 2048.0
        return [h, lo]
    raise ValueError(MODE)


def _chunked(a, b):
    """sum_k a[..., i, k] b[..., j, k] with k in 16-deep slices, slice sums exact (fp64),
    accumulated across slices in fp32."""
    K = a.shape[-1]
    acc = None
    for k0 in range(0, K, KCH):
        p = torch.matmul(a[..., k0:k0 + KCH], b[..., k0:k0 + KCH].transpose(-1, -2))
        acc = p.to(torch.float32) if acc is None else (acc + p.to(torch.float32))
    return acc


def mm(a, b):
    """a [..., M, K] @ b[..., N, K]^T under the current scheme, fp32 result."""
    if MODE == "f32":
        return torch.matmul(a.float(), b.float().transpose(-1, -2))
    if MODE == "f64":
        return torch.matmul(a.double(), b.double().transpose(-1, -2)).float()
    pa, pb = pieces(a.double()), pieces(b.double())
    if MODE == "x6":
        terms = [(2, 0), (1, 1), (0, 2), (1, 0), (0, 1), (0, 0)]
        acc = None
        for k0 in range(0, a.shape[-1], KCH):
            s = None
            for (i, j) in terms:  # each MFMA rounds into the fp32 accumulator
                p = torch.matmul(pa[i][..., k0:k0 + KCH], pb[j][..., k0:k0 + KCH].transpose(-1, -2))
                acc = p.float() if acc is None else acc + p.float()
        return acc
    if MODE == "x3":
        acc = None
        for k0 in range(0, a.shape[-1], KCH):
            for (i, j) in [(1, 0), (0, 1), (0, 0)]:
                p = torch.matmul(pa[i][..., k0:k0 + KCH], pb[j][..., k0:k0 + KCH].transpose(-1, -2))
                acc = p.float() if acc is None else acc + p.float()
        return acc
    if MODE in ("h3", "h4"):
        hh = _chunked(pa[0], pb[0])
        cr = None
        terms = [(1, 0), (0, 1)] + ([(1, 1)] if MODE == "h4" else [])
        for k0 in range(0, a.shape[-1], KCH):
            for (i, j) in terms:
                p = torch.matmul(pa[i][..., k0:k0 + KCH] * (2048.0 if i else 1.0),
                                 pb[j][..., k0:k0 + KCH].transpose(-1, -2) * (2048.0 if j else 1.0))
                if i and j:
                    p = p / 2048.0
                cr = p.float() if cr is None else cr + p.float()
        return hh + cr * np.float32(1.0 / 2048.0)
    raise ValueError(MODE)


def linear(x, w, b):
    y = mm(x, w)
    return y + b if b is not None else y


def sdpa(q, k, v, scale):
    s = mm(q, k) * scale
    mx = s.max(-1, keepdim=True).values
    p = torch.exp(s - mx)
    o = mm(p, v.transpose(-1, -2))
    return o / p.sum(-1, keepdim=True)


def cross_block(x0, x1, W, p, H):
    def heads(t):
        return t.unflatten(-1, (H, -1)).transpose(1, 2)

    qk0 = heads(linear(x0, W[p + ".to_qk.weight"], W[p + ".to_qk.bias"]))
    qk1 = heads(linear(x1, W[p + ".to_qk.weight"], W[p + ".to_qk.bias"]))
    v0 = heads(linear(x0, W[p + ".to_v.weight"], W[p + ".to_v.bias"]))
    v1 = heads(linear(x1, W[p + ".to_v.weight"], W[p + ".to_v.bias"]))
    s = (x0.shape[-1] // H) ** -0.5
    qk0, qk1 = qk0 * s ** 0.5, qk1 * s ** 0.5
    m0 = sdpa(qk0, qk1, v1, 1.0)
    m1 = sdpa(qk1, qk0, v0, 1.0)
    m0 = linear(m0.transpose(1, 2).flatten(-2), W[p + ".to_out.weight"], W[p + ".to_out.bias"])
    m1 = linear(m1.transpose(1, 2).flatten(-2), W[p + ".to_out.weight"], W[p + ".to_out.bias"])
    return R._ffn(x0, m0, W, p), R._ffn(x1, m1, W, p)


def match_assignment(d0, d1, W, p):
    md0 = linear(d0, W[p + ".final_proj.weight"], W[p + ".final_proj.bias"])
    md1 = linear(d1, W[p + ".final_proj.weight"], W[p + ".final_proj.bias"])
    dim = md0.shape[-1]
    md0, md1 = md0 / dim ** 0.25, md1 / dim ** 0.25
    sim = mm(md0, md1)
    z0 = F.linear(d0, W[p + ".matchability.weight"], W[p + ".matchability.bias"])
    z1 = F.linear(d1, W[p + ".matchability.weight"], W[p + ".matchability.bias"])
    return R.sigmoid_log_double_softmax(sim, z0, z1), sim


def install():
    R._linear = linear
    R._softmax_attention = lambda q, k, v, scale: sdpa(q, k, v, scale)
    R.cross_block = cross_block
    R.match_assignment = match_assignment


def run_case(name):
    g = load(name)
    conf, sd, data = case_inputs(g["meta"])
    t = time.time()
    out = oracle.lightglue_forward(sd, data, conf)
    dt = time.time() - t
    res = {}
    res["idx_mismatch"] = int((out["matches0"].numpy() != g["matches0"]).sum() + (out["matches1"].numpy() != g["matches1"]).sum())
    res["score"] = float(max(np.abs(out["matching_scores0"].numpy() - g["matching_scores0"]).max(),
                             np.abs(out["matching_scores1"].numpy() - g["matching_scores1"]).max()))
    la = out["log_assignment"]
    res["la_rowmax"] = float(np.abs(la[:, :-1, :-1].max(2).values.numpy() - g["la_row_max"]).max())
    res["prune_ok"] = bool((out["prune0"].numpy() == g["prune0"]).all() and (out["prune1"].numpy() == g["prune1"]).all())
    res["t"] = round(dt, 1)
    return res


def main():
    global MODE
    ap = argparse.ArgumentParser()
    ap.add_argument("--modes", default="f64,f32,x6,h3,h4,x3")
    ap.add_argument("--cases", default="tiny_ragged_b2,n300x257_b2,n512,prune_width_n512,n1024")
    a = ap.parse_args()
    install()
    torch.set_num_threads(os.cpu_count() or 8)
    for case in a.cases.split(","):
        for m in a.modes.split(","):
            MODE = m
            r = run_case(case)
            print(f"{case:24s} {m:4s} idx_mismatch={r['idx_mismatch']:3d} score={r['score']:.2e} "
                  f"la_rowmax={r['la_rowmax']:.2e} prune_ok={r['prune_ok']} ({r['t']}s)", flush=True)


if __name__ == "__main__":
    main()
