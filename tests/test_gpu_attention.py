"""Attention kernel (the SDPA of lightglue.py:139-149) in isolation, through the C-ABI entry
`lg_attention`, against a float64 reference — needs an MI355X.

The full-forward parity tests see the attention only through 9 layers of mixing; these cases
drive the kernel's own corner paths directly:
  * lazy softmax reference: keys ordered by increasing score force a reference raise (and the
    O / l rescale) on every 64-key tile; decreasing order never raises after the first tile;
  * large logits (|scale q.k| up to ~90) where a stale reference would overflow exp;
  * ragged key counts (last tile partly masked, a single key) and query blocks;
  * query rows at the smallest scale the h3g common (log2-unit, accumulator-seeded) form takes, and
    waves mixing such rows with tiny ones (exact form);
  * both operand formats (fp16x3 "auto", bf16x6).
Bar: |ctx - ref64| <= 2e-6 + 2^-21 * L * max|v|, L = max_{q,k} scale * sum_d |q_d k_d| -- twice the
fp16x3 piece-truncation bound (2^-22 relative) carried by the largest logit; fp32
arithmetic itself would give 2^-24 * L.  For O(1) logits the bar is ~2.5e-6 (the kernels measure
~5e-7, tools/kbench_attn.hip); the increasing-score case (logits up to ~100) measures 2.4e-5 in
fp16x3.
"""
import ctypes

import numpy as np
import pytest
import torch

import lgamd  # noqa: F401
from lightglue_amd import _lib

pytestmark = pytest.mark.gpu

TOL = 2e-6
H = 4


def run_attention(q, k, v, scale, precision):
    lib = _lib.load()
    B, _, Nq, _ = q.shape
    Nk = k.shape[2]
    qd, kd, vd = (t.float().contiguous().cuda() for t in (q, k, v))
    ctx = torch.empty(B, Nq, H * 64, device="cuda")
    nbytes = ctypes.c_size_t()
    _lib.check(lib.lg_attention_workspace_bytes(B, H, Nq, Nk, ctypes.byref(nbytes)), "workspace")
    ws = torch.empty(max(nbytes.value, 1), dtype=torch.uint8, device="cuda")
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    rc = lib.lg_attention(qd.data_ptr(), kd.data_ptr(), vd.data_ptr(), B, H, Nq, Nk, ctypes.c_float(scale),
                          _lib.PRECISIONS[precision], ctx.data_ptr(), ws.data_ptr(), nbytes.value, stream)
    _lib.check(rc, "lg_attention")
    return ctx.cpu().double()


def reference(q, k, v, scale):
    s = torch.einsum("bhqd,bhkd->bhqk", q.double(), k.double()) * scale
    o = torch.softmax(s, dim=-1) @ v.double()
    return o.permute(0, 2, 1, 3).reshape(q.shape[0], q.shape[2], -1)


def randn(*shape, seed):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(*shape, generator=g)


def case(name):
    B = 2
    if name == "random_ragged":
        q, k, v = randn(B, H, 300, 64, seed=1), randn(B, H, 520, 64, seed=2), randn(B, H, 520, 64, seed=3)
        return q, k, v, 0.125
    if name in ("increasing_scores", "decreasing_scores"):
        # every query has a large component along u; key j has u-component growing with j, so
        # scale*q.k rises by ~0.3 per key -> the running max jumps past the lazy threshold
        # (3 in log2 units) on every 64-key tile
        Nq, Nk = 256, 640
        u = torch.ones(64) / 8.0
        q = 0.3 * randn(B, H, Nq, 64, seed=4) + 8.0 * u
        ramp = torch.linspace(-12.0, 12.0, Nk)
        if name == "decreasing_scores":
            ramp = ramp.flip(0)
        k = 0.3 * randn(B, H, Nk, 64, seed=5) + ramp[None, None, :, None] * u
        v = randn(B, H, Nk, 64, seed=6)
        return q, k, v, 1.0
    if name == "large_logits":
        q, k, v = 3.0 * randn(B, H, 192, 64, seed=7), 3.0 * randn(B, H, 200, 64, seed=8), randn(B, H, 200, 64, seed=9)
        return q, k, v, 0.125
    if name == "single_key":
        return randn(B, H, 70, 64, seed=10), randn(B, H, 1, 64, seed=11), randn(B, H, 1, 64, seed=12), 0.125
    if name == "one_key_in_last_tile":
        return randn(B, H, 257, 64, seed=13), randn(B, H, 65, 64, seed=14), randn(B, H, 65, 64, seed=15), 0.125
    if name == "small_queries":
        # every row's max |q scale log2 e| just above 2^-4, the smallest the h3g common form takes
        # (its unscaled low pieces are mostly fp16 subnormals there)
        q = randn(B, H, 256, 64, seed=16)
        q = q / q.abs().amax(-1, keepdim=True) * (0.07 / (0.125 * 1.4426950408889634))
        return q, randn(B, H, 300, 64, seed=17), randn(B, H, 300, 64, seed=18), 0.125
    if name == "mixed_row_scales":
        # row scales from 1e-3 to 8 interleaved, so waves mix rows on both sides of the 2^-4
        # threshold (such a wave runs the exact form)
        q = randn(B, H, 256, 64, seed=19)
        f = torch.logspace(-3, np.log10(8.0), 256)[torch.randperm(256, generator=torch.Generator().manual_seed(20))]
        return q * f[None, None, :, None], randn(B, H, 320, 64, seed=21), randn(B, H, 320, 64, seed=22), 0.125
    raise KeyError(name)


CASES = ["random_ragged", "increasing_scores", "decreasing_scores", "large_logits", "single_key",
         "one_key_in_last_tile", "small_queries", "mixed_row_scales"]


@pytest.mark.parametrize("kernel", ["h3m", "h3g"])
@pytest.mark.parametrize("precision,waves", [("auto", "8"), ("auto", "4"), ("auto", "2"), ("bf16x6", "8")])
@pytest.mark.parametrize("name", CASES)
def test_attention_matches_float64(name, precision, waves, kernel, monkeypatch):
    # fp16x3 kernels (16x16x32 / 32x32x16 MFMAs) under every query-block shape (LG_ATTN_WAVES:
    # 256 / 128 / 64 queries per workgroup); the small shapes here would otherwise always pick 4
    if precision == "bf16x6" and kernel == "h3g":
        pytest.skip("bf16x6 has one kernel")
    monkeypatch.setenv("LG_ATTN_WAVES", waves)
    monkeypatch.setenv("LG_ATTN_KERNEL", kernel)
    q, k, v, scale = case(name)
    got = run_attention(q, k, v, scale, precision)
    ref = reference(q, k, v, scale)
    err = (got - ref).abs().max().item()
    L = (scale * torch.einsum("bhqd,bhkd->bhqk", q.double().abs(), k.double().abs())).max().item()
    tol = TOL + 2.0 ** -21 * L * v.abs().max().item()
    assert np.isfinite(err) and err <= tol, f"{name}/{precision}: max |d| = {err:.3g} > {tol:.3g}"


@pytest.mark.parametrize("splits", ["2", "8"])
@pytest.mark.parametrize("name", CASES)
def test_attention_key_splits_match_float64(name, splits, monkeypatch):
    """Small batches split each work item's keys over LG_ATTN_SPLIT workgroups (4-wave h3g) whose
    partials (O, m, l, c) attn_split_combine_kernel merges; the lazy references of the splits
    differ, empty key ranges (single_key, one_key_in_last_tile) weigh nothing."""
    monkeypatch.setenv("LG_ATTN_WAVES", "4")
    monkeypatch.setenv("LG_ATTN_KERNEL", "h3g")
    monkeypatch.setenv("LG_ATTN_SPLIT", splits)
    q, k, v, scale = case(name)
    got = run_attention(q, k, v, scale, "auto")
    ref = reference(q, k, v, scale)
    err = (got - ref).abs().max().item()
    L = (scale * torch.einsum("bhqd,bhkd->bhqk", q.double().abs(), k.double().abs())).max().item()
    tol = TOL + 2.0 ** -21 * L * v.abs().max().item()
    assert np.isfinite(err) and err <= tol, f"{name}/split {splits}: max |d| = {err:.3g} > {tol:.3g}"


def test_increasing_scores_really_rescale():
    """The adversarial case is adversarial: the per-tile max of scale*q.k rises by more than the
    lazy threshold (3 log2 units = 2.08 nats) between consecutive 64-key tiles."""
    q, k, _, scale = case("increasing_scores")
    s = torch.einsum("bhqd,bhkd->bhqk", q.double(), k.double()) * scale
    tile_max = s.unflatten(-1, (-1, 64)).amax(-1)  # [B,H,Nq,tiles]
    assert (tile_max.diff(dim=-1) > 3 * np.log(2)).float().mean() > 0.9


@pytest.mark.parametrize("precision,kernel", [("auto", "h3m"), ("auto", "h3g"), ("bf16x6", "h3m")])
def test_values_beyond_fp16_range_are_range_scaled(precision, kernel, monkeypatch):
    """Keys up to ~4e5 and values up to ~4e6 (far past fp16's 65504): the fp16x3 planes are
    written scaled by a device-chosen power of two (kernels.h RangeOut), the key exponent folds
    into the softmax scale and the value exponent into the output, so the result keeps the same
    relative accuracy as O(1) data -- no refusal, no host round trip."""
    monkeypatch.setenv("LG_ATTN_KERNEL", kernel)
    q, k, v, scale = case("random_ragged")
    k, v, scale = k * 1.0e5, v * 1.0e6, scale / 1.0e5
    got = run_attention(q, k, v, scale, precision)
    ref = reference(q, k, v, scale)
    L = (scale * torch.einsum("bhqd,bhkd->bhqk", q.double().abs(), k.double().abs())).max().item()
    vmax = v.abs().max().item()
    err = (got - ref).abs().max().item() / vmax
    assert np.isfinite(err) and err <= TOL + 2.0 ** -21 * L, f"{precision}: relative max |d| = {err:.3g}"
