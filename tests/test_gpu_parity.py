"""HIP path vs the reference's golden vectors (and the oracle) — needs an MI355X.

Bar (BASELINE north star): match indices bit-exact, matching scores |d| <= 1e-4,
log-assignment |d| <= 1e-3 (fp32 vs fp64 already differs by 2.2e-3), prune counts exact.
Near-ties: a row / column whose fp64 top-1 / top-2 margin (fixture keys margin0 / margin1) is below
NEAR_TIE = 1e-4 is not decidable by fp32 arithmetic (the reference's own fp32 result differs from
fp64 by more than that in log-assignment units); its index may flip and is counted, never silently
skipped: every forward test reports (rows below NEAR_TIE, flips among them) and asserts that NO
index flips at a margin >= NEAR_TIE.  With LG_PARITY_REPORT=<path> the counts are appended there
as JSON lines (profiles/<round>/parity_report.jsonl).
Both matrix-core operand formats are held to the same bar: "auto" (fp16x3, the default) and
"bf16x6" (the guarded fallback).
"""
import json
import os

import numpy as np
import pytest
import torch

import lgamd  # noqa: F401
from golden_util import case_inputs, case_names, load, sinkhorn_inputs, sinkhorn_names

NEAR_TIE = 1e-4
SCORE_TOL = 1e-4
LA_TOL = 1e-3
# descriptors (every layer): |d| <= DESC_ATOL + DESC_RTOL * |ref| (measured max 1.1e-5, profiles/r02/parity_report.jsonl)
DESC_ATOL, DESC_RTOL = 5e-5, 1e-5

pytestmark = pytest.mark.gpu


def _model(conf, sd, precision="auto"):
    from lightglue_amd import LightGlue

    m = LightGlue({**dict(conf), "precision": precision}).eval().cuda()
    res = m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
    assert not res.missing_keys and not res.unexpected_keys
    return m


def _gpu_data(data):
    d = {k: torch.from_numpy(v).cuda() for k, v in data.items() if not k.startswith("image_size")}
    d["view0"] = {"image_size": torch.from_numpy(data["image_size0"]).cuda()}
    d["view1"] = {"image_size": torch.from_numpy(data["image_size1"]).cuda()}
    return d


def _report(**kw):
    path = os.environ.get("LG_PARITY_REPORT")
    if path:
        with open(path, "a") as f:
            f.write(json.dumps(kw) + "\n")


def check_against_golden(pred, g, label=""):
    """Assert the golden bar; return the near-tie / error report of this forward."""
    m0, m1 = pred["matches0"].cpu().numpy(), pred["matches1"].cpu().numpy()
    ok0 = np.ones_like(m0, dtype=bool)
    ok1 = np.ones_like(m1, dtype=bool)
    if "margin0" in g:
        ok0 = g["margin0"] >= NEAR_TIE
        ok1 = g["margin1"] >= NEAR_TIE
    f0, f1 = m0 != g["matches0"], m1 != g["matches1"]
    rep = {
        "case": label,
        "near_tie_rows": int((~ok0).sum()), "near_tie_cols": int((~ok1).sum()),
        "flips_near_tie": int((f0 & ~ok0).sum() + (f1 & ~ok1).sum()),
        "flips_decidable": int((f0 & ok0).sum() + (f1 & ok1).sum()),
    }
    if "margin0" in g:
        rep["min_margin"] = float(min(g["margin0"].min(), g["margin1"].min()))
        rep["rows_margin_below_1e-3"] = int((g["margin0"] < 1e-3).sum() + (g["margin1"] < 1e-3).sum())
    np.testing.assert_array_equal(m0[ok0], g["matches0"][ok0])
    np.testing.assert_array_equal(m1[ok1], g["matches1"][ok1])
    s0, s1 = pred["matching_scores0"].cpu().numpy(), pred["matching_scores1"].cpu().numpy()
    same0 = ok0 & ((m0 > -1) == (g["matches0"] > -1))
    same1 = ok1 & ((m1 > -1) == (g["matches1"] > -1))
    np.testing.assert_allclose(s0[same0], g["matching_scores0"][same0], atol=SCORE_TOL, rtol=0)
    np.testing.assert_allclose(s1[same1], g["matching_scores1"][same1], atol=SCORE_TOL, rtol=0)
    rep["max_score_err"] = float(max(np.abs(s0[same0] - g["matching_scores0"][same0]).max(initial=0),
                                     np.abs(s1[same1] - g["matching_scores1"][same1]).max(initial=0)))
    p0, p1 = pred["prune0"].cpu().numpy(), pred["prune1"].cpu().numpy()
    np.testing.assert_array_equal(p0, g["prune0"])
    np.testing.assert_array_equal(p1, g["prune1"])
    assert p0.dtype == g["prune0"].dtype
    la = pred["log_assignment"]
    inner = la[:, :-1, :-1]
    np.testing.assert_allclose(inner.max(2).values.cpu().numpy(), g["la_row_max"], atol=LA_TOL)
    np.testing.assert_allclose(inner.max(1).values.cpu().numpy(), g["la_col_max"], atol=LA_TOL)
    np.testing.assert_allclose(la[:, :-1, -1].cpu().numpy(), g["la_dustbin_col"], atol=1e-4)
    np.testing.assert_allclose(la[:, -1, :-1].cpu().numpy(), g["la_dustbin_row"], atol=1e-4)
    assert float(la[0, -1, -1]) == 0.0
    if "log_assignment" in g:
        np.testing.assert_allclose(la.cpu().numpy(), g["log_assignment"], atol=LA_TOL)
    if "ref_descriptors0" in g:
        k0, k1 = g["ref_descriptors0"].shape[2], g["ref_descriptors1"].shape[2]
        r0 = pred["ref_descriptors0"][:, :, :k0].cpu().numpy()
        r1 = pred["ref_descriptors1"][:, :, :k1].cpu().numpy()
        np.testing.assert_allclose(r0, g["ref_descriptors0"], atol=DESC_ATOL, rtol=DESC_RTOL)
        np.testing.assert_allclose(r1, g["ref_descriptors1"], atol=DESC_ATOL, rtol=DESC_RTOL)
        rep["max_desc_err"] = float(max(np.abs(r0 - g["ref_descriptors0"]).max(), np.abs(r1 - g["ref_descriptors1"]).max()))
    _report(**rep)
    return rep


@pytest.mark.parametrize("precision", ["auto", "bf16x6"])
@pytest.mark.parametrize("name", case_names())
def test_forward_matches_reference_golden(name, precision):
    g = load(name)
    conf, sd, data = case_inputs(g["meta"])
    model = _model(conf, sd, precision)
    with torch.no_grad():
        pred = model(_gpu_data(data))
    torch.cuda.synchronize()
    assert model.last_precision_used == ("fp16x3" if precision == "auto" else "bf16x6")
    assert int(pred["stop_layer"][0]) + 1 == int(g["n_layers_run"])
    check_against_golden(pred, g, f"{name}/{precision}")


@pytest.mark.parametrize("tile,waves,assign,kernel,ksplit,asplit", [("big", "8", "sim_h3", "h3g", "4", "auto"),
                                                                     ("small", "4", "x6_fused", "h3m", "4", "auto"),
                                                                     ("small", "2", "x6_unfused", "h3g", "1", "auto"),
                                                                     ("small", "8", "sim_h3", "h3g", "2", "auto"),
                                                                     ("big", "2", "sim_h3", "h3m", "4", "auto"),
                                                                     ("medium", "4", "sim_h3", "h3g", "4", "1"),
                                                                     ("small", "4", "sim_h3", "h3g", "4", "8"),
                                                                     ("big", "8", "sim_h3", "h3g", "nt", "auto")])
@pytest.mark.parametrize("name", case_names())
def test_forward_golden_all_launch_shapes(name, tile, waves, assign, kernel, ksplit, asplit, monkeypatch):
    """The fp16x3 GEMM picks 256x256 tiles (throughput), 128x128 tiles (fewer big tiles than CUs)
    or 64x64 tiles (fewer than a quarter, e.g. B = 1) by row count, and the attention 8, 4 or 2 waves (256/128/64 queries) per
    workgroup, and the assignment either recomputes the similarity inside two fp16x3 GEMM passes
    (M, N multiples of 16, no pruning: sim_h3) or materialises it with the bf16x6 GEMM and runs
    the two-read fused passes (N % 4 == 0, N <= 2048) or the four-read ones; LG_GEMM_TILE /
    LG_ATTN_WAVES / LG_ASSIGN_SIM_X6 / LG_ASSIGN_UNFUSED force each so that every launch shape is
    checked against the reference on every golden case.  The 64x64 tiles split the k-tiles over
    LG_GEMM_KSPLIT waves (4 by default at small row counts; 1 = the unsplit single-wave tile), and
    the 4-wave attention splits the keys of small batches over LG_ATTN_SPLIT workgroups (auto: up
    to 8, merged by attn_split_combine_kernel; 1 = unsplit)."""
    monkeypatch.setenv("LG_GEMM_TILE", tile)
    if ksplit == "nt":  # the streamed-once hints at every size, ffn.3 walking front to back
        monkeypatch.setenv("LG_NT_MIN_MB", "0")
        monkeypatch.setenv("LG_FFN3_REVERSE", "0")
    else:
        monkeypatch.setenv("LG_GEMM_KSPLIT", ksplit)
    if asplit != "auto":
        monkeypatch.setenv("LG_ATTN_SPLIT", asplit)
    monkeypatch.setenv("LG_ATTN_WAVES", waves)
    monkeypatch.setenv("LG_ATTN_KERNEL", kernel)  # fp16x3 attention: 16x16x32 (h3g) / 32x32x16 (h3m) MFMAs
    if assign != "sim_h3":  # the materialised bf16x6 similarity
        monkeypatch.setenv("LG_ASSIGN_SIM_X6", "1")
    if assign == "x6_unfused":  # its four-read assignment passes (N % 4 != 0 or N > 2048)
        monkeypatch.setenv("LG_ASSIGN_UNFUSED", "1")
    g = load(name)
    conf, sd, data = case_inputs(g["meta"])
    model = _model(conf, sd, "auto")
    with torch.no_grad():
        pred = model(_gpu_data(data))
    torch.cuda.synchronize()
    assert model.last_precision_used == "fp16x3"
    check_against_golden(pred, g, f"{name}/tile={tile},waves={waves},{assign},{kernel},ksplit={ksplit},asplit={asplit}")


def test_weight_changes_after_first_forward_are_picked_up():
    """The forward re-uploads weights when a parameter changes in place (version bump) or is
    replaced by a new tensor object, like a torch module would use its current parameters."""
    from lightglue_amd.weights import synthetic_pair, synthetic_state_dict

    conf = {"filter_threshold": 0.1}
    sd = synthetic_state_dict(conf, seed=0)
    data = _gpu_data(synthetic_pair(B=1, M=200, N=180, seed=4))
    model = _model(conf, sd)
    with torch.no_grad():
        model(data)
        model.log_assignment[-1].final_proj.weight.mul_(0.5)  # in place
        a = model(data)
        model.log_assignment[-1].matchability.bias = torch.nn.Parameter(  # new object
            model.log_assignment[-1].matchability.bias.detach() + 1.0)
        b = model(data)
    sd2 = {k: v.copy() for k, v in sd.items()}
    sd2["log_assignment.8.final_proj.weight"] = sd2["log_assignment.8.final_proj.weight"] * np.float32(0.5)
    ref_a = _model(conf, sd2)
    sd2["log_assignment.8.matchability.bias"] = sd2["log_assignment.8.matchability.bias"] + np.float32(1.0)
    ref_b = _model(conf, sd2)
    with torch.no_grad():
        ra, rb = ref_a(data), ref_b(data)
    for got, ref in ((a, ra), (b, rb)):
        assert torch.equal(got["matches0"], ref["matches0"])
        assert torch.equal(got["log_assignment"], ref["log_assignment"])


def _assert_same_result(a, b, tol=SCORE_TOL):
    for k in ("matches0", "matches1", "prune0", "prune1"):
        assert torch.equal(a[k], b[k]), k
    for k in ("matching_scores0", "matching_scores1"):
        assert torch.allclose(a[k], b[k], atol=tol, rtol=0), k


def test_values_beyond_fp16_range_are_range_scaled():
    """Descriptors beyond the fp16 range (|x| up to ~2e4 x 2e5): every run-time plane image
    picks its power-of-two scale on the device (kernels.h RangeOut), so the fp16x3 forward needs no
    guard, no read-back and no rerun, and gives the bf16x6 (full fp32 range) result."""
    from lightglue_amd.weights import synthetic_pair, synthetic_state_dict

    conf = {"filter_threshold": 0.1}
    sd = synthetic_state_dict(conf, seed=0)
    data = synthetic_pair(B=1, M=128, N=120, seed=2)
    data["descriptors0"] = data["descriptors0"] * np.float32(2.0e5)
    auto, x6 = _model(conf, sd, "auto"), _model(conf, sd, "bf16x6")
    with torch.no_grad():
        a = auto(_gpu_data(data))
        b = x6(_gpu_data(data))
    assert auto.last_precision_used == "fp16x3"
    _assert_same_result(a, b)


def test_forward_batched_equals_single():
    """B=3 batch gives the same result per pair as three B=1 calls (no cross-pair leakage)."""
    from lightglue_amd.weights import synthetic_pair, synthetic_state_dict

    conf = {"filter_threshold": 0.1}
    model = _model(conf, synthetic_state_dict(conf, seed=0))
    data = synthetic_pair(B=3, M=200, N=170, seed=4)
    with torch.no_grad():
        full = model(_gpu_data(data))
        for b in range(3):
            one = model(_gpu_data({k: v[b : b + 1] for k, v in data.items()}))
            assert torch.equal(one["matches0"][0], full["matches0"][b])
            assert torch.equal(one["matches1"][0], full["matches1"][b])
            assert torch.allclose(one["matching_scores0"][0], full["matching_scores0"][b], atol=1e-6)


def test_forward_deterministic():
    from lightglue_amd.weights import synthetic_pair, synthetic_state_dict

    conf = {"filter_threshold": 0.1}
    model = _model(conf, synthetic_state_dict(conf, seed=0))
    d = _gpu_data(synthetic_pair(B=2, M=300, N=310, seed=9))
    with torch.no_grad():
        a = model(d)
        b = model(d)
    for k in ("matches0", "matches1", "matching_scores0", "matching_scores1", "log_assignment"):
        assert torch.equal(a[k], b[k]), k


def test_no_image_size_fallback_matches_oracle():
    """Without view*/image_size the keypoints are normalised by their extent (lightglue.py:25-26)."""
    import oracle
    from lightglue_amd.weights import synthetic_pair, synthetic_state_dict

    conf = {"filter_threshold": 0.1}
    sd = synthetic_state_dict(conf, seed=0)
    data = synthetic_pair(B=1, M=150, N=140, seed=3)
    ref = oracle.lightglue_forward(sd, {k: v for k, v in data.items() if not k.startswith("image_size")}, conf)
    model = _model(conf, sd)
    with torch.no_grad():
        pred = model({k: torch.from_numpy(v).cuda() for k, v in data.items() if not k.startswith("image_size")})
    np.testing.assert_array_equal(pred["matches0"].cpu().numpy(), ref["matches0"].numpy())
    np.testing.assert_array_equal(pred["matches1"].cpu().numpy(), ref["matches1"].numpy())
    np.testing.assert_allclose(pred["matching_scores0"].cpu().numpy(), ref["matching_scores0"].numpy(), atol=SCORE_TOL)


def test_empty_keypoints_raise_like_reference():
    from lightglue_amd.weights import synthetic_pair, synthetic_state_dict

    conf = {}
    model = _model(conf, synthetic_state_dict(conf, seed=0))
    data = _gpu_data(synthetic_pair(B=1, M=16, N=16, seed=3))
    data["keypoints1"] = data["keypoints1"][:, :0]
    data["descriptors1"] = data["descriptors1"][:, :0]
    with pytest.raises(IndexError):
        model(data)


def test_cpu_inputs_fail_loudly():
    from lightglue_amd.weights import synthetic_pair, synthetic_state_dict

    model = _model({}, synthetic_state_dict({}, seed=0))
    data = {k: torch.from_numpy(v) for k, v in synthetic_pair(B=1, M=8, seed=3).items()}
    with pytest.raises(RuntimeError):
        model(data)


@pytest.mark.parametrize("name", sinkhorn_names())
def test_sinkhorn_matches_reference_golden(name):
    """configs[4]'s assignment head against the reference: the small cases compare all of Z, the
    4096 x 4096 x B=2 50-iteration case (the configs[4] shape) 16 sampled rows, the dustbin
    column, every row / column maximum and every argmax whose top-1 / top-2 margin is >= 1e-4."""
    from lightglue_amd import log_optimal_transport

    g = load(name)
    meta = g["meta"]
    scores = torch.from_numpy(sinkhorn_inputs(meta)).cuda()
    Z = log_optimal_transport(scores, torch.tensor(meta["alpha"]), meta["iters"]).cpu()
    inner = Z[:, :-1, :-1]
    if "Z" in g:
        np.testing.assert_allclose(Z.numpy(), g["Z"], atol=1e-4, rtol=1e-5)
        np.testing.assert_array_equal(inner.max(2).indices.numpy(), g["row_argmax"])
        np.testing.assert_array_equal(inner.max(1).indices.numpy(), g["col_argmax"])
        return
    np.testing.assert_allclose(Z[:, g["sample_rows"]].numpy(), g["Z_rows"], atol=1e-4, rtol=1e-5)
    np.testing.assert_allclose(Z[:, :, -1].numpy(), g["Z_dustbin_col"], atol=1e-4, rtol=1e-5)
    np.testing.assert_allclose(inner.max(2).values.numpy(), g["row_max"], atol=1e-4, rtol=1e-5)
    np.testing.assert_allclose(inner.max(1).values.numpy(), g["col_max"], atol=1e-4, rtol=1e-5)
    r_ok, c_ok = g["row_margin"] >= NEAR_TIE, g["col_margin"] >= NEAR_TIE
    np.testing.assert_array_equal(inner.max(2).indices.numpy()[r_ok], g["row_argmax"][r_ok])
    np.testing.assert_array_equal(inner.max(1).indices.numpy()[c_ok], g["col_argmax"][c_ok])
    _report(case=name, near_tie_rows=int((~r_ok).sum()), near_tie_cols=int((~c_ok).sum()),
            flips_near_tie=int((inner.max(2).indices.numpy() != g["row_argmax"])[~r_ok].sum()
                               + (inner.max(1).indices.numpy() != g["col_argmax"])[~c_ok].sum()))


@pytest.mark.parametrize(
    "B,M,N,alpha,iters",
    [
        (2, 300, 4096, 1.0, 20),   # fused path, 16 float4 chunks per lane (4-wave workgroups)
        (1, 4095, 777, 0.3, 10),   # fused, unaligned rows (scalar loads), many row runs
        (3, 33, 257, 2.0, 50),     # fused, ragged last chunk
        (1, 1, 1, -1.0, 7),        # fused, single real row / column
        (8, 64, 2048, 1.0, 5),     # fused, many pairs
        (1, 40, 4100, 1.0, 10),    # N > 4096: two-read general path
    ],
)
def test_sinkhorn_matches_oracle_shapes(B, M, N, alpha, iters):
    """Both Sinkhorn paths (one-read fused N <= 4096, transposed two-read otherwise) against the
    torch-CPU restatement of superglue.py:173-201 on seeded scores; |dZ| <= 1e-4, argmaxes exact
    outside fp32 near-ties."""
    import oracle
    from lightglue_amd import log_optimal_transport

    g = torch.Generator().manual_seed(B * 7919 + M * 31 + N)
    scores = torch.randn((B, M, N), generator=g) * 2.0
    ref = oracle.log_optimal_transport(scores, alpha, iters)
    Z = log_optimal_transport(scores.cuda(), alpha, iters).cpu()
    np.testing.assert_allclose(Z.numpy(), ref.numpy(), atol=1e-4, rtol=1e-5)
    inner, rinner = Z[:, :-1, :-1], ref[:, :-1, :-1]
    top = rinner.topk(min(2, N), dim=2).values
    clear = (top[..., 0] - top[..., -1] > 1e-4) if N > 1 else torch.ones(top.shape[:2], dtype=torch.bool)
    assert torch.equal(inner.max(2).indices[clear], rinner.max(2).indices[clear])


@pytest.mark.parametrize("N", [72, 4096])
def test_sinkhorn_underflow_column_takes_exact_path(N):
    """A column ~300 below every row's maximum: its exponentials underflow in the scaled
    one-FMA column statistics, the merge flags it and the exact running-max kernel reruns; the
    result must still match the oracle."""
    import oracle
    from lightglue_amd import log_optimal_transport

    g = torch.Generator().manual_seed(11)
    scores = torch.randn((2, 50, N), generator=g) * 2.0
    scores[:, :, 5] = -300.0
    scores[1, 7, :] = -250.0
    ref = oracle.log_optimal_transport(scores, 1.0, 20)
    Z = log_optimal_transport(scores.cuda(), 1.0, 20).cpu()
    assert torch.isfinite(ref).all()
    np.testing.assert_allclose(Z.numpy(), ref.numpy(), atol=1e-4, rtol=1e-5)


def test_filter_matches_matches_oracle():
    import oracle
    from lightglue_amd import filter_matches

    rng = np.random.default_rng(5)
    for (B, M, N, th) in [(2, 70, 90, 0.1), (1, 300, 257, 0.0), (3, 5, 1, 0.2)]:
        la = torch.from_numpy((rng.standard_normal((B, M + 1, N + 1)) * 3).astype(np.float32))
        la[0, 3, :] = la[0, 3, 0]  # exact ties -> first index
        ref = oracle.filter_matches(la, th)
        got = filter_matches(la.cuda(), th)
        np.testing.assert_array_equal(got[0].cpu().numpy(), ref[0].numpy())
        np.testing.assert_array_equal(got[1].cpu().numpy(), ref[1].numpy())
        # exp() of the same fp32 value: GPU expf vs torch-CPU differ by <= 1 ulp
        np.testing.assert_allclose(got[2].cpu().numpy(), ref[2].numpy(), rtol=3e-7, atol=0)
        np.testing.assert_allclose(got[3].cpu().numpy(), ref[3].numpy(), rtol=3e-7, atol=0)


def test_profile_family_mask():
    """lg_profile_enable: 1 times every family; LG_PROFILE_ONLY(k) masks time only family k."""
    from lightglue_amd.weights import synthetic_pair, synthetic_state_dict

    conf = {"filter_threshold": 0.1}
    m = _model(conf, synthetic_state_dict(conf, seed=0))
    d = _gpu_data(synthetic_pair(B=1, M=128, N=96, seed=3))
    with torch.no_grad():
        m(d)
        m.profile_enable(True, only=("attention",))
        m(d)
        att = m.profile_read("attention")
        gem = m.profile_read("gemm")
        m.profile_enable(True)
        m(d)
        gem_all = m.profile_read("gemm")
        m.profile_enable(False)
    assert att[1] == 2 * 9 and att[0] > 0  # self + cross per layer
    assert gem[1] == 0
    assert gem_all[1] > 0 and gem_all[2] > 0


def test_configs2_batch32_equals_golden():
    """configs[2] shape (N = 2048, 9 layers, B = 32 pairs in one forward): the n2048 golden pair
    tiled 32 times, every odd pair with its image-1 keypoints permuted.  Every pair must give the
    golden matches exactly (mapped through its permutation) and scores within 1e-4."""
    g = load("n2048")
    conf, sd, data = case_inputs(g["meta"])
    B, N = 32, data["keypoints1"].shape[1]
    rng = np.random.default_rng(0)
    batch = {k: np.repeat(v, B, axis=0) for k, v in data.items()}
    perms = []
    for b in range(B):
        perm = rng.permutation(N) if b % 2 else np.arange(N)
        batch["keypoints1"][b] = data["keypoints1"][0][perm]
        batch["descriptors1"][b] = data["descriptors1"][0][perm]
        perms.append(perm)
    model = _model(conf, sd)
    with torch.no_grad():
        pred = model(_gpu_data(batch))
    m0, m1 = pred["matches0"].cpu().numpy(), pred["matches1"].cpu().numpy()
    s0, s1 = pred["matching_scores0"].cpu().numpy(), pred["matching_scores1"].cpu().numpy()
    for b, perm in enumerate(perms):
        inv = np.argsort(perm)
        e0 = np.where(g["matches0"][0] > -1, inv[np.maximum(g["matches0"][0], 0)], -1)
        np.testing.assert_array_equal(m0[b], e0, err_msg=f"pair {b}")
        np.testing.assert_array_equal(m1[b], g["matches1"][0][perm], err_msg=f"pair {b}")
        np.testing.assert_allclose(s0[b], g["matching_scores0"][0], atol=SCORE_TOL, rtol=0)
        np.testing.assert_allclose(s1[b], g["matching_scores1"][0][perm], atol=SCORE_TOL, rtol=0)


@pytest.mark.parametrize("name", [n for n in case_names() if "layer0_desc0" in load(n)])
def test_every_layer_matches_reference_layers(name):
    """Training mode returns every layer's descriptors (lightglue.py:521-524,572); each layer is
    compared with the reference's per-layer outputs stored in the tiny fixtures, so a layer-local
    regression shows at its own layer instead of after 9 layers of mixing."""
    g = load(name)
    conf, sd, data = case_inputs(g["meta"])
    model = _model(conf, sd).train()
    with torch.no_grad():
        pred = model(_gpu_data(data))
    L = model.conf.n_layers
    assert pred["ref_descriptors0"].shape[1] == L
    errs = []
    for i in range(L):
        for s in (0, 1):
            got = pred[f"ref_descriptors{s}"][:, i].cpu().numpy()
            ref = g[f"layer{i}_desc{s}"]
            np.testing.assert_allclose(got, ref, atol=DESC_ATOL, rtol=DESC_RTOL, err_msg=f"layer {i} image {s}")
            errs.append(float(np.abs(got - ref).max()))
    _report(case=f"{name}/layers", max_desc_err_per_layer=[max(errs[2 * i], errs[2 * i + 1]) for i in range(L)])
    # training mode: the final outputs are those of the full-depth eval forward
    model.eval()
    with torch.no_grad():
        ev = model(_gpu_data(data))
    assert torch.equal(ev["matches0"], pred["matches0"])
    assert torch.equal(ev["ref_descriptors0"][:, 0], pred["ref_descriptors0"][:, -1])


def test_training_mode_gates_pruning_and_early_stop():
    """lightglue.py:502-503: early stop and point pruning only run in eval mode."""
    g = load("prune_depth_width_n512")
    conf, sd, data = case_inputs(g["meta"])
    model = _model(conf, sd)
    with torch.no_grad():
        ev = model(_gpu_data(data))
        model.train()
        tr = model(_gpu_data(data))
    assert ev["prune0"].dtype == torch.int64 and int(ev["prune0"].min()) < model.conf.n_layers
    assert tr["prune0"].dtype == torch.float32 and bool((tr["prune0"] == model.conf.n_layers).all())
    assert int(tr["stop_layer"][0]) == model.conf.n_layers - 1
    assert tr["ref_descriptors0"].shape[1] == model.conf.n_layers
    off = _model({k: v for k, v in conf.items() if k not in ("width_confidence", "depth_confidence")}, sd)
    with torch.no_grad():
        full = off(_gpu_data(data))
    assert torch.equal(tr["matches0"], full["matches0"])


def test_training_mode_with_autograd_is_differentiable():
    """Training mode with gradients enabled runs the autograd training path (tests/test_gpu_train.py
    pins its gradients): every layer's descriptors and the log assignment carry a graph, and a
    backward reaches every parameter."""
    from lightglue_amd.weights import synthetic_pair, synthetic_state_dict

    model = _model({"n_layers": 2}, synthetic_state_dict({"n_layers": 2}, seed=0)).train()
    pred = model(_gpu_data(synthetic_pair(B=1, M=16, seed=3)))
    assert pred["ref_descriptors0"].requires_grad and pred["log_assignment"].requires_grad
    assert pred["ref_descriptors0"].shape[1] == 2
    (pred["ref_descriptors0"].sum() + pred["log_assignment"][:, :-1, :-1].sum()).backward()
    missing = [n for n, p in model.named_parameters() if p.grad is None and not n.startswith(("token_confidence", "log_assignment.0"))]
    assert not missing, missing


@pytest.mark.parametrize("name", ["tiny_ragged_b2", "input_proj_n128"])
def test_unaligned_descriptor_views(name):
    """Descriptors passed as views 4 bytes past a 16-byte boundary (input_dim 256 and != 256)
    give exactly the result of the aligned copies."""
    g = load(name)
    conf, sd, data = case_inputs(g["meta"])
    model = _model(conf, sd)
    d = _gpu_data(data)
    with torch.no_grad():
        ref = model(d)
        for k in ("descriptors0", "descriptors1"):
            t = d[k]
            buf = torch.empty(t.numel() + 1, device=t.device, dtype=t.dtype)
            view = buf[1:].view(t.shape)
            view.copy_(t)
            assert view.data_ptr() % 16 == 4
            d[k] = view
        got = model(d)
    for k in ("matches0", "matches1", "matching_scores0", "matching_scores1", "log_assignment"):
        assert torch.equal(got[k], ref[k]), k


def test_submodule_replacement_and_data_writes_are_picked_up():
    """a replaced submodule is seen by the next forward; writes through p.data are not
    (they bypass the version counter) until reload_weights()."""
    from lightglue_amd import LightGlue
    from lightglue_amd.weights import synthetic_pair, synthetic_state_dict

    conf = {"filter_threshold": 0.1}
    sd = synthetic_state_dict(conf, seed=0)
    data = _gpu_data(synthetic_pair(B=1, M=200, N=180, seed=4))
    model = _model(conf, sd)
    sd2 = {k: v.copy() for k, v in sd.items()}
    sd2["log_assignment.8.final_proj.weight"] = sd2["log_assignment.8.final_proj.weight"] * np.float32(0.5)
    ref = _model(conf, sd2)
    with torch.no_grad():
        base = model(data)
        new = type(model.log_assignment[8])(256).cuda()
        new.load_state_dict({"matchability.weight": torch.from_numpy(sd2["log_assignment.8.matchability.weight"]),
                             "matchability.bias": torch.from_numpy(sd2["log_assignment.8.matchability.bias"]),
                             "final_proj.weight": torch.from_numpy(sd2["log_assignment.8.final_proj.weight"]),
                             "final_proj.bias": torch.from_numpy(sd2["log_assignment.8.final_proj.bias"])})
        model.log_assignment[8] = new
        swapped = model(data)
        r = ref(data)
        assert torch.equal(swapped["log_assignment"], r["log_assignment"])
        assert not torch.equal(swapped["log_assignment"], base["log_assignment"])
        # .data write: invisible until reload_weights()
        model2 = _model(conf, sd)
        model2(data)
        model2.log_assignment[8].final_proj.weight.data.mul_(0.5)
        model2.reload_weights()
        assert torch.equal(model2(data)["log_assignment"], r["log_assignment"])
    assert isinstance(model, LightGlue)


def test_values_beyond_fp16_range_with_pruning():
    """with width pruning on, an out-of-range forward gives the bf16x6 result (the
    range scaling also covers the re-planed, compacted residual stream)."""
    from lightglue_amd.weights import synthetic_pair

    g = load("prune_width_n512")
    conf, sd, data = case_inputs(g["meta"])
    data = synthetic_pair(B=1, M=256, N=240, seed=2)
    data["descriptors0"] = data["descriptors0"] * np.float32(2.0e5)
    auto, x6 = _model(conf, sd, "auto"), _model(conf, sd, "bf16x6")
    with torch.no_grad():
        a = auto(_gpu_data(data))
        b = x6(_gpu_data(data))
    _assert_same_result(a, b)


def _stack_pairs(datas):
    return {k: np.concatenate([d[k] for d in datas], 0) for k in datas[0]}


@pytest.mark.parametrize("precision", ["auto", "bf16x6"])
@pytest.mark.parametrize("name,seeds", [("prune_depth_width_n512", (22, 5, 9)), ("prune_width_n512", (21, 3)),
                                        ("early_stop_n256", (23, 4, 6, 8))])
def test_batched_pruning_equals_per_pair(name, seeds, precision):
    """Pruning / early stop for B > 1 (the reference asserts B == 1, lightglue.py:528,533): every
    pair prunes and stops on its own with device-side counts, so a batch gives exactly what each
    pair gives alone -- matches, prune counts, stop layers, its log-assignment block and its kept
    descriptors."""
    from lightglue_amd.weights import synthetic_pair

    g = load(name)
    conf, sd, data = case_inputs(g["meta"])
    pkw = dict(g["meta"]["pair"])
    pairs = []
    for sd_ in seeds:
        pkw["seed"] = sd_
        pairs.append(synthetic_pair(**pkw))
    model = _model(conf, sd, precision)
    with torch.no_grad():
        full = model(_gpu_data(_stack_pairs(pairs)))
        singles = [model(_gpu_data(p)) for p in pairs]
    for i, one in enumerate(singles):
        for k in ("matches0", "matches1", "prune0", "prune1"):
            assert torch.equal(one[k][0], full[k][i]), (i, k)
        assert int(one["stop_layer"][0]) == int(full["stop_layer"][i])
        assert torch.allclose(one["matching_scores0"][0], full["matching_scores0"][i], atol=1e-6)
        la1, laB = one["log_assignment"][0], full["log_assignment"][i]
        assert la1.shape == laB.shape, (i, la1.shape, laB.shape)
        assert torch.allclose(la1, laB, atol=1e-5)
        assert torch.allclose(one["ref_descriptors0"][0, 0], full["ref_descriptors0"][i][0], atol=1e-6)
    # the batch really exercises ragged sets: the pairs keep different numbers of points
    if "width" in conf and conf.get("width_confidence", -1) > 0:
        assert len({int(k) for k in full["kept0"].tolist()}) > 1


def test_configs3_batched_pruning_equals_golden():
    """configs[3] shape (N = 2048, width = depth = 0.95) batched: the reference golden pair (prunes
    ~10 % per layer, stops after layer 5) four times in one forward, with image 1 permuted in two of
    them; every pair must give the golden matches and prune counts exactly."""
    g = load("prune_depth_width_n2048")
    conf, sd, data = case_inputs(g["meta"])
    N = data["keypoints1"].shape[1]
    rng = np.random.default_rng(1)
    batch = {k: np.repeat(v, 4, axis=0) for k, v in data.items()}
    perms = []
    for b in range(4):
        perm = rng.permutation(N) if b % 2 else np.arange(N)
        batch["keypoints1"][b] = data["keypoints1"][0][perm]
        batch["descriptors1"][b] = data["descriptors1"][0][perm]
        perms.append(perm)
    model = _model(conf, sd)
    with torch.no_grad():
        pred = model(_gpu_data(batch))
    assert [int(s) + 1 for s in pred["stop_layer"].tolist()] == [int(g["n_layers_run"])] * 4
    m0, m1 = pred["matches0"].cpu().numpy(), pred["matches1"].cpu().numpy()
    p0, p1 = pred["prune0"].cpu().numpy(), pred["prune1"].cpu().numpy()
    for b, perm in enumerate(perms):
        inv = np.argsort(perm)
        e0 = np.where(g["matches0"][0] > -1, inv[np.maximum(g["matches0"][0], 0)], -1)
        np.testing.assert_array_equal(m0[b], e0, err_msg=f"pair {b}")
        np.testing.assert_array_equal(m1[b], g["matches1"][0][perm], err_msg=f"pair {b}")
        np.testing.assert_array_equal(p0[b], g["prune0"][0], err_msg=f"pair {b}")
        np.testing.assert_array_equal(p1[b], g["prune1"][0][perm], err_msg=f"pair {b}")


def test_compile_replays_hip_graphs():
    """compile(): the first forward of a signature is captured into a hipGraph, later ones replay
    it on fresh inputs -- identical to eager forwards; a new shape captures a new graph."""
    from lightglue_amd.weights import synthetic_pair, synthetic_state_dict

    conf = {"filter_threshold": 0.1}
    sd = synthetic_state_dict(conf, seed=0)
    eager = _model(conf, sd, "auto")
    graphed = _model(conf, sd, "auto").compile()
    for M, N, seed in ((256, 230, 1), (256, 230, 2), (256, 230, 3), (192, 200, 4)):
        data = _gpu_data(synthetic_pair(B=2, M=M, N=N, seed=seed))
        with torch.no_grad():
            ref = eager(data)
            got = graphed(data)
        torch.cuda.synchronize()
        for k in ("matches0", "matches1", "matching_scores0", "matching_scores1", "log_assignment"):
            assert torch.equal(got[k], ref[k]), (k, M, N, seed)
    assert len(graphed._graphs) == 2


def test_compile_graphs_follow_conf_and_weight_changes():
    """a replayed graph must never run against stale weights, a stale config or device
    memory a later upload freed.  Capture two signatures, then (1) change the config, (2) write a
    parameter through p.data + reload_weights(), (3) change a weight in place and run the OTHER
    signature first (its eager forward re-uploads the weights): every replay equals a fresh eager
    model with the same config and weights."""
    from lightglue_amd.weights import synthetic_pair, synthetic_state_dict

    conf = {"filter_threshold": 0.1}
    sd = synthetic_state_dict(conf, seed=0)
    graphed = _model(conf, sd, "auto").compile()
    da = _gpu_data(synthetic_pair(B=2, M=256, N=230, seed=1))
    db = _gpu_data(synthetic_pair(B=1, M=192, N=200, seed=2))

    def expect(model_conf, state, data, got):
        ref = _model(model_conf, {k: v.detach().cpu().numpy() for k, v in state.items()}, "auto")
        with torch.no_grad():
            r = ref(data)
        torch.cuda.synchronize()
        for k in ("matches0", "matches1", "matching_scores0", "matching_scores1", "log_assignment"):
            assert torch.equal(got[k], r[k]), k

    with torch.no_grad():
        graphed(da)
        graphed(db)
        # (1) config change: the handle is recreated, both graphs are stale
        graphed.conf.filter_threshold = 0.3
        got = {k: v.clone() for k, v in graphed(da).items() if torch.is_tensor(v)}
        expect({"filter_threshold": 0.3}, graphed.state_dict(), da, got)
        # (2) a write the version counter cannot see, then reload_weights()
        graphed.log_assignment[-1].final_proj.weight.data.mul_(0.5)
        graphed.reload_weights()
        got = {k: v.clone() for k, v in graphed(da).items() if torch.is_tensor(v)}
        expect({"filter_threshold": 0.3}, graphed.state_dict(), da, got)
        # (3) an in-place change, picked up by the other signature first
        graphed.log_assignment[-1].matchability.bias.add_(0.5)
        graphed(db)
        got = {k: v.clone() for k, v in graphed(da).items() if torch.is_tensor(v)}
        expect({"filter_threshold": 0.3}, graphed.state_dict(), da, got)


@pytest.mark.parametrize("prune", [False, True])
def test_deep_config_matches_oracle(prune):
    """a 32-layer model needs more range-table slots than the round-2 fixed table had
    (9 L + 2 with pruning); the table is sized from n_layers, so a deep forward matches the oracle
    (indices exact outside fp64 near-ties, scores within 1e-4)."""
    import oracle
    from lightglue_amd.weights import synthetic_pair, synthetic_state_dict

    conf = {"filter_threshold": 0.1, "n_layers": 32}
    if prune:
        conf.update(width_confidence=0.99, depth_confidence=-1)
    sd = synthetic_state_dict(conf, seed=0)
    data = synthetic_pair(B=1, M=96, N=80, seed=5)
    ref = oracle.lightglue_forward(sd, data, conf)
    ref64 = oracle.lightglue_forward(sd, data, conf, dtype=torch.float64)
    model = _model(conf, sd)
    with torch.no_grad():
        pred = model(_gpu_data(data))
    m0, m1 = pred["matches0"].cpu().numpy(), pred["matches1"].cpu().numpy()
    r0, r1 = ref["matches0"].numpy(), ref["matches1"].numpy()
    ok0, ok1 = np.ones_like(m0, dtype=bool), np.ones_like(m1, dtype=bool)
    la = ref64["log_assignment"][:, :-1, :-1]
    if la.shape[1:] == (m0.shape[1], m1.shape[1]):  # every point kept: fp64 margins per row / column
        t0, t1 = la.topk(2, dim=2).values, la.topk(2, dim=1).values
        ok0 = (t0[..., 0] - t0[..., 1] >= NEAR_TIE).numpy()
        ok1 = (t1[:, 0] - t1[:, 1] >= NEAR_TIE).numpy()
    np.testing.assert_array_equal(m0[ok0], r0[ok0])
    np.testing.assert_array_equal(m1[ok1], r1[ok1])
    if prune:
        np.testing.assert_array_equal(pred["prune0"].cpu().numpy(), ref["prune0"].numpy())
        np.testing.assert_array_equal(pred["prune1"].cpu().numpy(), ref["prune1"].numpy())
    same = ok0 & ((m0 > -1) == (r0 > -1))
    np.testing.assert_allclose(pred["matching_scores0"].cpu().numpy()[same], ref["matching_scores0"].numpy()[same],
                               atol=SCORE_TOL)


def test_profile_flops_count_kept_points_only():
    """lg_profile_read on a pruned forward: each attention launch's algorithmic flops come from the
    per-pair kept counts at launch time (stopped pairs excluded), so they equal what the prune
    counts imply -- point i of a pair takes part in layers l < prune[i] (lightglue.py:540)."""
    g = load("prune_depth_width_n512")
    conf, sd, data = case_inputs(g["meta"])
    from lightglue_amd.weights import synthetic_pair

    pkw = dict(g["meta"]["pair"])
    pairs = []
    for s_ in (22, 5):
        pkw["seed"] = s_
        pairs.append(synthetic_pair(**pkw))
    model = _model(conf, sd)
    batch = _gpu_data(_stack_pairs(pairs))
    with torch.no_grad():
        model(batch)
        model.profile_enable(True, only=("attention",))
        pred = model(batch)
        ms, n, fl, _ = model.profile_read("attention")
        model.profile_enable(False)
    p0, p1 = pred["prune0"].cpu().numpy(), pred["prune1"].cpu().numpy()
    want = 0.0
    for b in range(2):
        for li in range(int(pred["stop_layer"][b]) + 1):
            m_, n_ = float((p0[b] > li).sum()), float((p1[b] > li).sum())
            want += 4.0 * 256 * (m_ * m_ + n_ * n_) + 6.0 * 256 * m_ * n_
    assert n >= 2 * int(pred["stop_layer"].max() + 1)
    assert fl == pytest.approx(want, rel=1e-12)
