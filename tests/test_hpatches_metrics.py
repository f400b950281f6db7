"""HPatches DLT metric restatement (lightglue_amd.hpatches_metrics) — CPU.

cal_error_auc is pinned against the reference's own function (golden vectors made by
tests/golden/make_metric_golden.py).  find_homography_dlt restates kornia's weighted DLT; kornia is
not installed, so it is pinned by properties: exact recovery from noise-free correspondences,
zero-weight outliers ignored, invariance to correspondence order and to a common weight scale.
"""
import json
import os

import numpy as np
import pytest
import torch

import lgamd  # noqa: F401
from lightglue_amd import hpatches_metrics as hm

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "metric_auc.json")


def random_homography(g, perturb=0.2):
    H = torch.eye(3, dtype=torch.float64) + perturb * torch.randn(3, 3, generator=g, dtype=torch.float64) * torch.tensor(
        [[1, 1, 100], [1, 1, 100], [1e-3, 1e-3, 0]], dtype=torch.float64)
    return H / H[2, 2]


def warp(H, pts):
    return hm.from_homogeneous(hm.to_homogeneous(pts) @ H.transpose(-1, -2))


def test_cal_error_auc_matches_reference_golden():
    g = json.load(open(GOLDEN))
    for name, c in g["cases"].items():
        got = hm.cal_error_auc(np.array(c["errors"]), g["thresholds"])
        np.testing.assert_allclose(got, c["auc"], atol=0, rtol=0, err_msg=name)


def test_summarize_dlt_keys():
    s = hm.summarize_dlt([0.5, 2.0, 10.0])
    assert set(s) == {"H_error_dlt@1px", "H_error_dlt@3px", "H_error_dlt@5px"}
    assert all(np.isnan(v) for v in hm.summarize_dlt([]).values())


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_dlt_recovers_exact_homography(seed):
    g = torch.Generator().manual_seed(seed)
    H = random_homography(g)
    p0 = torch.rand(1, 50, 2, generator=g, dtype=torch.float64) * 640
    p1 = warp(H, p0)
    Hd = hm.find_homography_dlt(p0, p1, torch.rand(1, 50, generator=g, dtype=torch.float64) + 0.1)[0]
    np.testing.assert_allclose(Hd.numpy(), H.numpy(), rtol=1e-7, atol=1e-9)
    err = hm.homography_corner_error(Hd, H, torch.tensor([640.0, 480.0], dtype=torch.float64))
    assert err.item() < 1e-6


def test_dlt_zero_weight_outliers_are_ignored():
    g = torch.Generator().manual_seed(3)
    H = random_homography(g)
    p0 = torch.rand(1, 40, 2, generator=g, dtype=torch.float64) * 640
    p1 = warp(H, p0)
    p1[0, :8] += 50.0  # gross outliers
    w = torch.ones(1, 40, dtype=torch.float64)
    w[0, :8] = 0.0
    Hd = hm.find_homography_dlt(p0, p1, w)[0]
    assert hm.homography_corner_error(Hd, H, torch.tensor([640.0, 480.0], dtype=torch.float64)).item() < 1e-6
    Hu = hm.find_homography_dlt(p0, p1, torch.ones_like(w))[0]
    assert hm.homography_corner_error(Hu, H, torch.tensor([640.0, 480.0], dtype=torch.float64)).item() > 1.0


def test_dlt_invariances():
    g = torch.Generator().manual_seed(4)
    H = random_homography(g)
    p0 = torch.rand(1, 30, 2, generator=g, dtype=torch.float64) * 640
    p1 = warp(H, p0) + 0.5 * torch.randn(1, 30, 2, generator=g, dtype=torch.float64)
    w = torch.rand(1, 30, generator=g, dtype=torch.float64) + 0.1
    Ha = hm.find_homography_dlt(p0, p1, w)
    perm = torch.randperm(30, generator=g)
    Hb = hm.find_homography_dlt(p0[:, perm], p1[:, perm], w[:, perm])
    Hc = hm.find_homography_dlt(p0, p1, 7.0 * w)
    np.testing.assert_allclose(Hb.numpy(), Ha.numpy(), rtol=1e-8, atol=1e-10)
    np.testing.assert_allclose(Hc.numpy(), Ha.numpy(), rtol=1e-8, atol=1e-10)


def test_corner_error_known_translation():
    T = torch.eye(3, dtype=torch.float64)
    T[0, 2], T[1, 2] = 3.0, 4.0
    err = hm.homography_corner_error(T, torch.eye(3, dtype=torch.float64), torch.tensor([640.0, 480.0], dtype=torch.float64))
    assert err.item() == pytest.approx(5.0)


def test_eval_homography_dlt_pipeline():
    g = torch.Generator().manual_seed(5)
    H = random_homography(g)
    k0 = torch.rand(60, 2, generator=g, dtype=torch.float64) * 640
    k1 = warp(H, k0)
    m0 = torch.arange(60)
    m0[::7] = -1  # unmatched keypoints are dropped
    data = {"H_0to1": H, "view0": {"image_size": torch.tensor([640.0, 480.0], dtype=torch.float64)}}
    pred = {"keypoints0": k0, "keypoints1": k1, "matches0": m0, "matching_scores0": torch.rand(60, generator=g, dtype=torch.float64)}
    assert hm.eval_homography_dlt(data, pred)["H_error_dlt"] < 1e-6
    # no matches: the DLT asserts and the reference substitutes H = inf everywhere; its corner
    # error then evaluates to nan (inf/inf in from_homogeneous), which we reproduce
    pred["matches0"] = torch.full((60,), -1)
    assert np.isnan(hm.eval_homography_dlt(data, pred)["H_error_dlt"])


def test_homography_corner_error_matches_reference_golden():
    """Pinned against the reference's own homography_corner_error (geometry/homography.py:336-342)
    on committed vectors (tests/golden/make_metric_golden.py): single and batched homographies,
    float64 and float32."""
    g = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "metric_corner_error.json")))
    for i, c in enumerate(g["cases"]):
        dt = getattr(torch, c["dtype"])
        T = torch.tensor(c["T"], dtype=torch.float64).to(dt)
        T_gt = torch.tensor(c["T_gt"], dtype=torch.float64).to(dt)
        size = torch.tensor(c["image_size"], dtype=torch.float64).to(dt)
        got = hm.homography_corner_error(T, T_gt, size).double().reshape(-1).numpy()
        tol = 1e-12 if dt == torch.float64 else 1e-6
        np.testing.assert_allclose(got, c["error"], rtol=tol, atol=tol, err_msg=f"case {i}")
