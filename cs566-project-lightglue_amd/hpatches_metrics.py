"""HPatches homography metric of the north-star (``H_error_dlt@{1,3,5}px`` AUC), restated.

SURVEY.md §8f rank 2: the evaluation that consumes the matcher's output on HPatches
(``gluefactory/eval/hpatches.py:143-149``):

    matches -> weighted DLT homography (kornia ``find_homography_dlt``, weights = matching scores)
            -> mean corner error against the ground-truth homography
            -> AUC of the per-pair errors at 1 / 3 / 5 px

Host-side evaluation code (numpy / torch-CPU or any torch device): it runs once per pair on a few
hundred matches, outside the measured hot path.  ``find_homography_dlt`` restates kornia's published
algorithm (kornia is not installed here, so its parity is pinned by properties in
``tests/test_hpatches_metrics.py`` -- exact recovery, weighting, invariances -- not by kornia's own
outputs); ``cal_error_auc`` is pinned against the reference's own function on committed vectors
(``tests/golden/metric_auc.json``).
"""
import numpy as np
import torch

AUC_THRESHOLDS = [1, 3, 5]  # eval/hpatches.py:143


def get_matches_scores(kpts0, kpts1, matches0, mscores0):
    """Matched keypoint pairs and their scores (eval/utils.py:21-27)."""
    m0 = matches0 > -1
    m1 = matches0[m0]
    return kpts0[m0], kpts1[m1], mscores0[m0]


def to_homogeneous(points):
    """(..., N) -> (..., N+1) (geometry/utils.py:5-19)."""
    return torch.cat([points, points.new_ones(points.shape[:-1] + (1,))], dim=-1)


def from_homogeneous(points, eps=0.0):
    """(..., N+1) -> (..., N) (geometry/utils.py:22-30)."""
    return points[..., :-1] / (points[..., -1:] + eps)


def normalize_points(points, eps=1e-8):
    """Hartley normalisation used by kornia's DLT: centre on the mean, scale so that the mean
    distance to the centre is sqrt(2).  points [B,N,2] -> (normalised points, transform [B,3,3])."""
    mean = points.mean(dim=1, keepdim=True)
    scale = (points - mean).norm(dim=-1).mean(dim=-1)
    scale = np.sqrt(2.0) / (scale + eps)
    z, o = torch.zeros_like(scale), torch.ones_like(scale)
    T = torch.stack([scale, z, -scale * mean[:, 0, 0], z, scale, -scale * mean[:, 0, 1], z, z, o], dim=-1)
    T = T.view(-1, 3, 3)
    return from_homogeneous(to_homogeneous(points) @ T.transpose(-1, -2)), T


def find_homography_dlt(points1, points2, weights=None):
    """Weighted DLT homography H with points2 ~ H points1 (kornia ``find_homography_dlt``,
    called at eval/utils.py:188 with the matching scores as weights).

    points1, points2: [B,N,2] (N >= 4), weights: [B,N] or None.  Returns [B,3,3] normalised so
    that H[2,2] = 1.  Each correspondence contributes the two rows of the DLT system, weighted by
    its score; the solution is the right singular vector of the smallest singular value of
    A^T W A, de-normalised.  Raises AssertionError for fewer than 4 points (the reference
    catches it and reports an infinite error)."""
    assert points1.shape == points2.shape and points1.dim() == 3 and points1.shape[-1] == 2
    assert points1.shape[1] >= 4, "need at least 4 correspondences"
    B, N = points1.shape[:2]
    p1, T1 = normalize_points(points1)
    p2, T2 = normalize_points(points2)
    x1, y1 = p1[..., 0:1], p1[..., 1:2]
    x2, y2 = p2[..., 0:1], p2[..., 1:2]
    one, zero = torch.ones_like(x1), torch.zeros_like(x1)
    ax = torch.cat([zero, zero, zero, -x1, -y1, -one, y2 * x1, y2 * y1, y2], dim=-1)
    ay = torch.cat([x1, y1, one, zero, zero, zero, -x2 * x1, -x2 * y1, -x2], dim=-1)
    A = torch.cat([ax, ay], dim=-1).reshape(B, 2 * N, 9)
    if weights is None:
        AtA = A.transpose(-2, -1) @ A
    else:
        w = weights.to(A).unsqueeze(-1).repeat(1, 1, 2).reshape(B, 2 * N, 1)
        AtA = A.transpose(-2, -1) @ (w * A)
    _, _, Vh = torch.linalg.svd(AtA)
    H = Vh[..., -1, :].reshape(B, 3, 3)
    H = torch.linalg.inv(T2) @ (H @ T1)
    return H / (H[..., -1:, -1:] + 1e-8)


def homography_corner_error(T, T_gt, image_size):
    """Mean distance of the four image corners warped by T and by T_gt
    (geometry/homography.py:336-342).  image_size = (W, H)."""
    image_size = torch.as_tensor(image_size, dtype=T.dtype, device=T.device)
    W, H = image_size[..., 0], image_size[..., 1]
    corners0 = torch.stack([torch.stack([0 * W, 0 * H]), torch.stack([W, 0 * H]), torch.stack([W, H]),
                            torch.stack([0 * W, H])]).to(T)
    c1_gt = from_homogeneous(to_homogeneous(corners0) @ T_gt.transpose(-1, -2))
    c1 = from_homogeneous(to_homogeneous(corners0) @ T.transpose(-1, -2))
    return torch.sqrt(((c1 - c1_gt) ** 2).sum(-1)).mean(-1)


def eval_homography_dlt(data, pred):
    """Per-pair ``H_error_dlt`` (eval/utils.py:176-196): data has ``H_0to1`` [3,3] and
    ``view0.image_size``; pred has keypoints0/1, matches0, matching_scores0 (one pair)."""
    H_gt = data["H_0to1"]
    pts0, pts1, scores = get_matches_scores(pred["keypoints0"], pred["keypoints1"], pred["matches0"],
                                            pred["matching_scores0"])
    scores = scores.to(pts0)
    try:
        squeeze = H_gt.ndim == 2
        if squeeze:
            pts0, pts1, scores = pts0[None], pts1[None], scores[None]
        h_dlt = find_homography_dlt(pts0, pts1, scores)
        if squeeze:
            h_dlt = h_dlt[0]
    except AssertionError:
        h_dlt = torch.full_like(H_gt, float("inf"))
    error = homography_corner_error(h_dlt, H_gt, data["view0"]["image_size"])
    return {"H_error_dlt": error.item()}


def cal_error_auc(errors, thresholds):
    """Area under the error-recall curve up to each threshold, / threshold, rounded to 4 decimals
    (utils/tools.py:137-149)."""
    errors = np.sort(np.asarray(errors, dtype=np.float64))
    recall = (np.arange(len(errors)) + 1) / len(errors)
    errors = np.r_[0.0, errors]
    recall = np.r_[0.0, recall]
    aucs = []
    for t in thresholds:
        last = np.searchsorted(errors, t)
        r = np.r_[recall[:last], recall[last - 1]]
        e = np.r_[errors[:last], t]
        aucs.append(np.round(np.trapezoid(r, x=e) / t, 4))
    return aucs


def summarize_dlt(errors, thresholds=AUC_THRESHOLDS):
    """``H_error_dlt@{t}px`` summaries of a list of per-pair errors (eval/hpatches.py:146-149)."""
    if len(errors) == 0:
        return {f"H_error_dlt@{t}px": float("nan") for t in thresholds}
    aucs = cal_error_auc(errors, thresholds)
    return {f"H_error_dlt@{t}px": float(a) for t, a in zip(thresholds, aucs)}
