"""The north star's accuracy clause -- HPatches ``H_error_dlt`` AUC within +-0.002 of the reference
-- on synthetic HPatches-style pairs (HPatches images and trained weights are not available here).

Pairs (16 x 1024 points, and the bench's 32 x 2048): 640 x 480 views related by a random
homography (corners moved up to 64 px, the HPatches viewpoint range), 0.5 px keypoint noise, 20 % of the second view's points replaced by unrelated
points and descriptors, the second view shuffled; descriptors unit vectors, the second view's a
noisy copy.  Weights: the seeded random trunk with each block's ffn.3 scaled by 0.03 (the layers
move the descriptors a little, so the transformer matters to the result) and assignment heads that
score descriptor similarity (final_proj = 20 I, matchability bias +5).  Each pair's matches and
scores go through the reference's HPatches evaluation (eval/utils.py:176-196: weighted DLT on the
matches, corner error; utils/tools.py:137-149: AUC at 1 / 3 / 5 px), once from the HIP forward and
once from the float32 CPU oracle (oracle/lightglue_ref.py), and the AUCs must agree within 0.002."""
import json

import numpy as np
import pytest
import torch

import lgamd  # noqa: F401

pytestmark = pytest.mark.gpu

FFN_SCALE, ALPHA, MATCHABLE = 0.03, 20.0, 5.0
AUC_TOL = 0.002


def crafted_state_dict(conf):
    from lightglue_amd.weights import synthetic_state_dict

    sd = synthetic_state_dict(conf, seed=0)
    for i in range(int(conf.get("n_layers", 9))):
        for blk in ("self_attn", "cross_attn"):
            for p in ("weight", "bias"):
                k = f"transformers.{i}.{blk}.ffn.3.{p}"
                sd[k] = (sd[k] * FFN_SCALE).astype(np.float32)
        sd[f"log_assignment.{i}.final_proj.weight"] = (ALPHA * np.eye(256)).astype(np.float32)
        sd[f"log_assignment.{i}.final_proj.bias"] = np.zeros(256, np.float32)
        sd[f"log_assignment.{i}.matchability.weight"] = np.zeros((1, 256), np.float32)
        sd[f"log_assignment.{i}.matchability.bias"] = np.full(1, MATCHABLE, np.float32)
    return sd


def homography_pairs(B, N, seed, W=640.0, H=480.0, outliers=0.2, px_noise=0.5, desc_noise=0.2):
    rng = np.random.Generator(np.random.PCG64(seed))
    keys = ("keypoints0", "keypoints1", "descriptors0", "descriptors1", "image_size0", "image_size1")
    out = {k: [] for k in keys}
    Hs = []
    for _ in range(B):
        c = np.array([[0, 0], [W, 0], [W, H], [0, H]], np.float64)
        c1 = c + rng.uniform(-64, 64, c.shape)
        A = []
        for (x, y), (u, v) in zip(c, c1):
            A.append([x, y, 1, 0, 0, 0, -u * x, -u * y, -u])
            A.append([0, 0, 0, x, y, 1, -v * x, -v * y, -v])
        h = np.linalg.svd(np.array(A))[2][-1].reshape(3, 3)
        h /= h[2, 2]
        k0 = rng.uniform([0, 0], [W, H], (N, 2))
        k1 = np.c_[k0, np.ones(N)] @ h.T
        k1 = k1[:, :2] / k1[:, 2:] + rng.normal(0, px_noise, (N, 2))
        d0 = rng.normal(size=(N, 256))
        d0 /= np.linalg.norm(d0, axis=1, keepdims=True)
        d1 = d0 + desc_noise * rng.normal(size=(N, 256)) / 16.0
        d1 /= np.linalg.norm(d1, axis=1, keepdims=True)
        bad = rng.random(N) < outliers
        k1[bad] = rng.uniform([0, 0], [W, H], (int(bad.sum()), 2))
        r = rng.normal(size=(int(bad.sum()), 256))
        d1[bad] = r / np.linalg.norm(r, axis=1, keepdims=True)
        perm = rng.permutation(N)
        for k, v in zip(keys, (k0, k1[perm], d0, d1[perm], [W, H], [W, H])):
            out[k].append(v)
        Hs.append(h)
    return {k: np.asarray(v, np.float32) for k, v in out.items()}, np.asarray(Hs)


def dlt_errors(pred, data, Hs):
    from lightglue_amd import hpatches_metrics as hm

    errs = []
    for b in range(len(Hs)):
        d = {"H_0to1": torch.from_numpy(Hs[b]),
             "view0": {"image_size": torch.tensor(data["image_size0"][b], dtype=torch.float64)}}
        p = {"keypoints0": torch.from_numpy(data["keypoints0"][b]).double(),
             "keypoints1": torch.from_numpy(data["keypoints1"][b]).double(),
             "matches0": pred["matches0"][b].cpu(), "matching_scores0": pred["matching_scores0"][b].cpu().double()}
        errs.append(hm.eval_homography_dlt(d, p)["H_error_dlt"])
    return np.asarray(errs)


@pytest.mark.parametrize("B,N,seed", [(16, 1024, 2), (32, 2048, 3)], ids=["16x1024", "configs2_32x2048"])
def test_synthetic_hpatches_auc_equals_the_oracle(B, N, seed):
    import oracle
    from lightglue_amd import LightGlue
    from lightglue_amd import hpatches_metrics as hm

    conf = {"filter_threshold": 0.1}
    sd = crafted_state_dict(conf)
    data, Hs = homography_pairs(B, N, seed=seed)
    dev = torch.device("cuda", 0)
    model = LightGlue(conf).eval().to(dev)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
    feed = {k: torch.from_numpy(v).to(dev) for k, v in data.items() if not k.startswith("image_size")}
    feed["view0"] = {"image_size": torch.from_numpy(data["image_size0"]).to(dev)}
    feed["view1"] = {"image_size": torch.from_numpy(data["image_size1"]).to(dev)}
    with torch.no_grad():
        hip = model(feed)
    ref = oracle.lightglue_forward(sd, data, conf)
    e_hip, e_ref = dlt_errors(hip, data, Hs), dlt_errors(ref, data, Hs)
    a_hip, a_ref = hm.summarize_dlt(list(e_hip)), hm.summarize_dlt(list(e_ref))
    print(json.dumps({"auc_hip": a_hip, "auc_oracle": a_ref, "max_pair_error_diff_px": float(np.abs(e_hip - e_ref).max()),
                      "pairs": len(Hs), "npts": N}))
    for k in a_ref:
        assert abs(a_hip[k] - a_ref[k]) <= AUC_TOL, (k, a_hip[k], a_ref[k])
    # a discriminating case: sub-pixel to pixel errors, so the AUCs move with the matches
    assert 0.2 < a_ref["H_error_dlt@1px"] < 0.95 and a_ref["H_error_dlt@5px"] > 0.8, a_ref
    np.testing.assert_array_equal(hip["matches0"].cpu().numpy(), ref["matches0"].numpy())
