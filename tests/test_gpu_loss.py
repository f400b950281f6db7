"""LightGlue.loss (reference lightglue.py:614-663, losses.py:6-73, metrics.py) on the HIP library vs
golden vectors from the reference itself (tests/golden/make_loss_golden.py) -- needs an MI355X.

Bar: every NLL term within 1e-5 relative (the per-layer heads run from this library's own
fp32-accurate per-layer descriptors, ~1e-5 from the reference's); the token-confidence BCE counts
argmax agreements per point, so a near-tie row that flips moves it by ~1/M: it is held to 1e-5
relative plus 2 such flips; metrics exact up to fp32 rounding (they are ratios of match counts).
Also: the similarity output and ``assignment_head`` agree with the forward's own log assignment.
"""
import glob
import json
import os
import sys

import numpy as np
import pytest
import torch

import lgamd  # noqa: F401
from golden_util import HERE

sys.path.insert(0, HERE)
from make_superglue_golden import ground_truth  # noqa: E402

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _names():
    return sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(HERE, "loss_*.npz")))


def _case(name):
    from lightglue_amd import LightGlue
    from lightglue_amd.weights import synthetic_pair, synthetic_state_dict

    z = np.load(os.path.join(HERE, name + ".npz"))
    g = {k: z[k] for k in z.files if k != "meta_json"}
    meta = json.loads(str(z["meta_json"]))
    conf = meta["conf"]
    sd = synthetic_state_dict(conf, **meta["weights"])
    pair = synthetic_pair(**meta["pair"])
    B, M = meta["pair"]["B"], meta["pair"]["M"]
    gt = ground_truth(B, M, M, meta["gt_seed"])
    model = LightGlue(conf).to(DEV)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
    model.train(meta["training"])
    data = {k: torch.from_numpy(v).to(DEV) for k, v in pair.items() if not k.startswith("image_size")}
    data["view0"] = {"image_size": torch.from_numpy(pair["image_size0"]).to(DEV)}
    data["view1"] = {"image_size": torch.from_numpy(pair["image_size1"]).to(DEV)}
    data.update({k: torch.from_numpy(v).to(DEV) for k, v in gt.items()})
    return model, data, g, meta


@pytest.mark.parametrize("name", _names())
def test_lightglue_loss_matches_reference(name):
    model, data, g, meta = _case(name)
    with torch.no_grad():
        pred = model(data)
        losses, metrics = model.loss(pred, data)
    assert sorted(losses) == meta["loss_keys"] and sorted(metrics) == meta["metric_keys"]
    M = meta["pair"]["M"]
    for k, v in losses.items():
        got = np.asarray(v.detach().cpu().numpy() if torch.is_tensor(v) else v, np.float64)
        want = g[f"loss_{k}"]
        if k == "confidence":
            np.testing.assert_allclose(got, want, rtol=1e-5, atol=2.0 * np.log(2.0) / M, err_msg=k)
        elif k == "total" and meta["training"]:  # total includes the confidence term in training mode
            np.testing.assert_allclose(got, want, rtol=1e-5, atol=2.0 * np.log(2.0) / M, err_msg=k)
        else:
            np.testing.assert_allclose(got, want, rtol=1e-5, atol=1e-6, err_msg=k)
    np.testing.assert_array_equal(pred["matches0"].cpu().numpy(), g["matches0"])
    for k, v in metrics.items():
        np.testing.assert_allclose(v.cpu().numpy(), g[f"metric_{k}"], rtol=1e-5, atol=1e-7, err_msg=k)


def test_assignment_head_and_similarity_agree_with_forward():
    """assignment_head(-1) on the forward's final descriptors reproduces the forward's log
    assignment, and conf return_similarity returns the similarity that log assignment came from."""
    from lightglue_amd import LightGlue
    from lightglue_amd.weights import synthetic_pair, synthetic_state_dict

    conf = {"filter_threshold": 0.1, "return_similarity": True}
    sd = synthetic_state_dict(conf, seed=0)
    model = LightGlue(conf).eval().to(DEV)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
    p = synthetic_pair(B=2, M=200, N=176, seed=3)
    data = {k: torch.from_numpy(v).to(DEV) for k, v in p.items() if not k.startswith("image_size")}
    data["view0"] = {"image_size": torch.from_numpy(p["image_size0"]).to(DEV)}
    data["view1"] = {"image_size": torch.from_numpy(p["image_size1"]).to(DEV)}
    with torch.no_grad():
        pred = model(data)
        la, sim = model.assignment_head(-1, pred["ref_descriptors0"][:, 0], pred["ref_descriptors1"][:, 0])
    assert pred["similarity"].shape == (2, 200, 176)
    # both are fp32-accurate (|sim| ~ 1e2 with the sharpened recipe): relative agreement
    torch.testing.assert_close(sim, pred["similarity"], atol=1e-5, rtol=2e-6)
    torch.testing.assert_close(la, pred["log_assignment"], atol=1e-4, rtol=1e-5)
    # float64 check of the similarity itself: md = final_proj(x) / 256**0.25 (lightglue.py:308-311)
    W = model.log_assignment[-1].final_proj.weight.double()
    bb = model.log_assignment[-1].final_proj.bias.double()
    md0 = (pred["ref_descriptors0"][:, 0].double() @ W.T + bb) / 4.0
    md1 = (pred["ref_descriptors1"][:, 0].double() @ W.T + bb) / 4.0
    torch.testing.assert_close(pred["similarity"].double(), md0 @ md1.transpose(1, 2), atol=2e-5, rtol=1e-5)


@pytest.mark.parametrize("B", [1, 3])
def test_similarity_with_pruning_is_the_kept_block(B):
    """With width pruning and return_similarity, pred["similarity"] is sliced like log_assignment
    (b == 1: [1, M', N']; b > 1: per-pair list of [M_b, N_b], as the [M_b+1, N_b+1] log-assignment
    list) and holds md0 md1^T of the kept descriptors (ref_descriptors*, same compacted order) --
    ADVICE r3."""
    from golden_util import PRUNE_BIAS
    from lightglue_amd import LightGlue
    from lightglue_amd.weights import synthetic_pair, synthetic_state_dict

    conf = {"filter_threshold": 0.1, "width_confidence": 0.95, "return_similarity": True}
    sd = synthetic_state_dict(conf, seed=6)
    for i, v in enumerate(PRUNE_BIAS):
        sd[f"log_assignment.{i}.matchability.bias"][:] = v
    model = LightGlue(conf).eval().to(DEV)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
    p = synthetic_pair(B=B, M=512, N=480, seed=21)
    data = {k: torch.from_numpy(v).to(DEV) for k, v in p.items() if not k.startswith("image_size")}
    data["view0"] = {"image_size": torch.from_numpy(p["image_size0"]).to(DEV)}
    data["view1"] = {"image_size": torch.from_numpy(p["image_size1"]).to(DEV)}
    with torch.no_grad():
        pred = model(data)
    W = model.log_assignment[-1].final_proj.weight.double()
    bb = model.log_assignment[-1].final_proj.bias.double()
    sims = pred["similarity"] if B > 1 else [pred["similarity"]]
    las = pred["log_assignment"] if B > 1 else [pred["log_assignment"]]
    rd0s = pred["ref_descriptors0"] if B > 1 else [pred["ref_descriptors0"]]
    rd1s = pred["ref_descriptors1"] if B > 1 else [pred["ref_descriptors1"]]
    assert len(sims) == B
    pruned = False
    for sim, la, r0, r1 in zip(sims, las, rd0s, rd1s):
        k0, k1 = r0.shape[-2], r1.shape[-2]
        pruned |= k0 < 512 or k1 < 480
        assert tuple(sim.shape[-2:]) == (k0, k1) and tuple(la.shape[-2:]) == (k0 + 1, k1 + 1)
        assert sim.dim() == la.dim()
        md0 = (r0.reshape(k0, 256).double() @ W.T + bb) / 4.0
        md1 = (r1.reshape(k1, 256).double() @ W.T + bb) / 4.0
        torch.testing.assert_close(sim.reshape(k0, k1).double(), md0 @ md1.T, atol=2e-5, rtol=1e-5)
    assert pruned
