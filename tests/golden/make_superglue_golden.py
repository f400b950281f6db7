#!/usr/bin/env python3
"""Golden vectors for the SuperGlue matcher (GNN + Sinkhorn) and the NLL losses, made by running
the REAL reference here.

Run from the repo root (needs ``/root/reference``, which does not exist on the GPU box)::

    python tests/golden/make_superglue_golden.py

Harness only (nothing here ships):

* the ``omegaconf`` stand-in and package objects of ``make_superpoint_golden.py``, so the REAL
  ``gluefactory.models.base_model.BaseModel`` loads without the training stack;
* ``SuperGlue({... "weights": None})`` (the trained checkpoint is a download, ``superglue.py:
  248-251``), then ``load_state_dict(strict=True)`` of the recipe weights
  (``lightglue_amd.sg_weights.superglue_state_dict``);
* eval-mode ``model(data)`` on ``lightglue_amd.weights.synthetic_pair`` keypoints/descriptors and
  ``sg_weights.synthetic_scores``; a forward hook on ``final_proj`` also records the GNN output;
* ``model.loss(pred, data)`` (``superglue.py:309-339``) and ``losses.NLLLoss`` (``models/utils/
  losses.py``) on a seeded ground truth.

Inputs and weights are regenerated from the recipe in the tests (their SHA-256 is stored).  Each
case records, per row and per column of the assignment, the gap between the best and the
second-best log-assignment value and the distance of exp(max) from the filter threshold, so a
test can tell a decision fp32 rounding could flip from a real mismatch.
"""
import hashlib
import importlib
import json
import os
import sys
import types

import numpy as np
import torch

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)
import lgamd  # noqa: E402,F401
from lightglue_amd.sg_weights import superglue_state_dict, synthetic_scores  # noqa: E402
from lightglue_amd.weights import synthetic_pair  # noqa: E402
from make_golden import _ADict, _merge  # noqa: E402

CASES = {
    # name: (B, M, N, conf, image_size (w, h) per pair or None -> image shape (H, W), seed, w_seed)
    "sg_b1_n128": (1, 128, 128, {}, [[640.0, 480.0]], 21, 1),
    "sg_b2_m96_n160": (2, 96, 160, {}, [[640.0, 480.0], [640.0, 640.0]], 22, 2),
    "sg_noscore_l4_b1_n200": (1, 200, 200, {"use_scores": False, "GNN_layers": ["self", "cross"] * 2,
                                             "filter_threshold": 0.1, "num_sinkhorn_iterations": 30}, None, 23, 3),
    "sg_b1_m300_n257": (1, 300, 257, {"GNN_layers": ["cross", "self", "self"]}, [[700.0, 500.0]], 24, 4),
}
IMAGE_HW = (480, 640)


def install_shim():
    om = types.ModuleType("omegaconf")

    class OmegaConf:
        merge = staticmethod(_merge)
        create = staticmethod(lambda d=None: _merge(d or {}))
        to_container = staticmethod(lambda d: dict(d))
        set_struct = staticmethod(lambda *a, **k: None)
        set_readonly = staticmethod(lambda *a, **k: None)

    om.OmegaConf = OmegaConf
    om.DictConfig = _ADict
    sys.modules["omegaconf"] = om
    for name, path in [
        ("gluefactory", "gluefactory"),
        ("gluefactory.models", "gluefactory/models"),
        ("gluefactory.models.utils", "gluefactory/models/utils"),
        ("gluefactory_nonfree", "gluefactory_nonfree"),
    ]:
        m = types.ModuleType(name)
        m.__path__ = [os.path.join(REF, path)]
        sys.modules[name] = m
    if REF not in sys.path:
        sys.path.insert(0, REF)
    return importlib.import_module("gluefactory_nonfree.superglue"), importlib.import_module("gluefactory.models.utils.losses")


def sha(arrs):
    h = hashlib.sha256()
    for k in sorted(arrs):
        h.update(k.encode())
        h.update(np.ascontiguousarray(arrs[k]).tobytes())
    return h.hexdigest()


def case_inputs(B, M, N, conf, isz, seed):
    """The recipe inputs of a case (also used by the tests)."""
    p = synthetic_pair(B, M, N, seed=seed, width=IMAGE_HW[1], height=IMAGE_HW[0])
    data = {
        "keypoints0": p["keypoints0"], "keypoints1": p["keypoints1"],
        "descriptors0": p["descriptors0"], "descriptors1": p["descriptors1"],
        "keypoint_scores0": synthetic_scores(B, M, seed=seed + 100),
        "keypoint_scores1": synthetic_scores(B, N, seed=seed + 200),
    }
    if isz is not None:
        data["image_size"] = np.asarray(isz, np.float32)
    return data


def ground_truth(B, M, N, seed):
    """Seeded one-to-one ground truth: gt_matches0/1 (int64, -1 unmatched), gt_assignment (bool)."""
    rng = np.random.Generator(np.random.PCG64(seed + 1000))
    m0 = -np.ones((B, M), np.int64)
    m1 = -np.ones((B, N), np.int64)
    a = np.zeros((B, M, N), bool)
    for b in range(B):
        k = min(M, N) * 2 // 3
        i = rng.permutation(M)[:k]
        j = rng.permutation(N)[:k]
        m0[b, i] = j
        m1[b, j] = i
        a[b, i, j] = True
    return {"gt_matches0": m0, "gt_matches1": m1, "gt_assignment": a}


def margins(la, th):
    """Per row / column: best - second best of la[:-1, :-1], and |exp(best) - th|."""
    s = la[:, :-1, :-1].astype(np.float64)
    r = np.sort(s, axis=2)
    c = np.sort(s, axis=1)
    return {"row_gap": r[:, :, -1] - r[:, :, -2], "col_gap": c[:, -1, :] - c[:, -2, :],
            "row_th": np.abs(np.exp(r[:, :, -1]) - th), "col_th": np.abs(np.exp(c[:, -1, :]) - th)}


def run_case(sg_mod, loss_mod, name, spec):
    B, M, N, conf, isz, seed, w_seed = spec
    sd = superglue_state_dict(conf, seed=w_seed)
    model = sg_mod.SuperGlue({**conf, "weights": None}).eval()
    model.load_state_dict({k: torch.from_numpy(np.asarray(v).copy()) for k, v in sd.items()}, strict=True)
    inp = case_inputs(B, M, N, conf, isz, seed)
    gt = ground_truth(B, M, N, seed)
    t = {k: torch.from_numpy(v) for k, v in inp.items() if k != "image_size"}
    view = {"image": torch.zeros(B, 1, *IMAGE_HW)}
    if isz is not None:
        view["image_size"] = torch.from_numpy(inp["image_size"])
    data = {**t, "view0": view, "view1": dict(view)}
    seen = {}
    def keep(mod, a, o):  # returns None: the output is left alone
        seen[len(seen)] = a[0].detach().clone()

    hook = model.final_proj.register_forward_hook(keep)
    with torch.no_grad():
        pred = model(data)
        data_gt = {**data, **{k: torch.from_numpy(v) for k, v in gt.items()}}
        losses = model.loss(pred, data_gt)
        nll = loss_mod.NLLLoss({})
        try:  # losses.py:72 writes neg1 into [:, -1, :m]: only M == N runs
            nll_total, _, nll_metrics = nll({"log_assignment": pred["log_assignment"]}, data_gt)
            nll_error = None
        except RuntimeError as e:
            nll_total, nll_metrics, nll_error = None, {}, str(e)
    hook.remove()
    out = {f"out_{k}": v.numpy() for k, v in pred.items()}
    out["gnn_desc0"] = seen[0].numpy()  # [B, D, M] input of final_proj for view 0
    out["gnn_desc1"] = seen[1].numpy()
    for k, v in losses.items():
        out[f"sgloss_{k}"] = v.detach().numpy() if torch.is_tensor(v) else np.asarray(v)
    if nll_total is not None:
        out["nll_total"] = nll_total.numpy()
    for k, v in nll_metrics.items():
        out[f"nll_{k}"] = v.numpy()
    th = {**{"filter_threshold": 0.2}, **conf}["filter_threshold"]
    mg = margins(out["out_log_assignment"], th)
    meta = {"B": B, "M": M, "N": N, "conf": conf, "image_size": isz, "seed": seed, "w_seed": w_seed,
            "image_hw": list(IMAGE_HW), "inputs_sha256": sha(inp), "weights_sha256": sha(sd),
            "min_row_gap": float(mg["row_gap"].min()), "min_col_gap": float(mg["col_gap"].min()),
            "min_row_th": float(mg["row_th"].min()), "min_col_th": float(mg["col_th"].min()),
            "matches": int((out["out_matches0"] >= 0).sum()), "nll_error": nll_error}
    out.update({f"margin_{k}": v for k, v in mg.items()})
    out["meta_json"] = np.array(json.dumps(meta))
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **out)
    print(name, meta)


def main():
    sg_mod, loss_mod = install_shim()
    only = sys.argv[1:]
    for name, spec in CASES.items():
        if not only or name in only:
            run_case(sg_mod, loss_mod, name, spec)


if __name__ == "__main__":
    main()
