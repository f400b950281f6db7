#!/usr/bin/env python3
"""Golden vectors for the SuperPoint extractor, made by running the REAL reference here.

Run from the repo root (needs ``/root/reference``, which does not exist on the GPU box)::

    python tests/golden/make_superpoint_golden.py

Harness only (nothing here ships):

* an ``omegaconf`` stand-in (``OmegaConf.create/merge/set_struct/set_readonly``, attribute
  dicts) and synthetic package objects whose ``__path__`` points into ``/root/reference``, so the
  REAL ``gluefactory.models.base_model.BaseModel`` and ``gluefactory.models.utils.misc`` load
  without the training stack;
* ``torch.hub.load_state_dict_from_url`` (called by ``SuperPoint._init``, ``superpoint.py:198-200``)
  is replaced by a function returning the recipe weights
  (``lightglue_amd.sp_weights.superpoint_state_dict``): the trained checkpoint is a download;
* ``SuperPoint(conf).eval()(data)`` runs on the recipe images (``synthetic_images``); the outputs
  go to ``tests/golden/<case>.npz``.  Inputs and weights are regenerated from the recipe in the
  tests (their SHA-256 is stored).  Each case also stores, per image, the gap between the k-th and
  (k+1)-th best post-NMS candidate score (``kth_gap``) so a test can tell a selection that fp32
  rounding could flip from a real mismatch.

With B > 1 the reference's sparse path returns only with ``force_num_keypoints`` (otherwise
``desc`` is a list and ``desc.transpose`` raises, ``superpoint.py:330-344``), so the B = 2 case sets
it with a keypoint budget every image fills (no random padding is drawn).
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
from lightglue_amd.sp_weights import superpoint_state_dict, synthetic_images  # noqa: E402
from make_golden import _ADict, _merge  # noqa: E402

CASES = {
    # name: (B, C, H, W, conf, image_size or None, img_seed, w_seed, store_dense)
    "sp_gray_b1_120x160": (1, 1, 120, 160, {}, None, 11, 1, True),
    "sp_rgb_b2_96x128_k100": (2, 3, 96, 128, {"max_num_keypoints": 100, "force_num_keypoints": True}, [[120.0, 90.0], [128.0, 96.0]], 12, 2, True),
    "sp_odd_b1_100x132_fix": (1, 1, 100, 132, {"max_num_keypoints": 150, "legacy_sampling": False}, None, 13, 3, True),
    "sp_refine_b1_96x96": (1, 1, 96, 96, {"max_num_keypoints": 100, "refinement_radius": 2, "nms_radius": 3}, None, 14, 4,
                           False),
    "sp_dense_b2_64x80": (2, 1, 64, 80, {"sparse_outputs": False}, None, 15, 5, False),
    "sp_b1_480x640_k1024": (1, 1, 480, 640, {"max_num_keypoints": 1024}, None, 16, 6, False),
}


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
    return importlib.import_module("gluefactory_nonfree.superpoint")


def sha(arrs):
    h = hashlib.sha256()
    for k in sorted(arrs):
        h.update(k.encode())
        h.update(np.ascontiguousarray(arrs[k]).tobytes())
    return h.hexdigest()


def run_case(sp_mod, name, spec):
    B, C, H, W, conf, isz, img_seed, w_seed, store_dense = spec
    sd = superpoint_state_dict(conf, seed=w_seed)
    image = synthetic_images(B, C, H, W, seed=img_seed)
    real_hub = torch.hub.load_state_dict_from_url
    torch.hub.load_state_dict_from_url = lambda *a, **k: {n: torch.from_numpy(v.copy()) for n, v in sd.items()}
    try:
        model = sp_mod.SuperPoint(dict(conf)).eval()
    finally:
        torch.hub.load_state_dict_from_url = real_hub
    data = {"image": torch.from_numpy(image)}
    if isz is not None:
        data["image_size"] = torch.tensor(isz, dtype=torch.float32)
    with torch.no_grad():
        pred = model(data)
        dense_model = sp_mod.SuperPoint.__new__(sp_mod.SuperPoint)
        dense_model.__dict__.update(model.__dict__)
        dense_model.conf = _merge(model.conf, {"sparse_outputs": False})
        dense = dense_model(data)
    out = {f"out_{k}": v.numpy() for k, v in pred.items()}
    if store_dense and "out_dense_keypoint_scores" not in out:
        out["dense_keypoint_scores"] = dense["keypoint_scores"].numpy()
        out["dense_descriptors"] = dense["descriptors"].numpy()
    meta = {"B": B, "C": C, "H": H, "W": W, "conf": conf, "image_size": isz, "img_seed": img_seed, "w_seed": w_seed,
            "inputs_sha256": sha({"image": image}), "weights_sha256": sha(sd)}
    if conf.get("sparse_outputs", True):
        # selection margin at the top-k boundary (post-NMS, borders removed), per image
        s = sp_mod.simple_nms(dense["keypoint_scores"].clone(), model.conf.nms_radius)
        r = model.conf.remove_borders
        s[:, :r] = -1
        s[:, :, :r] = -1
        if isz is not None:
            for i in range(B):
                w, h = isz[i]
                s[i, int(h) - r:] = -1
                s[i, :, int(w) - r:] = -1
        else:
            s[:, -r:] = -1
            s[:, :, -r:] = -1
        k = conf.get("max_num_keypoints", -1)
        gaps = []
        for i in range(B):
            c = s[i][s[i] > model.conf.detection_threshold]
            if 0 < k < len(c):
                v = torch.sort(c, descending=True).values
                gaps.append(float(v[k - 1] - v[k]))
            else:
                gaps.append(float("inf"))
        meta["kth_gap"] = gaps
        meta["counts"] = [int((s[i] > model.conf.detection_threshold).sum()) for i in range(B)]
    out["meta_json"] = np.array(json.dumps(meta))
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **out)
    print(name, {k: v.shape for k, v in out.items() if k != "meta_json"}, meta.get("counts"), meta.get("kth_gap"))


def main():
    sp_mod = install_shim()
    only = sys.argv[1:]
    for name, spec in CASES.items():
        if not only or name in only:
            run_case(sp_mod, name, spec)


if __name__ == "__main__":
    main()
