#!/usr/bin/env python3
"""Generate golden vectors by running the REAL reference in the build container.

Run from the repo root (needs ``/root/reference``, which does not exist on the GPU box)::

    python tests/golden/make_golden.py

What it does (harness only; nothing here ships):

* registers a minimal ``omegaconf`` stand-in (``OmegaConf.merge/create`` returning an
  attribute dict) and synthetic ``gluefactory`` / ``gluefactory.models`` /
  ``gluefactory.models.matchers`` / ``gluefactory.models.utils`` package objects whose
  ``__path__`` points into ``/root/reference`` so their training-stack ``__init__`` files are
  skipped;
* imports ``gluefactory.models.matchers.lightglue`` and ``gluefactory_nonfree.superglue``;
* builds ``LightGlue(conf)``, loads the deterministic recipe weights
  (``lightglue_amd.weights.synthetic_state_dict``) with ``strict=True``, runs the seeded
  ``synthetic_pair`` inputs through ``forward`` in eval mode, and writes the outputs into
  ``tests/golden/<case>.npz``.  Inputs and weights are NOT stored (they are regenerated from
  the recipe); their SHA-256 is, so recipe drift is detected.

Early-stop cases: the reference reads an undefined ``self.confidence_thresholds``
(``lightglue.py:592,604``); the harness sets that attribute on the instance to
``[confidence_threshold(i) for i in range(L)]``.  When the stop fires, the reference then fails
in ``torch.stack([])`` (``:572``) after the matches were computed; the harness swaps the
module's ``torch`` for a proxy whose ``stack`` returns an empty tensor for an empty list, and the
fixture omits ``ref_descriptors*``.
"""
import copy
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
import lgamd  # noqa: E402,F401
from lightglue_amd.weights import PRUNE2K_MATCH_BIAS, PRUNE2K_TOKEN_BIAS, synthetic_pair, synthetic_state_dict  # noqa: E402,F401


class _ADict(dict):
    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __setattr__(self, k, v):
        self[k] = v


def _merge(*cfgs):
    out = _ADict()
    for c in cfgs:
        for k, v in (c or {}).items():
            if isinstance(v, dict):
                out[k] = _merge(out.get(k, {}) if isinstance(out.get(k), dict) else {}, v)
            else:
                out[k] = v
    return out


def install_shim():
    om = types.ModuleType("omegaconf")

    class OmegaConf:
        merge = staticmethod(_merge)
        create = staticmethod(lambda d=None: _merge(d or {}))
        to_container = staticmethod(lambda d: dict(d))

    om.OmegaConf = OmegaConf
    om.DictConfig = _ADict
    sys.modules["omegaconf"] = om
    for name, path in [
        ("gluefactory", "gluefactory"),
        ("gluefactory.models", "gluefactory/models"),
        ("gluefactory.models.matchers", "gluefactory/models/matchers"),
        ("gluefactory.models.utils", "gluefactory/models/utils"),
        ("gluefactory_nonfree", "gluefactory_nonfree"),
    ]:
        m = types.ModuleType(name)
        m.__path__ = [os.path.join(REF, path)]
        sys.modules[name] = m
    bm = types.ModuleType("gluefactory.models.base_model")
    bm.BaseModel = torch.nn.Module
    sys.modules["gluefactory.models.base_model"] = bm
    if REF not in sys.path:
        sys.path.insert(0, REF)
    lg = importlib.import_module("gluefactory.models.matchers.lightglue")
    sg = importlib.import_module("gluefactory_nonfree.superglue")
    return lg, sg


class _TorchProxy:
    def __init__(self, real):
        self._real = real

    def __getattr__(self, k):
        return getattr(self._real, k)

    def stack(self, ts, *a, **kw):
        if len(ts) == 0:
            return self._real.empty(0)
        return self._real.stack(ts, *a, **kw)


def sha(arrs):
    h = hashlib.sha256()
    for k in sorted(arrs):
        h.update(k.encode())
        h.update(np.ascontiguousarray(arrs[k]).tobytes())
    return h.hexdigest()


# Per-layer matchability biases that prune ~10 % of the points per layer under the seed-6
# recipe (keep iff sigmoid(z) > 1 - 0.95, i.e. z > -2.944; offsets from the 10 % quantile of the
# unpruned logits).
PRUNE_BIAS = [-2.97, -2.32, -2.90, -2.29, -3.00, -2.80, -2.14, -2.37]

# configs[3]-shaped case (N = 2048, width = depth = 0.95): PRUNE2K_TOKEN_BIAS / PRUNE2K_MATCH_BIAS
# (lightglue_amd.weights, from tools/tune_prune_golden.py) -- layers 0..4 prune ~10 % of the points
# each, layer 5 stops early.

# name -> (conf overrides, pair kwargs, weight kwargs, weight overrides, store_full)
CASES = {
    "tiny_ragged_b2": ({"filter_threshold": 0.1}, dict(B=2, M=48, N=40, seed=11), dict(seed=0), {}, True),
    "tiny_b1_n64": ({"filter_threshold": 0.0}, dict(B=1, M=64, N=64, seed=12), dict(seed=3), {}, True),
    "n512": ({"filter_threshold": 0.1}, dict(B=1, M=512, seed=1), dict(seed=0), {}, False),
    "n1024": ({"filter_threshold": 0.1}, dict(B=1, M=1024, seed=1), dict(seed=0), {}, False),
    "n2048": ({"filter_threshold": 0.1}, dict(B=1, M=2048, seed=1), dict(seed=0), {}, False),
    "n300x257_b2": ({"filter_threshold": 0.1}, dict(B=2, M=300, N=257, seed=5), dict(seed=1), {}, False),
    "default_init_n256": ({"filter_threshold": 0.0}, dict(B=1, M=256, seed=7), dict(seed=2, sharpen=False), {}, False),
    "scale_ori_n128": ({"filter_threshold": 0.1, "add_scale_ori": True}, dict(B=1, M=128, N=96, seed=8), dict(seed=4), {}, False),
    "input_proj_n128": ({"filter_threshold": 0.1, "input_dim": 128}, dict(B=1, M=128, N=112, seed=9, dim=128), dict(seed=5), {}, False),
    "prune_width_n512": (
        {"filter_threshold": 0.1, "width_confidence": 0.95},
        dict(B=1, M=512, N=480, seed=21),
        dict(seed=6),
        {"matchability_bias": PRUNE_BIAS},
        False,
    ),
    "prune_depth_width_n512": (
        {"filter_threshold": 0.1, "width_confidence": 0.95, "depth_confidence": 0.95},
        dict(B=1, M=512, N=500, seed=22),
        dict(seed=6),
        {"matchability_bias": PRUNE_BIAS},
        False,
    ),
    "prune_depth_width_n2048": (
        {"filter_threshold": 0.1, "width_confidence": 0.95, "depth_confidence": 0.95},
        dict(B=1, M=2048, N=2048, seed=41),
        dict(seed=8),
        {"token_bias": PRUNE2K_TOKEN_BIAS, "matchability_bias": PRUNE2K_MATCH_BIAS},
        False,
    ),
    # configs[4]-shaped forward (N = 4096, the Sinkhorn config's matcher size)
    "n4096": ({"filter_threshold": 0.1}, dict(B=1, M=4096, seed=1), dict(seed=0), {}, False),
    # near-tie stress: unsharpened (default-init-like) weights and noisy view-1 descriptors, so
    # the assignment is nearly flat and many rows / columns have tiny top-1 / top-2 margins
    "unsharp_n1024": ({"filter_threshold": 0.0}, dict(B=1, M=1024, seed=51, noise=0.3), dict(seed=9, sharpen=False), {}, False),
    "unsharp_n2048": ({"filter_threshold": 0.0}, dict(B=1, M=2048, seed=52, noise=2.0), dict(seed=10, sharpen=False), {}, False),
    # near-tie stress, round 3: final_proj scaled down on unsharpened weights so the assignment is
    # flat and many rows / columns have fp64 top-1 / top-2 margins inside [1e-5, 1e-4]
    # (tools/.. probes: ~10 per 2048 rows+columns at x0.25, N = 1024)
    "tie_fp025_b4_n1024": ({"filter_threshold": 0.0}, dict(B=4, M=1024, seed=71, noise=0.3), dict(seed=9, sharpen=False),
                           {"final_proj_scale": 0.25}, False),
    "tie_fp005_b2_n2048": ({"filter_threshold": 0.0}, dict(B=2, M=2048, seed=72, noise=0.3), dict(seed=10, sharpen=False),
                           {"final_proj_scale": 0.05}, False),
    "tie_fp025_b32_n1024": ({"filter_threshold": 0.0}, dict(B=32, M=1024, seed=73, noise=0.3),
                            dict(seed=12, sharpen=False), {"final_proj_scale": 0.25}, False),
    # matching scores O(0.1-1) around the threshold (the sharpened recipe on a noisy view 1): the
    # 1e-4 score bar and the strict '>' threshold on values that matter
    "scores_mid_b2_n1024": ({"filter_threshold": 0.3}, dict(B=2, M=1024, seed=74, noise=0.6), dict(seed=9), {}, False),
    "early_stop_n256": (
        {"filter_threshold": 0.1, "depth_confidence": 0.9},
        dict(B=1, M=256, N=240, seed=23),
        dict(seed=7),
        {"token_bias_layer": (3, 6.0)},
        False,
    ),
}


def make_weights(conf, wkw, over):
    sd = synthetic_state_dict(conf, **wkw)
    L = conf.get("n_layers", 9)
    if "matchability_bias" in over:
        for i in range(L - 1):
            if over["matchability_bias"][i] is not None:
                sd[f"log_assignment.{i}.matchability.bias"][:] = over["matchability_bias"][i]
    if "token_bias" in over:
        for i in range(L - 1):
            if over["token_bias"][i] is not None:
                sd[f"token_confidence.{i}.token.0.bias"][:] = over["token_bias"][i]
    if "token_bias_layer" in over:
        li, val = over["token_bias_layer"]
        sd[f"token_confidence.{li}.token.0.bias"][:] = val
    if "final_proj_scale" in over:
        for k in sd:
            if k.startswith("log_assignment.") and ".final_proj." in k:
                sd[k] = (sd[k] * np.float32(over["final_proj_scale"])).astype(np.float32)
    return sd


def scale_ori(B, M, N, seed):
    rng = np.random.Generator(np.random.PCG64(seed + 1000))
    return {
        "scales0": (rng.random((B, M)) * 2).astype(np.float32),
        "oris0": (rng.random((B, M)) * 6.28 - 3.14).astype(np.float32),
        "scales1": (rng.random((B, N)) * 2).astype(np.float32),
        "oris1": (rng.random((B, N)) * 6.28 - 3.14).astype(np.float32),
    }


def run_case(lg_mod, name, spec):
    conf, pkw, wkw, over, full = spec
    sd = make_weights(conf, wkw, over)
    pair = synthetic_pair(**pkw)
    B, M = pkw["B"], pkw["M"]
    N = pkw.get("N", M)
    if conf.get("add_scale_ori"):
        pair.update(scale_ori(B, M, N, pkw["seed"]))
    model = lg_mod.LightGlue(dict(conf)).eval()
    L = model.conf.n_layers
    model.confidence_thresholds = [model.confidence_threshold(i) for i in range(L)]
    missing = model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
    assert not missing.missing_keys and not missing.unexpected_keys
    data = {k: torch.from_numpy(v) for k, v in pair.items() if not k.startswith("image_size")}
    data["view0"] = {"image_size": torch.from_numpy(pair["image_size0"])}
    data["view1"] = {"image_size": torch.from_numpy(pair["image_size1"])}
    layers = []
    hooks = [
        t.register_forward_hook(lambda mod, inp, out: layers.append((out[0].clone(), out[1].clone())))
        for t in model.transformers
    ]
    real_torch = lg_mod.torch
    lg_mod.torch = _TorchProxy(real_torch)
    try:
        with torch.no_grad():
            pred = model(data)
    finally:
        lg_mod.torch = real_torch
        for h in hooks:
            h.remove()
    out = {
        "matches0": pred["matches0"].numpy(),
        "matches1": pred["matches1"].numpy(),
        "matching_scores0": pred["matching_scores0"].numpy(),
        "matching_scores1": pred["matching_scores1"].numpy(),
        "prune0": pred["prune0"].numpy(),
        "prune1": pred["prune1"].numpy(),
        "n_layers_run": np.array(len(layers)),
    }
    la = pred["log_assignment"]
    inner = la[:, :-1, :-1]
    out["la_row_max"] = inner.max(2).values.numpy()
    out["la_col_max"] = inner.max(1).values.numpy()
    out["la_dustbin_col"] = la[:, :-1, -1].numpy()
    out["la_dustbin_row"] = la[:, -1, :-1].numpy()
    if conf.get("width_confidence", -1) <= 0 and conf.get("depth_confidence", -1) <= 0:
        # The same reference run in float64: top-1 / top-2 margins of every row and column of
        # the inner log assignment.  Rows/columns with a margin below the fp32 noise floor are
        # near-ties whose argmax no fp32 implementation decides reliably.
        m64 = copy.deepcopy(model).double()
        d64 = {k: (v.double() if isinstance(v, torch.Tensor) else {kk: vv.double() for kk, vv in v.items()}) for k, v in data.items()}
        torch.set_default_dtype(torch.float64)  # the reference builds its condition tensor with torch.ones
        try:
            with torch.no_grad():
                la64 = m64(d64)["log_assignment"][:, :-1, :-1]
        finally:
            torch.set_default_dtype(torch.float32)
        t0, t1 = la64.topk(min(2, la64.shape[2]), dim=2).values, la64.topk(min(2, la64.shape[1]), dim=1).values
        out["margin0"] = (t0[..., 0] - t0[..., -1]).float().numpy()
        out["margin1"] = (t1[:, 0] - t1[:, -1]).float().numpy()
    if pred["ref_descriptors0"].numel():
        out["ref_descriptors0"] = pred["ref_descriptors0"].numpy() if full else pred["ref_descriptors0"][:, :, :8].numpy()
        out["ref_descriptors1"] = pred["ref_descriptors1"].numpy() if full else pred["ref_descriptors1"][:, :, :8].numpy()
    if full:
        out["log_assignment"] = la.numpy()
        for li, (a, b) in enumerate(layers):
            out[f"layer{li}_desc0"] = a.numpy()
            out[f"layer{li}_desc1"] = b.numpy()
    meta = {
        "conf": conf,
        "pair": pkw,
        "weights": wkw,
        "overrides": {k: list(v) if isinstance(v, tuple) else v for k, v in over.items()},
        "inputs_sha256": sha(pair),
        "weights_sha256": sha(sd),
        "store_full": full,
    }
    out["meta_json"] = np.array(json.dumps(meta))
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **out)
    nm = int((out["matches0"] > -1).sum())
    print(f"{name}: layers_run={len(layers)} matches={nm} prune0_min={out['prune0'].min()}", flush=True)


# Sinkhorn cases: (B, M, N, alpha, iters, seed, full).  Large cases (configs[4]: 4096 x 4096,
# 50 iterations) store the dustbin row / column, every row's and column's max and argmax with
# their top-1 / top-2 margins, and 16 evenly spaced full rows instead of the 134 MB Z.
SINKHORN_CASES = {
    "sinkhorn_b2_60x50": (2, 60, 50, 1.0, 50, 31, True),
    "sinkhorn_b1_257x300": (1, 257, 300, 0.5, 50, 32, True),
    "sinkhorn_b1_64x64_it3": (1, 64, 64, 2.0, 3, 33, True),
    "sinkhorn_b2_4096x4096": (2, 4096, 4096, 1.0, 50, 34, False),
}


def run_sinkhorn(sg_mod, only=()):
    for name, (B, M, N, alpha, iters, seed, full) in SINKHORN_CASES.items():
        if only and name not in only and "sinkhorn" not in only:
            continue
        rng = np.random.Generator(np.random.PCG64(seed))
        scores = (rng.standard_normal((B, M, N)) * 2.0).astype(np.float32)
        with torch.no_grad():
            Z = sg_mod.log_optimal_transport(torch.from_numpy(scores), torch.tensor(alpha), iters)
        Zi = Z[:, :-1, :-1]
        max0, max1 = Zi.max(2), Zi.max(1)
        meta = {"B": B, "M": M, "N": N, "alpha": alpha, "iters": iters, "seed": seed, "scale": 2.0, "full": full}
        out = dict(
            scores_sha256=np.array(sha({"scores": scores})),
            row_argmax=max0.indices.numpy(),
            col_argmax=max1.indices.numpy(),
            meta_json=np.array(json.dumps(meta)),
        )
        if full:
            out["Z"] = Z.numpy()
        else:
            rows = np.linspace(0, M, 16).round().astype(np.int64)  # includes the dustbin row M
            out["sample_rows"] = rows
            out["Z_rows"] = Z[:, rows].numpy()
            out["Z_dustbin_col"] = Z[:, :, -1].numpy()
            out["row_max"] = max0.values.numpy()
            out["col_max"] = max1.values.numpy()
            t0, t1 = Zi.topk(2, dim=2).values, Zi.topk(2, dim=1).values
            out["row_margin"] = (t0[..., 0] - t0[..., 1]).numpy()
            out["col_margin"] = (t1[:, 0] - t1[:, 1]).numpy()
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **out)
        print(f"{name}: Z range [{Z.min().item():.3f}, {Z.max().item():.3f}]", flush=True)


def main():
    torch.set_num_threads(8)
    lg_mod, sg_mod = install_shim()
    only = set(sys.argv[1:])
    for name, spec in CASES.items():
        if only and name not in only:
            continue
        run_case(lg_mod, name, spec)
    if not only or any(o.startswith("sinkhorn") for o in only):
        run_sinkhorn(sg_mod, only)


if __name__ == "__main__":
    main()
