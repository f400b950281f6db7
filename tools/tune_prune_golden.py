#!/usr/bin/env python3
"""Pick the per-layer token-confidence / matchability biases of the configs[3]-shaped golden
case (tests/golden/make_golden.py, case ``prune_depth_width_n2048``) by running the REAL
reference (build container only: needs /root/reference, imported through make_golden's harness).

Goal of the recipe: at N = 2048 with width_confidence = depth_confidence = 0.95 the reference
really prunes (about 10 % of the points per layer, layers 0..4) and then stops early (layer 5),
so the fixture exercises compaction, the remap, the per-layer prune counts and the early stop.
Every decision threshold is placed in the middle of a gap of the sorted decision logits (at least
1e-3 wide), so no point sits within fp32 noise of a pruning / confidence threshold and the
decisions are reproducible by any fp32-accurate implementation.

    python tools/tune_prune_golden.py      # prints TOKEN_BIAS / MATCH_BIAS for make_golden.py
"""
import math
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
sys.path.insert(0, ROOT)
import make_golden  # noqa: E402
from lightglue_amd.weights import synthetic_pair, synthetic_state_dict  # noqa: E402

CONF = {"filter_threshold": 0.1, "width_confidence": 0.95, "depth_confidence": 0.95}
PAIR = dict(B=1, M=2048, N=2048, seed=41)
WEIGHTS = dict(seed=8)
PRUNE_LAYERS = 5      # layers 0..4 prune
STOP_LAYER = 5        # early stop fires here
CONFIDENT_FRAC = 0.7  # tokens above the layer threshold at the pruning layers
PRUNE_FRAC = 0.14     # of the confident points (~10 % of all points)


def logit(p):
    return math.log(p / (1 - p))


def gap_value(v, q, lo=0.05):
    """A value near quantile q of v lying in the middle of the widest gap within +-lo quantiles."""
    s = np.sort(v)
    n = len(s)
    a, b = max(1, int((q - lo) * n)), min(n - 1, int((q + lo) * n))
    k = a + int(np.argmax(s[a:b] - s[a - 1 : b - 1]))
    return 0.5 * (s[k] + s[k - 1]), s[k] - s[k - 1]


def run(lg_mod, sd, data):
    model = lg_mod.LightGlue(dict(CONF)).eval()
    L = model.conf.n_layers
    model.confidence_thresholds = [model.confidence_threshold(i) for i in range(L)]
    model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
    layers = []
    hooks = [t.register_forward_hook(lambda mod, inp, out: layers.append((out[0].clone(), out[1].clone())))
             for t in model.transformers]
    real = lg_mod.torch
    lg_mod.torch = make_golden._TorchProxy(real)
    try:
        with torch.no_grad():
            pred = model(data)
    finally:
        lg_mod.torch = real
        for h in hooks:
            h.remove()
    return pred, layers, model


def main():
    torch.set_num_threads(8)
    lg_mod, _ = make_golden.install_shim()
    base = synthetic_state_dict(CONF, **WEIGHTS)
    pair = synthetic_pair(**PAIR)
    data = {k: torch.from_numpy(v) for k, v in pair.items() if not k.startswith("image_size")}
    data["view0"] = {"image_size": torch.from_numpy(pair["image_size0"])}
    data["view1"] = {"image_size": torch.from_numpy(pair["image_size1"])}
    L = 9
    tok = [-20.0] * (L - 1)   # token ~0: never confident -> nothing pruned, no stop
    mat = [20.0] * (L - 1)    # matchability ~1: kept
    for i in range(PRUNE_LAYERS + 1):
        sd = {k: v.copy() for k, v in base.items()}
        for j in range(L - 1):
            sd[f"token_confidence.{j}.token.0.bias"][:] = tok[j]
            sd[f"log_assignment.{j}.matchability.bias"][:] = mat[j]
        _, layers, model = run(lg_mod, sd, data)
        d = torch.cat([layers[i][0][0], layers[i][1][0]]).double().numpy()
        thr = float(model.confidence_thresholds[i])
        wt = base[f"token_confidence.{i}.token.0.weight"].astype(np.float64)[0]
        wm = base[f"log_assignment.{i}.matchability.weight"].astype(np.float64)[0]
        t = d @ wt
        z = d @ wm
        if i == STOP_LAYER:
            tok[i] = float(logit(thr) - np.min(t) + 4.0)  # every token confident -> ratio 1 > 0.95
            print(f"layer {i}: stop, token bias {tok[i]:.4f}", flush=True)
            break
        v, g = gap_value(t, 1 - CONFIDENT_FRAC)
        tok[i] = float(np.float32(logit(thr) - v))
        conf = t + tok[i] > logit(thr)
        vz, gz = gap_value(z[conf], PRUNE_FRAC)
        mat[i] = float(np.float32(logit(0.05) - vz))
        kept = (~conf) | (z + mat[i] > logit(0.05))
        print(f"layer {i}: rows {len(t)} token bias {tok[i]:.4f} (gap {g:.2e}) confident {conf.mean():.3f}; "
              f"matchability bias {mat[i]:.4f} (gap {gz:.2e}) kept {kept.mean():.3f}", flush=True)
    print("TOKEN_BIAS =", [round(x, 4) for x in tok])
    print("MATCH_BIAS =", [round(x, 4) for x in mat])


if __name__ == "__main__":
    main()
