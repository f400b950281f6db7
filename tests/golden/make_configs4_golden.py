#!/usr/bin/env python3
"""configs[4] END TO END from the REAL reference (harness only; needs ``/root/reference``)::

    python tests/golden/make_configs4_golden.py

The composition ``bench.py --workload configs4`` times (``lightglue_amd.assignment.sinkhorn_match``):
the in-tree LightGlue forward in eval mode (no pruning) on N = 4096 keypoints, its final
``MatchAssignment`` similarity (``lightglue.py:306-315``: the second output, which ``forward``
discards -- the harness calls ``model.log_assignment[-1]`` on ``pred["ref_descriptors*"][:, 0]``,
the final descriptors, ``:550``), ``log_optimal_transport`` with the SuperGlue dustbin score 1.0 and
50 iterations (``gluefactory_nonfree/superglue.py:181-201,214``) and the mutual filter at 0.2
(``superglue.py:288-298``).  B = 8 pairs (configs[4]: 8 pairs per GPU).

Run once in float32 (the values) and once in float64 (every row's / column's top-1 / top-2 margin
of the transport's inner block, so index flips on near-ties can be told apart, and the float32
run's own spread of Z against float64).  Stored: matches / scores, 4 evenly spaced full Z rows per
pair, the dustbin column, row / column maxima, the margins, the spread; inputs and weights are
the committed recipes (SHA-256 stored).
"""
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import install_shim, sha  # noqa: E402

from lightglue_amd.weights import synthetic_pair, synthetic_state_dict  # noqa: E402

NAME = "configs4_b8_n4096"
B, N, SEED, WSEED = 8, 4096, 1, 0
ALPHA, ITERS, TH = 1.0, 50, 0.2


def run(lg_mod, sg_mod, dtype):
    torch.set_default_dtype(dtype)
    try:
        conf = {"filter_threshold": 0.1}
        sd = synthetic_state_dict(conf, seed=WSEED)
        model = lg_mod.LightGlue(dict(conf))
        model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
        model = model.to(dtype).eval()
        pair = synthetic_pair(B=B, M=N, seed=SEED)
        data = {k: torch.from_numpy(v).to(dtype) for k, v in pair.items() if not k.startswith("image_size")}
        data["view0"] = {"image_size": torch.from_numpy(pair["image_size0"]).to(dtype)}
        data["view1"] = {"image_size": torch.from_numpy(pair["image_size1"]).to(dtype)}
        with torch.no_grad():
            pred = model(data)
            _, sim = model.log_assignment[-1](pred["ref_descriptors0"][:, 0], pred["ref_descriptors1"][:, 0])
            Z = sg_mod.log_optimal_transport(sim, torch.tensor(ALPHA, dtype=dtype), ITERS)
        return sd, pair, Z
    finally:
        torch.set_default_dtype(torch.float32)


def mutual_filter(Z, th):
    """superglue.py:288-298 (identical to lightglue.py:321-337)."""
    inner = Z[:, :-1, :-1]
    max0, max1 = inner.max(2), inner.max(1)
    m0, m1 = max0.indices, max1.indices
    mutual0 = torch.arange(m0.shape[1])[None] == m1.gather(1, m0)
    mutual1 = torch.arange(m1.shape[1])[None] == m0.gather(1, m1)
    zero = Z.new_tensor(0)
    ms0 = torch.where(mutual0, max0.values.exp(), zero)
    ms1 = torch.where(mutual1, ms0.gather(1, m1), zero)
    valid0 = mutual0 & (ms0 > th)
    valid1 = mutual1 & valid0.gather(1, m1)
    return torch.where(valid0, m0, -1), torch.where(valid1, m1, -1), ms0, ms1


def main():
    torch.set_num_threads(8)
    lg_mod, sg_mod = install_shim()
    sd, pair, Z = run(lg_mod, sg_mod, torch.float32)
    _, _, Z64 = run(lg_mod, sg_mod, torch.float64)
    m0, m1, s0, s1 = mutual_filter(Z, TH)
    Zi, Z64i = Z[:, :-1, :-1], Z64[:, :-1, :-1]
    rows = np.linspace(0, N, 4).round().astype(np.int64)  # includes the dustbin row N
    t0, t1 = Z64i.topk(2, dim=2).values, Z64i.topk(2, dim=1).values
    s64 = mutual_filter(Z64, TH)[2]
    out = {
        "matches0": m0.numpy(), "matches1": m1.numpy(),
        "matching_scores0": s0.numpy(), "matching_scores1": s1.numpy(),
        "sample_rows": rows, "Z_rows": Z[:, rows].numpy(), "Z_dustbin_col": Z[:, :, -1].numpy(),
        "row_max": Zi.max(2).values.numpy(), "col_max": Zi.max(1).values.numpy(),
        "row_margin": (t0[..., 0] - t0[..., 1]).float().numpy(), "col_margin": (t1[:, 0] - t1[:, 1]).float().numpy(),
        # |exp(max) - threshold| per row in float64: rows whose validity the fp32 rounding can decide
        "row_th_margin": (s64 - TH).abs().float().numpy(),
        "spread_Z": np.float64((Z.double() - Z64).abs().max()),
        "spread_scores0": np.float64((s0.double() - s64).abs().max()),
    }
    meta = {"B": B, "N": N, "pair_seed": SEED, "weights_seed": WSEED, "conf": {"filter_threshold": 0.1},
            "alpha": ALPHA, "iters": ITERS, "threshold": TH,
            "inputs_sha256": sha(pair), "weights_sha256": sha(sd)}
    out["meta_json"] = np.array(json.dumps(meta))
    np.savez_compressed(os.path.join(HERE, f"{NAME}.npz"), **out)
    print(NAME, "matches/pair", float((m0 > -1).float().sum(1).mean()), "spread_Z", out["spread_Z"],
          "spread_scores0", out["spread_scores0"], "min row margin", float(out["row_margin"].min()),
          "min col margin", float(out["col_margin"].min()), flush=True)


if __name__ == "__main__":
    main()
