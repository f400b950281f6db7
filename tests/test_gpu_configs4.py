"""configs[4] END TO END on the HIP library against the reference (tests/golden/configs4_b8_n4096.npz,
make_configs4_golden.py) -- needs an MI355X.

The composition is ``lightglue_amd.assignment.sinkhorn_match``, exactly what ``bench.py --workload
configs4`` times: LightGlue forward (N = 4096, B = 8, no pruning) -> its final similarity ->
log_optimal_transport (dustbin 1.0, 50 iterations) -> mutual filter (0.2).

Bars: matching scores within 1e-4 (the north star's score bar; the reference's own fp32-vs-fp64
spread is 3.2e-5); match indices exact on every row / column whose float64 top-1 / top-2 margin in
Z and |exp(max) - 0.2| are at least 1e-3 (the rest are reported; none may flip beyond that
count); Z rows, the dustbin column and the row / column maxima within max(1e-4, 2 x the reference's
own fp32-vs-fp64 spread of Z, 6.3e-4): Z carries the similarity's absolute rounding (|sim| ~ 1e2
with the sharpened recipe) through 50 iterations.
"""
import json
import os

import numpy as np
import pytest
import torch

import lgamd  # noqa: F401
from golden_util import HERE, sha

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def test_configs4_end_to_end_matches_reference():
    from lightglue_amd import LightGlue
    from lightglue_amd.assignment import sinkhorn_match
    from lightglue_amd.weights import synthetic_pair, synthetic_state_dict

    z = np.load(os.path.join(HERE, "configs4_b8_n4096.npz"))
    g = {k: z[k] for k in z.files if k != "meta_json"}
    meta = json.loads(str(z["meta_json"]))
    B, N = meta["B"], meta["N"]
    conf = dict(meta["conf"])
    sd = synthetic_state_dict(conf, seed=meta["weights_seed"])
    pair = synthetic_pair(B=B, M=N, seed=meta["pair_seed"])
    assert sha(pair) == meta["inputs_sha256"] and sha(sd) == meta["weights_sha256"]
    model = LightGlue({**conf, "return_similarity": True}).eval().to(DEV)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
    data = {k: torch.from_numpy(v).to(DEV) for k, v in pair.items() if not k.startswith("image_size")}
    data["view0"] = {"image_size": torch.from_numpy(pair["image_size0"]).to(DEV)}
    data["view1"] = {"image_size": torch.from_numpy(pair["image_size1"]).to(DEV)}
    with torch.no_grad():
        out, Z = sinkhorn_match(model, data, meta["alpha"], meta["iters"], meta["threshold"])
    Zc = Z.cpu().numpy()
    ztol = max(1e-4, 2 * float(g["spread_Z"]))
    np.testing.assert_allclose(Zc[:, g["sample_rows"]], g["Z_rows"], atol=ztol, rtol=0)
    np.testing.assert_allclose(Zc[:, :, -1], g["Z_dustbin_col"], atol=ztol, rtol=0)
    inner = Zc[:, :-1, :-1]
    np.testing.assert_allclose(inner.max(2), g["row_max"], atol=ztol, rtol=0)
    np.testing.assert_allclose(inner.max(1), g["col_max"], atol=ztol, rtol=0)
    for k in ("matching_scores0", "matching_scores1"):
        np.testing.assert_allclose(out[k].cpu().numpy(), g[k], atol=1e-4, rtol=0)
    m0 = out["matches0"].cpu().numpy()
    m1 = out["matches1"].cpu().numpy()
    # decidable rows: clear fp64 argmax margin, clear threshold margin, and the matched column's
    # own argmax clear as well (the mutual check reads it)
    ref0 = g["matches0"]
    col_ok = np.ones_like(g["col_margin"], dtype=bool)
    col_ok &= g["col_margin"] >= 1e-3
    arg0 = inner.argmax(2)
    dec0 = (g["row_margin"] >= 1e-3) & (g["row_th_margin"] >= 1e-3) & np.take_along_axis(col_ok, arg0, 1)
    flips = int(((m0 != ref0) & dec0).sum())
    undecided = int((m0 != ref0).sum()) - flips
    print(f"configs4: {int((m0 > -1).sum())} matches, {flips} decidable flips, {undecided} near-tie flips, "
          f"{int((~dec0).sum())} near-tie rows; Z max err {np.abs(Zc[:, g['sample_rows']] - g['Z_rows']).max():.2e}")
    assert flips == 0
    assert undecided <= int((~dec0).sum())
    # matches1 follows from matches0 on mutual pairs: consistency of the two sides
    b, i = np.nonzero(m0 > -1)
    assert (m1[b, m0[b, i]] == i).all()
