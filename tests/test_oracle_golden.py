"""Pin the CPU oracle (oracle/lightglue_ref.py) to the reference's own outputs (tests/golden).

The fixtures were produced by running /root/reference through tests/golden/make_golden.py.
Tolerances: indices exact; scores |d| <= 1e-5 (same torch-CPU fp32 arithmetic, different op
grouping); log-assignment rows |d| <= 1e-4.
"""
import numpy as np
import pytest
import torch

import oracle
from golden_util import case_inputs, case_names, load, sha, sinkhorn_inputs, sinkhorn_names


@pytest.mark.parametrize("name", case_names())
def test_oracle_matches_reference(name):
    g = load(name)
    meta = g["meta"]
    conf, sd, data = case_inputs(meta)
    assert sha(data) == meta["inputs_sha256"], "input recipe drifted"
    assert sha(sd) == meta["weights_sha256"], "weight recipe drifted"
    out = oracle.lightglue_forward(sd, data, conf)
    assert out["stop_layer"] + 1 == int(g["n_layers_run"])
    np.testing.assert_array_equal(out["matches0"].numpy(), g["matches0"])
    np.testing.assert_array_equal(out["matches1"].numpy(), g["matches1"])
    np.testing.assert_allclose(out["matching_scores0"].numpy(), g["matching_scores0"], atol=1e-4)
    np.testing.assert_allclose(out["matching_scores1"].numpy(), g["matching_scores1"], atol=1e-4)
    np.testing.assert_array_equal(out["prune0"].numpy(), g["prune0"])
    np.testing.assert_array_equal(out["prune1"].numpy(), g["prune1"])
    la = out["log_assignment"]
    np.testing.assert_allclose(la[:, :-1, :-1].max(2).values.numpy(), g["la_row_max"], atol=1e-3)
    np.testing.assert_allclose(la[:, :-1, :-1].max(1).values.numpy(), g["la_col_max"], atol=1e-3)
    np.testing.assert_allclose(la[:, :-1, -1].numpy(), g["la_dustbin_col"], atol=1e-4)
    np.testing.assert_allclose(la[:, -1, :-1].numpy(), g["la_dustbin_row"], atol=1e-4)
    if "log_assignment" in g:
        np.testing.assert_allclose(la.numpy(), g["log_assignment"], atol=1e-3)
    if "ref_descriptors0" in g:
        # non-full fixtures keep only the first 8 keypoints' descriptors
        k0, k1 = g["ref_descriptors0"].shape[2], g["ref_descriptors1"].shape[2]
        np.testing.assert_allclose(out["ref_descriptors0"][:, :, :k0].numpy(), g["ref_descriptors0"], atol=1e-4, rtol=1e-5)
        np.testing.assert_allclose(out["ref_descriptors1"][:, :, :k1].numpy(), g["ref_descriptors1"], atol=1e-4, rtol=1e-5)


@pytest.mark.parametrize("name", sinkhorn_names())
def test_oracle_sinkhorn_matches_reference(name):
    g = load(name)
    meta = g["meta"]
    scores = sinkhorn_inputs(meta)
    assert sha({"scores": scores}) == str(g["scores_sha256"])
    Z = oracle.log_optimal_transport(torch.from_numpy(scores), meta["alpha"], meta["iters"])
    inner = Z[:, :-1, :-1]
    if "Z" in g:
        np.testing.assert_allclose(Z.numpy(), g["Z"], atol=2e-5, rtol=1e-5)
        np.testing.assert_array_equal(inner.max(2).indices.numpy(), g["row_argmax"])
        np.testing.assert_array_equal(inner.max(1).indices.numpy(), g["col_argmax"])
    else:  # large case: sampled rows, dustbin column, row / column maxima (make_golden.py)
        np.testing.assert_allclose(Z[:, g["sample_rows"]].numpy(), g["Z_rows"], atol=2e-5, rtol=1e-5)
        np.testing.assert_allclose(Z[:, :, -1].numpy(), g["Z_dustbin_col"], atol=2e-5, rtol=1e-5)
        np.testing.assert_allclose(inner.max(2).values.numpy(), g["row_max"], atol=2e-5, rtol=1e-5)
        np.testing.assert_allclose(inner.max(1).values.numpy(), g["col_max"], atol=2e-5, rtol=1e-5)
        r_ok, c_ok = g["row_margin"] > 1e-4, g["col_margin"] > 1e-4
        np.testing.assert_array_equal(inner.max(2).indices.numpy()[r_ok], g["row_argmax"][r_ok])
        np.testing.assert_array_equal(inner.max(1).indices.numpy()[c_ok], g["col_argmax"][c_ok])
