"""Pin the SuperGlue oracle (oracle/superglue_ref.py) to the reference's own outputs
(tests/golden/sg_*.npz, made by tests/golden/make_superglue_golden.py from
/root/reference/gluefactory_nonfree/superglue.py and gluefactory/models/utils/losses.py).

Same torch-CPU fp32 operations in the same order, up to the einsum/conv summation order of the
1x1 convolutions, so outputs agree to a few fp32 ulps; matches are compared exactly.
"""
import numpy as np
import pytest
import torch

from oracle.superglue_ref import nll_loss, superglue_forward, superglue_loss
from sg_golden_util import sg_case, sg_case_names, sg_load, sha


@pytest.mark.parametrize("name", sg_case_names())
def test_superglue_oracle_matches_reference(name):
    g = sg_load(name)
    meta = g["meta"]
    conf, sd, data, gt = sg_case(meta)
    assert sha({k: v for k, v in data.items() if k != "image_hw"}) == meta["inputs_sha256"], "input recipe drifted"
    assert sha(sd) == meta["weights_sha256"], "weight recipe drifted"
    with torch.no_grad():
        out = superglue_forward(sd, data, conf)
    np.testing.assert_allclose(out["gnn_desc0"].numpy(), g["gnn_desc0"], rtol=0, atol=2e-5)
    np.testing.assert_allclose(out["gnn_desc1"].numpy(), g["gnn_desc1"], rtol=0, atol=2e-5)
    np.testing.assert_allclose(out["sinkhorn_cost"].numpy(), g["out_sinkhorn_cost"], rtol=0, atol=1e-4)
    np.testing.assert_allclose(out["log_assignment"].numpy(), g["out_log_assignment"], rtol=0, atol=1e-4)
    np.testing.assert_array_equal(out["matches0"].numpy(), g["out_matches0"])
    np.testing.assert_array_equal(out["matches1"].numpy(), g["out_matches1"])
    np.testing.assert_allclose(out["matching_scores0"].numpy(), g["out_matching_scores0"], rtol=0, atol=1e-5)
    # losses on the reference's own log assignment
    la = torch.from_numpy(g["out_log_assignment"])
    sl = superglue_loss(la, gt["gt_assignment"], gt["gt_matches0"], gt["gt_matches1"], bin_score=sd["bin_score"])
    for k, v in sl.items():
        np.testing.assert_allclose(v.numpy(), g[f"sgloss_{k}"], rtol=1e-6, atol=0, err_msg=k)
    if meta["nll_error"] is None:
        total, metrics = nll_loss(la, gt["gt_assignment"], gt["gt_matches0"], gt["gt_matches1"])
        np.testing.assert_allclose(total.numpy(), g["nll_total"], rtol=1e-6)
        for k, v in metrics.items():
            np.testing.assert_allclose(v.numpy(), g[f"nll_{k}"], rtol=1e-6, err_msg=k)
    else:
        with pytest.raises(RuntimeError, match="must match the existing size"):
            nll_loss(la, gt["gt_assignment"], gt["gt_matches0"], gt["gt_matches1"])


def test_superglue_oracle_no_keypoints():
    """superglue.py:257-264: an empty view returns -1 matches (int32) and zero scores."""
    from lightglue_amd.sg_weights import superglue_state_dict

    sd = superglue_state_dict({}, seed=0)
    data = {"keypoints0": np.zeros((2, 0, 2), np.float32), "keypoints1": np.zeros((2, 5, 2), np.float32),
            "descriptors0": np.zeros((2, 0, 256), np.float32), "descriptors1": np.zeros((2, 5, 256), np.float32),
            "image_hw": (480, 640)}
    out = superglue_forward(sd, data, {})
    assert out["matches0"].shape == (2, 0) and out["matches1"].dtype == torch.int32
    assert (out["matches1"] == -1).all() and (out["matching_scores1"] == 0).all()
