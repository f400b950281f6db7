"""Pin the SuperPoint oracle (oracle/superpoint_ref.py) to the reference's own outputs
(tests/golden/sp_*.npz, made by tests/golden/make_superpoint_golden.py from
/root/reference/gluefactory_nonfree/superpoint.py).

Same torch-CPU fp32 arithmetic, so keypoints and scores are compared exactly and descriptors at
1e-6.  The B = 2 fixture uses force_num_keypoints with a budget every image fills (the reference
returns B > 1 sparse outputs only then, superpoint.py:330-344); the oracle stacks per-image
samples, which is the same arithmetic.
"""
import numpy as np
import pytest
import torch

from oracle.superpoint_ref import superpoint_forward
from sp_golden_util import sha, sp_case_inputs, sp_case_names, sp_load


@pytest.mark.parametrize("name", sp_case_names())
def test_superpoint_oracle_matches_reference(name):
    g = sp_load(name)
    meta = g["meta"]
    conf, sd, data = sp_case_inputs(meta)
    assert sha({"image": data["image"]}) == meta["inputs_sha256"], "image recipe drifted"
    assert sha(sd) == meta["weights_sha256"], "weight recipe drifted"
    conf = {k: v for k, v in conf.items() if k != "force_num_keypoints"}
    with torch.no_grad():
        out = superpoint_forward(sd, data, conf)
    if conf.get("sparse_outputs", True):
        np.testing.assert_array_equal(out["keypoints"].numpy(), g["out_keypoints"])
        np.testing.assert_array_equal(out["keypoint_scores"].numpy(), g["out_keypoint_scores"])
        np.testing.assert_allclose(out["descriptors"].numpy(), g["out_descriptors"], atol=1e-6)
    else:
        np.testing.assert_array_equal(out["keypoint_scores"].numpy(), g["out_keypoint_scores"])
        np.testing.assert_allclose(out["descriptors"].numpy(), g["out_descriptors"], atol=1e-6)
