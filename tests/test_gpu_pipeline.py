"""The HIP matcher behind the reference's callers — needs an MI355X.
TwoViewPipeline (two_view_pipeline.py:79-97) with cached features feeds lightglue_amd.LightGlue
through the registry name "matchers.lightglue"; the batched export loop
(export_predictions.py:17-85, every pair written) stores exactly what the matcher returned, and the
result equals the reference's golden vectors."""
import numpy as np
import pytest
import torch

import lgamd  # noqa: F401
from golden_util import case_inputs, load

pytestmark = pytest.mark.gpu


def _pipeline_data(data, names):
    d = {}
    for i in (0, 1):
        d[f"view{i}"] = {
            "image_size": torch.from_numpy(data[f"image_size{i}"]).cuda(),
            "scales": torch.ones(data[f"image_size{i}"].shape, device="cuda"),
            "cache": {"keypoints": torch.from_numpy(data[f"keypoints{i}"]).cuda(),
                      "descriptors": torch.from_numpy(data[f"descriptors{i}"]).cuda()},
        }
    d["name"] = names
    return d


def test_pipeline_and_export_match_golden():
    from lightglue_amd import export, pipeline

    g = load("tiny_ragged_b2")
    conf, sd, data = case_inputs(g["meta"])
    pipe = pipeline.get_model("two_view_pipeline")({"matcher": {"name": "matchers.lightglue", **conf}}).eval().cuda()
    res = pipe.matcher.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
    assert not res.missing_keys
    batch = _pipeline_data(data, ["pair/a", "pair/b"])
    with torch.no_grad():
        pred = pipe(batch)
    np.testing.assert_array_equal(pred["matches0"].cpu().numpy(), g["matches0"])
    np.testing.assert_array_equal(pred["matches1"].cpu().numpy(), g["matches1"])
    w = export.MemoryWriter()
    export.export_predictions([batch, _pipeline_data(data, ["pair/c", "pair/d"])], pipe, writer=w,
                              keys=["keypoints0", "keypoints1", "matches0", "matches1", "matching_scores0",
                                    "matching_scores1"], device="cuda")
    assert sorted(w.groups) == ["pair/a", "pair/b", "pair/c", "pair/d"]
    for b, name in enumerate(["pair/a", "pair/b"]):
        np.testing.assert_array_equal(w.groups[name]["matches0"], g["matches0"][b])
        np.testing.assert_allclose(w.groups[name]["matching_scores0"], g["matching_scores0"][b], atol=1e-4)
        np.testing.assert_array_equal(w.groups[name]["keypoints0"], data["keypoints0"][b])
    np.testing.assert_array_equal(w.groups["pair/d"]["matches1"], g["matches1"][1])
