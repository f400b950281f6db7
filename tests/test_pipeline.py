"""Callers around the matcher: the two-view pipeline / registry
(reference models/two_view_pipeline.py:21-97, models/__init__.py:7-30) and the batched export
loop (utils/export_predictions.py:17-85).  CPU: stand-in extractor and matcher registered through
register_model; the GPU test in test_gpu_pipeline.py runs the HIP matcher through the same code."""
import numpy as np
import pytest
import torch
from torch import nn

import lgamd  # noqa: F401
from lightglue_amd import export, pipeline


class FakeExtractor(nn.Module):
    """Keypoints = a fixed grid scaled by the image content, descriptors = one-hot rows."""

    def __init__(self, conf):
        super().__init__()
        self.conf = conf

    def forward(self, view):
        img = view["image"]
        b = img.shape[0]
        n = 5
        k = torch.arange(n, dtype=torch.float32)[None, :, None].repeat(b, 1, 2) * img.mean((1, 2, 3))[:, None, None]
        return {"keypoints": k, "descriptors": torch.eye(n)[None].repeat(b, 1, 1), "keypoint_scores": torch.ones(b, n)}


class FakeMatcher(nn.Module):
    def __init__(self, conf):
        super().__init__()
        self.conf = conf
        self.seen = []

    def forward(self, data):
        self.seen.append(sorted(data))
        m0 = torch.arange(data["keypoints0"].shape[1])[None].repeat(data["keypoints0"].shape[0], 1)
        return {"matches0": m0, "matches1": m0.clone(), "matching_scores0": torch.ones(m0.shape),
                "matching_scores1": torch.ones(m0.shape)}


pipeline.register_model("extractors.fake", FakeExtractor)
pipeline.register_model("matchers.fake", FakeMatcher)


def _data(b, names):
    g = torch.Generator().manual_seed(0)
    v = lambda: {"image": torch.rand(b, 1, 8, 8, generator=g), "scales": torch.rand(b, 2, generator=g) + 0.5}
    return {"view0": v(), "view1": v(), "name": names}


def test_registry_resolves_reference_names():
    from lightglue_amd.lightglue import LightGlue

    assert pipeline.get_model("matchers.lightglue") is LightGlue
    assert pipeline.get_model("lightglue") is LightGlue  # matchers. prefix fallback
    assert pipeline.get_model("two_view_pipeline") is pipeline.TwoViewPipeline
    assert pipeline.get_model("fake") is FakeMatcher
    with pytest.raises(RuntimeError, match="not found"):
        pipeline.get_model("matchers.nope")


def test_two_view_pipeline_merges_like_reference():
    m = pipeline.TwoViewPipeline({"extractor": {"name": "extractors.fake"}, "matcher": {"name": "fake"}})
    data = _data(2, ["a", "b"])
    pred = m(data)
    for k in ("keypoints0", "descriptors1", "keypoint_scores0", "matches0", "matching_scores1"):
        assert k in pred
    # the matcher sees {**data, **pred}: views and the extractor outputs of both images
    assert {"view0", "view1", "keypoints0", "keypoints1", "descriptors0"} <= set(m.matcher.seen[0])
    with pytest.raises(AssertionError, match="Missing key view1"):
        m({"view0": data["view0"]})
    # frozen extractor (trainable: False by default for the extractor, two_view_pipeline.py:24-27)
    assert m.conf.extractor.trainable is False


def test_cache_and_allow_no_extract():
    m = pipeline.TwoViewPipeline({"extractor": {"name": "extractors.fake"}, "matcher": {"name": "fake"},
                                  "allow_no_extract": True})
    data = _data(1, ["a"])
    cache = {"keypoints": torch.zeros(1, 3, 2), "descriptors": torch.zeros(1, 3, 5)}
    data["view0"]["cache"] = cache
    pred = m(data)
    assert pred["keypoints0"].shape[1] == 3 and pred["keypoints1"].shape[1] == 5


def test_mine_wrapper_builds_lightglue_with_features_key():
    w = pipeline.get_model("matchers.lightglue_pretrained_MINE")({"filter_threshold": 0.2})
    assert w.conf.features == "superpoint" and w.net.conf.filter_threshold == 0.2
    assert len(w.net.transformers) == 9


def test_export_writes_every_pair_of_a_batch(tmp_path):
    """The reference keeps v[0] only (export_predictions.py:68); every pair is written here, with
    keypoints divided by ITS view's scales."""
    m = pipeline.TwoViewPipeline({"extractor": {"name": "extractors.fake"}, "matcher": {"name": "fake"}})
    loader = [_data(3, ["s/0", "s/1", "s/2"]), _data(2, ["t/0", "t/1"])]
    w = export.MemoryWriter()
    export.export_predictions(loader, m, writer=w, keys=["keypoints0", "matches0"], optional_keys=["matching_scores0"],
                              device="cpu")
    assert sorted(w.groups) == ["s/0", "s/1", "s/2", "t/0", "t/1"]
    for bi, batch in enumerate(loader):
        pred = m(batch)
        for b, name in enumerate(batch["name"]):
            got = w.groups[name]
            assert set(got) == {"keypoints0", "matches0", "matching_scores0"}
            exp = (pred["keypoints0"][b] / batch["view0"]["scales"][b]).numpy()
            np.testing.assert_allclose(got["keypoints0"], exp, rtol=1e-6)
            np.testing.assert_array_equal(got["matches0"], pred["matches0"][b].numpy())
    with pytest.raises(ValueError, match="Missing key"):
        export.export_predictions(loader, m, writer=export.MemoryWriter(), keys=["nope"], device="cpu")


def test_export_npz_writer_and_duplicates(tmp_path):
    m = pipeline.TwoViewPipeline({"extractor": {"name": "extractors.fake"}, "matcher": {"name": "fake"}})
    loader = [_data(2, ["seq/1_2", "seq/1_3"]), _data(1, ["seq/1_2"])]  # duplicate name is skipped
    export.export_predictions(loader, m, writer=export.NpzWriter(tmp_path), as_half=True, device="cpu")
    z = np.load(tmp_path / "seq" / "1_2.npz")
    assert z["keypoints0"].dtype == np.float16 and z["matches0"].dtype == np.int64
    assert (tmp_path / "seq" / "1_3.npz").exists()


def test_h5_writer_is_unavailable_here():
    try:
        import h5py  # noqa: F401
    except ImportError:
        with pytest.raises(ImportError):
            export.H5Writer("/tmp/nope.h5")


class ListMatcher(FakeMatcher):
    """A pruned B > 1 batch: per-pair LISTS of kept blocks for log_assignment / ref_descriptors,
    plus a scalar that has no per-pair form (lightglue_amd.LightGlue with pruning)."""

    def forward(self, data):
        out = super().forward(data)
        b = data["keypoints0"].shape[0]
        out["log_assignment"] = [torch.full((i + 2, i + 3), float(i)) for i in range(b)]
        out["stop_note"] = 7
        return out


def test_export_writes_per_pair_lists_and_names_skipped_keys():
    pipeline.register_model("matchers.fake_lists", ListMatcher)
    m = pipeline.TwoViewPipeline({"extractor": {"name": "extractors.fake"}, "matcher": {"name": "fake_lists"}})
    loader = [_data(3, ["a/0", "a/1", "a/2"])]
    w = export.MemoryWriter()
    with pytest.warns(UserWarning, match="stop_note"):
        export.export_predictions(loader, m, writer=w, device="cpu")
    for i in range(3):
        la = w.groups[f"a/{i}"]["log_assignment"]
        assert la.shape == (i + 2, i + 3) and float(la[0, 0]) == i
        assert "stop_note" not in w.groups[f"a/{i}"]
