"""CPU-only checks: the C-ABI library loads and exports what include/*.h declares, the drop-in
module keeps the reference's config keys and state-dict schema, and the host helpers behave."""
import ctypes
import glob
import os
import re

import numpy as np
import pytest
import torch

import lgamd  # noqa: F401
from lightglue_amd import _lib
from lightglue_amd.weights import DEFAULT_CONF, state_dict_schema, synthetic_pair, synthetic_state_dict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    syms = set()
    for h in glob.glob(os.path.join(ROOT, "include", "*.h")):
        src = open(h).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        syms |= set(re.findall(r"\b((?:lg|sp|sg)_[a-z_0-9]+)\s*\(", src))
    return syms


def test_library_loads_and_exports_every_declared_symbol():
    lib = _lib.load()
    declared = declared_symbols()
    assert declared, "no declarations found"
    for s in sorted(declared):
        assert hasattr(lib, s), f"{s} declared in include/ but not exported"
    assert declared == set(_lib.EXPORTED_SYMBOLS)
    assert lib.lg_abi_version() == _lib.ABI_VERSION


def test_ctypes_structs_match_header_layout(tmp_path):
    """Every field offset and struct size of the ctypes mirrors equals what a C compiler makes of
    include/lightglue_mi355x.h (gcc on a generated offsetof table)."""
    import subprocess

    structs = {"lg_config_t": _lib.LGConfig, "lg_inputs_t": _lib.LGInputs, "lg_outputs_t": _lib.LGOutputs,
               "sp_config_t": _lib.SPConfig, "sp_inputs_t": _lib.SPInputs, "sp_outputs_t": _lib.SPOutputs,
               "sg_config_t": _lib.SGConfig, "sg_inputs_t": _lib.SGInputs, "sg_outputs_t": _lib.SGOutputs}
    lines = ["#include <stdio.h>", "#include <stddef.h>", f'#include "{os.path.join(ROOT, "include", "lightglue_mi355x.h")}"',
             f'#include "{os.path.join(ROOT, "include", "superpoint_mi355x.h")}"',
             f'#include "{os.path.join(ROOT, "include", "superglue_mi355x.h")}"', "int main(void) {"]
    for cname, py in structs.items():
        lines.append(f'printf("{cname} size %zu\\n", sizeof({cname}));')
        for f, _ in py._fields_:
            lines.append(f'printf("{cname} {f} %zu\\n", offsetof({cname}, {f}));')
    lines += ["return 0; }"]
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-o", str(exe), str(src)], check=True)
    got = {}
    for line in subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.splitlines():
        c, f, v = line.split()
        got[(c, f)] = int(v)
    for cname, py in structs.items():
        assert got[(cname, "size")] == ctypes.sizeof(py), cname
        for f, _ in py._fields_:
            assert got[(cname, f)] == getattr(py, f).offset, (cname, f)


def test_error_path_without_gpu_reports_message():
    lib = _lib.load()
    b = ctypes.c_size_t()
    assert lib.lg_filter_workspace_bytes(2, 10, 12, ctypes.byref(b)) == 0 and b.value > 0
    rc = lib.lg_filter_matches(None, 1, 1, 1, 0.0, None, None, None, None, None, 0, None)
    assert rc == _lib.LG_E_INVALID
    assert b"null" in lib.lg_last_error()


def test_module_schema_matches_reference_schema():
    from lightglue_amd import LightGlue

    for conf in ({}, {"add_scale_ori": True}, {"input_dim": 128}, {"n_layers": 3}):
        m = LightGlue(conf)
        sd = m.state_dict()
        schema = state_dict_schema(conf)
        assert list(sd.keys()) == [n for n, _ in schema]
        for n, shape in schema:
            assert tuple(sd[n].shape) == tuple(shape), n


def test_default_conf_keys_match_reference():
    # lightglue.py:341-361
    assert set(DEFAULT_CONF) == {
        "name", "input_dim", "add_scale_ori", "descriptor_dim", "n_layers", "num_heads", "flash", "mp",
        "depth_confidence", "width_confidence", "filter_threshold", "checkpointed", "weights",
        "weights_from_version", "loss",
    }


def test_checkpoint_key_renames(tmp_path):
    """Old 'self_attn.{i}' / 'cross_attn.{i}' keys are renamed like lightglue.py:424-429."""
    from lightglue_amd import LightGlue

    sd = synthetic_state_dict({}, seed=3)
    old = {}
    for k, v in sd.items():
        k2 = re.sub(r"^transformers\.(\d+)\.self_attn", r"self_attn.\1", k)
        k2 = re.sub(r"^transformers\.(\d+)\.cross_attn", r"cross_attn.\1", k2)
        old[k2] = torch.from_numpy(v)
    p = tmp_path / "w.pth"
    torch.save(old, p)
    m = LightGlue({"weights": str(p)})
    got = m.state_dict()
    for k, v in sd.items():
        assert torch.equal(got[k], torch.from_numpy(v)), k


def test_forward_refuses_cpu_inputs():
    from lightglue_amd import LightGlue

    m = LightGlue({})
    data = {k: torch.from_numpy(v) for k, v in synthetic_pair(B=1, M=8, seed=0).items()}
    with pytest.raises((RuntimeError, AssertionError)):
        m(data)


def test_assignment_helpers_refuse_cpu():
    from lightglue_amd import filter_matches, log_optimal_transport

    with pytest.raises(RuntimeError):
        filter_matches(torch.zeros(1, 3, 3), 0.1)
    with pytest.raises(RuntimeError):
        log_optimal_transport(torch.zeros(1, 3, 3), 1.0, 3)


def test_synthetic_recipes_are_deterministic():
    a = synthetic_state_dict({}, seed=0)
    b = synthetic_state_dict({}, seed=0)
    assert all(np.array_equal(a[k], b[k]) for k in a)
    p, q = synthetic_pair(B=2, M=20, N=30, seed=1), synthetic_pair(B=2, M=20, N=30, seed=1)
    assert all(np.array_equal(p[k], q[k]) for k in p)
    assert p["keypoints1"].shape == (2, 30, 2)
    np.testing.assert_allclose(np.linalg.norm(p["descriptors1"], axis=-1), 1.0, atol=1e-5)


def test_superpoint_module_schema_matches_reference_schema():
    """lightglue_amd.SuperPoint registers the reference's conv modules (superpoint.py:174-196), so
    its state dict has the recipe schema's keys, order and shapes for every head combination."""
    from lightglue_amd.sp_weights import SP_DEFAULT_CONF, superpoint_schema
    from lightglue_amd.superpoint import SuperPoint

    for conf in ({}, {"has_detector": False, "sparse_outputs": False}, {"has_descriptor": False, "sparse_outputs": False}):
        sd = SuperPoint(conf).state_dict()
        schema = superpoint_schema(conf)
        assert list(sd.keys()) == [n for n, _ in schema]
        for n, shape in schema:
            assert tuple(sd[n].shape) == tuple(shape), n
    assert set(SP_DEFAULT_CONF) == {  # superpoint.py:153-169 + base_model.py:54-59
        "name", "trainable", "freeze_batch_normalization", "timeit", "has_detector", "has_descriptor",
        "descriptor_dim", "sparse_outputs", "dense_outputs", "nms_radius", "refinement_radius",
        "detection_threshold", "max_num_keypoints", "max_num_keypoints_val", "force_num_keypoints",
        "randomize_keypoints_training", "remove_borders", "legacy_sampling"}


def test_superpoint_registered_in_pipeline():
    from lightglue_amd import pipeline
    from lightglue_amd.superpoint import SuperPoint

    for name in ("gluefactory_nonfree.superpoint", "extractors.superpoint", "superpoint"):
        assert pipeline.get_model(name) is SuperPoint


def test_superpoint_cpu_input_raises():
    from lightglue_amd.superpoint import SuperPoint

    with pytest.raises(RuntimeError, match="HIP device"):
        SuperPoint({})({"image": torch.zeros(1, 1, 64, 64)})


def test_superglue_module_schema_matches_reference_schema():
    """The parameter containers' state dict is the reference's (superglue.py:63-139,239-247)."""
    from lightglue_amd import SuperGlue
    from lightglue_amd.sg_weights import superglue_schema

    for conf in ({}, {"use_scores": False, "GNN_layers": ["cross", "self"]}, {"keypoint_encoder": [16, 64]}):
        sd = SuperGlue(conf).state_dict()
        schema = superglue_schema(conf)
        assert list(sd.keys()) == [n for n, _, _ in schema]
        for n, shape, _ in schema:
            assert tuple(sd[n].shape) == tuple(shape), n


def test_superglue_registry_and_cpu_inputs_raise():
    import torch

    from lightglue_amd import SuperGlue
    from lightglue_amd.pipeline import get_model

    assert get_model("gluefactory_nonfree.superglue") is SuperGlue and get_model("superglue") is SuperGlue
    m = SuperGlue({"GNN_layers": ["self"]}).eval()
    view = {"image": torch.zeros(1, 1, 48, 64)}
    data = {"view0": view, "view1": view, "keypoints0": torch.rand(1, 5, 2) * 40,
            "keypoints1": torch.rand(1, 6, 2) * 40, "descriptors0": torch.rand(1, 5, 256),
            "descriptors1": torch.rand(1, 6, 256), "keypoint_scores0": torch.rand(1, 5),
            "keypoint_scores1": torch.rand(1, 6)}
    with pytest.raises(RuntimeError, match="HIP device"):
        m(data)
    # empty view: the reference's early return (superglue.py:257-264), int32 matches
    out = m({**data, "keypoints1": torch.zeros(1, 0, 2), "descriptors1": torch.zeros(1, 0, 256),
             "keypoint_scores1": torch.zeros(1, 0)})
    assert out["matches0"].dtype == torch.int32 and (out["matches0"] == -1).all() and out["matches1"].shape == (1, 0)
    with pytest.raises(ValueError):
        SuperGlue({"GNN_layers": ["self", "both"]})


def test_bench_training_ground_truth_is_one_to_one():
    """bench.py --workload train*: the seeded ground truth of the synthetic pairs is one-to-one,
    consistent across gt_matches0 / gt_matches1 / gt_assignment, and leaves about a third unmatched;
    the training flop model counts the forward linears three times (y, dx, dW)."""
    import bench

    d = bench.gpu_pairs(3, 96, 256, 1, torch.device("cpu"))
    g = bench.gpu_ground_truth(d, 7)
    m0, m1, a = g["gt_matches0"], g["gt_matches1"], g["gt_assignment"]
    b, i = torch.nonzero(m0 > -1, as_tuple=True)
    assert (m1[b, m0[b, i]] == i).all()
    b, j = torch.nonzero(m1 > -1, as_tuple=True)
    assert (m0[b, m1[b, j]] == j).all()
    assert int(a.sum()) == int((m0 > -1).sum()) == int((m1 > -1).sum())
    assert (a.sum(2) <= 1).all() and (a.sum(1) <= 1).all()
    frac = float((m0 > -1).float().mean())
    assert 0.45 < frac < 0.8
    assert bench.train_flops_per_pair(2048) > 3 * 9 * 76 * 2048 * 256 * 256


def test_layer_slices_gradient_matches_indexing():
    """lightglue._LayerSlices (loss(): the per-layer head inputs) gives the same slices and the same
    [B, L, M, D] gradient as indexing rd[:, i], including layers whose slice gets no gradient."""
    import torch
    from lightglue_amd.lightglue import _LayerSlices

    g = torch.Generator().manual_seed(3)
    rd = torch.randn(2, 4, 5, 3, generator=g, dtype=torch.float64)
    r = [torch.randn(2, 5, 3, generator=g, dtype=torch.float64) for _ in range(4)]
    a = rd.clone().requires_grad_()
    sl = _LayerSlices.apply(a)
    assert all(s.is_contiguous() and torch.equal(s, rd[:, i]) for i, s in enumerate(sl))
    sum((sl[i] * r[i]).sum() * (i + 1) for i in (0, 1, 3)).backward()  # layer 2 unused
    b = rd.clone().requires_grad_()
    sum((b[:, i] * r[i]).sum() * (i + 1) for i in (0, 1, 3)).backward()
    assert torch.equal(a.grad, b.grad)
