"""The C-ABI from a non-Python host (examples/c_host/lg_c_host.c: plain C99 + the HIP runtime's C
API): the reference's LightGlue.__init__ + forward (gluefactory/models/matchers/lightglue.py:367-430,
444-579) driven through include/lightglue_mi355x.h alone -- state dict in, matches and scores out --
gives the same matches0/1 and matching_scores0/1 as the Python drop-in class on the same weights
and inputs (both run the same deterministic kernels: bit for bit), and those match the CPU oracle's
indices.  The binary is built in-tree by the library's Makefile (__graft_entry__.build())."""
import os
import struct
import subprocess

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "examples", "c_host", "lg_c_host")
pytestmark = pytest.mark.gpu


def _write_weights(path, sd):
    with open(path, "wb") as f:
        f.write(b"LGW1" + struct.pack("<I", len(sd)))
        for k, v in sd.items():
            a = np.ascontiguousarray(v, dtype=np.float32)
            f.write(struct.pack("<I", len(k)) + k.encode() + struct.pack("<q", a.size) + a.tobytes())


def _write_inputs(path, d):
    B, M, _ = d["keypoints0"].shape
    N = d["keypoints1"].shape[1]
    with open(path, "wb") as f:
        f.write(b"LGI1" + struct.pack("<iii", B, M, N))
        for k in ("keypoints0", "keypoints1", "descriptors0", "descriptors1", "image_size0", "image_size1"):
            f.write(np.ascontiguousarray(d[k], dtype=np.float32).tobytes())


def _read_outputs(path):
    raw = open(path, "rb").read()
    assert raw[:4] == b"LGO1"
    B, M, N = struct.unpack("<iii", raw[4:16])
    o = 16
    out = {}
    for k, n, dt in (("matches0", B * M, np.int64), ("matches1", B * N, np.int64),
                     ("matching_scores0", B * M, np.float32), ("matching_scores1", B * N, np.float32)):
        a = np.frombuffer(raw, dtype=dt, count=n, offset=o)
        o += a.nbytes
        out[k] = a.reshape(B, -1)
    return out


@pytest.mark.parametrize("adaptive", [False, True], ids=["fixed_depth", "early_stop_and_pruning"])
def test_c_host_forward_equals_python_forward(tmp_path, adaptive):
    """adaptive: the golden case prune_depth_width_n2048 (depth / width confidence 0.95, weights that
    make the reference stop early and prune, lightglue.py:502-540, from tests/golden/make_golden.py):
    the C host against the Python class bit for bit, and against the reference's own matches and
    stop layer stored in the golden."""
    import lgamd  # noqa: F401
    import oracle
    from golden_util import case_inputs, load
    from lightglue_amd import LightGlue
    from lightglue_amd.weights import synthetic_pair, synthetic_state_dict

    assert os.path.exists(EXE), "examples/c_host/lg_c_host is built by make -C cs566-project-lightglue_amd/csrc"
    if adaptive:
        g = load("prune_depth_width_n2048")
        conf, sd, data = case_inputs(g["meta"])
        args = [repr(conf["filter_threshold"]), repr(conf["depth_confidence"]), repr(conf["width_confidence"])]
    else:
        conf = {"filter_threshold": 0.1}
        sd = synthetic_state_dict(conf, seed=0)
        data = synthetic_pair(B=2, M=300, N=277, seed=9)
        args = ["0.1"]
    w, i, o = (str(tmp_path / n) for n in ("w.bin", "i.bin", "o.bin"))
    _write_weights(w, sd)
    _write_inputs(i, data)
    r = subprocess.run([EXE, w, i, o] + args, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    got = _read_outputs(o)

    dev = torch.device("cuda", 0)
    model = LightGlue(conf).eval().to(dev)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
    feed = {k: torch.from_numpy(v).to(dev) for k, v in data.items() if not k.startswith("image_size")}
    feed["view0"] = {"image_size": torch.from_numpy(data["image_size0"]).to(dev)}
    feed["view1"] = {"image_size": torch.from_numpy(data["image_size1"]).to(dev)}
    with torch.no_grad():
        pred = model(feed)
    for k in ("matches0", "matches1", "matching_scores0", "matching_scores1"):
        np.testing.assert_array_equal(got[k], pred[k].cpu().numpy(), err_msg=k)
    if adaptive:
        # lg_outputs_t.stop_layer as the C host printed it; the golden's layer count is the reference's
        stop = int(r.stdout.split("stop layer ")[1].split()[0])
        assert stop + 1 == int(g["n_layers_run"]) < conf.get("n_layers", 9), (stop, g["n_layers_run"])
        assert np.asarray(g["prune0"]).min() < np.asarray(g["prune0"]).max()  # the case does prune
        np.testing.assert_array_equal(got["matches0"], np.asarray(g["matches0"]))
        return
    ref = oracle.lightglue_forward(sd, data, conf)
    np.testing.assert_array_equal(got["matches0"], ref["matches0"].numpy())
    np.testing.assert_allclose(got["matching_scores0"], ref["matching_scores0"].numpy(), atol=1e-4)
    assert (got["matches0"] > -1).sum() > 0
