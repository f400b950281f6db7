"""Load golden fixtures and regenerate their inputs/weights from the committed recipe."""
import glob
import json
import os

import numpy as np

import lgamd  # noqa: F401
from lightglue_amd.weights import synthetic_pair, synthetic_state_dict

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
PRUNE_BIAS = [-2.97, -2.32, -2.90, -2.29, -3.00, -2.80, -2.14, -2.37]


def case_names(prefix=""):
    return sorted(
        os.path.basename(p)[:-4]
        for p in glob.glob(os.path.join(HERE, "*.npz"))
        if os.path.basename(p).startswith(prefix) and not os.path.basename(p).startswith(("sinkhorn", "sp_", "sg_", "loss_", "grad_", "configs4", "sgtrain_"))
    )


def sinkhorn_names():
    return sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(HERE, "sinkhorn*.npz")))


def load(name):
    z = np.load(os.path.join(HERE, name + ".npz"), allow_pickle=False)
    out = {k: z[k] for k in z.files}
    out["meta"] = json.loads(str(out.pop("meta_json")))
    return out


def case_inputs(meta):
    """(conf, weights, data) exactly as tests/golden/make_golden.py built them."""
    conf = dict(meta["conf"])
    sd = synthetic_state_dict(conf, **meta["weights"])
    over = meta.get("overrides", {})
    L = conf.get("n_layers", 9)
    if "matchability_bias" in over:
        for i in range(L - 1):
            if over["matchability_bias"][i] is not None:
                sd[f"log_assignment.{i}.matchability.bias"][:] = over["matchability_bias"][i]
    if "token_bias" in over:
        for i in range(L - 1):
            if over["token_bias"][i] is not None:
                sd[f"token_confidence.{i}.token.0.bias"][:] = over["token_bias"][i]
    if "token_bias_layer" in over:
        li, val = over["token_bias_layer"]
        sd[f"token_confidence.{li}.token.0.bias"][:] = val
    if "final_proj_scale" in over:
        for k in sd:
            if k.startswith("log_assignment.") and ".final_proj." in k:
                sd[k] = (sd[k] * np.float32(over["final_proj_scale"])).astype(np.float32)
    pkw = dict(meta["pair"])
    data = synthetic_pair(**pkw)
    if conf.get("add_scale_ori"):
        B, M = pkw["B"], pkw["M"]
        N = pkw.get("N", M)
        rng = np.random.Generator(np.random.PCG64(pkw["seed"] + 1000))
        data.update(
            {
                "scales0": (rng.random((B, M)) * 2).astype(np.float32),
                "oris0": (rng.random((B, M)) * 6.28 - 3.14).astype(np.float32),
                "scales1": (rng.random((B, N)) * 2).astype(np.float32),
                "oris1": (rng.random((B, N)) * 6.28 - 3.14).astype(np.float32),
            }
        )
    return conf, sd, data


def sinkhorn_inputs(meta):
    rng = np.random.Generator(np.random.PCG64(meta["seed"]))
    return (rng.standard_normal((meta["B"], meta["M"], meta["N"])) * meta["scale"]).astype(np.float32)


def sha(arrs):
    import hashlib

    h = hashlib.sha256()
    for k in sorted(arrs):
        h.update(k.encode())
        h.update(np.ascontiguousarray(arrs[k]).tobytes())
    return h.hexdigest()
