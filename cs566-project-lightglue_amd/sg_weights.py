"""SuperGlue configuration, state-dict schema and deterministic recipe weights.

The schema is the reference module tree (``gluefactory_nonfree/superglue.py``):

* ``kenc.encoder`` -- ``MLP([3 or 2] + keypoint_encoder + [D])`` (``:63-72,89-104``): Conv1d(k=1)
  layers at indices 0, 3, 6, ... with BatchNorm1d + ReLU between them;
* ``gnn.layers.<i>.attn.proj.{0,1,2}`` / ``attn.merge`` -- the q/k/v projections and the head
  merge of ``MultiHeadedAttention`` (``:113-128``), Conv1d(D, D, 1) each;
* ``gnn.layers.<i>.mlp`` -- ``MLP([2D, 2D, D])`` (``:131-139``): Conv1d, BatchNorm1d, ReLU, Conv1d;
* ``final_proj`` (Conv1d(D, D, 1)) and the scalar ``bin_score`` (``:244-248``).

Conv1d weights are ``[out, in, 1]``; BatchNorm1d carries ``weight``, ``bias``, ``running_mean``,
``running_var`` and the int64 ``num_batches_tracked`` buffer (state-dict only, not used in eval).

The recipe (NumPy PCG64, host only) draws Conv1d weights and biases uniform(+-1/sqrt(fan_in))
like torch's default init, BatchNorm affine parameters and running statistics away from the
identity (so folding them is exercised), and ``sharpen`` scales the residual MLP outputs and the
keypoint encoding down and ``final_proj`` up, so the final descriptors stay distinctive after 18
random layers (the Sinkhorn assignment then keeps confident matches whose argmaxes have margins
well above fp32 rounding).
"""
from collections import OrderedDict

import numpy as np

SG_DEFAULT_CONF = {
    "descriptor_dim": 256,
    "weights": "outdoor",
    "keypoint_encoder": [32, 64, 128, 256],
    "GNN_layers": ["self", "cross"] * 9,
    "num_sinkhorn_iterations": 50,
    "filter_threshold": 0.2,
    "use_scores": True,
    "loss": {"nll_balancing": 0.5},
}


def merged_conf(conf=None):
    c = dict(SG_DEFAULT_CONF)
    for k, v in (conf or {}).items():
        if k == "loss":
            c["loss"] = {**SG_DEFAULT_CONF["loss"], **(v or {})}
        else:
            c[k] = v
    c["keypoint_encoder"] = list(c["keypoint_encoder"])
    c["GNN_layers"] = list(c["GNN_layers"])
    return c


def _mlp(prefix, channels):
    """(name, shape, kind) of ``MLP(channels)`` (superglue.py:63-72)."""
    out, idx = [], 0
    for i in range(1, len(channels)):
        out += [(f"{prefix}.{idx}.weight", (channels[i], channels[i - 1], 1), "conv_w"),
                (f"{prefix}.{idx}.bias", (channels[i],), "conv_b")]
        idx += 1
        if i < len(channels) - 1:
            n = channels[i]
            out += [(f"{prefix}.{idx}.weight", (n,), "bn_w"), (f"{prefix}.{idx}.bias", (n,), "bn_b"),
                    (f"{prefix}.{idx}.running_mean", (n,), "bn_mean"), (f"{prefix}.{idx}.running_var", (n,), "bn_var"),
                    (f"{prefix}.{idx}.num_batches_tracked", (), "bn_count")]
            idx += 2  # BatchNorm1d, ReLU
    return out


def superglue_schema(conf=None):
    """[(name, shape, kind)] in the reference's state-dict order."""
    c = merged_conf(conf)
    d = c["descriptor_dim"]
    # the module's own parameter (registered last, :246-247) comes first in a state dict
    out = [("bin_score", (), "scalar")]
    out += _mlp("kenc.encoder", [3 if c["use_scores"] else 2] + c["keypoint_encoder"] + [d])
    for i in range(len(c["GNN_layers"])):
        p = f"gnn.layers.{i}"
        out += [(f"{p}.attn.merge.weight", (d, d, 1), "conv_w"), (f"{p}.attn.merge.bias", (d,), "conv_b")]
        for j in range(3):
            out += [(f"{p}.attn.proj.{j}.weight", (d, d, 1), "conv_w"), (f"{p}.attn.proj.{j}.bias", (d,), "conv_b")]
        out += _mlp(f"{p}.mlp", [2 * d, 2 * d, d])
    out += [("final_proj.weight", (d, d, 1), "conv_w"), ("final_proj.bias", (d,), "conv_b")]
    return out


def superglue_state_dict(conf=None, seed=0, sharpen=True):
    """Deterministic weights keyed like the reference state dict (float32; the BatchNorm counters
    int64)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    sd = OrderedDict()
    for name, shape, kind in superglue_schema(conf):
        if kind == "conv_w":
            bound = 1.0 / np.sqrt(shape[1])
            v = (rng.random(shape) * 2.0 - 1.0) * bound
        elif kind == "conv_b":
            bound = 1.0 / np.sqrt(sd[name[: -len("bias")] + "weight"].shape[1])
            v = (rng.random(shape) * 2.0 - 1.0) * bound
        elif kind == "bn_w":
            v = 0.5 + rng.random(shape)
        elif kind == "bn_b":
            v = (rng.random(shape) - 0.5) * 0.2
        elif kind == "bn_mean":
            v = rng.standard_normal(shape) * 0.1
        elif kind == "bn_var":
            v = 0.5 + 1.5 * rng.random(shape)
        elif kind == "bn_count":
            sd[name] = np.array(0, np.int64)
            continue
        else:  # bin_score (superglue.py:246)
            v = np.array(1.0)
        sd[name] = np.asarray(v, np.float32)
    if sharpen:
        last_kenc = f"kenc.encoder.{3 * len(merged_conf(conf)['keypoint_encoder'])}."
        for name in sd:
            if ".mlp.3." in name:
                sd[name] = (sd[name] * 0.05).astype(np.float32)
            if name.startswith(last_kenc):
                sd[name] = (sd[name] * 0.1).astype(np.float32)
            if name.startswith("final_proj."):
                sd[name] = (sd[name] * 20.0).astype(np.float32)
    return sd


def synthetic_scores(B, N, seed=3):
    """Keypoint scores in (0, 1) for the keypoint encoder's third input channel."""
    rng = np.random.Generator(np.random.PCG64(seed))
    return rng.random((B, N)).astype(np.float32)
