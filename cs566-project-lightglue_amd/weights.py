"""State-dict schema of the reference LightGlue and deterministic weight/input recipes.

Schema: the parameter names and shapes that ``gluefactory.models.matchers.lightglue.LightGlue``
registers, in registration order (reference ``lightglue.py:367-398``):

* ``input_proj.{weight,bias}`` only when ``input_dim != descriptor_dim`` (``:370-373``)
* ``posenc.Wr.weight`` [F/2, 2+2*add_scale_ori] and ``posenc.condition_modulation.{weight,bias}``
  [F/2, 1], [F/2] with F = head_dim (``:50-61,380-381``)
* ``transformers.{i}.self_attn.{Wqkv,out_proj}``, ``...self_attn.ffn.{0,1,3}`` (``:159-176``)
* ``transformers.{i}.cross_attn.{to_qk,to_v,to_out}``, ``...cross_attn.ffn.{0,1,3}`` (``:194-211``)
* ``log_assignment.{i}.{matchability,final_proj}`` (``:299-304``)
* ``token_confidence.{i}.token.0`` for i < n_layers-1 (``:96-99``)

Recipes (used by tests, smoke and bench; never by the product path):

* :func:`synthetic_state_dict` draws every tensor, in schema order, from one NumPy PCG64
  stream: uniform(-1/sqrt(fan_in), 1/sqrt(fan_in)) like PyTorch's default ``nn.Linear`` init,
  LayerNorm weight 1 / bias 0, ``Wr`` standard normal (``:58``), ``condition_modulation``
  uniform(-1, 1) (its fan_in is 1).  ``sharpen=True`` scales ``final_proj`` by 4 and sets the
  matchability bias to 2, so the assignment is decisive instead of ~1e-4 flat.
* :func:`synthetic_pair` makes a pair batch per SURVEY §8(d): keypoints uniform in the image,
  L2-normalised N(0,1) descriptors, view 1 a permuted, noised copy of view 0.
"""
from collections import OrderedDict

import numpy as np

DEFAULT_CONF = {
    "name": "lightglue",
    "input_dim": 256,
    "add_scale_ori": False,
    "descriptor_dim": 256,
    "n_layers": 9,
    "num_heads": 4,
    "flash": False,
    "mp": False,
    "depth_confidence": -1,
    "width_confidence": -1,
    "filter_threshold": 0.0,
    "checkpointed": False,
    "weights": None,
    "weights_from_version": "v0.1_arxiv",
    "loss": {"gamma": 1.0, "fn": "nll", "nll_balancing": 0.5},
}


def _ffn(prefix, d):
    return [
        (f"{prefix}.ffn.0.weight", (2 * d, 2 * d)),
        (f"{prefix}.ffn.0.bias", (2 * d,)),
        (f"{prefix}.ffn.1.weight", (2 * d,)),
        (f"{prefix}.ffn.1.bias", (2 * d,)),
        (f"{prefix}.ffn.3.weight", (d, 2 * d)),
        (f"{prefix}.ffn.3.bias", (d,)),
    ]


def state_dict_schema(conf=None):
    """List of (name, shape) in the reference's registration order (lightglue.py:367-398)."""
    c = dict(DEFAULT_CONF)
    c.update(conf or {})
    d, h, L = int(c["descriptor_dim"]), int(c["num_heads"]), int(c["n_layers"])
    din = int(c["input_dim"])
    hd = d // h
    m_in = 2 + 2 * int(bool(c["add_scale_ori"]))
    out = []
    if din != d:
        out += [("input_proj.weight", (d, din)), ("input_proj.bias", (d,))]
    out += [
        ("posenc.Wr.weight", (hd // 2, m_in)),
        ("posenc.condition_modulation.weight", (hd // 2, 1)),
        ("posenc.condition_modulation.bias", (hd // 2,)),
    ]
    for i in range(L):
        s = f"transformers.{i}.self_attn"
        out += [
            (f"{s}.Wqkv.weight", (3 * d, d)),
            (f"{s}.Wqkv.bias", (3 * d,)),
            (f"{s}.out_proj.weight", (d, d)),
            (f"{s}.out_proj.bias", (d,)),
        ] + _ffn(s, d)
        x = f"transformers.{i}.cross_attn"
        out += [
            (f"{x}.to_qk.weight", (d, d)),
            (f"{x}.to_qk.bias", (d,)),
            (f"{x}.to_v.weight", (d, d)),
            (f"{x}.to_v.bias", (d,)),
            (f"{x}.to_out.weight", (d, d)),
            (f"{x}.to_out.bias", (d,)),
        ] + _ffn(x, d)
    for i in range(L):
        a = f"log_assignment.{i}"
        out += [
            (f"{a}.matchability.weight", (1, d)),
            (f"{a}.matchability.bias", (1,)),
            (f"{a}.final_proj.weight", (d, d)),
            (f"{a}.final_proj.bias", (d,)),
        ]
    for i in range(L - 1):
        out += [
            (f"token_confidence.{i}.token.0.weight", (1, d)),
            (f"token_confidence.{i}.token.0.bias", (1,)),
        ]
    return out


def _fan_in(name, shape, schema_shapes):
    if name.endswith(".weight"):
        return shape[1] if len(shape) == 2 else None
    wshape = schema_shapes.get(name[: -len("bias")] + "weight")
    return wshape[1] if wshape is not None and len(wshape) == 2 else None


def synthetic_state_dict(conf=None, seed=0, sharpen=True):
    """Deterministic fp32 weights (NumPy PCG64), keyed like the reference state dict."""
    schema = state_dict_schema(conf)
    shapes = dict(schema)
    rng = np.random.Generator(np.random.PCG64(seed))
    sd = OrderedDict()
    for name, shape in schema:
        if ".ffn.1." in name:  # LayerNorm(elementwise_affine=True) default init
            v = np.ones(shape) if name.endswith("weight") else np.zeros(shape)
            rng.random(shape)  # keep the stream position independent of the branch
        elif name == "posenc.Wr.weight":
            v = rng.standard_normal(shape)
        else:
            fan = _fan_in(name, shape, shapes)
            bound = 1.0 / np.sqrt(fan) if fan else 1.0
            v = (rng.random(shape) * 2.0 - 1.0) * bound
        sd[name] = v.astype(np.float32)
    if sharpen:
        for name in sd:
            if name.startswith("log_assignment.") and ".final_proj." in name:
                sd[name] = (sd[name] * 4.0).astype(np.float32)
            if name.startswith("log_assignment.") and name.endswith("matchability.bias"):
                sd[name] = np.full_like(sd[name], 2.0)
    return sd


# configs[3] recipe (N = 2048, width = depth = 0.95): per-layer token-confidence and matchability
# biases on top of the seed-8 weights, found by tools/tune_prune_golden.py -- layers 0..4 prune
# ~10 % of the points each, layer 5 fires the early stop; every decision threshold sits in a
# >= 1e-3 gap of the sorted decision logits.  None = keep the recipe value.
PRUNE2K_TOKEN_BIAS = [2.0127, 2.2824, 1.7838, 1.715, 0.9317, 6.3066, None, None]
PRUNE2K_MATCH_BIAS = [-2.5056, -2.4873, -1.8882, -3.3078, -2.4224, None, None, None]


def prune_recipe_state_dict(conf=None, seed=8):
    """Weights that really prune and stop early at N = 2048 (the configs[3] workload and the
    ``prune_depth_width_n2048`` golden): ``synthetic_state_dict(conf, seed)`` with the biases above."""
    sd = synthetic_state_dict(conf, seed=seed)
    for i, (tb, mb) in enumerate(zip(PRUNE2K_TOKEN_BIAS, PRUNE2K_MATCH_BIAS)):
        if tb is not None and f"token_confidence.{i}.token.0.bias" in sd:
            sd[f"token_confidence.{i}.token.0.bias"][:] = tb
        if mb is not None and f"log_assignment.{i}.matchability.bias" in sd:
            sd[f"log_assignment.{i}.matchability.bias"][:] = mb
    return sd


def synthetic_pair(B, M, N=None, dim=256, seed=1, width=640, height=640, noise=0.05, kpt_noise=1.0):
    """Synthetic pair batch.  Returns a dict of NumPy arrays.

    keypoints0 [B,M,2] uniform in [0,width)x[0,height); descriptors0 [B,M,dim] L2-normalised
    N(0,1); view 1 takes a random permutation of view 0 (padded with fresh points when N > M),
    adds pixel noise to keypoints and Gaussian noise to descriptors, then re-normalises.
    """
    N = M if N is None else N
    rng = np.random.Generator(np.random.PCG64(seed))
    size = np.array([width, height], np.float64)
    k0 = rng.random((B, M, 2)) * size
    d0 = rng.standard_normal((B, M, dim))
    d0 /= np.linalg.norm(d0, axis=-1, keepdims=True)
    k1 = np.empty((B, N, 2))
    d1 = np.empty((B, N, dim))
    for b in range(B):
        perm = rng.permutation(max(M, N))[:N]
        hit = perm < M
        src = np.minimum(perm, M - 1)
        kn = rng.standard_normal((N, 2)) * kpt_noise
        dn = rng.standard_normal((N, dim)) * noise
        kf = rng.random((N, 2)) * size
        df = rng.standard_normal((N, dim))
        k1[b] = np.where(hit[:, None], k0[b, src] + kn, kf)
        d1[b] = np.where(hit[:, None], d0[b, src] + dn, df)
    k1 = np.clip(k1, 0.0, size - 1e-3)
    d1 /= np.linalg.norm(d1, axis=-1, keepdims=True)
    isz = np.tile(size[None], (B, 1))
    return {
        "keypoints0": k0.astype(np.float32),
        "keypoints1": k1.astype(np.float32),
        "descriptors0": d0.astype(np.float32),
        "descriptors1": d1.astype(np.float32),
        "image_size0": isz.astype(np.float32),
        "image_size1": isz.astype(np.float32),
    }
