"""Functional torch-CPU restatement of the reference SuperGlue matcher and the NLL losses — TEST
ORACLE.

Test infrastructure only (see ``oracle/__init__.py``).  Every function cites the reference lines
it restates; paths are relative to ``/root/reference``.  Weights are a plain dict keyed like the
reference state dict (``lightglue_amd.sg_weights.superglue_schema``).  Pinned against the
reference's own outputs in ``tests/golden/sg_*.npz`` (``tests/test_oracle_superglue.py``).

``dtype=torch.float64`` runs the same algorithm in double precision.
"""
import numpy as np
import torch

from .lightglue_ref import filter_matches, log_optimal_transport

BN_EPS = 1e-5  # torch.nn.BatchNorm1d default


def _t(w, dtype):
    return torch.as_tensor(np.asarray(w)).to(dtype)


def _conv1(W, name, x, dtype):
    """Conv1d(kernel_size=1) on [B, C, N]."""
    w = _t(W[name + ".weight"], dtype)[:, :, 0]
    return torch.einsum("oc,bcn->bon", w, x) + _t(W[name + ".bias"], dtype)[None, :, None]


def _bn(W, name, x, dtype):
    """BatchNorm1d in eval mode (running statistics)."""
    m, v = _t(W[name + ".running_mean"], dtype), _t(W[name + ".running_var"], dtype)
    g, b = _t(W[name + ".weight"], dtype), _t(W[name + ".bias"], dtype)
    return (x - m[None, :, None]) / torch.sqrt(v[None, :, None] + BN_EPS) * g[None, :, None] + b[None, :, None]


def mlp(W, prefix, channels, x, dtype):
    """superglue.py:63-72: Conv1d / BatchNorm1d / ReLU stacks, no activation after the last."""
    idx = 0
    for i in range(1, len(channels)):
        x = _conv1(W, f"{prefix}.{idx}", x, dtype)
        idx += 1
        if i < len(channels) - 1:
            x = torch.relu(_bn(W, f"{prefix}.{idx}", x, dtype))
            idx += 2
    return x


def normalize_keypoints(kpts, size):
    """superglue.py:75-86; ``size`` [B, 2] (w, h)."""
    shift = size / 2
    scale = size.max(1).values * 0.7
    return (kpts - shift[:, None]) / scale[:, None, None]


def attention(q, k, v):
    """superglue.py:107-111 on [B, dim, H, N]."""
    dim = q.shape[1]
    scores = torch.einsum("bdhn,bdhm->bhnm", q, k) / dim ** 0.5
    prob = torch.softmax(scores, dim=-1)
    return torch.einsum("bhnm,bdhm->bdhn", prob, v)


def propagation(W, p, x, source, dtype, heads=4):
    """AttentionalPropagation (superglue.py:131-139) with MultiHeadedAttention (:113-128)."""
    b, d = x.shape[0], x.shape[1]
    q, k, v = [_conv1(W, f"{p}.attn.proj.{j}", t, dtype).view(b, d // heads, heads, -1) for j, t in
               enumerate((x, source, source))]
    msg = _conv1(W, f"{p}.attn.merge", attention(q, k, v).contiguous().view(b, d, -1), dtype)
    return mlp(W, f"{p}.mlp", [2 * d, 2 * d, d], torch.cat([x, msg], dim=1), dtype)


def superglue_forward(W, data, conf, dtype=torch.float32):
    """SuperGlue._forward (superglue.py:253-307) in eval mode.

    ``data``: keypoints0/1 [B, N, 2], descriptors0/1 [B, N, D], keypoint_scores0/1 [B, N], and
    ``image_size`` [B, 2] (w, h) or ``image_hw`` (H, W) for the image-shape fallback (:78-83).
    """
    from lightglue_amd.sg_weights import merged_conf

    c = merged_conf(conf)
    k0, k1 = _t(data["keypoints0"], dtype), _t(data["keypoints1"], dtype)
    B, M, N = k0.shape[0], k0.shape[1], k1.shape[1]
    if M == 0 or N == 0:  # :257-264
        return {"matches0": torch.full((B, M), -1, dtype=torch.int32), "matches1": torch.full((B, N), -1, dtype=torch.int32),
                "matching_scores0": torch.zeros(B, M, dtype=dtype), "matching_scores1": torch.zeros(B, N, dtype=dtype)}
    if data.get("image_size") is not None:
        size = _t(data["image_size"], dtype)
    else:
        h, w = data["image_hw"]
        size = torch.tensor([[float(w), float(h)]], dtype=dtype)
    n0, n1 = normalize_keypoints(k0, size), normalize_keypoints(k1, size)
    enc = [3 if c["use_scores"] else 2] + c["keypoint_encoder"] + [c["descriptor_dim"]]

    def kenc(kp, sc):  # :89-104
        inputs = [kp.transpose(1, 2)] + ([_t(sc, dtype)[:, None]] if c["use_scores"] else [])
        return mlp(W, "kenc.encoder", enc, torch.cat(inputs, dim=1), dtype)

    d0 = _t(data["descriptors0"], dtype).transpose(1, 2) + kenc(n0, data.get("keypoint_scores0"))
    d1 = _t(data["descriptors1"], dtype).transpose(1, 2) + kenc(n1, data.get("keypoint_scores1"))
    for i, name in enumerate(c["GNN_layers"]):  # AttentionalGNN (:148-170)
        p = f"gnn.layers.{i}"
        if name == "self":
            e0, e1 = propagation(W, p, d0, d0, dtype), propagation(W, p, d1, d1, dtype)
        elif name == "cross":
            e0, e1 = propagation(W, p, d0, d1, dtype), propagation(W, p, d1, d0, dtype)
        else:
            raise ValueError(name)
        d0, d1 = d0 + e0, d1 + e1
    md0, md1 = _conv1(W, "final_proj", d0, dtype), _conv1(W, "final_proj", d1, dtype)
    cost = torch.einsum("bdn,bdm->bnm", md0, md1) / c["descriptor_dim"] ** 0.5
    la = log_optimal_transport(cost, _t(W["bin_score"], dtype), c["num_sinkhorn_iterations"])
    m0, m1, s0, s1 = filter_matches(la, c["filter_threshold"])
    return {"sinkhorn_cost": cost, "log_assignment": la, "matches0": m0, "matches1": m1, "matching_scores0": s0,
            "matching_scores1": s1, "gnn_desc0": d0, "gnn_desc1": d1}


def superglue_loss(la, gt_assignment, gt_matches0, gt_matches1, nll_balancing=0.5, bin_score=None):
    """SuperGlue.loss (superglue.py:309-339): positives normalised by max(#positives, 1), the two
    dustbin terms together by max(#negatives0 + #negatives1, 1)."""
    la = torch.as_tensor(la)
    positive = torch.as_tensor(gt_assignment).to(la.dtype)
    num_pos = torch.max(positive.sum((1, 2)), positive.new_tensor(1))
    neg0 = (torch.as_tensor(gt_matches0) == -1).to(la.dtype)
    neg1 = (torch.as_tensor(gt_matches1) == -1).to(la.dtype)
    num_neg = torch.max(neg0.sum(1) + neg1.sum(1), neg0.new_tensor(1))
    nll_pos = -(la[:, :-1, :-1] * positive).sum((1, 2)) / num_pos
    nll_neg = (-(la[:, :-1, -1] * neg0).sum(1) - (la[:, -1, :-1] * neg1).sum(1)) / num_neg
    nll = nll_balancing * nll_pos + (1 - nll_balancing) * nll_neg
    out = {"total": nll, "assignment_nll": nll, "nll_pos": nll_pos, "nll_neg": nll_neg, "num_matchable": num_pos,
           "num_unmatchable": num_neg}
    if bin_score is not None:
        out["bin_score"] = torch.as_tensor(bin_score).reshape(1)
    return out


def nll_loss(la, gt_assignment, gt_matches0, gt_matches1, nll_balancing=0.5):
    """losses.py:6-73 NLLLoss: weights built by ``nll_loss`` (the column dustbin row is written at
    ``[:, -1, :m]``, so only M == N runs -- the reference raises otherwise), then ``weight_loss``
    with the two negative counts clamped separately."""
    la = torch.as_tensor(la)
    b, m1, n1 = la.shape
    m, n = m1 - 1, n1 - 1
    if m != n:
        raise RuntimeError(f"The expanded size of the tensor ({m}) must match the existing size ({n}) at non-singleton "
                           f"dimension 1.  Target sizes: [{b}, {m}].  Tensor sizes: [{b}, {n}]")
    w = torch.zeros_like(la)
    w[:, :m, :n] = torch.as_tensor(gt_assignment).to(la.dtype)
    w[:, :m, -1] = (torch.as_tensor(gt_matches0) == -1).to(la.dtype)
    w[:, -1, :m] = (torch.as_tensor(gt_matches1) == -1).to(la.dtype)
    sc = la * w
    num_neg0 = w[:, :m, -1].sum(-1).clamp(min=1.0)
    num_neg1 = w[:, -1, :n].sum(-1).clamp(min=1.0)
    num_pos = w[:, :m, :n].sum((-1, -2)).clamp(min=1.0)
    nll_pos = -sc[:, :m, :n].sum((-1, -2)) / num_pos.clamp(min=1.0)
    nll_neg = (-sc[:, :m, -1].sum(-1) - sc[:, -1, :n].sum(-1)) / (num_neg0 + num_neg1)
    nll = nll_balancing * nll_pos + (1 - nll_balancing) * nll_neg
    return nll, {"assignment_nll": nll, "nll_pos": nll_pos, "nll_neg": nll_neg, "num_matchable": num_pos,
                 "num_unmatchable": (num_neg0 + num_neg1) / 2.0}
