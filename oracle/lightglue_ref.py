"""Functional torch-CPU restatement of the reference LightGlue eval forward — TEST ORACLE.

Test infrastructure only (see ``oracle/__init__.py``).  Every function cites the reference
lines it restates; paths are relative to ``/root/reference``.  Weights are a plain dict keyed
like the reference state dict (``lightglue_amd.weights.state_dict_schema``).

Deliberate differences from the reference, all documented in DESIGN.md §2:

* early stop (``lightglue.py:527-531``): the reference reads an undefined
  ``self.confidence_thresholds`` (``:592,604``); here the thresholds are
  ``[confidence_threshold(i) for i in range(L)]`` (``:581-584``).  When the stop fires, the
  reference then crashes on ``torch.stack([])`` (``:572``); here ``ref_descriptors*`` hold the
  descriptors of the stopping layer.
* ``image_size`` missing: the reference raises ``UnboundLocalError`` (``:452-455``); here the
  min/max fallback of ``normalize_keypoints`` (``:25-26``) is used.

``dtype=torch.float64`` runs the same algorithm in double precision; the tests use it to find
near-tie rows whose argmax is not decidable at fp32.
"""
import math

import numpy as np
import torch
import torch.nn.functional as F


def _t(w, dtype):
    return torch.as_tensor(np.asarray(w)).to(dtype)


def normalize_keypoints(kpts, size=None):
    """lightglue.py:21-33: (k - size/2) / (max(size)/2); min/max fallback when size is None."""
    if size is None:
        size = 1 + kpts.max(-2).values - kpts.min(-2).values
    size = size.to(kpts)
    shift = size / 2
    scale = size.max(-1).values / 2
    return (kpts - shift[..., None, :]) / scale[..., None, None]


def positional_encoding(kpts_n, n_points, Wr, Wc, bc):
    """lightglue.py:63-77 (conditional Fourier PE), condition = float(N) per pair (:490-491).

    Returns (cos, sin), each [B, N, F/2]; the reference's ``repeat_interleave(2)`` (:77) is
    implicit: dims 2i and 2i+1 share frequency i.
    """
    proj = kpts_n @ Wr.T  # [B,N,F/2]
    cond = torch.full((kpts_n.shape[0], 1), float(n_points), dtype=kpts_n.dtype)
    cond = F.relu(cond) @ Wc.T + bc  # [B,F/2]
    proj = proj + cond[:, None, :]
    return torch.cos(proj), torch.sin(proj)


def _rotary(t, cos, sin):
    """lightglue.py:36-43: t*cos + rotate_half(t)*sin with interleaved pairs (2i, 2i+1)."""
    c = cos.repeat_interleave(2, dim=-1)[:, None]  # [B,1,N,hd]
    s = sin.repeat_interleave(2, dim=-1)[:, None]
    pairs = t.unflatten(-1, (-1, 2))
    rot = torch.stack((-pairs[..., 1], pairs[..., 0]), dim=-1).flatten(-2)
    return t * c + rot * s


def _linear(x, w, b):
    return F.linear(x, w, b)


def _ffn(x, msg, W, p):
    """lightglue.py:171-176,191: x + Lin(512->256)(GELU(LN(Lin(512->512)(cat[x,msg]))))."""
    h = _linear(torch.cat([x, msg], -1), W[p + ".ffn.0.weight"], W[p + ".ffn.0.bias"])
    h = F.layer_norm(h, (h.shape[-1],), W[p + ".ffn.1.weight"], W[p + ".ffn.1.bias"], eps=1e-5)
    h = F.gelu(h)
    return x + _linear(h, W[p + ".ffn.3.weight"], W[p + ".ffn.3.bias"])


def _softmax_attention(q, k, v, scale):
    """lightglue.py:146-149: softmax(q k^T * scale) v via torch's CPU SDPA (math backend)."""
    assert abs(scale - q.shape[-1] ** -0.5) < 1e-12
    return F.scaled_dot_product_attention(q.contiguous(), k.contiguous(), v.contiguous())


def self_block(x, cos, sin, W, p, H):
    """lightglue.py:178-191 SelfBlock.forward (eval, no mask)."""
    B, N, D = x.shape
    qkv = _linear(x, W[p + ".Wqkv.weight"], W[p + ".Wqkv.bias"])
    qkv = qkv.unflatten(-1, (H, -1, 3)).transpose(1, 2)  # [B,H,N,hd,3], layout [head][dh][qkv]
    q, k, v = qkv[..., 0], qkv[..., 1], qkv[..., 2]
    q, k = _rotary(q, cos, sin), _rotary(k, cos, sin)
    ctx = _softmax_attention(q, k, v, (D // H) ** -0.5)
    msg = _linear(ctx.transpose(1, 2).flatten(-2), W[p + ".out_proj.weight"], W[p + ".out_proj.bias"])
    return _ffn(x, msg, W, p)


def cross_block(x0, x1, W, p, H):
    """lightglue.py:220-249 CrossBlock.forward (non-flash path, eval, no mask)."""
    def heads(t):
        return t.unflatten(-1, (H, -1)).transpose(1, 2)

    qk0 = heads(_linear(x0, W[p + ".to_qk.weight"], W[p + ".to_qk.bias"]))
    qk1 = heads(_linear(x1, W[p + ".to_qk.weight"], W[p + ".to_qk.bias"]))
    v0 = heads(_linear(x0, W[p + ".to_v.weight"], W[p + ".to_v.bias"]))
    v1 = heads(_linear(x1, W[p + ".to_v.weight"], W[p + ".to_v.bias"]))
    s = (x0.shape[-1] // H) ** -0.5
    qk0, qk1 = qk0 * s ** 0.5, qk1 * s ** 0.5
    sim = torch.einsum("bhid,bhjd->bhij", qk0, qk1)
    m0 = torch.einsum("bhij,bhjd->bhid", torch.softmax(sim, -1), v1)
    m1 = torch.einsum("bhji,bhjd->bhid", torch.softmax(sim.transpose(-2, -1), -1).transpose(-2, -1), v0)
    m0 = _linear(m0.transpose(1, 2).flatten(-2), W[p + ".to_out.weight"], W[p + ".to_out.bias"])
    m1 = _linear(m1.transpose(1, 2).flatten(-2), W[p + ".to_out.weight"], W[p + ".to_out.bias"])
    return _ffn(x0, m0, W, p), _ffn(x1, m1, W, p)


def sigmoid_log_double_softmax(sim, z0, z1):
    """lightglue.py:284-296: [B,M+1,N+1] log assignment with dustbins."""
    b, m, n = sim.shape
    cert = F.logsigmoid(z0) + F.logsigmoid(z1).transpose(1, 2)
    s0 = F.log_softmax(sim, 2)
    s1 = F.log_softmax(sim.transpose(-1, -2), 2).transpose(-1, -2)
    out = sim.new_zeros((b, m + 1, n + 1))
    out[:, :m, :n] = s0 + s1 + cert
    out[:, :-1, -1] = F.logsigmoid(-z0.squeeze(-1))
    out[:, -1, :-1] = F.logsigmoid(-z1.squeeze(-1))
    return out


def match_assignment(d0, d1, W, p):
    """lightglue.py:306-315 MatchAssignment.forward."""
    md0 = _linear(d0, W[p + ".final_proj.weight"], W[p + ".final_proj.bias"])
    md1 = _linear(d1, W[p + ".final_proj.weight"], W[p + ".final_proj.bias"])
    dim = md0.shape[-1]
    md0, md1 = md0 / dim ** 0.25, md1 / dim ** 0.25
    sim = torch.einsum("bmd,bnd->bmn", md0, md1)
    z0 = _linear(d0, W[p + ".matchability.weight"], W[p + ".matchability.bias"])
    z1 = _linear(d1, W[p + ".matchability.weight"], W[p + ".matchability.bias"])
    return sigmoid_log_double_softmax(sim, z0, z1), sim


def filter_matches(scores, th):
    """lightglue.py:321-337 (identical to superglue.py:288-298): mutual NN + threshold.

    Ties resolve to the first index (torch CPU ``max`` semantics).
    """
    inner = scores[:, :-1, :-1]
    max0, max1 = inner.max(2), inner.max(1)
    m0, m1 = max0.indices, max1.indices
    i0 = torch.arange(m0.shape[1])[None]
    i1 = torch.arange(m1.shape[1])[None]
    mutual0 = i0 == m1.gather(1, m0)
    mutual1 = i1 == m0.gather(1, m1)
    ms0 = torch.where(mutual0, max0.values.exp(), max0.values.new_tensor(0))
    ms1 = torch.where(mutual1, ms0.gather(1, m1), ms0.new_tensor(0))
    valid0 = mutual0 & (ms0 > th)
    valid1 = mutual1 & valid0.gather(1, m1)
    return torch.where(valid0, m0, -1), torch.where(valid1, m1, -1), ms0, ms1


def confidence_threshold(i, n_layers):
    """lightglue.py:581-584."""
    return float(np.clip(0.8 + 0.1 * np.exp(-4.0 * i / n_layers), 0, 1))


def lightglue_forward(W, data, conf, dtype=torch.float32, return_layers=False):
    """lightglue.py:444-579 LightGlue.forward in eval mode.

    ``W``: dict name -> array (reference state-dict keys).  ``data``: dict with keypoints0/1
    [B,M,2], descriptors0/1 [B,M,D], and optionally image_size0/1 [B,2] (the reference reads
    ``data['view*']['image_size']``), scales*/oris* when ``add_scale_ori``.
    """
    W = {k: _t(v, dtype) for k, v in W.items()}
    L, H = int(conf.get("n_layers", 9)), int(conf.get("num_heads", 4))
    depth_conf = float(conf.get("depth_confidence", -1))
    width_conf = float(conf.get("width_confidence", -1))
    th = float(conf.get("filter_threshold", 0.0))

    k0, k1 = _t(data["keypoints0"], dtype), _t(data["keypoints1"], dtype)
    b, m, _ = k0.shape
    n = k1.shape[1]
    s0 = _t(data["image_size0"], dtype) if data.get("image_size0") is not None else None
    s1 = _t(data["image_size1"], dtype) if data.get("image_size1") is not None else None
    k0, k1 = normalize_keypoints(k0, s0), normalize_keypoints(k1, s1)
    if conf.get("add_scale_ori", False):  # :458-476
        def ext(k, sc, o):
            sc, o = _t(sc, dtype), _t(o, dtype)
            return torch.cat([k, sc if sc.dim() == 3 else sc[..., None], o if o.dim() == 3 else o[..., None]], -1)
        k0 = ext(k0, data["scales0"], data["oris0"])
        k1 = ext(k1, data["scales1"], data["oris1"])
    d0, d1 = _t(data["descriptors0"], dtype), _t(data["descriptors1"], dtype)
    if "input_proj.weight" in W:  # :370-373,486-487
        d0 = _linear(d0, W["input_proj.weight"], W["input_proj.bias"])
        d1 = _linear(d1, W["input_proj.weight"], W["input_proj.bias"])

    pe = ("posenc.Wr.weight", "posenc.condition_modulation.weight", "posenc.condition_modulation.bias")
    cos0, sin0 = positional_encoding(k0, m, *(W[k] for k in pe))
    cos1, sin1 = positional_encoding(k1, n, *(W[k] for k in pe))

    do_stop = depth_conf > 0
    do_prune = width_conf > 0
    if do_prune:
        ind0, ind1 = torch.arange(m)[None], torch.arange(n)[None]
        prune0, prune1 = torch.ones_like(ind0), torch.ones_like(ind1)
    thr = [confidence_threshold(i, L) for i in range(L)]
    layers = []
    token0 = token1 = None
    for i in range(L):
        p = f"transformers.{i}"
        d0 = self_block(d0, cos0, sin0, W, p + ".self_attn", H)
        d1 = self_block(d1, cos1, sin1, W, p + ".self_attn", H)
        d0, d1 = cross_block(d0, d1, W, p + ".cross_attn", H)
        if return_layers:
            layers.append((d0.clone(), d1.clone()))
        if i == L - 1:
            break
        if do_stop:  # :527-531, with thresholds per confidence_threshold (:581-584)
            assert b == 1
            tw, tb = W[f"token_confidence.{i}.token.0.weight"], W[f"token_confidence.{i}.token.0.bias"]
            token0 = torch.sigmoid(_linear(d0, tw, tb)).squeeze(-1)
            token1 = torch.sigmoid(_linear(d1, tw, tb)).squeeze(-1)
            conf_all = torch.cat([token0, token1], -1)
            ratio = 1.0 - (conf_all < thr[i]).float().sum() / (m + n)
            if ratio > depth_conf:
                break
        if do_prune:  # :532-547, get_pruning_mask :586-593
            assert b == 1
            a = f"log_assignment.{i}"
            mw, mb = W[a + ".matchability.weight"], W[a + ".matchability.bias"]

            def keep_of(d, tok):
                keep = torch.sigmoid(_linear(d, mw, mb)).squeeze(-1) > (1 - width_conf)
                if tok is not None:
                    keep |= tok <= thr[i]
                return torch.where(keep)[1]

            keep0 = keep_of(d0, token0)
            ind0 = ind0.index_select(1, keep0)
            d0 = d0.index_select(1, keep0)
            cos0, sin0 = cos0.index_select(1, keep0), sin0.index_select(1, keep0)
            prune0[:, ind0] += 1
            keep1 = keep_of(d1, token1)
            ind1 = ind1.index_select(1, keep1)
            d1 = d1.index_select(1, keep1)
            cos1, sin1 = cos1.index_select(1, keep1), sin1.index_select(1, keep1)
            prune1[:, ind1] += 1

    scores, sim = match_assignment(d0, d1, W, f"log_assignment.{i}")
    m0, m1, ms0, ms1 = filter_matches(scores, th)
    if do_prune:  # :553-562
        m0_ = torch.full((b, m), -1, dtype=m0.dtype)
        m1_ = torch.full((b, n), -1, dtype=m1.dtype)
        m0_[:, ind0] = torch.where(m0 == -1, -1, ind1.gather(1, m0.clamp(min=0)))
        m1_[:, ind1] = torch.where(m1 == -1, -1, ind0.gather(1, m1.clamp(min=0)))
        ms0_ = torch.zeros((b, m), dtype=ms0.dtype)
        ms1_ = torch.zeros((b, n), dtype=ms1.dtype)
        ms0_[:, ind0] = ms0
        ms1_[:, ind1] = ms1
        m0, m1, ms0, ms1 = m0_, m1_, ms0_, ms1_
    else:
        prune0 = torch.full((b, m), float(L), dtype=ms0.dtype)
        prune1 = torch.full((b, n), float(L), dtype=ms1.dtype)
    out = {
        "matches0": m0,
        "matches1": m1,
        "matching_scores0": ms0,
        "matching_scores1": ms1,
        "ref_descriptors0": d0[:, None],
        "ref_descriptors1": d1[:, None],
        "log_assignment": scores,
        "sim": sim,
        "prune0": prune0,
        "prune1": prune1,
        "stop_layer": i,
    }
    if return_layers:
        out["layers"] = layers
    return out


def log_optimal_transport(scores, alpha, iters):
    """superglue.py:173-201: log-domain Sinkhorn with a dustbin row/column of score ``alpha``."""
    scores = torch.as_tensor(scores)
    b, m, n = scores.shape
    alpha = torch.as_tensor(alpha, dtype=scores.dtype)
    ms, ns = torch.tensor(float(m), dtype=scores.dtype), torch.tensor(float(n), dtype=scores.dtype)
    couplings = torch.cat(
        [torch.cat([scores, alpha.expand(b, m, 1)], -1), torch.cat([alpha.expand(b, 1, n), alpha.expand(b, 1, 1)], -1)], 1
    )
    norm = -(ms + ns).log()
    log_mu = torch.cat([norm.expand(m), ns.log()[None] + norm])[None].expand(b, -1)
    log_nu = torch.cat([norm.expand(n), ms.log()[None] + norm])[None].expand(b, -1)
    u, v = torch.zeros_like(log_mu), torch.zeros_like(log_nu)
    for _ in range(iters):
        u = log_mu - torch.logsumexp(couplings + v.unsqueeze(1), dim=2)
        v = log_nu - torch.logsumexp(couplings + u.unsqueeze(2), dim=1)
    return couplings + u.unsqueeze(2) + v.unsqueeze(1) - norm


def near_tie_rows(scores64, eps):
    """Rows / columns whose top-1 vs top-2 margin in the fp64 inner block is below ``eps``."""
    inner = scores64[:, :-1, :-1]
    top0 = inner.topk(2, dim=2).values if inner.shape[2] > 1 else None
    top1 = inner.topk(2, dim=1).values if inner.shape[1] > 1 else None
    r = (top0[..., 0] - top0[..., 1] < eps) if top0 is not None else torch.zeros(inner.shape[:2], dtype=torch.bool)
    c = (top1[:, 0] - top1[:, 1] < eps) if top1 is not None else torch.zeros((inner.shape[0], inner.shape[2]), dtype=torch.bool)
    return r, c


__all__ = [
    "normalize_keypoints",
    "positional_encoding",
    "self_block",
    "cross_block",
    "sigmoid_log_double_softmax",
    "match_assignment",
    "filter_matches",
    "confidence_threshold",
    "lightglue_forward",
    "log_optimal_transport",
    "near_tie_rows",
    "math",
]
