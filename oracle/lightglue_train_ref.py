"""Functional torch-CPU restatement of the reference LightGlue TRAINING loss — TEST ORACLE.

Test infrastructure only (see ``oracle/__init__.py``): the GPU backward tests differentiate this
restatement with torch autograd (in float64) and compare every parameter gradient and both
descriptor gradients with the HIP backward.  It is pinned to the reference's own autograd
gradients by ``tests/golden/make_grad_golden.py`` / ``tests/test_oracle_grad.py``.

Restates (paths relative to ``/root/reference``):
* ``gluefactory/models/matchers/lightglue.py:444-579`` ``LightGlue.forward`` in training mode
  (no pruning, no early stop, every layer's descriptors kept, :502-503,521-524);
* ``:614-663`` ``LightGlue.loss`` (gamma-weighted NLL of every layer's assignment head on that
  layer's descriptors, the token-confidence BCE of :108-122, ``row_norm``);
* ``gluefactory/models/utils/losses.py:6-73`` ``weight_loss`` / ``NLLLoss``;
* ``gluefactory/train.py:436`` ``loss = torch.mean(losses["total"])``.

``W`` is a dict name -> torch tensor (reference state-dict keys); tensors that require grad get
gradients through ``torch.autograd``.  ``dtype`` casts every weight and input.
"""
import numpy as np
import torch
import torch.nn.functional as F

from .lightglue_ref import cross_block, match_assignment, normalize_keypoints, positional_encoding, self_block


def _tt(x, dtype):
    if torch.is_tensor(x):
        return x.to(dtype)
    return torch.as_tensor(np.asarray(x)).to(dtype)


def train_forward(W, data, conf, dtype=torch.float64):
    """lightglue.py:444-579 in training mode.  Returns (layers, la_final): ``layers[i]`` is the
    (desc0, desc1) pair after transformer layer i (``ref_descriptors*[:, i]``, :521-524,572) and
    ``la_final`` the last head's log assignment (``pred["log_assignment"]``, :550)."""
    L, H = int(conf.get("n_layers", 9)), int(conf.get("num_heads", 4))
    k0, k1 = _tt(data["keypoints0"], dtype), _tt(data["keypoints1"], dtype)
    m, n = k0.shape[1], k1.shape[1]
    s0 = _tt(data["image_size0"], dtype) if data.get("image_size0") is not None else None
    s1 = _tt(data["image_size1"], dtype) if data.get("image_size1") is not None else None
    k0, k1 = normalize_keypoints(k0, s0), normalize_keypoints(k1, s1)
    if conf.get("add_scale_ori", False):  # :458-476
        def ext(k, sc, o):
            sc, o = _tt(sc, dtype), _tt(o, dtype)
            return torch.cat([k, sc if sc.dim() == 3 else sc[..., None], o if o.dim() == 3 else o[..., None]], -1)
        k0 = ext(k0, data["scales0"], data["oris0"])
        k1 = ext(k1, data["scales1"], data["oris1"])
    d0, d1 = _tt(data["descriptors0"], dtype), _tt(data["descriptors1"], dtype)
    if "input_proj.weight" in W:  # :370-373,486-487
        d0 = F.linear(d0, W["input_proj.weight"], W["input_proj.bias"])
        d1 = F.linear(d1, W["input_proj.weight"], W["input_proj.bias"])
    pe = ("posenc.Wr.weight", "posenc.condition_modulation.weight", "posenc.condition_modulation.bias")
    cos0, sin0 = positional_encoding(k0, m, *(W[k] for k in pe))
    cos1, sin1 = positional_encoding(k1, n, *(W[k] for k in pe))
    layers = []
    for i in range(L):  # :514-524
        p = f"transformers.{i}"
        d0 = self_block(d0, cos0, sin0, W, p + ".self_attn", H)
        d1 = self_block(d1, cos1, sin1, W, p + ".self_attn", H)
        d0, d1 = cross_block(d0, d1, W, p + ".cross_attn", H)
        layers.append((d0, d1))
    la_final, _ = match_assignment(d0, d1, W, f"log_assignment.{L - 1}")  # :550
    return layers, la_final


def nll_weights(la, gt_matches0, gt_matches1, gt_assignment):
    """losses.py:60-73 NLLLoss.nll_loss: [B, M+1, N+1] weights (column dustbin at [:, -1, :m])."""
    m, n = gt_matches0.shape[-1], gt_matches1.shape[-1]
    w = torch.zeros_like(la)
    w[:, :m, :n] = gt_assignment.to(la.dtype)
    w[:, :m, -1] = (gt_matches0 == -1).to(la.dtype)
    w[:, -1, :m] = (gt_matches1 == -1).to(la.dtype)
    return w


def weight_loss(la, w):
    """losses.py:6-27."""
    b, m, n = la.shape
    m -= 1
    n -= 1
    sc = la * w
    num_neg0 = w[:, :m, -1].sum(-1).clamp(min=1.0)
    num_neg1 = w[:, -1, :n].sum(-1).clamp(min=1.0)
    num_pos = w[:, :m, :n].sum((-1, -2)).clamp(min=1.0)
    nll_pos = -sc[:, :m, :n].sum((-1, -2)) / num_pos.clamp(min=1.0)
    nll_neg = (-sc[:, :m, -1].sum(-1) - sc[:, -1, :n].sum(-1)) / (num_neg0 + num_neg1)
    return nll_pos, nll_neg, num_pos, (num_neg0 + num_neg1) / 2.0


def nll(la, w, balancing):
    """losses.py:40-58 NLLLoss.forward (the loss value)."""
    nll_pos, nll_neg, _, _ = weight_loss(la, w)
    return balancing * nll_pos + (1 - balancing) * nll_neg


def train_loss(W, data, gt, conf, dtype=torch.float64):
    """lightglue.py:614-663 LightGlue.loss in training mode on the training forward; returns
    (mean total -- train.py:436 --, losses dict)."""
    L = int(conf.get("n_layers", 9))
    lconf = {"gamma": 1.0, "nll_balancing": 0.5, **conf.get("loss", {})}
    gamma, bal = float(lconf["gamma"]), float(lconf["nll_balancing"])
    layers, la_final = train_forward(W, data, conf, dtype)
    g0 = torch.as_tensor(np.asarray(gt["gt_matches0"]))
    g1 = torch.as_tensor(np.asarray(gt["gt_matches1"]))
    ga = torch.as_tensor(np.asarray(gt["gt_assignment"]))
    la_last, _ = match_assignment(layers[-1][0], layers[-1][1], W, f"log_assignment.{L - 1}")
    w = nll_weights(la_last, g0, g1, ga)
    total = nll(la_last, w, bal)
    losses = {"last": total.detach().clone()}
    sum_weights = 1.0
    conf_loss = 0.0
    la_fd = la_final.detach()
    for i in range(L - 1):
        la_i, _ = match_assignment(layers[i][0], layers[i][1], W, f"log_assignment.{i}")
        weight = gamma ** (L - i - 1) if gamma > 0.0 else i + 1
        sum_weights += weight
        total = total + nll(la_i, w, bal) * weight
        # TokenConfidence.loss (:108-122): gradients reach the token Linear only (detached inputs)
        tw, tb = W[f"token_confidence.{i}.token.0.weight"], W[f"token_confidence.{i}.token.0.bias"]
        lg0 = F.linear(layers[i][0].detach(), tw, tb).squeeze(-1)
        lg1 = F.linear(layers[i][1].detach(), tw, tb).squeeze(-1)
        la_id = la_i.detach()
        c0 = la_fd[:, :-1, :].max(-1).indices == la_id[:, :-1, :].max(-1).indices
        c1 = la_fd[:, :, :-1].max(-2).indices == la_id[:, :, :-1].max(-2).indices
        bce = F.binary_cross_entropy_with_logits
        conf_loss = conf_loss + (bce(lg0, c0.to(lg0.dtype), reduction="none").mean(-1)
                                 + bce(lg1, c1.to(lg1.dtype), reduction="none").mean(-1)) / 2.0 / (L - 1)
    total = total / sum_weights + conf_loss
    losses.update({"total": total, "confidence": conf_loss})
    return total.mean(), losses
