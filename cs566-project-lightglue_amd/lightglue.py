"""Drop-in for ``gluefactory.models.matchers.lightglue.LightGlue`` (reference lightglue.py:340-666).

Same constructor config keys (``default_conf``, :341-361), same parameter names / state-dict
schema (so reference checkpoints load unchanged, including the old ``self_attn.{i}`` key renames,
:423-430), same ``forward(data) -> dict`` contract (:444-579).  The modules below are parameter
containers only: the whole eval forward runs in ``liblightglue_mi355x.so`` (hand-written gfx950
HIP kernels) through the C-ABI in ``include/lightglue_mi355x.h``.  There is no PyTorch compute
fallback; a CPU input or a missing library raises.

Deliberate behaviour differences from the reference:
* early stop uses ``[confidence_threshold(i) for i in range(L)]`` (the reference reads an
  undefined attribute, :592,604) and returns the stopping layer's descriptors (the reference
  crashes in ``torch.stack([])``, :572);
* without ``view*['image_size']`` the keypoints are normalised by their extent (:25-26) instead of
  raising ``UnboundLocalError`` (:452-455);
* ``ref_descriptors*`` is ``[B, 1, M', 256]`` in eval mode and ``[B, L, M, 256]`` (every layer) in
  training mode, as the reference (:521-524,572); training mode also turns early stop and pruning
  off (:502-503).  The training path computes in fp32 whatever ``mp`` says (the reference's
  autocast is not mirrored).
* with pruning and B > 1, ``log_assignment`` and ``ref_descriptors*`` are per-pair LISTS (pair b's
  kept block; the reference asserts B == 1, :528,533); ``kept0/1`` and ``stop_layer`` give the
  per-pair counts.

Training (the reference differentiates this module with torch autograd, gluefactory/train.py:450):
in training mode with gradients enabled, ``forward`` runs the activation-saving training forward
of the HIP library (``lg_train_forward``) inside a ``torch.autograd.Function`` whose backward is
the hand-written HIP backward (``lg_train_backward``); every ``MatchAssignment`` head is another
Function (``lg_assignment_head`` forward, ``lg_head_backward`` backward), and :meth:`loss` fuses
the NLL of each head into its head's backward (no dense d(loss)/d(log_assignment) is formed).
Gradients reach every parameter and both descriptor inputs.
"""
import ctypes
import os
import warnings
from pathlib import Path

import numpy as np
import torch
from torch import nn

from . import _lib
from .weights import DEFAULT_CONF

DATA_PATH = Path(__file__).resolve().parent.parent / "data"


class AttrDict(dict):
    """Minimal stand-in for the OmegaConf DictConfig the reference uses for ``self.conf``."""

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __setattr__(self, k, v):
        self[k] = v


def merge_conf(*cfgs):
    out = AttrDict()
    for c in cfgs:
        for k, v in dict(c or {}).items():
            if isinstance(v, dict):
                prev = out.get(k)
                out[k] = merge_conf(prev if isinstance(prev, dict) else {}, v)
            else:
                out[k] = v
    return out


# ---------------------------------------------------------------- parameter containers
class _PosEnc(nn.Module):  # lightglue.py:50-61
    def __init__(self, m_in, f_dim, gamma=1.0):
        super().__init__()
        self.Wr = nn.Linear(m_in, f_dim // 2, bias=False)
        nn.init.normal_(self.Wr.weight.data, mean=0, std=gamma**-2)
        self.condition_modulation = nn.Linear(1, f_dim // 2)


def _ffn(d):
    return nn.Sequential(nn.Linear(2 * d, 2 * d), nn.LayerNorm(2 * d, elementwise_affine=True), nn.GELU(), nn.Linear(2 * d, d))


class _SelfBlock(nn.Module):  # lightglue.py:159-176
    def __init__(self, d):
        super().__init__()
        self.Wqkv = nn.Linear(d, 3 * d)
        self.out_proj = nn.Linear(d, d)
        self.ffn = _ffn(d)


class _CrossBlock(nn.Module):  # lightglue.py:194-211
    def __init__(self, d):
        super().__init__()
        self.to_qk = nn.Linear(d, d)
        self.to_v = nn.Linear(d, d)
        self.to_out = nn.Linear(d, d)
        self.ffn = _ffn(d)


class _Layer(nn.Module):  # lightglue.py:252-256
    def __init__(self, d):
        super().__init__()
        self.self_attn = _SelfBlock(d)
        self.cross_attn = _CrossBlock(d)


class _MatchAssignment(nn.Module):  # lightglue.py:299-304
    def __init__(self, d):
        super().__init__()
        self.matchability = nn.Linear(d, 1, bias=True)
        self.final_proj = nn.Linear(d, d, bias=True)


class _TokenConfidence(nn.Module):  # lightglue.py:96-99
    def __init__(self, d):
        super().__init__()
        self.token = nn.Sequential(nn.Linear(d, 1), nn.Sigmoid())


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


# Extension keys (no reference counterpart).  "precision": matrix-core operand format of the HIP
# kernels, both fp32-accurate -- "auto" (fp16x3, run-time operands range-scaled on the device) or "bf16x6"
# (DESIGN.md §3).  "return_similarity": also return the final head's similarity md0 md1^T
# [B, M, N] as pred["similarity"] (MatchAssignment's second output, lightglue.py:311,315; the input
# of a Sinkhorn assignment head, configs[4]).
EXTENSION_CONF = {"precision": "auto", "return_similarity": False}


def _trunk_param(name):
    return name.startswith(("input_proj.", "posenc.", "transformers."))


class _TrainTrunk(torch.autograd.Function):
    """LightGlue.forward in training mode (lightglue.py:444-579, :502-503 gating) up to the
    per-layer descriptors ``ref_descriptors0/1`` [B, L, M, 256]; backward = lg_train_backward."""

    @staticmethod
    def forward(ctx, model, inputs, d0, d1, *params):
        lib = model._ensure_handle(d0.device, upload=False)
        ctx.model, ctx.inputs = model, inputs
        b, m, n = d0.shape[0], d0.shape[1], d1.shape[1]
        L, dd = int(model.conf.n_layers), int(model.conf.descriptor_dim)
        inp = model._lg_inputs(inputs, d0, d1)
        nb = ctypes.c_size_t()
        _lib.check(lib.lg_train_saved_bytes_ex(model._handle, b, m, n, inp.flags, ctypes.byref(nb)),
                   "lg_train_saved_bytes_ex")
        saved = torch.empty(max(nb.value, 1), dtype=torch.uint8, device=d0.device)
        rd0 = torch.empty((b, L, m, dd), dtype=torch.float32, device=d0.device)
        rd1 = torch.empty((b, L, n, dd), dtype=torch.float32, device=d0.device)
        stream = torch.cuda.current_stream(d0.device).cuda_stream
        _lib.check(lib.lg_train_forward(model._handle, model._param_array(params), ctypes.byref(inp), _ptr(rd0), _ptr(rd1),
                                        _ptr(saved), nb.value, ctypes.c_void_p(stream)), "lg_train_forward")
        ctx.saved_buf = saved
        ctx.save_for_backward(d0, d1, *params)
        return rd0, rd1

    @staticmethod
    def backward(ctx, g_rd0, g_rd1):
        model = ctx.model
        d0, d1, *params = ctx.saved_tensors
        lib = model._ensure_handle(d0.device, upload=False)
        b, m, n = d0.shape[0], d0.shape[1], d1.shape[1]
        names = model._schema_names()
        wanted = [_trunk_param(nm) and ctx.needs_input_grad[4 + i] for i, nm in enumerate(names)]
        ddp = getattr(model, "_ddp", None)  # ddp.DataParallel: per-layer all-reduces under the backward
        if ddp is not None:
            buckets = ddp.buckets(names, params, wanted, int(model.conf.n_layers), False, d0.device)
            grads = buckets.grads
            _lib.check(lib.lg_set_grad_ready_hook(model._handle, _lib.fnptr(buckets.callback(_lib.LG_GRAD_READY_FN)),
                                                   None),
                       "lg_set_grad_ready_hook")
        else:
            grads = [torch.empty_like(p) if w else None for w, p in zip(wanted, params)]
        gd0 = torch.empty_like(d0) if ctx.needs_input_grad[2] else None
        gd1 = torch.empty_like(d1) if ctx.needs_input_grad[3] else None
        nb = ctypes.c_size_t()
        _lib.check(lib.lg_train_scratch_bytes(model._handle, b, m, n, ctypes.byref(nb)), "lg_train_scratch_bytes")
        scratch = torch.empty(max(nb.value, 1), dtype=torch.uint8, device=d0.device)
        g_rd0 = None if g_rd0 is None else g_rd0.contiguous()
        g_rd1 = None if g_rd1 is None else g_rd1.contiguous()
        inp = model._lg_inputs(ctx.inputs, d0, d1)
        stream = torch.cuda.current_stream(d0.device).cuda_stream
        try:
            _lib.check(lib.lg_train_backward(model._handle, model._param_array(params), ctypes.byref(inp),
                                             _ptr(ctx.saved_buf), ctx.saved_buf.numel(), _ptr(g_rd0), _ptr(g_rd1),
                                             model._param_array(grads), _ptr(gd0), _ptr(gd1), _ptr(scratch), nb.value,
                                             ctypes.c_void_p(stream)), "lg_train_backward")
        except Exception as e:
            if ddp is not None:
                ddp.abort(e)  # fewer bucket collectives than the peers issue: fatal to the job, never a hang
            raise
        finally:
            if ddp is not None:
                lib.lg_set_grad_ready_hook(model._handle, None, None)
        if ddp is not None:
            grads = buckets.finish()  # wait for the layer buckets, average over the ranks
        ctx.saved_buf = None
        return (None, None, gd0, gd1, *grads)


def _head_backward(model, layer, d0, d1, params, needs, la_grad, s_in, s_dust, g_sim, g_t0, g_t1, fwd_scratch=None,
                   gt=None):
    """lg_head_backward for head ``layer``: (gd0, gd1, per-parameter grads or None).  ``fwd_scratch``:
    the scratch of this head's _head_forward (similarity not requested), whose md / z / similarity /
    LSEs the backward then reuses (lg_head_backward_from_forward) instead of recomputing them.
    ``gt``: nll_inputs' (gt_assignment uint8, gt_matches0, gt_matches1) in place of ``la_grad`` --
    the NLL weights read from the ground truth (lg_head_nll_backward), no dense weight tensor."""
    lib = model._ensure_handle(d0.device, upload=False)
    b, m, n = d0.shape[0], d0.shape[1], d1.shape[1]
    L = int(model.conf.n_layers)
    li = layer % L
    own = (f"log_assignment.{li}.",) + ((f"token_confidence.{li}.",) if (g_t0 is not None or g_t1 is not None) else ())
    names = model._schema_names()
    grads = [torch.empty_like(p) if (nm.startswith(own) and needs[i]) else None
             for i, (nm, p) in enumerate(zip(names, params))]
    gd0 = torch.empty_like(d0) if needs[-2] else None
    gd1 = torch.empty_like(d1) if needs[-1] else None
    nb = ctypes.c_size_t()
    _lib.check(lib.lg_head_scratch_bytes(model._handle, b, m, n, ctypes.byref(nb)), "lg_head_scratch_bytes")
    if fwd_scratch is not None:
        scratch, fn = fwd_scratch, lib.lg_head_backward_from_forward
    else:
        scratch, fn = torch.empty(max(nb.value, 1), dtype=torch.uint8, device=d0.device), lib.lg_head_backward
    stream = torch.cuda.current_stream(d0.device).cuda_stream
    c = lambda t: None if t is None else t.float().contiguous()  # noqa: E731
    la_grad, s_in, s_dust, g_sim, g_t0, g_t1 = map(c, (la_grad, s_in, s_dust, g_sim, g_t0, g_t1))
    if gt is not None:
        gta, g0, g1 = gt
        _lib.check(lib.lg_head_nll_backward(model._handle, model._param_array(params), int(li), _ptr(d0), _ptr(d1), b, m,
                                            n, _ptr(gta), _ptr(g0), _ptr(g1), _ptr(s_in), _ptr(s_dust), _ptr(g_t0),
                                            _ptr(g_t1), model._param_array(grads), _ptr(gd0), _ptr(gd1),
                                            int(fwd_scratch is not None), _ptr(scratch), nb.value,
                                            ctypes.c_void_p(stream)), "lg_head_nll_backward")
        return gd0, gd1, grads
    _lib.check(fn(model._handle, model._param_array(params), int(li), _ptr(d0), _ptr(d1), b, m, n,
                  _ptr(la_grad), _ptr(s_in), _ptr(s_dust), _ptr(g_sim), _ptr(g_t0), _ptr(g_t1),
                  model._param_array(grads), _ptr(gd0), _ptr(gd1), _ptr(scratch), nb.value,
                  ctypes.c_void_p(stream)), "lg_head_backward")
    return gd0, gd1, grads


def _head_forward(model, layer, d0, d1, params, tokens, similarity=False, keep_scratch=False):
    """lg_head_forward: MatchAssignment ``layer`` (+ the token logits) on raw parameters, fp32.
    ``keep_scratch``: also return the scratch (md, z, similarity, LSEs) for _head_backward."""
    lib = model._ensure_handle(d0.device, upload=False)
    b, m, n = d0.shape[0], d0.shape[1], d1.shape[1]
    dev = d0.device
    la = torch.empty((b, m + 1, n + 1), dtype=torch.float32, device=dev)
    sim = torch.empty((b, m, n), dtype=torch.float32, device=dev) if similarity else None
    t0 = torch.empty((b, m), dtype=torch.float32, device=dev) if tokens else None
    t1 = torch.empty((b, n), dtype=torch.float32, device=dev) if tokens else None
    nb = ctypes.c_size_t()
    _lib.check(lib.lg_head_scratch_bytes(model._handle, b, m, n, ctypes.byref(nb)), "lg_head_scratch_bytes")
    scratch = torch.empty(max(nb.value, 1), dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    _lib.check(lib.lg_head_forward(model._handle, model._param_array(params), int(layer), _ptr(d0), _ptr(d1), b, m, n,
                                   _ptr(la), _ptr(sim), _ptr(t0), _ptr(t1), _ptr(scratch), nb.value,
                                   ctypes.c_void_p(stream)), "lg_head_forward")
    return (la, sim, t0, t1, scratch) if keep_scratch else (la, sim, t0, t1)


class _Head(torch.autograd.Function):
    """``log_assignment[layer](desc0, desc1)`` (MatchAssignment + sigmoid_log_double_softmax,
    lightglue.py:284-315) -> (log_assignment, similarity, token logits 0, token logits 1); the
    token logits are TokenConfidence's Linear before its sigmoid (:109-110, detached inputs)."""

    @staticmethod
    def forward(ctx, model, layer, tokens, d0, d1, *params):
        d0c, d1c = d0.float().contiguous(), d1.float().contiguous()
        la, sim, t0, t1 = _head_forward(model, layer, d0c, d1c, params, tokens, similarity=True)
        if not tokens:
            t0, t1 = la.new_zeros(0), la.new_zeros(0)
        ctx.model, ctx.layer, ctx.tokens = model, layer, tokens
        ctx.save_for_backward(d0c, d1c, *params)
        return la, sim, t0, t1

    @staticmethod
    def backward(ctx, g_la, g_sim, g_t0, g_t1):
        d0, d1, *params = ctx.saved_tensors
        if g_la is None:
            b, m, n = d0.shape[0], d0.shape[1], d1.shape[1]
            g_la = torch.zeros((b, m + 1, n + 1), device=d0.device)
        if not ctx.tokens:
            g_t0 = g_t1 = None
        needs = list(ctx.needs_input_grad[5:]) + [ctx.needs_input_grad[3], ctx.needs_input_grad[4]]
        gd0, gd1, grads = _head_backward(ctx.model, ctx.layer, d0, d1, params, needs, g_la, None, None, g_sim, g_t0, g_t1)
        return (None, None, None, gd0, gd1, *grads)


# env LG_HEAD_REUSE=0: the loss heads' backward recomputes md / z / similarity / LSEs (A/B runs)
_HEAD_REUSE = os.environ.get("LG_HEAD_REUSE", "1") != "0"
# env LG_HEAD_FUSED=0: the loss heads store their log assignment and take NLL / argmaxes from it
_HEAD_FUSED = os.environ.get("LG_HEAD_FUSED", "1") != "0"
# env LG_HEAD_GT=0: LightGlue.loss builds the dense [B, M+1, N+1] NLL weights (nll_weights) and the
# heads' backward reads them, instead of reading the ground truth itself (lg_head_nll_backward)
_HEAD_GT = os.environ.get("LG_HEAD_GT", "1") != "0"


def _head_nll_forward(model, layer, d0, d1, params, tokens, prepared, balancing):
    """lg_head_nll_forward: head ``layer``'s NLL terms [5, B] and its log assignment's row / column
    argmaxes, the log assignment never stored; returns (terms, argmax0, argmax1, t0, t1, scratch)."""
    lib = model._ensure_handle(d0.device, upload=False)
    b, m, n = d0.shape[0], d0.shape[1], d1.shape[1]
    dev = d0.device
    gta, g0, g1 = prepared
    out = torch.empty((5, b), dtype=torch.float32, device=dev)
    am0 = torch.empty((b, m), dtype=torch.int64, device=dev)
    am1 = torch.empty((b, n), dtype=torch.int64, device=dev)
    t0 = torch.empty((b, m), dtype=torch.float32, device=dev) if tokens else None
    t1 = torch.empty((b, n), dtype=torch.float32, device=dev) if tokens else None
    nb = ctypes.c_size_t()
    _lib.check(lib.lg_head_scratch_bytes(model._handle, b, m, n, ctypes.byref(nb)), "lg_head_scratch_bytes")
    scratch = torch.empty(max(nb.value, 1), dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    rc = lib.lg_head_nll_forward(model._handle, model._param_array(params), int(layer), _ptr(d0), _ptr(d1), b, m, n,
                                 _ptr(gta), _ptr(g0), _ptr(g1), 1, float(balancing), _ptr(out), _ptr(am0), _ptr(am1),
                                 _ptr(t0), _ptr(t1), _ptr(scratch), nb.value, ctypes.c_void_p(stream))
    if rc == _lib.LG_E_INVALID and m != n:
        raise RuntimeError(lib.lg_last_error().decode(errors="replace"))  # the reference's own error type
    _lib.check(rc, "lg_head_nll_forward")
    return out, am0, am1, t0, t1, scratch


class _HeadNLL(torch.autograd.Function):
    """One term of LightGlue.loss (lightglue.py:614-640): the NLL (losses.py:6-58) of head
    ``layer`` on (desc0, desc1) with the ground-truth weights of losses.py:62-73.  Outputs (nll,
    nll_pos, nll_neg, num_pos, num_neg, row argmax [B, M], column argmax [B, N] of the head's log
    assignment -- what TokenConfidence.loss compares, :108-122 -- token logits 0, token logits 1);
    the log assignment itself is never stored (lg_head_nll_forward).  The loss is linear in the log
    assignment, so the backward hands lg_head_backward the weights and two per-pair scales instead
    of a dense gradient."""

    @staticmethod
    def forward(ctx, model, layer, gt, balancing, tokens, d0, d1, *params):
        from .superglue import _nll

        # gt = (data, NLLLoss weights [B, M+1, N+1] or None, nll_inputs(data)): built once per
        # loss(); without the dense weights the backward reads them from nll_inputs' ground truth
        data, w, prepared = gt
        d0c, d1c = d0.float().contiguous(), d1.float().contiguous()
        # the scratch keeps md / z / similarity / LSEs for the backward (saved activations, ~1 GB per
        # head at configs[2]): no recompute of the head there (unless conf.checkpointed)
        if _HEAD_FUSED and d1c.shape[1] <= 4096:
            terms, am0, am1, t0, t1, scratch = _head_nll_forward(model, layer, d0c, d1c, params, tokens, prepared, balancing)
        else:
            la, _, t0, t1, scratch = _head_forward(model, layer, d0c, d1c, params, tokens, keep_scratch=True)
            terms = _nll(la, data, 1, float(balancing), prepared)  # [5, B]: nll, nll_pos, nll_neg, num_pos, num_neg
            am0, am1 = la[:, :-1, :].max(-1).indices, la[:, :, :-1].max(-2).indices
            del la
        # conf.checkpointed asks for activation memory over speed: the head's backward then
        # recomputes md / z / similarity / LSEs instead of keeping this ~1 GB scratch (configs[2])
        ctx.scratch = scratch if (_HEAD_REUSE and not model.conf.checkpointed) else None
        del scratch
        if not tokens:
            t0, t1 = d0c.new_zeros(0), d0c.new_zeros(0)
        ctx.model, ctx.layer, ctx.tokens, ctx.bal = model, layer, tokens, float(balancing)
        ctx.gt = prepared if w is None else None
        ctx.set_materialize_grads(False)  # unused outputs' gradients arrive as None, not zero tensors
        ctx.save_for_backward(d0c, d1c, w, terms, *params)  # terms: never returned itself (clones below)
        ctx.mark_non_differentiable(am0, am1)
        nll, pos, neg, npos, nneg = (terms[i].clone() for i in range(5))
        ctx.mark_non_differentiable(npos, nneg)
        return nll, pos, neg, npos, nneg, am0, am1, t0, t1

    @staticmethod
    def backward(ctx, g_nll, g_pos, g_neg, _g_npos, _g_nneg, _g_am0, _g_am1, g_t0, g_t1):
        d0, d1, w, terms, *params = ctx.saved_tensors
        npos, nneg = terms[3], terms[4]

        def lin(a, wa, c):  # a * wa + c, an absent (None: unused output) term left out
            if a is None:
                return c if c is not None else torch.zeros(d0.shape[0], device=d0.device)
            return a * wa if c is None else a * wa + c

        gp = lin(g_nll, ctx.bal, g_pos)
        gn = lin(g_nll, 1.0 - ctx.bal, g_neg)
        # nll_pos = -sum(w la)_inner / num_pos, nll_neg = -sum(w la)_dustbins / (num_neg0 + num_neg1)
        s_in = -gp / npos
        s_dust = -gn / (2.0 * nneg)
        if not ctx.tokens:
            g_t0 = g_t1 = None
        needs = list(ctx.needs_input_grad[7:]) + [ctx.needs_input_grad[5], ctx.needs_input_grad[6]]
        gd0, gd1, grads = _head_backward(ctx.model, ctx.layer, d0, d1, params, needs, w, s_in, s_dust, None, g_t0, g_t1,
                                         fwd_scratch=ctx.scratch, gt=ctx.gt)
        # only the forward's scratch is dropped (a second backward through a retained graph then
        # recomputes the head); the ground truth stays: without the dense weights (w None) it is
        # what the backward reads its NLL weights from
        ctx.scratch = None
        return (None, None, None, None, None, gd0, gd1, *grads)


class _LayerSlices(torch.autograd.Function):
    """``rd`` [B, L, M, D] -> the L layer slices [B, M, D], each contiguous (what the heads take).
    Backward writes the slice gradients into one [B, L, M, D] tensor; indexing ``rd[:, i]`` per head
    instead lets autograd zero-fill a full [B, L, M, D] gradient for every slice and add them up."""

    @staticmethod
    def forward(ctx, rd):
        ctx.shape = rd.shape
        return tuple(rd[:, i].contiguous() for i in range(rd.shape[1]))

    @staticmethod
    def backward(ctx, *grads):
        ref = next((g for g in grads if g is not None), None)
        if ref is None:
            return None
        out = ref.new_empty(ctx.shape)
        for i, g in enumerate(grads):
            if g is None:
                out[:, i].zero_()
            else:
                out[:, i].copy_(g)
        return out


class LightGlue(nn.Module):
    default_conf = {**DEFAULT_CONF, **EXTENSION_CONF}
    required_data_keys = ["keypoints0", "keypoints1", "descriptors0", "descriptors1"]
    url = "https://github.com/cvg/LightGlue/releases/download/{}/{}_lightglue.pth"

    def __init__(self, conf) -> None:
        super().__init__()
        self.conf = conf = merge_conf(self.default_conf, conf)
        d, h, n = int(conf.descriptor_dim), int(conf.num_heads), int(conf.n_layers)
        if conf.input_dim != conf.descriptor_dim:
            self.input_proj = nn.Linear(conf.input_dim, d, bias=True)
        else:
            self.input_proj = nn.Identity()
        self.posenc = _PosEnc(2 + 2 * int(bool(conf.add_scale_ori)), d // h)
        self.transformers = nn.ModuleList([_Layer(d) for _ in range(n)])
        self.log_assignment = nn.ModuleList([_MatchAssignment(d) for _ in range(n)])
        self.token_confidence = nn.ModuleList([_TokenConfidence(d) for _ in range(n - 1)])
        self._handle = None
        self._handle_device = None
        self._weights_key = None
        self._weight_entries = None
        self._weight_modules = None
        self._graphs = None  # compile(): {signature: (hipGraph, static inputs, static outputs, generation, workspace)}
        # bumped whenever the native handle is (re)created or its weights are (re)uploaded: both
        # free device memory a captured graph may point at, so graphs of older generations are
        # recaptured instead of replayed
        self._gen = 0
        self._ws = None

        state_dict = None
        if conf.weights is not None:  # lightglue.py:402-421
            if Path(conf.weights).exists():
                state_dict = torch.load(conf.weights, map_location="cpu", weights_only=True)
            elif (DATA_PATH / conf.weights).exists():
                state_dict = torch.load(str(DATA_PATH / conf.weights), map_location="cpu", weights_only=True)
            else:
                fname = f"{conf.weights}_{conf.weights_from_version}".replace(".", "-") + ".pth"
                state_dict = torch.hub.load_state_dict_from_url(
                    self.url.format(conf.weights_from_version, conf.weights), file_name=fname
                )
        if state_dict:
            for i in range(n):  # lightglue.py:424-429
                pattern = f"self_attn.{i}", f"transformers.{i}.self_attn"
                state_dict = {k.replace(*pattern): v for k, v in state_dict.items()}
                pattern = f"cross_attn.{i}", f"transformers.{i}.cross_attn"
                state_dict = {k.replace(*pattern): v for k, v in state_dict.items()}
            self.load_state_dict(state_dict, strict=False)

    # ------------------------------------------------------------ reference helpers
    def confidence_threshold(self, layer_index: int) -> float:
        """lightglue.py:581-584."""
        threshold = 0.8 + 0.1 * np.exp(-4.0 * layer_index / self.conf.n_layers)
        return np.clip(threshold, 0, 1)

    @property
    def confidence_thresholds(self):
        return [self.confidence_threshold(i) for i in range(self.conf.n_layers)]

    def compile(self, mode="reduce-overhead"):
        """The reference torch.compile()s its layers (:432-442); its "reduce-overhead" mode is CUDA
        graphs.  The forward here is native HIP already, so compile() turns on HIP-graph replay:
        the first eval forward of each (shape, inputs present) signature without pruning / early
        stop runs once eagerly (weights upload, workspace) and is then captured into a hipGraph
        (torch.cuda.CUDAGraph); later forwards of that signature copy their inputs into the graph's
        static buffers and replay it -- one graph launch instead of ~100 kernel launches.  As with
        torch's CUDA graphs, a replayed forward returns the graph's static output tensors, which the
        next forward of the same signature overwrites (clone to keep).  ``mode`` is ignored."""
        self._graphs = {}
        return self

    def _graph_forward(self, inputs, key):
        """Replay (capturing on first use) the HIP graph of one forward signature.  The handle is
        validated first (config, weights): a re-upload or a new handle bumps ``self._gen`` and
        every graph captured before it is recaptured, never replayed against freed memory."""
        self._ensure_handle(inputs[0].device)
        ent = self._graphs.get(key)
        if ent is None or ent[3] != self._gen:
            static = [None if t is None else t.clone() for t in inputs]
            self._forward_native(*static)  # eager: weights upload, workspace sizing, lazy init
            torch.cuda.synchronize(static[0].device)
            gen = self._gen
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                pred = self._forward_native(*static)
            assert self._gen == gen, "lightglue_amd: the handle changed during graph capture"
            # the graph keeps the workspace it was captured with alive (a later, larger eager
            # forward replaces self._ws)
            ent = (g, static, pred, gen, self._ws)
            self._graphs[key] = ent
        g, static, pred = ent[0], ent[1], ent[2]
        for dst, src in zip(static, inputs):
            if dst is not None:
                dst.copy_(src)
        g.replay()
        return pred

    # ------------------------------------------------------------ native handle
    def _lib_config(self):
        c = self.conf
        return _lib.LGConfig(
            int(c.input_dim),
            int(c.descriptor_dim),
            int(c.n_layers),
            int(c.num_heads),
            int(bool(c.add_scale_ori)),
            float(c.depth_confidence),
            float(c.width_confidence),
            float(c.filter_threshold),
            _lib.PRECISIONS[str(c.precision)],
        )

    def _ensure_handle(self, device, upload=True):
        """The native handle for this config on ``device``; with ``upload`` the parameters are
        (re)packed into it when they changed.  The training path passes raw parameter pointers
        to every call and never needs the packed copy (upload=False)."""
        lib = _lib.load()
        cfg = self._lib_config()
        cfg_key = tuple(getattr(cfg, f) for f, _ in _lib.LGConfig._fields_)
        if self._handle is not None and (self._handle_device != device or self._cfg_key != cfg_key):
            lib.lg_destroy(self._handle)
            self._handle = None
        if self._handle is None:
            h = ctypes.c_void_p()
            _lib.check(lib.lg_create(ctypes.byref(cfg), device.index or 0, ctypes.byref(h)), "lg_create")
            self._handle, self._handle_device, self._cfg_key = h, device, cfg_key
            self._weights_key = None
            self._gen += 1
        if not upload:
            return lib
        key = self._weights_signature()
        if key != self._weights_key:
            sd = self.state_dict(keep_vars=True)
            names = [n for n in sd]
            ts = []
            for n in names:
                t = sd[n].detach()
                if t.device != device or t.dtype != torch.float32:
                    raise RuntimeError(
                        f"lightglue_amd: parameter {n} is {t.dtype} on {t.device}; move the module to {device} in fp32"
                    )
                ts.append(t.contiguous())
            arr_n = (ctypes.c_char_p * len(names))(*[n.encode() for n in names])
            arr_p = (ctypes.c_void_p * len(ts))(*[t.data_ptr() for t in ts])
            arr_k = (ctypes.c_int64 * len(ts))(*[t.numel() for t in ts])
            stream = torch.cuda.current_stream(device).cuda_stream
            _lib.check(lib.lg_load_weights(self._handle, len(ts), arr_n, arr_p, arr_k, ctypes.c_void_p(stream)), "lg_load_weights")
            torch.cuda.current_stream(device).synchronize()  # sources may be temporaries
            self._weights_key = self._weights_signature()
            self._gen += 1
        return lib

    def reload_weights(self):
        """Force the next forward to re-upload every parameter.  Needed only after writes the
        forward cannot see: in-place writes through ``p.data`` (``p.data.copy_(...)``, EMA
        updates) bump the version counter of a temporary tensor, not of ``p``.  Captured HIP graphs
        (:meth:`compile`) are dropped as well."""
        self._weights_key = None
        if self._graphs is not None:
            self._graphs = {}

    def _weights_signature(self):
        """(data_ptr, _version) of every parameter / persistent buffer plus the identity of every
        submodule, from a cached list of (owner dict, name, tensor): ~0.1 ms per forward instead of
        ~0.8 ms for state_dict() + key (the forward's host time sits between two GPU forwards).
        A replaced submodule (``model.log_assignment[3] = ...``) or tensor object rebuilds the list;
        .to()/.cuda() clear it through _apply.  Writes through ``p.data`` are not seen: call
        :meth:`reload_weights` after them."""
        while True:
            mods = tuple(map(id, self.modules()))
            if self._weight_entries is None or self._weight_modules != mods:
                ent = []
                for mod in self.modules():
                    for n, t in mod._parameters.items():
                        if t is not None:
                            ent.append((mod._parameters, n, t))
                    for n, t in mod._buffers.items():
                        if t is not None and n not in mod._non_persistent_buffers_set:
                            ent.append((mod._buffers, n, t))
                self._weight_entries = ent
                self._weight_modules = mods
            sig = [mods]
            for d, n, t in self._weight_entries:
                if d.get(n) is not t:
                    self._weight_entries = None
                    break
                sig.append((t.data_ptr(), t._version))
            else:
                return tuple(sig)

    def _apply(self, fn, *args, **kwargs):  # .to() / .cuda() / .float(): parameters may be new tensors
        self._weight_entries = None
        self._weights_key = None
        return super()._apply(fn, *args, **kwargs)

    def __del__(self):
        try:
            if self._handle is not None and _lib._lib is not None:
                _lib._lib.lg_destroy(self._handle)
        except Exception:
            pass

    # ------------------------------------------------------------ forward
    def forward(self, data: dict) -> dict:
        for key in self.required_data_keys:  # lightglue.py:445-446
            assert key in data, f"Missing key {key} in data"
        kpts0, kpts1 = data["keypoints0"], data["keypoints1"]
        device = kpts0.device
        if device.type != "cuda":
            raise RuntimeError("lightglue_amd: inputs must be on a HIP (cuda) device; there is no CPU path")
        b, m, _ = kpts0.shape
        _, n, _ = kpts1.shape
        c = self.conf
        desc0, desc1 = data["descriptors0"], data["descriptors1"]
        assert desc0.shape[-1] == c.input_dim  # :481-482
        assert desc1.shape[-1] == c.input_dim
        size0 = size1 = None
        if "view0" in data and "view1" in data:  # :452-454
            size0 = data["view0"].get("image_size")
            size1 = data["view1"].get("image_size")

        def f32(t):
            return None if t is None else torch.as_tensor(t, device=device).to(torch.float32).contiguous()

        def per_point(t):  # scales/oris may be [B,N] or [B,N,1] (:464-465)
            t = f32(t)
            return t.reshape(t.shape[0], t.shape[1]) if t is not None else None

        k0, k1, d0, d1 = f32(kpts0), f32(kpts1), f32(desc0), f32(desc1)
        s0 = f32(size0).reshape(b, 2) if size0 is not None else None
        s1 = f32(size1).reshape(b, 2) if size1 is not None else None
        sc0 = o0 = sc1 = o1 = None
        if c.add_scale_ori:
            sc0, o0 = per_point(data["scales0"]), per_point(data["oris0"])
            sc1, o1 = per_point(data["scales1"]), per_point(data["oris1"])

        if self.training and torch.is_grad_enabled() and (
                d0.requires_grad or d1.requires_grad or any(p.requires_grad for p in self.parameters())):
            return self._forward_train((k0, k1, s0, s1, sc0, o0, sc1, o1), d0, d1)
        inputs = (k0, k1, d0, d1, s0, s1, sc0, o0, sc1, o1)
        pruning = (c.width_confidence > 0 or c.depth_confidence > 0) and not self.training
        if self._graphs is not None and not pruning and not self.training:
            key = (str(device),) + tuple(None if t is None else tuple(t.shape) for t in inputs)
            return self._graph_forward(inputs, key)
        return self._forward_native(*inputs)

    # ------------------------------------------------------------ training forward (autograd)
    def _schema_names(self):
        """State-dict names in the library's schema order (lg_weight_name)."""
        if getattr(self, "_schema_for", None) is not self._handle:
            lib = _lib.load()
            n = lib.lg_weight_count(self._handle)
            self._schema_list = [lib.lg_weight_name(self._handle, i).decode() for i in range(n)]
            self._schema_for = self._handle
        return self._schema_list

    def _schema_params(self, device):
        self._ensure_handle(device, upload=False)
        named = dict(self.named_parameters())
        params = []
        for nm in self._schema_names():
            p = named[nm]
            if p.device != device or p.dtype != torch.float32 or not p.is_contiguous():
                raise RuntimeError(f"lightglue_amd: parameter {nm} must be a contiguous fp32 tensor on {device}")
            params.append(p)
        return params

    @staticmethod
    def _param_array(tensors):
        arr = (ctypes.c_void_p * len(tensors))(*[None if t is None else t.data_ptr() for t in tensors])
        return ctypes.cast(arr, ctypes.c_void_p)

    def _lg_inputs(self, inputs, d0, d1):
        k0, k1, s0, s1, sc0, o0, sc1, o1 = inputs
        # checkpointed (lightglue.py:515-518): the training call keeps layer outputs only and the
        # backward recomputes each layer (LG_FWD_CHECKPOINTED)
        flags = _lib.LG_FWD_TRAINING_GATE | (_lib.LG_FWD_CHECKPOINTED if self.conf.checkpointed else 0)
        return _lib.LGInputs(d0.shape[0], d0.shape[1], d1.shape[1],
                             *[_ptr(t) for t in (k0, k1, d0, d1, s0, s1, sc0, o0, sc1, o1)], flags)

    def _forward_train(self, inputs, d0, d1):
        """Training-mode forward with autograd (lightglue.py:444-579 with :502-503 gating): the HIP
        training forward keeps its activations for the HIP backward; the final head is a
        differentiable MatchAssignment; matches come from the detached log assignment."""
        from .assignment import filter_matches

        c = self.conf
        device = d0.device
        b, m, n = d0.shape[0], d0.shape[1], d1.shape[1]
        if m == 0 or n == 0:
            raise IndexError("max(): Expected reduction dim to have non-zero size (empty keypoint set)")
        L = int(c.n_layers)
        params = self._schema_params(device)
        rd0, rd1 = _TrainTrunk.apply(self, inputs, d0, d1, *params)
        la, _, _, _ = _Head.apply(self, -1, False, rd0[:, -1], rd1[:, -1], *params)
        m0, m1, ms0, ms1 = filter_matches(la.detach(), float(c.filter_threshold))
        self.last_precision_used = "fp32"
        return {
            "matches0": m0,
            "matches1": m1,
            "matching_scores0": ms0,
            "matching_scores1": ms1,
            "ref_descriptors0": rd0,
            "ref_descriptors1": rd1,
            "log_assignment": la,
            "prune0": torch.full((b, m), float(L), device=device),
            "prune1": torch.full((b, n), float(L), device=device),
            "stop_layer": torch.full((b,), L - 1, dtype=torch.int64),
        }

    def _forward_native(self, k0, k1, d0, d1, s0, s1, sc0, o0, sc1, o1):
        """One lg_forward call on prepared (fp32, contiguous, on-device) inputs."""
        c = self.conf
        device = k0.device
        b, m, _ = k0.shape
        _, n, _ = k1.shape
        lib = self._ensure_handle(device)
        # early stop / pruning only in eval mode (lightglue.py:502-503).  The reference asserts
        # b == 1 (:528,533); here each pair of a batch prunes and stops on its own.
        pruning = (c.width_confidence > 0 or c.depth_confidence > 0) and not self.training
        L, dd = int(c.n_layers), int(c.descriptor_dim)
        m0 = torch.empty((b, m), dtype=torch.int64, device=device)
        m1 = torch.empty((b, n), dtype=torch.int64, device=device)
        ms0 = torch.empty((b, m), dtype=torch.float32, device=device)
        ms1 = torch.empty((b, n), dtype=torch.float32, device=device)
        la = torch.empty((b, m + 1, n + 1), dtype=torch.float32, device=device)
        if self.training:  # every layer's descriptors, torch.stack(all_desc0, 1) (:521-524,572)
            rd0 = torch.empty((b, L, m, dd), dtype=torch.float32, device=device)
            rd1 = torch.empty((b, L, n, dd), dtype=torch.float32, device=device)
        else:
            rd0 = torch.empty((b, m, dd), dtype=torch.float32, device=device)
            rd1 = torch.empty((b, n, dd), dtype=torch.float32, device=device)
        p0 = torch.empty((b, m), dtype=torch.int64, device=device)
        p1 = torch.empty((b, n), dtype=torch.int64, device=device)

        ws_bytes = ctypes.c_size_t()
        _lib.check(lib.lg_workspace_bytes(self._handle, b, m, n, ctypes.byref(ws_bytes)), "lg_workspace_bytes")
        if self._ws is None or self._ws.numel() < ws_bytes.value or self._ws.device != device:
            self._ws = torch.empty(max(ws_bytes.value, 1), dtype=torch.uint8, device=device)
        flags = _lib.LG_FWD_TRAINING_GATE if self.training else 0
        inp = _lib.LGInputs(b, m, n, *[_ptr(t) for t in (k0, k1, d0, d1, s0, s1, sc0, o0, sc1, o1)], flags)
        final, layers = (None, rd0) if self.training else (rd0, None)
        final1, layers1 = (None, rd1) if self.training else (rd1, None)
        kept = torch.empty((2, b), dtype=torch.int32, device=device) if pruning else None
        stop = torch.empty((b,), dtype=torch.int32, device=device) if pruning else None
        sim = torch.empty((b, m, n), dtype=torch.float32, device=device) if c.return_similarity else None
        out = _lib.LGOutputs(*[_ptr(t) for t in (m0, m1, ms0, ms1, la, final, final1, p0, p1, layers, layers1, kept, stop)],
                             0, 0, 0, 0, _ptr(sim))
        stream = torch.cuda.current_stream(device).cuda_stream
        _lib.check(
            lib.lg_forward(self._handle, ctypes.byref(inp), ctypes.byref(out), _ptr(self._ws), ws_bytes.value, ctypes.c_void_p(stream)),
            "lg_forward",
        )
        self.last_precision_used = "fp16x3" if out.precision_used == 0 else "bf16x6"
        if c.width_confidence > 0 and not self.training:
            prune0, prune1 = p0, p1
        else:
            prune0 = torch.full((b, m), float(L), device=device)
            prune1 = torch.full((b, n), float(L), device=device)
        pred = {
            "matches0": m0,
            "matches1": m1,
            "matching_scores0": ms0,
            "matching_scores1": ms1,
            "ref_descriptors0": rd0 if self.training else rd0[:, None],
            "ref_descriptors1": rd1 if self.training else rd1[:, None],
            "log_assignment": la,
            "prune0": prune0,
            "prune1": prune1,
            # extension key (no reference counterpart): index of the last executed layer, per pair
            "stop_layer": torch.full((b,), out.stop_layer, dtype=torch.int64),
        }
        if sim is not None:
            pred["similarity"] = sim
        if pruning:
            # kept points per pair (the library synchronised once to return them): the
            # reference's outputs cover the kept points only -- its log_assignment is
            # [1, M'+1, N'+1] -- so they are sliced per pair; B > 1 gives per-pair lists
            k0, k1 = out.kept0, out.kept1
            pred["stop_layer"] = stop.to(torch.int64)
            pred["kept0"], pred["kept1"] = kept[0].to(torch.int64), kept[1].to(torch.int64)
            # the similarity (return_similarity) is the kept block too: rows / columns past the kept
            # counts are workspace, and its kept rows are in the same compacted order as la
            if b == 1:
                pred["log_assignment"] = la[:, : k0 + 1, : k1 + 1]
                pred["ref_descriptors0"] = rd0[:, None, :k0]
                pred["ref_descriptors1"] = rd1[:, None, :k1]
                if sim is not None:
                    pred["similarity"] = sim[:, :k0, :k1]
            else:
                ks = kept.tolist()
                pred["log_assignment"] = [la[i, : ks[0][i] + 1, : ks[1][i] + 1] for i in range(b)]
                pred["ref_descriptors0"] = [rd0[i, None, : ks[0][i]] for i in range(b)]
                pred["ref_descriptors1"] = [rd1[i, None, : ks[1][i]] for i in range(b)]
                if sim is not None:
                    pred["similarity"] = [sim[i, : ks[0][i], : ks[1][i]] for i in range(b)]
        return pred

    # ------------------------------------------------------------ profiling (bench.py)
    def profile_enable(self, enable=True, only=None):
        """Start timing the hot kernel families (all, or only the names in `only`)."""
        if self._handle is None:
            raise RuntimeError("run one forward first (the native handle is created lazily)")
        code = int(bool(enable))
        if enable and only:
            code = 0
            for k in only:
                code |= 1 << (_lib.KERNEL_IDS[k] + 1)
        _lib.check(_lib.load().lg_profile_enable(self._handle, code), "lg_profile_enable")

    def profile_read(self, kernel):
        """(total_ms, launches, algorithmic_flops, algorithmic_bytes) since profile_enable()."""
        ms, n, fl, by = ctypes.c_double(), ctypes.c_int64(), ctypes.c_double(), ctypes.c_double()
        _lib.check(
            _lib.load().lg_profile_read(self._handle, _lib.KERNEL_IDS[kernel], ctypes.byref(ms), ctypes.byref(n),
                                        ctypes.byref(fl), ctypes.byref(by)),
            "lg_profile_read",
        )
        return ms.value, n.value, fl.value, by.value

    # ------------------------------------------------------------ training loss (forward values)
    def assignment_head(self, layer, desc0, desc1, token_logits=False):
        """``self.log_assignment[layer](desc0, desc1)`` (MatchAssignment, lightglue.py:306-315 +
        :284-296) on the HIP library: returns (log_assignment [B, M+1, N+1], similarity [B, M, N])
        and, with ``token_logits``, the ``token_confidence[layer]`` logits (before the sigmoid) of
        both descriptor sets.  ``layer`` indexes like a list (-1 = the last head)."""
        device = desc0.device
        if device.type != "cuda":
            raise RuntimeError("lightglue_amd: inputs must be on a HIP (cuda) device; there is no CPU path")
        lib = self._ensure_handle(device)
        d0 = desc0.to(torch.float32).contiguous()
        d1 = desc1.to(torch.float32).contiguous()
        b, m, _ = d0.shape
        n = d1.shape[1]
        la = torch.empty((b, m + 1, n + 1), dtype=torch.float32, device=device)
        sim = torch.empty((b, m, n), dtype=torch.float32, device=device)
        t0 = torch.empty((b, m), dtype=torch.float32, device=device) if token_logits else None
        t1 = torch.empty((b, n), dtype=torch.float32, device=device) if token_logits else None
        nb = ctypes.c_size_t()
        _lib.check(lib.lg_assignment_workspace_bytes(self._handle, b, m, n, ctypes.byref(nb)), "lg_assignment_workspace_bytes")
        ws = torch.empty(max(nb.value, 1), dtype=torch.uint8, device=device)
        stream = torch.cuda.current_stream(device).cuda_stream
        _lib.check(lib.lg_assignment_head(self._handle, int(layer), _ptr(d0), _ptr(d1), b, m, n, _ptr(la), _ptr(sim),
                                          _ptr(t0), _ptr(t1), _ptr(ws), nb.value, ctypes.c_void_p(stream)),
                   "lg_assignment_head")
        return (la, sim, t0, t1) if token_logits else (la, sim)

    def loss(self, pred, data):
        """LightGlue.loss (lightglue.py:614-663): the NLL of every layer's assignment head on that
        layer's descriptors (``pred["ref_descriptors*"]`` is [B, L, M, 256] in training mode,
        [B, 1, M, 256] in eval mode, so eval evaluates the last head only), weighted by
        ``gamma ** (L - i - 1)`` (or ``i + 1`` when gamma <= 0); the token-confidence BCE of layers
        0..L-2 (:108-122; added to ``total`` in training mode); ``row_norm``; and, in eval mode,
        ``matcher_metrics`` (models/utils/metrics.py).  Differentiable: each head + NLL term is one
        autograd Function (:class:`_HeadNLL`) whose backward runs in the HIP library; what stays in
        torch is the reference's per-point glue (argmax agreement, BCE on [B, M] logits, the
        gamma-weighted sum, metric ratios)."""
        lconf = self.conf.loss
        if lconf.get("fn", "nll") != "nll":
            raise NotImplementedError(f"loss fn {lconf.fn!r} (the reference defines only 'nll')")
        from .superglue import nll_inputs, nll_weights

        bal = float(lconf.nll_balancing)
        rd0, rd1 = pred["ref_descriptors0"], pred["ref_descriptors1"]
        N = rd0.shape[1]
        params = self._schema_params(rd0.device)
        b, m, n = rd0.shape[0], rd0.shape[2], rd1.shape[2]
        # the ground truth's loss weights (losses.py:62-73) once, as the reference (gt_weights, :633);
        # by default never as a dense [B, M+1, N+1] tensor: the heads' backward reads them from the
        # ground truth (bit-identical, lg_head_nll_backward)
        w = nll_weights(rd0.new_empty((b, m + 1, n + 1)), data) if not _HEAD_GT else None
        gt = (data, w, nll_inputs(data, rd0.device))

        sl0, sl1 = _LayerSlices.apply(rd0), _LayerSlices.apply(rd1)

        def head(i, tokens):
            return _HeadNLL.apply(self, i, gt, bal, tokens, sl0[i], sl1[i], *params)

        nll, nll_pos, nll_neg, num_pos, num_neg, _, _, _, _ = head(-1, False)
        losses = {"total": nll, "last": nll.clone().detach(), "assignment_nll": nll, "nll_pos": nll_pos,
                  "nll_neg": nll_neg, "num_matchable": num_pos, "num_unmatchable": num_neg}
        sum_weights = 1.0
        if self.training:
            losses["confidence"] = 0.0
        la_final = pred["log_assignment"].detach()
        losses["row_norm"] = la_final.exp()[:, :-1].sum(2).mean(1)
        bce = torch.nn.functional.binary_cross_entropy_with_logits
        if N > 1:  # the final head's argmaxes, shared by every layer's TokenConfidence.loss
            fin0 = la_final[:, :-1, :].max(-1).indices
            fin1 = la_final[:, :, :-1].max(-2).indices
        for i in range(N - 1):
            nll_i, _, _, _, _, am0_i, am1_i, lg0, lg1 = head(i, True)
            weight = lconf.gamma ** (N - i - 1) if lconf.gamma > 0.0 else i + 1
            sum_weights += weight
            losses["total"] = losses["total"] + nll_i * weight
            # TokenConfidence.loss (:108-122): does layer i already pick the final argmax?
            hit0 = (fin0 == am0_i).float()
            hit1 = (fin1 == am1_i).float()
            tok = (bce(lg0, hit0, reduction="none").mean(-1) + bce(lg1, hit1, reduction="none").mean(-1)) / 2.0
            losses["confidence"] = losses.get("confidence", 0.0) + tok / (N - 1)
        losses["total"] = losses["total"] / sum_weights
        if self.training:
            losses["total"] = losses["total"] + losses["confidence"]
        metrics = {} if self.training else matcher_metrics(pred, data)
        return losses, metrics


@torch.no_grad()
def matcher_metrics(pred, data, prefix="", prefix_gt=None):
    """models/utils/metrics.py:4-50 (match recall / precision / accuracy / ranking AP of
    ``matches0`` against ``gt_matches0``), restated as ratios of per-pair counts over [B, M].
    The reference's ranking AP sums the consecutive steps of the score-sorted recall curve times the
    curve's LAST precision point (``p_pts[:, None, -1]``): the sum telescopes to
    precision * (recall - recall point of the best-scoring keypoint), computed here without the
    sort (ties for the best score resolve to the first index)."""
    pg = prefix if prefix_gt is None else prefix_gt
    m = pred[f"{prefix}matches0"]
    gt = data[f"gt_{pg}matches0"].to(m.device)
    hit = (m == gt).float()
    labelled = (gt >= -1).float()
    matchable = (gt > -1).float()
    claimed = ((m > -1) & (gt >= -1)).float()
    eps = 1e-8

    def rate(mask):
        return (hit * mask).sum(1) / (eps + mask.sum(1))

    recall, precision = rate(matchable), rate(claimed)
    best = pred[f"{prefix}matching_scores0"].argmax(1, keepdim=True)
    first = (hit * matchable).gather(1, best).squeeze(1) / (eps + matchable.sum(1))
    return {
        f"{prefix}match_recall": recall,
        f"{prefix}match_precision": precision,
        f"{prefix}accuracy": rate(labelled),
        f"{prefix}average_precision": precision * (recall - first),
    }


__main_model__ = LightGlue
