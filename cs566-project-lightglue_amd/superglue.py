"""MI355X-native SuperGlue matcher: drop-in for ``gluefactory_nonfree.superglue.SuperGlue``
(reference ``superglue.py:204-342``) and for the NLL loss of ``gluefactory/models/utils/losses.py``.

Same config keys (:205-217), same module tree (``kenc.encoder`` MLP, ``gnn.layers.<i>.attn``
{``proj``, ``merge``} / ``mlp``, ``final_proj``, ``bin_score``: checkpoints load unchanged), same
``forward(data) -> dict`` outputs (:300-307) and ``loss(pred, data)`` (:309-339).  The forward is
the HIP path of ``liblightglue_mi355x.so`` (``include/superglue_mi355x.h``): keypoint encoder
kernel, the LightGlue fp16x3 GEMM / attention kernels for the 18-layer GNN (merge and eval
BatchNorm folded into the MLP's first linear at load time), bf16x6 cost GEMM, the log-domain
Sinkhorn kernel and the mutual filter.  No CPU fallback: CPU inputs raise.

Deliberate differences from the reference:

* the trained checkpoint is a download (:248-251); the module starts from PyTorch's default init
  (``weights`` is ignored) and takes weights through ``load_state_dict``;
* training mode runs ``sg_train_forward`` / ``sg_train_backward`` (a ``torch.autograd.Function``
  over raw parameters): BatchNorm with batch statistics per image set and the running-statistics
  updates of the reference's step, including the second GNN update its
  ``torch.utils.checkpoint`` recomputation makes (:151-155); ``loss`` is differentiable through
  ``sg_nll_backward``;
* ``NLLLoss`` with explicit ``weights`` other than the ground truth's raises NotImplementedError
  (the kernel derives the weights from the ground truth, losses.py:46-73).
"""
import ctypes

import torch
from torch import nn

from . import _lib
from .lightglue import merge_conf
from .sg_weights import SG_DEFAULT_CONF


def _ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _mlp(channels):  # superglue.py:63-72 (parameter container)
    layers = []
    for i in range(1, len(channels)):
        layers.append(nn.Conv1d(channels[i - 1], channels[i], kernel_size=1, bias=True))
        if i < len(channels) - 1:
            layers.append(nn.BatchNorm1d(channels[i]))
            layers.append(nn.ReLU())
    return nn.Sequential(*layers)


class _KeypointEncoder(nn.Module):  # superglue.py:89-104
    def __init__(self, feature_dim, layers, use_scores=True):
        super().__init__()
        self.encoder = _mlp([3 if use_scores else 2] + list(layers) + [feature_dim])
        nn.init.constant_(self.encoder[-1].bias, 0.0)


class _MultiHeadedAttention(nn.Module):  # superglue.py:113-128
    def __init__(self, h, d_model):
        super().__init__()
        self.merge = nn.Conv1d(d_model, d_model, kernel_size=1)
        self.proj = nn.ModuleList([nn.Conv1d(d_model, d_model, kernel_size=1) for _ in range(3)])


class _AttentionalPropagation(nn.Module):  # superglue.py:131-139
    def __init__(self, num_dim, num_heads):
        super().__init__()
        self.attn = _MultiHeadedAttention(num_heads, num_dim)
        self.mlp = _mlp([num_dim * 2, num_dim * 2, num_dim])
        nn.init.constant_(self.mlp[-1].bias, 0.0)


class _AttentionalGNN(nn.Module):  # superglue.py:142-170
    def __init__(self, feature_dim, layer_names):
        super().__init__()
        self.layers = nn.ModuleList([_AttentionalPropagation(feature_dim, 4) for _ in range(len(layer_names))])
        self.names = list(layer_names)


class SuperGlue(nn.Module):
    default_conf = SG_DEFAULT_CONF
    required_data_keys = ["view0", "view1", "keypoints0", "keypoints1", "descriptors0", "descriptors1",
                          "keypoint_scores0", "keypoint_scores1"]
    checkpoint_url = "https://github.com/magicleap/SuperGluePretrainedNetwork/raw/master/models/weights/superglue_{}.pth"

    def __init__(self, conf=None):
        super().__init__()
        self.conf = conf = merge_conf(self.default_conf, conf or {})
        if int(conf.descriptor_dim) != 256:
            raise ValueError("lightglue_amd.SuperGlue: descriptor_dim must be 256")
        if len(conf.GNN_layers) > _lib.SG_MAX_LAYERS or len(conf.keypoint_encoder) > _lib.SG_MAX_KENC:
            raise ValueError("lightglue_amd.SuperGlue: too many GNN / keypoint-encoder layers")
        for n in conf.GNN_layers:
            if n not in ("self", "cross"):
                raise ValueError(n)
        self.kenc = _KeypointEncoder(conf.descriptor_dim, conf.keypoint_encoder, conf.use_scores)
        self.gnn = _AttentionalGNN(conf.descriptor_dim, conf.GNN_layers)
        self.final_proj = nn.Conv1d(conf.descriptor_dim, conf.descriptor_dim, kernel_size=1, bias=True)
        self.register_parameter("bin_score", nn.Parameter(torch.tensor(1.0)))
        self._handle = None
        self._handle_device = None
        self._weights_key = None
        self._ws = None

    # ------------------------------------------------------------ native handle
    def _lib_config(self):
        c = self.conf
        cfg = _lib.SGConfig()
        cfg.descriptor_dim = int(c.descriptor_dim)
        cfg.n_layers = len(c.GNN_layers)
        for i, n in enumerate(c.GNN_layers):
            cfg.layer_types[i] = 0 if n == "self" else 1
        cfg.n_kenc = len(c.keypoint_encoder)
        for i, w in enumerate(c.keypoint_encoder):
            cfg.keypoint_encoder[i] = int(w)
        cfg.use_scores = int(bool(c.use_scores))
        cfg.sinkhorn_iterations = int(c.num_sinkhorn_iterations)
        cfg.filter_threshold = float(c.filter_threshold)
        return cfg

    def _weights_signature(self):
        return tuple((id(m), n, t.data_ptr(), t._version) for m in self.modules()
                     for n, t in list(m._parameters.items()) + list(m._buffers.items()) if t is not None)

    def _ensure_handle(self, device, upload=True):
        lib = _lib.load()
        if self._handle is not None and self._handle_device != device:
            lib.sg_destroy(self._handle)
            self._handle = None
        if self._handle is None:
            h = ctypes.c_void_p()
            cfg = self._lib_config()
            _lib.check(lib.sg_create(ctypes.byref(cfg), device.index or 0, ctypes.byref(h)), "sg_create")
            self._handle, self._handle_device, self._weights_key = h, device, None
        if not upload:
            return lib
        key = self._weights_signature()
        if key != self._weights_key:
            sd = {k: v for k, v in self.state_dict(keep_vars=True).items() if not k.endswith("num_batches_tracked")}
            names = list(sd)
            ts = []
            for n in names:
                t = sd[n].detach()
                if t.device != device or t.dtype != torch.float32:
                    raise RuntimeError(f"lightglue_amd.SuperGlue: tensor {n} is {t.dtype} on {t.device}; "
                                       f"move the module to {device} in fp32")
                ts.append(t.contiguous())
            arr_n = (ctypes.c_char_p * len(names))(*[n.encode() for n in names])
            arr_p = (ctypes.c_void_p * len(ts))(*[t.data_ptr() for t in ts])
            arr_k = (ctypes.c_int64 * len(ts))(*[t.numel() for t in ts])
            stream = torch.cuda.current_stream(device).cuda_stream
            _lib.check(lib.sg_load_weights(self._handle, len(ts), arr_n, arr_p, arr_k, ctypes.c_void_p(stream)),
                       "sg_load_weights")
            torch.cuda.current_stream(device).synchronize()
            self._weights_key = key
        return lib

    def reload_weights(self):
        self._weights_key = None

    def _apply(self, fn, *args, **kwargs):
        self._weights_key = None
        return super()._apply(fn, *args, **kwargs)

    def __del__(self):
        try:
            if self._handle is not None and _lib._lib is not None:
                _lib._lib.sg_destroy(self._handle)
        except Exception:
            pass

    def _workspace(self, lib, device, B, M, N):
        nb = ctypes.c_size_t()
        _lib.check(lib.sg_workspace_bytes(self._handle, B, M, N, ctypes.byref(nb)), "sg_workspace_bytes")
        if self._ws is None or self._ws.numel() < nb.value or self._ws.device != device:
            self._ws = torch.empty(nb.value, dtype=torch.uint8, device=device)
        return self._ws, nb.value

    # ------------------------------------------------------------ forward (superglue.py:253-307)
    def forward(self, data: dict, return_descriptors: bool = False) -> dict:
        """``return_descriptors``: also return the GNN output (the input of ``final_proj``) as
        ``gnn_descriptors0/1`` [B, N, D] (a check point for tests; not a reference output)."""
        for k in self.required_data_keys:
            assert k in data, f"Missing key {k} in data"
        c = self.conf
        kpts0, kpts1 = data["keypoints0"], data["keypoints1"]
        if kpts0.shape[1] == 0 or kpts1.shape[1] == 0:  # no keypoints (:257-264)
            shape0, shape1 = kpts0.shape[:-1], kpts1.shape[:-1]
            return {
                "matches0": kpts0.new_full(shape0, -1, dtype=torch.int),
                "matches1": kpts1.new_full(shape1, -1, dtype=torch.int),
                "matching_scores0": kpts0.new_zeros(shape0),
                "matching_scores1": kpts1.new_zeros(shape1),
            }
        if not kpts0.is_cuda:
            raise RuntimeError("lightglue_amd.SuperGlue runs on a HIP device; inputs are on the CPU")
        device = kpts0.device
        B, M, N = kpts0.shape[0], kpts0.shape[1], kpts1.shape[1]

        def size_of(view):  # normalize_keypoints' size / image-shape fallback (:78-83)
            s = view.get("image_size")
            if s is not None:
                return s.to(device=device, dtype=torch.float32).contiguous(), 0, 0
            h, w = view["image"].shape[-2:]
            return None, int(w), int(h)

        s0, w0, h0 = size_of(data["view0"])
        s1, w1, h1 = size_of(data["view1"])
        # the reference asserts every normalised keypoint lies in [-1, 1] (:272-273)
        for k, s, w, h in ((kpts0, s0, w0, h0), (kpts1, s1, w1, h1)):
            size = s if s is not None else torch.tensor([[float(w), float(h)]], device=device)
            kn = (k.float() - (size / 2)[:, None]) / (size.max(1).values * 0.7)[:, None, None]
            assert torch.all(kn >= -1) and torch.all(kn <= 1)

        def f32(t):
            return t.to(device=device, dtype=torch.float32).contiguous()

        k0, k1 = f32(kpts0), f32(kpts1)
        d0, d1 = f32(data["descriptors0"]), f32(data["descriptors1"])
        sc0 = f32(data["keypoint_scores0"]) if c.use_scores else None
        sc1 = f32(data["keypoint_scores1"]) if c.use_scores else None
        if self.training:
            inp = _lib.SGInputs(B, M, N, _ptr(k0), _ptr(k1), _ptr(d0), _ptr(d1), _ptr(sc0), _ptr(sc1), _ptr(s0), _ptr(s1),
                                w0, h0, w1, h1)
            return self._forward_train(device, inp, (k0, k1, d0, d1, sc0, sc1, s0, s1), return_descriptors)
        lib = self._ensure_handle(device)
        ws, nb = self._workspace(lib, device, B, M, N)
        m0 = torch.empty((B, M), dtype=torch.int64, device=device)
        m1 = torch.empty((B, N), dtype=torch.int64, device=device)
        ms0 = torch.empty((B, M), device=device)
        ms1 = torch.empty((B, N), device=device)
        cost = torch.empty((B, M, N), device=device)
        la = torch.empty((B, M + 1, N + 1), device=device)
        inp = _lib.SGInputs(B, M, N, _ptr(k0), _ptr(k1), _ptr(d0), _ptr(d1), _ptr(sc0), _ptr(sc1), _ptr(s0), _ptr(s1),
                            w0, h0, w1, h1)
        g0 = torch.empty((B, M, 256), device=device) if return_descriptors else None
        g1 = torch.empty((B, N, 256), device=device) if return_descriptors else None
        out = _lib.SGOutputs(_ptr(m0), _ptr(m1), _ptr(ms0), _ptr(ms1), _ptr(cost), _ptr(la), _ptr(g0), _ptr(g1))
        stream = ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)
        _lib.check(lib.sg_forward(self._handle, ctypes.byref(inp), ctypes.byref(out), _ptr(ws), nb, stream), "sg_forward")
        pred = {"sinkhorn_cost": cost, "log_assignment": la, "matches0": m0, "matches1": m1, "matching_scores0": ms0,
                "matching_scores1": ms1}
        if return_descriptors:
            pred["gnn_descriptors0"], pred["gnn_descriptors1"] = g0, g1
        return pred

    # ------------------------------------------------------------ training (superglue.py:148-155,253-307)
    def _schema_tensors(self):
        """(name, tensor) in the library's schema order: parameters and BatchNorm running buffers."""
        lib = _lib.load()
        sd = dict(self.named_parameters())
        sd.update({n: b for n, b in self.named_buffers() if not n.endswith("num_batches_tracked")})
        out = []
        for i in range(lib.sg_weight_count(self._handle)):
            n = lib.sg_weight_name(self._handle, i).decode()
            out.append((n, sd[n]))
        return out

    def _forward_train(self, device, inp, keep, return_descriptors):
        for n, m in self.named_modules():
            # the training kernels update running statistics with nn.BatchNorm1d's defaults:
            # refuse a module configured otherwise instead of silently ignoring its settings
            if isinstance(m, nn.BatchNorm1d) and (m.momentum != 0.1 or not m.track_running_stats or not m.affine
                                                  or m.eps != 1e-5):
                raise NotImplementedError(
                    f"lightglue_amd.SuperGlue training: BatchNorm1d {n} must keep momentum=0.1, eps=1e-5, "
                    f"affine=True, track_running_stats=True (got momentum={m.momentum}, eps={m.eps})")
        self._ensure_handle(device, upload=False)
        self._weights_key = None  # the eval path re-uploads: parameters / running stats change in place
        named = self._schema_tensors()
        for n, t in named:
            if t.device != device or t.dtype != torch.float32 or not t.is_contiguous():
                raise RuntimeError(f"lightglue_amd.SuperGlue: tensor {n} must be contiguous fp32 on {device}")
        params = [t for _, t in named if isinstance(t, nn.Parameter)]
        la, cost, m0, m1, ms0, ms1, g0, g1 = _SGTrain.apply(self, (inp, keep, named, return_descriptors), keep[2], keep[3],
                                                            *params)
        for m in self.modules():  # one running-statistics update per image set (:274-275, :160-170)
            if isinstance(m, nn.BatchNorm1d) and m.num_batches_tracked is not None:
                m.num_batches_tracked.add_(2)
        pred = {"sinkhorn_cost": cost, "log_assignment": la, "matches0": m0, "matches1": m1, "matching_scores0": ms0,
                "matching_scores1": ms1}
        if return_descriptors:
            pred["gnn_descriptors0"], pred["gnn_descriptors1"] = g0, g1
        return pred

    def _relu_masks(self, lib, saved, B, M, N):
        """The training forward's ReLU decisions (``keep_relu_masks = True``; test instrumentation):
        {BatchNorm name: (image-0 mask [B, C, M], image-1 mask [B, C, N])} read from the saved
        post-ReLU activations (sg_train_saved_tensor)."""
        out = {}
        for name, m in self.named_modules():
            if not isinstance(m, nn.BatchNorm1d):
                continue
            off, n = ctypes.c_size_t(), ctypes.c_size_t()
            _lib.check(lib.sg_train_saved_tensor(self._handle, B, M, N, name.encode(), ctypes.byref(off), ctypes.byref(n)),
                       "sg_train_saved_tensor")
            g = saved[off.value:off.value + 4 * n.value].view(torch.float32).view(B * (M + N), -1)
            C = g.shape[1]
            out[name] = ((g[:B * M] > 0).view(B, M, C).permute(0, 2, 1).contiguous(),
                         (g[B * M:] > 0).view(B, N, C).permute(0, 2, 1).contiguous())
        return out

    def loss(self, pred, data):
        """superglue.py:309-339; differentiable in ``pred["log_assignment"]`` (sg_nll_backward)."""
        la = pred["log_assignment"]
        bal = float(self.conf.loss.nll_balancing)
        out = _SGNLL.apply(la, data, 0, bal) if la.requires_grad else _nll(la, data, 0, bal)
        losses = {"total": out[0], "assignment_nll": out[0], "nll_pos": out[1], "nll_neg": out[2],
                  "num_matchable": out[3], "num_unmatchable": out[4], "bin_score": self.bin_score[None]}
        return losses

    def metrics(self, pred, data):
        raise NotImplementedError


class _SGTrain(torch.autograd.Function):
    """sg_train_forward / sg_train_backward over the raw parameters (schema order)."""

    @staticmethod
    def forward(ctx, model, feed, d0, d1, *params):
        inp, keep, named, want_desc = feed
        lib = _lib.load()
        h = model._handle
        B, M, N = inp.B, inp.M, inp.N
        dev = d0.device
        nb = ctypes.c_size_t()
        _lib.check(lib.sg_train_saved_bytes(h, B, M, N, ctypes.byref(nb)), "sg_train_saved_bytes")
        saved = torch.empty(nb.value, dtype=torch.uint8, device=dev)
        la = torch.empty((B, M + 1, N + 1), device=dev)
        cost = torch.empty((B, M, N), device=dev)
        m0 = torch.empty((B, M), dtype=torch.int64, device=dev)
        m1 = torch.empty((B, N), dtype=torch.int64, device=dev)
        ms0 = torch.empty((B, M), device=dev)
        ms1 = torch.empty((B, N), device=dev)
        g0 = torch.empty((B, M, 256), device=dev) if want_desc else None
        g1 = torch.empty((B, N, 256), device=dev) if want_desc else None
        out = _lib.SGOutputs(_ptr(m0), _ptr(m1), _ptr(ms0), _ptr(ms1), _ptr(cost), _ptr(la), _ptr(g0), _ptr(g1))
        ptrs = (ctypes.c_void_p * len(named))(*[t.data_ptr() for _, t in named])
        stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
        ddp = getattr(model, "_ddp", None)  # ddp.DataParallel: SyncBatchNorm over the ranks
        if ddp is not None:
            ddp.attach_collective(lib, h, dev)
        else:
            _lib.check(lib.sg_set_collective(h, None, None, None, 0), "sg_set_collective")
        rc = lib.sg_train_forward(h, ptrs, ctypes.byref(inp), ctypes.byref(out), _ptr(saved), nb.value, stream)
        if ddp is not None:
            ddp.check_collective()
            if rc != _lib.LG_OK:  # a failure between SyncBatchNorm collectives strands the peers
                try:
                    _lib.check(rc, "sg_train_forward")
                except Exception as e:
                    ddp.abort(e)
        _lib.check(rc, "sg_train_forward")
        if getattr(model, "keep_relu_masks", False):
            model.last_relu_masks = model._relu_masks(lib, saved, B, M, N)
        ctx.model, ctx.inp, ctx.keep, ctx.named, ctx.saved = model, inp, keep, named, saved
        ctx.keep_desc = (d0, d1)
        nd = [m0, m1, ms0, ms1] + [t for t in (g0, g1) if t is not None]
        ctx.mark_non_differentiable(*nd)
        return la, cost, m0, m1, ms0, ms1, g0, g1

    @staticmethod
    def backward(ctx, g_la, g_cost, *_):
        lib = _lib.load()
        model, inp, named = ctx.model, ctx.inp, ctx.named
        B, M, N = inp.B, inp.M, inp.N
        dev = ctx.saved.device
        ddp = getattr(model, "_ddp", None)  # ddp.DataParallel: per-layer all-reduces under the backward
        if ddp is not None:
            names = [n for n, _ in named]
            tensors = [t for _, t in named]
            wanted = [isinstance(t, nn.Parameter) for t in tensors]
            buckets = ddp.buckets(names, tensors, wanted, len(model.conf.GNN_layers), True, dev)
            grads = buckets.grads
            _lib.check(lib.sg_set_grad_ready_hook(model._handle, _lib.fnptr(buckets.callback(_lib.SG_GRAD_READY_FN)),
                                                   None),
                       "sg_set_grad_ready_hook")
        else:
            grads = [torch.empty_like(t) if isinstance(t, nn.Parameter) else None for _, t in named]
        gd0 = torch.empty((B, M, 256), device=dev) if ctx.needs_input_grad[2] else None
        gd1 = torch.empty((B, N, 256), device=dev) if ctx.needs_input_grad[3] else None
        nb = ctypes.c_size_t()
        _lib.check(lib.sg_train_scratch_bytes(model._handle, B, M, N, ctypes.byref(nb)), "sg_train_scratch_bytes")
        scratch = torch.empty(nb.value, dtype=torch.uint8, device=dev)
        ptrs = (ctypes.c_void_p * len(named))(*[t.data_ptr() for _, t in named])
        gptrs = (ctypes.c_void_p * len(named))(*[g.data_ptr() if g is not None else None for g in grads])
        g_la = g_la.float().contiguous() if g_la is not None else None
        g_cost = g_cost.float().contiguous() if g_cost is not None else None
        stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
        try:
            rc = lib.sg_train_backward(model._handle, ptrs, ctypes.byref(inp), _ptr(ctx.saved), ctx.saved.numel(),
                                       _ptr(g_la), _ptr(g_cost), gptrs, _ptr(gd0), _ptr(gd1), _ptr(scratch), nb.value,
                                       stream)
            if ddp is not None:
                ddp.check_collective()
            _lib.check(rc, "sg_train_backward")
        except Exception as e:
            if ddp is not None:
                ddp.abort(e)  # fewer collectives than the peers issue: fatal to the job, never a hang
            raise
        finally:
            if ddp is not None:
                lib.sg_set_grad_ready_hook(model._handle, None, None)
        if ddp is not None:
            grads = buckets.finish()  # wait for the layer buckets, average over the ranks
        ctx.saved = None
        for n, m in model.named_modules():  # the checkpoint recomputation's second GNN update
            if n.startswith("gnn.") and isinstance(m, nn.BatchNorm1d) and m.num_batches_tracked is not None:
                m.num_batches_tracked.add_(2)
        return (None, None, gd0, gd1, *[g for g in grads if g is not None])


class _SGNLL(torch.autograd.Function):
    """sg_nll_loss with its gradient (sg_nll_backward): out [5, B]; rows 0-2 differentiable."""

    @staticmethod
    def forward(ctx, la, data, mode, balancing):
        prepared = nll_inputs(data, la.device)
        out = _nll(la.detach(), data, mode, balancing, prepared)
        ctx.prepared, ctx.mode, ctx.bal, ctx.shape = prepared, mode, balancing, la.shape
        ctx.save_for_backward(out)
        return out

    @staticmethod
    def backward(ctx, g):
        (out,) = ctx.saved_tensors
        B, M1, N1 = ctx.shape
        g = g.float().contiguous()
        gla = torch.empty((B, M1, N1), device=out.device)
        gta, g0, g1 = ctx.prepared
        lib = _lib.load()
        stream = ctypes.c_void_p(torch.cuda.current_stream(out.device).cuda_stream)
        _lib.check(lib.sg_nll_backward(_ptr(out), _ptr(g[0]), _ptr(g[1]), _ptr(g[2]), B, M1 - 1, N1 - 1, _ptr(gta),
                                       _ptr(g0), _ptr(g1), ctx.mode, ctx.bal, _ptr(gla), stream), "sg_nll_backward")
        return gla, None, None, None


def nll_inputs(data, device):
    """The ground truth in the layouts sg_nll_loss reads (uint8 assignment, int64 matches); convert
    once per loss() and pass ``prepared=`` to every head's _nll."""
    a = data["gt_assignment"].to(device=device)
    # a bool assignment is read as its uint8 bytes in place (no conversion pass over B x M x N)
    a = (a if a.dtype == torch.bool else a.bool()).contiguous().view(torch.uint8)
    return (a,
            data["gt_matches0"].to(device=device, dtype=torch.int64).contiguous(),
            data["gt_matches1"].to(device=device, dtype=torch.int64).contiguous())


def _nll(la, data, mode, balancing, prepared=None):
    if not la.is_cuda:
        raise RuntimeError("lightglue_amd NLL loss runs on a HIP device; inputs are on the CPU")
    device = la.device
    B, M1, N1 = la.shape
    gta, g0, g1 = prepared if prepared is not None else nll_inputs(data, device)
    la = la.float().contiguous()
    out = torch.empty((5, B), device=device)
    lib = _lib.load()
    stream = ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)
    nb = ctypes.c_size_t()
    _lib.check(lib.sg_nll_workspace_bytes(B, M1 - 1, ctypes.byref(nb)), "sg_nll_workspace_bytes")
    ws = torch.empty(max(nb.value, 8), dtype=torch.uint8, device=device)  # torch allocator, stream-ordered
    rc = lib.sg_nll_loss_ws(_ptr(la), B, M1 - 1, N1 - 1, _ptr(gta), _ptr(g0), _ptr(g1), mode, balancing, _ptr(out),
                            _ptr(ws), nb.value, stream)
    if rc == _lib.LG_E_INVALID and mode == 1 and M1 != N1:
        raise RuntimeError(lib.lg_last_error().decode(errors="replace"))  # the reference's own error type
    _lib.check(rc, "sg_nll_loss")
    return out


def nll_weights(la, data):
    """losses.py:62-73 (``NLLLoss.nll_loss``): the [B, M+1, N+1] loss weights of a ground truth,
    built on the device exactly as the reference builds them (column dustbin written at [:, -1, :m],
    so only M == N runs, as in the reference)."""
    m, n = data["gt_matches0"].size(-1), data["gt_matches1"].size(-1)
    dev = la.device
    weights = torch.zeros_like(la)
    weights[:, :m, :n] = data["gt_assignment"].to(dev).float()
    weights[:, :m, -1] = (data["gt_matches0"].to(dev) == -1).float()
    weights[:, -1, :m] = (data["gt_matches1"].to(dev) == -1).float()
    return weights


class NLLLoss(nn.Module):
    """losses.py:26-73, differentiable in ``log_assignment`` (sg_nll_backward): ``forward(pred, data, weights=None) ->
    (nll, weights, metrics)``.  The sums run in ``sg_nll_kernel`` (fp64), which derives the weights
    from the ground truth itself; the returned ``weights`` tensor is the reference's [B, M+1, N+1]
    one (losses.py:52-60).  Explicit ``weights`` must be those ground-truth weights (what
    LightGlue.loss passes back, lightglue.py:633); any other weighting raises NotImplementedError."""

    default_conf = {"nll_balancing": 0.5, "gamma_f": 0.0}

    def __init__(self, conf=None):
        super().__init__()
        self.conf = merge_conf(self.default_conf, conf or {})

    def forward(self, pred, data, weights=None):
        la = pred["log_assignment"]
        derived = nll_weights(la, data)
        if weights is not None and not (weights.shape == derived.shape and torch.equal(weights.to(la.device), derived)):
            raise NotImplementedError("explicit loss weights other than the ground truth's (the kernel derives them)")
        bal = float(self.conf.nll_balancing)
        out = _SGNLL.apply(la, data, 1, bal) if la.requires_grad else _nll(la, data, 1, bal)
        metrics = {"assignment_nll": out[0], "nll_pos": out[1], "nll_neg": out[2], "num_matchable": out[3],
                   "num_unmatchable": out[4]}
        return out[0], derived, metrics
