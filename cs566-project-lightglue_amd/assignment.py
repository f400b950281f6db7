"""Functional drop-ins for the reference's assignment helpers, on the HIP library.

* :func:`filter_matches`       == ``gluefactory/models/matchers/lightglue.py:321-337``
                                  (identical to ``gluefactory_nonfree/superglue.py:288-298``)
* :func:`log_optimal_transport` == ``gluefactory_nonfree/superglue.py:181-201``

Inputs must be fp32 CUDA (HIP) tensors; there is no CPU path.
"""
import ctypes

import torch

from . import _lib


def _stream(t):
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def _require_gpu(t, name):
    if not isinstance(t, torch.Tensor) or t.device.type != "cuda":
        raise RuntimeError(f"lightglue_amd: {name} must be a HIP (cuda) tensor; there is no CPU path")


def filter_matches(scores: torch.Tensor, th: float):
    """Mutual nearest neighbours + threshold on a [B, M+1, N+1] log assignment."""
    _require_gpu(scores, "scores")
    lib = _lib.load()
    scores = scores.to(torch.float32).contiguous()
    b, m1, n1 = scores.shape
    m, n = m1 - 1, n1 - 1
    dev = scores.device
    out = [
        torch.empty((b, m), dtype=torch.int64, device=dev),
        torch.empty((b, n), dtype=torch.int64, device=dev),
        torch.empty((b, m), dtype=torch.float32, device=dev),
        torch.empty((b, n), dtype=torch.float32, device=dev),
    ]
    ws_b = ctypes.c_size_t()
    _lib.check(lib.lg_filter_workspace_bytes(b, m, n, ctypes.byref(ws_b)), "lg_filter_workspace_bytes")
    ws = torch.empty(max(ws_b.value, 1), dtype=torch.uint8, device=dev)
    _lib.check(
        lib.lg_filter_matches(
            ctypes.c_void_p(scores.data_ptr()), b, m, n, float(th),
            *[ctypes.c_void_p(t.data_ptr()) for t in out],
            ctypes.c_void_p(ws.data_ptr()), ws_b.value, _stream(scores),
        ),
        "lg_filter_matches",
    )
    return tuple(out)


def log_optimal_transport(scores: torch.Tensor, alpha, iters: int) -> torch.Tensor:
    """Log-domain Sinkhorn with dustbins; returns Z [B, M+1, N+1] (already multiplied by M+N)."""
    _require_gpu(scores, "scores")
    lib = _lib.load()
    scores = scores.to(torch.float32).contiguous()
    b, m, n = scores.shape
    alpha = float(alpha.item() if isinstance(alpha, torch.Tensor) else alpha)
    Z = torch.empty((b, m + 1, n + 1), dtype=torch.float32, device=scores.device)
    ws_b = ctypes.c_size_t()
    _lib.check(lib.lg_sinkhorn_workspace_bytes(b, m, n, ctypes.byref(ws_b)), "lg_sinkhorn_workspace_bytes")
    ws = torch.empty(max(ws_b.value, 1), dtype=torch.uint8, device=scores.device)
    _lib.check(
        lib.lg_log_optimal_transport(
            ctypes.c_void_p(scores.data_ptr()), alpha, b, m, n, int(iters), ctypes.c_void_p(Z.data_ptr()),
            ctypes.c_void_p(ws.data_ptr()), ws_b.value, _stream(scores),
        ),
        "lg_log_optimal_transport",
    )
    return Z
