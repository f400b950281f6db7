"""Functional drop-ins for the reference's assignment helpers, on the HIP library.

* :func:`filter_matches`       == ``gluefactory/models/matchers/lightglue.py:321-337``
                                  (identical to ``gluefactory_nonfree/superglue.py:288-298``)
* :func:`log_optimal_transport` == ``gluefactory_nonfree/superglue.py:181-201``
* :func:`sinkhorn_match`        == configs[4]'s composition: a LightGlue forward's final similarity
                                  (``lightglue.py:306-315``) through the SuperGlue Sinkhorn head
                                  (``superglue.py:181-201,214``) and its mutual filter (``:288-298``)

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


# SuperGlue's head (superglue.py:214-215; bin_score initialised to 1.0): 50 iterations, threshold 0.2
SINKHORN_ALPHA, SINKHORN_ITERS, SINKHORN_THRESHOLD = 1.0, 50, 0.2


def sinkhorn_match(model, data, alpha=SINKHORN_ALPHA, iters=SINKHORN_ITERS, threshold=SINKHORN_THRESHOLD,
                   on_sinkhorn=None):
    """configs[4] (BASELINE.json): ``model`` (a LightGlue with ``return_similarity``) matches
    ``data``; its final head's similarity goes through ``log_optimal_transport`` and
    ``filter_matches``.  ``on_sinkhorn(t0, t1)`` (optional) is called with two recorded CUDA events
    around the Sinkhorn call (bench.py times the kernel with them).  Returns the matches dict and Z."""
    pred = model(data)
    sim = pred["similarity"]
    if isinstance(sim, list):
        raise ValueError("sinkhorn_match needs a dense similarity (pruning off)")
    e0 = e1 = None
    if on_sinkhorn is not None:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
    Z = log_optimal_transport(sim, alpha, iters)
    if on_sinkhorn is not None:
        e1.record()
        on_sinkhorn(e0, e1)
    m0, m1, s0, s1 = filter_matches(Z, threshold)
    return {"matches0": m0, "matches1": m1, "matching_scores0": s0, "matching_scores1": s1}, Z
