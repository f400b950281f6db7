#!/usr/bin/env python3
"""Training-GEMM shapes of one configs[2] step through lg_train_gemm (tools only; time it with
rocprofv3 --kernel-trace --stats).  Shapes (R = 32 x 4096 rows): forward linears (0, 1), input
gradients (0, 0), weight gradients (1, 0; split-K)."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import lgamd  # noqa: E402,F401
from lightglue_amd import _lib  # noqa: E402

R = int(os.environ.get("KB_ROWS", 131072))
REPS = int(os.environ.get("KB_REPS", 5))
lib = _lib.load()
dev = torch.device("cuda", 0)
st = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
g = torch.Generator(device=dev).manual_seed(0)


def run(tag, M, N, K, ta, tb):
    A = torch.randn((K, M) if ta else (M, K), device=dev, generator=g)
    B = torch.randn((N, K) if tb else (K, N), device=dev, generator=g)
    C = torch.empty((M, N), device=dev)
    nb = ctypes.c_size_t()
    _lib.check(lib.lg_train_gemm_workspace_bytes(M, N, K, 1, ctypes.byref(nb)), "ws")
    ws = torch.empty(max(nb.value, 4), dtype=torch.uint8, device=dev)
    lda = A.shape[1]
    ldb = B.shape[1]
    for _ in range(REPS):
        _lib.check(lib.lg_train_gemm(ctypes.c_void_p(A.data_ptr()), ctypes.c_void_p(B.data_ptr()),
                                     ctypes.c_void_p(C.data_ptr()), lda, ldb, N, 0, 0, 0, M, N, K, 1, 1.0, 0.0, None,
                                     ta, tb, ctypes.c_void_p(ws.data_ptr()), nb.value, st), tag)
    ref = (A.t() if ta else A).double() @ (B.t() if tb else B).double()
    err = float((C.double() - ref).abs().max() / ref.abs().max())
    print(f"{tag}: M={M} N={N} K={K} ta={ta} tb={tb} rel err {err:.1e}", flush=True)


run("fwd_qkv", R, 768, 256, 0, 1)
run("fwd_ffn0", R, 512, 512, 0, 1)
run("fwd_ffn3", R, 256, 512, 0, 1)
run("dgrad_qkv", R, 256, 768, 0, 0)
run("dgrad_ffn0", R, 512, 512, 0, 0)
run("wgrad_qkv", 768, 256, R, 1, 0)
run("wgrad_ffn0", 512, 512, R, 1, 0)
