#!/usr/bin/env python3
"""Sinkhorn schedule sweep (configs[4]: B=8, N=4096, 50 iterations): pair-group sizes (LG_SK_GROUP)
against the streaming schedule; one JSON line per setting, and Z compared with the first setting."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import lgamd  # noqa: E402,F401
from lightglue_amd import log_optimal_transport  # noqa: E402

B, N, IT = int(os.environ.get("B", 8)), int(os.environ.get("N", 4096)), 50
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(5)
scores = torch.randn((B, N, N), generator=g, device=dev) * 2.0
ref = None
for setting in os.environ.get("SK_SETTINGS", "0:1,1:1,1:2,1:3,2:2,2:1,4:2").split(","):
    grp, nstreams = setting.split(":")
    os.environ["LG_SK_GROUP"] = grp
    os.environ["LG_SK_STREAMS"] = nstreams
    for _ in range(2):
        Z = log_optimal_transport(scores, 1.0, IT)
    torch.cuda.synchronize()
    reps = 10
    t0 = time.perf_counter()
    for _ in range(reps):
        Z = log_optimal_transport(scores, 1.0, IT)
    torch.cuda.synchronize()
    s = (time.perf_counter() - t0) / reps
    by = float(IT * B * N * N * 4 + B * (N + 1) * (N + 1) * 4 + B * N * N * 4)
    if ref is None:
        ref = Z.clone()
    print(json.dumps({"group": int(grp), "streams": int(nstreams), "ms": round(s * 1e3, 3), "GBps": round(by / s / 1e9, 1),
                      "max_abs_diff_vs_first": float((Z - ref).abs().max())}), flush=True)
