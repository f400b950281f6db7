#!/usr/bin/env python3
"""Sinkhorn schedule sweep (configs[4]: B=8, N=4096, 50 iterations): pair-group sizes (LG_SK_GROUP)
and streams (LG_SK_STREAMS) against the streaming schedule, one JSON line per setting.  The
library reads those knobs once per process, so every setting runs in a child process (the parent
never touches the GPU).  LIGHTGLUE_MI355X_LIB selects the library build (A/B of build knobs)."""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child():
    import torch

    sys.path.insert(0, ROOT)
    import lgamd  # noqa: F401
    from lightglue_amd import log_optimal_transport

    B, N, IT = int(os.environ.get("B", 8)), int(os.environ.get("N", 4096)), 50
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(5)
    scores = torch.randn((B, N, N), generator=g, device=dev) * 2.0
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
    print(json.dumps({"group": int(os.environ.get("LG_SK_GROUP", 0)), "streams": int(os.environ.get("LG_SK_STREAMS", 1)),
                      "resident_mb": float(os.environ.get("LG_SK_RESIDENT_MB", 0)),
                      "lib": os.path.basename(os.environ.get("LIGHTGLUE_MI355X_LIB", "default")),
                      "ms": round(s * 1e3, 3), "GBps": round(by / s / 1e9, 1),
                      "Z_sum": float(Z.double().sum()), "Z_absmax": float(Z.abs().max())}), flush=True)


if __name__ == "__main__":
    if os.environ.get("SK_CHILD"):
        child()
        sys.exit(0)
    rc = 0
    for setting in os.environ.get("SK_SETTINGS", "0:1,1:2,2:2,3:3,4:2").split(","):
        f = setting.split(":")  # group:streams[:resident_mb]
        env = dict(os.environ, SK_CHILD="1", LG_SK_GROUP=f[0], LG_SK_STREAMS=f[1], LG_SK_RESIDENT_MB=f[2] if len(f) > 2 else "0")
        r = subprocess.run([sys.executable, os.path.abspath(__file__)], env=env, timeout=300)
        rc = rc or r.returncode
        if r.returncode != 0:
            break
    sys.exit(rc)
