#!/usr/bin/env python3
"""One timed TRAINING step on one MI355X (reference gluefactory/train.py:430-470: forward in
training mode, model.loss, torch.mean(total), backward, optimizer step) -- LightGlue (default) or
SuperGlue (``--model superglue``: the 18-layer GNN, 50 Sinkhorn iterations, SuperGlue.loss).

Default shape = BASELINE configs[2] (N = 2048 keypoints, 9 layers, 32 pairs per step), synthetic
inputs (SURVEY §8d recipe) and a seeded one-to-one ground truth, random-init weights of the
reference architecture.  Prints one JSON line: ms per step (forward / loss / backward / optimizer
split from HIP events), pairs/s, peak memory, and the algorithmic TFLOP/s of the step.

    python tools/bench_train.py [--model lightglue|superglue] [--batch 32] [--npts 2048] [--steps 5] [--warmup 2]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import lgamd  # noqa: E402,F401


def step_flops(B, N, L, d=256):
    """Algorithmic flops of one training step (fwd + bwd): linear layers 3x their forward flops
    (y, dx, dW); attention 4 N^2 d forward + 10 N^2 d backward per (pair, image) for self and
    4 + 10 per direction for cross (S recomputed per direction, as the forward); heads: the loss
    evaluates L assignment heads (final_proj + similarity forward, similarity recompute + two
    backward products)."""
    lin = L * 76 * N * d * d  # per pair, forward (76 N d^2 per layer)
    att = L * (2 * 14 * N * N * d + 2 * 14 * N * N * d) / 2  # self (2 images) + cross (2 dirs): 14 N^2 d each
    head = L * (2 * 2 * N * d * d + 2 * N * N * d)  # final_proj x2 images + sim
    fwd_head = head
    bwd_head = L * (2 * N * N * d + 2 * 2 * N * N * d + 3 * 2 * N * d * d)
    return B * (3 * lin + att + fwd_head + bwd_head)


def sg_step_flops(B, N, L=18, T=50, d=256):
    """SuperGlue: per layer and image set q/k/v/merge (4 N d^2 x 2) + mlp (2 N (2d)^2 + 2 N 2d d)
    forward, 3x for fwd + bwd; attention 4 N^2 d fwd + 10 N^2 d bwd per image; final_proj + cost;
    the Sinkhorn's exp work is not counted (memory-bound)."""
    lin = L * 2 * (2 * 4 * N * d * d + 2 * N * 4 * d * d + 2 * N * 2 * d * d)
    att = L * 2 * 14 * N * N * d
    head = 3 * (2 * 2 * N * d * d + 2 * N * N * d)
    return B * (3 * lin + att + head)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", choices=["lightglue", "superglue"], default="lightglue")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--npts", type=int, default=2048)
    ap.add_argument("--layers", type=int, default=9)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--no-optim", action="store_true")
    a = ap.parse_args()
    from lightglue_amd import LightGlue
    from lightglue_amd.weights import synthetic_pair, synthetic_state_dict

    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    from make_superglue_golden import ground_truth

    dev = torch.device("cuda", 0)
    B, N, L = a.batch, a.npts, a.layers
    if a.model == "lightglue":
        conf = {"filter_threshold": 0.1, "n_layers": L}
        model = LightGlue(conf).to(dev)
        model.load_state_dict({k: torch.from_numpy(v) for k, v in synthetic_state_dict(conf, seed=0).items()})
    else:
        from lightglue_amd import SuperGlue
        from lightglue_amd.sg_weights import superglue_state_dict, synthetic_scores

        model = SuperGlue({}).to(dev)
        full = model.state_dict()
        full.update({k: torch.from_numpy(v) for k, v in superglue_state_dict({}, seed=0).items()})
        model.load_state_dict(full)
    model.train()
    pair = synthetic_pair(B=B, M=N, seed=1)
    if a.model == "superglue":
        pair["keypoint_scores0"] = synthetic_scores(B, N, seed=2)
        pair["keypoint_scores1"] = synthetic_scores(B, N, seed=3)
    gt = ground_truth(B, N, N, 7)
    data = {k: torch.from_numpy(v).to(dev) for k, v in pair.items() if not k.startswith("image_size")}
    data["view0"] = {"image_size": torch.from_numpy(pair["image_size0"]).to(dev)}
    data["view1"] = {"image_size": torch.from_numpy(pair["image_size1"]).to(dev)}
    data.update({k: torch.from_numpy(v).to(dev) for k, v in gt.items()})
    opt = torch.optim.Adam(model.parameters(), lr=1e-4)
    ev = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731

    def one_step(times=None):
        e = [ev() for _ in range(5)]
        e[0].record()
        opt.zero_grad(set_to_none=True)
        pred = model(data)
        e[1].record()
        losses = model.loss(pred, data)
        losses = losses[0] if isinstance(losses, tuple) else losses
        loss = torch.mean(losses["total"])
        e[2].record()
        loss.backward()
        e[3].record()
        if not a.no_optim:
            opt.step()
            model.reload_weights()  # the optimizer writes through p.data-free in-place ops; re-upload for the head forwards
        e[4].record()
        if times is not None:
            times.append(e)
        return loss

    for _ in range(a.warmup):
        one_step()
    torch.cuda.synchronize()
    torch.cuda.reset_peak_memory_stats(dev)
    times = []
    t0, t1 = ev(), ev()
    t0.record()
    for _ in range(a.steps):
        loss = one_step(times)
    t1.record()
    torch.cuda.synchronize()
    ms = t0.elapsed_time(t1) / a.steps
    split = np.mean([[e[i].elapsed_time(e[i + 1]) for i in range(4)] for e in times], axis=0)
    fl = step_flops(B, N, L) if a.model == "lightglue" else sg_step_flops(B, N)
    out = {
        "metric": f"training step (forward + {'LightGlue' if a.model == 'lightglue' else 'SuperGlue'}.loss + backward + Adam)",
        "ms_per_step": round(ms, 2),
        "pairs_per_s": round(B * 1000.0 / ms, 2),
        "split_ms": {"forward": round(float(split[0]), 2), "loss": round(float(split[1]), 2),
                     "backward": round(float(split[2]), 2), "optimizer": round(float(split[3]), 2)},
        "algorithmic_tflops": round(fl / (ms * 1e-3) / 1e12, 1),
        "peak_mem_gb": round(torch.cuda.max_memory_allocated(dev) / 2**30, 2),
        "loss": float(loss.detach()),
        "dtype": "f32 (f32-input MFMA)",
        "config": {"workload": (f"configs[2] shape: N={N}, {L} layers, {B} pairs per step" if a.model == "lightglue"
                                else f"SuperGlue outdoor architecture (18 GNN layers, 50 Sinkhorn iterations), N={N}, "
                                     f"{B} pairs per step"), "data": "synthetic"},
    }
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
