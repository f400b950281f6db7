#!/usr/bin/env python3
"""Per-GPU measurements of the BASELINE.json configs other than the headline one (bench.py).

    python tools/bench_configs.py [--only 1,3,4,sp,sg,e2e] [--reps R]

One JSON line per config:
  configs[1]  N=1024, 9 layers, B=1 (latency-shaped: one pair per forward)
  configs[3]  N=2048, width/depth pruning on (0.95 / 0.95) with weights that really prune and stop
              early, 32 pairs per forward (each pair prunes / stops on its own; the reference asserts
              B == 1, lightglue.py:528,533); MegaDepth-like 1600x1200 keypoints; also the same
              batch unpruned and one pair per forward
  sp          SuperPoint (§8f row 3): 16 gray 640x480 images per forward, top-2048 keypoints
  e2e         configs[2] end to end: SuperPoint on both views + LightGlue, 32 pairs per forward
  configs[4]  N=4096, 8 pairs per GPU (64 over 8 GPUs): the LightGlue forward at N=4096 and the
              SuperGlue log-domain Sinkhorn (superglue.py:173-201, 50 iterations) on the
              [8, 4096, 4096] similarity, each timed on its own; Sinkhorn against the HBM roofline
              (algorithmic bytes = one read of the B*M*N fp32 scores per iteration + the Z write)
Synthetic inputs and random-init weights as in bench.py; inputs resident in HBM.
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import lgamd  # noqa: E402,F401
from bench import HBM_PEAK_GBS, gpu_pairs  # noqa: E402
from lightglue_amd import LightGlue, log_optimal_transport  # noqa: E402
from lightglue_amd.weights import synthetic_state_dict  # noqa: E402


def model_for(conf, device):
    m = LightGlue(conf).eval().to(device)
    sd = synthetic_state_dict({"filter_threshold": 0.1}, seed=0)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
    return m


def timed(fn, reps, warm=2):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        out = fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps, out


def cfg1(dev, reps):
    m = model_for({"filter_threshold": 0.1}, dev)
    data = gpu_pairs(1, 1024, 256, seed=1, device=dev)
    with torch.no_grad():
        s, pred = timed(lambda: m(data), reps)
        mg = model_for({"filter_threshold": 0.1}, dev).compile()  # HIP-graph replay
        sg, pg = timed(lambda: mg(data), reps)
    assert torch.equal(pg["matches0"], pred["matches0"])
    return {"config": "configs[1]: synthetic N=1024 d=256, 9 layers, batch=1, 1 GPU", "value": round(1 / s, 2),
            "unit": "image-pairs/s", "ms_per_pair": round(1e3 * s, 3),
            "graph_replay_pairs_per_s": round(1 / sg, 2), "graph_replay_ms_per_pair": round(1e3 * sg, 3),
            "matches": int((pred["matches0"] > -1).sum())}


def prune_recipe_model(conf, dev):
    """Weights that really prune and stop (weights.prune_recipe_state_dict, the configs[3] golden's
    recipe: layers 0..4 prune ~10 % of the points, layer 5 fires the early stop)."""
    from lightglue_amd.weights import prune_recipe_state_dict

    m = LightGlue(conf).eval().to(dev)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in prune_recipe_state_dict(conf).items()}, strict=True)
    return m


def cfg3(dev, reps, B=32):
    """configs[3]: N = 2048 with width + depth pruning 0.95, B pairs per forward (every pair prunes
    and stops on its own, device-side counts, one sync per forward), against the same batch
    unpruned and against one pair per forward (the reference's B == 1 regime)."""
    conf = {"filter_threshold": 0.1, "width_confidence": 0.95, "depth_confidence": 0.95}
    m = prune_recipe_model(conf, dev)
    m_full = prune_recipe_model({"filter_threshold": 0.1}, dev)
    data = gpu_pairs(B, 2048, 256, seed=3, device=dev, size=(1600.0, 1200.0))
    with torch.no_grad():
        s, pred = timed(lambda: m(data), reps)
        s_full, _ = timed(lambda: m_full(data), max(1, reps // 2), warm=1)
        ones = [{k: (v[i:i + 1] if torch.is_tensor(v) else {"image_size": v["image_size"][i:i + 1]})
                 for k, v in data.items()} for i in range(8)]
        s1, _ = timed(lambda: [m(d) for d in ones], max(1, reps // 4), warm=1)
    kept = (pred["kept0"].float() / 2048).tolist()
    return {"config": f"configs[3]: N=2048 (1600x1200 keypoints), width+depth pruning 0.95, batch={B} per forward",
            "value": round(B / s, 2), "unit": "image-pairs/s per GPU", "ms_per_pair": round(1e3 * s / B, 3),
            "unpruned_same_batch_pairs_per_s": round(B / s_full, 2),
            "one_pair_per_forward_pairs_per_s": round(8 / s1, 2),
            "layers_executed": sorted({int(x) + 1 for x in pred["stop_layer"].tolist()}),
            "kept_fraction_image0_mean": round(sum(kept) / len(kept), 3)}


def cfg4(dev, reps):
    B, N = 8, 4096
    m = model_for({"filter_threshold": 0.1}, dev)
    data = gpu_pairs(B, N, 256, seed=4, device=dev)
    with torch.no_grad():
        s_fwd, _ = timed(lambda: m(data), max(1, reps // 2), warm=1)
    g = torch.Generator(device=dev).manual_seed(5)
    scores = torch.randn((B, N, N), generator=g, device=dev) * 2.0
    iters = 50
    s_sk, Z = timed(lambda: log_optimal_transport(scores, 1.0, iters), reps)
    # algorithmic bytes: one streamed read of the B*N*N fp32 scores per iteration (both half-steps
    # from the same read) + the final Z write and its scores read
    by = float(iters * B * N * N * 4 + B * (N + 1) * (N + 1) * 4 + B * N * N * 4)
    gbs = by / s_sk / 1e9
    return {"config": "configs[4]: N=4096 d=256, 8 pairs per GPU (batch 64 over 8 GPUs), Sinkhorn 50 iters",
            "forward_pairs_per_s": round(B / s_fwd, 2), "forward_ms": round(1e3 * s_fwd, 3),
            "sinkhorn_ms": round(1e3 * s_sk, 3), "sinkhorn_pairs_per_s": round(B / s_sk, 2),
            "end_to_end_pairs_per_s": round(B / (s_fwd + s_sk), 2),
            "sinkhorn_roofline": {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                  "frac": round(gbs / HBM_PEAK_GBS, 4),
                                  "algorithmic_bytes": by,
                                  "note": "scores 537 MB > 256 MB Infinity Cache; >1 means cache reuse"},
            "Z_finite": bool(torch.isfinite(Z).all())}


def sp_flops(H, W):
    """Algorithmic flops of one SuperPoint dense forward (2 per MAC, superpoint.py:208-235)."""
    f, h, w = 0, H, W
    for i, (ci, co) in enumerate([(1, 64), (64, 64), (64, 64), (64, 64), (64, 128), (128, 128), (128, 128), (128, 128)]):
        f += 2 * h * w * ci * co * 9
        if i in (1, 3, 5):
            h, w = h // 2, w // 2
    return f + 2 * h * w * (2 * 128 * 256 * 9 + 256 * 65 + 256 * 256)


def cfg_sp(dev, reps, B=16, H=480, W=640, k=2048):
    """SuperPoint extractor (§8f row 3): B gray 640x480 images per forward, top-2048 keypoints."""
    from lightglue_amd import SuperPoint
    from lightglue_amd.sp_weights import superpoint_state_dict, synthetic_images

    m = SuperPoint({"max_num_keypoints": k}).eval().to(dev)
    m.load_state_dict({n: torch.from_numpy(v) for n, v in superpoint_state_dict({}, seed=0).items()})
    img = torch.from_numpy(synthetic_images(B, 1, H, W, seed=1)).to(dev)
    with torch.no_grad():
        s, pred = timed(lambda: m({"image": img}), reps)
    fl = sp_flops(H, W) * B
    return {"config": f"SuperPoint {W}x{H} gray, batch={B}, max_num_keypoints={k}", "value": round(B / s, 2),
            "unit": "images/s", "ms_per_image": round(1e3 * s / B, 3), "dense_tflops_wall": round(fl / s / 1e12, 1),
            "keypoints": list(pred["keypoints"].shape)}


def sg_flops(B, M, N, L=18, D=256):
    """Dense flops of a SuperGlue forward (GNN + final_proj + cost; the encoder and Sinkhorn are
    not counted): per layer q/k/v + mlp.0 (merge folded) + mlp.3 on both images, attention
    (QK^T and PV per head)."""
    R = B * (M + N)
    per_layer = 2 * R * D * (3 * D + 2 * D * 2 * D // D + 2 * D) + 2 * 2 * B * (M * N + N * M) * D
    return L * per_layer + 2 * R * D * D + 2 * B * M * N * D


def cfg_sg(dev, reps, B=16, N=1024):
    """SuperGlue (§8f row 4): B pairs of N keypoints, 18 GNN layers, 50 Sinkhorn iterations."""
    from lightglue_amd import SuperGlue
    from lightglue_amd.sg_weights import superglue_state_dict, synthetic_scores
    from lightglue_amd.weights import synthetic_pair

    m = SuperGlue({}).eval().to(dev)
    sd = m.state_dict()
    sd.update({n: torch.from_numpy(v) for n, v in superglue_state_dict({}, seed=0).items()})
    m.load_state_dict(sd)
    p = synthetic_pair(B, N, N, seed=1, width=640, height=480)
    view = {"image_size": torch.tensor([[640.0, 480.0]] * B, device=dev)}
    data = {k: torch.from_numpy(v).to(dev) for k, v in p.items() if not k.startswith("image_size")}
    data.update({"keypoint_scores0": torch.from_numpy(synthetic_scores(B, N, 2)).to(dev),
                 "keypoint_scores1": torch.from_numpy(synthetic_scores(B, N, 3)).to(dev), "view0": view, "view1": view})
    with torch.no_grad():
        s, pred = timed(lambda: m(data), reps)
    fl = sg_flops(B, N, N)
    return {"config": f"SuperGlue N={N}, 18 GNN layers, 50 Sinkhorn iterations, batch={B}", "value": round(B / s, 2),
            "unit": "image-pairs/s", "ms_per_pair": round(1e3 * s / B, 3), "dense_tflops_wall": round(fl / s / 1e12, 1),
            "matches_per_pair": float((pred["matches0"] >= 0).sum()) / B}


def cfg_e2e(dev, reps, B=32, H=480, W=640, k=2048):
    """configs[2] end to end (SuperPoint + LightGlue): B image pairs per forward through
    TwoViewPipeline (two_view_pipeline.py:79-97) -- SuperPoint on each view's B gray 640x480
    images (top-2048, force_num_keypoints so the pairs batch), then the 9-layer LightGlue on the
    B pairs at N = 2048."""
    from lightglue_amd.pipeline import TwoViewPipeline
    from lightglue_amd.sp_weights import superpoint_state_dict, synthetic_images

    conf = {"extractor": {"name": "gluefactory_nonfree.superpoint", "max_num_keypoints": k, "force_num_keypoints": True},
            "matcher": {"name": "matchers.lightglue", "filter_threshold": 0.1}}
    pipe = TwoViewPipeline(conf).eval().to(dev)
    pipe.extractor.load_state_dict({n: torch.from_numpy(v) for n, v in superpoint_state_dict({}, seed=0).items()})
    sd = synthetic_state_dict({"filter_threshold": 0.1}, seed=0)
    pipe.matcher.load_state_dict({n: torch.from_numpy(v) for n, v in sd.items()}, strict=True)
    size = torch.tensor([[float(W), float(H)]] * B, device=dev)
    # both views show the same synthetic images (so the random-weight matcher has something to
    # match; the work is the same for any pair of images)
    img = torch.from_numpy(synthetic_images(B, 1, H, W, seed=1)).to(dev)
    views = [{"image": img, "image_size": size} for _ in range(2)]
    with torch.no_grad():
        s, pred = timed(lambda: pipe({"view0": dict(views[0]), "view1": dict(views[1])}), reps)
    return {"config": f"configs[2] end to end: SuperPoint {W}x{H} (top-{k}) + LightGlue N={k}, 9 layers, "
                      f"batch={B} pairs, 1 GPU", "value": round(B / s, 2), "unit": "image-pairs/s",
            "ms_per_forward": round(1e3 * s, 2), "keypoints0": list(pred["keypoints0"].shape),
            "matches_per_pair": float((pred["matches0"] > -1).sum()) / B}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="1,3,4")
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    fns = {"1": cfg1, "3": cfg3, "4": cfg4, "sp": cfg_sp, "sg": cfg_sg, "e2e": cfg_e2e}
    for k in a.only.split(","):
        print(json.dumps(fns[k](dev, a.reps)), flush=True)


if __name__ == "__main__":
    main()
