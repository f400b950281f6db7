#!/usr/bin/env python3
"""Throughput of the MI355X LightGlue matcher: image-pairs/s at N=2048 keypoints, d=256.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--npts N] [--workload W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

With --gpus N > 1 and no WORLD_SIZE in the environment, bench.py spawns the N ranks itself
(torch.multiprocessing.spawn before the parent touches the GPU, like the reference's
gluefactory/train.py:696); under torch.distributed.run it joins the launcher's process group.

Workload (BASELINE.json configs[2]): SuperPoint-shaped synthetic pairs, N=2048 keypoints per
image, 9 layers, no pruning, B=32 pairs per GPU per step (weak scaling: every rank matches its own
32 pairs; a step also all-gathers the match results to every rank over RCCL when N > 1).
Weights: deterministic random init of the full architecture (no network for checkpoints).
One step = one full LightGlue.forward (positional encoding, 9 x self+cross layers, dual-softmax
assignment with the [B,N+1,N+1] log_assignment written, mutual filter).

Other BASELINE.json configs through the same multi-rank launch (--workload; the default line above
is unchanged):
  configs3  N=2048, width + depth pruning 0.95 (weights that prune ~10 % per layer and stop after
            layer 6; MegaDepth-like 1600x1200 keypoints), 64 pairs per GPU per step pulled from a
            shared queue in guided chunks of <= 32 pairs, each chunk one batched-pruning forward
            (parallel.match_dynamic; per-pair cost varies)
  configs4  N=4096, 8 pairs per GPU per step (64 over 8 GPUs), static shards (parallel.match_static):
            LightGlue forward -> its final similarity -> log-domain Sinkhorn (superglue.py:173-201,
            50 iterations, dustbin score 1.0) -> mutual filter (superglue.py:288-298, threshold 0.2)

Training steps (reference gluefactory/train.py:430-470) through the same launch:
  train     LightGlue in training mode on the configs[2] shape (N=2048, 9 layers, 32 pairs per GPU):
            forward, LightGlue.loss, torch.mean(total), backward, gradient all-reduce (RCCL, one
            flat bucket, N > 1), Adam -- the hand-written HIP backward
  train_sg  the same step for SuperGlue (outdoor architecture: 18 GNN layers, 50 Sinkhorn
            iterations)
  (seeded one-to-one ground truth from the synthetic pairs' own correspondence; their roofline
  object is the whole step's algorithmic flops against the f32 MFMA peak, and their CPU baseline
  the oracle's training step on one pair)

Prints ONE JSON line on rank 0 with the metric, the attention kernel's roofline (in-library HIP
events around every attention launch in the timed region; algorithmic flops per launch) and the
CPU oracle's throughput on this host (rank 0, N=1 only, bounded sample).
"""
import argparse
import json
import os
import socket
import sys
import time

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
import lgamd  # noqa: E402,F401
from lightglue_amd import parallel  # noqa: E402
from lightglue_amd.weights import synthetic_state_dict  # noqa: E402

FP32_MFMA_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: v_mfma_f32_32x32x2_f32 dense peak
BF16X6_PEAK_TFLOPS = 2500.0 / 6  # bf16 dense MFMA peak / 6 MFMAs per fp32-accurate (bf16x6) product
BF16_MFMA_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: dense bf16 MFMA peak
# The hot kernels compute fp32-accurate products as three fp16 MFMA products (fp16x3, the default)
# or six bf16 ones (bf16x6, the guarded fallback), so their fp32-equivalent matrix
# peak is the fp16/bf16 dense peak / 3 (or / 6).
PEAKS = {
    "fp16x3": (BF16_MFMA_PEAK_TFLOPS / 3.0, "lg::attention_h3g_kernel",
               "fp32-equivalent: fp16 dense 2500 TF/s / 3 fp16 products per fp32 product (fp32 MFMA peak is 157.3)"),
    "bf16x6": (BF16_MFMA_PEAK_TFLOPS / 6.0, "lg::attention_x6_kernel",
               "fp32-equivalent: bf16 dense 2500 TF/s / 6 bf16 products per fp32 product (fp32 MFMA peak is 157.3)"),
}
HBM_PEAK_GBS = 8000.0
# The fp16x3 MFMA rate this chip sustains under load on random operands, measured: a GEMM k-loop
# with no k-tile copies at all (operands re-read from LDS) runs at 434-470 TF/s fp32-equivalent
# (1.30-1.41 PF of raw fp16 MFMA work; profiles/r02/kbench_gemm_kloop_probes.txt, DIAG 2) -- the
# clock the chip holds on random data (MI355X_MICROARCH.md, DVFS give-back) caps it well below the
# 2.5 PF spec.  Reported beside the spec-sheet fraction as the achievable denominator.
FP16X3_MEASURED_CEILING_TFLOPS = 470.0
TRAFFIC_JSON = os.path.join(ROOT, "profiles", "traffic.json")


def measured_traffic(kernel_prefix):
    """HBM bytes per launch of a kernel from the committed rocprofv3 PMC passes (tools/profile.sh:
    separate FETCH_SIZE and WRITE_SIZE runs of this bench; FETCH_SIZE doubled per the gfx950
    correction in MI355X_MICROARCH.md §HBM).  None if no profile is committed."""
    try:
        with open(TRAFFIC_JSON) as f:
            t = json.load(f)
    except (OSError, ValueError):
        return None, None
    for name, v in t.get("kernels", {}).items():
        if name.startswith(kernel_prefix):
            return v.get("hbm_bytes_per_launch"), t.get("source")
    return None, None


def gpu_pairs(B, N, dim, seed, device, size=(640.0, 640.0)):
    g = torch.Generator(device=device).manual_seed(seed)
    wh = torch.tensor(size, device=device)
    k0 = torch.rand((B, N, 2), generator=g, device=device) * wh
    d0 = torch.randn((B, N, dim), generator=g, device=device)
    d0 = d0 / d0.norm(dim=-1, keepdim=True)
    perm = torch.argsort(torch.rand((B, N), generator=g, device=device), dim=1)
    k1 = (torch.gather(k0, 1, perm[..., None].expand(-1, -1, 2)) + torch.randn((B, N, 2), generator=g, device=device)).clamp(0, 639.9)
    d1 = torch.gather(d0, 1, perm[..., None].expand(-1, -1, dim)) + 0.05 * torch.randn((B, N, dim), generator=g, device=device)
    d1 = d1 / d1.norm(dim=-1, keepdim=True)
    isz = wh[None].expand(B, 2).contiguous()
    return {
        "keypoints0": k0, "keypoints1": k1, "descriptors0": d0, "descriptors1": d1,
        "view0": {"image_size": isz}, "view1": {"image_size": isz},
    }


def attention_flops_per_pair(N, d=256, L=9):
    return L * 14 * N * N * d  # SURVEY §8d attention term (self 8, cross 6 N^2 d per layer)


def total_flops_per_pair(N, d=256, L=9):
    return L * (76 * N * d * d + 14 * N * N * d) + 4 * N * d * d + 2 * N * N * d


def cpu_threads():
    """Host cores this process may use: the launcher's OMP_NUM_THREADS share when set (16 on the
    GPU box, whose os.cpu_count() reports the whole machine), else the affinity mask."""
    env = os.environ.get("OMP_NUM_THREADS")
    return int(env) if env and env.isdigit() and int(env) > 0 else len(os.sched_getaffinity(0))


def cpu_baseline(npts, budget_s):
    """The CPU oracle (torch-CPU restatement of the reference forward) on this host's cores, with
    the reference's benchmark() protocol (gluefactory/utils/benchmark.py:7-33): 10 warm-up
    forwards, then timed forwards (at most r = 100, bounded by `budget_s`), mean and std."""
    import oracle
    from lightglue_amd.weights import synthetic_pair

    torch.set_num_threads(cpu_threads())
    conf = {"filter_threshold": 0.1}
    sd = synthetic_state_dict(conf, seed=0)
    data = synthetic_pair(B=1, M=npts, seed=1)
    with torch.no_grad():
        for _ in range(10):  # benchmark.py:13-14
            oracle.lightglue_forward(sd, data, conf)
        times, t_start = [], time.perf_counter()
        while len(times) < 100 and (time.perf_counter() - t_start) < budget_s:
            t0 = time.perf_counter()
            oracle.lightglue_forward(sd, data, conf)
            times.append((time.perf_counter() - t0) * 1e3)
    t = np.array(times)
    return {
        "value": 1000.0 / t.mean(),
        "unit": "image-pairs/s",
        "cores": torch.get_num_threads(),
        "kind": "port",
        "mean_ms": round(float(t.mean()), 2),
        "std_ms": round(float(t.std()), 2),
        "sample": f"benchmark() protocol: 10 warm-ups + {len(t)} timed forwards of 1 pair x N={npts} "
                  f"(B=1, 9 layers, fp32), torch-CPU oracle (oracle/lightglue_ref.py), "
                  f"{torch.get_num_threads()} threads",
    }


class _CpuStandIn:
    """--selftest-cpu: a stand-in matcher with the forward() contract (no GPU, no compute) so the
    launch / sharding / gather / timing logic of this script runs on CPU with gloo."""

    last_precision_used = "none"

    def __call__(self, data):
        b, m = data["keypoints0"].shape[:2]
        n = data["keypoints1"].shape[1]
        return {
            "matches0": torch.full((b, m), -1, dtype=torch.int64),
            "matches1": torch.full((b, n), -1, dtype=torch.int64),
            "matching_scores0": torch.zeros((b, m)),
            "matching_scores1": torch.zeros((b, n)),
        }


def cpu_pairs(B, N, dim, seed):
    g = torch.Generator().manual_seed(seed)
    k = torch.rand((B, N, 2), generator=g) * 640
    d = torch.nn.functional.normalize(torch.randn((B, N, dim), generator=g), dim=-1)
    isz = torch.full((B, 2), 640.0)
    return {"keypoints0": k, "keypoints1": k.clone(), "descriptors0": d, "descriptors1": d.clone(),
            "view0": {"image_size": isz}, "view1": {"image_size": isz}}


# workload -> (pairs per GPU per step, keypoints, description)
WORKLOADS = {
    "configs2": (32, 2048, "configs[2]: SuperPoint+LightGlue N=2048, 9 layers, no pruning, batch=32 per GPU"),
    "configs3": (64, 2048, "configs[3]: MegaDepth-like N=2048 (1600x1200), adaptive depth/width pruning 0.95, "
                           "64 pairs per GPU from a shared queue in guided chunks of <= 32"),
    "configs4": (8, 4096, "configs[4]: N=4096 d=256, Sinkhorn assignment (50 iterations), 8 pairs per GPU "
                          "(batch 64 over 8 GPUs)"),
}
WORKLOADS["train"] = (32, 2048, "training step, configs[2] shape: LightGlue N=2048, 9 layers, 32 pairs per GPU "
                               "(forward + LightGlue.loss + backward + Adam)")
WORKLOADS["train_sg"] = (32, 2048, "training step: SuperGlue outdoor architecture (18 GNN layers, 50 Sinkhorn "
                                   "iterations), N=2048, 32 pairs per GPU (forward + SuperGlue.loss + backward + Adam)")
SINKHORN_ITERS, SINKHORN_ALPHA, SINKHORN_THRESHOLD = 50, 1.0, 0.2  # superglue.py:214-215, bin_score init 1.0


def train_flops_per_pair(N, sg=False, d=256, L=9):
    """Algorithmic flops of one training step per pair (forward + backward): linear layers 3x their
    forward flops (y, dx, dW), attention 4 N^2 d forward + 10 N^2 d backward per softmax direction,
    the assignment heads' products (LightGlue: every layer's head is evaluated by the loss)."""
    if sg:
        lin = 18 * 2 * (8 * N * d * d + 8 * N * d * d + 4 * N * d * d)
        return 3 * lin + 18 * 2 * 14 * N * N * d + 3 * (4 * N * d * d + 2 * N * N * d)
    lin = L * 76 * N * d * d
    # four softmax directions per layer: self-attention on each image + cross-attention both ways
    # (this was 2 directions, under-counting the attention by half)
    att = L * 4 * 14 * N * N * d
    head = L * (4 * N * d * d + 2 * N * N * d)
    bwd_head = L * (6 * N * N * d + 6 * N * d * d)
    return 3 * lin + att + head + bwd_head


def gpu_ground_truth(data, seed):
    """One-to-one ground truth of gpu_pairs' correspondence (image-1 point j is image-0 point
    perm[j], recovered from the keypoints), a third of each side left unmatched."""
    k0, k1 = data["keypoints0"], data["keypoints1"]
    B, M = k0.shape[:2]
    dev = k0.device
    near = torch.cdist(k1, k0).argmin(-1)  # [B, N] -> image-0 index
    g = torch.Generator(device=dev).manual_seed(seed)
    keep = torch.rand((B, k1.shape[1]), generator=g, device=dev) < 0.67
    m1 = torch.where(keep, near, torch.full_like(near, -1))
    m0 = torch.full((B, M), -1, dtype=torch.int64, device=dev)
    bi, ji = torch.nonzero(m1 > -1, as_tuple=True)
    m0[bi, m1[bi, ji]] = ji
    m1 = torch.full_like(m1, -1)  # keep the pairs one-to-one after collisions
    bi, ii = torch.nonzero(m0 > -1, as_tuple=True)
    m1[bi, m0[bi, ii]] = ii
    a = torch.zeros((B, M, k1.shape[1]), dtype=torch.bool, device=dev)
    a[bi, ii, m0[bi, ii]] = True
    return {"gt_matches0": m0, "gt_matches1": m1, "gt_assignment": a}


def cpu_baseline_train(npts, budget_s, sg):
    """The CPU oracle's training step (torch-CPU restatement of the reference forward in training
    mode + its loss, differentiated by torch autograd in fp32) on one pair, on this host's cores:
    one warm-up step, then timed steps until `budget_s` (at least one)."""
    from lightglue_amd.weights import synthetic_pair

    torch.set_num_threads(cpu_threads())
    pair = synthetic_pair(B=1, M=npts, seed=1)
    k0, k1 = pair["keypoints0"], pair["keypoints1"]
    d2 = ((k1[0][:, None, :] - k0[0][None, :, :]) ** 2).sum(-1)
    near = d2.argmin(-1)
    m1 = np.where(np.arange(npts) % 3 != 0, near, -1)[None]
    m0 = -np.ones((1, npts), np.int64)
    for j, i in enumerate(m1[0]):
        if i >= 0:
            m0[0, i] = j
    m1 = -np.ones((1, npts), np.int64)
    for i, j in enumerate(m0[0]):
        if j >= 0:
            m1[0, j] = i
    a = np.zeros((1, npts, npts), bool)
    for i, j in enumerate(m0[0]):
        if j >= 0:
            a[0, i, j] = True
    gt = {"gt_matches0": m0, "gt_matches1": m1, "gt_assignment": a}
    if sg:
        from oracle.superglue_train_ref import sg_train_forward, sg_train_loss
        from lightglue_amd.sg_weights import superglue_state_dict, synthetic_scores

        sd = superglue_state_dict({}, seed=0)

        def one():
            W = {k: torch.from_numpy(np.asarray(v).copy()).float().requires_grad_(
                not k.endswith(("running_mean", "running_var"))) for k, v in sd.items()
                 if not k.endswith("num_batches_tracked")}
            data = {"keypoints0": torch.from_numpy(k0), "keypoints1": torch.from_numpy(k1),
                    "descriptors0": torch.from_numpy(pair["descriptors0"]),
                    "descriptors1": torch.from_numpy(pair["descriptors1"]),
                    "keypoint_scores0": synthetic_scores(1, npts, seed=2), "keypoint_scores1": synthetic_scores(1, npts, seed=3),
                    "image_size": pair["image_size0"]}
            la, _, _, _ = sg_train_forward(W, data, {})
            loss, _ = sg_train_loss(la, {k: torch.from_numpy(v) for k, v in gt.items()})
            loss.backward()
        what = "oracle/superglue_train_ref.py (18 GNN layers, 50 Sinkhorn iterations)"
    else:
        from oracle.lightglue_train_ref import train_loss

        conf = {"filter_threshold": 0.1}
        sd = synthetic_state_dict(conf, seed=0)

        def one():
            W = {k: torch.from_numpy(np.asarray(v).copy()).float().requires_grad_() for k, v in sd.items()}
            data = {k: torch.from_numpy(v) for k, v in pair.items()}
            loss, _ = train_loss(W, data, gt, conf, torch.float32)
            loss.backward()
        what = "oracle/lightglue_train_ref.py (9 layers, LightGlue.loss over every layer's head)"
    one()  # warm-up
    times, t_start = [], time.perf_counter()
    while not times or (time.perf_counter() - t_start) < budget_s:
        t0 = time.perf_counter()
        one()
        times.append((time.perf_counter() - t0) * 1e3)
    t = np.array(times)
    return {
        "value": 1000.0 / t.mean(),
        "unit": "image-pairs/s",
        "cores": torch.get_num_threads(),
        "kind": "port",
        "mean_ms": round(float(t.mean()), 2),
        "sample": f"1 warm-up + {len(t)} timed training steps (forward + loss + autograd backward, fp32) of 1 pair "
                  f"x N={npts}, torch-CPU {what}, {torch.get_num_threads()} threads",
    }


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="configs2", choices=sorted(WORKLOADS))
    ap.add_argument("--batch", type=int, default=None, help="pairs per GPU per step (default: the workload's)")
    ap.add_argument("--npts", type=int, default=None, help="keypoints per image (default: the workload's)")
    ap.add_argument("--chunk", type=int, default=32, help="configs3: largest chunk of pairs per forward")
    ap.add_argument("--cpu-budget", type=float, default=15.0, help="seconds of timed CPU-baseline work (0 = skip)")
    ap.add_argument("--precision", default="auto", choices=["auto", "bf16x6"])
    ap.add_argument("--checkpointed", action="store_true",
                    help="--workload train: LightGlue conf checkpointed (layer recompute in the backward)")
    ap.add_argument("--selftest-cpu", action="store_true",
                    help="CPU/gloo rehearsal of the launch and gather logic with a stand-in matcher")
    a = ap.parse_args(argv)
    b, n, _ = WORKLOADS[a.workload]
    a.batch = b if a.batch is None else a.batch
    a.npts = n if a.npts is None else a.npts
    return a


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _spawned(rank, args, port):
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(args.gpus),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    run(args)


def main(argv=None):
    args = parse_args(argv)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # one process per GPU; the parent never touches the GPU (no exec after GPU init)
        mp.spawn(_spawned, nprocs=args.gpus, args=(args, _free_port()), join=True)
        return
    run(args)


def run(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks")
    # LG_BENCH_DIST=1: the process-group path (RCCL all-gather / DataParallel buckets) at one rank
    # too -- how tests/test_gpu_bench_dist.py exercises RCCL on a one-GPU box
    distributed = world > 1 or os.environ.get("LG_BENCH_DIST") == "1"
    selftest = args.selftest_cpu
    if distributed:
        if selftest:
            dist.init_process_group("gloo")
        else:
            os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    B, N = args.batch, args.npts
    wl = args.workload
    if wl in ("train", "train_sg"):
        return run_train(args, world, rank, local, distributed)
    conf = {"filter_threshold": 0.1}
    if wl == "configs3":
        conf.update(width_confidence=0.95, depth_confidence=0.95)
    if wl == "configs4":
        conf["return_similarity"] = True
    size = (1600.0, 1200.0) if wl == "configs3" else (640.0, 640.0)
    if selftest:
        device = torch.device("cpu")
        model = _CpuStandIn()
        data = cpu_pairs(B * world, N, 256, seed=1)
    else:
        from lightglue_amd import LightGlue
        from lightglue_amd.weights import prune_recipe_state_dict

        device = torch.device("cuda", local)
        model = LightGlue({**conf, "precision": args.precision}).eval().to(device)
        sd = prune_recipe_state_dict(conf) if wl == "configs3" else synthetic_state_dict(conf, seed=0)
        model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
        # every rank holds the same global batch (B pairs per GPU) and matches its shard
        data = gpu_pairs(B * world, N, 256, seed=3 if wl == "configs3" else 1, device=device, size=size)

    sk_events = []

    def sinkhorn_matcher(d):
        """configs[4]: the matcher's final similarity through the Sinkhorn head (superglue.py:173-201,
        288-298) instead of the dual softmax."""
        if selftest:
            return model(d)
        from lightglue_amd.assignment import sinkhorn_match

        n = d["keypoints0"].shape[0]
        out, _ = sinkhorn_match(model, d, SINKHORN_ALPHA, SINKHORN_ITERS, SINKHORN_THRESHOLD,
                                on_sinkhorn=lambda e0, e1: sk_events.append((e0, e1, n)))
        return out

    matcher = sinkhorn_matcher if wl == "configs4" else model

    def sync():
        if not selftest:
            torch.cuda.synchronize()

    def step():
        if wl == "configs3":  # shared queue of guided chunks, one batched-pruning forward per chunk
            return parallel.match_dynamic(matcher, data, chunk=args.chunk)[0]
        if distributed:  # this rank's B pairs, then the RCCL all-gather of the match results
            return parallel.match_static(matcher, data)
        with torch.no_grad():
            return matcher(data)

    for _ in range(args.warmup):
        step()
    sync()
    if distributed:
        dist.barrier()
    # timed region: HIP events only around the roofline kernel (the attention launches)
    if not selftest:
        model.profile_enable(True, only=("attention",))
    sync()
    if distributed:
        dist.barrier()
    sk_events.clear()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        pred = step()
    sync()
    if distributed:
        dist.barrier()
    el = time.perf_counter() - t0
    sk_timed = list(sk_events)
    result_kernels, roofline = None, None
    if not selftest:
        att_ms, att_n, att_fl, att_by = model.profile_read("attention")
        # per-family breakdown from a separate, untimed pass with every family evented
        bsteps = min(args.steps, 3)
        model.profile_enable(True)
        for _ in range(bsteps):
            step()
        sync()
        gem_ms, gem_n, gem_fl, _ = model.profile_read("gemm")
        asg_ms, asg_n, _, asg_by = model.profile_read("assign")
        model.profile_enable(False)
        prec = model.last_precision_used
        peak, kname, peak_note = PEAKS[prec]
        if prec == "fp16x3" and os.environ.get("LG_ATTN_KERNEL") == "h3m":
            kname = "lg::attention_h3m_kernel"
        traffic, traffic_src = measured_traffic(kname)
        roofline = {
            "kernel": f"{kname} (flash self/cross attention, {prec} fp32-accurate products)",
            "bound": "mfma",
            "achieved": round(att_fl / (att_ms * 1e-3) / 1e12, 2) if att_ms > 0 else None,
            "peak": round(peak, 1),
            "peak_note": peak_note,
            "unit": "TFLOP/s",
            "frac": round(att_fl / (att_ms * 1e-3) / 1e12 / peak, 4) if att_ms > 0 else None,
            "achievable_peak": FP16X3_MEASURED_CEILING_TFLOPS if prec == "fp16x3" else None,
            "frac_of_achievable": (round(att_fl / (att_ms * 1e-3) / 1e12 / FP16X3_MEASURED_CEILING_TFLOPS, 4)
                                   if att_ms > 0 and prec == "fp16x3" else None),
            "achievable_note": "measured fp16x3 MFMA ceiling under load on random operands (copy-free GEMM k-loop, "
                               "profiles/r02/kbench_gemm_kloop_probes.txt); 'frac' uses the 2.5 PF spec / 3",
            "traffic": traffic,
            "traffic_source": traffic_src,
            "launches": att_n,
            "avg_launch_ms": round(att_ms / max(att_n, 1), 4),
            "algorithmic_flops_per_launch": att_fl / max(att_n, 1),
        }
        if wl == "configs3":
            roofline["flops_note"] = ("pruned forwards: each launch's flops over the kept points of the running pairs "
                                      "(per-pair counts copied at launch time, lg_profile_read)")
        result_kernels = {
            "attention_ms_per_step": round(att_ms / args.steps, 3),
            "breakdown_note": f"gemm/assign from {bsteps} untimed steps with every kernel family evented",
            "gemm_ms_per_step": round(gem_ms / bsteps, 3),
            "gemm_tflops": round(gem_fl / (gem_ms * 1e-3) / 1e12, 2) if gem_ms > 0 else None,
            "assign_ms_per_step": round(asg_ms / bsteps, 3),
            "assign_gbs": round(asg_by / (asg_ms * 1e-3) / 1e9, 1) if asg_ms > 0 else None,
        }
    if distributed:  # max over ranks of the timed region
        t = torch.tensor([el], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())

    if sk_timed:  # configs4: the Sinkhorn kernel against the HBM roofline (one read of the scores per iteration)
        sk_ms = sum(a.elapsed_time(b) for a, b, _ in sk_timed)
        sk_pairs = sum(n for _, _, n in sk_timed)
        by = sk_pairs * (SINKHORN_ITERS * N * N * 4.0 + (N + 1) * (N + 1) * 4.0 + N * N * 4.0)
        result_kernels["sinkhorn_ms_per_step"] = round(sk_ms / args.steps, 3)
        result_kernels["sinkhorn_roofline"] = {
            "bound": "hbm", "achieved": round(by / (sk_ms * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(by / (sk_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "algorithmic_bytes_per_pair": by / sk_pairs,
            "note": "scores read once per iteration + final read and Z write; > 1 means on-die cache reuse"}
    pairs = B * args.steps * world  # every rank matched B pairs per step
    value = pairs / el
    result = {
        "metric": "image-pairs/sec at N=2048 kpts, d=256; HPatches AUC@3px parity",
        "value": round(value, 3),
        "unit": "image-pairs/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1000.0 * el / args.steps, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (SuperPoint-shaped keypoints/descriptors, random-init weights)"
                + (" [CPU self-test: stand-in matcher, no compute]" if selftest else ""),
        "config": {
            "workload": WORKLOADS[wl][2] if (B, N) == WORKLOADS[wl][:2] else f"{wl} shape, N={N}, batch={B} per GPU",
            "npts": N, "descriptor_dim": 256, "n_layers": 9, "pairs_per_gpu_per_step": B,
            "global_batch": B * world,
            "parallelism": f"pair-sharded x{world}" + (
                f" (parallel.match_dynamic: guided chunks <= {args.chunk} from a c10d-store queue, one all_reduce merge)"
                if wl == "configs3" else (" (parallel.match_static: RCCL all-gather of matches)" if distributed else "")),
            "matrix_operands": model.last_precision_used,
        },
        "achieved_tflops_total": round(total_flops_per_pair(N) * pairs / el / 1e12, 2),
        "roofline": roofline,
        "kernels": result_kernels,
        "pairs_timed": pairs,
        "matches_per_pair": float((pred["matches0"] > -1).float().sum(1).mean()),
    }
    if wl == "configs3":
        # pruned forwards do a data-dependent fraction of the 9-layer work: the unpruned-model count
        # would overstate the rate, so it is reported only under its own name
        result["unpruned_equivalent_tflops"] = result.pop("achieved_tflops_total")
        result["unpruned_equivalent_note"] = ("total_flops_per_pair(N) of the UNPRUNED 9-layer forward per matched pair; "
                                              "the kernels' live-row flops are in roofline.achieved")
    if wl == "configs3" and not selftest:
        result["config"]["pruning"] = "width 0.95, depth 0.95 (weights: weights.prune_recipe_state_dict)"
    if rank == 0 and world == 1 and args.cpu_budget > 0 and wl == "configs2":
        result["cpu_baseline"] = cpu_baseline(N, args.cpu_budget)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if distributed:
        dist.destroy_process_group()


def _train_selftest_step(args, world, rank, sg):
    """--selftest-cpu for the training workloads: the float32 ORACLE training step on this rank's
    pairs as the stand-in for the HIP step (no GPU), with the data-parallel semantics of
    ddp.DataParallel: SuperGlue's BatchNorms synchronised over the ranks through a differentiable
    all-reduce (oracle/superglue_train_ref.py ``sync``), gradients averaged over the ranks, Adam."""
    import torch.distributed.nn.functional as dfn
    from lightglue_amd.weights import synthetic_pair

    B, N = args.batch, args.npts
    pair = synthetic_pair(B=B, M=N, seed=1 + rank)
    rng = np.random.Generator(np.random.PCG64(7 + rank))
    m0 = -np.ones((B, N), np.int64)
    m1 = -np.ones((B, N), np.int64)
    a = np.zeros((B, N, N), bool)
    for b in range(B):
        k = 2 * N // 3
        i, j = rng.permutation(N)[:k], rng.permutation(N)[:k]
        m0[b, i], m1[b, j], a[b, i, j] = j, i, True
    gt = {"gt_matches0": m0, "gt_matches1": m1, "gt_assignment": a}
    sync = (lambda t: dfn.all_reduce(t)) if world > 1 else None
    if sg:
        from lightglue_amd.sg_weights import superglue_state_dict, synthetic_scores
        from oracle.superglue_train_ref import sg_train_forward, sg_train_loss

        sd = superglue_state_dict({}, seed=0)
        W = {k: torch.from_numpy(np.asarray(v).copy()).float().requires_grad_(
            not k.endswith(("running_mean", "running_var"))) for k, v in sd.items() if not k.endswith("num_batches_tracked")}
        data = {k: torch.from_numpy(pair[k]) for k in ("keypoints0", "keypoints1", "descriptors0", "descriptors1")}
        data.update(keypoint_scores0=synthetic_scores(B, N, seed=2), keypoint_scores1=synthetic_scores(B, N, seed=3),
                    image_size=pair["image_size0"])

        def loss_fn():
            la, _, _, _ = sg_train_forward(W, data, {}, sync=sync)
            return sg_train_loss(la, {k: torch.from_numpy(v) for k, v in gt.items()})[0]
    else:
        from oracle.lightglue_train_ref import train_loss

        conf = {"filter_threshold": 0.1}
        W = {k: torch.from_numpy(np.asarray(v).copy()).float().requires_grad_()
             for k, v in synthetic_state_dict(conf, seed=0).items()}
        data = {k: torch.from_numpy(v) for k, v in pair.items()}

        def loss_fn():
            return train_loss(W, data, gt, conf, torch.float32)[0]
    params = [w for w in W.values() if w.requires_grad]
    opt = torch.optim.Adam(params, lr=1e-4)

    def step():
        opt.zero_grad(set_to_none=True)
        loss = loss_fn()
        loss.backward()
        if world > 1:  # DDP: average over the ranks (one bucket: the CPU stand-in has no overlap to gain)
            for p in params:
                dist.all_reduce(p.grad)
                p.grad.div_(world)
        opt.step()
        return loss
    return step, torch.device("cpu")


def run_train(args, world, rank, local, distributed):
    """--workload train / train_sg: one data-parallel training step per timed step (train.py:430-470);
    with N > 1 ranks ddp.DataParallel (train.py:307-309: DDP, per-layer gradient buckets all-reduced
    under the backward, and SyncBatchNorm for SuperGlue)."""
    B, N, sg = args.batch, args.npts, args.workload == "train_sg"
    if args.selftest_cpu:
        step, device = _train_selftest_step(args, world, rank, sg)
    else:
        device = torch.device("cuda", local)
        if sg:
            from lightglue_amd import SuperGlue
            from lightglue_amd.sg_weights import superglue_state_dict

            model = SuperGlue({}).to(device)
            full = model.state_dict()
            full.update({k: torch.from_numpy(v) for k, v in superglue_state_dict({}, seed=0).items()})
            model.load_state_dict(full, strict=True)
        else:
            from lightglue_amd import LightGlue

            conf = {"filter_threshold": 0.1}
            model = LightGlue({**conf, "checkpointed": bool(args.checkpointed)}).to(device)
            model.load_state_dict({k: torch.from_numpy(v) for k, v in synthetic_state_dict(conf, seed=0).items()},
                                  strict=True)
        model.train()
        if distributed:
            from lightglue_amd.ddp import DataParallel

            DataParallel(model)
        # this rank's B pairs (its shard of the global batch: every rank draws its own seeded pairs)
        data = gpu_pairs(B, N, 256, seed=1 + rank, device=device)
        data.update(gpu_ground_truth(data, seed=7 + rank))
        if sg:
            g = torch.Generator(device=device).manual_seed(11 + rank)
            data["keypoint_scores0"] = torch.rand((B, N), generator=g, device=device)
            data["keypoint_scores1"] = torch.rand((B, N), generator=g, device=device)
        params = [p for p in model.parameters() if p.requires_grad]
        opt = torch.optim.Adam(params, lr=1e-4)

        def step():
            opt.zero_grad(set_to_none=True)
            pred = model(data)
            losses = model.loss(pred, data)
            losses = losses[0] if isinstance(losses, tuple) else losses
            loss = torch.mean(losses["total"])  # train.py:436
            loss.backward()  # train.py:450 (with DataParallel: gradients averaged over the ranks)
            opt.step()
            return loss

    def cuda_sync():
        if not args.selftest_cpu:
            torch.cuda.synchronize()

    for _ in range(args.warmup):
        step()
    cuda_sync()
    if distributed:
        dist.barrier()
    cuda_sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    cuda_sync()
    if distributed:
        dist.barrier()
    el = time.perf_counter() - t0
    if distributed:
        t = torch.tensor([el], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    pairs = B * args.steps * world
    tf = train_flops_per_pair(N, sg) * pairs / el / 1e12
    result = {
        "metric": f"training image-pairs/sec ({'SuperGlue' if sg else 'LightGlue'} forward + loss + backward + Adam)",
        "value": round(pairs / el, 3),
        "unit": "image-pairs/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1000.0 * el / args.steps, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (SuperPoint-shaped keypoints/descriptors, seeded one-to-one ground truth, random-init weights)",
        "config": {"workload": WORKLOADS[args.workload][2] if (B, N) == WORKLOADS[args.workload][:2]
                   else f"{args.workload} shape, N={N}, batch={B} per GPU",
                   "npts": N, "pairs_per_gpu_per_step": B, "global_batch": B * world,
                   "parallelism": f"data-parallel x{world}" + ((" (gloo, CPU stand-in: oracle step + gradient all-reduce"
                                                           + (" + SyncBatchNorm)" if sg else ")")) if args.selftest_cpu else
                                                          (" (ddp.DataParallel: per-layer gradient buckets all-reduced over RCCL "
                                                           "under the backward" + (" + SyncBatchNorm)" if sg else ")"))
                                                          if distributed else "")
                   + (", checkpointed (layer recompute in the backward)" if args.checkpointed and not sg else "")},
        "roofline": {"kernel": "whole training step (every kernel; f32-input MFMA, bf16x6 attention and input / weight gradients)", "bound": "mfma",
                     "achieved": round(tf, 2), "peak": BF16X6_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": round(tf / BF16X6_PEAK_TFLOPS, 4), "traffic": None,
                     "peak_note": "bf16x6 fp32-equivalent (2.5 PF/s dense bf16 / 6 MFMAs per fp32-accurate product): the "
                                  "route of the attention forward / backward, the input / weight gradients and (LightGlue) "
                                  "the trunk forward linears; SuperGlue's forward linears and the attention backward's dQ "
                                  "run on the f32 MFMA (157.3 TF/s, frac_of_f32_peak)",
                     "frac_of_f32_peak": round(tf / FP32_MFMA_PEAK_TFLOPS, 4),
                     "note": "step-average over all kernels (algorithmic flops of bench.train_flops_per_pair); per-kernel "
                             "rates in DESIGN.md §10c/§10d and profiles/r04, profiles/r05"},
        "loss": float(loss.detach()),
        "peak_mem_gb": None if args.selftest_cpu else round(torch.cuda.max_memory_allocated(device) / 2**30, 2),
    }
    if args.selftest_cpu:
        result["data"] += " [CPU self-test: float32 oracle step stand-in]"
    if rank == 0 and world == 1 and args.cpu_budget > 0 and not args.selftest_cpu:
        result["cpu_baseline"] = cpu_baseline_train(N, args.cpu_budget, sg)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
