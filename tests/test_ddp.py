"""Data-parallel TRAINING semantics on CPU with gloo, world size 2 (the reference's
gluefactory/train.py:307-309: SyncBatchNorm + DistributedDataParallel; cs566-project-lightglue_amd/
ddp.py is the HIP path's counterpart, exercised on the GPU by tools/ddp_check.py).

The per-rank step is the float64 ORACLE training step (test stand-in for the HIP step, which needs a
GPU): each rank takes one pair of a two-pair batch, its loss is the per-rank mean
(train.py:436), SuperGlue's BatchNorms take the global batch's statistics through a differentiable
all-reduce (oracle/superglue_train_ref.py ``sync``), and the parameter gradients are averaged over
the ranks as DDP averages them.  The result must equal ONE world-size-1 step on the concatenated
two-pair batch: every parameter gradient and (SuperGlue) every BatchNorm running statistic.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _sg_case():
    sys.path.insert(0, HERE)
    import lgamd  # noqa: F401
    from lightglue_amd.sg_weights import superglue_state_dict, synthetic_scores
    from lightglue_amd.weights import synthetic_pair
    from sg_golden_util import ground_truth

    conf = {"GNN_layers": ["self", "cross"], "num_sinkhorn_iterations": 8, "keypoint_encoder": [16, 32]}
    sd = superglue_state_dict(conf, seed=21)
    B, M, N = 2, 30, 26
    p = synthetic_pair(B, M, N, seed=22, width=640, height=480)
    data = {"keypoints0": p["keypoints0"], "keypoints1": p["keypoints1"], "descriptors0": p["descriptors0"],
            "descriptors1": p["descriptors1"], "keypoint_scores0": synthetic_scores(B, M, seed=23),
            "keypoint_scores1": synthetic_scores(B, N, seed=24), "image_hw": (480, 640)}
    return conf, sd, data, ground_truth(B, M, N, 25)


def _lg_case():
    sys.path.insert(0, HERE)
    import lgamd  # noqa: F401
    from lightglue_amd.weights import synthetic_pair, synthetic_state_dict
    from sg_golden_util import ground_truth

    conf = {"filter_threshold": 0.1, "n_layers": 2}
    sd = synthetic_state_dict(conf, seed=3)
    pair = synthetic_pair(B=2, M=32, seed=4)
    return conf, sd, pair, ground_truth(2, 32, 32, 5)


def _slice(d, r):
    return {k: (v[r:r + 1] if isinstance(v, np.ndarray) and v.ndim >= 1 and v.shape[0] == 2 else v) for k, v in d.items()}


def _sg_step(conf, sd, data, gt, sync=None):
    from lightglue_amd.sg_weights import merged_conf
    from oracle.superglue_train_ref import running_stats_after_step, sg_train_forward, sg_train_loss

    buf = ("running_mean", "running_var")
    W = {k: (torch.from_numpy(np.asarray(v).copy()).double() if k.endswith(buf)
             else torch.from_numpy(np.asarray(v).copy()).double().requires_grad_())
         for k, v in sd.items() if not k.endswith("num_batches_tracked")}
    feed = {k: (torch.from_numpy(v).double() if isinstance(v, np.ndarray) else v) for k, v in data.items()}
    la, _, calls, _ = sg_train_forward(W, feed, conf, sync=sync)
    loss, _ = sg_train_loss(la, {k: torch.from_numpy(v) for k, v in gt.items()},
                            merged_conf(conf)["loss"]["nll_balancing"])
    loss.backward()
    grads = {k: w.grad.clone() if w.grad is not None else torch.zeros_like(w) for k, w in W.items() if not k.endswith(buf)}
    return grads, running_stats_after_step(W, calls)


def _lg_step(conf, sd, pair, gt):
    from oracle.lightglue_train_ref import train_loss

    W = {k: torch.from_numpy(np.asarray(v)).double().requires_grad_() for k, v in sd.items()}
    data = {k: torch.from_numpy(v).double() for k, v in pair.items()}
    loss, _ = train_loss(W, data, gt, conf, torch.float64)
    loss.backward()
    return {k: w.grad.clone() if w.grad is not None else torch.zeros_like(w) for k, w in W.items()}, {}


def _worker(rank, world, port, model, out_dir):
    sys.path.insert(0, os.path.dirname(HERE))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import torch.distributed.nn.functional as dfn

        torch.set_num_threads(1)
        if model == "superglue":
            conf, sd, data, gt = _sg_case()
            grads, stats = _sg_step(conf, sd, _slice(data, rank), _slice(gt, rank), sync=lambda t: dfn.all_reduce(t))
        else:
            conf, sd, pair, gt = _lg_case()
            grads, stats = _lg_step(conf, sd, _slice(pair, rank), _slice(gt, rank))
        for g in grads.values():  # DDP: average the gradients over the ranks
            dist.all_reduce(g)
            g.div_(world)
        torch.save({"grads": grads, "stats": stats}, os.path.join(out_dir, f"r{rank}.pt"))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("model", ["superglue", "lightglue"])
def test_data_parallel_step_equals_one_step_on_the_concatenated_batch(tmp_path, model):
    sys.path.insert(0, os.path.dirname(HERE))
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), model, str(tmp_path)), nprocs=world, join=True)
    if model == "superglue":
        conf, sd, data, gt = _sg_case()
        ref_g, ref_s = _sg_step(conf, sd, data, gt)
        # the per-rank (unsynchronised) statistics differ: the test would not be vacuous
        _, loc_s = _sg_step(conf, sd, _slice(data, 0), _slice(gt, 0))
        assert any((loc_s[k] - ref_s[k]).abs().max() > 1e-6 for k in ref_s)
    else:
        conf, sd, pair, gt = _lg_case()
        ref_g, ref_s = _lg_step(conf, sd, pair, gt)
    for r in range(world):
        got = torch.load(os.path.join(str(tmp_path), f"r{r}.pt"))
        assert set(got["grads"]) == set(ref_g)
        for k, g in ref_g.items():
            scale = float(g.abs().max()) + 1e-30
            err = float((got["grads"][k] - g).abs().max())
            assert err <= 1e-10 * scale + 1e-14, (r, k, err, scale)
        assert set(got["stats"]) == set(ref_s)
        for k, s in ref_s.items():
            assert float((got["stats"][k] - s).abs().max()) <= 1e-12 * max(float(s.abs().max()), 1.0), (r, k)


def _abort_worker(rank, world, port, out_dir):
    """Rank 1 fails after its first gradient bucket (as a library error mid-backward would); rank 0
    goes on to its second bucket's all-reduce, which rank 1 never issues."""
    import time

    sys.path.insert(0, os.path.dirname(HERE))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import lgamd  # noqa: F401
    from lightglue_amd.ddp import DataParallel

    class Tiny(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.transformers = torch.nn.ModuleList([torch.nn.Linear(4, 4) for _ in range(2)])

    model = Tiny()
    ddp = DataParallel(model)
    names = [n for n, _ in model.named_parameters()]
    params = [p for _, p in model.named_parameters()]
    b = ddp.buckets(names, params, [True] * len(params), 2, False, torch.device("cpu"))
    for g in b.grads:
        g.fill_(rank + 1.0)
    ready = b.callback(lambda f: f)  # the Python callback itself (the library would call it)
    ready(None, 1, None)  # layer 1's bucket: both ranks issue it
    t0 = time.time()
    try:
        if rank == 1:
            ddp.abort(RuntimeError("injected failure"))
        ready(None, 0, None)  # rank 0 only
        b.finish()
        res = "finished"
    except Exception as e:  # noqa: BLE001
        res = f"raised {type(e).__name__}"
    with open(os.path.join(out_dir, f"abort{rank}.txt"), "w") as f:
        f.write(f"{res} {time.time() - t0:.1f}")
    if dist.is_initialized():
        dist.destroy_process_group()


def test_data_parallel_rank_failure_fails_the_peers_instead_of_hanging(tmp_path):
    """ddp.DataParallel.abort: a failing rank drains what it issued and destroys the
    process group, so a peer blocked in a collective the failed rank never issues raises."""
    import time

    ctx = mp.spawn(_abort_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=False)
    deadline = time.time() + 120
    while not ctx.join(timeout=1):
        if time.time() > deadline:
            for p in ctx.processes:
                p.kill()
            pytest.fail("a rank hung after its peer failed")
    r0 = open(os.path.join(str(tmp_path), "abort0.txt")).read()
    print("rank 0:", r0)
    r1 = open(os.path.join(str(tmp_path), "abort1.txt")).read()
    assert r1.startswith("raised RuntimeError"), r1
    assert r0.startswith("raised"), r0
    assert float(r0.split()[-1]) < 60, r0  # promptly: the closed group, not a collective timeout
