"""Pair-batch sharding across GPUs (one process per GPU, torch.distributed over RCCL/xGMI).

SURVEY §8(e): image pairs are independent, so a batch of B pairs is split across ranks with no
collective on the data path; the only exchange is the final gather of fixed-size match results
(``matches0/1`` int64, ``matching_scores0/1`` fp32) so that every rank — or rank 0 for export —
holds the whole batch.

* :func:`match_static`  — contiguous B/world slices, one ``all_gather_into_tensor`` of the packed
  results (configs[2]/[4]: uniform per-pair cost).
* :func:`match_dynamic` — pruning makes per-pair cost data dependent (configs[3], B == 1 per
  launch per reference semantics, lightglue.py:528,533): ranks pull pair indices from an atomic
  counter in the process group's c10d store (``store.add``), then one ``all_reduce(MAX)`` merges
  the outputs (each pair is written by exactly one rank; the rest of the buffer holds -2 / -inf).

``matcher`` is any callable with the ``LightGlue.forward`` contract; in production it is
``lightglue_amd.LightGlue`` on this rank's GPU (the gather then runs on RCCL).  The CPU tests
drive the same code with gloo and a CPU stand-in matcher.
"""
import torch
import torch.distributed as dist

RESULT_KEYS = ("matches0", "matches1", "matching_scores0", "matching_scores1")


def shard_range(B, world, rank):
    """Contiguous [start, stop) of pair indices owned by ``rank`` (sizes differ by at most 1)."""
    base, extra = divmod(B, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def _slice(data, a, b):
    out = {}
    for k, v in data.items():
        if isinstance(v, dict):
            out[k] = _slice(v, a, b)
        elif isinstance(v, torch.Tensor) and v.dim() > 0:
            out[k] = v[a:b]
        else:
            out[k] = v
    return out


def _pack(pred, M, N, rows, device):
    """[rows, 2M+2N] float64 rows: matches as exact small integers, scores widened."""
    buf = torch.empty((rows, 2 * M + 2 * N), dtype=torch.float64, device=device)
    buf[:, :M] = pred["matches0"].to(torch.float64)
    buf[:, M : M + N] = pred["matches1"].to(torch.float64)
    buf[:, M + N : 2 * M + N] = pred["matching_scores0"].to(torch.float64)
    buf[:, 2 * M + N :] = pred["matching_scores1"].to(torch.float64)
    return buf


def _unpack(buf, M, N):
    return {
        "matches0": buf[:, :M].to(torch.int64),
        "matches1": buf[:, M : M + N].to(torch.int64),
        "matching_scores0": buf[:, M + N : 2 * M + N].to(torch.float32),
        "matching_scores1": buf[:, 2 * M + N :].to(torch.float32),
    }


def match_static(matcher, data, group=None):
    """Run this rank's contiguous share of the pair batch, then all-gather the results."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    B, M = data["keypoints0"].shape[:2]
    N = data["keypoints1"].shape[1]
    a, b = shard_range(B, world, rank)
    per = -(-B // world)  # padded rows per rank so the all-gather is fixed-size
    device = data["keypoints0"].device
    local = torch.full((per, 2 * M + 2 * N), -2.0, dtype=torch.float64, device=device)
    if b > a:
        with torch.no_grad():
            pred = matcher(_slice(data, a, b))
        local[: b - a] = _pack(pred, M, N, b - a, device)
    out = torch.empty((world * per, 2 * M + 2 * N), dtype=torch.float64, device=device)
    dist.all_gather_into_tensor(out, local, group=group)
    rows = torch.cat([out[r * per : r * per + (shard_range(B, world, r)[1] - shard_range(B, world, r)[0])] for r in range(world)])
    return _unpack(rows, M, N)


def match_dynamic(matcher, data, group=None, store=None, key="lightglue_amd/next_pair"):
    """Work-queue sharding: each rank pulls single pairs until the batch is exhausted."""
    world_rank = dist.get_rank(group)
    B, M = data["keypoints0"].shape[:2]
    N = data["keypoints1"].shape[1]
    device = data["keypoints0"].device
    if store is None:
        store = dist.distributed_c10d._get_default_store()
    dist.barrier(group)
    if world_rank == 0:
        store.set(key, "0")
    dist.barrier(group)
    buf = torch.full((B, 2 * M + 2 * N), -2.0, dtype=torch.float64, device=device)
    buf[:, M + N :] = float("-inf")
    done = []
    while True:
        i = store.add(key, 1) - 1
        if i >= B:
            break
        with torch.no_grad():
            pred = matcher(_slice(data, i, i + 1))
        buf[i : i + 1] = _pack(pred, M, N, 1, device)
        done.append(i)
    dist.all_reduce(buf, op=dist.ReduceOp.MAX, group=group)
    return _unpack(buf, M, N), done
