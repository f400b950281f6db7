"""Pair-batch sharding across GPUs (one process per GPU, torch.distributed over RCCL/xGMI).

SURVEY §8(e): image pairs are independent, so a batch of B pairs is split across ranks with no
collective on the data path; the only exchange is the final gather of fixed-size match results
(``matches0/1`` int64, ``matching_scores0/1`` fp32) so that every rank — or rank 0 for export —
holds the whole batch.

* :func:`match_static`  — contiguous B/world slices, one ``all_gather_into_tensor`` of the packed
  results (configs[2]/[4]: uniform per-pair cost).
* :func:`match_dynamic` — pruning makes per-pair cost data dependent (configs[3]): ranks pull
  CHUNKS of pair indices (guided self-scheduling) from an atomic counter in the process group's
  c10d store (``store.add``) and match each chunk in one batched forward -- the reference asserts
  B == 1 when pruning (lightglue.py:528,533); the HIP forward prunes and stops every pair of a batch
  on its own -- then one ``all_reduce(MAX)`` merges the outputs (each pair is written by exactly one
  rank; the rest of the buffer holds -2 / -inf).

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


_dynamic_calls = 0


def guided_chunk(remaining, world, chunk, min_chunk=1):
    """Guided self-scheduling: a rank takes ceil(remaining / world) pairs, capped at ``chunk`` (the
    per-forward batch that maximises pruned pairs/s) and floored at ``min_chunk``.  Early pulls are
    full chunks (batched pruning runs at ~4.8x the pairs/s of one pair per forward,
    profiles/r02/configs.jsonl); near the end of the queue the chunks shrink so the ranks finish
    together when per-pair cost varies."""
    return max(min_chunk, min(chunk, -(-remaining // max(world, 1))))


def match_dynamic(matcher, data, group=None, store=None, key="lightglue_amd/next_pair", chunk=32, min_chunk=1):
    """Work-queue sharding in chunks of pairs: each rank pulls a contiguous chunk of pair indices
    from an atomic counter in the process group's c10d store (``store.add``), matches it in ONE
    batched forward (pruning / early stop are per pair inside the batch), and repeats until the
    batch is exhausted; one ``all_reduce(MAX)`` then merges the outputs (each pair is written by
    exactly one rank; the rest of the buffer holds -2 / -inf).  Chunk sizes follow
    :func:`guided_chunk`.  Without an initialised process group the same loop runs on a local
    counter (world size 1).  Returns (results, [(start, stop) chunks this rank matched])."""
    global _dynamic_calls
    B, M = data["keypoints0"].shape[:2]
    N = data["keypoints1"].shape[1]
    device = data["keypoints0"].device
    distributed = dist.is_available() and dist.is_initialized()
    world = dist.get_world_size(group) if distributed else 1
    # a fresh counter per call: every rank makes the same sequence of calls, so the key needs no
    # reset and no barrier (TCPStore.add creates a missing key at 0)
    _dynamic_calls += 1
    ckey = f"{key}/{_dynamic_calls}"
    if distributed and store is None:
        store = dist.distributed_c10d._get_default_store()
    local = [0]

    def pull(n):  # atomic fetch-and-add; returns the counter value before the add
        if not distributed:
            local[0] += n
            return local[0] - n
        return store.add(ckey, n) - n

    buf = torch.full((B, 2 * M + 2 * N), -2.0, dtype=torch.float64, device=device)
    buf[:, M + N :] = float("-inf")
    done = []
    while True:
        seen = pull(0)
        if seen >= B:
            break
        c = guided_chunk(B - seen, world, chunk, min_chunk)
        a = pull(c)
        if a >= B:
            break
        b = min(B, a + c)
        with torch.no_grad():
            pred = matcher(_slice(data, a, b))
        buf[a:b] = _pack(pred, M, N, b - a, device)
        done.append((a, b))
    if distributed:
        dist.all_reduce(buf, op=dist.ReduceOp.MAX, group=group)
    return _unpack(buf, M, N), done
