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
  on its own -- then the ranks all-gather only the rows they matched, each tagged with its pair
  index (a tiny count exchange first, so the gather is fixed-size), and scatter them into place.

Results travel packed: one int32 row per pair, ``[pair | matches0 (M) | matches1 (N) | scores0 (M) |
scores1 (N)]`` with the fp32 scores bit-cast (8 (M + N) + 4 bytes per pair; matches are < 2^31).

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


def _pack(pred, M, N, rows, first, device):
    """[rows, 1 + 2M + 2N] int32: pair index, matches as int32, fp32 scores bit-cast."""
    buf = torch.empty((rows, 1 + 2 * M + 2 * N), dtype=torch.int32, device=device)
    buf[:, 0] = torch.arange(first, first + rows, dtype=torch.int32, device=device)
    buf[:, 1 : 1 + M] = pred["matches0"].to(torch.int32)
    buf[:, 1 + M : 1 + M + N] = pred["matches1"].to(torch.int32)
    buf[:, 1 + M + N : 1 + 2 * M + N] = pred["matching_scores0"].to(torch.float32).contiguous().view(torch.int32)
    buf[:, 1 + 2 * M + N :] = pred["matching_scores1"].to(torch.float32).contiguous().view(torch.int32)
    return buf


def _unpack(buf, M, N):
    return {
        "matches0": buf[:, 1 : 1 + M].to(torch.int64),
        "matches1": buf[:, 1 + M : 1 + M + N].to(torch.int64),
        "matching_scores0": buf[:, 1 + M + N : 1 + 2 * M + N].contiguous().view(torch.float32),
        "matching_scores1": buf[:, 1 + 2 * M + N :].contiguous().view(torch.float32),
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
    local = torch.zeros((per, 1 + 2 * M + 2 * N), dtype=torch.int32, device=device)
    if b > a:
        with torch.no_grad():
            pred = matcher(_slice(data, a, b))
        local[: b - a] = _pack(pred, M, N, b - a, a, device)
    out = torch.empty((world * per, 1 + 2 * M + 2 * N), dtype=torch.int32, device=device)
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
    batch is exhausted; the ranks then all-gather the rows they matched (tagged with their pair
    indices, padded to the largest count) and scatter them into place: about the result size
    through the collective (:func:`exchange_bytes`) instead of a whole-batch reduction.  Chunk sizes
    follow :func:`guided_chunk`.  Without an initialised process group the same loop runs on a local
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

    width = 1 + 2 * M + 2 * N
    parts, done = [], []
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
        parts.append(_pack(pred, M, N, b - a, a, device))
        done.append((a, b))
    mine = torch.cat(parts) if parts else torch.empty((0, width), dtype=torch.int32, device=device)
    if not distributed:
        return _unpack(mine[mine[:, 0].argsort()], M, N), done
    # fixed-size gather of exactly the rows each rank matched: counts first (one int per rank), then
    # the tagged rows padded to the largest count; every pair arrives exactly once
    n = torch.tensor([mine.shape[0]], dtype=torch.int64, device=device)
    counts = torch.empty(world, dtype=torch.int64, device=device)
    dist.all_gather_into_tensor(counts, n, group=group)
    cl = counts.tolist()
    cap = max(cl)
    padded = torch.zeros((cap, width), dtype=torch.int32, device=device)
    padded[: mine.shape[0]] = mine
    every = torch.empty((world * cap, width), dtype=torch.int32, device=device)
    dist.all_gather_into_tensor(every, padded, group=group)
    rows = torch.cat([every[r * cap : r * cap + cl[r]] for r in range(world)])
    out = torch.empty((B, width), dtype=torch.int32, device=device)
    out[rows[:, 0].long()] = rows
    return _unpack(out, M, N), done


def exchange_bytes(B, M, N, world, counts=None):
    """Bytes one match_static / match_dynamic call moves through the collective (all ranks'
    contributions of the final gather; the count exchange of match_dynamic adds 8 per rank).
    ``counts`` = rows matched per rank (dynamic); None = static shards."""
    width = 4 * (1 + 2 * M + 2 * N)
    if counts is None:
        return world * (-(-B // world)) * width
    return world * max(counts) * width + 8 * world
