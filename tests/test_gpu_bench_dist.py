"""bench.py's multi-GPU path on RCCL (the backend the driver's N = 2, 4, 8 runs use), exercised on a
one-GPU box: ``python -m torch.distributed.run --nproc-per-node 1 bench.py --gpus 1`` with
LG_BENCH_DIST=1 runs the same code as each rank of an N-rank job -- ``init_process_group("nccl")``,
the barriers, ``parallel.match_static``'s all_gather_into_tensor of the match results, configs[3]'s
c10d-store chunk queue and all-gather merge, ``ddp.DataParallel``'s per-layer gradient buckets and
SuperGlue's SyncBatchNorm collective, and the max-over-ranks all_reduce of the timed region.  The
launcher never touches the GPU; each run is a child process with its own time limit."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _bench(*args):
    env = dict(os.environ, LG_BENCH_DIST="1", HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="4")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "1", "--steps", "2", "--warmup", "1", "--cpu-budget", "0", *args]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


@pytest.mark.parametrize("workload,extra,marker", [
    ("configs2", ["--batch", "4", "--npts", "1024"], "RCCL all-gather"),
    ("configs3", ["--batch", "4", "--npts", "1024", "--chunk", "2"], "c10d-store queue"),
    ("configs4", ["--batch", "2", "--npts", "1024"], "RCCL all-gather"),
    ("train", ["--batch", "2", "--npts", "512"], "ddp.DataParallel"),
    ("train_sg", ["--batch", "2", "--npts", "512"], "SyncBatchNorm"),
])
def test_bench_process_group_path_on_rccl(workload, extra, marker):
    d = _bench("--workload", workload, *extra)
    assert d["n_gpus"] == 1 and d["value"] > 0, d
    assert marker in d["config"]["parallelism"], d["config"]
    if workload == "configs2":
        assert d["matches_per_pair"] > 0 and d["roofline"]["achieved"] > 0
    if workload.startswith("train"):
        assert d["loss"] == d["loss"]  # finite
