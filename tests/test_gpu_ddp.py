"""ddp.DataParallel itself on the GPU: the per-layer gradient buckets all-reduced from
the library's grad-ready hooks, the assignment heads' post-accumulate hooks, SuperGlue's
SyncBatchNorm collective (sg_set_collective) and the finish / average step -- the reference's
``train.py:307-309`` (convert_sync_batchnorm + DistributedDataParallel).

``tools/ddp_check.py`` runs one training step of each matcher as two gloo ranks on cuda:0 (one pair
each) and as one process on both pairs, and compares every parameter gradient and running
statistic with the float64 oracle of the concatenated batch (bar per tensor: 8x the float32
oracle's spread + 1e-6 of the tensor's scale) and the two HIP runs with each other.  It runs as a
child process whose parent never touches the GPU (it spawns every GPU process itself)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_data_parallel_two_ranks_equal_one_process_on_the_concatenated_batch(tmp_path):
    out = os.path.join(str(tmp_path), "ddp_check.json")
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="4")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "ddp_check.py"), "--out", out], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=150)
    assert os.path.exists(out), r.stdout[-3000:] + r.stderr[-3000:]
    reps = json.load(open(out))
    assert {rep["model"] for rep in reps} == {"superglue", "lightglue"}
    for rep in reps:
        assert rep["ok"], (rep["model"], rep["bad"][:6], rep["worst_err_over_tol"][:4])
        assert rep["n_checked"] > 0
        # rank losses are per-rank means; their average is the one-process loss of both pairs
        assert abs(sum(rep["loss_ranks"]) / 2 - rep["loss_single"]) <= 1e-5 * max(1.0, abs(rep["loss_single"]))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
