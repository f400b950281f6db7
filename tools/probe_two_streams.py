"""Probe (tools only): does splitting the 32-pair bench batch into two 16-pair forwards on two
HIP streams (one host thread each) overlap the HBM-heavy GEMM epilogues of one half with the
MFMA/VALU-bound attention of the other?  Prints ms per 32 pairs for both schedules."""
import os
import sys
import threading
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import lgamd  # noqa: F401,E402
from bench import gpu_pairs  # noqa: E402
from lightglue_amd import LightGlue  # noqa: E402
from lightglue_amd.weights import synthetic_state_dict  # noqa: E402

dev = torch.device("cuda", 0)
conf = {"filter_threshold": 0.1}
sd = {k: torch.from_numpy(v) for k, v in synthetic_state_dict(conf, seed=0).items()}
N = 2048


def mk():
    m = LightGlue(conf).eval().to(dev)
    m.load_state_dict(sd, strict=True)
    return m


full = gpu_pairs(32, N, 256, seed=1, device=dev)
halves = [{k: (v[i * 16:(i + 1) * 16] if torch.is_tensor(v) else {"image_size": v["image_size"][i * 16:(i + 1) * 16]})
           for k, v in full.items()} for i in range(2)]
m1, ma, mb = mk(), mk(), mk()
streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]


def one():
    with torch.no_grad():
        return m1(full)


def two():
    res = [None, None]

    def run(i, m):
        with torch.cuda.stream(streams[i]), torch.no_grad():
            res[i] = m(halves[i])

    ts = [threading.Thread(target=run, args=(i, m)) for i, m in ((0, ma), (1, mb))]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    torch.cuda.synchronize()
    return res


for name, fn in (("one stream, 32 pairs", one), ("two streams, 2 x 16 pairs", two), ("one stream, 32 pairs", one),
                 ("two streams, 2 x 16 pairs", two)):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        r = fn()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / 5 * 1e3
    print(f"{name:28s} {ms:8.2f} ms per 32 pairs  ({32e3 / ms:7.1f} pairs/s)", flush=True)
a = one()
b = two()
same = all(torch.equal(a["matches0"][i * 16:(i + 1) * 16], b[i]["matches0"]) for i in range(2))
print("two-stream matches identical to one-stream:", same)
