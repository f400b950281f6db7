"""Probe (tools only): split the 32-pair bench batch into two 16-pair forwards on two CU-masked HIP
streams (each stream owns half of the CUs), one stream started DELAY_MS later, so that one half's
store-bound GEMM epilogues overlap the other half's MFMA work instead of every CU storing at once.
Prints ms per 32 pairs for the one-stream and the two-stream schedules, alternating."""
import ctypes
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
ncu = torch.cuda.get_device_properties(dev).multi_processor_count
hip = ctypes.CDLL("libamdhip64.so")


def masked_stream(bits):
    words = (ctypes.c_uint32 * ((ncu + 31) // 32))()
    for b in bits:
        words[b // 32] |= 1 << (b % 32)
    s = ctypes.c_void_p()
    rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), ctypes.c_uint32(len(words)), words)
    assert rc == 0, rc
    return torch.cuda.ExternalStream(s.value, device=dev)


def mk():
    m = LightGlue(conf).eval().to(dev)
    m.load_state_dict(sd, strict=True)
    return m


full = gpu_pairs(32, N, 256, seed=1, device=dev)
halves = [{k: (v[i * 16:(i + 1) * 16] if torch.is_tensor(v) else {"image_size": v["image_size"][i * 16:(i + 1) * 16]})
           for k, v in full.items()} for i in range(2)]
m1, ma, mb = mk(), mk(), mk()
masks = {
    "contiguous halves": (range(0, ncu // 2), range(ncu // 2, ncu)),
    "even/odd CUs": (range(0, ncu, 2), range(1, ncu, 2)),
}
delay_ms = float(os.environ.get("DELAY_MS", "1.3"))
cyc_per_ms = 100e3  # torch.cuda._sleep counts s_memrealtime-ish ticks: calibrated below


def one():
    with torch.no_grad():
        return m1(full)


def calibrate():
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    torch.cuda._sleep(1_000_000)
    e1.record()
    torch.cuda.synchronize()
    return 1_000_000 / e0.elapsed_time(e1)


def make_two(streams, delay):
    def two():
        res = [None, None]

        def run(i, m):
            with torch.cuda.stream(streams[i]), torch.no_grad():
                if i == 1 and delay > 0:
                    torch.cuda._sleep(int(delay * cyc_per_ms))
                res[i] = m(halves[i])

        ts = [threading.Thread(target=run, args=(i, m)) for i, m in ((0, ma), (1, mb))]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        torch.cuda.synchronize()
        return res
    return two


def timeit(fn, reps=5):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        r = fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3, r


cyc_per_ms = calibrate()
print(f"{ncu} CUs; sleep ticks per ms {cyc_per_ms:.0f}", flush=True)
plain = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
cands = [("one stream, 32 pairs", one)]
cands.append(("two unmasked streams, delay 0", make_two(plain, 0.0)))
for name, (a, b) in masks.items():
    st = [masked_stream(a), masked_stream(b)]
    for d in (0.0, delay_ms):
        cands.append((f"two masked ({name}), delay {d}", make_two(st, d)))
for rnd in range(2):
    for name, fn in cands:
        ms, _ = timeit(fn)
        print(f"{name:48s} {ms:8.2f} ms per 32 pairs  ({32e3 / ms:7.1f} pairs/s)", flush=True)
a = one()
b = cands[-1][1]()
same = all(torch.equal(a["matches0"][i * 16:(i + 1) * 16], b[i]["matches0"]) and
           torch.equal(a["matching_scores0"][i * 16:(i + 1) * 16], b[i]["matching_scores0"]) for i in range(2))
print("two-stream outputs identical to one-stream:", same)
