"""Diagnostic: fp16x3 (range-scaled) vs bf16x6 vs the CPU oracle on inputs scaled past fp16."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
import lgamd  # noqa
import oracle
from lightglue_amd import LightGlue
from lightglue_amd.weights import synthetic_pair, synthetic_state_dict

conf = {"filter_threshold": 0.1}
sd = synthetic_state_dict(conf, seed=0)
def mk(p):
    m = LightGlue({**conf, "precision": p}).eval().cuda()
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}); return m
auto, x6 = mk("auto"), mk("bf16x6")
for scale in [1.0, 1e2, 1e3, 1e4, 3e4, 1e5, 2e5]:
    data = synthetic_pair(B=1, M=128, N=120, seed=2)
    data["descriptors0"] = data["descriptors0"] * np.float32(scale)
    g = {k: torch.from_numpy(v).cuda() for k, v in data.items() if not k.startswith("image_size")}
    g["view0"] = {"image_size": torch.from_numpy(data["image_size0"]).cuda()}
    g["view1"] = {"image_size": torch.from_numpy(data["image_size1"]).cuda()}
    with torch.no_grad():
        a, b = auto(g), x6(g)
    r = oracle.lightglue_forward(sd, data, conf)
    am, bm, rm = a["matches0"].cpu().numpy(), b["matches0"].cpu().numpy(), r["matches0"].numpy()
    da = np.abs(a["ref_descriptors0"].cpu().numpy() - r["ref_descriptors0"].numpy()).max()
    db = np.abs(b["ref_descriptors0"].cpu().numpy() - r["ref_descriptors0"].numpy()).max()
    print(f"scale {scale:8.0e}: auto!=x6 {int((am!=bm).sum())}  auto!=cpu {int((am!=rm).sum())}  x6!=cpu {int((bm!=rm).sum())}"
          f"  desc err auto {da:.3e} x6 {db:.3e} (max|desc| {np.abs(r['ref_descriptors0'].numpy()).max():.3e})", flush=True)
