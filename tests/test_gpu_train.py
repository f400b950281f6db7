"""LightGlue backward pass on the HIP library (training path, include/lightglue_mi355x.h
"Training") -- needs an MI355X.

Gradients are checked two ways:
* against the reference's own autograd gradients (tests/golden/grad_*.npz, make_grad_golden.py:
  float64 values at seeded sample positions), and
* against the float64 autograd gradients of the oracle restatement (oracle/lightglue_train_ref.py,
  itself pinned to those goldens by tests/test_oracle_grad.py) on EVERY entry of every tensor.
Bar per tensor: max |g_gpu - g64| <= 8 * spread32 + 1e-6 * max|g64| + 1e-12, where spread32 is
how far a float32 autograd gradient lies from float64: the larger of the reference's own float32
run (stored in the golden) and the oracle's float32 run (round 5; one run's rounding luck is not
the scale -- at N = 512 the two differ by up to 8x on single tensors).
The HIP path is fp32 arithmetic like the reference's float32 run, with different summation orders
(and float-atomic dQ sums), so a few spreads of headroom are the right scale.
Kernel-level checks: the f32 matrix-core GEMM in every transpose form (split-k included) and the
training attention forward / backward against float64 torch.
"""
import ctypes

import numpy as np
import pytest
import torch

import lgamd  # noqa: F401
from grad_golden_util import desc_golden, desc_pick, golden_entries, grad_case, grad_names, load_grad, oracle_grads

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _p(t):
    return ctypes.c_void_p(0 if t is None else t.data_ptr())


def _lib():
    from lightglue_amd import _lib

    return _lib, _lib.load()


# ------------------------------------------------------------------ kernel level
@pytest.mark.parametrize("ta,tb", [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize("M,N,K,batch", [(200, 136, 72, 1), (37, 300, 129, 3), (256, 512, 5000, 1), (33, 17, 4100, 2)])
def test_train_gemm_matches_fp64(ta, tb, M, N, K, batch):
    L, lib = _lib()
    g = torch.Generator().manual_seed(M * 7 + N + K)
    A = torch.randn((batch, K, M) if ta else (batch, M, K), generator=g)
    Bm = torch.randn((batch, N, K) if tb else (batch, K, N), generator=g)
    C0 = torch.randn((batch, M, N), generator=g)
    bias = torch.randn(N, generator=g)
    alpha, beta = 0.75, 1.0
    ref = alpha * ((A.transpose(1, 2) if ta else A).double() @ (Bm.transpose(1, 2) if tb else Bm).double()
                   + bias.double()) + beta * C0.double()
    Ad, Bd, Cd, bd = A.to(DEV), Bm.to(DEV), C0.to(DEV), bias.to(DEV)
    nb = ctypes.c_size_t()
    L.check(lib.lg_train_gemm_workspace_bytes(M, N, K, batch, ctypes.byref(nb)), "ws")
    ws = torch.empty(max(nb.value, 4), dtype=torch.uint8, device=DEV)
    lda = A.shape[2]
    ldb = Bm.shape[2]
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    L.check(lib.lg_train_gemm(_p(Ad), _p(Bd), _p(Cd), lda, ldb, N, A[0].numel(), Bm[0].numel(), M * N, M, N, K, batch,
                              alpha, beta, _p(bd), ta, tb, _p(ws), nb.value, st), "lg_train_gemm")
    err = (Cd.cpu().double() - ref).abs().max().item()
    # fp32 accumulation over K terms of |a b| ~ 1: a few ulps of sqrt(K)-scale sums
    assert err <= 2e-6 * max(K, 64) ** 0.5 * 8, err


def _attn_ref(q, k, v, scale):
    s = torch.einsum("bhid,bhjd->bhij", q, k) * scale
    return torch.softmax(s, -1) @ v


@pytest.mark.parametrize("B,Nq,Nk", [(2, 96, 96), (1, 200, 77), (3, 33, 300), (1, 1, 5)])
def test_train_attention_forward_backward_fp64(B, Nq, Nk):
    L, lib = _lib()
    H, scale = 4, 0.125
    g = torch.Generator().manual_seed(B * 1000 + Nq + Nk)
    q = torch.randn(B, Nq, 256, generator=g) * 2
    k = torch.randn(B, Nk, 256, generator=g) * 2
    v = torch.randn(B, Nk, 256, generator=g)
    go = torch.randn(B, Nq, 256, generator=g)

    def heads(t):
        return t.double().unflatten(-1, (H, 64)).transpose(1, 2)

    qd, kd, vd = (heads(t).requires_grad_() for t in (q, k, v))
    o = _attn_ref(qd, kd, vd, scale)
    o.backward(heads(go))
    o_ref = o.detach().transpose(1, 2).flatten(-2)
    dq_ref, dk_ref, dv_ref = (t.grad.transpose(1, 2).flatten(-2) for t in (qd, kd, vd))

    qg, kg, vg, gog = (t.to(DEV).contiguous() for t in (q, k, v, go))
    og = torch.empty(B, Nq, 256, device=DEV)
    lse = torch.empty(B * H * Nq, device=DEV)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    L.check(lib.lg_train_attention(_p(qg), _p(kg), _p(vg), B, H, Nq, Nk, scale, _p(og), _p(lse), st), "fwd")
    np.testing.assert_allclose(og.cpu().double().numpy(), o_ref.numpy(), atol=2e-5, rtol=1e-5)
    s = torch.einsum("bhid,bhjd->bhij", heads(q), heads(k)) * scale
    lse_ref = torch.logsumexp(s, -1).flatten() / np.log(2.0)
    np.testing.assert_allclose(lse.cpu().double().numpy(), lse_ref.numpy(), atol=2e-5, rtol=1e-6)
    dq, dk, dv = (torch.empty_like(t) for t in (qg, kg, vg))
    delta = torch.empty(B * H * Nq, device=DEV)
    L.check(lib.lg_train_attention_backward(_p(qg), _p(kg), _p(vg), _p(og), _p(lse), _p(gog), B, H, Nq, Nk, scale,
                                            _p(dq), _p(dk), _p(dv), _p(delta), st), "bwd")
    for got, ref in ((dq, dq_ref), (dk, dk_ref), (dv, dv_ref)):
        r = ref.numpy()
        np.testing.assert_allclose(got.cpu().double().numpy(), r, atol=2e-5 * max(1.0, np.abs(r).max()), rtol=1e-5)


# ------------------------------------------------------------------ full backward
REF_ONLY_CANARY = 2.0  # see test_gpu_sg_train.py


def _gpu_grads(conf, sd, pair, gt):
    from lightglue_amd import LightGlue

    model = LightGlue(conf).to(DEV)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
    model.train()
    data = {k: torch.from_numpy(v).to(DEV) for k, v in pair.items()
            if not k.startswith(("image_size", "descriptors"))}
    d0 = torch.from_numpy(pair["descriptors0"]).to(DEV).requires_grad_()
    d1 = torch.from_numpy(pair["descriptors1"]).to(DEV).requires_grad_()
    data["descriptors0"], data["descriptors1"] = d0, d1
    data["view0"] = {"image_size": torch.from_numpy(pair["image_size0"]).to(DEV)}
    data["view1"] = {"image_size": torch.from_numpy(pair["image_size1"]).to(DEV)}
    data.update({k: torch.from_numpy(v).to(DEV) for k, v in gt.items()})
    pred = model(data)
    losses, _ = model.loss(pred, data)
    loss = torch.mean(losses["total"])  # train.py:436
    loss.backward()  # train.py:450
    grads = {n: (p.grad.detach().double().cpu().numpy() if p.grad is not None else None)
             for n, p in model.named_parameters()}
    return float(loss.detach()), grads, d0.grad.double().cpu().numpy(), d1.grad.double().cpu().numpy(), pred


@pytest.mark.parametrize("name", grad_names())
def test_backward_matches_reference_and_oracle(name):
    g, meta = load_grad(name)
    conf, sd, pair, gt = grad_case(meta)
    loss, grads, gd0, gd1, pred = _gpu_grads(conf, sd, pair, gt)
    assert abs(loss - float(g["loss64"])) <= 1e-4 * abs(float(g["loss64"]))
    _, og, ogd0, ogd1 = oracle_grads(conf, sd, pair, gt)
    # spread32 = the larger distance from float64 of two float32 implementations: the reference's
    # own run (golden) and the oracle's (round 5: one fp32 run's rounding luck is not the scale)
    _, og32, o32d0, o32d1 = oracle_grads(conf, sd, pair, gt, dtype=torch.float32)

    def spread(ref32, r64, o32):
        return max(float(ref32), float(np.abs(np.asarray(o32) - r64).max()))
    worst, bad, canary = [], [], []
    for n in meta["names"]:
        assert grads[n] is not None, f"no gradient for {n}"
        tol = 8 * spread(g[f"spread32:{n}"], og[n], og32[n]) + 1e-6 * float(g[f"max64:{n}"]) + 1e-12
        idx, ref = golden_entries(g, n)
        got = grads[n].reshape(-1)
        e_gold = np.abs((got if idx is None else got[idx]) - ref).max()
        e_full = np.abs(got - og[n].reshape(-1)).max()
        worst.append((max(e_gold, e_full) / tol, n))
        if e_gold > tol or e_full > tol:
            bad.append((n, float(e_gold), float(e_full), tol, float(g[f"max64:{n}"])))
        # canary on the bar of the reference's own float32 spread alone (round 5's
        # default routes reached 1.19 of it, profiles/r05/grad_routes/)
        canary.append((float(e_gold) / (8 * float(g[f"spread32:{n}"]) + 1e-6 * float(g[f"max64:{n}"]) + 1e-12), n))
    for got, ref, r32, key in ((gd0, ogd0, o32d0, "gdesc0"), (gd1, ogd1, o32d1, "gdesc1")):
        idx, gref, gmax = desc_golden(g, key)
        tol = 8 * spread(g[f"spread_{key}"], ref, r32) + 1e-6 * gmax + 1e-12
        e_gold, e_full = np.abs(desc_pick(got, idx) - gref).max(), np.abs(got - ref).max()
        worst.append((max(e_gold, e_full) / tol, key))
        if e_gold > tol or e_full > tol:
            bad.append((key, float(e_gold), float(e_full), tol, gmax))
    worst.sort(reverse=True)
    canary.sort(reverse=True)
    print(name, "loss", loss, "worst err/tol:", [(n, round(r, 3)) for r, n in worst[:6]],
          "reference-spread-only:", [(n, round(r, 3)) for r, n in canary[:3]])
    assert not bad, bad[:12]
    assert canary[0][0] <= REF_ONLY_CANARY, canary[:4]


@pytest.mark.parametrize("name", ["grad_train_b2_n64", "grad_train_l3_b2_n96_proj_ori"])
def test_checkpointed_step_matches_full_step(name):
    """conf ``checkpointed`` (lightglue.py:353,515-518; LG_FWD_CHECKPOINTED): the training call keeps
    each layer's output only and the backward recomputes every layer's activations before
    differentiating it.  The forward kernels are deterministic, so the loss and the log assignment
    equal the full step's bit for bit; the gradients equal it up to the float-atomic dQ sums'
    order (checked at the golden's bar form); the saved buffer at the configs[2] shape shrinks
    below a quarter."""
    g, meta = load_grad(name)
    conf, sd, pair, gt = grad_case(meta)
    loss_f, grads_f, gd0_f, gd1_f, pred_f = _gpu_grads(conf, sd, pair, gt)
    loss_c, grads_c, gd0_c, gd1_c, pred_c = _gpu_grads({**conf, "checkpointed": True}, sd, pair, gt)
    assert loss_c == loss_f
    assert torch.equal(pred_c["log_assignment"], pred_f["log_assignment"])
    bad = []
    for n in meta["names"]:
        tol = 8 * float(g[f"spread32:{n}"]) + 1e-6 * float(g[f"max64:{n}"]) + 1e-12
        e = float(np.abs(grads_c[n] - grads_f[n]).max())
        if e > tol:
            bad.append((n, e, tol))
    for key, a, b in (("gdesc0", gd0_c, gd0_f), ("gdesc1", gd1_c, gd1_f)):
        _, _, gmax = desc_golden(g, key)
        tol = 8 * float(g[f"spread_{key}"]) + 1e-6 * gmax + 1e-12
        if float(np.abs(a - b).max()) > tol:
            bad.append((key, float(np.abs(a - b).max()), tol))
    assert not bad, bad[:8]
    from lightglue_amd import LightGlue
    from lightglue_amd import _lib as L

    model = LightGlue({"n_layers": 9}).to(DEV)
    lib = model._ensure_handle(DEV, upload=False)
    full, ck = ctypes.c_size_t(), ctypes.c_size_t()
    L.check(lib.lg_train_saved_bytes_ex(model._handle, 32, 2048, 2048, L.LG_FWD_TRAINING_GATE, ctypes.byref(full)), "sb")
    L.check(lib.lg_train_saved_bytes_ex(model._handle, 32, 2048, 2048, L.LG_FWD_TRAINING_GATE | L.LG_FWD_CHECKPOINTED,
                                        ctypes.byref(ck)), "sb")
    plain = ctypes.c_size_t()
    L.check(lib.lg_train_saved_bytes(model._handle, 32, 2048, 2048, ctypes.byref(plain)), "sb")
    assert plain.value == full.value
    print(name, f"saved bytes at configs[2]: full {full.value / 2**30:.2f} GiB, checkpointed {ck.value / 2**30:.2f} GiB")
    assert ck.value < full.value / 4


def test_training_forward_matches_eval_forward_descriptors():
    """The autograd training forward (fp32 f32-MFMA kernels) and the no-grad training-mode forward
    (the fp16x3 eval kernels with the training gate) produce the same per-layer descriptors."""
    from lightglue_amd import LightGlue
    from lightglue_amd.weights import synthetic_pair, synthetic_state_dict

    conf = {"filter_threshold": 0.1, "n_layers": 3}
    sd = synthetic_state_dict(conf, seed=2)
    pair = synthetic_pair(B=2, M=100, N=90, seed=5)
    model = LightGlue(conf).to(DEV)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    model.train()
    data = {k: torch.from_numpy(v).to(DEV) for k, v in pair.items() if not k.startswith("image_size")}
    data["view0"] = {"image_size": torch.from_numpy(pair["image_size0"]).to(DEV)}
    data["view1"] = {"image_size": torch.from_numpy(pair["image_size1"]).to(DEV)}
    with torch.no_grad():
        ref = model(data)
    pred = model(data)
    assert pred["ref_descriptors0"].requires_grad
    for k in ("ref_descriptors0", "ref_descriptors1", "log_assignment"):
        np.testing.assert_allclose(pred[k].detach().cpu().numpy(), ref[k].cpu().numpy(), atol=1e-4, rtol=1e-4)
    assert torch.equal(pred["matches0"], ref["matches0"])


@pytest.mark.parametrize("tokens", [True, False])
def test_head_backward_from_forward_equals_recompute(tokens):
    """lg_head_backward_from_forward (the loss heads reuse their forward's md / z / similarity /
    LSEs) gives the recomputing lg_head_backward's gradients bit for bit: the forward kernels are
    deterministic, so the saved values are the recomputed ones."""
    from lightglue_amd import LightGlue
    from lightglue_amd.lightglue import _head_backward, _head_forward
    from lightglue_amd.weights import synthetic_state_dict

    conf = {"n_layers": 3}
    model = LightGlue(conf).to(DEV)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in synthetic_state_dict(conf, seed=9).items()})
    params = model._schema_params(DEV)
    g = torch.Generator(device="cpu").manual_seed(4)
    B, M, N = 2, 150, 97
    d0 = torch.randn(B, M, 256, generator=g).to(DEV)
    d1 = torch.randn(B, N, 256, generator=g).to(DEV)
    la, _, t0, t1, scratch = _head_forward(model, 1, d0, d1, params, tokens, keep_scratch=True)
    w = torch.rand((B, M + 1, N + 1), generator=g).to(DEV)
    s_in, s_dust = torch.rand(B, generator=g).to(DEV), torch.rand(B, generator=g).to(DEV)
    gt0 = torch.randn(B, M, generator=g).to(DEV) if tokens else None
    gt1 = torch.randn(B, N, generator=g).to(DEV) if tokens else None
    needs = [True] * len(params) + [True, True]
    ref = _head_backward(model, 1, d0, d1, params, needs, w, s_in, s_dust, None, gt0, gt1)
    got = _head_backward(model, 1, d0, d1, params, needs, w, s_in, s_dust, None, gt0, gt1, fwd_scratch=scratch)
    torch.cuda.synchronize()
    assert torch.equal(got[0], ref[0]) and torch.equal(got[1], ref[1])
    n = 0
    for a, b in zip(got[2], ref[2]):
        assert (a is None) == (b is None)
        if a is not None:
            assert torch.equal(a, b)
            n += 1
    assert n >= (6 if tokens else 4)


@pytest.mark.parametrize("B,N,layer", [(2, 150, 1), (1, 2048, 0), (3, 33, 2)])
def test_head_nll_forward_matches_stored_log_assignment(B, N, layer):
    """lg_head_nll_forward (the loss heads without a stored log assignment) against lg_head_forward
    + sg_nll_loss + torch argmaxes on the stored log assignment: the NLL terms to fp32 rounding (the
    fp64 sums are grouped differently), the argmaxes and token logits exactly; M != N raises the
    reference's error (losses.py:66-70)."""
    from lightglue_amd import LightGlue
    from lightglue_amd.lightglue import _head_forward, _head_nll_forward
    from lightglue_amd.superglue import _nll, nll_inputs
    from lightglue_amd.weights import synthetic_state_dict
    from sg_golden_util import ground_truth

    conf = {"n_layers": 3}
    model = LightGlue(conf).to(DEV)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in synthetic_state_dict(conf, seed=12).items()})
    params = model._schema_params(DEV)
    g = torch.Generator(device="cpu").manual_seed(6)
    d0 = torch.randn(B, N, 256, generator=g).to(DEV)
    d1 = torch.randn(B, N, 256, generator=g).to(DEV)
    gt = {k: torch.from_numpy(v).to(DEV) for k, v in ground_truth(B, N, N, 8).items()}
    prepared = nll_inputs(gt, DEV)
    tokens = layer < 2
    terms, am0, am1, t0, t1, _ = _head_nll_forward(model, layer, d0, d1, params, tokens, prepared, 0.5)
    la, _, r0, r1 = _head_forward(model, layer, d0, d1, params, tokens)
    ref = _nll(la, gt, 1, 0.5, prepared)
    torch.cuda.synchronize()
    torch.testing.assert_close(terms, ref, rtol=2e-6, atol=1e-6)
    assert torch.equal(am0, la[:, :-1, :].max(-1).indices)
    assert torch.equal(am1, la[:, :, :-1].max(-2).indices)
    if tokens:
        assert torch.equal(t0, r0) and torch.equal(t1, r1)
    with pytest.raises(RuntimeError):
        _head_nll_forward(model, layer, d0, d1[:, : N - 1].contiguous(), params, False, prepared, 0.5)


@pytest.mark.parametrize("B,N,layer,reuse", [(2, 150, 1, False), (2, 148, 0, True), (1, 2048, 2, True), (3, 33, 1, True),
                                               (1, 3072, 0, True)])
def test_head_nll_backward_from_ground_truth_equals_dense_weights(B, N, layer, reuse):
    """lg_head_nll_backward (the NLL weights read from gt_assignment / gt_matches0/1, never a dense
    tensor) gives lg_head_backward's gradients on nll_weights (losses.py:62-73) bit for bit: every
    sum adds 0/1 values and every product is the same weight * scale.  M != N raises."""
    from lightglue_amd import LightGlue
    from lightglue_amd.lightglue import _head_backward, _head_forward
    from lightglue_amd.superglue import nll_inputs, nll_weights
    from lightglue_amd.weights import synthetic_state_dict
    from sg_golden_util import ground_truth

    conf = {"n_layers": 3}
    model = LightGlue(conf).to(DEV)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in synthetic_state_dict(conf, seed=13).items()})
    params = model._schema_params(DEV)
    g = torch.Generator(device="cpu").manual_seed(7)
    d0 = torch.randn(B, N, 256, generator=g).to(DEV)
    d1 = torch.randn(B, N, 256, generator=g).to(DEV)
    gt = {k: torch.from_numpy(v).to(DEV) for k, v in ground_truth(B, N, N, 8).items()}
    prepared = nll_inputs(gt, DEV)
    w = nll_weights(d0.new_empty((B, N + 1, N + 1)), gt)
    s_in, s_dust = -torch.rand(B, generator=g).to(DEV), -torch.rand(B, generator=g).to(DEV)
    tokens = layer < 2
    gt0 = torch.randn(B, N, generator=g).to(DEV) if tokens else None
    gt1 = torch.randn(B, N, generator=g).to(DEV) if tokens else None
    needs = [True] * len(params) + [True, True]
    ref = _head_backward(model, layer, d0, d1, params, needs, w, s_in, s_dust, None, gt0, gt1)
    scratch = _head_forward(model, layer, d0, d1, params, tokens, keep_scratch=True)[4] if reuse else None
    got = _head_backward(model, layer, d0, d1, params, needs, None, s_in, s_dust, None, gt0, gt1, fwd_scratch=scratch,
                         gt=prepared)
    torch.cuda.synchronize()
    assert torch.equal(got[0], ref[0]) and torch.equal(got[1], ref[1])
    n = 0
    for a, b in zip(got[2], ref[2]):
        assert (a is None) == (b is None)
        if a is not None:
            assert torch.equal(a, b)
            n += 1
    assert n >= (6 if tokens else 4)
    with pytest.raises(RuntimeError):
        _head_backward(model, layer, d0, d1[:, : N - 1].contiguous(), params, needs, None, s_in, s_dust, None, None, None,
                       gt=prepared)


def test_head_backward_dense_and_similarity_gradients():
    """_Head (plain autograd through log_assignment and similarity) against float64 torch."""
    from lightglue_amd import LightGlue
    from lightglue_amd.lightglue import _Head
    from lightglue_amd.weights import synthetic_state_dict
    from oracle.lightglue_ref import match_assignment

    conf = {"n_layers": 2}
    sd = synthetic_state_dict(conf, seed=4)
    model = LightGlue(conf).to(DEV)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    gen = torch.Generator().manual_seed(3)
    B, M, N = 2, 70, 45
    d0 = torch.randn(B, M, 256, generator=gen)
    d1 = torch.randn(B, N, 256, generator=gen)
    gla = torch.randn(B, M + 1, N + 1, generator=gen)
    gsim = torch.randn(B, M, N, generator=gen) * 0.1
    W = {k: torch.from_numpy(v).double().requires_grad_() for k, v in sd.items()}
    x0, x1 = d0.double().requires_grad_(), d1.double().requires_grad_()
    la, sim = match_assignment(x0, x1, W, "log_assignment.0")
    ((la * gla.double()).sum() + (sim * gsim.double()).sum()).backward()
    params = model._schema_params(DEV)
    g0, g1 = d0.to(DEV).requires_grad_(), d1.to(DEV).requires_grad_()
    la_g, sim_g, _, _ = _Head.apply(model, 0, False, g0, g1, *params)
    ((la_g * gla.to(DEV)).sum() + (sim_g * gsim.to(DEV)).sum()).backward()
    for got, ref in ((g0.grad, x0.grad), (g1.grad, x1.grad)):
        r = ref.numpy()
        np.testing.assert_allclose(got.cpu().double().numpy(), r, atol=1e-5 * np.abs(r).max(), rtol=0)
    named = dict(model.named_parameters())
    for n in ("log_assignment.0.final_proj.weight", "log_assignment.0.final_proj.bias",
              "log_assignment.0.matchability.weight", "log_assignment.0.matchability.bias"):
        r = W[n].grad.numpy()
        np.testing.assert_allclose(named[n].grad.cpu().double().numpy(), r, atol=1e-5 * np.abs(r).max(), rtol=0)


@pytest.mark.parametrize("conf,B,M,N", [({"n_layers": 2}, 2, 70, 45), ({"n_layers": 1, "input_dim": 64}, 1, 33, 130),
                                        ({"n_layers": 2, "add_scale_ori": True}, 3, 40, 40)])
def test_trunk_backward_ragged_vs_oracle(conf, B, M, N):
    """The training trunk (lg_train_forward / lg_train_backward) on ragged sets (M != N, sizes that
    are no multiple of any tile), input_proj and scale/ori positions, under an arbitrary loss on
    every layer's descriptors: every parameter gradient and both descriptor gradients against
    float64 autograd of the oracle (oracle/lightglue_train_ref.train_forward).  Bar: 2e-5 of each
    tensor's largest entry (fp32 arithmetic through <= 2 layers)."""
    from lightglue_amd import LightGlue
    from lightglue_amd.weights import synthetic_pair, synthetic_state_dict
    from oracle.lightglue_train_ref import train_forward

    sd = synthetic_state_dict(conf, seed=11)
    pair = synthetic_pair(B=B, M=M, N=N, seed=12, dim=int(conf.get("input_dim", 256)))
    if conf.get("add_scale_ori"):
        rng = np.random.Generator(np.random.PCG64(5))
        for k, n in (("0", M), ("1", N)):
            pair["scales" + k] = (rng.random((B, n)) * 2).astype(np.float32)
            pair["oris" + k] = (rng.random((B, n)) * 6.28 - 3.14).astype(np.float32)
    L = int(conf["n_layers"])
    gen = torch.Generator().manual_seed(7)
    w0 = torch.randn(B, L, M, 256, generator=gen)
    w1 = torch.randn(B, L, N, 256, generator=gen)
    # float64 oracle
    W = {k: torch.from_numpy(v).double().requires_grad_() for k, v in sd.items()}
    data64 = {k: torch.from_numpy(v).double() for k, v in pair.items() if not k.startswith("descriptors")}
    x0 = torch.from_numpy(pair["descriptors0"]).double().requires_grad_()
    x1 = torch.from_numpy(pair["descriptors1"]).double().requires_grad_()
    data64["descriptors0"], data64["descriptors1"] = x0, x1
    layers, _ = train_forward(W, data64, conf)
    loss64 = sum((a * w0[:, i].double()).sum() + (b * w1[:, i].double()).sum() for i, (a, b) in enumerate(layers))
    loss64.backward()
    # HIP
    model = LightGlue(conf).to(DEV)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
    model.train()
    data = {k: torch.from_numpy(v).to(DEV) for k, v in pair.items() if not k.startswith(("image_size", "descriptors"))}
    g0 = torch.from_numpy(pair["descriptors0"]).to(DEV).requires_grad_()
    g1 = torch.from_numpy(pair["descriptors1"]).to(DEV).requires_grad_()
    data["descriptors0"], data["descriptors1"] = g0, g1
    data["view0"] = {"image_size": torch.from_numpy(pair["image_size0"]).to(DEV)}
    data["view1"] = {"image_size": torch.from_numpy(pair["image_size1"]).to(DEV)}
    pred = model(data)
    ((pred["ref_descriptors0"] * w0.to(DEV)).sum() + (pred["ref_descriptors1"] * w1.to(DEV)).sum()).backward()
    named = dict(model.named_parameters())
    bad = []
    for n, w in W.items():
        if not n.startswith(("input_proj", "posenc.Wr", "transformers")):
            continue
        r = w.grad.numpy()
        got = named[n].grad.double().cpu().numpy()
        err, scale = np.abs(got - r).max(), np.abs(r).max()
        if err > 2e-5 * scale + 1e-9:
            bad.append((n, float(err), float(scale)))
    for got, ref, key in ((g0, x0, "d0"), (g1, x1, "d1")):
        r = ref.grad.numpy()
        err = np.abs(got.grad.double().cpu().numpy() - r).max()
        if err > 2e-5 * np.abs(r).max() + 1e-9:
            bad.append((key, float(err), float(np.abs(r).max())))
    assert not bad, bad[:8]


@pytest.mark.parametrize("frozen", ["posenc.Wr.weight", "posenc.condition_modulation.bias"])
def test_trunk_backward_with_one_posenc_parameter_frozen(frozen):
    """Freezing one positional-encoding parameter: the others still get their
    gradients -- equal to the run with every parameter trainable -- and the frozen one gets none
    (the library used to skip the posenc backward unless all three were requested, leaving the
    requested ones uninitialised)."""
    from lightglue_amd import LightGlue
    from lightglue_amd.weights import synthetic_pair, synthetic_state_dict

    conf = {"n_layers": 2}
    sd = synthetic_state_dict(conf, seed=11)
    pair = synthetic_pair(B=2, M=70, N=45, seed=12)
    gen = torch.Generator().manual_seed(7)
    w0 = torch.randn(2, 2, 70, 256, generator=gen).to(DEV)
    w1 = torch.randn(2, 2, 45, 256, generator=gen).to(DEV)

    def run(freeze):
        model = LightGlue(conf).to(DEV)
        model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
        model.train()
        named = dict(model.named_parameters())
        if freeze:
            named[freeze].requires_grad_(False)
        data = {k: torch.from_numpy(v).to(DEV) for k, v in pair.items() if not k.startswith("image_size")}
        data["view0"] = {"image_size": torch.from_numpy(pair["image_size0"]).to(DEV)}
        data["view1"] = {"image_size": torch.from_numpy(pair["image_size1"]).to(DEV)}
        pred = model(data)
        ((pred["ref_descriptors0"] * w0).sum() + (pred["ref_descriptors1"] * w1).sum()).backward()
        return {n: (p.grad.clone() if p.grad is not None else None) for n, p in named.items() if n.startswith("posenc.")}

    full = run(None)
    part = run(frozen)
    assert part[frozen] is None
    # run-to-run noise: the attention backward's dQ sums are float atomics, and the
    # condition_modulation gradient is zero in exact arithmetic (a common phase cancels in q.k),
    # so compare on the scale of the Wr gradient
    scale = float(full["posenc.Wr.weight"].abs().max())
    for n, g in part.items():
        if n == frozen:
            continue
        assert g is not None and torch.isfinite(g).all(), n
        err = float((g - full[n]).abs().max())
        assert err <= 1e-4 * scale, (n, err, scale)


def test_loss_heads_backward_twice_through_a_retained_graph():
    """_HeadNLL's backward drops only the forward's scratch, not the ground truth its NLL
    weights come from, so a second backward through a retained graph recomputes the head
    (lg_head_nll_backward, from_forward = 0) and gives the first backward's gradients."""
    g, meta = load_grad("grad_train_b2_n64")
    conf, sd, pair, gt = grad_case(meta)
    from lightglue_amd import LightGlue

    model = LightGlue(conf).to(DEV)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
    model.train()
    data = {k: torch.from_numpy(v).to(DEV) for k, v in pair.items() if not k.startswith("image_size")}
    data["view0"] = {"image_size": torch.from_numpy(pair["image_size0"]).to(DEV)}
    data["view1"] = {"image_size": torch.from_numpy(pair["image_size1"]).to(DEV)}
    data.update({k: torch.from_numpy(v).to(DEV) for k, v in gt.items()})
    pred = model(data)
    # the trunk's saved activations go with its first backward: differentiate the heads only
    rd0 = pred["ref_descriptors0"].detach().requires_grad_()
    rd1 = pred["ref_descriptors1"].detach().requires_grad_()
    losses, _ = model.loss({**pred, "ref_descriptors0": rd0, "ref_descriptors1": rd1}, data)
    loss = torch.mean(losses["total"])
    loss.backward(retain_graph=True)
    first = (rd0.grad.clone(), rd1.grad.clone())
    rd0.grad = rd1.grad = None
    loss.backward()
    for a, b in zip(first, (rd0.grad, rd1.grad)):
        scale = float(a.abs().max())
        assert scale > 0
        assert float((a - b).abs().max()) <= 1e-6 * scale
