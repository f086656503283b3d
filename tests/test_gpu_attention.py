"""AttentionMechanism drop-in contract on the GPU (attention.py:12-35,57-360):
``build_attention(cfg)(query, key, value, key_padding_mask[, memory_state, cell_state])``
for every module type, query [B, D] / [B, 1, D] / [B, 20, D], with and without a
key-padding mask, key is value and distinct key / value, against the reference's own
outputs and gradients (tests/golden/attention_standalone.npz, written by
oracle/gen_golden.py from the reference modules).  Loss = <context, gc> + <weights, gw>,
so the returned weights' gradient (MHA's head mean included) is checked too.
fp32: context / weights rtol 1e-4, every gradient rtol 2e-4 (atol 2e-4 * max|ref|, floored at
1e-6 of the largest parameter gradient for the analytically-zero MHA key bias gradient).
bf16: norm-relative error <= 3e-2 (outputs) and <= 6e-2 (gradients; the analytically-zero MHA key
bias gradient against 1e-2 of the largest parameter-gradient norm)."""
import os

import numpy as np
import pytest
import torch

from test_oracle_attention import FORMS, GOLD, VARIANTS, load_case

pytestmark = pytest.mark.gpu
cuda = pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a GPU")


def _module(name, p, precision):
    import capk
    from capk import config as C
    from capk.models.attention import build_attention
    kind, heads, temp = VARIANTS[name]
    cfg = C.AttentionConfig(attention_type=kind, num_heads=heads, temperature=temp)
    cfg.hidden_dim = int(p["sentinel_proj.weight" if kind == "adaptive" else "query_proj.weight"].shape[1])
    mod = build_attention(cfg)
    mod.load_state_dict(p, strict=True)
    capk.prepare(mod, "cuda", precision)
    return mod


def _run(name, form, precision):
    z = np.load(GOLD, allow_pickle=False)
    p, t = load_case(z, name, form)
    mod = _module(name, p, precision)
    for prm in mod.parameters():
        prm._capk_grad.zero_()
    dt = torch.float32 if precision == "fp32" else torch.bfloat16
    dev = lambda x: x.cuda().to(dt).requires_grad_(True)  # noqa: E731
    q, k = dev(t["query"]), dev(t["key"])
    v = k if form == "q1" else dev(t["value"])
    h, c = dev(t["memory_state"]), dev(t["cell_state"])
    mask = t["mask"].cuda() if t["mask"] is not None else None
    kw = {"memory_state": h, "cell_state": c} if VARIANTS[name][0] == "adaptive" else {}
    ctx, w = mod(q, k, v, mask, **kw)
    assert ctx.shape == tuple(z[f"{name}/{form}/context"].shape) and w.shape == tuple(z[f"{name}/{form}/weights"].shape)
    ((ctx.float() * t["gc"].cuda()).sum() + (w.float() * t["gw"].cuda()).sum()).backward()
    got = {"context": ctx, "weights": w, "dquery": q.grad, "dkey": k.grad}
    if form != "q1":
        got["dvalue"] = v.grad
    if kw:
        got["dmemory_state"], got["dcell_state"] = h.grad, c.grad
    for n, prm in mod.named_parameters():
        got["grad/" + n] = prm._capk_grad
    return z, got


@cuda
@pytest.mark.parametrize("form", FORMS)
@pytest.mark.parametrize("name", sorted(VARIANTS))
def test_attention_standalone_fp32(name, form):
    z, got = _run(name, form, "fp32")
    pre = f"{name}/{form}/"
    # floor for analytically-zero gradients (MHA key_proj.bias: softmax is shift-invariant, the
    # reference's values are fp32 rounding noise ~1e-8): 1e-6 of the module's largest gradient
    gmax = max(float(np.abs(z[k]).max()) for k in z.files if k.startswith(pre + "grad/"))
    for n, g in got.items():
        ref = z[pre + n]
        assert g is not None, n
        g = g.detach().float().cpu().numpy()
        if n in ("context", "weights"):
            np.testing.assert_allclose(g, ref, rtol=1e-4, atol=1e-6, err_msg=n)
        else:
            atol = 2e-4 * max(float(np.abs(ref).max()), 5e-3 * gmax)
            np.testing.assert_allclose(g, ref, rtol=2e-4, atol=atol, err_msg=n)


@cuda
@pytest.mark.parametrize("form", ("q1m", "qT"))
@pytest.mark.parametrize("name", sorted(VARIANTS))
def test_attention_standalone_bf16(name, form):
    z, got = _run(name, form, "bf16")
    pre = f"{name}/{form}/"
    # MHA's key_proj.bias gradient is analytically zero (its reference values are fp32 noise): its
    # bf16 error is measured against 1e-2 of the module's largest parameter-gradient norm
    gnorm = max(float(np.linalg.norm(z[k])) for k in z.files if k.startswith(pre + "grad/"))
    for n, g in got.items():
        ref = z[pre + n]
        g = g.detach().float().cpu().numpy()
        floor = 1e-2 * gnorm if n.startswith("grad/") else 1e-12
        err = np.linalg.norm(g - ref) / max(np.linalg.norm(ref), floor)
        tol = 3e-2 if n in ("context", "weights") else 6e-2
        assert err <= tol, f"{n}: rel {err:.3g} > {tol}"
