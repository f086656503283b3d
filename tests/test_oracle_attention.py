"""Pin the oracle's attention restatements (oracle/lstm.py) against the reference's own
standalone modules (tests/golden/attention_standalone.npz, oracle/gen_golden.py
case_attention_standalone): query [B, D], [B, 1, D] and [B, 20, D], key-padding mask,
AdaptiveAttention's memory_state / cell_state, outputs and every gradient.  CPU only."""
import os

import numpy as np
import pytest
import torch

from oracle import lstm as olstm

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "attention_standalone.npz")
VARIANTS = {"soft": ("soft", 1, 0.7), "multi_head": ("multi_head", 4, 1.0), "aoa": ("aoa", 4, 1.0),
            "aoa_soft": ("aoa", 1, 1.0), "adaptive": ("adaptive", 4, 1.3), "adaptive_soft": ("adaptive", 1, 1.0)}
FORMS = ("q1", "q1m", "qT")


def load_case(z, name, form):
    """(params, inputs dict) of one fixture case as torch tensors."""
    pre = name + "/p0/"
    p = {k[len(pre):]: torch.from_numpy(z[k].copy()) for k in z.files if k.startswith(pre)}
    t = {n: torch.from_numpy(z[f"in/{form}/{n}"].copy())
         for n in ("query", "key", "value", "memory_state", "cell_state", "gc", "gw")}
    t["mask"] = None if form == "q1" else torch.from_numpy(z["in/mask"].copy())
    return p, t


@pytest.mark.parametrize("form", FORMS)
@pytest.mark.parametrize("name", sorted(VARIANTS))
def test_oracle_attention_standalone_matches_reference(name, form):
    z = np.load(GOLD, allow_pickle=False)
    kind, heads, temp = VARIANTS[name]
    p, t = load_case(z, name, form)
    p = {k: v.requires_grad_(True) for k, v in p.items()}
    q = t["query"].requires_grad_(True)
    k = t["key"].requires_grad_(True)
    v = k if form == "q1" else t["value"].requires_grad_(True)
    h = t["memory_state"].requires_grad_(True)
    c = t["cell_state"].requires_grad_(True)
    ctx, w = olstm.standalone(kind, p, q, k, v, heads, temp, t["mask"], h, c)
    ((ctx * t["gc"]).sum() + (w * t["gw"]).sum()).backward()
    pre = f"{name}/{form}/"
    np.testing.assert_allclose(ctx.detach().numpy(), z[pre + "context"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(w.detach().numpy(), z[pre + "weights"], rtol=1e-5, atol=1e-7)
    got = {"dquery": q.grad, "dkey": k.grad}
    if form != "q1":
        got["dvalue"] = v.grad
    if kind == "adaptive":
        got["dmemory_state"], got["dcell_state"] = h.grad, c.grad
    for n, g in got.items():
        np.testing.assert_allclose(g.numpy(), z[pre + n], rtol=1e-4, atol=1e-6, err_msg=n)
    for n, prm in p.items():
        g = prm.grad if prm.grad is not None else torch.zeros_like(prm)
        np.testing.assert_allclose(g.numpy(), z[pre + "grad/" + n], rtol=1e-4, atol=1e-6, err_msg=n)
