"""AdamW over the flat parameter store + the reference's LR schedule.

Restates CaptioningTrainer._create_optimizer (src/train/trainer.py:111-134):
two groups (weight decay 0.01 / 0.0 for names containing 'bias' or
'LayerNorm.weight'), torch AdamW betas (0.9, 0.999), eps 1e-8 — and
get_cosine_schedule_with_warmup (trainer.py:136-162).  One fused HIP kernel per
group segment updates fp32 master, m, v and refreshes the bf16 shadow.
"""
import math

import torch

from .. import ops


def cosine_schedule_with_warmup(step, base_lr, warmup, total, num_cycles=0.5):
    if step < warmup:
        return base_lr * float(step) / float(max(1, warmup))
    progress = float(step - warmup) / float(max(1, total - warmup))
    return base_lr * max(0.0, 0.5 * (1.0 + math.cos(math.pi * float(num_cycles) * 2.0 * progress)))


class CapkAdamW:
    def __init__(self, store, lr=5e-5, weight_decay=0.01, betas=(0.9, 0.999), eps=1e-8):
        self.store = store
        self.lr = lr
        self.wd = {"decay": weight_decay, "no_decay": 0.0}
        self.betas = betas
        self.eps = eps
        self.m = {g: torch.zeros_like(store.master[g]) for g in store.groups}
        self.v = {g: torch.zeros_like(store.master[g]) for g in store.groups}
        self.steps = {}  # per (group, start) segment -> step count (torch keeps per-param 'step')

    def step(self, lr=None):
        lr = self.lr if lr is None else lr
        st = self.store
        for g in st.groups:
            for key, s, e in st.segments(g):
                n = self.steps.get(key, 0) + 1
                self.steps[key] = n
                sh = None if st.bf16[g] is None else st.bf16[g][s:e]
                ops.adamw(st.master[g][s:e], st.grad[g][s:e], self.m[g][s:e], self.v[g][s:e], sh, lr, self.wd[g],
                          self.betas[0], self.betas[1], self.eps, n)
        st.written_optional.clear()

    def zero_grad(self, set_to_none=False):
        # capk backward passes overwrite every gradient they produce; nothing to clear.
        self.store.relink_grads()

    def state_dict(self):
        return {"m": self.m, "v": self.v, "steps": dict(self.steps), "lr": self.lr}

    def load_state_dict(self, sd):
        for g in self.m:
            self.m[g].copy_(sd["m"][g])
            self.v[g].copy_(sd["v"][g])
        self.steps = dict(sd["steps"])
        self.lr = sd["lr"]
