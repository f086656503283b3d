"""AdamW over the flat parameter store + the reference's LR schedules.

Restates CaptioningTrainer._create_optimizer (src/train/trainer.py:111-134):
two groups (weight decay 0.01 / 0.0 for names containing 'bias' or
'LayerNorm.weight'), torch AdamW betas (0.9, 0.999), eps 1e-8 — and
_create_scheduler (trainer.py:136-162): HF get_cosine_schedule_with_warmup /
get_linear_schedule_with_warmup (both torch LambdaLR) or StepLR(total//3, 0.1).
One fused HIP kernel per group segment updates fp32 master, m, v and refreshes
the bf16 shadow.

Checkpoint compatibility (trainer.py:569-620): ``state_dict()`` is torch.optim.AdamW's
layout — ``{"state": {i: {"step", "exp_avg", "exp_avg_sq"}}, "param_groups": [...]}``
with parameter indices numbered the way the reference's optimizer numbers them
(``named_parameters()`` order, requires_grad only, decay group first) — and the
schedulers' ``state_dict()`` is LambdaLR's / StepLR's, so the optimizer / scheduler entries
of a checkpoint written by the reference trainer load here and vice versa (the file itself
through ``capk.train.trainer.load_checkpoint_file``, which maps the reference's pickled
``src.config`` classes onto capk.config under ``weights_only=True``).
"""
import math

import torch

from .. import ops
from ..params import no_decay


def cosine_schedule_with_warmup(step, base_lr, warmup, total, num_cycles=0.5):
    """transformers get_cosine_schedule_with_warmup lambda x base_lr."""
    if step < warmup:
        return base_lr * float(step) / float(max(1, warmup))
    progress = float(step - warmup) / float(max(1, total - warmup))
    return base_lr * max(0.0, 0.5 * (1.0 + math.cos(math.pi * float(num_cycles) * 2.0 * progress)))


def linear_schedule_with_warmup(step, base_lr, warmup, total):
    """transformers get_linear_schedule_with_warmup lambda x base_lr."""
    if step < warmup:
        return base_lr * float(step) / float(max(1, warmup))
    return base_lr * max(0.0, float(total - step) / float(max(1, total - warmup)))


def _reference_param_order(named_parameters):
    """trainer.py:117-126: [decay params..., no-decay params...] in named_parameters order,
    requires_grad only — the index space of torch's optimizer.state_dict()."""
    named = [(n, p) for n, p in named_parameters if p.requires_grad]
    dec = [(n, p) for n, p in named if not no_decay(n)]
    nod = [(n, p) for n, p in named if no_decay(n)]
    return dec, nod


class CapkAdamW:
    """torch.optim.AdamW semantics (decoupled weight decay, bias-corrected moments, one step
    count per parameter) over the ParamStore's flat buffers."""

    GROUP_KEYS = ("decay", "no_decay")

    def __init__(self, store, lr=5e-5, weight_decay=0.01, betas=(0.9, 0.999), eps=1e-8):
        self.store = store
        self.betas = betas
        self.eps = eps
        self.m = {g: torch.zeros_like(store.master[g]) for g in store.groups}
        self.v = {g: torch.zeros_like(store.master[g]) for g in store.groups}
        self.steps = {}  # per (group, start) segment -> step count (torch keeps per-param 'step')
        # torch-style groups: the scheduler writes 'lr' here (trainer.py:129-132 group order)
        self.param_groups = [{"lr": lr, "initial_lr": lr, "weight_decay": weight_decay, "betas": betas, "eps": eps},
                             {"lr": lr, "initial_lr": lr, "weight_decay": 0.0, "betas": betas, "eps": eps}]

    @property
    def lr(self):
        return self.param_groups[0]["lr"]

    @lr.setter
    def lr(self, v):
        for pg in self.param_groups:
            pg["lr"] = v

    @property
    def wd(self):
        return {g: pg["weight_decay"] for g, pg in zip(self.GROUP_KEYS, self.param_groups)}

    def step(self, lr=None):
        """One AdamW step; `lr` overrides the groups' current learning rate for this step."""
        from ..models.common import join_dw
        join_dw()  # (weight gradients still in flight on the side stream, if any)
        st = self.store
        for g, pg in zip(self.GROUP_KEYS, self.param_groups):
            glr = pg["lr"] if lr is None else lr
            for key, s, e in st.segments(g):
                n = self.steps.get(key, 0) + 1
                self.steps[key] = n
                sh = None if st.bf16[g] is None else st.bf16[g][s:e]
                ops.adamw(st.master[g][s:e], st.grad[g][s:e], self.m[g][s:e], self.v[g][s:e], sh, glr,
                          pg["weight_decay"], self.betas[0], self.betas[1], self.eps, n)
        st.written_optional.clear()
        ops.FP8.weights_changed()  # fp8 weight copies are re-quantised on their next use
        ops.WT.weights_changed()   # and the K-major dX copies re-transposed (ops.WeightT),
        ops.WT.refresh_async()     # now, on a side stream under the next forward

    def zero_grad(self, set_to_none=False):
        # capk backward passes overwrite every gradient they produce (no accumulation
        # across backward calls); nothing to clear.
        self.store.relink_grads()

    # ------------------------------------------------------------ checkpoints --
    def _step_key(self, p):
        g, off = self.store.offsets[id(p)]
        return (g, off) if id(p) in self.store.optional else (g, "required")

    def _order(self):
        return _reference_param_order(self.store.named)

    def state_dict(self):
        """torch.optim.AdamW.state_dict() layout (tensors copied to the CPU)."""
        dec, nod = self._order()
        state, groups, idx = {}, [], 0
        for plist, pg in ((dec, self.param_groups[0]), (nod, self.param_groups[1])):
            ids = []
            for _, p in plist:
                n = self.steps.get(self._step_key(p), 0)
                if n > 0:  # torch creates per-parameter state at its first step
                    state[idx] = {"step": torch.tensor(float(n)),
                                  "exp_avg": self.store.param_view(p, self.m).detach().cpu().clone(),
                                  "exp_avg_sq": self.store.param_view(p, self.v).detach().cpu().clone()}
                ids.append(idx)
                idx += 1
            groups.append({"weight_decay": pg["weight_decay"], "lr": pg["lr"], "betas": tuple(self.betas),
                           "eps": self.eps, "amsgrad": False, "maximize": False, "foreach": None,
                           "capturable": False, "differentiable": False, "fused": None,
                           "decoupled_weight_decay": True, "initial_lr": pg.get("initial_lr", pg["lr"]),
                           "params": ids})
        return {"state": state, "param_groups": groups}

    def load_state_dict(self, sd):
        """Load a torch.optim.AdamW state dict (written by the reference trainer or by
        ``state_dict``).  capk keeps one step count per contiguous update range, so the
        required parameters of a group must share their step count (true for any
        checkpoint of the reference's training loop)."""
        dec, nod = self._order()
        groups = sd["param_groups"]
        if len(groups) != 2 or len(groups[0]["params"]) != len(dec) or len(groups[1]["params"]) != len(nod):
            raise ValueError("optimizer state dict does not match this model's parameter groups "
                             f"({[len(g['params']) for g in groups]} vs {[len(dec), len(nod)]})")
        state = sd["state"]
        steps = {}
        for plist, pg, mine in ((dec, groups[0], self.param_groups[0]), (nod, groups[1], self.param_groups[1])):
            for (_, p), i in zip(plist, pg["params"]):
                s = state.get(i, state.get(str(i)))
                key = self._step_key(p)
                n = 0 if s is None else int(float(s["step"]))
                if key in steps and steps[key] != n:
                    raise ValueError(f"parameter {self.store.names[id(p)]}: step {n} differs from its range's "
                                     f"{steps[key]} (capk keeps one AdamW step count per range)")
                steps[key] = n
                with torch.no_grad():
                    mv, vv = self.store.param_view(p, self.m), self.store.param_view(p, self.v)
                    if s is None:
                        mv.zero_()
                        vv.zero_()
                    else:
                        mv.copy_(s["exp_avg"].to(mv.device, mv.dtype))
                        vv.copy_(s["exp_avg_sq"].to(vv.device, vv.dtype))
            mine["lr"] = pg["lr"]
            mine["weight_decay"] = pg["weight_decay"]
            mine["initial_lr"] = pg.get("initial_lr", pg["lr"])
            self.betas = tuple(pg["betas"])
            self.eps = pg["eps"]
        self.steps = {k: n for k, n in steps.items() if n > 0}


class LambdaSchedule:
    """torch.optim.lr_scheduler.LambdaLR over CapkAdamW (state_dict layout identical, so
    the reference's HF cosine / linear warmup schedulers round-trip through checkpoints)."""

    def __init__(self, optimizer, lr_lambda):
        self.optimizer = optimizer
        self.lr_lambda = lr_lambda
        self.base_lrs = [pg.get("initial_lr", pg["lr"]) for pg in optimizer.param_groups]
        for pg, b in zip(optimizer.param_groups, self.base_lrs):
            pg["initial_lr"] = b
        self.last_epoch = 0
        self._step_count = 1
        self._apply()

    def _apply(self):
        for pg, b in zip(self.optimizer.param_groups, self.base_lrs):
            pg["lr"] = b * self.lr_lambda(self.last_epoch)
        self._last_lr = [pg["lr"] for pg in self.optimizer.param_groups]

    def step(self):
        self._step_count += 1
        self.last_epoch += 1
        self._apply()

    def get_last_lr(self):
        return list(self._last_lr)

    def state_dict(self):
        return {"base_lrs": list(self.base_lrs), "last_epoch": self.last_epoch, "_step_count": self._step_count,
                "_is_initial": False, "_get_lr_called_within_step": False, "_last_lr": list(self._last_lr),
                "lr_lambdas": [{} for _ in self.base_lrs]}

    def load_state_dict(self, sd):
        self.base_lrs = list(sd["base_lrs"])
        self.last_epoch = int(sd["last_epoch"])
        self._step_count = int(sd.get("_step_count", self.last_epoch + 1))
        self._apply()


class StepSchedule(LambdaSchedule):
    """torch StepLR(step_size, gamma) — the reference's fallback scheduler (trainer.py:154-160)."""

    def __init__(self, optimizer, step_size, gamma=0.1):
        self.step_size, self.gamma = max(1, int(step_size)), gamma
        super().__init__(optimizer, lambda e: self.gamma ** (e // self.step_size))

    def state_dict(self):
        sd = super().state_dict()
        del sd["lr_lambdas"]
        sd.update(step_size=self.step_size, gamma=self.gamma)
        return sd


def build_scheduler(kind, optimizer, warmup, total):
    """trainer.py:136-162."""
    if kind == "linear":
        return LambdaSchedule(optimizer, lambda s: linear_schedule_with_warmup(s, 1.0, warmup, total))
    if kind == "cosine":
        return LambdaSchedule(optimizer, lambda s: cosine_schedule_with_warmup(s, 1.0, warmup, total))
    return StepSchedule(optimizer, total // 3, 0.1)
