"""Oracle restatement of the training-step arithmetic.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).
"""
import math

import torch
import torch.nn.functional as F


def shifted_ce(logits, targets, pad_token_id):
    """CombinedLoss.forward CE part (src/train/losses.py:236-247): shift
    logits[:, :-1] vs targets[:, 1:], CrossEntropyLoss(ignore_index=pad) = mean
    over non-pad target tokens."""
    V = logits.shape[-1]
    return F.cross_entropy(logits[:, :-1].reshape(-1, V), targets[:, 1:].reshape(-1),
                           ignore_index=pad_token_id)


def no_decay(name):
    """CaptioningTrainer._create_optimizer group rule (src/train/trainer.py:114-128):
    a parameter skips weight decay iff its name contains 'bias' or
    'LayerNorm.weight' (case-sensitive substring test, so transformers-5.15
    'layernorm_before.weight' and torch 'norm1.weight' DO get decay)."""
    return any(nd in name for nd in ("bias", "LayerNorm.weight"))


def cosine_warmup_lr(step, base_lr, warmup, total, num_cycles=0.5):
    """transformers.get_cosine_schedule_with_warmup lr_lambda (used by
    trainer.py:150-154): linear warmup then half-cosine to 0."""
    if step < warmup:
        return base_lr * float(step) / float(max(1, warmup))
    progress = float(step - warmup) / float(max(1, total - warmup))
    return base_lr * max(0.0, 0.5 * (1.0 + math.cos(math.pi * float(num_cycles) * 2.0 * progress)))


def adamw_step(param, grad, m, v, step, lr, wd, beta1=0.9, beta2=0.999, eps=1e-8):
    """torch.optim.AdamW single-tensor update (torch/optim/adamw.py, _single_tensor_adam
    with decoupled weight decay), betas (0.9, 0.999), eps 1e-8 (trainer.py:131-134).
    In-place on param/m/v; `step` is the 1-based step count after increment."""
    param.mul_(1.0 - lr * wd)
    m.lerp_(grad, 1.0 - beta1)
    v.mul_(beta2).addcmul_(grad, grad, value=1.0 - beta2)
    bc1 = 1.0 - beta1 ** step
    bc2 = 1.0 - beta2 ** step
    step_size = lr / bc1
    denom = (v.sqrt() / math.sqrt(bc2)).add_(eps)
    param.addcdiv_(m, denom, value=-step_size)
