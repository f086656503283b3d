"""Checkpoints and frozen parameters on the GPU:
* a torch.optim.AdamW + HF cosine-schedule checkpoint of the reference's optimizer
  (trainer.py:111-162) loads into CapkAdamW and the next capk step equals torch's next
  step (fp32 kernels, rtol 1e-6);
* CaptioningTrainer.save_checkpoint -> load_checkpoint resumes bit-identically;
* EncoderConfig.freeze: the frozen encoder's weights stay bit-identical through a step
  (the reference's AdamW never sees them, trainer.py:117-126)."""
import pytest
import torch

from test_checkpoint import reference_optimizer, tiny_model, torch_checkpoint

pytestmark = pytest.mark.gpu
cuda = pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a GPU")


@cuda
def test_resume_torch_adamw_checkpoint_and_continue():
    import capk
    from capk.train.optim import CapkAdamW, build_scheduler
    model, cfg, opt, sch = torch_checkpoint(steps=2)
    capk_model, _ = tiny_model()
    capk_model.load_state_dict(model.state_dict())
    store = capk.prepare(capk_model, "cuda", "fp32")
    copt = CapkAdamW(store, lr=5e-5, weight_decay=0.01)
    csch = build_scheduler("cosine", copt, 3, 20)
    copt.load_state_dict(opt.state_dict())
    csch.load_state_dict(sch.state_dict())
    # third step, same gradients on both sides
    g = torch.Generator().manual_seed(7)
    named = dict(capk_model.named_parameters())
    for n, p in model.named_parameters():
        if "pooler" in n:
            p.grad = None
            continue
        p.grad = torch.randn(p.shape, generator=g)
        named[n]._capk_grad.copy_(p.grad)
    opt.step()
    sch.step()
    copt.step()
    csch.step()
    torch.cuda.synchronize()
    for n, p in model.named_parameters():
        torch.testing.assert_close(named[n].detach().cpu(), p.detach(), rtol=1e-6, atol=1e-9, msg=n)
    assert csch.get_last_lr() == sch.get_last_lr()


def _batch(B=3, T=9, V=70, pad=69, seed=3):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(B, 3, 32, 32, generator=g).cuda(), torch.randint(0, pad, (B, T), generator=g).cuda()


@cuda
def test_trainer_save_load_resumes_bit_identically(tmp_path):
    from capk.train.trainer import CaptioningTrainer
    images, caps = _batch()
    m1, cfg = tiny_model()
    cfg.checkpoint_dir = str(tmp_path)
    cfg.training.warmup_steps = 2
    t1 = CaptioningTrainer(cfg, m1, device="cuda", precision="fp32", total_steps=10)
    m1.eval()  # dropout off: the comparison is of the optimizer / checkpoint path
    t1.train_step(images, caps)
    path = t1.save_checkpoint(epoch=0)
    m2, _ = tiny_model()
    t2 = CaptioningTrainer(cfg, m2, device="cuda", precision="fp32", total_steps=10)
    m2.eval()
    t2.load_checkpoint(path)
    for t in (t1, t2):
        for _ in range(2):
            t.train_step(images, caps)
    torch.cuda.synchronize()
    for (n, a), (_, b) in zip(m1.state_dict().items(), m2.state_dict().items()):
        assert torch.equal(a, b), n
    assert t1.scheduler.get_last_lr() == t2.scheduler.get_last_lr()
    ck = torch.load(path, weights_only=True)
    assert set(ck) == {"epoch", "model_state_dict", "optimizer_state_dict", "scheduler_state_dict", "config",
                       "best_val_score", "rl_updates"}


@cuda
def test_frozen_encoder_weights_unchanged_by_step():
    import capk
    from capk.train import CapkAdamW, CombinedLoss
    model, cfg = tiny_model(freeze=True)
    store = capk.prepare(model, "cuda", "fp32")
    before = {n: p.detach().clone() for n, p in model.encoder.named_parameters()}
    dec_before = {n: p.detach().clone() for n, p in model.decoder.named_parameters()}
    opt = CapkAdamW(store, lr=1e-2, weight_decay=0.1)
    images, caps = _batch()
    model.eval()
    out = model(images=images, captions=caps)
    CombinedLoss(69)(out["logits"], caps)["total_loss"].backward()
    opt.step()
    torch.cuda.synchronize()
    for n, p in model.encoder.named_parameters():
        assert torch.equal(p.detach(), before[n]), n
    moved = [n for n, p in model.decoder.named_parameters() if not torch.equal(p.detach(), dec_before[n])]
    assert len(moved) > 5
