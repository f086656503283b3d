"""Checkpoint format (src/train/trainer.py:569-620): capk's optimizer and
scheduler state dicts are torch.optim.AdamW's and LambdaLR's, numbered the way the
reference's _create_optimizer numbers parameters (trainer.py:111-134), so a checkpoint
written by the reference loads into capk and capk's own state dict reproduces it bit for
bit.  CPU only (ParamStore on the CPU; the GPU continuation is tests/test_gpu_checkpoint.py)."""
import pytest
import torch
from transformers import get_cosine_schedule_with_warmup

from capk import config as C
from capk.params import attach
from capk.train.optim import CapkAdamW, LambdaSchedule, build_scheduler, cosine_schedule_with_warmup


def tiny_model(freeze=False):
    from capk.models import captioning_model as cm
    from capk.models import encoders as E
    cfg = C.Config()
    cfg.model.encoder = C.EncoderConfig(encoder_type="vit", feature_dim=64, freeze=freeze)
    cfg.model.decoder = C.DecoderConfig(decoder_type="transformer", hidden_dim=64, num_layers=1, num_heads=2)
    cfg.model.vocab_size, cfg.model.pad_token_id = 70, 69
    arch = dict(hidden_size=64, num_hidden_layers=1, num_attention_heads=2, intermediate_size=128, image_size=32,
                patch_size=16, num_channels=3, layer_norm_eps=1e-12)
    orig = E.VIT_ARCHS["google/vit-base-patch16-224"]
    E.VIT_ARCHS["google/vit-base-patch16-224"] = arch
    try:
        torch.manual_seed(0)
        return cm.ImageCaptioningModel(cfg), cfg
    finally:
        E.VIT_ARCHS["google/vit-base-patch16-224"] = orig


def reference_optimizer(model, lr=5e-5, wd=0.01):
    """trainer.py:111-134 verbatim in structure."""
    nd = ["bias", "LayerNorm.weight"]
    with_wd = [p for n, p in model.named_parameters() if not any(x in n for x in nd) and p.requires_grad]
    without = [p for n, p in model.named_parameters() if any(x in n for x in nd) and p.requires_grad]
    return torch.optim.AdamW([{"params": with_wd, "weight_decay": wd}, {"params": without, "weight_decay": 0.0}],
                             lr=lr)


def torch_checkpoint(freeze=False, steps=2, skip_pooler=True):
    """Run the reference's optimizer + scheduler for `steps` steps on random gradients."""
    model, cfg = tiny_model(freeze)
    opt = reference_optimizer(model)
    sch = get_cosine_schedule_with_warmup(opt, num_warmup_steps=3, num_training_steps=20)
    g = torch.Generator().manual_seed(1)
    for _ in range(steps):
        for n, p in model.named_parameters():
            if not p.requires_grad or (skip_pooler and "pooler" in n):
                p.grad = None  # decoder ignores pooled features: torch AdamW skips the pooler
                continue
            p.grad = torch.randn(p.shape, generator=g)
        opt.step()
        sch.step()
    return model, cfg, opt, sch


def _assert_same(a, b, path="sd"):
    if isinstance(a, dict):
        assert set(a) == set(b), (path, set(a) ^ set(b))
        for k in a:
            _assert_same(a[k], b[k], f"{path}.{k}")
    elif isinstance(a, (list, tuple)):
        assert len(a) == len(b), path
        for i, (x, y) in enumerate(zip(a, b)):
            _assert_same(x, y, f"{path}[{i}]")
    elif torch.is_tensor(a):
        assert torch.equal(a, b.to(a.dtype)), path
    else:
        assert a == b, (path, a, b)


@pytest.mark.parametrize("freeze", [False, True])
def test_torch_adamw_checkpoint_round_trips_bit_identically(freeze):
    model, cfg, opt, sch = torch_checkpoint(freeze)
    sd, ssd = opt.state_dict(), sch.state_dict()
    # a fresh capk model holding the same weights
    capk_model, _ = tiny_model(freeze)
    capk_model.load_state_dict(model.state_dict())
    store = attach(capk_model, "cpu")
    copt = CapkAdamW(store, lr=5e-5, weight_decay=0.01)
    csch = build_scheduler("cosine", copt, 3, 20)
    copt.load_state_dict(sd)
    csch.load_state_dict(ssd)
    _assert_same(sd, copt.state_dict())
    _assert_same(ssd, csch.state_dict())
    assert copt.param_groups[0]["lr"] == opt.param_groups[0]["lr"]
    # the moments sit in the flat buffers at the parameters' places
    named = dict(capk_model.named_parameters())
    idx = 0
    for gi, group in enumerate(sd["param_groups"]):
        for i in group["params"]:
            st = sd["state"].get(i)
            if st is not None:
                p = [q for q in opt.param_groups[gi]["params"]][group["params"].index(i)]
                name = [n for n, q in model.named_parameters() if q is p][0]
                assert torch.equal(store.param_view(named[name], copt.m), st["exp_avg"]), name
            idx += 1
    if freeze:
        assert all(not p.requires_grad for p in capk_model.encoder.parameters())


def test_scheduler_matches_hf_lambda_lr():
    model, _ = tiny_model()
    opt = reference_optimizer(model, lr=1e-3)
    sch = get_cosine_schedule_with_warmup(opt, num_warmup_steps=5, num_training_steps=40)
    store = attach(tiny_model()[0], "cpu")
    copt = CapkAdamW(store, lr=1e-3)
    csch = LambdaSchedule(copt, lambda s: cosine_schedule_with_warmup(s, 1.0, 5, 40))
    for _ in range(45):
        assert csch.get_last_lr() == sch.get_last_lr()
        assert copt.param_groups[1]["lr"] == opt.param_groups[1]["lr"]
        sch.step()
        csch.step()
    _assert_same(sch.state_dict(), csch.state_dict())


def test_mismatched_state_dict_is_rejected():
    model, cfg, opt, sch = torch_checkpoint()
    other, _ = tiny_model(freeze=True)  # frozen encoder: different group sizes
    copt = CapkAdamW(attach(other, "cpu"))
    with pytest.raises(ValueError):
        copt.load_state_dict(opt.state_dict())


def test_reference_checkpoint_file_loads_weights_only(golden_dir):
    """A checkpoint in the reference trainer's layout, with the reference's own pickled
    src.config.Config (oracle/gen_ref_checkpoint.py), loads under weights_only=True: the ten
    src.config classes come back as capk.config's, nothing else is allowlisted."""
    import os
    import pickle

    from capk import config as C
    from capk.train.trainer import load_checkpoint_file
    path = os.path.join(golden_dir, "ref_checkpoint.pth")
    ck = load_checkpoint_file(path)
    cfg = ck["config"]
    assert isinstance(cfg, C.Config) and isinstance(cfg.model.encoder, C.EncoderConfig)
    assert cfg.model.encoder.encoder_type is C.EncoderType.CLIP
    assert cfg.model.decoder.decoder_type is C.DecoderType.LSTM
    assert cfg.model.attention.attention_type is C.AttentionType.AOA
    assert cfg.training.batch_size == 48 and ck["epoch"] == 2 and ck["best_val_score"] == 0.625
    assert set(ck["model_state_dict"]) == {"weight", "bias"}
    assert ck["optimizer_state_dict"]["state"][0]["step"] == 1
    with pytest.raises(pickle.UnpicklingError):  # the plain weights-only load refuses the file
        torch.load(path, weights_only=True)
