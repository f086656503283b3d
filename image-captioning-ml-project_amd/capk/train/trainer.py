"""CaptioningTrainer on capk — mirrors src/train/trainer.py:22-620.

Same loop structure and state as the reference trainer, with the compute on libcapk:

* ``train_step``      — one batch of ``_train_epoch`` (trainer.py:218-289): forward, shifted
  CE, backward, (DP: bucketed gradient all-reduce overlapped with the backward), AdamW,
  ``scheduler.step()``.  bf16 storage / fp32 master weights replace fp16 autocast +
  GradScaler (bf16 has fp32's exponent range: no loss scaling, no inf checks).
* ``rl_step``         — one batch of ``_train_reinforcement_learning`` (trainer.py:340-381)
  with the SURVEY D8/D9 fixes (capk.train.scst).
* ``validate``        — ``_validate_epoch`` (trainer.py:486-567): CE on the first caption
  of each image + captions from ``model.generate`` scored with CIDEr-D.
* ``save_checkpoint`` / ``load_checkpoint`` — trainer.py:569-620, the reference's layout
  ``{epoch, model_state_dict, optimizer_state_dict, scheduler_state_dict, config,
  best_val_score}`` with torch-AdamW / LambdaLR state dicts, written by rank 0 only
  under DP.  ``config`` is stored as a plain dict; reference checkpoints (which pickle the
  dataclass) load through ``load_checkpoint_file``'s weights-only class mapping.
"""
import logging
from pathlib import Path

import torch
import torch.distributed as dist

from .. import prepare
from ..config import Config, _serialize
from .dp import GradBucketer
from .losses import CombinedLoss
from .optim import CapkAdamW, build_scheduler
from .scst import scst_step, strip_special

log = logging.getLogger("capk.trainer")


_REF_CONFIG_CLASSES = ("EncoderType", "DecoderType", "AttentionType", "EncoderConfig", "DecoderConfig",
                       "AttentionConfig", "TrainingConfig", "InferenceConfig", "ModelConfig", "Config")


def _set_epoch(loader, tag):
    """Tag the loader's sampler (capk.data.EpochSampler / DistributedSampler) with an explicit
    pass number, so a pass's permutation and augmentations are a function of the training epoch
    (and a resumed run repeats nothing) instead of the count of earlier iterations."""
    sampler = getattr(loader, "sampler", None)
    if sampler is not None and hasattr(sampler, "set_epoch"):
        sampler.set_epoch(tag)


def load_checkpoint_file(path, map_location="cpu"):
    """torch.load(weights_only=True) of a checkpoint written by this trainer or by the
    reference trainer (trainer.py:578-585, which pickles its ``src.config.Config`` dataclass
    and Enums).  Nothing from the file is executed: only those ten class names are
    allowlisted, each mapped to capk.config's class of the same name and fields, so the
    reference's config comes back as a capk Config."""
    from .. import config as C
    safe = [(getattr(C, n), f"src.config.{n}") for n in _REF_CONFIG_CLASSES]
    with torch.serialization.safe_globals(safe):
        return torch.load(path, map_location=map_location, weights_only=True)


def _rank():
    return dist.get_rank() if dist.is_available() and dist.is_initialized() else 0


class CaptioningTrainer:
    def __init__(self, config: Config, model, train_loader=None, val_loader=None, tokenizer=None, device=None,
                 precision="bf16", total_steps=None):
        self.config = config
        self.model = model
        self.train_loader = train_loader
        self.val_loader = val_loader
        self.tokenizer = tokenizer
        self.device = torch.device(device or config.device)
        self.store = prepare(model, self.device, precision)
        tc = config.training
        self.optimizer = CapkAdamW(self.store, lr=tc.learning_rate, weight_decay=tc.weight_decay)
        if total_steps is None:  # trainer.py:139
            total_steps = (len(train_loader) if train_loader is not None else 1) * tc.num_epochs
        self.total_steps = int(total_steps)
        self.scheduler = build_scheduler(tc.lr_scheduler, self.optimizer, tc.warmup_steps, self.total_steps)
        dec = model.decoder
        self.loss_fn = CombinedLoss(dec.pad_token_id)
        dp = dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1
        # bf16 wire format (fp32 master kept) except on the fp32 parity path
        # fp32 gradient average (the reduction the reference's DDP-free trainer would need to
        # match); 442 MB -> 884 MB per step on xGMI, overlapped with the backward
        self.bucketer = GradBucketer(self.store, exchange="fp32") if dp else None
        self.output_dir = Path(config.output_dir)
        self.checkpoint_dir = Path(config.checkpoint_dir)
        self.best_val_score = 0.0
        self.global_step = 0
        self.rl_updates = 0

    # ------------------------------------------------------------------ CE -----
    def train_step(self, images, captions):
        """trainer.py:223-286 for one batch; returns the loss as a device tensor (no host sync)."""
        self.optimizer.zero_grad()
        out = self.model(images=images, captions=captions, caption_lengths=None)
        loss = self.loss_fn(logits=out["logits"], targets=captions)["total_loss"]
        loss.backward()
        if self.bucketer is not None:
            self.bucketer.finish()
        self.optimizer.step()
        self.scheduler.step()
        self.global_step += 1
        return loss.detach()

    def train_epoch(self, epoch, loader=None):
        """_train_epoch (trainer.py:200-317): mean CE over the loader, then SCST when enabled."""
        loader = loader or self.train_loader
        _set_epoch(loader, 2 * epoch)  # crop / flip draws and the permutation follow the training epoch
        self.model.train()
        total, n = None, 0
        for i, batch in enumerate(loader):
            images = batch["image"].to(self.device, non_blocking=True)
            caps = batch["caption_tokens"].to(self.device, non_blocking=True)
            loss = self.train_step(images, caps)
            total = loss if total is None else total + loss
            n += 1
            if (i + 1) % self.config.log_every == 0:
                log.info(f"Epoch {epoch + 1}, Batch {i + 1}, Loss: {float(loss):.4f}, "
                         f"LR: {self.scheduler.get_last_lr()[0]:.6f}")
        avg = float(total) / max(n, 1) if total is not None else 0.0
        tc = self.config.training
        if tc.use_rl and epoch >= tc.rl_start_epoch:  # trainer.py:314-315
            self.rl_epoch(epoch, loader)
        return avg

    # ---------------------------------------------------------------- SCST -----
    def _baseline_kwargs(self):
        # trainer.py:353-356 -> model.generate: greedy for LSTM/Transformer, and
        # GPT2Decoder.generate's fixed num_beams=4 (decoders.py:645-654)
        from ..models.decoders import GPT2Decoder
        return {"num_beams": 4} if isinstance(self.model.decoder, GPT2Decoder) else {}

    def rl_step(self, images, references):
        """One SCST update.  references: per image, a list of token-id lists."""
        self.optimizer.zero_grad()
        loss, rs, rb = scst_step(self.model, images, references, self.optimizer, lr=None,
                                 seed=0x5C57 + self.rl_updates, max_length=self.config.inference.max_length,
                                 baseline_kwargs=self._baseline_kwargs(), bucketer=self.bucketer)
        self.scheduler.step()
        self.rl_updates += 1
        self.global_step += 1
        return loss, rs, rb

    def rl_epoch(self, epoch, loader):
        _set_epoch(loader, 2 * epoch + 1)  # the SCST pass of an epoch draws its own permutation
        self.model.train()
        dec = self.model.decoder
        for batch in loader:
            images = batch["image"].to(self.device, non_blocking=True)
            refs = batch.get("references")
            if refs is None:  # trainer.py:363-364: the batch's own caption is the reference
                refs = [[strip_special(c, dec.eos_token_id, dec.pad_token_id, dec.bos_token_id)]
                        for c in batch["caption_tokens"].tolist()]
            self.rl_step(images, refs)

    # ----------------------------------------------------------- validation ----
    @torch.no_grad()
    def validate(self, loader=None):
        """_validate_epoch (trainer.py:486-567): CE on caption 0 + CIDEr-D of generate()."""
        from ..cider import cider_d
        loader = loader or self.val_loader
        self.model.eval()
        dec = self.model.decoder
        losses, cands, refs = [], [], []
        for batch in loader:
            images = batch["image"].to(self.device, non_blocking=True)
            caps = batch["caption_tokens"].to(self.device, non_blocking=True)
            first = caps[:, 0, :] if caps.dim() == 3 else caps
            out = self.model(images=images, captions=first, caption_lengths=None)
            losses.append(self.loss_fn(logits=out["logits"], targets=first)["total_loss"].float())
            ids, _ = self.model.generate(images=images, max_length=self.config.inference.max_length)
            cands += [strip_special(r, dec.eos_token_id, dec.pad_token_id, dec.bos_token_id) for r in ids.tolist()]
            all_caps = caps if caps.dim() == 3 else caps[:, None, :]
            nref = batch.get("num_references")
            nref = nref.tolist() if nref is not None else [all_caps.shape[1]] * all_caps.shape[0]
            refs += [[strip_special(c, dec.eos_token_id, dec.pad_token_id, dec.bos_token_id) for c in img[:n]]
                     for img, n in zip(all_caps.tolist(), nref)]
        self.model.train()
        val_loss = float(torch.stack(losses).mean()) if losses else 0.0
        cider = float(cider_d(cands, refs).mean()) if cands else 0.0
        return val_loss, {"CIDEr": cider}

    # ---------------------------------------------------------- checkpoints ----
    def checkpoint(self, epoch):
        return {"epoch": epoch,
                "model_state_dict": {k: v.detach().cpu() for k, v in self.model.state_dict().items()},
                "optimizer_state_dict": self.optimizer.state_dict(),
                "scheduler_state_dict": self.scheduler.state_dict(),
                "config": _serialize(self.config),
                "best_val_score": self.best_val_score,
                "rl_updates": self.rl_updates}

    def save_checkpoint(self, epoch, is_best=False, path=None):
        """trainer.py:569-598; rank 0 writes (every rank holds identical weights under DP)."""
        if _rank() != 0:
            return None
        ck = self.checkpoint(epoch)
        self.checkpoint_dir.mkdir(parents=True, exist_ok=True)
        path = Path(path) if path else self.checkpoint_dir / f"checkpoint_epoch_{epoch + 1}.pth"
        torch.save(ck, path)
        if is_best:
            torch.save(ck, self.checkpoint_dir / "best_model.pth")
        return path

    def load_checkpoint(self, path):
        """trainer.py:600-620 -- a checkpoint of this trainer or of the reference trainer
        (load_checkpoint_file: weights_only=True, src.config classes mapped)."""
        ck = load_checkpoint_file(path)
        self.load_state(ck)
        return ck

    def load_state(self, ck):
        missing, unexpected = self.model.load_state_dict(ck["model_state_dict"], strict=True)
        self.store.refresh_shadow()
        self.optimizer.load_state_dict(ck["optimizer_state_dict"])
        if ck.get("scheduler_state_dict") is not None:
            self.scheduler.load_state_dict(ck["scheduler_state_dict"])
        self.best_val_score = ck.get("best_val_score", 0.0)
        self.global_step = int(self.scheduler.last_epoch)
        # SCST sampler seeds continue where the run stopped (reference checkpoints: none ran)
        self.rl_updates = int(ck.get("rl_updates", 0))

    # --------------------------------------------------------------- epochs ----
    def train(self):
        """trainer.py:164-198."""
        for epoch in range(self.config.training.num_epochs):
            train_loss = self.train_epoch(epoch)
            val_loss, metrics = self.validate() if self.val_loader is not None else (0.0, {"CIDEr": 0.0})
            log.info(f"Epoch {epoch + 1}: Train Loss: {train_loss:.4f}, Val Loss: {val_loss:.4f}, "
                     f"Val CIDEr: {metrics['CIDEr']:.4f}")
            if metrics["CIDEr"] > self.best_val_score:
                self.best_val_score = metrics["CIDEr"]
                self.save_checkpoint(epoch, is_best=True)
            if (epoch + 1) % self.config.save_every == 0:
                self.save_checkpoint(epoch)
