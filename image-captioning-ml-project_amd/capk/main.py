"""capk command line — the reference's CLI flag surface (src/main.py:17-130) on libcapk.

    python -m capk.main --mode train --encoder_type vit --decoder_type transformer \\
        --attention_type multi_head --batch_size 256 --steps 100

Every reference flag is kept with its name, choices and meaning (src/main.py:23-63);
``_update_config_from_args`` (src/main.py:105-130) is restated with the SURVEY fixes:

* D2  — assigning a flag string to an Enum field coerces it (capk.config), so
        ``--encoder_type vit`` reaches the factories as EncoderType.VIT;
* D17 — ``--encoder_type`` / ``--decoder_type`` change the family but the reference keeps
        ``pretrained_model_name`` (a ViT name under ``--encoder_type resnet`` makes its
        ResNetModel.from_pretrained load the wrong checkpoint): when the configured name
        is not an architecture of the selected family, the family's reference default
        is used (encoders.py:42-44,191-193; decoders.py:511-513).

Offline additions (no COCO download, no tokenizer download in this environment):
``--steps N`` runs N train (or eval) batches on synthetic 224x224 images and
20-token captions when no COCO annotations exist under ``--data_root`` (0 = build
the model and stop); ``--precision`` picks the bf16 throughput or fp32 parity
kernels; ``--seed``.  Without a tokenizer the GPT-2 vocabulary layout of
src/main.py:160-168 is used (50257 ids, pad = bos = eos = 50256).
"""
import argparse
import logging
import os
import sys

import torch

from .config import EncoderType, DecoderType, get_default_config, load_config, save_config

log = logging.getLogger("capk.main")

GPT2_VOCAB, GPT2_EOS = 50257, 50256


def build_parser():
    """src/main.py:19-63 (same flags, choices and defaults) + the offline extras."""
    p = argparse.ArgumentParser(description="Image Captioning with Transformers (capk, MI355X)")
    p.add_argument("--mode", type=str, default="train", choices=["train", "eval", "demo"])
    p.add_argument("--config", type=str, default=None)
    p.add_argument("--save_config", type=str, default=None)
    p.add_argument("--checkpoint", type=str, default=None)
    p.add_argument("--output_dir", type=str, default=None)
    p.add_argument("--batch_size", type=int, default=None)
    p.add_argument("--num_epochs", type=int, default=None)
    p.add_argument("--learning_rate", type=float, default=None)
    p.add_argument("--encoder_type", type=str, default=None, choices=["resnet", "vit", "swin", "clip"])
    p.add_argument("--decoder_type", type=str, default=None, choices=["lstm", "transformer", "gpt2"])
    p.add_argument("--attention_type", type=str, default=None, choices=["soft", "multi_head", "adaptive", "aoa"])
    p.add_argument("--use_rl", action="store_true")
    p.add_argument("--data_root", type=str, default=None)
    p.add_argument("--image_path", type=str, default=None)
    # offline extras
    p.add_argument("--steps", type=int, default=None,
                   help="synthetic batches to run (train: CE steps; eval: generate); 0 = build only")
    p.add_argument("--precision", type=str, default="bf16", choices=["bf16", "fp32", "fp8"])
    p.add_argument("--seed", type=int, default=None)
    return p


_FAMILY_DEFAULT_ENCODER = {EncoderType.VIT: "google/vit-base-patch16-224", EncoderType.RESNET: "microsoft/resnet-50",
                           EncoderType.CLIP: "openai/clip-vit-base-patch32",
                           EncoderType.SWIN: "microsoft/swin-base-patch4-window7-224"}


def _known_encoder_archs(et):
    from .models.clip import CLIP_ARCHS
    from .models.resnet import RESNET_ARCHS
    from .models.swin import SWIN_ARCHS
    from .models.vit import VIT_ARCHS
    return {EncoderType.VIT: VIT_ARCHS, EncoderType.RESNET: RESNET_ARCHS, EncoderType.CLIP: CLIP_ARCHS,
            EncoderType.SWIN: SWIN_ARCHS}.get(et, {})


def update_config_from_args(config, args):
    """src/main.py:105-130 (+ D17 family defaults)."""
    if args.output_dir:
        config.output_dir = args.output_dir
        config.checkpoint_dir = os.path.join(args.output_dir, "checkpoints")
    if args.batch_size:
        config.training.batch_size = args.batch_size
    if args.num_epochs:
        config.training.num_epochs = args.num_epochs
    if args.learning_rate:
        config.training.learning_rate = args.learning_rate
    if args.encoder_type:
        config.model.encoder.encoder_type = args.encoder_type  # D2: coerced to EncoderType on assignment
        et = config.model.encoder.encoder_type
        if et in _FAMILY_DEFAULT_ENCODER and config.model.encoder.pretrained_model_name not in _known_encoder_archs(et):
            config.model.encoder.pretrained_model_name = _FAMILY_DEFAULT_ENCODER[et]
    if args.decoder_type:
        config.model.decoder.decoder_type = args.decoder_type
        if config.model.decoder.decoder_type == DecoderType.GPT2 and not config.model.decoder.pretrained_model_name:
            config.model.decoder.pretrained_model_name = "gpt2"
    if args.attention_type:
        config.model.attention.attention_type = args.attention_type
    if args.use_rl:
        config.training.use_rl = True
    if args.data_root:
        config.data_root = args.data_root
    if args.seed is not None:
        config.seed = args.seed
    return config


def apply_tokenizer(config, tokenizer=None):
    """src/main.py:160-168: vocabulary and special ids from the tokenizer (pad := eos when
    unset); without one, the GPT-2 tokenizer's layout."""
    if tokenizer is not None:
        if getattr(tokenizer, "pad_token", None) is None:
            tokenizer.pad_token = tokenizer.eos_token
        config.model.vocab_size = len(tokenizer)
        config.model.pad_token_id = tokenizer.pad_token_id
        config.model.bos_token_id = getattr(tokenizer, "bos_token_id", None) or tokenizer.cls_token_id
        config.model.eos_token_id = tokenizer.eos_token_id
    else:
        config.model.vocab_size = GPT2_VOCAB
        config.model.pad_token_id = config.model.bos_token_id = config.model.eos_token_id = GPT2_EOS
    return config


class SyntheticCaptionLoader:
    """Synthetic batches of the benchmark's shape: randn 224x224x3 images and
    uniform caption ids without pad tokens, generated on the device (no host traffic)."""

    def __init__(self, batch, steps, vocab, pad, device, image_size=224, seq_len=20, seed=0, refs_per_image=0):
        self.batch, self.steps, self.vocab, self.pad = batch, steps, vocab, pad
        self.device, self.image_size, self.seq_len, self.seed = device, image_size, seq_len, seed
        self.refs_per_image = refs_per_image

    def __len__(self):
        return self.steps

    def __iter__(self):
        g = torch.Generator(device=self.device).manual_seed(self.seed)
        hi = self.pad if 0 <= self.pad < self.vocab else self.vocab
        for _ in range(self.steps):
            images = torch.randn(self.batch, 3, self.image_size, self.image_size, device=self.device, generator=g)
            shape = (self.batch, self.refs_per_image, self.seq_len) if self.refs_per_image else (self.batch,
                                                                                               self.seq_len)
            caps = torch.randint(0, hi, shape, device=self.device, generator=g)
            yield {"image": images, "caption_tokens": caps}


def build_model(config, tokenizer=None):
    from .models.captioning_model import ImageCaptioningModel
    torch.manual_seed(config.seed)
    return ImageCaptioningModel(config, tokenizer)


def _loaders(config, args, device, tokenizer):
    """COCO loaders when annotations exist under data_root (src/main.py:170-177), else synthetic."""
    ann = os.path.join(config.data_root, config.train_json)
    if os.path.exists(ann) and tokenizer is not None:
        from .data import build_coco_dataloaders
        train_loader, val_loader, _ = build_coco_dataloaders(config, tokenizer)
        return train_loader, val_loader
    steps = args.steps if args.steps is not None else 10
    m = config.model
    train = SyntheticCaptionLoader(config.training.batch_size, steps, m.vocab_size, m.pad_token_id, device,
                                   config.image_size, seed=config.seed)
    val = SyntheticCaptionLoader(config.training.batch_size, max(1, min(steps, 2)), m.vocab_size, m.pad_token_id,
                                 device, config.image_size, seed=config.seed + 1, refs_per_image=5)
    return train, val


def main(argv=None, tokenizer=None):
    """src/main.py:17-102.  Returns (config, model, trainer-or-None)."""
    parser = build_parser()
    args = parser.parse_args(argv)
    config = load_config(args.config) if args.config else get_default_config()
    apply_tokenizer(config, tokenizer)
    update_config_from_args(config, args)
    if args.save_config:
        save_config(config, args.save_config)
    logging.basicConfig(format="%(asctime)s - %(levelname)s - %(message)s", datefmt="%m/%d/%Y %H:%M:%S",
                        level=logging.INFO)
    model = build_model(config, tokenizer)
    if args.steps == 0:
        return config, model, None
    if not torch.cuda.is_available():
        raise RuntimeError("capk runs on an MI355X GPU (no CPU path); use --steps 0 to only build the model")
    from .train.trainer import CaptioningTrainer
    device = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")))
    torch.cuda.set_device(device)
    train_loader, val_loader = _loaders(config, args, device, tokenizer)
    trainer = CaptioningTrainer(config, model, train_loader, val_loader, tokenizer, device, precision=args.precision)
    if args.checkpoint:
        trainer.load_checkpoint(args.checkpoint)
    if args.mode == "train":
        if args.steps is not None:
            # synthetic run: one epoch of `steps` CE batches (+ SCST over the same batches with --use_rl)
            loss = trainer.train_epoch(epoch=config.training.rl_start_epoch if config.training.use_rl else 0)
            log.info(f"train: {args.steps} steps, mean loss {loss:.4f}")
        else:
            trainer.train()
    elif args.mode == "eval":
        val_loss, metrics = trainer.validate()
        log.info(f"eval: loss {val_loss:.4f}, CIDEr-D {metrics['CIDEr']:.4f}")
    else:  # demo (src/main.py:270-343) — caption ids for one image
        if not args.image_path:
            parser.error("--image_path is required for demo mode")
        from .data import load_image
        img = load_image(args.image_path, config.image_size).to(device)[None]
        model.eval()
        with torch.no_grad():
            ids, _ = model.generate(images=img, max_length=config.inference.max_length)
        text = tokenizer.decode(ids[0], skip_special_tokens=True) if tokenizer is not None else ids[0].tolist()
        log.info(f"Generated caption: {text}")
    return config, model, trainer


if __name__ == "__main__":
    main(sys.argv[1:])
