"""The reference CLI flag surface (src/main.py:23-63, _update_config_from_args 105-130)
on capk: every --encoder_type x --decoder_type x --attention_type combination builds
through the plugin factories with the D2 (string -> Enum on assignment) and D17
(family-default architecture) fixes, and --save_config / --config round-trip.  CPU only
(--steps 0 builds the model and stops; no kernel runs)."""
import itertools
import json

import pytest

from capk import config as C
from capk.main import build_parser, main, update_config_from_args

ENC = ["resnet", "vit", "swin", "clip"]
DEC = ["lstm", "transformer", "gpt2"]
ATT = ["soft", "multi_head", "adaptive", "aoa"]


def test_parser_matches_reference_flags():
    p = build_parser()
    acts = {a.dest: a for a in p._actions}
    for flag in ("mode", "config", "save_config", "checkpoint", "output_dir", "batch_size", "num_epochs",
                 "learning_rate", "encoder_type", "decoder_type", "attention_type", "use_rl", "data_root",
                 "image_path"):
        assert flag in acts, flag
    assert acts["mode"].choices == ["train", "eval", "demo"] and acts["mode"].default == "train"
    assert acts["encoder_type"].choices == ENC
    assert acts["decoder_type"].choices == DEC
    assert acts["attention_type"].choices == ATT
    with pytest.raises(SystemExit):
        p.parse_args(["--encoder_type", "convnext"])


def test_update_config_assigns_strings_and_coerces():
    """D2: the reference assigns the flag strings after construction (main.py:119-124)."""
    args = build_parser().parse_args(["--encoder_type", "clip", "--decoder_type", "lstm", "--attention_type",
                                      "adaptive", "--batch_size", "7", "--learning_rate", "0.001", "--use_rl",
                                      "--output_dir", "/tmp/capk_o", "--num_epochs", "3"])
    cfg = update_config_from_args(C.get_default_config(), args)
    assert cfg.model.encoder.encoder_type is C.EncoderType.CLIP
    assert cfg.model.decoder.decoder_type is C.DecoderType.LSTM
    assert cfg.model.attention.attention_type is C.AttentionType.ADAPTIVE
    assert cfg.model.encoder.pretrained_model_name == "openai/clip-vit-base-patch32"  # D17
    assert cfg.training.batch_size == 7 and cfg.training.learning_rate == 0.001 and cfg.training.use_rl
    assert cfg.training.num_epochs == 3
    assert cfg.output_dir == "/tmp/capk_o" and cfg.checkpoint_dir == "/tmp/capk_o/checkpoints"


@pytest.mark.parametrize("enc,dec,att", list(itertools.product(ENC, DEC, ATT)))
def test_every_cli_combination_builds_and_round_trips(enc, dec, att, tmp_path):
    from capk.models.attention import AttentionOnAttention, AdaptiveAttention, MultiHeadAttention, SoftAttention
    from capk.models.decoders import GPT2Decoder, LSTMDecoder, TransformerDecoder
    from capk.models.encoders import CLIPEncoder, ResNetEncoder, SwinEncoder, ViTEncoder
    cfg_path = tmp_path / "cfg.json"
    argv = ["--encoder_type", enc, "--decoder_type", dec, "--attention_type", att, "--save_config", str(cfg_path),
            "--steps", "0"]
    cfg, model, trainer = main(argv)
    assert trainer is None
    assert isinstance(model.encoder, {"resnet": ResNetEncoder, "vit": ViTEncoder, "clip": CLIPEncoder,
                                      "swin": SwinEncoder}[enc])
    assert isinstance(model.decoder, {"lstm": LSTMDecoder, "transformer": TransformerDecoder,
                                      "gpt2": GPT2Decoder}[dec])
    if dec == "lstm":  # only the LSTM decoder builds an attention plugin
        want = {"soft": SoftAttention, "multi_head": MultiHeadAttention, "adaptive": AdaptiveAttention,
                "aoa": AttentionOnAttention}[att]
        assert isinstance(model.decoder.attention, want), type(model.decoder.attention)
    assert model.decoder.vocab_size == 50257 and model.decoder.pad_token_id == 50256
    saved = json.loads(cfg_path.read_text())
    assert saved["model"]["encoder"]["encoder_type"] == enc and saved["model"]["decoder"]["decoder_type"] == dec
    assert saved["model"]["attention"]["attention_type"] == att
    # --config round trip: the loaded config equals the saved one (Enums, nested dataclasses)
    args2 = build_parser().parse_args(["--config", str(cfg_path)])
    cfg2 = update_config_from_args(C.load_config(args2.config), args2)
    assert C._serialize(cfg2) == C._serialize(cfg)
    if att == "aoa":  # and it rebuilds the same model (state-dict names)
        _, model2, _ = main(["--config", str(cfg_path), "--steps", "0"])
        assert list(model2.state_dict()) == list(model.state_dict())
