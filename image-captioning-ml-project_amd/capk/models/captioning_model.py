"""ImageCaptioningModel — mirrors src/models/captioning_model.py:13-150 (encoder ->
decoder glue; the optional QFormer is out of scope: use_q_former=False default)."""
import torch.nn as nn

from ..config import Config
from .decoders import build_decoder
from .encoders import build_encoder


class ImageCaptioningModel(nn.Module):
    def __init__(self, config: Config, tokenizer=None):
        super().__init__()
        self.config = config
        self.model_config = config.model
        self.encoder = build_encoder(config.model.encoder)
        if tokenizer:
            vocab_size = len(tokenizer)
            pad, bos, eos = tokenizer.pad_token_id, tokenizer.bos_token_id, tokenizer.eos_token_id
        else:
            m = config.model
            vocab_size, pad, bos, eos = m.vocab_size, m.pad_token_id, m.bos_token_id, m.eos_token_id
        self.decoder = build_decoder(config.model.decoder, config.model.attention, vocab_size, pad, bos, eos)
        if config.model.use_q_former:
            raise NotImplementedError("capk: QFormer is outside the hot path (SURVEY §2)")

    def forward(self, images, captions=None, caption_lengths=None, return_dict=True, **kwargs):
        """captioning_model.py:56-104."""
        encoder_features = self.encoder(images)
        out = self.decoder(encoder_features=encoder_features, captions=captions, caption_lengths=caption_lengths,
                           **kwargs)
        return out if return_dict else out["logits"]

    def generate(self, images, max_length=None, **kwargs):
        """captioning_model.py:106-150."""
        if max_length is None:
            max_length = self.config.inference.max_length
        encoder_features = self.encoder(images)
        return self.decoder.generate(encoder_features=encoder_features, max_length=max_length, **kwargs)
