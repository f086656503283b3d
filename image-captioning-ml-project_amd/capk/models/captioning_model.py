"""ImageCaptioningModel — mirrors src/models/captioning_model.py:13-150 (encoder ->
[QFormer] -> decoder glue)."""
import torch
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
        if config.model.use_q_former:  # captioning_model.py:49-54
            from .qformer import QFormer
            self.q_former = QFormer(query_dim=config.model.projection_dim,
                                    vision_dim=config.model.encoder.feature_dim,
                                    num_queries=config.model.q_former_num_queries)

    def _with_q_former(self, encoder_features):
        """captioning_model.py:79-91: the queries replace the features, all-ones mask."""
        if not hasattr(self, "q_former"):
            return encoder_features
        q = self.q_former(encoder_features["features"], encoder_features.get("attention_mask"))["queries"]
        out = dict(encoder_features)
        out["features"] = q
        out["attention_mask"] = torch.ones(q.shape[0], q.shape[1], device=q.device)
        return out

    def forward(self, images, captions=None, caption_lengths=None, return_dict=True, **kwargs):
        """captioning_model.py:56-104."""
        encoder_features = self._with_q_former(self.encoder(images))
        out = self.decoder(encoder_features=encoder_features, captions=captions, caption_lengths=caption_lengths,
                           **kwargs)
        return out if return_dict else out["logits"]

    def generate(self, images, max_length=None, **kwargs):
        """captioning_model.py:106-150."""
        if max_length is None:
            max_length = self.config.inference.max_length
        encoder_features = self._with_q_former(self.encoder(images))
        return self.decoder.generate(encoder_features=encoder_features, max_length=max_length, **kwargs)
