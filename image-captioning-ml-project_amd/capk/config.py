"""Configuration surface — mirrors src/config.py of the reference (same dataclasses,
field names, defaults and Enums) with the documented fixes of SURVEY §0.1:

* D2: string values coming from the CLI are coerced to the Enum members, both at
  construction (``EncoderConfig(encoder_type="vit")``) and on later assignment
  (``cfg.model.encoder.encoder_type = "vit"``, what src/main.py:119-124
  ``_update_config_from_args`` does); the reference stored the string and its
  factories, comparing 'vit' against EncoderType.VIT, raised ValueError.
* D13: ``save_config`` serialises nested Enums; ``load_config`` rebuilds the
  nested dataclasses and Enums (the reference left them as dicts).
* Mutable dataclass defaults use ``default_factory`` (the reference's
  ``ModelConfig()`` defaults only work on Python <= 3.10).
"""
import dataclasses
import json
from dataclasses import dataclass, field
from enum import Enum


class EncoderType(Enum):
    RESNET = "resnet"
    VIT = "vit"
    SWIN = "swin"
    CONVNEXT = "convnext"
    EFFICIENTNET = "efficientnet"
    CLIP = "clip"


class DecoderType(Enum):
    LSTM = "lstm"
    TRANSFORMER = "transformer"
    GPT2 = "gpt2"
    T5 = "t5"
    BART = "bart"


class AttentionType(Enum):
    SOFT = "soft"
    MULTI_HEAD = "multi_head"
    ADAPTIVE = "adaptive"
    AOA = "aoa"
    OBJECT = "object"


def _coerce(enum_cls, v):
    return v if isinstance(v, enum_cls) else enum_cls(v)


class _EnumFields:
    """Coerce the Enum-typed field on every assignment (D2), not only in __init__."""
    _ENUM_FIELDS = {}

    def __setattr__(self, name, value):
        cls = self._ENUM_FIELDS.get(name)
        super().__setattr__(name, _coerce(cls, value) if cls is not None else value)


@dataclass
class EncoderConfig(_EnumFields):
    _ENUM_FIELDS = {"encoder_type": EncoderType}

    encoder_type: EncoderType = EncoderType.VIT
    pretrained_model_name: str = "google/vit-base-patch16-224"
    freeze: bool = False
    feature_dim: int = 768
    use_object_features: bool = False



@dataclass
class DecoderConfig(_EnumFields):
    _ENUM_FIELDS = {"decoder_type": DecoderType}

    decoder_type: DecoderType = DecoderType.GPT2
    pretrained_model_name: str = "gpt2"
    hidden_dim: int = 768
    num_layers: int = 6
    num_heads: int = 8
    dropout: float = 0.1
    max_length: int = 50



@dataclass
class AttentionConfig(_EnumFields):
    _ENUM_FIELDS = {"attention_type": AttentionType}

    attention_type: AttentionType = AttentionType.MULTI_HEAD
    num_heads: int = 8
    temperature: float = 1.0
    use_geometric: bool = False
    # D3: the reference attention modules read config.hidden_dim, which the reference
    # AttentionConfig lacks; build_decoder fills it from DecoderConfig.hidden_dim.
    hidden_dim: int = 768



@dataclass
class TrainingConfig:
    batch_size: int = 64
    num_epochs: int = 15
    learning_rate: float = 5e-5
    weight_decay: float = 0.01
    lr_scheduler: str = "cosine"
    warmup_steps: int = 2000
    use_rl: bool = True
    rl_start_epoch: int = 10
    rl_reward: str = "cider"
    rl_weight: float = 1.0
    use_amp: bool = True
    use_curriculum: bool = False
    curriculum_strategy: str = "caption_length"
    use_contrastive_loss: bool = False
    use_itm_loss: bool = False
    use_obj_cls_loss: bool = False


@dataclass
class InferenceConfig:
    decoding_strategy: str = "beam"
    beam_size: int = 5
    top_p: float = 0.9
    temperature: float = 1.0
    min_length: int = 5
    max_length: int = 20
    length_penalty: float = 0.8
    num_beam_groups: int = 1
    diversity_penalty: float = 0.5
    use_clip_reranking: bool = False
    num_candidates: int = 5


@dataclass
class ModelConfig:
    encoder: EncoderConfig = field(default_factory=EncoderConfig)
    decoder: DecoderConfig = field(default_factory=DecoderConfig)
    attention: AttentionConfig = field(default_factory=AttentionConfig)
    projection_dim: int = 768
    use_q_former: bool = False
    q_former_num_queries: int = 32
    vocab_size: int = 50257
    pad_token_id: int = 0
    bos_token_id: int = 1
    eos_token_id: int = 2


@dataclass
class Config:
    model: ModelConfig = field(default_factory=ModelConfig)
    training: TrainingConfig = field(default_factory=TrainingConfig)
    inference: InferenceConfig = field(default_factory=InferenceConfig)
    data_root: str = "data"
    train_json: str = "annotations/captions_train2014.json"
    val_json: str = "annotations/captions_val2014.json"
    train_image_dir: str = "train2014"
    val_image_dir: str = "val2014"
    image_size: int = 224
    output_dir: str = "outputs"
    checkpoint_dir: str = "checkpoints"
    log_every: int = 100
    save_every: int = 1
    device: str = "cuda"
    num_workers: int = 4
    seed: int = 42


def get_default_config() -> Config:
    return Config()


def _serialize(obj):
    if dataclasses.is_dataclass(obj):
        return {f.name: _serialize(getattr(obj, f.name)) for f in dataclasses.fields(obj)}
    if isinstance(obj, Enum):
        return obj.value
    return obj


def save_config(config: Config, path: str):
    with open(path, "w") as f:
        json.dump(_serialize(config), f, indent=2)


def load_config(path: str) -> Config:
    with open(path) as f:
        d = json.load(f)
    m = d.get("model", {})
    model = ModelConfig(
        encoder=EncoderConfig(**m.get("encoder", {})),
        decoder=DecoderConfig(**m.get("decoder", {})),
        attention=AttentionConfig(**m.get("attention", {})),
        **{k: v for k, v in m.items() if k not in ("encoder", "decoder", "attention")})
    cfg = Config(model=model, training=TrainingConfig(**d.get("training", {})),
                 inference=InferenceConfig(**d.get("inference", {})))
    for k, v in d.items():
        if k not in ("model", "training", "inference"):
            setattr(cfg, k, v)
    return cfg
