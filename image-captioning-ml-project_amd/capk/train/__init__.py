from .losses import CombinedLoss, shifted_cross_entropy  # noqa: F401
from .optim import CapkAdamW, cosine_schedule_with_warmup  # noqa: F401
