"""Stable coverage of the bf16-vs-fp32 beam-5 precision check (tests/test_gpu_beam.py
_bf16_vs_fp32_margins) for several peaked-LM-head settings of the config-3 model, 256 images.
PROBE_SETTINGS="n_hot:gain:eos_hot:round_bf16:bias_step:cold_bias:bias_spread[:bias_offset];..." overrides
the list."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "image-captioning-ml-project_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import torch  # noqa: E402

import test_gpu_beam as tb  # noqa: E402

DEFAULT = "8:3:0:1:0:-20:10;8:4:0:1:0:-20:12;12:3:0:1:0:-20:16;6:2:0:1:0:-20:8;8:2.5:0:1:0:-20:8;16:3:0:1:0:-20:24;8:2:0:1:0:-20:8"


def main():
    B = int(os.environ.get("PROBE_B", "256"))
    images = torch.randn(B, 3, 224, 224, generator=torch.Generator().manual_seed(3)).cuda()
    for item in os.environ.get("PROBE_SETTINGS", DEFAULT).split(";"):
        f = item.split(":")
        n_hot, gain, eos_hot, rb, bstep, cold, spread = f[:7]
        kw = dict(n_hot=int(n_hot), gain=float(gain), eos_hot=eos_hot == "1", round_bf16=rb == "1",
                  bias_step=float(bstep), cold_bias=float(cold), bias_spread=float(spread),
                  bias_offset=float(f[7]) if len(f) > 7 else 0.0)
        m32, cfg = tb._config3_peaked("fp32", **kw)
        m16, _ = tb._config3_peaked("bf16", **kw)
        same, stable, ids16, err = tb._bf16_vs_fp32_margins(m32, m16, cfg, images)
        lens = (ids16 != cfg.model.pad_token_id).sum(1).float()
        print(f"{kw}: identical {float(same.float().mean()):.3f}  stable {float(stable.float().mean()):.3f}  "
              f"stable steps {tb._bf16_vs_fp32_margins.step_cov:.3f}  "
              f"stable&different {int((stable & ~same).sum())}  median err {float(err.median()):.4f}  "
              f"mean output length {float(lens.mean()):.1f}  distinct best sequences {len(set(map(tuple, ids16.tolist())))}",
              flush=True)
        del m32, m16
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
