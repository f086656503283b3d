"""Writes tests/golden/ref_checkpoint.pth: a checkpoint in the reference trainer's layout
(src/train/trainer.py:578-585) with the reference's own pickled ``src.config.Config``
(non-default Enum / field values), a small model state dict and a torch AdamW + LambdaLR
state -- the input of tests/test_checkpoint.py's reference-checkpoint load test.
Run in the build container (imports /root/reference); the GPU box only reads the file."""
import os
import sys

import torch

REF = "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden", "ref_checkpoint.pth")


def main():
    sys.path.insert(0, REF)
    from src import config as RC
    cfg = RC.Config()
    cfg.model.encoder.encoder_type = RC.EncoderType.CLIP
    cfg.model.decoder.decoder_type = RC.DecoderType.LSTM
    cfg.model.attention.attention_type = RC.AttentionType.AOA
    cfg.training.batch_size = 48
    torch.manual_seed(0)
    lin = torch.nn.Linear(4, 3)
    opt = torch.optim.AdamW(lin.parameters(), lr=1e-3)
    sch = torch.optim.lr_scheduler.LambdaLR(opt, lambda s: 1.0)
    lin(torch.randn(2, 4)).sum().backward()
    opt.step()
    sch.step()
    ck = {"epoch": 2, "model_state_dict": lin.state_dict(), "optimizer_state_dict": opt.state_dict(),
          "scheduler_state_dict": sch.state_dict(), "config": cfg, "best_val_score": 0.625}
    torch.save(ck, OUT)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
