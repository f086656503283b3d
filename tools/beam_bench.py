#!/usr/bin/env python3
"""Beam-5 only timing/profiling harness (config-3 model, bf16): python tools/beam_bench.py [--batch 256] [--reps 3]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "image-captioning-ml-project_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from bench import build  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--beams", type=int, default=5)
    ap.add_argument("--encoder-only", action="store_true")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    cfg, model, store, opt, loss_fn, _ = build(args.batch, dev)
    model.eval()
    images = torch.randn(args.batch, 3, 224, 224, device=dev)
    if args.encoder_only:
        with torch.no_grad():
            for _ in range(2):
                model.encoder(images)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.reps):
                model.encoder(images)
            torch.cuda.synchronize()
        t = (time.perf_counter() - t0) / args.reps
        print(f"encoder fwd batch {args.batch}: {t*1e3:.2f} ms", flush=True)
        return
    with torch.no_grad():
        model.generate(images=images, max_length=20, num_beams=args.beams)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.reps):
            enc = model.encoder(images)
        torch.cuda.synchronize()
        t_enc = (time.perf_counter() - t0) / args.reps
        t0 = time.perf_counter()
        for _ in range(args.reps):
            ids, info = model.generate(images=images, max_length=20, num_beams=args.beams)
        torch.cuda.synchronize()
        t_all = (time.perf_counter() - t0) / args.reps
    print(f"batch {args.batch} beams {args.beams}: total {t_all*1e3:.2f} ms/batch ({args.batch/t_all:.1f} captions/s), "
          f"encoder {t_enc*1e3:.2f} ms, decode {(t_all-t_enc)*1e3:.2f} ms, out len {ids.shape[1]}", flush=True)


if __name__ == "__main__":
    main()
