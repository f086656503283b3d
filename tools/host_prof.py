#!/usr/bin/env python3
"""Host-side cost of the config-3 encoder forward / beam decode: wall time to issue the launches
(no sync) vs. wall time with the device drained, and a cProfile of the issue path.
python tools/host_prof.py [--what encoder|beam] [--batch 256]"""
import argparse
import cProfile
import os
import pstats
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
    ap.add_argument("--what", default="encoder")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    cfg, model, store, opt, loss_fn, _ = build(args.batch, dev)
    model.eval()
    images = torch.randn(args.batch, 3, 224, 224, device=dev)
    if args.what == "encoder":
        fn = lambda: model.encoder(images)  # noqa: E731
    else:
        fn = lambda: model.generate(images=images, max_length=20, num_beams=5)  # noqa: E731
    with torch.no_grad():
        for _ in range(2):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        t_issue = time.perf_counter() - t0
        torch.cuda.synchronize()
        t_all = time.perf_counter() - t0
        print(f"{args.what}: host issue {t_issue * 1e3:.2f} ms, issue + drain {t_all * 1e3:.2f} ms", flush=True)
        pr = cProfile.Profile()
        pr.enable()
        fn()
        pr.disable()
        torch.cuda.synchronize()
    pstats.Stats(pr).sort_stats("tottime").print_stats(18)


if __name__ == "__main__":
    main()
