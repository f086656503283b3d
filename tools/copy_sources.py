"""Where the device-to-device copies of a config-3 train step and of a beam-5 generate come from:
torch.profiler (CPU activity, Python stacks) over one step / one search, aten::copy_ / clone /
contiguous / cat / index ops grouped by the innermost capk (or bench) source line.

usage: python tools/copy_sources.py [--batch 256] [--what train,beam]
"""
import argparse
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "image-captioning-ml-project_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

from bench import build  # noqa: E402

OPS = ("aten::copy_", "aten::clone", "aten::contiguous", "aten::cat", "aten::index", "aten::index_select",
       "aten::_to_copy", "aten::zeros", "aten::zero_", "aten::fill_", "aten::add", "aten::mul", "aten::where",
       "aten::masked_fill", "aten::gather", "aten::scatter", "aten::cumsum", "aten::eq", "aten::ne")


def site(stack):
    for fr in stack:
        if "capk" in fr or "bench.py" in fr:
            return fr.split("/repo/")[-1]
    return stack[0] if stack else "?"


def report(prof, tag):
    agg = collections.Counter()
    names = collections.Counter()
    for ev in prof.events():
        names[ev.name] += 1
        if ev.name in OPS:
            agg[(ev.name, site(ev.stack or []))] += 1
    print(f"== {tag}: {sum(agg.values())} ops of interest")
    for (name, s), n in agg.most_common(60):
        print(f"{n:5d}  {name:22s} {s}")
    print("-- most frequent events:")
    for name, n in names.most_common(40):
        print(f"{n:5d}  {name}")
    try:
        print(prof.key_averages(group_by_stack_n=6).table(sort_by="count", row_limit=40, max_name_column_width=40))
    except Exception as e:  # noqa: BLE001
        print("key_averages:", e)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--what", default="train,beam")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    cfg, model, store, opt, loss_fn, _ = build(a.batch, dev)
    images = torch.randn(a.batch, 3, 224, 224, device=dev)
    captions = torch.randint(0, 50256, (a.batch, 20), device=dev)

    def step():
        out = model(images=images, captions=captions, caption_lengths=None)
        loss = loss_fn(logits=out["logits"], targets=captions)["total_loss"]
        loss.backward()
        opt.step(lr=1e-4)

    if "train" in a.what:
        model.train()
        step()
        torch.cuda.synchronize()
        with profile(activities=[ProfilerActivity.CPU], with_stack=True, record_shapes=True, acc_events=True) as prof:
            step()
            torch.cuda.synchronize()
        report(prof, "train step")
    if "beam" in a.what:
        model.eval()
        with torch.no_grad():
            model.generate(images=images, max_length=20, num_beams=5)
            torch.cuda.synchronize()
            with profile(activities=[ProfilerActivity.CPU], with_stack=True, record_shapes=True, acc_events=True) as prof:
                model.generate(images=images, max_length=20, num_beams=5)
                torch.cuda.synchronize()
        report(prof, "beam-5 generate")


if __name__ == "__main__":
    main()
