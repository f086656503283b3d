"""In-process A/B of libcapk GEMM knobs on the config-3 shapes (HIP events, graph-replayed).

Variants are interleaved round by round in ONE process (guide §5.4 rule 24) and the median /
min per variant are printed.  AB_KNOB selects the knob:
  group  capk_gemm_set_group(v)   (persistent-GEMM raster: 0 row-major, -1 auto, n rows)
  tail   capk_gemm_set_tail(v)
AB_VALUES="0,-1" the values; AB_ROUNDS rounds; GEMM_ONLY / GEMM_SHAPES as tools/gemm_bench.py.
"""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "image-captioning-ml-project_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402

import gemm_bench as gb  # noqa: E402
from capk import _lib  # noqa: E402


def make_fn(name, M, N, K, kind):
    from capk import ops
    from capk._lib import ACT_DERIV, ACT_GELU_ERF
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    if kind.startswith("fwd"):
        x = torch.rand(M, K, device=dev, generator=g).mul_(2).sub_(1).bfloat16()
        w = (torch.rand(N, K, device=dev, generator=g).mul_(2).sub_(1) * 0.05).bfloat16()
        b = torch.zeros(N, device=dev)
        pre = torch.empty(M, N, device=dev, dtype=torch.bfloat16) if "gelu" in kind else None
        res = torch.randn(M, N, device=dev, generator=g).bfloat16() if "res" in kind else None
        act = (ACT_GELU_ERF | (ACT_DERIV if "deriv" in kind else 0)) if pre is not None else 0
        return lambda: ops.linear(x, w, b, act=act, preact=pre, residual=res)
    if kind.startswith("dx"):
        dy = torch.rand(M, K, device=dev, generator=g).mul_(2).sub_(1).bfloat16()
        w = (torch.rand(K, N, device=dev, generator=g).mul_(2).sub_(1) * 0.05).bfloat16()
        aux = torch.randn(M, N, device=dev, generator=g).bfloat16() if "gelu" in kind else None
        act = (ACT_GELU_ERF | (ACT_DERIV if "deriv" in kind else 0)) if aux is not None else 0
        return lambda: ops.linear_dx(dy, w, act_bwd=act, aux=aux)
    dy = torch.rand(M, N, device=dev, generator=g).mul_(2).sub_(1).bfloat16()
    x = torch.rand(M, K, device=dev, generator=g).mul_(2).sub_(1).bfloat16()
    dw = torch.empty(N, K, device=dev)
    return lambda: ops.linear_dw(dy, x, dw)


def main():
    lib = _lib.load()
    knob = os.environ.get("AB_KNOB", "group")
    setter = {"group": lib.capk_gemm_set_group, "tail": lib.capk_gemm_set_tail}[knob]
    reset = {"group": -2, "tail": -1}[knob]
    values = [int(v) for v in os.environ.get("AB_VALUES", "0,-1").split(",")]
    rounds = int(os.environ.get("AB_ROUNDS", "5"))
    iters = int(os.environ.get("GEMM_ITERS", "20"))
    only = os.environ.get("GEMM_ONLY")
    shapes = gb.SHAPES
    extra = os.environ.get("GEMM_SHAPES")
    if extra:
        shapes = [(f[0], int(f[1]), int(f[2]), int(f[3]), f[4]) for f in (x.split(":") for x in extra.split(","))]
    for name, M, N, K, kind in shapes:
        if only and name not in only.split(","):
            continue
        fn = make_fn(name, M, N, K, kind)
        graphs = {}
        for v in values:  # one graph per variant (the knob is read at capture time)
            setter(v)
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr):
                for _ in range(iters):
                    fn()
            gr.replay()
            torch.cuda.synchronize()
            graphs[v] = gr
        setter(reset)
        times = {v: [] for v in values}
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for _ in range(rounds):
            for v in values:
                e0.record()
                graphs[v].replay()
                e1.record()
                torch.cuda.synchronize()
                times[v].append(e0.elapsed_time(e1) / iters * 1e3)
        fl = 2.0 * M * N * K
        parts = []
        for v in values:
            med = statistics.median(times[v])
            parts.append(f"{knob}={v}: med {med:7.1f} us min {min(times[v]):7.1f} ({fl / med / 1e6:6.1f} TF/s)")
        print(f"{name:22s} M={M:6d} N={N:6d} K={K:6d}  " + " | ".join(parts), flush=True)
        del graphs


if __name__ == "__main__":
    main()
