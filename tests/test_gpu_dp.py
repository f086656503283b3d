"""Data-parallel step on the GPU through the real model code.

Two ranks share cuda:0 over gloo (RCCL needs one GPU per rank; the 8-GPU run uses
"nccl" with the same code).  Each rank runs the capk forward + backward of the
tiny config-3 model (fp32 parity path) on its half of the batch with a
GradBucketer installed: the ViT layer / head backward notifications launch
asynchronous all-reduce buckets while the rest of the backward is still queued.
After ``finish()`` every gradient must equal the single-process gradient of the
full batch, and buckets must have been launched before the backward ended."""
import os

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from test_dp_gloo import _free_port, _tiny

pytestmark = pytest.mark.gpu


def _grads(m):
    return {n: p._capk_grad.detach().cpu().clone() for n, p in m.named_parameters()}


def _step(m, images, caps, pad):
    from capk.train import CombinedLoss
    out = m(images=images, captions=caps, caption_lengths=None)
    CombinedLoss(pad)(out["logits"], caps)["total_loss"].backward()


def _worker(rank, world, port, golden, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    import capk
    from capk.train.dp import GradBucketer
    m, sd, dims = _tiny(golden)
    D, Le, He, Ld, Hd, V, pad, patch, img = dims
    store = capk.prepare(m, "cuda", "fp32")
    m.eval()
    bucketer = GradBucketer(store, bucket_elems=1000)
    g = torch.Generator().manual_seed(123)
    images = torch.randn(4, 3, img, img, generator=g).cuda()
    caps = torch.randint(0, V - 1, (4, 7), generator=g).cuda()  # no pad: equal token counts per shard
    shard = slice(rank * 2, rank * 2 + 2)
    _step(m, images[shard], caps[shard], pad)
    early = len(bucketer.works)
    bucketer.finish()
    torch.cuda.synchronize()
    got = _grads(m)
    if rank == 0:
        m2, _, _ = _tiny(golden)
        capk.prepare(m2, "cuda", "fp32")
        m2.eval()
        _step(m2, images, caps, pad)
        torch.cuda.synchronize()
        ref = _grads(m2)
        # relative to the parameter's own scale, floored at 1e-3 of the largest gradient: the
        # attention key bias has an analytically zero gradient (softmax shift invariance), so
        # its values are rounding noise on both sides
        top = max(float(t.abs().max()) for t in ref.values())
        errs = {n: float((got[n] - ref[n]).abs().max()) / max(float(ref[n].abs().max()), 1e-3 * top) for n in ref}
        bad = sorted((n for n in errs if errs[n] >= 1e-5), key=lambda n: -errs[n])[:12]
        torch.save({"err": max(errs.values()), "early": early, "bad": [(n, errs[n]) for n in bad]}, out)
    dist.barrier()
    dist.destroy_process_group()


def test_dp_two_ranks_overlapped_equals_full_batch(tmp_path, golden_dir):
    out = str(tmp_path / "dp_gpu.pt")
    golden = os.path.join(golden_dir, "vit_transformer_step.npz")
    mp.spawn(_worker, args=(2, _free_port(), golden, out), nprocs=2, join=True)
    res = torch.load(out, weights_only=True)
    assert res["err"] < 1e-5, res
    assert res["early"] > 0, res
