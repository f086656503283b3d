"""Data-parallel semantics on CPU (gloo, world_size 2): the flat-gradient all-reduce
of capk.train.dp makes a DP step equal to a single-process step on the
concatenated batch.  Gradients are produced by the CPU oracle on
each rank's shard and written into the ParamStore's flat buffers, then averaged
with the same bucketed all_reduce bench.py uses (RCCL on the GPU node)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _tiny(golden):
    import sys
    for p in (ROOT, os.path.join(ROOT, "image-captioning-ml-project_amd")):
        if p not in sys.path:
            sys.path.insert(0, p)
    z = np.load(golden, allow_pickle=False)
    from capk import config as C
    from capk.models import captioning_model as cm
    from capk.models import encoders as E
    D, Le, He, Ld, Hd, V, pad, patch, img = [int(x) for x in z["meta/dims"]]
    cfg = C.Config()
    cfg.model.encoder = C.EncoderConfig(encoder_type="vit", feature_dim=D)
    cfg.model.decoder = C.DecoderConfig(decoder_type="transformer", hidden_dim=D, num_layers=Ld, num_heads=Hd)
    cfg.model.vocab_size, cfg.model.pad_token_id = V, pad
    arch = dict(hidden_size=D, num_hidden_layers=Le, num_attention_heads=He, intermediate_size=2 * D,
                image_size=img, patch_size=patch, num_channels=3, layer_norm_eps=1e-12)
    orig = E.VIT_ARCHS["google/vit-base-patch16-224"]
    E.VIT_ARCHS["google/vit-base-patch16-224"] = arch
    try:
        m = cm.ImageCaptioningModel(cfg)
    finally:
        E.VIT_ARCHS["google/vit-base-patch16-224"] = orig
    sd = {k[3:]: torch.from_numpy(z[k].copy()) for k in z.files if k.startswith("p0/")}
    m.load_state_dict(sd)
    return m, sd, (D, Le, He, Ld, Hd, V, pad, patch, img)


def _oracle_grads(sd, dims, images, caps):
    from oracle import decoders as odec
    from oracle import encoders as oenc
    from oracle import train as otrain
    D, Le, He, Ld, Hd, V, pad, patch, img = dims
    p = {k: v.clone().requires_grad_(True) for k, v in sd.items()}
    sub = lambda pre: {k[len(pre):]: v for k, v in p.items() if k.startswith(pre)}
    enc = oenc.vit_encoder(sub("encoder.model."), images, Le, He, patch)
    logits = odec.transformer_decoder(sub("decoder."), enc["features"], caps, Ld, Hd, pad)
    otrain.shifted_ce(logits, caps, pad).backward()
    return {k: (v.grad if v.grad is not None else torch.zeros_like(v)) for k, v in p.items()}


def _worker(rank, world, port, golden, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    m, sd, dims = _tiny(golden)
    from capk.params import attach
    from capk.train.dp import allreduce_grads
    store = attach(m, "cpu")
    D, Le, He, Ld, Hd, V, pad, patch, img = dims
    g = torch.Generator().manual_seed(123)
    images = torch.randn(4, 3, img, img, generator=g)
    caps = torch.randint(0, V - 1, (4, 7), generator=g)  # no pad: equal token counts per shard
    shard = slice(rank * 2, rank * 2 + 2)
    grads = _oracle_grads(sd, dims, images[shard], caps[shard])
    named = dict(m.named_parameters())
    with torch.no_grad():
        for n, t in grads.items():
            named[n]._capk_grad.copy_(t)
    allreduce_grads(store, bucket_elems=1000)  # small buckets: exercise the chunking
    if rank == 0:
        full = _oracle_grads(sd, dims, images, caps)
        err = max(float((named[n]._capk_grad - full[n]).abs().max()) for n in full)
        torch.save({"err": err}, out)
    dist.barrier()
    dist.destroy_process_group()


def _worker_overlap(rank, world, port, golden, out, exchange="fp32"):
    """GradBucketer: gradients become final in reverse registration order (as in the
    backward), each followed by a notification; buckets launch asynchronously while
    later gradients are still being written."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    m, sd, dims = _tiny(golden)
    from capk.params import attach, notify_final
    from capk.train.dp import GradBucketer
    store = attach(m, "cpu")
    bucketer = GradBucketer(store, bucket_elems=1000, exchange=exchange)
    D, Le, He, Ld, Hd, V, pad, patch, img = dims
    g = torch.Generator().manual_seed(123)
    images = torch.randn(4, 3, img, img, generator=g)
    caps = torch.randint(0, V - 1, (4, 7), generator=g)
    shard = slice(rank * 2, rank * 2 + 2)
    named = dict(m.named_parameters())
    full = _oracle_grads(sd, dims, images, caps)
    for step in range(2):  # the bucketer resets between steps
        grads = _oracle_grads(sd, dims, images[shard], caps[shard])
        for buf in store.grad.values():
            buf.fill_(float("nan"))  # a bucket launched before its gradients were written would poison the result
        launched = []
        # the optional pooler (buffer tail) is final with the encoder head, before the encoder layers
        order = [n for n in reversed(list(named)) if id(named[n]) in store.optional]
        order += [n for n in reversed(list(named)) if id(named[n]) not in store.optional]
        for n in order:
            with torch.no_grad():
                named[n]._capk_grad.copy_(grads[n])
            notify_final(store, [named[n]])
            launched.append(len(bucketer.works))
        bucketer.finish()
        err = max(float((named[n]._capk_grad - full[n]).abs().max()) for n in full)
        gmax = max(float(full[n].abs().max()) for n in full)
        if rank == 0:
            torch.save({"err": err, "gmax": gmax, "early": launched[len(launched) // 2]}, out)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("exchange,tol", [("fp32", 1e-5), ("bf16", 1e-2)])
def test_dp_overlapped_buckets_equal_full_batch(tmp_path, golden_dir, exchange, tol):
    """fp32 exchange: equal to the full-batch gradient to fp32 rounding.  bf16 exchange:
    every gradient element within 1e-2 x the largest gradient magnitude (one bf16 rounding
    per rank and per reduction step, 8 significant bits)."""
    out = str(tmp_path / "dpo.pt")
    golden = os.path.join(golden_dir, "vit_transformer_step.npz")
    mp.spawn(_worker_overlap, args=(2, _free_port(), golden, out, exchange), nprocs=2, join=True)
    res = torch.load(out, weights_only=True)
    assert res["err"] < tol * max(1.0, res["gmax"]), res
    assert res["early"] > 0, res  # collectives were in flight before the last gradient was written


def _backward_groups(m):
    """The notify_final points of the real backward, in its order (capk/models/transformer.py
    _DecoderFn.backward, vit.py _ViTLayerFn / _ViTHeadFn / _ViTEmbedFn): the decoder's LM head,
    its layers last to first, its embeddings, its visual projection; then the encoder head
    (every parameter but the encoder's embeddings and layers), the encoder layers last to first."""
    dec, enc = m.decoder, m.encoder.model
    groups = [("dec_head", [dec.output_layer.weight, dec.output_layer.bias])]
    for i in reversed(range(len(dec.transformer_decoder.layers))):
        groups.append((f"dec_layer{i}", list(dec.transformer_decoder.layers[i].parameters())))
    groups.append(("dec_emb", [dec.embedding.weight, dec.position_encoding.weight]))
    groups.append(("dec_vproj", [dec.visual_projection.weight, dec.visual_projection.bias]))
    groups.append(("enc_head", None))  # all_except: the encoder's embeddings and layers
    for i in reversed(range(len(enc.layers))):
        groups.append((f"enc_layer{i}", list(enc.layers[i].parameters())))
    groups.append(("enc_emb", list(enc.embeddings.parameters())))
    return groups


def _worker_decoder_buckets(rank, world, port, golden, out):
    """GradBucketer with the model's own notification points: the decoder's buckets (LM head,
    each layer) launch while the decoder backward still runs -- the visual projection, finished
    last, sits in front of the decoder's run (params._capk_store_first) and the optional ViT
    pooler at the buffer tail is exchanged by finish() -- and the result is the full-batch
    gradient (NaN-poisoned buffers catch any premature launch)."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    m, sd, dims = _tiny(golden)
    from capk.params import attach, notify_final
    from capk.train.dp import GradBucketer
    store = attach(m, "cpu")
    bucketer = GradBucketer(store, bucket_elems=1000)
    D, Le, He, Ld, Hd, V, pad, patch, img = dims
    g = torch.Generator().manual_seed(321)
    images = torch.randn(4, 3, img, img, generator=g)
    caps = torch.randint(0, V - 1, (4, 7), generator=g)
    shard = slice(rank * 2, rank * 2 + 2)
    named = dict(m.named_parameters())
    name_of = {id(p): n for n, p in named.items()}
    full = _oracle_grads(sd, dims, images, caps)
    grads = _oracle_grads(sd, dims, images[shard], caps[shard])
    for buf in store.grad.values():
        buf.fill_(float("nan"))
    launched = {}
    enc_skip = list(m.encoder.model.embeddings.parameters()) + list(m.encoder.model.layers.parameters())
    done = set()
    for tag, params in _backward_groups(m):
        if params is None:  # the encoder head: everything not written yet but the encoder body
            skip = {id(p) for p in enc_skip}
            params = [p for p in named.values() if id(p) not in skip and id(p) not in done]
        with torch.no_grad():
            for p in params:
                p._capk_grad.copy_(grads[name_of[id(p)]])
                done.add(id(p))
        if tag == "enc_head":
            notify_final(store, all_except=enc_skip)
        else:
            notify_final(store, params)
        launched[tag] = len(bucketer.works)
    bucketer.finish()
    err = max(float((named[n]._capk_grad - full[n]).abs().max()) for n in full)
    gmax = max(float(full[n].abs().max()) for n in full)
    if rank == 0:
        torch.save({"err": err, "gmax": gmax, "launched": launched}, out)
    dist.barrier()
    dist.destroy_process_group()


def test_dp_decoder_layer_buckets_launch_early(tmp_path, golden_dir):
    out = str(tmp_path / "dpd.pt")
    golden = os.path.join(golden_dir, "vit_transformer_step.npz")
    mp.spawn(_worker_decoder_buckets, args=(2, _free_port(), golden, out), nprocs=2, join=True)
    res = torch.load(out, weights_only=True)
    assert res["err"] < 1e-5 * max(1.0, res["gmax"]), res
    L = res["launched"]
    # decoder buckets in flight before the decoder backward is over (its embeddings and visual
    # projection), and more launched while the encoder layers still run
    assert L["dec_layer0"] > 0, L
    assert L["dec_head"] <= L["dec_layer0"] <= L["enc_head"] <= L["enc_layer0"], L


def test_dp_allreduce_equals_full_batch(tmp_path, golden_dir):
    out = str(tmp_path / "dp.pt")
    golden = os.path.join(golden_dir, "vit_transformer_step.npz")
    mp.spawn(_worker, args=(2, _free_port(), golden, out), nprocs=2, join=True)
    res = torch.load(out, weights_only=True)
    assert res["err"] < 1e-5, res


def _worker_bench(rank, world, port, golden, out):
    """bench.py's own N>1 path on CPU: dist_init (torchrun env vars), the backward-overlapped
    GradBucketer with the bf16 exchange bench.py uses by default, timed_steps' barrier +
    MAX-over-ranks timing, and the whole-job throughput formula."""
    import importlib.util
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    spec = importlib.util.spec_from_file_location("bench", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    w, r, local = bench.dist_init("gloo")
    assert (w, r, local) == (world, rank, rank)
    torch.manual_seed(0)
    m, sd, dims = _tiny(golden)
    from capk.params import attach, notify_final
    from capk.train.dp import GradBucketer
    store = attach(m, "cpu")
    bucketer = GradBucketer(store, bucket_elems=4096, exchange="bf16")
    D, Le, He, Ld, Hd, V, pad, patch, img = dims
    g = torch.Generator().manual_seed(7)
    images = torch.randn(4, 3, img, img, generator=g)
    caps = torch.randint(0, V - 1, (4, 7), generator=g)
    shard = slice(rank * 2, rank * 2 + 2)
    named = dict(m.named_parameters())
    order = [n for n in reversed(list(named)) if id(named[n]) in store.optional]
    order += [n for n in reversed(list(named)) if id(named[n]) not in store.optional]
    n_steps = [0]

    def step():  # the backward writes gradients in reverse order and notifies, then finish()
        grads = _oracle_grads(sd, dims, images[shard], caps[shard])
        for n in order:
            with torch.no_grad():
                named[n]._capk_grad.copy_(grads[n])
            notify_final(store, [named[n]])
        bucketer.finish()
        n_steps[0] += 1
        if rank == 1:
            import time
            time.sleep(0.05)  # the slower rank sets the reported time

    elapsed = bench.timed_steps(step, 2, 1, world, sync=lambda: None, device="cpu")
    full = _oracle_grads(sd, dims, images, caps)
    err = max(float((named[n]._capk_grad - full[n]).abs().max()) for n in full)
    gmax = max(float(full[n].abs().max()) for n in full)
    value = bench.throughput(2, world, 2, elapsed)
    torch.save({"elapsed": elapsed, "err": err, "gmax": gmax, "steps": n_steps[0], "value": value},
               out + f".{rank}")
    dist.barrier()
    dist.destroy_process_group()


def test_bench_dp_path_gloo(tmp_path, golden_dir):
    out = str(tmp_path / "bench")
    golden = os.path.join(golden_dir, "vit_transformer_step.npz")
    mp.spawn(_worker_bench, args=(2, _free_port(), golden, out), nprocs=2, join=True)
    r0 = torch.load(out + ".0", weights_only=True)
    r1 = torch.load(out + ".1", weights_only=True)
    assert r0["steps"] == r1["steps"] == 3  # 1 warm-up + 2 timed
    assert r0["elapsed"] == r1["elapsed"] >= 0.1  # MAX over ranks: rank 1's 2 x 50 ms sleeps
    assert abs(r0["value"] - 2 * 2 * 2 / r0["elapsed"]) < 1e-9
    assert r0["err"] < 1e-2 * max(1.0, r0["gmax"]), r0  # bf16 exchange of the averaged gradient


def test_bench_gpus2_self_launch():
    """`python bench.py --gpus 2` with no torchrun environment starts 2 ranks itself (a child
    torch.distributed.run, before any GPU call) and the printed line reports 2 ranks -- here
    in the CPU/gloo self-test mode, which runs the same launch, dist_init, GradBucketer and
    MAX-over-ranks timing as the GPU workloads."""
    import json
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dp-selftest", "--steps",
                        "2", "--warmup", "1", "--batch", "4"], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 prints ONE line
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["process_group"] == {"backend": "gloo", "world_size": 2}, rec
    assert rec["config"]["global_batch"] == 8 and rec["steps"] == 2
    assert abs(rec["value"] - 8 * 2 / (rec["ms_per_step"] * 2 / 1e3)) < 0.01 * rec["value"]
