"""Data parallelism: one process per GPU, gradient all-reduce over RCCL/xGMI.

The reference has no distributed code; the build adds plain DP:
every rank computes the full train step on its own batch shard and the flat
fp32 gradient buffers of the ParamStore are averaged with bucketed
``all_reduce`` (backend "nccl" = RCCL on ROCm).  Buckets are contiguous slices
of the flat buffers (no packing copies).  Buckets can be launched while the
backward is still running (``GradBucketer.launch_ready``) on a side stream so
the exchange overlaps the remaining backward; ``finish()`` joins them before the
optimizer step.
"""
import torch
import torch.distributed as dist

BUCKET_ELEMS = 16 * 1024 * 1024  # 64 MiB of fp32 per all-reduce


def _avg_op():
    if dist.get_backend() == "nccl":
        return dist.ReduceOp.AVG, False
    return dist.ReduceOp.SUM, True  # gloo has no AVG: sum, then scale


def allreduce_grads(store, bucket_elems=BUCKET_ELEMS):
    """Average every gradient buffer across ranks (blocking on the current stream)."""
    if not dist.is_available() or not dist.is_initialized() or dist.get_world_size() == 1:
        return
    op, need_scale = _avg_op()
    world = dist.get_world_size()
    for g in store.groups:
        buf = store.grad[g]
        n = buf.numel()
        for s in range(0, n, bucket_elems):
            chunk = buf[s:s + bucket_elems]
            dist.all_reduce(chunk, op=op)
            if need_scale:
                chunk.div_(world)
