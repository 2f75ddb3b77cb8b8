"""Data-parallel training over the GPUs of one node (RCCL over xGMI).

The reference is single-device.  The SD-VAE step
shards naturally: every swap group (``bs`` base meshes -> ``bs^2`` swapped
meshes) is self-contained (the latent-consistency loss is intra-group,
``model_manager.py:360-393``; no batch norm), so each rank trains on its own
groups and the only exchange is ONE all-reduce of the flat fp32 gradient
bucket (1 081 881 parameters = 4.3 MB) per step, followed by an identical
Adam on every rank.  One process per GPU; ``backend="nccl"`` is RCCL on ROCm.
"""
import os

import torch
import torch.distributed as dist


def env_world():
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def init_from_env(backend=None, device_id=None):
    """Initialise the default process group from torchrun's environment
    (MASTER_ADDR defaults to 127.0.0.1).  Returns (world, rank, local_rank)."""
    world, rank, local = env_world()
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29511")
        backend = backend or ("nccl" if torch.cuda.is_available() else "gloo")
        kw = {}
        if backend == "nccl" and device_id is not None:
            kw["device_id"] = device_id
        dist.init_process_group(backend, rank=rank, world_size=world, **kw)
    return world, rank, local


def barrier():
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.barrier()


def destroy():
    if dist.is_initialized():
        dist.destroy_process_group()


def broadcast_parameters(flat, src=0):
    """Make every rank start from rank ``src``'s parameters."""
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.broadcast(flat, src)


class GradientAverager:
    """All-reduce(SUM) of the flat gradient, then x 1/world.

    Two ways to use it (both give the same numbers):
    * ``avg(grad)``: one blocking all-reduce of the whole bucket;
    * bucketed, overlapped with the backward (``SDVAEEngine.train_step_on``
      does this when handed an averager): ``bucket_ready(view)`` starts an
      asynchronous all-reduce of one contiguous slice as soon as the backward
      has finalised it (RCCL runs on its own stream, ordered after the work
      already queued), ``finish(grad)`` joins them and scales.
    ``scale`` is the in-place scaling routine: libcfsd's ``cfsd_scale`` for
    device buffers (default), or any callable ``(tensor, alpha)``.
    ``always``: issue the collectives even at world 1 (a one-rank RCCL group
    runs the data-parallel step structure on one GPU: the test that RCCL
    loads, runs and captures into the step graph, bit-equal to the
    single-process step)."""

    def __init__(self, world=None, scale=None, group=None, always=False):
        self.world = world if world is not None else (dist.get_world_size() if dist.is_initialized() else 1)
        self.group = group
        self.always = bool(always)
        if scale is None:
            from . import ops
            scale = ops.scale
        self.scale = scale
        self._works = []

    @property
    def active(self):
        """True when the step must exchange gradients (world > 1, or forced)."""
        return self.world > 1 or self.always

    @property
    def capturable(self):
        """The collectives can be recorded into a hipGraph: RCCL supports
        stream capture (gloo runs on the host and cannot be captured)."""
        return dist.is_initialized() and dist.get_backend(self.group) == "nccl"

    def __call__(self, grad):
        if not self.active:
            return grad
        dist.all_reduce(grad, op=dist.ReduceOp.SUM, group=self.group)
        self.scale(grad, 1.0 / self.world)
        return grad

    def bucket_ready(self, view):
        if self.active:
            self._works.append(dist.all_reduce(view, op=dist.ReduceOp.SUM, group=self.group,
                                               async_op=True))

    def finish(self, grad, scale=True):
        """Join the bucket all-reduces; ``scale=False`` leaves the 1/world
        factor to the caller (``TrainStep`` folds it into Adam)."""
        works, self._works = self._works, []
        for w in works:
            w.wait()
        if self.active and scale and self.world > 1:
            self.scale(grad, 1.0 / self.world)
        return grad


def shard_range(n_items, rank, world):
    """Contiguous shard [lo, hi) of ``n_items`` for ``rank`` (sizes differ by <= 1)."""
    per, rem = divmod(n_items, world)
    lo = rank * per + min(rank, rem)
    return lo, lo + per + (1 if rank < rem else 0)


def steps_per_epoch(n_items, world, bs):
    """Train steps per epoch that EVERY rank runs over its :func:`shard_range`
    shard: the smallest shard's ``len // bs`` (= (n_items // world) // bs).
    Each step issues the gradient all-reduces, so ranks running different
    counts would pair one rank's step collective with the other's end-of-epoch
    loss all-reduce (RCCL hangs, gloo errors).  Depends on the sizes only, so
    all ranks agree without communicating."""
    return (n_items // world) // bs


def max_over_ranks(value, device=None):
    """Max of a Python float over ranks (timing: the slowest rank defines the step)."""
    if not (dist.is_initialized() and dist.get_world_size() > 1):
        return value
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
