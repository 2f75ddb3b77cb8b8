"""The replayable training step: one ``ModelManager._do_iteration``
(``model_manager.py:274-326``) from an HBM-resident dataset, on one GPU or
data-parallel over the GPUs of a node, captured as hipGraphs.

This is the object ``bench.py``, ``manager.ModelManager`` (and so
``train.py``) and the data-parallel GPU tests all run, so the step that is
timed is the step that is tested.

Step anatomy (every launch on one stream; nothing synchronises with the host):

* ``part_a``: ``cfsd_step_begin`` (device counter -> epoch-shuffled batch
  pick, swap key, VAE noise, Adam's t), the feature swap, the forward with its
  four losses, and the backward from the losses through the decoder, the
  latent head and the encoder Linear.  After it the gradient of everything
  from the encoder Linear on (~96 % of the parameters) is final;
* ``part_b``: the encoder conv backward and the batched weight-gradient
  reduce.  On one GPU Adam rides in that reduce (``cfsd_dw_reduce_batch_adam``);
* ``part_c``: (data-parallel only) Adam, after the gradient all-reduce.

One graph per step whenever the collectives can be captured: on one GPU the
three parts are ONE graph; data-parallel over RCCL the two bucket all-reduces
are recorded INTO that graph (RCCL supports stream capture: the decoder /
bottleneck bucket forks onto RCCL's stream right after ``part_a`` and overlaps
``part_b``, the encoder-conv bucket follows ``part_b``, both join before
Adam, which folds in the 1/world averaging -- ``cfsd_adam_scaled``).  A
second graph, recorded on the first :meth:`TrainStep.run` of
``steps_per_graph`` or more steps, holds that many whole steps back to back:
the host gap between consecutive replays (~8 us) is paid once per replay
instead of once per step.  A backend that cannot be captured (gloo: the
one-GPU rehearsals and CPU tests) keeps three graphs with the all-reduces
issued by the host between their replays (``CFSD_DP_GRAPH=three`` forces that
structure over RCCL for A/B).  The
justification for data parallelism is that every loss term is intra-swap-group
(``model_manager.py:360-393``): each rank trains its own groups and the only
exchange is the flat fp32 gradient.
"""
import os

import torch

from . import ops

# Capture in thread-local mode: with the default ("global") mode a CUDA/HIP
# call from ANY thread that is unsafe during capture fails -- and the RCCL
# process group's watchdog thread polls the events of finished collectives
# (cudaEventQuery) at its own pace, so a capture that overlaps one of its
# polls aborted the process (a watchdog exception in one of round 6's
# one-rank RCCL capture tests).  The capturing thread itself is still checked.
_CAPTURE_MODE = "thread_local"


class TrainStep:
    """``TrainStep(engine, data, averager=None, acc=None)``.

    ``engine``: :class:`engine.SDVAEEngine`; ``data``: :class:`engine.
    ResidentData` (this rank's shard); ``averager``: a
    :class:`dist.GradientAverager` (``None``, or world 1 without ``always``: single GPU);
    ``acc``: the device loss accumulator (default ``engine.loss_acc``).

    ``step()`` runs one training step -- eagerly until :meth:`capture` was
    called, then by graph replay.  ``capture()`` first runs ONE real step
    eagerly on a side stream (that step counts: it advances the counter,
    the parameters and the epoch position exactly like any other), then
    records the graphs; nothing executes while recording, so the k-th step
    of a captured runner equals the k-th step of an eager one, bit for bit."""

    def __init__(self, engine, data, averager=None, acc=None):
        self.eng = engine
        self.data = data
        self.avg = averager if (averager is not None and averager.active) else None
        self.b = engine.buffers(engine.step_rows)
        self.acc = engine.loss_acc if acc is None else acc
        self.graphs = None
        self.graph_multi = None
        # steps recorded into the multi-step graph run(k) replays (env: A/B)
        self.steps_per_graph = max(1, int(os.environ.get("CFSD_STEPS_PER_GRAPH", "16")))
        self._split = engine.enc_conv_numel()
        # the whole step (collectives included) as one graph, unless the
        # backend cannot be captured or the three-graph structure is forced
        self.one_graph = self.avg is None or (os.environ.get("CFSD_DP_GRAPH", "one") != "three"
                                              and self.avg.capturable)
        self.fallback = None  # why a capturable backend ended up with the three-graph structure

    @property
    def world(self):
        return self.avg.world if self.avg is not None else 1

    @property
    def captured(self):
        return self.graphs is not None

    # ------------------------------------------------------------ the parts
    def part_a(self):
        eng, b, T, d = self.eng, self.b, self.eng.topo, self.data
        ops.step_begin(eng.counter, eng.seed, eps=b.eps if eng.spec.is_vae else None, key=b.key,
                       n_regions=max(T.n_regions, 1), batch_idx=b.batch_idx, bs=eng.swap_bs,
                       n_batches=d.n_batches, perm=d.rows, n_items=d.n_items, shuffle=d.shuffle,
                       adam_step=eng.params.step)
        eng.load_batch(b, d)
        eng.forward(b, train=True, acc=self.acc, finalize=False)
        eng.backward_head(b, split=self.avg is not None, fuse_adam=self.avg is None)

    def part_b(self):
        self.eng.backward_tail(self.b, fuse_adam=self.avg is None)

    def part_c(self):
        if self.avg is not None:  # the 1/world averaging rides in the Adam launch
            self.eng.adam_step(grad_scale=1.0 / self.avg.world)

    # ------------------------------------------------------------ buckets
    def _bucket_dec(self):
        self.avg.bucket_ready(self.eng.params.grad[self._split:])

    def _bucket_enc_and_finish(self):
        grad = self.eng.params.grad
        self.avg.bucket_ready(grad[:self._split])
        self.avg.finish(grad, scale=False)

    # ------------------------------------------------------------ running
    def eager_step(self):
        """One whole step in stream order (also what a one-graph capture records)."""
        self.part_a()
        if self.avg is not None:
            self._bucket_dec()
        self.part_b()
        if self.avg is not None:
            self._bucket_enc_and_finish()
        self.part_c()

    def capture(self):
        """One real eager step on a side stream (lazy initialisation of
        everything the launches touch, RCCL's communicator included), then
        record the graph(s)."""
        dev = self.eng.device
        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            self.eager_step()
        torch.cuda.current_stream(dev).wait_stream(s)
        torch.cuda.synchronize(dev)
        if self.one_graph:
            try:
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, capture_error_mode=_CAPTURE_MODE):
                    self.eager_step()
                self.graphs = [g]
                return
            except RuntimeError as e:
                # a collective the backend refused to record (nothing ran
                # during the capture): fall back to the three-graph structure,
                # the collectives issued by the host between the replays
                if self.avg is None:
                    raise
                self.avg._works.clear()
                self.fallback = f"collectives not capturable: {e!r}"[:300]
                self.one_graph = False
                torch.cuda.synchronize(dev)
        self.graphs = [torch.cuda.CUDAGraph() for _ in range(3)]
        for g, fn in zip(self.graphs, (self.part_a, self.part_b, self.part_c)):
            with torch.cuda.graph(g, capture_error_mode=_CAPTURE_MODE):
                fn()

    def capture_multi(self):
        """Record (once) the graph holding ``steps_per_graph`` whole steps,
        which :meth:`run` replays k // steps_per_graph times: the per-replay
        host gap (~8 us between consecutive replays) is paid once per that
        many steps.  Nothing runs while recording."""
        if self.graph_multi is None and self.graphs is not None and self.one_graph and self.steps_per_graph > 1:
            try:
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, capture_error_mode=_CAPTURE_MODE):
                    for _ in range(self.steps_per_graph):
                        self.eager_step()
                self.graph_multi = g
            except RuntimeError as e:  # keep replaying the one-step graph
                if self.avg is None:
                    raise
                self.avg._works.clear()
                self.fallback = f"multi-step graph not capturable: {e!r}"[:300]
                self.steps_per_graph = 1
                torch.cuda.synchronize(self.eng.device)

    capture_pair = capture_multi  # (round-4 name)

    def step(self):
        if self.graphs is None:
            return self.eager_step()
        if self.one_graph:
            self.graphs[0].replay()
            return
        ga, gb, gc = self.graphs
        ga.replay()
        self._bucket_dec()          # overlaps with gb
        gb.replay()
        self._bucket_enc_and_finish()
        gc.replay()

    __call__ = step

    def run(self, k):
        """``k`` training steps (the same steps as ``k`` calls of :meth:`step`);
        a one-graph runner replays the multi-step graph."""
        if self.graphs is not None and self.one_graph:
            if k >= self.steps_per_graph > 1:
                self.capture_multi()
            n = self.steps_per_graph if self.graph_multi is not None else 1
            if n > 1:
                for _ in range(k // n):
                    self.graph_multi.replay()
                k %= n
            for _ in range(k):
                self.graphs[0].replay()
            return
        for _ in range(k):
            self.step()
