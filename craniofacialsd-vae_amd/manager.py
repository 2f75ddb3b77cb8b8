"""``ModelManager`` for the libcfsd training path: the reference's
orchestration (``model_manager.py:34-148`` construction, ``:176-238``
precompute / latent regions, ``:257-326`` run_epoch / _do_iteration,
``:575-592`` loss bookkeeping, ``:682-706`` checkpoints) driving
:class:`engine.SDVAEEngine` on resident data.

Differences by design (the reference's CPU loader and per-step host syncs are
what the MI355X path removes): batches come from :class:`engine.ResidentData`
(device-drawn epoch shuffle + on-device swap inside the step), the seven
``.item()`` per step become one device accumulator read per epoch, and the
train step can be replayed from a hipGraph.  Rendering, TensorBoard images
and the sklearn classifiers are out of scope.
"""
import json
import os

import numpy as np
import torch

from . import engine as E
from . import ops, precompute, refcache, topology
from .step import TrainStep

LOSS_KEYS = ["reconstruction", "kl", "latent_consistency", "laplacian", "classification",
             "classification_acc", "tot"]


def load_config(path):
    """``utils.get_config`` (utils.py:64-66)."""
    import yaml
    with open(path) as f:
        return yaml.safe_load(f)


def prepare_sub_folder(output_directory):
    """``utils.prepare_sub_folder`` (utils.py:69-74)."""
    d = os.path.join(output_directory, "checkpoints")
    os.makedirs(d, exist_ok=True)
    return d


def load_or_build_topology(config, template, precomputed_path):
    """The static geometry the model consumes (model_manager.py:176-230):
    ``topology.npz`` in ``precomputed_path`` (this package's cache), else the
    reference's own ``spirals.pkl`` + ``transforms.pkl`` (read without
    executing them), else built from the template by
    :func:`precompute.build_hierarchy` and cached.  Regions and Laplacian
    always come from the template (utils.py:77-144)."""
    os.makedirs(precomputed_path, exist_ok=True)
    cache = os.path.join(precomputed_path, "topology.npz")
    if os.path.exists(cache):
        return dict(np.load(cache))
    mp = config["model"]
    if os.path.exists(os.path.join(precomputed_path, "spirals.pkl")) and \
            os.path.exists(os.path.join(precomputed_path, "transforms.pkl")):
        h = refcache.load_precomputed(precomputed_path)
        h["pos_0"], h["face_0"] = template.pos, template.faces.astype(np.int32)
    else:
        h = precompute.build_hierarchy(template.pos, template.faces, template.colors,
                                       mp["sampling"]["sampling_factors"], mp["spirals"]["length"],
                                       mp["spirals"].get("dilation"), mp["sampling"].get("type", "basic"))
    if template.feat_and_cont is not None and "region_keys" not in h:  # (a fresh build wrote its own,
        keys = list(template.feat_and_cont.keys())                   # r_weighted-extended ones)
        h["region_keys"] = np.asarray(keys)
        for i, k in enumerate(keys):
            h[f"region_{i}_feature"] = np.asarray(template.feat_and_cont[k]["feature"], np.int32)
            h[f"region_{i}_contour"] = np.asarray(template.feat_and_cont[k]["contour"], np.int32)
    h["lap_row"], h["lap_col"], h["lap_val"] = template.laplacian
    np.savez(cache, **h)
    return h


class JsonlWriter:
    """``SummaryWriter.add_scalar`` subset writing JSON lines (tensorboard is
    not installed in this image)."""

    def __init__(self, log_dir):
        os.makedirs(log_dir, exist_ok=True)
        self.path = os.path.join(log_dir, "scalars.jsonl")

    def add_scalar(self, tag, value, step):
        with open(self.path, "a") as f:
            f.write(json.dumps({"tag": tag, "value": float(value), "step": int(step)}) + "\n")


class ModelManager:
    def __init__(self, configurations, device="cuda", precomputed_storage_path="precomputed",
                 precision="fp32", seed=0, use_graph=True, averager=None):
        self._model_params = configurations["model"]
        self._optimization_params = op = configurations["optimization"]
        self._precomputed_storage_path = precomputed_storage_path
        self._normalized_data = configurations["data"].get("normalize_data", True)
        self.to_mm_const = configurations["data"].get("to_mm_constant", 1.0)
        self.device = torch.device(device)
        self._swap_features = bool(configurations["data"].get("swap_features", True))
        if float(configurations["optimization"]["latent_consistency_weight"]) > 0 and not self._swap_features:
            # model_manager.py:93-94 (assert self._swap_features): the latent
            # consistency loss is defined on swapped bs x bs groups only
            raise ValueError("latent_consistency_weight > 0 needs data.swap_features: True")
        self.template = precompute.load_template(configurations["data"]["template_path"])
        self.topology_arrays = load_or_build_topology(configurations, self.template, precomputed_storage_path)
        self.topology = topology.DeviceTopology.from_npz(self.topology_arrays, device=self.device)
        self._w_latent_cons_loss = float(op["latent_consistency_weight"])
        self._w_laplacian_loss = float(op["laplacian_weight"])
        self._w_kl_loss = float(op["kl_weight"])
        mp = self._model_params
        spec = E.ModelSpec(mp["in_channels"], mp["out_channels"], mp["latent_size"],
                           is_vae=self._w_kl_loss > 0, pre_z_sigmoid=mp.get("pre_z_sigmoid", False))
        self.bs = int(op["batch_size"])
        self.engine = E.SDVAEEngine(
            self.topology, spec, lr=float(op["lr"]), weight_decay=float(op["weight_decay"]),
            w_kl=self._w_kl_loss, w_lc=self._w_latent_cons_loss, w_lap=self._w_laplacian_loss,
            eta1=float(op.get("latent_consistency_eta1", 0.5)), eta2=float(op.get("latent_consistency_eta2", 0.5)),
            swap_bs=self.bs, seed=seed, device=self.device, precision=precision,
            swap_features=self._swap_features)
        self._latent_regions = self._compute_latent_regions()
        self._batch_diagonal_idx = [(self.bs + 1) * i for i in range(self.bs)]
        self._losses = None
        self.use_graph = use_graph
        self._steps = {}
        # data-parallel (one process per GPU, train.py under torchrun): every
        # rank starts from rank 0's parameters and averages the gradient
        self.averager = averager
        if averager is not None and averager.world > 1:
            from .dist import broadcast_parameters
            broadcast_parameters(self.engine.params.data, 0)
            self.engine.sync_shadow()
        self.val_acc = torch.zeros(6, dtype=torch.float32, device=self.device)
        self.val_counter = torch.zeros(1, dtype=torch.int32, device=self.device)

    # ------------------------------------------------------------ properties
    @property
    def loss_keys(self):
        return list(LOSS_KEYS)

    @property
    def latent_regions(self):
        return self._latent_regions

    @property
    def is_vae(self):
        return self._w_kl_loss > 0

    @property
    def batch_diagonal_idx(self):
        return self._batch_diagonal_idx

    def _compute_latent_regions(self):
        """model_manager.py:232-238: latent dims [i*size, (i+1)*size) per region."""
        names = list(self.template.feat_and_cont.keys())
        latent = self._model_params["latent_size"]
        assert latent % len(names) == 0
        size = latent // len(names)
        return {k: [i * size, (i + 1) * size] for i, k in enumerate(names)}

    # ------------------------------------------------------------ epochs
    def _train_step(self, b, data):
        """One training step from ``data`` through :class:`step.TrainStep`
        (the object bench.py times).  With ``use_graph`` the first step of a
        data set runs eagerly on a side stream and is captured; later steps
        replay the graph(s)."""
        ts = self._steps.get(id(data))
        if ts is None or ts.data is not data:
            ts = TrainStep(self.engine, data, self.averager, acc=self.engine.loss_acc)
            self._steps[id(data)] = ts
            if self.use_graph:
                ts.capture()  # includes one real (eager) step
                return "captured"
        ts.step()

    def _eval_step(self, b, data):
        """_do_iteration(train=False) (model_manager.py:274-326 under
        torch.no_grad(), eval mode: z = mu): the validation loader's shuffled,
        swapped batch on the device, forward + the four losses only."""
        eng, T = self.engine, self.topology
        ops.step_begin(self.val_counter, eng.seed + 7919, key=b.key, n_regions=max(T.n_regions, 1),
                       batch_idx=b.batch_idx, bs=self.bs, n_batches=data.n_batches, perm=data.rows,
                       n_items=data.n_items, shuffle=data.shuffle)
        eng.load_batch(b, data)
        eng.forward(b, train=False, acc=self.val_acc, finalize=True)

    def run_epoch(self, data, train=True, record=None):
        """``ModelManager.run_epoch`` (model_manager.py:257-272): every batch
        of one (shuffled, drop_last) epoch; returns and stores the per-batch
        mean of the losses (``_reset/_add/_divide_losses``).  ``record`` (a
        list) receives (batch_idx, key, eps) of every step (parity tests)."""
        b = self.engine.buffers(self.engine.step_rows)
        acc = self.engine.loss_acc if train else self.val_acc
        acc.zero_()
        # writes made through ``net`` (a torch optimizer on its parameters,
        # net.load_state_dict) reach the fp32 master but not the bf16 shadow
        # the bf16 kernels read: refresh it once per epoch (one cast launch)
        self.engine.sync_shadow()
        steps_done = 0
        while steps_done < data.n_batches:
            if train:
                r = self._train_step(b, data)
                steps_done += 1
                if record is not None and r == "captured":
                    raise RuntimeError("record=... needs use_graph=False")
            else:
                self._eval_step(b, data)
                steps_done += 1
            if record is not None:
                record.append((b.batch_idx.cpu().numpy().copy(), int(b.key.item()),
                               b.eps.cpu().numpy().copy() if (train and self.is_vae) else None))
        if self.averager is not None and self.averager.world > 1:
            import torch.distributed as dist
            dist.all_reduce(acc)  # every rank's batches: sums and the batch count
        a = acc.cpu().numpy().astype(np.float64)
        if train:
            self.engine.check_health()  # a timed-out device wait invalidates the epoch: fail loudly
        n = max(a[5], 1.0)
        self._losses = {"reconstruction": a[0] / n, "kl": a[1] / n, "latent_consistency": a[2] / n,
                        "laplacian": a[3] / n, "classification": 0.0, "classification_acc": 0.0,
                        "tot": a[4] / n}
        return dict(self._losses)

    def log_losses(self, writer, epoch, phase="train", losses=None):
        """model_manager.py:587-592 (``losses``: a run_epoch result; default
        the last one)."""
        losses = self._losses if losses is None else losses
        for k in self.loss_keys:
            writer.add_scalar(phase + "/" + str(k), losses[k], epoch + 1)

    # ------------------------------------------------------------ model access
    @property
    def net(self):
        """The drop-in :class:`model.Model` (``ModelManager._net``,
        ``model_manager.py:60-67``) over the engine's parameter STORAGE: its
        ``nn.Parameter``s are views of the flat buffer, so the engine's Adam
        updates are what it computes with.  Autograd runs through libcfsd
        (``model.py`` autograd Functions); parameter gradients it produces
        land in the module's own ``.grad`` tensors, not in the engine's.
        Read-mostly: a write through it (an optimizer step on its parameters,
        ``load_state_dict``) updates the fp32 master; in bf16 mode call
        :meth:`sync_from_net` afterwards (``run_epoch`` also refreshes the
        bf16 shadow at every epoch start)."""
        if getattr(self, "_net", None) is None:
            self._net = _engine_model(self.engine, self.topology_arrays, self._model_params, self.device)
        return self._net

    def sync_from_net(self):
        """Refresh the engine's bf16 weight shadow after writes made through
        :attr:`net` (no-op in fp32)."""
        self.engine.sync_shadow()

    def forward(self, data):
        """``ModelManager.forward`` (``model_manager.py:240-241``):
        ``self._net(data.x)`` in the module's current train / eval mode, with
        autograd.  ``data``: an object with ``.x`` [B, V, 3] (a ``Data``
        batch) or the tensor itself."""
        x = data.x if hasattr(data, "x") else data
        return self.net(x.to(self.device))

    def generate_for_opt(self, z):
        """``ModelManager.generate_for_opt`` (``model_manager.py:253-255``):
        decode in train mode WITH autograd, so a caller can optimise ``z``
        (the reference's latent fitting).  Returns [N, V, 3]."""
        self.net.train()
        return self.net.decode(z.to(self.device))

    def encode(self, x):
        """Eval-mode latents of device meshes [N, V, 3] (model_manager.py:243-246)."""
        return self.engine.encode_all(x, batch_size=self.bs * self.bs)

    def generate(self, z):
        """Decoder output for latents [N, latent] (model_manager.py:248-251)."""
        outs = []
        for s in range(0, z.shape[0], self.bs * self.bs):
            zz = z[s:s + self.bs * self.bs].contiguous()
            b = self.engine.buffers(zz.shape[0])
            self.engine.decode(b, z=zz)
            outs.append(b.out.clone())
        return torch.cat(outs)

    def compute_vertex_errors(self, out, gt):
        """model_manager.py:395-400 (on device)."""
        return ops.vertex_errors(out.contiguous(), gt.contiguous(), to_mm=self.to_mm_const)

    def save_weights(self, checkpoint_dir, epoch):
        return self.engine.save_weights(checkpoint_dir, epoch)

    def resume(self, checkpoint_dir):
        return self.engine.resume(checkpoint_dir)


def _engine_model(engine, arrays, model_params, device):
    """A :class:`model.Model` built from the precomputed topology (int64
    spirals, sparse-COO transforms in file order, as the reference unpickles
    them) whose parameters are re-bound to views of ``engine.params.data``."""
    import torch.nn as nn

    from . import model as M
    n = int(arrays["n_levels"])
    spirals = [torch.from_numpy(np.asarray(arrays[f"spiral_{l}"], np.int64)).to(device) for l in range(n)]

    def sp(name, l):
        idx = np.stack([arrays[f"{name}_{l}_row"], arrays[f"{name}_{l}_col"]]).astype(np.int64)
        return torch.sparse_coo_tensor(torch.from_numpy(idx),
                                       torch.from_numpy(np.asarray(arrays[f"{name}_{l}_val"], np.float32)),
                                       tuple(np.asarray(arrays[f"{name}_{l}_shape"]).tolist()))

    S = engine.spec
    net = M.Model(S.in_ch, S.out_ch, S.latent, spirals, [sp("down", l) for l in range(n)],
                  [sp("up", l) for l in range(n)], pre_z_sigmoid=bool(model_params.get("pre_z_sigmoid", False)),
                  is_vae=S.is_vae).to(device)
    for name, _ in list(net.named_parameters()):
        *path, leaf = name.split(".")
        mod = net
        for p in path:
            mod = getattr(mod, p)
        setattr(mod, leaf, nn.Parameter(engine.params.view(name)))  # shares the flat buffer's storage
    return net
