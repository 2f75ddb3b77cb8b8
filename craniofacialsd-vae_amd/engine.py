"""The SD-VAE training step as an explicit launch sequence on libcfsd.

Reference call stack being replaced: ``ModelManager._do_iteration``
(``model_manager.py:274-326``) -> ``Model.forward`` (``model.py:175-182``) ->
losses -> ``loss_tot.backward()`` -> ``Adam.step()``, with the batch built by
``SwapFeatures`` in DataLoader workers (``swap_batch_transform.py:13-42``).

MI355X design:
* parameters, gradients and Adam moments live in ONE flat fp32 buffer each
  (named views keep the reference ``state_dict`` keys), so data-parallel
  training all-reduces one contiguous bucket and Adam is one launch;
* every activation/gradient buffer is allocated once per batch size, so the
  whole step (swap -> forward -> 4 losses -> backward -> Adam) is a fixed
  sequence of ~60 kernel launches that is captured once into a hipGraph and
  replayed; nothing in the step synchronises with the host (losses are
  accumulated on device, unlike the reference's seven ``.item()`` calls);
* the backward is hand-derived and fused (ELU backward in the producer's
  epilogue, deterministic gather-based transposes, no atomics).
"""
import math
import os

import numpy as np
import torch

from . import ops
from .ops import ACT_ELU, ACT_NONE


class ModelSpec:
    """Architecture of ``Model`` (``model.py:88-137``)."""

    def __init__(self, in_channels=3, out_channels=(32, 32, 32, 64), latent_size=75,
                 is_vae=True, pre_z_sigmoid=False):
        self.in_ch = int(in_channels)
        self.out_ch = [int(c) for c in out_channels]
        self.latent = int(latent_size)
        self.is_vae = bool(is_vae)
        self.sigmoid = bool(pre_z_sigmoid) and not self.is_vae
        self.n = len(self.out_ch)

    def enc_layers(self):
        """(cin, cout, level) of the Enblock convs."""
        return [((self.in_ch if i == 0 else self.out_ch[i - 1]), self.out_ch[i], i)
                for i in range(self.n)]

    def dec_layers(self):
        """(cin, cout, level, up_index) of de_layers[1..n] (model.py:125-134)."""
        out = []
        for idx in range(self.n):
            if idx == 0:
                cin, cout = self.out_ch[-1], self.out_ch[-1]
            else:
                cin, cout = self.out_ch[-idx], self.out_ch[-idx - 1]
            level = self.n - 1 - idx
            out.append((cin, cout, level, self.n - (idx + 1)))
        return out

    def param_specs(self, num_vert, seq):
        """(name, shape) in FLAT-BUFFER order.  The two encoder Linears are
        stacked [logvar; mu] so one GEMM produces both (mu = en_layers[-1],
        logvar = en_layers[-2], model.py:153-156)."""
        n, lat, c_last = self.n, self.latent, self.out_ch[-1]
        flat_in = num_vert * c_last
        specs = []
        for (cin, cout, lv) in self.enc_layers():
            specs.append((f"en_layers.{lv}.conv.layer.weight", (cout, seq[lv] * cin)))
            specs.append((f"en_layers.{lv}.conv.layer.bias", (cout,)))
        if self.is_vae:
            specs += [(f"en_layers.{n}.weight", (lat, flat_in)), (f"en_layers.{n + 1}.weight", (lat, flat_in)),
                      (f"en_layers.{n}.bias", (lat,)), (f"en_layers.{n + 1}.bias", (lat,))]
        else:
            specs += [(f"en_layers.{n}.weight", (lat, flat_in)), (f"en_layers.{n}.bias", (lat,))]
        specs += [("de_layers.0.weight", (flat_in, lat)), ("de_layers.0.bias", (flat_in,))]
        for i, (cin, cout, lv, _) in enumerate(self.dec_layers()):
            specs.append((f"de_layers.{i + 1}.conv.layer.weight", (cout, seq[lv] * cin)))
            specs.append((f"de_layers.{i + 1}.conv.layer.bias", (cout,)))
        specs.append((f"de_layers.{n + 1}.layer.weight", (self.in_ch, seq[0] * self.out_ch[0])))
        specs.append((f"de_layers.{n + 1}.layer.bias", (self.in_ch,)))
        return specs

    def reference_order(self, num_vert, seq):
        """Parameter names in the reference ``named_parameters`` order."""
        n = self.n
        names = [k for k, _ in self.param_specs(num_vert, seq)]
        enc_lin = [f"en_layers.{n}.weight", f"en_layers.{n}.bias"]
        if self.is_vae:
            enc_lin += [f"en_layers.{n + 1}.weight", f"en_layers.{n + 1}.bias"]
        convs = [k for k in names if k.startswith("en_layers") and ".conv." in k]
        rest = [k for k in names if k.startswith("de_layers")]
        return convs + enc_lin + rest


class FlatParams:
    """One contiguous fp32 buffer for params / grads / Adam moments."""

    def __init__(self, specs, device):
        self.specs = list(specs)
        self.offsets = {}
        off = 0
        for name, shape in self.specs:
            self.offsets[name] = (off, tuple(shape))
            off += int(np.prod(shape))
        self.numel = off
        self.data = torch.zeros(off, dtype=torch.float32, device=device)
        self.grad = torch.zeros(off, dtype=torch.float32, device=device)
        self.exp_avg = torch.zeros(off, dtype=torch.float32, device=device)
        self.exp_avg_sq = torch.zeros(off, dtype=torch.float32, device=device)
        self.step = torch.zeros(1, dtype=torch.int32, device=device)
        self.shadow = None  # bf16 copy of `data` (precision "bf16"), refreshed by Adam

    def view(self, name, buf=None):
        off, shape = self.offsets[name]
        b = self.data if buf is None else buf
        return b[off:off + int(np.prod(shape))].view(shape)

    def gview(self, name):
        return self.view(name, self.grad)

    def span(self, first, last, buf=None):
        """Contiguous view from the start of ``first`` to the end of ``last``."""
        b = self.data if buf is None else buf
        o0, _ = self.offsets[first]
        o1, s1 = self.offsets[last]
        return b[o0:o1 + int(np.prod(s1))]


class _Buffers:
    pass


class SDVAEEngine:
    """Forward/backward/Adam of the SD-VAE on one device, for a fixed
    topology and any number of batch sizes (buffers cached per batch)."""

    def __init__(self, topo, spec=None, lr=1e-4, weight_decay=0.0, w_kl=1e-4, w_lc=0.5,
                 w_lap=0.1, eta1=0.5, eta2=0.5, swap_bs=4, seed=0, device="cuda", precision="fp32",
                 vertex_major=True, swap_features=True):
        """``precision``: "fp32" (the reference's arithmetic, the parity
        configuration) or "bf16" (configs C3/C5: the level-0/1 activations
        and gradients -- the large tensors -- stored in bf16 and VERTEX-MAJOR
        (``ops.is_vm``: the 16 mesh rows of a vertex are one contiguous 1-KiB
        block, so every spiral gather is a coalesced wave load), their convs
        on bf16 MFMA with the bf16 shadow of the fp32 master weights, fp32
        accumulation; the network input / output, coarse levels, bottleneck,
        losses, gradients and Adam stay fp32 batch-major).

        ``vertex_major`` (fp32): store the level-0/1 32-channel tensors
        vertex-major too, for batches that are a multiple of 16 (the fp32
        vertex-major kernels: same forward outputs bit for bit, the data
        gradient through the flat inverse list); False keeps every fp32 tensor
        batch-major (the reference's [B, V, C])."""
        if precision not in ("fp32", "bf16"):
            raise ValueError(f"precision must be 'fp32' or 'bf16', got {precision!r}")
        self.precision = precision
        self.topo = topo
        self.spec = spec or ModelSpec()
        self.device = torch.device(device)
        self.lr, self.weight_decay = float(lr), float(weight_decay)
        self.w_kl = float(w_kl) if self.spec.is_vae else 0.0
        self.w_lc, self.w_lap = float(w_lc), float(w_lap)
        self.eta1, self.eta2 = float(eta1), float(eta2)
        self.swap_bs = int(swap_bs)
        # data config swap_features (data_loading.py:38): a train step is the
        # bs^2 swapped meshes of bs base meshes, or (False) the bs meshes
        # themselves with the latent-consistency term 0 (model_manager.py:290-293)
        self.swap = bool(swap_features)
        self.seed = int(seed)
        if topo.n_levels != self.spec.n:
            raise ValueError(f"topology has {topo.n_levels} levels, model {self.spec.n}")
        if topo.lap_csr is None:
            raise ValueError("SDVAEEngine needs the template's Laplacian (utils.load_template, "
                             "utils.py:88-89): the training losses are MSE + Laplacian (+ KL, LC)")
        self.num_vert = topo.n_verts[-1]
        self.params = FlatParams(self.spec.param_specs(self.num_vert, topo.seq), self.device)
        # levels whose tensors are bf16 (the two finest; never the bottleneck)
        self.lp_levels = set()
        if precision == "bf16":
            if not all(topo.enc_select) or self.spec.n < 3:
                raise ValueError("bf16 precision needs 0/1 selection down-sampling and >= 3 levels")
            self.lp_levels = {0, 1}
            self.params.shadow = torch.zeros(self.params.numel, dtype=torch.bfloat16, device=self.device)
        self.vertex_major = bool(vertex_major)
        self.fuse_up = True  # coarse Deblocks: Pool(up) fused into the conv gather (False: separate SpMM)
        self.fuse_latent = True  # latent head + decoder Linear in one launch (False: two)
        # One default path per layer.  The attributes below select the fused
        # launches; the separate launches they replace stay as the general
        # fallback (shapes the fused kernels do not take) and as the bit-identity
        # references of the GPU tests.
        # the bottleneck backward (coarsest Pool(up)^T, decoder Linear, latent
        # head, encoder Linear) as one launch (cfsd_bottleneck_bwd).  Its
        # workgroups wait on counters for lower-index workgroups, which is
        # deadlock-free only while no OTHER such launch holds the device's
        # slots: ranks sharing one GPU (CFSD_SHARE_DEVICE rehearsals) take the
        # four bit-identical launches instead (a world-2 shared-device bench hit
        # the kernel's timed-out-wait guard)
        self.fuse_bottleneck = not os.environ.get("CFSD_SHARE_DEVICE")
        # the feature swap and the first Enblock's conv as one launch (cfsd_spiral_conv_fwd_in_swap)
        self.fuse_swap = True
        # vertex-major levels whose fp32 Deblock backward runs as one dx + dW launch
        # (cfsd_spiral_conv_bwd_flat_pair): level 1 (D2: 37.8 vs 20.8 + 19.9 us,
        # step 0.563 vs 0.568 ms same-box); at level 0 the pair is slower (117.5 vs
        # 51.4 + 52.0 us: the dx role's 12-wave workgroups lose to its 2-per-CU kernel)
        self.vm_pair_levels = {1}
        # the bf16 step's pair (cfsd_spiral_conv_bwd_flat_pair_bf16) at both vertex-major
        # levels: D3 29.0 vs 20.0 + 19.0 us, D2 14.7 vs 10.4 + 11.6 us, step 0.427 -> 0.409 ms;
        # and the bf16 Enblock's dx + dW pair (cfsd_spiral_conv_bwd_rowsub_pair_bf16)
        self.rowsub_pair16 = True
        self.vm_pair_levels16 = {0, 1}
        n_reg = topo.n_regions if topo.n_regions else 1
        self.region_size = self.spec.latent // n_reg if topo.n_regions else 0
        if topo.n_regions and self.w_lc and self.spec.latent % n_reg:
            raise ValueError("latent_size must be a multiple of the number of regions")
        self.reset_parameters()
        self._bufs = {}
        self.loss_acc = torch.zeros(6, dtype=torch.float32, device=self.device)
        self.betas, self.adam_eps = (0.9, 0.999), 1e-8
        # device step counter: drives the VAE noise, swap key and batch order
        # of cfsd_step_begin (one per engine, re-seeded by resume())
        self.counter = torch.zeros(1, dtype=torch.int32, device=self.device)

    # ----------------------------------------------------------- parameters
    def reset_parameters(self, generator=None):
        """``Model.reset_parameters`` (model.py:139-144): xavier-uniform
        weights, zero biases."""
        for name, shape in self.params.specs:
            v = self.params.view(name)
            if name.endswith("bias"):
                v.zero_()
            else:
                fan_out, fan_in = shape
                a = math.sqrt(6.0 / (fan_in + fan_out))
                v.uniform_(-a, a, generator=generator)
        self.sync_shadow()

    def sync_shadow(self):
        """Refresh the bf16 weight shadow from the fp32 master (bf16 mode)."""
        if self.params.shadow is not None and self.device.type == "cuda":
            ops.cast(self.params.data, self.params.shadow)

    def state_dict(self):
        n, order = self.spec.n, self.spec.reference_order(self.num_vert, self.topo.seq)
        return {k: self.params.view(k).detach().clone() for k in order}

    def load_state_dict(self, sd):
        for name, shape in self.params.specs:
            t = sd[name]
            if tuple(t.shape) != tuple(shape):
                raise ValueError(f"{name}: shape {tuple(t.shape)} != {shape}")
            self.params.view(name).copy_(t.to(self.device, torch.float32))
        self.sync_shadow()

    def grads(self):
        return {k: self.params.gview(k) for k, _ in self.params.specs}

    # ----------------------------------------------------------- evaluation
    def encode_all(self, meshes, batch_size=16):
        """``ModelManager.encode_all`` / ``encode`` (``model_manager.py:244-246,
        402-426``): eval-mode latents (mu; sigmoid(mu) for a pre_z_sigmoid AE)
        of device meshes ``[N, V, 3]`` (already un-swapped), in batches
        (ragged tail allowed).  Returns a device tensor ``[N, latent]``."""
        out = []
        for s in range(0, meshes.shape[0], batch_size):
            b = self.set_batch(meshes[s:s + batch_size])
            self.encode(b)
            self.latent(b, train=False)
            out.append(b.z.clone())
        return torch.cat(out, dim=0)

    @staticmethod
    def latent_stats(latents):
        """``Tester.compute_latent_stats`` (``test.py:95-117``) of device
        latents: per-dimension means / stds / mins / maxs (torch reductions)."""
        return {"means": torch.mean(latents, dim=0), "stds": torch.std(latents, dim=0),
                "mins": torch.min(latents, dim=0)[0], "maxs": torch.max(latents, dim=0)[0]}

    # ----------------------------------------------------------- checkpoints
    def optimizer_state_dict(self):
        """The ``torch.optim.Adam.state_dict()`` the reference's optimiser
        (``model_manager.py:69-72``, over ``Model.parameters()``) would hold
        after the same steps: parameter ids in ``named_parameters`` order,
        per-parameter ``step`` / ``exp_avg`` / ``exp_avg_sq`` (CPU tensors)."""
        P, order = self.params, self.spec.reference_order(self.num_vert, self.topo.seq)
        t = int(P.step.item())
        group = dict(torch.optim.Adam([torch.zeros(1)], lr=self.lr,
                                      weight_decay=self.weight_decay).state_dict()["param_groups"][0])
        group["params"] = list(range(len(order)))
        state = {}
        if t > 0:
            for i, k in enumerate(order):
                state[i] = {"step": torch.tensor(float(t)),
                            "exp_avg": P.view(k, P.exp_avg).detach().cpu().clone(),
                            "exp_avg_sq": P.view(k, P.exp_avg_sq).detach().cpu().clone()}
        return {"state": state, "param_groups": [group]}

    def load_optimizer_state_dict(self, sd):
        """Inverse of :meth:`optimizer_state_dict` (accepts a reference
        ``optimizer.pt`` payload); all parameters must share one ``step``."""
        P, order = self.params, self.spec.reference_order(self.num_vert, self.topo.seq)
        groups = sd["param_groups"]
        ids = [i for g in groups for i in g["params"]]
        if len(ids) != len(order):
            raise ValueError(f"optimizer state has {len(ids)} parameters, model {len(order)}")
        self.lr = float(groups[0]["lr"])
        self.weight_decay = float(groups[0]["weight_decay"])
        self.betas = tuple(float(b) for b in groups[0].get("betas", (0.9, 0.999)))
        self.adam_eps = float(groups[0].get("eps", 1e-8))
        if groups[0].get("amsgrad", False) or groups[0].get("maximize", False):
            raise ValueError("amsgrad / maximize Adam variants are not supported")
        steps = set()
        for i, k in zip(ids, order):
            st = sd["state"].get(i)
            if st is None:
                P.view(k, P.exp_avg).zero_()
                P.view(k, P.exp_avg_sq).zero_()
                steps.add(0)
                continue
            _, shape = P.offsets[k]
            for key, buf in (("exp_avg", P.exp_avg), ("exp_avg_sq", P.exp_avg_sq)):
                if tuple(st[key].shape) != tuple(shape):
                    raise ValueError(f"{k}.{key}: shape {tuple(st[key].shape)} != {shape}")
                P.view(k, buf).copy_(st[key].to(self.device, torch.float32))
            steps.add(int(float(st["step"])))
        if len(steps) != 1:
            raise ValueError(f"parameters at different Adam steps {sorted(steps)}")
        P.step.fill_(steps.pop())
        # the noise / swap-key / batch stream continues where it stopped
        self.counter.copy_(P.step)

    def save_weights(self, checkpoint_dir, epoch):
        """``ModelManager.save_weights`` (``model_manager.py:682-688``):
        ``model_%08d.pt`` = {'model': state_dict} (reference keys) and
        ``optimizer.pt`` = {'optimizer': Adam state_dict}."""
        import os
        net_name = os.path.join(checkpoint_dir, "model_%08d.pt" % (epoch + 1))
        torch.save({"model": {k: v.cpu() for k, v in self.state_dict().items()}}, net_name)
        torch.save({"optimizer": self.optimizer_state_dict()},
                   os.path.join(checkpoint_dir, "optimizer.pt"))
        return net_name

    def resume(self, checkpoint_dir):
        """``ModelManager.resume`` (``model_manager.py:690-706``, last model by
        ``utils.get_model_list`` ``utils.py:180-190``); loads with
        ``weights_only=True``.  Returns the epoch count."""
        import os
        names = sorted(f for f in os.listdir(checkpoint_dir)
                       if os.path.isfile(os.path.join(checkpoint_dir, f)) and "model" in f and ".pt" in f)
        if not names:
            raise FileNotFoundError(f"no model checkpoint in {checkpoint_dir}")
        last = os.path.join(checkpoint_dir, names[-1])
        self.load_state_dict(torch.load(last, map_location="cpu", weights_only=True)["model"])
        opt = torch.load(os.path.join(checkpoint_dir, "optimizer.pt"), map_location="cpu",
                         weights_only=True)
        self.load_optimizer_state_dict(opt["optimizer"])
        return int(last[-11:-3])

    # ----------------------------------------------------------- buffers
    def vm_levels(self, bsz):
        """Levels whose 32-channel tensors are stored vertex-major (and routed
        through the mixed / vertex-major entry points) at batch ``bsz``: the
        bf16 levels always; in fp32 levels 0 and 1 when the batch is a
        multiple of 16, every down-sampling is a 0/1 selection, and the level's
        convs fit the fp32 vertex-major kernels (32 -> 32/64 with flat
        inverse lists)."""
        if self.lp_levels:
            return set(self.lp_levels)
        T, S = self.topo, self.spec
        if not (self.vertex_major and bsz % 16 == 0 and all(T.enc_select) and S.n >= 3):
            return set()
        for (cin, cout, lv, _) in S.dec_layers():
            if lv in (0, 1) and not (cin == 32 and cout in (32, 64) and T.spiral_flat[lv] is not None):
                return set()
        for (cin, cout, lv) in S.enc_layers():
            if lv == 1 and not (cin == 32 and cout in (32, 64) and T.enc_flat[1] is not None):
                return set()
        if S.enc_layers()[0][0] > 3 or S.out_ch[0] != 32:
            return set()
        return {0, 1}

    def buffers(self, bsz):
        if bsz in self._bufs:
            return self._bufs[bsz]
        T, S, dev = self.topo, self.spec, self.device
        f = lambda *shape: torch.empty(shape, dtype=torch.float32, device=dev)  # noqa: E731
        lp = self.vm_levels(bsz)  # vertex-major levels (bf16 in bf16 mode)
        ldt = torch.bfloat16 if self.lp_levels else torch.float32

        def fl(level, *shape):  # storage of a level's activation / gradient
            if level in lp:  # vertex-major (ops.is_vm): a vertex's 16 mesh rows = one contiguous block
                return ops.vm_empty(*shape, dtype=ldt, device=dev)
            return torch.empty(shape, dtype=torch.float32, device=dev)

        b = _Buffers()
        b.bsz = bsz
        b.xl = lp
        nv = T.n_verts
        lat = S.latent
        last_enc = S.enc_layers()[-1][2]
        # the xyz tensors of level 0 (input, output, Laplacian unit vectors,
        # output gradient) share level 0's layout; fp32 always
        f0 = ((lambda *shape: ops.vm_empty(*shape, dtype=torch.float32, device=dev)) if 0 in lp else f)
        b.x = f0(bsz, nv[0], S.in_ch)
        b.enc_full = [None] * S.n     # full-resolution conv outputs (non-selection path)
        b.enc_out = []                # pooled Enblock outputs [B, V_{i+1}, C_i]
        for (cin, cout, lv) in S.enc_layers():
            if not T.enc_select[lv]:
                b.enc_full[lv] = f(bsz, nv[lv], cout)
            b.enc_out.append(f(bsz, nv[lv + 1], cout) if lv == last_enc else fl(lv + 1, bsz, nv[lv + 1], cout))
        nmulv = 2 * lat if S.is_vae else lat
        b.mulv, b.z = f(bsz, nmulv), f(bsz, lat)
        b.dlat, b.terms = f(bsz, 3 * lat), f(2)
        b.eps = torch.zeros(bsz, lat, dtype=torch.float32, device=dev)
        b.eps_fixed = False  # True: injected by inject()/set_batch(eps=...)
        b.key = torch.zeros(1, dtype=torch.int32, device=dev)
        b.h = f(bsz, self.num_vert, S.out_ch[-1])
        b.dec_up, b.dec_out = [], []
        for (cin, cout, lv, ui) in S.dec_layers():
            b.dec_up.append(fl(lv, bsz, nv[lv], cin))
            b.dec_out.append(fl(lv, bsz, nv[lv], cout))
        b.out = f0(bsz, nv[0], S.in_ch)
        b.unit = f0(bsz, nv[0], S.in_ch)
        b.partials = f(2 * ops.recon_lap_blocks(bsz, nv[0]))
        b.losses = f(5)
        # backward
        b.dout = f0(bsz, nv[0], S.in_ch)
        b.g_dec_up = [fl(lv, bsz, nv[lv], cin) for (cin, cout, lv, ui) in S.dec_layers()]   # grad wrt dec_up
        b.dpre_dec = [fl(lv, bsz, nv[lv], cout) for (cin, cout, lv, ui) in S.dec_layers()]  # grad wrt pre-ELU
        b.dh = torch.empty_like(b.h)
        b.dz = f(bsz, lat)
        flat_out = self.num_vert * S.out_ch[-1]
        b.dz_parts = (f(ops.linear_bwd_split_parts(flat_out), bsz, lat)
                      if bsz <= 16 and lat <= 128 else None)
        b.dmulv = torch.empty_like(b.mulv)
        b.bn_sync = torch.zeros(ops.BN_SYNC_INTS, dtype=torch.int32, device=dev)  # cfsd_bottleneck_bwd's counters
        b.bn_xchg = (f(ops.bottleneck_exchange_floats(bsz, lat, flat_out, nmulv)) if b.dz_parts is not None
                     else None)  # cfsd_bottleneck_bwd's line-exclusive hand-off area
        b.dpre_enc = [f(bsz, nv[lv + 1], cout) if (lv == last_enc or not T.enc_select[lv])
                      else fl(lv + 1, bsz, nv[lv + 1], cout) for (cin, cout, lv) in S.enc_layers()]
        b.g_enc_in = [None] + [f(bsz, nv[lv], cin) if not T.enc_select[lv - 1] else None
                               for (cin, cout, lv) in S.enc_layers()[1:]]
        b.g_pooled = [f(bsz, nv[lv + 1], cout) if not T.enc_select[lv] else None
                      for (cin, cout, lv) in S.enc_layers()]
        ws = 0
        for (cin, cout, lv) in S.enc_layers():
            rows = nv[lv + 1] if T.enc_select[lv] else nv[lv]
            ws = max(ws, ops.spiral_conv_bwd_weight_workspace(bsz, rows, T.seq[lv], cin, cout))
        for (cin, cout, lv, _) in S.dec_layers():
            ws = max(ws, ops.spiral_conv_bwd_weight_workspace(bsz, nv[lv], T.seq[lv], cin, cout))
        ws = max(ws, ops.spiral_conv_bwd_weight_workspace(bsz, nv[0], T.seq[0], S.out_ch[0], S.in_ch))
        for (cin, cout, lv) in S.enc_layers():
            rows = nv[lv + 1] if T.enc_select[lv] else nv[lv]
            ws = max(ws, ops.spiral_conv_workspace(bsz, nv[lv], rows, T.seq[lv], cin, cout))
        for (cin, cout, lv, _) in S.dec_layers():
            ws = max(ws, ops.spiral_conv_workspace(bsz, nv[lv], nv[lv], T.seq[lv], cin, cout))
        ws = max(ws, ops.spiral_conv_workspace(bsz, nv[0], nv[0], T.seq[0], S.out_ch[0], S.in_ch))
        ws = max(ws, ops.spiral_conv_bwd_workspace(bsz, nv[0], nv[0], T.seq[0], S.out_ch[0], S.in_ch))
        # bf16 Enblocks whose dpre is fp32: dx by the row-subset dG + gather
        b.rowsub_x = {}
        for (cin, cout, lv) in S.enc_layers():
            if lv in lp and lv > 0 and T.enc_select[lv] and T.enc_flat[lv] is not None and lv + 1 not in lp:
                need = ops.spiral_conv_bwd_data_rowsub_workspace(bsz, nv[lv + 1], T.seq[lv], cin)
                b.rowsub_x[lv] = need > 0
                ws = max(ws, need)
        b.ws = torch.empty(ws // 4 + 64, dtype=torch.float32, device=dev)
        # weight-gradient partials: one region per layer, all reduced by ONE
        # cfsd_dw_reduce_batch launch at the end of the backward
        # (coarse layers whose dx and dW run as one paired launch keep the
        # paired call's workspace: dW slabs in the same region)
        regions = [("out", ops.spiral_conv_bwd_workspace(bsz, nv[0], nv[0], T.seq[0], S.out_ch[0],
                                                         S.in_ch))]
        b.paired = {}

        b.rowsub = {}
        b.rowsub_vm = {}

        def dw_region(key, vsrc, rows, seq, cin, cout, has_dx, low, flat=None):
            b.paired[key] = (not low) and has_dx and ops.spiral_conv_bwd_paired(bsz, vsrc, rows, seq, cin, cout)
            # Enblock conv on a row subset: dG at the kept rows + flat-list gather
            rs = ops.spiral_conv_bwd_rowsub_workspace(bsz, vsrc, rows, seq, cin, cout)
            # fp32 vertex-major input (E1 of the fp32 step): the same paired
            # dG + dW-slab launch reading x vertex-major (few-row layers)
            b.rowsub_vm[key] = (low and not self.lp_levels and has_dx and flat is not None and rs > 0
                                and bsz * rows < 65536)
            b.rowsub[key] = ((not low) or b.rowsub_vm[key]) and has_dx and flat is not None and rs > 0
            if b.rowsub[key]:
                regions.append((key, rs))
                return
            if low:
                nb = ops.spiral_conv_bwd_weight_x_workspace(bsz, rows, seq, cin, cout, ldt if cin > 3 else torch.float32)
                if b.vm_pair.get(key):
                    nb = max(nb, ops.spiral_conv_bwd_flat_pair_workspace(bsz, rows, seq, cin, cout))
            else:
                nb = (ops.spiral_conv_bwd_workspace(bsz, vsrc, rows, seq, cin, cout) if b.paired[key]
                      else ops.spiral_conv_bwd_weight_workspace(bsz, rows, seq, cin, cout))
            regions.append((key, nb))

        # fp32 vertex-major Deblocks (levels in vm_pair_levels): dx + dW slabs in one launch
        b.vm_pair = {}
        for i, (cin, cout, lv, _) in enumerate(S.dec_layers()):
            flat_ok = lv in lp and cin == 32 and cout == 32 and self._flat_dx(b, lv, cin, cout)
            if ldt == torch.float32:
                b.vm_pair[("dec", i)] = (flat_ok and lv in self.vm_pair_levels
                                         and ops.spiral_conv_bwd_flat_pair_workspace(bsz, nv[lv], T.seq[lv], cin,
                                                                                     cout) > 0)
            else:
                b.vm_pair[("dec", i)] = flat_ok and lv in self.vm_pair_levels16
        for i, (cin, cout, lv, _) in enumerate(S.dec_layers()):
            dw_region(("dec", i), nv[lv], nv[lv], T.seq[lv], cin, cout, True, lv in lp)
        for (cin, cout, lv) in S.enc_layers():
            rows = nv[lv + 1] if T.enc_select[lv] else nv[lv]
            dw_region(("enc", lv), nv[lv], rows, T.seq[lv], cin, cout, lv > 0, lv in lp,
                      T.enc_flat[lv] if T.enc_select[lv] else None)
        total = sum((nb // 4 + 64) // 64 * 64 for _, nb in regions)
        b.ws_dw_all = torch.empty(total, dtype=torch.float32, device=dev)
        b.ws_dw, off = {}, 0
        for key, nb in regions:
            n = (nb // 4 + 64) // 64 * 64
            b.ws_dw[key] = b.ws_dw_all[off:off + n]
            off += n
        flat_in = self.num_vert * S.out_ch[-1]
        nmu = lat * (2 if S.is_vae else 1)
        lws = max(ops.linear_workspace(bsz, flat_in, nmu), ops.linear_workspace(bsz, lat, flat_in))
        b.lin_ws = torch.empty(lws // 4 + 64, dtype=torch.float32, device=dev)
        # step bookkeeping for the resident-dataset path
        b.batch_idx = torch.zeros(self.swap_bs, dtype=torch.int32, device=dev)
        self._bufs[bsz] = b
        return b

    # ----------------------------------------------------------- names
    def _enc_w(self, i):
        return (self.params.view(f"en_layers.{i}.conv.layer.weight"),
                self.params.view(f"en_layers.{i}.conv.layer.bias"))

    def _dec_w(self, i):  # de_layers[i + 1]
        return (self.params.view(f"de_layers.{i + 1}.conv.layer.weight"),
                self.params.view(f"de_layers.{i + 1}.conv.layer.bias"))

    def _w16(self, wname):
        """bf16 shadow view of a conv weight (bf16 mode)."""
        return self.params.view(wname, self.params.shadow)

    def _wx(self, wname):
        """The weights the vertex-major kernels read: the bf16 shadow in bf16
        mode, the fp32 master in fp32 mode."""
        return self._w16(wname) if self.lp_levels else self.params.view(wname)

    @staticmethod
    def _plain(*ts):
        """fp32 batch-major operands: the plain fp32 entry points apply."""
        return all(t.dtype == torch.float32 and not ops.is_vm(t) for t in ts)

    def _conv_fwd(self, b, x, idx, wname, act, out):
        """SpiralConv forward on fp32, vertex-major or mixed/bf16 operands."""
        P = self.params
        w, bias = P.view(wname + ".weight"), P.view(wname + ".bias")
        if self._plain(x, out):
            ops.spiral_conv_fwd(x, idx, w, bias, act, out=out, workspace=b.ws)
        else:
            w16 = self._w16(wname + ".weight") if self.lp_levels else None
            ops.spiral_conv_fwd_x(x, idx, w, w16, bias, act, out)

    @classmethod
    def _spmm(cls, csr, x, m, out, elu_y=None, sched=None, uniform=0):
        if cls._plain(x, out):
            ops.spmm(csr, x, m, elu_y=elu_y, out=out, sched=sched, uniform=uniform)
        else:
            ops.spmm_x(csr, x, m, elu_y=elu_y, out=out, sched=sched, uniform=uniform)

    def _lin_names(self):
        n = self.spec.n
        if self.spec.is_vae:
            return (f"en_layers.{n}.weight", f"en_layers.{n + 1}.weight",
                    f"en_layers.{n}.bias", f"en_layers.{n + 1}.bias")
        return (f"en_layers.{n}.weight", f"en_layers.{n}.weight",
                f"en_layers.{n}.bias", f"en_layers.{n}.bias")

    def _enc_lin(self, buf=None):
        w0, w1, b0, b1 = self._lin_names()
        P = self.params
        flat_in = self.num_vert * self.spec.out_ch[-1]
        nout = self.spec.latent * (2 if self.spec.is_vae else 1)
        W = P.span(w0, w1, buf).view(nout, flat_in)
        B = P.span(b0, b1, buf)
        return W, B

    # ----------------------------------------------------------- forward
    def encode(self, b):
        """Enblocks + stacked mu/logvar Linear (model.py:146-160)."""
        T, S = self.topo, self.spec
        h = b.x
        swap_from, b.swap_from = getattr(b, "swap_from", None), None
        for (cin, cout, lv) in S.enc_layers():
            w, bias = self._enc_w(lv)
            if lv == 0 and swap_from is not None:  # feature swap + this conv in one launch
                ops.spiral_conv_fwd_in_swap(swap_from, b.batch_idx, T.region_mask, b.key, self.swap_bs, b.x,
                                            T.enc_rows[0], w, bias, ACT_ELU, b.enc_out[0])
            elif T.enc_select[lv]:
                self._conv_fwd(b, h, T.enc_rows[lv], f"en_layers.{lv}.conv.layer", ACT_ELU, b.enc_out[lv])
            else:
                ops.spiral_conv_fwd(h, T.spiral[lv], w, bias, ACT_ELU, out=b.enc_full[lv],
                                    workspace=b.ws)
                ops.spmm(T.down_csr[lv], b.enc_full[lv], T.n_verts[lv + 1], out=b.enc_out[lv])
            h = b.enc_out[lv]
        W, B = self._enc_lin()
        ops.linear_fwd(h.view(b.bsz, -1), W, B, out=b.mulv, workspace=b.lin_ws)

    @property
    def step_rows(self):
        """Meshes in one train step: bs^2 swapped meshes, or bs without the swap."""
        return self.swap_bs ** 2 if self.swap else self.swap_bs

    def _lc_on(self, b):
        """Latent consistency needs a swapped bs x bs group (model_manager.py:360-367);
        without the swap it is 0 (model_manager.py:290-293)."""
        return (self.swap and bool(self.region_size) and self.w_lc != 0.0
                and b.bsz == self.swap_bs ** 2)

    def latent(self, b, train, dec_linear=False):
        """Latent head (model.py:184-188 + the KL / LC terms); with
        ``dec_linear`` also the decoder Linear in the same launch
        (cfsd_latent_linear_fwd; decode() then starts at the first Deblock)."""
        S = self.spec
        lc = self._lc_on(b)
        args = (b.mulv, b.eps if (train and S.is_vae) else None,
                b.key if lc else None, b.z, b.dlat, b.terms, S.latent,
                self.region_size if lc else 0, train, S.is_vae, S.sigmoid, self.w_kl,
                self.w_lc if lc else 0.0, self.eta1, self.eta2)
        if dec_linear:
            ops.latent_linear_fwd(*args, self.params.view("de_layers.0.weight"),
                                  self.params.view("de_layers.0.bias"), out=b.h.view(b.bsz, -1))
        else:
            ops.latent_fwd(*args)

    def _fused_latent(self, b):
        return self.fuse_latent and ops.latent_linear_fwd_supported(
            b.bsz, self.spec.latent, self.params.view("de_layers.0.weight").shape[0])

    def decode(self, b, z=None, linear=True):
        """de_layers: Linear -> 4x (Pool up -> conv -> ELU) -> conv (model.py:162-173).
        ``linear=False``: b.h already holds the Linear's output."""
        T, S = self.topo, self.spec
        if linear:
            ops.linear_fwd(b.z if z is None else z, self.params.view("de_layers.0.weight"),
                           self.params.view("de_layers.0.bias"), out=b.h.view(b.bsz, -1),
                           workspace=b.lin_ws)
        h = b.h
        for i, (cin, cout, lv, ui) in enumerate(S.dec_layers()):
            wname = f"de_layers.{i + 1}.conv.layer"
            if self._fused_up(b, h, i, lv, ui, cin, cout):  # Pool(up) inside the conv gather
                ops.spiral_conv_fwd_up(h, T.up_comp[ui], T.spiral[lv], self.params.view(wname + ".weight"),
                                       self.params.view(wname + ".bias"), ACT_ELU, out=b.dec_out[i],
                                       up_out=b.dec_up[i])
            else:
                self._spmm(T.up_csr[ui], h, T.n_verts[lv], out=b.dec_up[i], uniform=T.up_uniform[ui])
                self._conv_fwd(b, b.dec_up[i], T.spiral[lv], wname, ACT_ELU, b.dec_out[i])
            h = b.dec_out[i]
        n = S.n
        self._conv_fwd(b, h, T.spiral[0], f"de_layers.{n + 1}.layer", ACT_NONE, b.out)

    def _fused_up(self, b, h, i, lv, ui, cin, cout):
        """The coarse Deblocks (fp32 batch-major, uniform 3-entry up rows,
        spirals starting at their own vertex) fuse Pool(up) into the conv's
        gather (cfsd_spiral_conv_fwd_up: bit-identical up-sampled rows, one
        launch instead of two)."""
        T = self.topo
        return (self.fuse_up and lv not in b.xl and T.up_comp[ui] is not None
                and self._plain(h, b.dec_up[i], b.dec_out[i])
                and ops.spiral_conv_fwd_up_supported(b.bsz, T.n_verts[lv], T.seq[lv], cin, cout))

    def losses_fwd(self, b, acc=None, finalize=True):
        T = self.topo
        ops.recon_lap_fwd(b.out, b.x, T.lap_csr, b.unit, b.partials)
        if finalize:
            ops.loss_finalize(b.partials, b.terms, b.losses, acc, b.bsz, T.n_verts[0], self.spec.in_ch,
                              self.w_kl, self.w_lc if self._lc_on(b) else 0.0, self.w_lap)

    def forward(self, b, train=True, acc=None, finalize=True):
        """``finalize=False``: the loss reduction is left to backward(), whose
        first launch finalises it (one launch less per train step)."""
        self.encode(b)
        fused = self._fused_latent(b)
        self.latent(b, train, dec_linear=fused)
        self.decode(b, linear=not fused)
        if self.topo.lap_csr is not None:
            self.losses_fwd(b, acc, finalize)
        b.pending_finalize = (not finalize, acc)

    # ----------------------------------------------------------- backward
    def enc_conv_numel(self):
        """Length of the flat-buffer prefix holding the encoder conv
        parameters (the last gradients the backward produces)."""
        return self.params.offsets[f"en_layers.{self.spec.n}.weight"][0]

    def backward(self, b, bucket_hook=None, fuse_adam=False):
        """Hand-derived backward of forward() (the reference's
        ``loss_tot.backward()``).  With ``bucket_hook`` the gradient becomes
        final in two contiguous buckets and the hook is called on each as soon
        as it is (data-parallel all-reduce overlapped with the rest of the
        backward): first everything from the encoder Linear on (decoder,
        bottleneck: ~96 % of the parameters), after the encoder-Linear
        backward; then the encoder convs at the end.  ``fuse_adam`` (no hook):
        the Adam step runs in the final weight-gradient reduce launch."""
        fuse = fuse_adam and bucket_hook is None
        self.backward_head(b, split=bucket_hook is not None, fuse_adam=fuse)
        if bucket_hook is not None:
            bucket_hook(self.params.grad[self.enc_conv_numel():])
        self.backward_tail(b, fuse_adam=fuse)
        if bucket_hook is not None:
            bucket_hook(self.params.grad[:self.enc_conv_numel()])

    def backward_head(self, b, split=False, fuse_adam=False):
        """Losses -> decoder -> latent head -> encoder Linear.  ``split``:
        reduce the decoder conv weight gradients here (their bucket is then
        final) instead of in backward_tail's single batched reduce.
        ``fuse_adam``: single process, nothing between gradient and update
        (Adam then rides in backward_tail's batched reduce)."""
        T, S, P = self.topo, self.spec, self.params
        n = S.n
        side_items = []  # deferred weight-gradient slab sets (reduced in one launch later)
        pending, acc = getattr(b, "pending_finalize", (False, None))
        if pending:
            ops.recon_lap_bwd_finalize(b.out, b.x, b.unit, T.lapT_csr, b.dout, 1.0, self.w_lap,
                                       b.partials, b.terms, b.losses, acc, self.w_kl,
                                       self.w_lc if self._lc_on(b) else 0.0)
            b.pending_finalize = (False, None)
        else:
            ops.recon_lap_bwd(b.out, b.x, b.unit, T.lapT_csr, b.dout, 1.0, self.w_lap)
        # final SpiralConv (no activation): dpre = dout
        last_in = b.dec_out[-1]
        # dX and dW/db of the output conv in one source-row pass.  Every conv
        # weight gradient is deferred (partials left in b.ws_dw[...]) and all
        # of them are reduced by one launch at the end.
        # (weight gradients on a side stream overlapping the dx chain were
        # measured slower on MI355X, 16.3k vs 17.5k meshes/s: the persistent
        # level-0 kernels slow ~2x when sharing the chip and every fork/join
        # costs 6-17 us inside the graph -> one stream)
        def defer(d, name):
            side_items.append((d, P.gview(name + ".weight"), P.gview(name + ".bias")))

        weight_grad = ops.spiral_conv_bwd_weight

        w_out = P.view(f"de_layers.{n + 1}.layer.weight")
        if self._flat_out(b):  # vertex-major: one walk of each vertex's flat inverse list
            _, d = ops.spiral_conv_bwd_out_flat(last_in, T.spiral[0], b.dout, T.spiral_flat[0], w_out, None, None,
                                                dx=b.dpre_dec[-1], elu_y=last_in, workspace=b.ws_dw["out"])
        else:
            bwd_out = ops.spiral_conv_bwd_x if 0 in b.xl else ops.spiral_conv_bwd
            _, d = bwd_out(last_in, T.spiral[0], b.dout, T.spiral_inv[0], w_out, None, None,
                           dx=b.dpre_dec[-1], elu_y=last_in, workspace=b.ws_dw["out"])
        defer(d, f"de_layers.{n + 1}.layer")
        dec = S.dec_layers()
        fused_bn = self._fused_bottleneck_ok(b)
        for i in reversed(range(len(dec))):
            cin, cout, lv, ui = dec[i]
            w, _ = self._dec_w(i)
            if b.vm_pair.get(("dec", i)) and b.dec_up[i].dtype == torch.bfloat16:  # bf16: the same pair
                defer(ops.spiral_conv_bwd_flat_pair_bf16(b.dec_up[i], T.spiral[lv], b.dpre_dec[i], T.spiral_flat[lv],
                                                         self._wx(f"de_layers.{i + 1}.conv.layer.weight"),
                                                         b.g_dec_up[i], workspace=b.ws_dw[("dec", i)]),
                      f"de_layers.{i + 1}.conv.layer")
            elif b.vm_pair.get(("dec", i)):  # fp32 vertex-major: flat dx + dW slabs in one launch
                defer(ops.spiral_conv_bwd_flat_pair(b.dec_up[i], T.spiral[lv], b.dpre_dec[i], T.spiral_flat[lv],
                                                    w, None, None, b.g_dec_up[i],
                                                    workspace=b.ws_dw[("dec", i)]), f"de_layers.{i + 1}.conv.layer")
            elif lv in b.xl:  # vertex-major (bf16 or fp32) operands: dW slabs + dx
                defer(ops.spiral_conv_bwd_weight_x(b.dec_up[i], T.spiral[lv], b.dpre_dec[i], None, None,
                                                   b.ws_dw[("dec", i)]), f"de_layers.{i + 1}.conv.layer")
                w16 = self._wx(f"de_layers.{i + 1}.conv.layer.weight")
                if self._flat_dx(b, lv, cin, cout):  # vertex-major, batch % 16: one MFMA per list entry
                    ops.spiral_conv_bwd_data_flat(b.dpre_dec[i], T.spiral_flat[lv], w16, T.n_verts[lv],
                                                  out=b.g_dec_up[i])
                else:
                    ops.spiral_conv_bwd_data_x(b.dpre_dec[i], T.spiral_inv[lv], w16, T.n_verts[lv],
                                               out=b.g_dec_up[i])
            elif b.paired[("dec", i)]:  # dx + dW slabs in one launch
                _, d = ops.spiral_conv_bwd(b.dec_up[i], T.spiral[lv], b.dpre_dec[i], T.spiral_inv[lv],
                                           w, None, None, dx=b.g_dec_up[i], workspace=b.ws_dw[("dec", i)])
                defer(d, f"de_layers.{i + 1}.conv.layer")
            else:
                defer(weight_grad(b.dec_up[i], T.spiral[lv], b.dpre_dec[i], None, None,
                                  b.ws_dw[("dec", i)]), f"de_layers.{i + 1}.conv.layer")
                ops.spiral_conv_bwd_data(b.dpre_dec[i], T.spiral_inv[lv], w, T.n_verts[lv],
                                         out=b.g_dec_up[i], workspace=b.ws)
            # a vertex-major source is swept in natural row order, XCD k taking the
            # k-th eighth of the rows (neighbouring rows share source blocks in its L2):
            # 17-19 vs 21.6 us at level 0; batch-major keeps the longest-rows-first order
            sch = T.upT_nat[ui] if lv in b.xl else T.upT_sched[ui]
            if i > 0:  # through Pool(up) into the previous Deblock's ELU
                self._spmm(T.upT_csr[ui], b.g_dec_up[i], T.n_verts[lv + 1], out=b.dpre_dec[i - 1],
                           elu_y=b.dec_out[i - 1], sched=sch)
            elif not fused_bn:
                self._spmm(T.upT_csr[ui], b.g_dec_up[i], T.n_verts[lv + 1], out=b.dh, sched=sch)
        if fused_bn:  # Pool(up)^T + decoder Linear + latent head + encoder Linear: one launch
            self._bottleneck_bwd_fused(b)
            if split:
                ops.dw_reduce_batch(side_items)
                side_items.clear()
            b.deferred = list(side_items)
            return
        # decoder Linear: dW/db and dz (as 64-row-slice partial products,
        # summed by the latent head's backward) in one launch
        if b.dz_parts is not None:
            ops.linear_bwd_split(b.z, P.view("de_layers.0.weight"), b.dh.view(b.bsz, -1), b.dz_parts,
                                 P.gview("de_layers.0.weight"), P.gview("de_layers.0.bias"))
            dz = b.dz_parts
        else:
            ops.linear_bwd(b.z, P.view("de_layers.0.weight"), b.dh.view(b.bsz, -1), dx=b.dz,
                           dw=P.gview("de_layers.0.weight"), db=P.gview("de_layers.0.bias"),
                           workspace=b.lin_ws)
            dz = b.dz
        ops.latent_bwd(b.mulv, b.eps, b.z, dz, b.dlat, b.dmulv, S.latent, True, S.is_vae, S.sigmoid)
        if split:
            ops.dw_reduce_batch(side_items)
            side_items.clear()
        b.deferred = list(side_items)
        # stacked encoder Linear; ELU of the last Enblock folded into dx
        W, _ = self._enc_lin()
        gW, gB = self._enc_lin(P.grad)
        enc = S.enc_layers()
        last = enc[-1][2]
        flat = b.enc_out[last].view(b.bsz, -1)
        if T.enc_select[last]:
            ops.linear_bwd(flat, W, b.dmulv, dx=b.dpre_enc[last].view(b.bsz, -1), dw=gW.view(W.shape),
                           db=gB, elu_y=flat, workspace=b.lin_ws)
        else:
            ops.linear_bwd(flat, W, b.dmulv, dx=b.g_pooled[last].view(b.bsz, -1), dw=gW.view(W.shape),
                           db=gB, workspace=b.lin_ws)
            ops.spmm(T.downT_csr[last], b.g_pooled[last], T.n_verts[last], elu_y=b.enc_full[last],
                     out=b.dpre_enc[last])

    def _fused_bottleneck_ok(self, b):
        """cfsd_bottleneck_bwd applies: partial-products decoder Linear, the
        coarsest Deblock's gradient
        batch-major fp32 with 64-multiple channels, batch <= 16, latent <= 128."""
        S = self.spec
        g = b.g_dec_up[0]
        ne = S.latent * (2 if S.is_vae else 1)
        return (self.fuse_bottleneck and b.dz_parts is not None
                and g.dtype == torch.float32 and not ops.is_vm(g) and g.is_contiguous()
                and g.shape[2] % 64 == 0 and b.h.numel() // b.bsz <= 5120 and b.bsz <= 16 and S.latent <= 128
                and ne <= 160)

    def _bottleneck_bwd_fused(self, b):
        T, S, P = self.topo, self.spec, self.params
        ui = S.dec_layers()[0][3]
        W, _ = self._enc_lin()
        gW, gB = self._enc_lin(P.grad)
        last = S.enc_layers()[-1][2]
        flat = b.enc_out[last].view(b.bsz, -1)
        select = T.enc_select[last]
        dxe = b.dpre_enc[last].view(b.bsz, -1) if select else b.g_pooled[last].view(b.bsz, -1)
        ops.bottleneck_bwd(T.upT_csr[ui], b.g_dec_up[0], b.z, P.view("de_layers.0.weight"), b.bn_xchg,
                           P.gview("de_layers.0.weight"), P.gview("de_layers.0.bias"), b.mulv, b.eps, b.dlat,
                           b.dmulv, S.is_vae, S.sigmoid, flat, W, dxe, gW.view(W.shape), gB, b.bn_sync,
                           elu_y=flat if select else None)
        if not select:
            ops.spmm(T.downT_csr[last], b.g_pooled[last], T.n_verts[last], elu_y=b.enc_full[last],
                     out=b.dpre_enc[last])

    def check_health(self):
        """Raise CfsdError if a device-side wait of any batch's one-launch
        bottleneck backward timed out (the sticky word of cfsd_bottleneck_bwd:
        those steps' gradients are invalid).  One device read per batch size:
        ModelManager.run_epoch calls it once per epoch, bench.py after the
        timed steps."""
        for b in self._bufs.values():
            ops.bottleneck_check(b.bn_sync)

    def _flat_out(self, b):
        """The flat-list output-conv backward applies (vertex-major level 0,
        batch % 16, the 32 -> 3 xyz conv)."""
        S = self.spec
        return (0 in b.xl and b.bsz % 16 == 0 and S.out_ch[0] == 32 and S.in_ch == 3
                and self.topo.spiral_flat[0] is not None)

    def _flat_dx(self, b, lv, cin, cout):
        """The flat-list bf16 data gradient applies (vertex-major level,
        batch a multiple of 16, 32 -> 32/64 channels, fan-in <= 20)."""
        return (lv in b.xl and b.bsz % 16 == 0 and cin == 32 and cout in (32, 64)
                and self.topo.spiral_flat[lv] is not None)

    def adam_args(self):
        P = self.params
        return dict(param=P.data, grad=P.grad, m=P.exp_avg, v=P.exp_avg_sq, step=P.step, lr=self.lr,
                    beta1=self.betas[0], beta2=self.betas[1], eps=self.adam_eps,
                    weight_decay=self.weight_decay, shadow=P.shadow)

    def backward_tail(self, b, fuse_adam=False):
        """Encoder convs (E_{n-1} .. E0), then ONE batched reduce of every
        still-deferred conv weight gradient -- with ``fuse_adam`` (nothing
        exchanges the gradient before the update) the Adam step runs in the
        same launch (``cfsd_dw_reduce_batch_adam``) and adam_step is skipped."""
        T, S, P = self.topo, self.spec, self.params
        deferred, b.deferred = b.deferred, []

        def defer(d, name):
            deferred.append((d, P.gview(name + ".weight"), P.gview(name + ".bias")))

        weight_grad = ops.spiral_conv_bwd_weight
        for (cin, cout, lv) in reversed(S.enc_layers()):
            w, _ = self._enc_w(lv)
            x_in = b.x if lv == 0 else b.enc_out[lv - 1]
            rows_tab = T.enc_rows[lv]
            prev = lv - 1
            if lv in b.xl and b.rowsub_vm.get(("enc", lv)) and T.enc_select[prev]:
                pass  # fp32 vertex-major x / dx: the paired row-subset launch below
            elif (lv in b.xl and self.rowsub_pair16 and lv > 0 and b.rowsub_x.get(lv) and T.enc_select[prev]
                  and x_in.dtype == torch.bfloat16 and b.dpre_enc[lv].dtype == torch.float32 and cin == 32
                  and cout == 32 and b.bsz % 16 == 0 and T.enc_flat[lv][1] <= 16):
                # bf16 Enblock: its flat dx and dW slabs in one launch
                defer(ops.spiral_conv_bwd_rowsub_pair_bf16(x_in, rows_tab, b.dpre_enc[lv], T.enc_flat[lv], w,
                                                           b.dpre_enc[prev], elu_y=b.enc_out[prev],
                                                           workspace=b.ws_dw[("enc", lv)]),
                      f"en_layers.{lv}.conv.layer")
                continue
            elif lv in b.xl:  # vertex-major (bf16 or fp32) operands (selection down-sampling)
                defer(ops.spiral_conv_bwd_weight_x(x_in, rows_tab, b.dpre_enc[lv], None, None,
                                                   b.ws_dw[("enc", lv)]), f"en_layers.{lv}.conv.layer")
                if lv > 0 and b.dpre_enc[lv].dtype == torch.float32 and b.rowsub_x.get(lv):
                    # fp32 dpre: dG = dpre.W at the kept rows (fp32), then the
                    # flat gather rounded once to bf16
                    ops.spiral_conv_bwd_data_rowsub(b.dpre_enc[lv], T.enc_flat[lv], w, T.n_verts[lv],
                                                    elu_y=b.enc_out[prev], out=b.dpre_enc[prev],
                                                    workspace=b.ws)
                elif lv > 0:
                    ops.spiral_conv_bwd_data_x(b.dpre_enc[lv], T.enc_inv[lv],
                                               self._w16(f"en_layers.{lv}.conv.layer.weight"), T.n_verts[lv],
                                               elu_y=b.enc_out[prev], out=b.dpre_enc[prev])
                continue
            if b.rowsub[("enc", lv)]:  # dG at the kept rows (+ dW slabs), then the flat gather
                sel = T.enc_select[prev]
                _, d = ops.spiral_conv_bwd_rowsub(x_in, rows_tab, b.dpre_enc[lv], T.enc_flat[lv], w, None, None,
                                                  dx=b.dpre_enc[prev] if sel else b.g_pooled[prev],
                                                  elu_y=b.enc_out[prev] if sel else None,
                                                  workspace=b.ws_dw[("enc", lv)])
                defer(d, f"en_layers.{lv}.conv.layer")
                if not sel:
                    ops.spmm(T.downT_csr[prev], b.g_pooled[prev], T.n_verts[prev],
                             elu_y=b.enc_full[prev], out=b.dpre_enc[prev])
                continue
            if b.paired[("enc", lv)]:  # dx + dW slabs in one launch
                sel = T.enc_select[prev]
                _, d = ops.spiral_conv_bwd(x_in, rows_tab, b.dpre_enc[lv], T.enc_inv[lv], w, None, None,
                                           dx=b.dpre_enc[prev] if sel else b.g_pooled[prev],
                                           elu_y=b.enc_out[prev] if sel else None,
                                           workspace=b.ws_dw[("enc", lv)])
                defer(d, f"en_layers.{lv}.conv.layer")
                if not sel:
                    ops.spmm(T.downT_csr[prev], b.g_pooled[prev], T.n_verts[prev],
                             elu_y=b.enc_full[prev], out=b.dpre_enc[prev])
                continue
            defer(weight_grad(x_in, rows_tab, b.dpre_enc[lv], None, None,
                              b.ws_dw[("enc", lv)]), f"en_layers.{lv}.conv.layer")
            if lv == 0:
                break
            if T.enc_select[prev]:
                # input of this conv IS the ELU output of the previous Enblock
                ops.spiral_conv_bwd_data(b.dpre_enc[lv], T.enc_inv[lv], w, T.n_verts[lv],
                                         elu_y=b.enc_out[prev], out=b.dpre_enc[prev], workspace=b.ws)
            else:
                ops.spiral_conv_bwd_data(b.dpre_enc[lv], T.enc_inv[lv], w, T.n_verts[lv],
                                         out=b.g_pooled[prev], workspace=b.ws)
                ops.spmm(T.downT_csr[prev], b.g_pooled[prev], T.n_verts[prev], elu_y=b.enc_full[prev],
                         out=b.dpre_enc[prev])
        ops.dw_reduce_batch(deferred, adam=self.adam_args() if fuse_adam else None)

    def adam_step(self, grad_scale=None):
        """Adam over the flat buffers; ``grad_scale`` (data-parallel: 1/world
        after the all-reduce SUM) scales the gradient in the same launch."""
        P = self.params
        kw = dict(beta1=self.betas[0], beta2=self.betas[1], eps=self.adam_eps, weight_decay=self.weight_decay,
                  shadow=P.shadow)
        if grad_scale is None:
            ops.adam(P.data, P.grad, P.exp_avg, P.exp_avg_sq, P.step, self.lr, **kw)
        else:
            ops.adam_scaled(P.data, P.grad, P.exp_avg, P.exp_avg_sq, P.step, grad_scale, self.lr, **kw)

    def advance_step(self, b=None):
        """t += 1 on device (the Adam bias-correction step) and, for a VAE
        batch whose noise was not injected, a fresh eps ~ N(0, 1) drawn on
        the device (``torch.randn_like``, model.py:187) from the step counter."""
        draw = b is not None and self.spec.is_vae and not b.eps_fixed
        ops.step_begin(self.counter, self.seed, eps=b.eps if draw else None,
                       adam_step=self.params.step)

    # ----------------------------------------------------------- entry points
    def set_batch(self, x, key_index=None, eps=None):
        """Copy an already-swapped batch [B, V, C] (+ injected key / eps).
        Without ``eps`` a VAE train step draws its own noise on the device."""
        b = self.buffers(x.shape[0])
        b.x.copy_(x)
        self.inject(b, key_index, eps)
        return b

    def inject(self, b, key_index=None, eps=None):
        """Fix the swap key and/or the VAE noise of batch buffers ``b`` (parity
        tests inject the reference's values).  ``eps=None`` returns the batch to
        device-drawn noise."""
        if key_index is not None:
            b.key.fill_(int(key_index))
        if eps is not None:
            b.eps.copy_(eps)
        b.eps_fixed = eps is not None
        return b

    def train_step_on(self, b, acc=None, grad_hook=None, advance=True):
        """forward + losses + backward + (grad_hook, e.g. all-reduce) + Adam.
        ``advance=False`` when cfsd_step_begin already advanced Adam's t (and
        drew the noise).  With ``advance`` the noise is drawn first."""
        if advance:
            self.advance_step(b)
        self.forward(b, train=True, acc=acc, finalize=False)
        if hasattr(grad_hook, "bucket_ready"):  # dist.GradientAverager: overlapped buckets
            self.backward(b, bucket_hook=grad_hook.bucket_ready)
            grad_hook.finish(self.params.grad)
        elif grad_hook is not None:
            self.backward(b)
            grad_hook(self.params.grad)
        else:  # nothing between the gradient and the update: Adam fused into the reduce
            self.backward(b, fuse_adam=True)
            return
        self.adam_step()

    def resident_step(self, b, data, acc=None, grad_hook=None):
        """Full reference step from a resident dataset (:class:`ResidentData`):
        device-side epoch-shuffled batch pick + swap key + VAE noise
        (cfsd_step_begin), on-device feature swap, then train_step_on.  No
        host input -> graph-capturable."""
        T = self.topo
        ops.step_begin(self.counter, self.seed, eps=b.eps if self.spec.is_vae else None, key=b.key,
                       n_regions=max(T.n_regions, 1), batch_idx=b.batch_idx, bs=self.swap_bs,
                       n_batches=data.n_batches, perm=data.rows, n_items=data.n_items,
                       shuffle=data.shuffle, adam_step=self.params.step)
        self.load_batch(b, data)
        self.train_step_on(b, acc=acc, grad_hook=grad_hook, advance=False)

    def load_batch(self, b, data):
        """The step's input from the picked base meshes: the on-device feature
        swap (bs -> bs^2) or, with ``swap_features`` False, the bs meshes.
        With the swap fused into the first Enblock's conv (the default,
        ``_swap_in_conv_ok``) nothing is written here: ``b.x`` holds the
        swapped batch only after :meth:`encode` / :meth:`forward` ran (that
        launch writes it); ``b.swap_from`` marks the pending swap."""
        b.swap_from = None
        if self.swap and self._swap_in_conv_ok(b, data):
            b.swap_from = data.meshes  # the swap rides in the first Enblock's conv launch (encode)
        elif self.swap:
            ops.swap_features(data.meshes, b.batch_idx, self.topo.region_mask, b.key, self.swap_bs, out=b.x)
        else:
            ops.gather_meshes(data.meshes, b.batch_idx, self.swap_bs, out=b.x)

    def _swap_in_conv_ok(self, b, data):
        """cfsd_spiral_conv_fwd_in_swap applies: the first Enblock is the xyz
        conv evaluated at its kept rows (3 -> 32/64), fp32 input meshes."""
        S, T = self.spec, self.topo
        cin, cout, lv = S.enc_layers()[0]
        return (self.fuse_swap and lv == 0 and cin == 3 and cout in (32, 64) and T.enc_select[0]
                and data.meshes.dtype == torch.float32 and data.meshes.shape[2] == 3
                and b.x.dtype == torch.float32 and b.bsz == self.swap_bs ** 2)


class ResidentData:
    """A training set resident in HBM (the MeshInMemoryDataset + MeshLoader of
    ``data_loading.py:23-51, 86-283``, without disk or worker processes).

    ``meshes`` [N, V, 3] device fp32 (normalised on the device with
    ``norm`` = {'mean', 'std'} [V, 3] when given, data_loading.py:259-260);
    ``rows`` optional int32 subset of mesh indices (e.g. this rank's shard);
    batches of ``bs`` base meshes with ``shuffle`` (a fresh device-drawn order
    every epoch) and ``drop_last`` semantics (data_loading.py:40-48).
    ``n_batches`` caps the steps per epoch (data-parallel shards whose sizes
    differ by one must all run the same number of steps, each step issuing
    the same gradient all-reduces: :func:`dist.steps_per_epoch`)."""

    def __init__(self, meshes, bs, rows=None, shuffle=True, norm=None, n_batches=None, inplace=False):
        if not meshes.is_cuda or meshes.dim() != 3:
            raise ValueError("meshes must be a [N, V, C] device tensor")
        if norm is not None:
            # into a buffer of its own (the caller's tensor is left unchanged),
            # or -- ``inplace``, for a caller that hands the set over (e.g. a
            # 50k-mesh augmented set) -- over the caller's contiguous fp32
            # tensor, so only one copy is resident
            mean = norm["mean"].to(meshes.device, torch.float32).contiguous()
            std = norm["std"].to(meshes.device, torch.float32).contiguous()
            if inplace and not (meshes.is_contiguous() and meshes.dtype == torch.float32):
                raise ValueError("inplace normalisation needs a contiguous fp32 tensor")
            dst = meshes if inplace else torch.empty(meshes.shape, dtype=torch.float32, device=meshes.device)
            self.meshes = ops.normalize(meshes.contiguous(), mean, std, out=dst)
        else:
            self.meshes = meshes.contiguous()
        n = meshes.shape[0]
        if rows is not None:
            rows = torch.as_tensor(rows).to(torch.int64).cpu()
            if rows.numel() and (int(rows.min()) < 0 or int(rows.max()) >= n):
                raise ValueError("rows index outside the dataset")
            self.rows = rows.to(torch.int32).to(meshes.device)
            self.n_items = int(rows.numel())
        else:
            self.rows, self.n_items = None, n
        self.bs = int(bs)
        self.n_batches = self.n_items // self.bs
        if n_batches is not None:
            if not 1 <= int(n_batches) <= self.n_batches:
                raise ValueError(f"n_batches {n_batches} outside [1, {self.n_batches}]")
            self.n_batches = int(n_batches)
        if self.n_batches < 1:
            raise ValueError(f"{self.n_items} meshes < one batch of {self.bs}")
        self.shuffle = bool(shuffle)
