"""CPU oracle for the spiral-convolution mesh-VAE training step.

TEST INFRASTRUCTURE.  Only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg may import this module, and only as the
checker / the timed CPU baseline.  The product path
(``craniofacialsd-vae_amd/``) never imports it and fails loudly when its HIP
library is missing.

This is a restatement of the reference algorithm in PyTorch-CPU fp32 (the
same ATen ops the reference dispatches: ``index_select``, ``addmm``,
``scatter_add_``, sparse ``mm``; backward via autograd exactly as the
reference's ``loss_tot.backward()``), written from the reference's documented
semantics.  Every function cites the reference line it restates.  Parity of
this oracle with the reference itself is pinned by ``tests/golden/*.npz``,
produced by running the reference's own code (``tests/golden/make_golden.py``)
and checked in ``tests/test_oracle_golden.py``.

Integer/byte work (feature swap, index tables) is restated in NumPy and is
bit-exact by construction.
"""
import numpy as np
import torch
import torch.nn.functional as F

SEQ = 9


# --------------------------------------------------------------- topology
class Topology:
    """Plain-array view of ``topology_craniofacial.npz`` (the reference's
    ``spirals.pkl`` / ``transforms.pkl`` / template)."""

    def __init__(self, npz):
        self.n_levels = int(npz["n_levels"])
        self.spirals = [np.asarray(npz[f"spiral_{l}"], np.int64) for l in range(self.n_levels)]
        self.down = [self._coo(npz, "down", l) for l in range(self.n_levels)]
        self.up = [self._coo(npz, "up", l) for l in range(self.n_levels)]
        self.region_keys = [str(k) for k in npz["region_keys"]]
        self.region_features = [np.asarray(npz[f"region_{i}_feature"], np.int64)
                                for i in range(len(self.region_keys))]
        self.n_verts = [int(self.spirals[0].shape[0])] + [int(d[3][0]) for d in self.down]
        n = self.n_verts[0]
        self.lap = (np.asarray(npz["lap_row"], np.int64), np.asarray(npz["lap_col"], np.int64),
                    np.asarray(npz["lap_val"], np.float32), (n, n))

    @staticmethod
    def _coo(npz, name, l):
        return (np.asarray(npz[f"{name}_{l}_row"], np.int64),
                np.asarray(npz[f"{name}_{l}_col"], np.int64),
                np.asarray(npz[f"{name}_{l}_val"], np.float32),
                tuple(int(s) for s in npz[f"{name}_{l}_shape"]))


# ---------------------------------------------------------------- ops
def spiral_conv(x, indices, weight, bias):
    """``SpiralConv.forward`` (``model.py:27-41``): gather the spiral of every
    vertex (``index_select`` along the vertex dim), view as
    ``[.., V, S*Cin]`` (s-major), then ``nn.Linear``."""
    idx = torch.as_tensor(indices, dtype=torch.long)
    n = idx.shape[0]
    if x.dim() == 2:
        g = torch.index_select(x, 0, idx.reshape(-1)).view(n, -1)
    elif x.dim() == 3:
        g = torch.index_select(x, 1, idx.reshape(-1)).view(x.shape[0], n, -1)
    else:
        raise RuntimeError(f"x.dim() is expected to be 2 or 3, but received {x.dim()}")
    return F.linear(g, weight, bias)


def pool(x, coo, dim=1):
    """``Pool`` (``model.py:50-55``): ``out[r] += val[k] * x[col[k]]`` for the
    nnz of the sparse transform in file order (torch-scatter ``scatter_add``
    into zeros of ``dim_size = M``)."""
    row, col, val, shape = coo
    row = torch.as_tensor(row, dtype=torch.long)
    col = torch.as_tensor(col, dtype=torch.long)
    v = torch.as_tensor(val).unsqueeze(-1)
    out = torch.index_select(x, dim, col) * v
    size = list(out.shape)
    size[dim] = shape[0]
    bshape = [1] * out.dim()
    bshape[dim] = -1
    idx = row.view(bshape).expand_as(out)
    return torch.zeros(size, dtype=out.dtype).scatter_add_(dim, idx, out)


def elu(x):
    return F.elu(x)


# ---------------------------------------------------------------- model
def param_names(n_enc=4):
    """Reference ``named_parameters`` order (``model.py:103-137``)."""
    names = []
    for i in range(n_enc):
        names += [f"en_layers.{i}.conv.layer.weight", f"en_layers.{i}.conv.layer.bias"]
    names += [f"en_layers.{n_enc}.weight", f"en_layers.{n_enc}.bias",
              f"en_layers.{n_enc + 1}.weight", f"en_layers.{n_enc + 1}.bias",
              "de_layers.0.weight", "de_layers.0.bias"]
    for i in range(1, n_enc + 1):
        names += [f"de_layers.{i}.conv.layer.weight", f"de_layers.{i}.conv.layer.bias"]
    names += [f"de_layers.{n_enc + 1}.layer.weight", f"de_layers.{n_enc + 1}.layer.bias"]
    return names


def _q(t):
    """bf16 storage of a tensor (round to nearest even), widened back."""
    return t.to(torch.bfloat16).to(t.dtype)


def _w(P, name, low):
    """A conv weight as the bf16 path reads it: the bf16 shadow when the layer
    runs on bf16 MFMA (``low``), else the fp32 master."""
    return _q(P[name]) if low else P[name]


def encode(P, x, topo, is_vae=True, lp=()):
    """``Model.encode`` (``model.py:146-160``): 4x (conv -> ELU -> Pool down),
    vertex-major flatten, Linear mu = en_layers[-1], logvar = en_layers[-2].
    ``lp``: levels stored in bf16 (emulates the engine's bf16 precision: those
    activations rounded to bf16, 32/64-channel convs reading them use bf16
    weights); empty = the reference's fp32."""
    n = topo.n_levels
    h = x
    for i in range(n):
        wname = f"en_layers.{i}.conv.layer.weight"
        low = i in lp and h.shape[-1] >= 16
        h = elu(spiral_conv(h, topo.spirals[i], _w(P, wname, low), P[f"en_layers.{i}.conv.layer.bias"]))
        h = pool(h, topo.down[i])
        if (i + 1) in lp and i + 1 < n:
            h = _q(h)
    last = n + 1 if is_vae else n
    flat = h.reshape(-1, P[f"en_layers.{last}.weight"].shape[1])
    mu = F.linear(flat, P[f"en_layers.{last}.weight"], P[f"en_layers.{last}.bias"])
    logvar = F.linear(flat, P[f"en_layers.{n}.weight"], P[f"en_layers.{n}.bias"]) if is_vae else None
    return mu, logvar


def decode(P, z, topo, c_last=None, lp=()):
    """``Model.decode`` (``model.py:162-173``): Linear -> view [B, V4, C];
    4x (Pool up -> conv -> ELU); final SpiralConv without activation.
    ``lp`` as in :func:`encode`."""
    n = topo.n_levels
    if c_last is None:
        c_last = P["de_layers.0.weight"].shape[0] // topo.n_verts[-1]
    h = F.linear(z, P["de_layers.0.weight"], P["de_layers.0.bias"])
    h = h.view(-1, topo.n_verts[-1], c_last)
    for i in range(1, n + 1):
        lv = n - i
        h = pool(h, topo.up[lv])
        if lv in lp:
            h = _q(h)
        h = elu(spiral_conv(h, topo.spirals[lv], _w(P, f"de_layers.{i}.conv.layer.weight", lv in lp),
                            P[f"de_layers.{i}.conv.layer.bias"]))
        if lv in lp:
            h = _q(h)
    return spiral_conv(h, topo.spirals[0], P[f"de_layers.{n + 1}.layer.weight"],
                       P[f"de_layers.{n + 1}.layer.bias"])


def forward(P, x, topo, eps=None, train=True, is_vae=True, lp=()):
    """``Model.forward`` + ``_reparameterize`` (``model.py:175-188``), with
    the noise ``eps`` injected instead of ``torch.randn_like``.  AE
    (``is_vae=False``, kl_weight 0 at ``model_manager.py:67``): z = mu."""
    mu, logvar = encode(P, x, topo, is_vae, lp)
    if train and is_vae:
        z = mu + eps * torch.exp(0.5 * logvar)
    else:
        z = mu
    return decode(P, z, topo, lp=lp), z, mu, logvar


# ---------------------------------------------------------------- losses
def mse_loss(pred, gt):
    """``compute_mse_loss`` (``model_manager.py:333-334``)."""
    return F.mse_loss(pred, gt)


def laplacian_loss(pred, lap):
    """``_compute_laplacian_regularizer`` + ``utils.batch_mm``
    (``model_manager.py:343-349``, ``utils.py:153-165``)."""
    row, col, val, shape = lap
    L = torch.sparse_coo_tensor(torch.as_tensor(np.stack([row, col])), torch.as_tensor(val), shape)
    b, n = pred.shape[0], pred.shape[1]
    m = pred.transpose(0, 1).reshape(n, -1)
    lx = L.mm(m).reshape(n, b, -1).transpose(1, 0)
    return (lx.norm(dim=-1) / n).sum() / b


def kl_loss(mu, logvar):
    """``_compute_kl_divergence_loss`` (``model_manager.py:352-354``)."""
    return torch.mean(-0.5 * torch.sum(1 + logvar - mu.pow(2) - logvar.exp(), dim=1), dim=0)


def latent_consistency(z, region, bs, eta1=0.5, eta2=0.5):
    """``_compute_latent_consistency`` (``model_manager.py:360-393``).

    ``z`` rows are ``i*bs + j`` (base mesh i, donor j).  For every base pair
    p<q and every t:  lg = |zf[q,t]-zf[p,t]|^2 (same donor),
    dg = |zf[t,q]-zf[t,p]|^2 (same base), likewise dr/lr on the other dims;
    loss = (sum relu(lr-dr+eta2) + sum relu(lg-dg+eta1)) / (bs^3 - bs^2)."""
    a, b = region
    zf = z[:, a:b].view(bs, bs, -1)
    ze = torch.cat([z[:, :a], z[:, b:]], dim=1).view(bs, bs, -1)
    p, q = torch.triu_indices(bs, bs, 1)
    lg = ((zf[q] - zf[p]) ** 2).sum(-1).reshape(-1)
    dg = ((zf[:, q].transpose(0, 1) - zf[:, p].transpose(0, 1)) ** 2).sum(-1).reshape(-1)
    dr = ((ze[q] - ze[p]) ** 2).sum(-1).reshape(-1)
    lr = ((ze[:, q].transpose(0, 1) - ze[:, p].transpose(0, 1)) ** 2).sum(-1).reshape(-1)
    return (1.0 / (bs ** 3 - bs ** 2)) * (torch.clamp(lr - dr + eta2, min=0).sum()
                                          + torch.clamp(lg - dg + eta1, min=0).sum())


def vertex_errors(out, gt, to_mm=89.11):
    """``compute_vertex_errors`` (``model_manager.py:395-400``)."""
    return torch.sqrt(((out - gt) ** 2).sum(-1)) * to_mm


# ---------------------------------------------------------------- swap
def swap_features(x, features, key_index):
    """``SwapFeatures.__call__`` / ``swap`` (``swap_batch_transform.py:13-52``):
    ``out[i*bs + j] = x[i]`` with the region's feature vertices taken from
    ``x[j]``; the diagonal holds the originals.  Bit-exact copy semantics."""
    x = np.asarray(x)
    bs = x.shape[0]
    feat = features[key_index]
    out = np.empty((bs * bs,) + x.shape[1:], x.dtype)
    for i in range(bs):
        for j in range(bs):
            o = x[i].copy()
            if i != j:
                o[feat] = x[j][feat]
            out[i * bs + j] = o
    return out


def swap_labels(bs, y, augmented, age, gender):
    """Label bookkeeping of ``SwapFeatures.__call__`` (``:18-38``)."""
    n = bs * bs
    ny, ng = [None] * n, ["n/a"] * n
    na = np.ones((n, 1), np.asarray(augmented).dtype)
    nage = -np.ones((n, 1), np.asarray(age).dtype)
    for i in range(bs):
        k = i * bs + i
        ny[k], ng[k] = y[i], gender[i]
        na[k] = augmented[i]
        nage[k] = age[i]
    return ny, na, nage, ng


# ---------------------------------------------------------------- train step
LOSS_W = {"kl": 1e-4, "lc": 0.5, "lap": 0.1}


def latent_regions(n_regions, latent=75):
    """``_compute_latent_regions`` (``model_manager.py:232-238``)."""
    rs = latent // n_regions
    return [(i * rs, (i + 1) * rs) for i in range(n_regions)]


def losses(P, x16, topo, key_index, eps, bs=4, w=LOSS_W, is_vae=True, train=True, lp=()):
    """Forward + the four losses of ``_do_iteration``
    (``model_manager.py:281-312``); KL only when ``w_kl > 0`` (``:285-288``),
    latent consistency only with swapped batches (``:290-293``).
    ``train=False``: the validation pass (eval mode, z = mu); ``lp``: bf16
    storage emulation (see :func:`encode`)."""
    rec, z, mu, lv = forward(P, x16, topo, eps=eps, train=train, is_vae=is_vae, lp=lp)
    l_rec = mse_loss(rec, x16)
    l_lap = laplacian_loss(rec, topo.lap)
    l_kl = kl_loss(mu, lv) if w["kl"] > 0 else torch.tensor(0.0)
    if w["lc"] and key_index is not None:
        region = latent_regions(len(topo.region_keys), z.shape[1])[key_index]
        l_lc = latent_consistency(z, region, bs)
    else:
        l_lc = torch.tensor(0.0)
    tot = l_rec + w["kl"] * l_kl + w["lc"] * l_lc + w["lap"] * l_lap
    return {"rec": l_rec, "kl": l_kl, "lc": l_lc, "lap": l_lap, "tot": tot,
            "out": rec, "z": z, "mu": mu, "logvar": lv}


class Adam:
    """``torch.optim.Adam`` update rule (lr, betas=(0.9, 0.999), eps=1e-8,
    weight_decay=0), restated (``model_manager.py:69-72, 316``)."""

    def __init__(self, params, lr=1e-4, betas=(0.9, 0.999), eps=1e-8):
        self.lr, self.b1, self.b2, self.eps = lr, betas[0], betas[1], eps
        self.m = {k: torch.zeros_like(v) for k, v in params.items()}
        self.v = {k: torch.zeros_like(v) for k, v in params.items()}
        self.t = 0

    @torch.no_grad()
    def step(self, params, grads):
        self.t += 1
        bc1 = 1 - self.b1 ** self.t
        bc2 = 1 - self.b2 ** self.t
        for k, p in params.items():
            g = grads[k]
            self.m[k].mul_(self.b1).add_(g, alpha=1 - self.b1)
            self.v[k].mul_(self.b2).addcmul_(g, g, value=1 - self.b2)
            denom = (self.v[k].sqrt() / (bc2 ** 0.5)).add_(self.eps)
            p.addcdiv_(self.m[k], denom, value=-self.lr / bc1)


def train_step(P, opt, x4, topo, key_index, eps, w=LOSS_W, is_vae=True, swap=True):
    """One ``_do_iteration(train=True)``: swap -> forward -> losses ->
    backward -> Adam.  ``P`` holds leaf tensors (requires_grad).  ``swap``
    False: a ``swap_features: False`` configuration (no SwapFeatures in the
    collater, data_loading.py:38, 81-82): the batch is ``x4`` itself and the
    latent-consistency term is 0 (``model_manager.py:290-293``)."""
    if not swap:
        key_index = None
    x16 = torch.from_numpy(swap_features(x4, topo.region_features, key_index) if swap
                           else np.ascontiguousarray(x4, dtype=np.float32))
    for p in P.values():
        p.grad = None
    out = losses(P, x16, topo, key_index, None if eps is None else torch.as_tensor(eps),
                 bs=len(x4), w=w, is_vae=is_vae)
    out["tot"].backward()
    grads = {k: p.grad.detach().clone() for k, p in P.items()}
    opt.step(P, grads)
    return out, grads, x16


def make_params(weights):
    return {k: torch.tensor(np.asarray(v), dtype=torch.float32, requires_grad=True)
            for k, v in weights.items()}


# --------------------------------------------------------------- data order
M64 = (1 << 64) - 1


def _mix32(x):
    """The 64 -> 32-bit finaliser of libcfsd's step_begin_k (train_ops.hip)."""
    x &= M64
    x ^= x >> 33
    x = (x * 0xff51afd7ed558ccd) & M64
    x ^= x >> 33
    x = (x * 0xc4ceb9fe1a85ec53) & M64
    x ^= x >> 33
    return x & 0xFFFFFFFF


def epoch_permutation(seed, epoch, n):
    """Order in which one epoch visits the n dataset positions: the keyed
    Feistel permutation libcfsd draws on the device for MeshLoader(shuffle=True)
    (data_loading.py:40-48; the reference's torch.randperm is a host RNG stream
    this restatement does not reproduce -- the contract pinned here is "a
    permutation per epoch", bit-exact to the kernel)."""
    key = (((seed ^ 0x5DEECE66D) * 0xD6E8FEB86659FD93) + epoch) & M64
    bits = 2
    while (1 << bits) < n:
        bits += 2
    h = bits // 2
    mask = (1 << h) - 1
    out = np.empty(n, np.int64)
    for i in range(n):
        x = i
        while True:
            l, r = x >> h, x & mask
            for rnd in range(4):
                f = _mix32(key + 0x9E3779B97F4A7C15 * (rnd + 1) + r) & mask
                l, r = r, l ^ f
            x = (l << h) | r
            if x < n:
                break
        out[i] = x
    return out


def epoch_batches(seed, epoch, n_items, bs, perm=None):
    """The drop_last batches of one epoch: [n_items // bs, bs] dataset rows."""
    order = epoch_permutation(seed, epoch, n_items)[: (n_items // bs) * bs]
    if perm is not None:
        order = np.asarray(perm)[order]
    return order.reshape(-1, bs)


def normalize(x, mean, std):
    """data_loading.py:259-260: (verts - mean) / std (torch fp32 ops)."""
    return (torch.as_tensor(x) - torch.as_tensor(mean)) / torch.as_tensor(std)


# --------------------------------------------------------------- augmentation
def spectral_interpolation(u, x1, x2, values, interp_until=30):
    """``spectral_interpolation`` (utils.py:256-267) in float64 NumPy with the
    random ``values`` [k] injected (the reference draws N(0.5, 0.5))."""
    u = np.asarray(u, np.float64)
    s1 = u.T @ np.asarray(x1, np.float64)
    s2 = u.T @ np.asarray(x2, np.float64)
    s3 = s1 + np.asarray(values, np.float64).reshape(-1, 1) * (s2 - s1)
    s4 = s1.copy()
    s4[:interp_until] = s3[:interp_until]
    return u @ s4


def augment_counts(train_names, aug_factor, balanced=True):
    """Augmented meshes per class of ``_augment`` (data_loading.py:314-335):
    classes are first letters, 'b' merged into 'n' (:322-324); the balanced
    target is aug_factor * len(initial_list) // len(data_classes) with
    data_classes taken BEFORE the merge (:314, :331-333); range(negative)
    draws nothing."""
    data_classes = set(n[0] for n in train_names)
    per = {c: [n for n in train_names if n[0] == c] for c in data_classes}
    per["n"] = per.get("n", []) + per.pop("b", [])
    out = {}
    for c, info in per.items():
        if balanced:
            n = aug_factor * len(train_names) // len(data_classes) - len(info)
        else:
            n = (aug_factor - 1) * len(info)
        out[c] = max(0, n)
    return out


def augmented_name(name1, name2, mode, i):
    """data_loading.py:359-371: name1[:-4] + '_' + name2[2:-4] + tag + ext."""
    tag = {"spectral_comb": "_spectral_comb", "spectral_interp": "_spectral_interp"}.get(mode)
    if tag is None:
        raise ValueError("interpolate names carry the drawn value, not an index")
    return name1[:-4] + "_" + name2[2:-4] + tag + str(i) + name1[-4:]


def mean_std(verts):
    """compute_mean_and_std (data_loading.py:247-249) over a [N, V, 3] fp32 stack."""
    verts = torch.as_tensor(verts)
    std = torch.std(verts, dim=0)
    return torch.mean(verts, dim=0), torch.where(std > 0, std, torch.tensor(1e-8))
