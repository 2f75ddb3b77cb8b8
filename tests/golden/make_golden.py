"""Generate golden vectors by running the REFERENCE's own Python code.

TEST INFRASTRUCTURE — runs only in the build container, where
``/root/reference`` exists.  Nothing here ships to the GPU box except the
``.npz`` files it writes.

How the reference is run:
* ``model.py`` and ``swap_batch_transform.py`` are compiled from their source
  text and executed in fresh module objects (the ``__pycache__`` in the
  reference is never loaded).
* Their absent third-party imports get minimal restatements:
  ``torch_scatter.scatter_add`` (torch-scatter, version unpinned by
  ``install_env.sh:17``; published semantics: ``out[index[i]] += src[i]`` along
  ``dim`` into a zero tensor of ``dim_size``) and an attribute-bag
  ``torch_geometric.data.Data``.
* ``model_manager.py`` cannot be imported (trimesh/pytorch3d/torchvision), so
  its loss methods (``:333-393``) and ``utils.batch_mm`` (``utils.py:153-165``)
  are extracted with :mod:`ast` and executed verbatim against a namespace
  that supplies ``self``.

Outputs (``tests/golden/``):
* ``golden_ops.npz``    per-op vectors (SpiralConv fwd/bwd, Pool fwd/bwd)
* ``golden_eval.npz``   C1: encode+decode of 8 demo meshes, eval mode
* ``golden_train.npz``  C2: three full train steps (swap, fwd, 4 losses, bwd,
                         Adam) with injected swap keys and VAE noise
* ``golden_swap.npz``   swap outputs (sha256 per region key)
"""
import ast
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import recipe  # noqa: E402

REF = os.environ.get("CFSD_REFERENCE", "/root/reference")
torch.set_num_threads(1)


# ----------------------------------------------------------------- shims
def _scatter_add(src, index, dim=-1, out=None, dim_size=None):
    dim = dim if dim >= 0 else src.dim() + dim
    shape = [1] * src.dim()
    shape[dim] = -1
    idx = index.view(shape).expand_as(src)
    size = list(src.size())
    size[dim] = dim_size if dim_size is not None else int(index.max()) + 1
    if out is None:
        out = torch.zeros(size, dtype=src.dtype, device=src.device)
    return out.scatter_add_(dim, idx, src)


class _Data:
    def __init__(self, **kw):
        for k, v in kw.items():
            setattr(self, k, v)


def _install_shims():
    ts = types.ModuleType("torch_scatter")
    ts.scatter_add = _scatter_add
    sys.modules["torch_scatter"] = ts
    tg = types.ModuleType("torch_geometric")
    tgd = types.ModuleType("torch_geometric.data")
    tgd.Data = _Data
    tg.data = tgd
    sys.modules["torch_geometric"] = tg
    sys.modules["torch_geometric.data"] = tgd


def _load_source_module(name, fname):
    path = os.path.join(REF, fname)
    mod = types.ModuleType(name)
    mod.__file__ = path
    src = open(path).read()
    exec(compile(src, path, "exec"), mod.__dict__)
    return mod


def _extract_functions(fname, names, cls=None):
    path = os.path.join(REF, fname)
    tree = ast.parse(open(path).read(), path)
    body = tree.body
    if cls is not None:
        body = [n for n in body if isinstance(n, ast.ClassDef) and n.name == cls][0].body
    fns = {}
    for node in body:
        if isinstance(node, ast.FunctionDef) and node.name in names:
            node.decorator_list = []
            mod = ast.Module(body=[node], type_ignores=[])
            ns = {"torch": torch, "np": np}
            exec(compile(mod, path, "exec"), ns)
            fns[node.name] = ns[node.name]
    missing = set(names) - set(fns)
    assert not missing, missing
    return fns


# ------------------------------------------------------------ reference
class RefLosses:
    """``self`` stand-in for the extracted ModelManager loss methods."""

    def __init__(self, topo, bs=4, eta1=0.5, eta2=0.5, latent=75):
        fns = _extract_functions("model_manager.py", [
            "compute_mse_loss", "_compute_laplacian_regularizer",
            "_compute_kl_divergence_loss", "_compute_latent_consistency",
            "compute_vertex_errors"], cls="ModelManager")
        ufns = _extract_functions("utils.py", ["batch_mm"])
        utils_ns = types.SimpleNamespace(batch_mm=ufns["batch_mm"])
        for f in fns.values():
            f.__globals__["utils"] = utils_ns
        self.f = fns
        n = topo["pos_0"].shape[0]
        lap = torch.sparse_coo_tensor(
            torch.from_numpy(np.stack([topo["lap_row"], topo["lap_col"]]).astype(np.int64)),
            torch.from_numpy(topo["lap_val"]), (n, n))
        self.template = types.SimpleNamespace(laplacian=lap)
        self._optimization_params = {"batch_size": bs,
                                      "latent_consistency_eta1": eta1,
                                      "latent_consistency_eta2": eta2}
        keys = list(topo["region_keys"])
        rs = latent // len(keys)
        self._latent_regions = {k: [i * rs, (i + 1) * rs] for i, k in enumerate(keys)}
        self.to_mm_const = 89.11

    def mse(self, p, g):
        return self.f["compute_mse_loss"](p, g)

    def lap(self, p):
        return self.f["_compute_laplacian_regularizer"](self, p)

    def kl(self, mu, lv):
        return self.f["_compute_kl_divergence_loss"](mu, lv)

    def lc(self, z, key):
        return self.f["_compute_latent_consistency"](self, z, key)


def ref_transforms(topo):
    downs, ups = [], []
    for l in range(int(topo["n_levels"])):
        for name, lst in (("down", downs), ("up", ups)):
            idx = np.stack([topo[f"{name}_{l}_row"], topo[f"{name}_{l}_col"]]).astype(np.int64)
            lst.append(torch.sparse_coo_tensor(
                torch.from_numpy(idx), torch.from_numpy(topo[f"{name}_{l}_val"]),
                tuple(topo[f"{name}_{l}_shape"].tolist())))
    return downs, ups


def build_ref_model(modmodel, topo, weights, is_vae=True):
    spirals = [torch.from_numpy(topo[f"spiral_{l}"].astype(np.int64))
               for l in range(int(topo["n_levels"]))]
    downs, ups = ref_transforms(topo)
    m = modmodel.Model(3, [32, 32, 32, 64], 75, spirals, downs, ups,
                       pre_z_sigmoid=False, is_vae=is_vae)
    sd = m.state_dict()
    assert list(sd.keys()) == list(weights.keys()), (list(sd.keys()), list(weights.keys()))
    m.load_state_dict({k: torch.from_numpy(v) for k, v in weights.items()})
    return m


def stats(t):
    a = t.detach().double().numpy().ravel()
    return np.array([a.sum(), np.abs(a).sum(), np.sqrt((a * a).sum())])


def main():
    _install_shims()
    modmodel = _load_source_module("ref_model", "model.py")
    modswap = _load_source_module("ref_swap", "swap_batch_transform.py")
    topo = recipe.load_topology()
    weights = recipe.golden_weights()
    keys = list(topo["region_keys"])
    feat = {k: {"feature": topo[f"region_{i}_feature"].tolist()} for i, k in enumerate(keys)}

    # ---------------- per-op goldens (small, stored in full)
    ops = {}
    rs = np.random.RandomState(42)
    sp3 = torch.from_numpy(topo["spiral_3"].astype(np.int64))
    conv = modmodel.SpiralConv(32, 64, sp3)
    w = rs.uniform(-0.1, 0.1, (64, 9 * 32)).astype(np.float32)
    b = rs.uniform(-0.1, 0.1, 64).astype(np.float32)
    conv.layer.weight.data.copy_(torch.from_numpy(w))
    conv.layer.bias.data.copy_(torch.from_numpy(b))
    x = torch.from_numpy(rs.randn(2, 267, 32).astype(np.float32)).requires_grad_()
    dy = torch.from_numpy(rs.randn(2, 267, 64).astype(np.float32))
    y = conv(x)
    y.backward(dy)
    ops.update(conv_w=w, conv_b=b, conv_x=x.detach().numpy(), conv_dy=dy.numpy(),
               conv_y=y.detach().numpy(), conv_dx=x.grad.numpy(),
               conv_dw=conv.layer.weight.grad.numpy(), conv_db=conv.layer.bias.grad.numpy())
    # 2-D input path (model.py:29-31)
    x2 = x.detach()[0].clone().requires_grad_()
    conv.zero_grad()
    y2 = conv(x2)
    ops.update(conv2d_y=y2.detach().numpy())
    downs, ups = ref_transforms(topo)
    for name, tr, n_in in (("down3", downs[3], 267), ("up3", ups[3], 67),
                           ("up2", ups[2], 267)):
        xp = torch.from_numpy(rs.randn(2, n_in, 64).astype(np.float32)).requires_grad_()
        out = modmodel.Pool(xp, tr)
        dout = torch.from_numpy(rs.randn(*out.shape).astype(np.float32))
        out.backward(dout)
        ops.update({f"pool_{name}_x": xp.detach().numpy(), f"pool_{name}_out": out.detach().numpy(),
                    f"pool_{name}_dout": dout.numpy(), f"pool_{name}_dx": xp.grad.numpy()})
    np.savez_compressed(os.path.join(HERE, "golden_ops.npz"), **ops)

    # ---------------- swap goldens (bit-exact, sha256 per key)
    swapper = modswap.SwapFeatures(types.SimpleNamespace(feat_and_cont=feat))
    base = recipe.normalized_meshes(4)
    shas = []
    for k in keys:
        outb = np.stack([np.asarray(base[i]) if i == j else
                         swapper.swap(base[i], base[j], k).numpy()
                         for i in range(4) for j in range(4)])
        # reference output index is i*bs+j; comprehension above is i-major
        shas.append(recipe.sha256(outb.astype(np.float32)))
    # full __call__ path once (key drawn by random.choice, seeded)
    import random
    random.seed(0)
    bd = _Data(x=torch.from_numpy(base), y=["a", "b", "c", "n"],
               augmented=torch.zeros(4, 1), age=torch.arange(4.).view(4, 1),
               gender=["M", "F", "M", "F"])
    sw = swapper(bd)
    np.savez_compressed(os.path.join(HERE, "golden_swap.npz"),
                        sha=np.asarray(shas), call_key=np.asarray(sw.swapped),
                        call_x_sha=np.asarray(recipe.sha256(sw.x.numpy())),
                        call_age=sw.age.numpy(), call_aug=sw.augmented.numpy(),
                        call_y=np.asarray([str(v) for v in sw.y]),
                        call_gender=np.asarray(sw.gender))

    # ---------------- C1 eval golden
    model = build_ref_model(modmodel, topo, weights)
    model.eval()
    x8 = torch.from_numpy(recipe.normalized_meshes(8))
    with torch.no_grad():
        out, z, mu, lv = model(x8)
    np.savez_compressed(os.path.join(HERE, "golden_eval.npz"),
                        weights_sha=np.asarray(recipe.weights_sha256(weights)),
                        recon=out.numpy(), z=z.numpy(), mu=mu.numpy(), logvar=lv.numpy())

    # ---------------- C2 train goldens: 3 steps with Adam
    losses = RefLosses(topo)
    model = build_ref_model(modmodel, topo, weights)
    model.train()
    opt = torch.optim.Adam(model.parameters(), lr=1e-4, weight_decay=0)
    tr = {"weights_sha": np.asarray(recipe.weights_sha256(weights))}
    names = list(weights.keys())
    orig_randn_like = torch.randn_like
    for step in range(3):
        base = recipe.normalized_meshes(12)[4 * step:4 * step + 4] if step < 3 else None
        key = keys[recipe.train_key_index(step)]
        bd = _Data(x=torch.from_numpy(base.copy()), y=["a"] * 4,
                   augmented=torch.zeros(4, 1), age=torch.zeros(4, 1), gender=["M"] * 4)
        random_choice = random.choice
        random.choice = lambda seq, _k=key: _k
        try:
            data = swapper(bd)
        finally:
            random.choice = random_choice
        assert data.swapped == key
        eps = torch.from_numpy(recipe.train_eps(step))
        torch.randn_like = lambda t, _e=eps: _e.clone()
        try:
            opt.zero_grad()
            rec, z, mu, lv = model(data.x)
        finally:
            torch.randn_like = orig_randn_like
        l_rec = losses.mse(rec, data.x)
        l_lap = losses.lap(rec)
        l_kl = losses.kl(mu, lv)
        l_lc = losses.lc(z, data.swapped)
        tot = l_rec + 1e-4 * l_kl + 0.5 * l_lc + 0.1 * l_lap
        tot.backward()
        p = f"s{step}_"
        tr[p + "x_sha"] = np.asarray(recipe.sha256(data.x.numpy()))
        tr[p + "losses"] = np.array([l_rec.item(), l_kl.item(), l_lc.item(),
                                     l_lap.item(), tot.item()])
        tr[p + "rec_stats"] = stats(rec)
        tr[p + "rec_sample"] = rec.detach().numpy().reshape(-1)[recipe.sample_idx(rec.numel(), 256)]
        tr[p + "z"] = z.detach().numpy()
        for name, prm in zip(names, model.parameters()):
            g = prm.grad
            tr[p + "grad_stats_" + name] = stats(g)
            tr[p + "grad_sample_" + name] = g.numpy().reshape(-1)[recipe.sample_idx(g.numel())]
        opt.step()
        for name, prm in zip(names, model.parameters()):
            tr[p + "param_stats_" + name] = stats(prm)
            tr[p + "param_sample_" + name] = prm.detach().numpy().reshape(-1)[
                recipe.sample_idx(prm.numel())]
        print("step", step, "key", key, "losses", tr[p + "losses"])
    np.savez_compressed(os.path.join(HERE, "golden_train.npz"), **tr)


if __name__ == "__main__":
    main()
