"""On-device data path: device normalisation, per-epoch
shuffled drop_last batches, device-drawn VAE noise, range-guarded swap.

References: data_loading.py:40-48 (MeshLoader shuffle=True, drop_last=True),
data_loading.py:259-260 (normalisation), model.py:184-188 (randn_like noise),
swap_batch_transform.py:13-42 (swap)."""
import numpy as np
import pytest
import torch

import cfsd_loader
import recipe
from oracle import cfsd_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module")
def mods():
    cfsd_loader.load()
    from craniofacialsd_vae_amd import engine as E
    from craniofacialsd_vae_amd import ops, topology
    return E, ops, topology


@pytest.fixture(scope="module")
def dtopo(mods):
    _, _, topology = mods
    return topology.DeviceTopology.from_npz(recipe.load_topology(), device=DEV)


def test_normalize_bit_exact(mods):
    _, ops, _ = mods
    m = np.load(f"{recipe.HERE}/demo_meshes.npz")
    x = torch.from_numpy(m["verts"]).float()
    mean = torch.from_numpy(m["norm_mean"]).float()
    std = torch.from_numpy(m["norm_std"]).float()
    got = ops.normalize(x.to(DEV), mean.to(DEV), std.to(DEV)).cpu()
    ref = O.normalize(x, mean, std)
    assert torch.equal(got, ref)
    # the committed goldens were normalised the same way
    assert np.array_equal(got[:8].numpy(), recipe.normalized_meshes(8))


@pytest.mark.parametrize("n_items,bs,rows", [(256, 4, None), (10, 4, None), (7, 2, [9, 3, 5, 1, 0, 8, 2])])
def test_epoch_shuffle_visits_each_mesh_once(mods, n_items, bs, rows):
    """Every epoch visits each position exactly once (drop_last tail
    excluded), the order changes between epochs, and the device order is
    bit-exact to the oracle's restated permutation."""
    _, ops, _ = mods
    seed = 77
    counter = torch.zeros(1, dtype=torch.int32, device=DEV)
    bidx = torch.zeros(bs, dtype=torch.int32, device=DEV)
    perm = torch.tensor(rows, dtype=torch.int32, device=DEV) if rows is not None else None
    nb = n_items // bs
    seen = []
    for _ in range(3 * nb):
        ops.step_begin(counter, seed, batch_idx=bidx, bs=bs, n_batches=nb, perm=perm, n_items=n_items,
                       shuffle=True)
        seen.append(bidx.cpu().numpy().copy())
    seen = np.stack(seen).reshape(3, nb, bs)
    for e in range(3):
        exp = O.epoch_batches(seed, e, n_items, bs, perm=rows)
        assert np.array_equal(seen[e], exp), f"epoch {e}"
        flat = seen[e].ravel()
        assert len(np.unique(flat)) == nb * bs
    assert not np.array_equal(seen[0], seen[1])


def test_device_noise_drawn_when_not_injected(mods, dtopo):
    """a VAE train step without injected eps draws fresh finite
    noise on the device every step (the reference's randn_like)."""
    E, _, _ = mods
    eng = E.SDVAEEngine(dtopo, E.ModelSpec(), device=DEV)
    eng.load_state_dict({k: torch.from_numpy(v) for k, v in recipe.golden_weights().items()})
    x = torch.from_numpy(O.swap_features(recipe.normalized_meshes(4),
                                         O.Topology(recipe.load_topology()).region_features, 3)).to(DEV)
    b = eng.set_batch(x, key_index=3)
    eng.train_step_on(b)
    e1 = b.eps.clone()
    b = eng.set_batch(x, key_index=3)
    eng.train_step_on(b)
    e2 = b.eps.clone()
    torch.cuda.synchronize()
    assert torch.isfinite(e1).all() and torch.isfinite(e2).all()
    assert not torch.equal(e1, e2)
    assert 0.5 < e1.std().item() < 1.5 and abs(e1.mean().item()) < 0.3
    assert torch.isfinite(b.losses).all()
    # injected noise is kept as given
    eps = torch.from_numpy(recipe.train_eps(0)).to(DEV)
    b = eng.set_batch(x, key_index=3, eps=eps)
    eng.train_step_on(b)
    assert torch.equal(b.eps, eps)


def test_swap_guards_out_of_range_device_values(mods, dtopo):
    """A key outside [0, n_regions) swaps nothing; a mesh index outside the
    dataset is clamped (no GPU fault).  In-range values stay bit-exact."""
    _, ops, _ = mods
    meshes = torch.from_numpy(recipe.normalized_meshes(4)).to(DEV)
    bidx = torch.arange(4, dtype=torch.int32, device=DEV)
    key = torch.tensor([99], dtype=torch.int32, device=DEV)
    out = ops.swap_features(meshes, bidx, dtopo.region_mask, key, 4)
    ref = meshes.repeat_interleave(4, dim=0)  # out[i*4 + j] = mesh i
    assert torch.equal(out, ref)
    bidx = torch.tensor([0, 1, 2, 1000], dtype=torch.int32, device=DEV)
    key = torch.tensor([2], dtype=torch.int32, device=DEV)
    out = ops.swap_features(meshes, bidx, dtopo.region_mask, key, 4)
    bidx_ok = torch.tensor([0, 1, 2, 3], dtype=torch.int32, device=DEV)
    assert torch.equal(out, ops.swap_features(meshes, bidx_ok, dtopo.region_mask, key, 4))


def test_resident_data_normalises_and_trains(mods, dtopo):
    """ResidentData (normalised on device) + resident_step: the batch the step
    trained on is the swap of the oracle's epoch batch of normalised meshes."""
    E, ops, _ = mods
    m = np.load(f"{recipe.HERE}/demo_meshes.npz")
    raw = torch.from_numpy(m["verts"]).float().to(DEV)
    norm = {"mean": torch.from_numpy(m["norm_mean"]), "std": torch.from_numpy(m["norm_std"])}
    data = E.ResidentData(raw.clone(), bs=4, shuffle=True, norm=norm)
    assert data.n_batches == 3
    eng = E.SDVAEEngine(dtopo, E.ModelSpec(), device=DEV, seed=5)
    eng.load_state_dict({k: torch.from_numpy(v) for k, v in recipe.golden_weights().items()})
    b = eng.buffers(16)
    xs = O.normalize(torch.from_numpy(m["verts"]).float(), norm["mean"].float(), norm["std"].float())
    for step in range(4):
        eng.resident_step(b, data)
        torch.cuda.synchronize()
        epoch, bt = divmod(step, 3)
        base = O.epoch_batches(5, epoch, 12, 4)[bt]
        assert np.array_equal(b.batch_idx.cpu().numpy(), base)
        key = int(b.key.item())
        exp = O.swap_features(xs.numpy()[base], O.Topology(recipe.load_topology()).region_features, key)
        assert np.array_equal(b.x.cpu().numpy(), exp)
        assert torch.isfinite(b.losses).all()
