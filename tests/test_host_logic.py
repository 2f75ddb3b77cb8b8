"""CPU tests of the host side: C-ABI exports, index-table builders, engine
parameter layout.  No kernel is launched here (no GPU in the build container)."""
import ctypes
import os
import re

import numpy as np
import pytest

import cfsd_loader

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
cfsd_loader.load()
from craniofacialsd_vae_amd import _abi, topology  # noqa: E402


def header_functions():
    src = open(os.path.join(ROOT, "include", "cfsd.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(cfsd_[a-z0-9_]+)\s*\(", src)))


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(_abi.LIB_PATH):
        pytest.skip("libcfsd.so not built (run __graft_entry__.build())")
    return _abi.load()


def test_library_exports_every_header_symbol(lib):
    names = header_functions()
    assert len(names) >= 20
    for n in names:
        assert hasattr(lib, n), n
    assert set(names) == set(_abi.SIGNATURES), set(names) ^ set(_abi.SIGNATURES)


def test_version_and_error_reporting(lib):
    assert lib.cfsd_version() >> 16 == 4  # 4.0: CFSD_VM vertex-major operands
    # argument validation happens before any HIP call: safe without a GPU
    rc = lib.cfsd_spiral_conv_fwd(None, None, None, None, None, None, 0, 1, 1, 1, 9, 32, 32, 0, None)
    assert rc == -1
    assert b"null" in lib.cfsd_last_error_string()
    rc = lib.cfsd_spiral_conv_fwd(ctypes.c_void_p(16), ctypes.c_void_p(16), ctypes.c_void_p(16), None,
                                  ctypes.c_void_p(16), None, 0, 1, 10, 10, 7, 32, 32, 0, None)
    assert rc == -1 and b"spiral length" in lib.cfsd_last_error_string()
    assert lib.cfsd_spiral_conv_bwd_weight_workspace(16, 17039, 9, 32, 32) > 0
    assert lib.cfsd_spiral_conv_bwd_weight_workspace(16, 17039, 9, 7, 5) == 0


def test_inverse_spiral_matches_bruteforce():
    rs = np.random.RandomState(0)
    idx = rs.randint(0, 50, size=(80, 9))
    ptr, rows, head = topology.inverse_spiral(idx, 50)
    assert head.shape == (50 * 9, topology.INV_HEAD)
    longest = 0
    for u in range(50):
        for s in range(9):
            k = u * 9 + s
            got = rows[ptr[k]:ptr[k + 1]].tolist()
            exp = [r for r in range(80) if idx[r, s] == u]
            assert got == exp
            longest = max(longest, len(exp))
            for j in range(topology.INV_HEAD):
                assert head[k, j] == (exp[j] if len(exp) > j else -1)
    assert longest > topology.INV_HEAD  # the overflow path is exercised


def test_inverse_flat_matches_bruteforce(topo_npz):
    """Flattened spiral positions p = r*9 + s per source vertex, ascending
    (the reference's index_add_ order), -1 padded to a multiple of 4."""
    rs = np.random.RandomState(1)
    idx = rs.randint(0, 60, size=(30, 9))
    flat, width = topology.inverse_flat(idx, 60)
    assert width % 4 == 0 and flat.shape == (60, width)
    for u in range(60):
        exp = [p for p in range(30 * 9) if idx.reshape(-1)[p] == u]
        assert flat[u].tolist() == exp + [-1] * (width - len(exp))
    # the craniofacial Enblock subsets (levels 1-3) fit in 8 entries
    T = topology.DeviceTopology.from_npz(topo_npz, device="cpu")
    for lv in (1, 2, 3):
        tab, w = T.enc_flat[lv]
        assert w == 8 and tuple(tab.shape) == (T.n_verts[lv], 8)
    assert topology.inverse_flat(np.zeros((20, 9), np.int64), 1) == (None, 0)


def test_csr_keeps_file_order_and_transpose():
    row = np.array([2, 0, 2, 1, 0, 2])
    col = np.array([5, 1, 0, 3, 4, 2])
    val = np.arange(6, dtype=np.float32)
    ptr, c, v = topology.csr_from_coo(row, col, val, 3)
    assert ptr.tolist() == [0, 2, 3, 6]
    assert c.tolist() == [1, 4, 3, 5, 0, 2] and v.tolist() == [1, 4, 3, 0, 2, 5]
    tp, tc, tv = topology.csr_transpose_from_coo(row, col, val, 6)
    assert tp.tolist() == [0, 1, 2, 3, 4, 5, 6]
    assert tc.tolist() == [2, 0, 2, 1, 0, 2]


def test_selection_detection(topo_npz):
    for l in range(4):
        sel = topology.selection_rows(topo_npz[f"down_{l}_row"], topo_npz[f"down_{l}_col"],
                                      topo_npz[f"down_{l}_val"], int(topo_npz[f"down_{l}_shape"][0]))
        assert sel is not None and len(np.unique(sel)) == len(sel)
        up = topology.selection_rows(topo_npz[f"up_{l}_row"], topo_npz[f"up_{l}_col"],
                                     topo_npz[f"up_{l}_val"], int(topo_npz[f"up_{l}_shape"][0]))
        assert up is None


def test_device_topology_tables_on_cpu(topo_npz):
    T = topology.DeviceTopology.from_npz(topo_npz, device="cpu")
    assert T.n_verts == [17039, 4260, 1065, 267, 67]
    assert all(T.enc_select)
    assert T.n_regions == 15 and tuple(T.region_mask.shape) == (15, 17039)
    # row subset of level 0 == spiral rows of the kept vertices
    sel = topology.selection_rows(topo_npz["down_0_row"], topo_npz["down_0_col"],
                                  topo_npz["down_0_val"], 4260)
    np.testing.assert_array_equal(T.enc_rows[0].numpy(), topo_npz["spiral_0"][sel])
    # Laplacian rows sum to zero (random walk: 1 - sum 1/deg)
    ptr, col, val = (t.numpy() for t in T.lap_csr)
    sums = np.add.reduceat(val.astype(np.float64), ptr[:-1])
    assert np.abs(sums).max() < 1e-6


def test_engine_parameter_layout():
    from craniofacialsd_vae_amd.engine import ModelSpec
    import recipe
    spec = ModelSpec()
    specs = spec.param_specs(67, [9, 9, 9, 9])
    ref = recipe.param_shapes()
    assert sorted(specs) == sorted(ref)
    assert spec.reference_order(67, [9, 9, 9, 9]) == [k for k, _ in ref]
    names = [k for k, _ in specs]
    # stacked encoder Linears: logvar (en_layers.4) then mu (en_layers.5), adjacent
    i = names.index("en_layers.4.weight")
    assert names[i + 1] == "en_layers.5.weight"
    assert names[i + 2: i + 4] == ["en_layers.4.bias", "en_layers.5.bias"]
    assert sum(int(np.prod(s)) for _, s in specs) == 1081881


def test_checkpoint_format_round_trip(topo_npz, tmp_path):
    """f4 host side: save_weights / resume (model_manager.py:682-706) on an
    engine held in host memory (no kernel runs): reference file names and
    payload keys, bit-identical round trip, and the optimizer.pt payload is
    accepted by torch.optim.Adam over the reference parameter order."""
    import torch
    from craniofacialsd_vae_amd import engine as E
    topo = topology.DeviceTopology.from_npz(topo_npz, device="cpu")
    a = E.SDVAEEngine(topo, E.ModelSpec(), device="cpu")
    g = torch.Generator().manual_seed(0)
    a.params.exp_avg.normal_(generator=g)
    a.params.exp_avg_sq.uniform_(generator=g)
    a.params.step.fill_(7)
    assert a.save_weights(str(tmp_path), 4).endswith("model_00000005.pt")
    assert sorted(os.listdir(tmp_path)) == ["model_00000005.pt", "optimizer.pt"]
    b = E.SDVAEEngine(topo, E.ModelSpec(), device="cpu")
    assert b.resume(str(tmp_path)) == 5
    for buf in ("data", "exp_avg", "exp_avg_sq", "step"):
        assert torch.equal(getattr(a.params, buf), getattr(b.params, buf)), buf
    ck = torch.load(tmp_path / "model_00000005.pt", weights_only=True)["model"]
    assert list(ck) == list(a.state_dict())
    opt = torch.optim.Adam([v.clone().requires_grad_() for v in ck.values()], lr=1e-4)
    opt.load_state_dict(torch.load(tmp_path / "optimizer.pt", weights_only=True)["optimizer"])
    assert len(opt.state) == len(ck)
    st = opt.state_dict()["state"][3]
    assert float(st["step"]) == 7.0
    bad = a.optimizer_state_dict()
    bad["state"][0]["step"] = torch.tensor(3.0)
    with pytest.raises(ValueError):
        b.load_optimizer_state_dict(bad)


def test_epoch_permutation_is_a_permutation_per_epoch():
    """Oracle restatement of the device epoch shuffle (cfsd_step_begin): each
    epoch is a permutation of [0, n), epochs differ, drop_last batching."""
    from oracle import cfsd_oracle as O
    for n in (1, 2, 3, 7, 64, 250, 1000):
        p0, p1 = O.epoch_permutation(9, 0, n), O.epoch_permutation(9, 1, n)
        assert sorted(p0.tolist()) == list(range(n)) == sorted(p1.tolist())
        if n > 3:
            assert not np.array_equal(p0, p1)
    b = O.epoch_batches(9, 2, 10, 4, perm=np.arange(100, 110))
    assert b.shape == (2, 4) and len(np.unique(b)) == 8 and b.min() >= 100


def test_engine_requires_laplacian(topo_npz):
    from craniofacialsd_vae_amd import engine as E
    npz = {k: v for k, v in topo_npz.items() if not k.startswith("lap_")}
    topo = topology.DeviceTopology.from_npz(npz, device="cpu")
    with pytest.raises(ValueError, match="Laplacian"):
        E.SDVAEEngine(topo, E.ModelSpec(), device="cpu")
