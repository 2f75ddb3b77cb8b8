"""Host side of the training driver (no kernel launches): dataset split rule,
labels, OBJ reading, config/log helpers, and the execution-free reader of the
reference's precomputed cache (checked against the committed fixture)."""
import json
import os

import numpy as np
import pytest
import torch

import cfsd_loader

cfsd_loader.load()
from craniofacialsd_vae_amd import data as D  # noqa: E402
from craniofacialsd_vae_amd import manager as M  # noqa: E402
from craniofacialsd_vae_amd import refcache  # noqa: E402


def test_split_rule_and_labels(tmp_path):
    for i in range(130):
        (tmp_path / f"{'abcn'[i % 4]}_{i:03d}.obj").write_text("v 0 0 0\n")
    (tmp_path / "aug").mkdir()
    (tmp_path / "aug" / "n_x.obj").write_text("v 0 0 0\n")
    train, test, val = D.split_data(str(tmp_path), str(tmp_path / "split.json"))
    names = sorted(f for f in os.listdir(tmp_path) if f.endswith(".obj"))
    assert test == [n for i, n in enumerate(names) if i % 100 <= 5]
    assert val == [n for i, n in enumerate(names) if 5 < i % 100 <= 10]
    assert len(train) == 130 - len(test) - len(val) and "n_x.obj" not in train
    assert json.load(open(tmp_path / "split.json"))["val"] == val
    # a second call reuses the file
    (tmp_path / "z_999.obj").write_text("v 0 0 0\n")
    assert D.split_data(str(tmp_path), str(tmp_path / "split.json"))[0] == train
    assert D.labels_of("b_001.obj") == ("n", False)
    assert D.labels_of("augmented/c_1_2_spectral_interp3.obj") == ("c", True)


def test_obj_reader_and_jsonl(tmp_path):
    p = tmp_path / "m.obj"
    p.write_text("# c\nv 1 2 3\nvn 0 0 1\nv 4.5 -1e-3 7\nf 1 2 1\n")
    assert np.array_equal(D.read_obj_vertices(str(p)), [[1, 2, 3], [4.5, -1e-3, 7]])
    w = M.JsonlWriter(str(tmp_path / "logs"))
    w.add_scalar("train/tot", 0.5, 1)
    assert json.loads(open(w.path).read()) == {"tag": "train/tot", "value": 0.5, "step": 1}


def test_refcache_reads_reference_precomputed(topo_npz):
    ref = "/root/reference/demo_files"
    if not os.path.exists(os.path.join(ref, "spirals.pkl")):
        pytest.skip("reference demo_files not present (build container only)")
    h = refcache.load_precomputed(ref)
    for l in range(4):
        assert np.array_equal(h[f"spiral_{l}"], topo_npz[f"spiral_{l}"])
        for k in ("down", "up"):
            for f in ("row", "col", "val", "shape"):
                assert np.array_equal(h[f"{k}_{l}_{f}"], topo_npz[f"{k}_{l}_{f}"])
        assert np.array_equal(h[f"face_{l + 1}"], topo_npz[f"face_{l + 1}"])


def _tiny_dataset(root, letters):
    """Small OBJ meshes (6 vertices, 4 faces) named '<letter>_<id>.obj'."""
    rs = np.random.RandomState(5)
    base = rs.normal(size=(6, 3))
    faces = np.array([[0, 1, 2], [0, 2, 3], [0, 3, 4], [0, 4, 5]])
    for i, c in enumerate(letters):
        D.write_obj(str(root / f"{c}_{i:03d}.obj"), base + rs.normal(0, 0.1, base.shape), faces)
    return base, faces


def test_balanced_counts_unmerged_divisor():
    """data_loading.py:314-335: 'b' is merged into 'n' for the per-class
    loop, but the balanced target divides by the letters BEFORE the merge."""
    from craniofacialsd_vae_amd import augment as A
    from oracle import cfsd_oracle as O
    names = [f"{c}_{i}.obj" for i, c in enumerate("aabbbnnnccm")]
    letters = [n[0] for n in names]
    exp = O.augment_counts(names, 5, True)
    assert exp == {"a": 9, "n": 5, "c": 9, "m": 10}   # 5 * 11 // 5 = 11 per class
    got = {c: max(0, v) for c, v in A.balanced_counts(letters, 5, True).items()}
    assert got == exp
    assert {c: max(0, v) for c, v in A.balanced_counts(letters, 3, False).items()} == O.augment_counts(names, 3, False)


def test_split_with_factor_interpolate(tmp_path):
    """(The test name avoids "aug": find_filenames skips any directory path
    containing it, data_loading.py:171, and pytest names tmp_path after the
    test.)  split_data with augmentation_factor > 0 (data_loading.py:207-218,
    292-374; mode 'interpolate', the one mode without eigenpairs, so it runs
    on the CPU here -- the spectral modes are GPU-tested):
    per-class counts as the reference's rule, names
    name1[:-4]_name2[2:-4]_interp<v.2f>.ext in the train split and
    data_split.json, norm.pt over the AUGMENTED train list, the augmented
    label, and reuse of an existing 'augmented' folder."""
    from craniofacialsd_vae_amd import precompute
    from oracle import cfsd_oracle as O
    root = tmp_path / "meshes"
    root.mkdir()
    letters = "aaabbnnnncccmmm" * 2
    base, faces = _tiny_dataset(root, letters)
    pre = tmp_path / "pre"
    pre.mkdir()
    cfg = {"dataset_path": str(root), "precomputed_path": str(pre), "augmentation_factor": 3,
           "augmentation_mode": "interpolate", "augmentation_balanced": True}
    tpl = precompute.Template(base.astype(np.float32), faces)
    train, test, val, norm, summary = D.prepare_split(cfg, template=tpl, device="cpu", seed=4)
    assert summary is None
    orig = [n for n in train if not n.startswith("augmented/")]
    augn = [n for n in train if n.startswith("augmented/")]
    assert len(orig) + len(test) + len(val) == len(letters)
    exp = O.augment_counts(orig, 3, True)
    got = {}
    for n in augn:
        base_name = n.split("/")[1]
        got[D.labels_of(n)[0]] = got.get(D.labels_of(n)[0], 0) + 1
        assert D.labels_of(n)[1] is True
        stem, ext = base_name[:-4], base_name[-4:]
        assert ext == ".obj" and "_interp" in stem and stem[-3] == "." and (root / n).exists()
        # the first name part is a training mesh of the same merged class
        assert any(stem.startswith(o[:-4] + "_") for o in orig if D.labels_of(o)[0] == D.labels_of(n)[0])
    assert got == {c: v for c, v in exp.items() if v}
    assert json.load(open(pre / "data_split.json"))["train"] == train
    verts = torch.stack([D.load_mesh(str(root / n)) for n in train])
    m, s = O.mean_std(verts)
    assert torch.equal(norm["mean"], m) and torch.equal(norm["std"], s)
    # interpolation between the pair: every augmented mesh lies on a segment
    # between two same-class originals (value in [0, 1))
    # an existing augmented folder is reused (no new draws)
    os.remove(pre / "data_split.json")
    n_files = len(os.listdir(root / "augmented"))
    tr2, _, _ = D.split_data(str(root), str(pre / "data_split.json"), False, cfg, tpl, "cpu", None, 9)
    assert len(os.listdir(root / "augmented")) == n_files
    assert sorted(tr2) == sorted(train)


def test_dataset_summary_csv(tmp_path):
    """utils.py:193-231 on a CSV summary with the spreadsheet's columns:
    mesh_name '<letter>_<id>', the 'Head Used' filter in find_filenames, ages
    in months (years * 12 + 6 when only years are known), (-1, 'n/a') for
    unlisted meshes."""
    import pandas as pd
    p = tmp_path / "summary.csv"
    pd.DataFrame({"Dataset": ["Apert", "Paeds", "LSFM", "Crouzon"], "ID": [1, 2, 3, 4],
                  "PID": [11, 12, 13, 14], "AgeMonths": [30, np.nan, 100, 12],
                  "AgeYears": [2.5, 4, 8.3, 1], "Gender": ["M", "F", "F", "M"],
                  "Head Used": ["y", "y", "n", "y"]}).to_csv(p, index=False)
    summ = D.get_dataset_summary({"dataset_summary_path": str(p)}, "heads")
    assert list(summ["mesh_name"]) == ["a_1", "b_2", "n_3", "c_4"]
    used = D.find_data_used_from_summary(summ, "heads")
    assert used == ["a_1", "b_2", "c_4"]
    assert D.get_age_and_gender_from_summary(summ, "b_2") == (54.0, "F")
    assert D.get_age_and_gender_from_summary(summ, "a_1") == (30.0, "M")
    assert D.get_age_and_gender_from_summary(summ, "augmented/x") == (-1, "n/a")
    root = tmp_path / "m"
    root.mkdir()
    for n in ("a_1", "b_2", "n_3", "c_4"):
        (root / f"{n}.obj").write_text("v 0 0 0\n")
    assert sorted(D.find_filenames(str(root), used)) == ["a_1.obj", "b_2.obj", "c_4.obj"]
