"""Host side of the training driver (no kernel launches): dataset split rule,
labels, OBJ reading, config/log helpers, and the execution-free reader of the
reference's precomputed cache (checked against the committed fixture)."""
import json
import os

import numpy as np
import pytest

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
