"""Data side of the training path: the reference's dataset / loader / feature
swap (``data_loading.py:23-283``, ``swap_batch_transform.py:7-52``) with the
swap on the GPU.

Two ways in:

* drop-in objects with the reference's interface -- :class:`Data` (the
  attribute bag ``torch_geometric.data.Data`` is used as),
  :class:`SwapFeatures` ``(template)(batched_data)`` and
  :class:`MeshCollater` -- for a host DataLoader: the collated batch is moved
  to the device once and swapped there by ``cfsd_swap_features``, and the
  label fields (y / augmented / age / gender / swapped) are built exactly as
  the reference builds them;
* the resident path the training driver uses: :func:`load_mesh_dataset` reads
  the mesh files once, splits and normalises them as the reference does, and
  returns :class:`engine.ResidentData` sets (whole set in HBM, device-drawn
  epoch shuffle, swap fused into the step).
"""
import json
import os
import random

import numpy as np
import torch
from torch.utils.data.dataloader import default_collate

from . import ops
from .engine import ResidentData


class Data:
    """Attribute bag standing in for ``torch_geometric.data.Data`` (the
    reference stores x / y / augmented / age / gender / swapped on it)."""

    def __init__(self, **kwargs):
        for k, v in kwargs.items():
            setattr(self, k, v)

    @property
    def keys(self):
        return [k for k in vars(self)]

    def __getitem__(self, k):
        return getattr(self, k)

    def __setitem__(self, k, v):
        setattr(self, k, v)

    def to(self, device):
        for k in self.keys:
            v = getattr(self, k)
            if torch.is_tensor(v):
                setattr(self, k, v.to(device))
        return self


def _region_mask(feat_and_cont, nv, device):
    keys = list(feat_and_cont.keys())
    mask = np.zeros((len(keys), nv), np.uint8)
    for i, k in enumerate(keys):
        mask[i, np.asarray(feat_and_cont[k]["feature"], np.int64)] = 1
    return torch.from_numpy(mask).to(device)


class SwapFeatures:
    """``SwapFeatures`` (swap_batch_transform.py:7-42): ``bs`` meshes ->
    ``bs**2``; output ``i*bs + j`` is mesh ``i`` with the feature vertices of
    one random region (``random.choice`` over the template's regions, as the
    reference) taken from mesh ``j``.  ``batched_data.x`` must be a device
    tensor (the swap runs on the GPU, bit-exact); labels as the reference:
    diagonal entries keep the originals, off-diagonal ones get y None,
    augmented 1, age -1, gender 'n/a'; ``swapped`` = the region key."""

    def __init__(self, template):
        self._template = template
        self._features_and_contours = template.feat_and_cont
        self._zones_keys = list(template.feat_and_cont.keys())
        self._masks = {}

    def __call__(self, batched_data, key=None):
        x = batched_data.x
        if not x.is_cuda:
            raise RuntimeError("SwapFeatures runs on the GPU: move the collated batch to the device first")
        bs = x.shape[0]
        nv = x.shape[1]
        dev = x.device
        if dev not in self._masks:
            self._masks[dev] = _region_mask(self._features_and_contours, nv, dev)
        key = random.choice(self._zones_keys) if key is None else key
        kidx = torch.tensor([self._zones_keys.index(key)], dtype=torch.int32, device=dev)
        new_batch = ops.swap_features(x.contiguous().float(), torch.arange(bs, dtype=torch.int32, device=dev),
                                      self._masks[dev], kidx, bs)
        aug = batched_data.augmented
        age = batched_data.age
        aug_t = torch.as_tensor(aug)
        age_t = torch.as_tensor(age)
        new_y = [None] * (bs ** 2)
        new_aug = torch.ones([bs ** 2, 1], device=aug_t.device, dtype=aug_t.dtype)
        new_gender = ["n/a"] * (bs ** 2)
        new_age = -torch.ones([bs ** 2, 1], device=age_t.device, dtype=age_t.dtype)
        for i in range(bs):
            d = i * bs + i
            new_y[d] = batched_data.y[i]
            new_aug[d] = aug_t[i]
            new_gender[d] = batched_data.gender[i]
            new_age[d] = age_t[i]
        return Data(x=new_batch, y=new_y, swapped=key, augmented=new_aug, age=new_age, gender=new_gender)


class MeshCollater:
    """``MeshCollater`` (data_loading.py:62-83): default-collate every field
    of a list of :class:`Data`, move the batch to ``device`` and swap there.
    Use it with ``num_workers=0`` (the swap needs the GPU; the reference
    swapped on CPU in 8 worker processes)."""

    def __init__(self, feature_swapper=None, device="cuda"):
        self._swapper = feature_swapper
        self._device = torch.device(device)

    def __call__(self, data_list):
        return self.collate(data_list)

    def collate(self, data_list):
        if not isinstance(data_list[0], Data):
            raise TypeError(f"DataLoader found invalid type: {type(data_list[0])}. "
                            f"Expected craniofacialsd_vae_amd.data.Data instead")
        keys = list(set.union(*[set(d.keys) for d in data_list]))
        batched = Data()
        for key in keys:
            batched[key] = default_collate([d[key] for d in data_list])
        batched.x = batched.x.to(self._device)
        if self._swapper is not None:
            batched = self._swapper(batched)
        return batched


# ------------------------------------------------------------------ dataset files
def read_obj_vertices(path):
    """Vertices of an OBJ file in file order (trimesh ``process=False``)."""
    vs = []
    with open(path) as f:
        for ln in f:
            if ln.startswith("v "):
                vs.append([float(t) for t in ln.split()[1:4]])
    return np.asarray(vs, np.float64)


def write_obj(path, verts, faces=None):
    """OBJ with ``v`` lines (9 significant digits: fp32 round-trips) and
    1-based ``f`` lines (what ``mesh1.export`` of the augmented mesh writes,
    data_loading.py:369-372)."""
    v = np.asarray(verts, np.float64)
    lines = ["v %.9g %.9g %.9g" % tuple(p) for p in v]
    if faces is not None:
        lines += ["f %d %d %d" % tuple(t) for t in (np.asarray(faces, np.int64) + 1)]
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")


def load_mesh(path):
    """``MeshInMemoryDataset.load_mesh`` (data_loading.py:220-229): vertices
    as float32."""
    if path.endswith(".ply"):
        from .precompute import read_ply
        return torch.tensor(read_ply(path)[0], dtype=torch.float)
    return torch.tensor(read_obj_vertices(path), dtype=torch.float)


# ------------------------------------------------------------------ dataset summary
def get_dataset_summary(data_config, data_type="heads"):
    """``utils.get_dataset_summary`` (utils.py:193-208): the spreadsheet of
    subjects (Dataset / ID|PID / AgeMonths / AgeYears / Gender / "Head Used"|
    "Face Used") with a ``mesh_name`` column '<class letter>_<id>'; ``None``
    without ``dataset_summary_path``.  ``.xlsx`` goes through pandas'
    ``read_excel`` (needs openpyxl, absent from this image: the error is
    pandas' own); a ``.csv`` with the same columns is read with
    ``read_csv``."""
    path = data_config.get("dataset_summary_path")
    if not path:
        return None
    import pandas as pd
    d = pd.read_csv(path) if path.endswith(".csv") else pd.read_excel(path)
    d["mesh_name"] = "nan"
    for ds, letter in (("Paeds", "b"), ("Apert", "a"), ("Crouzon", "c"), ("Muenke", "m"), ("LSFM", "n"),
                       ("LYHM", "n")):
        d.loc[d["Dataset"] == ds, "mesh_name"] = letter
    id_column = "ID" if data_type == "heads" else "PID"
    d["mesh_name"] = d["mesh_name"] + "_" + d[id_column].fillna(-1).astype(int).astype(str)
    return d


def find_data_used_from_summary(summary, data_type="heads"):
    """``utils.find_data_used_from_summary`` (utils.py:211-217)."""
    if summary is None:
        return None
    col = "Head Used" if data_type == "heads" else "Face Used"
    return list(summary.loc[summary[col] == "y"]["mesh_name"])


def get_age_and_gender_from_summary(summary, mesh_id):
    """``utils.get_age_and_gender_from_summary`` (utils.py:220-231): age in
    months (years * 12 + 6 when only years are known), gender; (-1, 'n/a')
    for meshes the summary does not list (augmented meshes) -- and, here,
    when there is no summary at all (the reference would raise)."""
    if summary is None:
        return -1, "n/a"
    try:
        rows = summary.loc[summary["mesh_name"] == mesh_id]
        age = rows["AgeMonths"].values[0]
        if np.isnan(age):
            age = rows["AgeYears"].values[0] * 12 + 6
        gender = rows["Gender"].values[0]
    except IndexError:
        age, gender = -1, "n/a"
    return age, gender


def find_filenames(root, data_to_use=None, find_augmented=False):
    """``MeshInMemoryDataset.find_filenames`` (data_loading.py:166-178): every
    .ply / .obj outside 'aug' folders whose stem the dataset summary marks as
    used (all of them without a summary); with ``find_augmented`` also those
    inside, as 'augmented/<name>'."""
    files = []
    for dirpath, _, fnames in os.walk(root):
        for f in fnames:
            if f.endswith(".ply") or f.endswith(".obj"):
                if "aug" not in dirpath:
                    if data_to_use is None or f[:-4] in data_to_use:
                        files.append(f)
                elif find_augmented:
                    files.append(os.path.join("augmented", f))
    return files


# ------------------------------------------------------------------ augmentation
def augment_train_list(root, train_list, data_config, template=None, device="cuda", summary=None,
                       precomputed_path=None, seed=0):
    """``MeshInMemoryDataset._augment`` (data_loading.py:292-374) with the
    meshes generated on the GPU (:mod:`augment`).

    * ``<root>/augmented`` exists and is non-empty: its meshes are appended
      (in sorted order; the reference takes ``os.listdir`` order) and nothing
      is generated (:295-303);
    * else: pairs per (merged) class and age group, balanced counts
      (:314-335), eigenpairs k = 1000 of the template's combinatorial
      Laplacian (cached as ``laplacian_eig_k1000.npz`` in the precomputed
      folder), one batched GPU blend per 1024 pairs, and every result is
      written to ``<root>/augmented/<name1>_<id2><_spectral_interp|..><i><ext>``
      (:371-373) with the template's faces, then appended to the list.
    Returns the extended train list (a new list)."""
    from . import augment as A
    train_list = list(train_list)
    aug_dir = os.path.join(root, "augmented")
    if os.path.isdir(aug_dir) and os.listdir(aug_dir):
        for name in sorted(os.listdir(aug_dir)):
            if name.endswith(".obj") or name.endswith(".ply"):
                train_list.append(os.path.join("augmented", name))
        return train_list
    mode = data_config.get("augmentation_mode", "interpolate")
    factor = int(data_config["augmentation_factor"])
    balanced = bool(data_config.get("augmentation_balanced", True))
    if template is None:
        from .precompute import load_template
        template = load_template(data_config["template_path"])
    initial = list(train_list)
    raw = torch.stack([load_mesh(os.path.join(root, n)) for n in initial]).to(device)
    letters = [n[0] for n in initial]
    ages = [get_age_and_gender_from_summary(summary, n[:-4])[0] for n in initial]
    ages = None if summary is None else ages
    u = None
    if mode in ("spectral_interp", "spectral_comb"):
        cache = os.path.join(precomputed_path, "laplacian_eig_k1000.npz") if precomputed_path else None
        k = min(1000, template.num_nodes - 1)
        _, u = A.laplacian_eigendecomposition(template.faces, template.num_nodes, k=k, device=device,
                                              cache=cache)
    aug, cls, (i1, i2, idx, tv) = A.augment(u, raw, letters, ages, aug_factor=factor, balanced=balanced,
                                        mode=mode, seed=seed)
    os.makedirs(aug_dir, exist_ok=True)
    suffix = {"spectral_comb": "_spectral_comb", "spectral_interp": "_spectral_interp"}
    host = aug.cpu().numpy()
    for j in range(len(cls)):
        n1, n2 = initial[int(i1[j])], initial[int(i2[j])]
        tag = (suffix[mode] + str(int(idx[j]))) if mode in suffix else f"_interp{float(tv[j]):.2f}"
        name = n1[:-4] + "_" + n2[2:-4] + tag + n1[-4:]
        path = os.path.join(aug_dir, name)
        if name.endswith(".ply"):
            from .precompute import write_ply
            write_ply(path, host[j], template.faces)
        else:
            write_obj(path, host[j], template.faces)
        train_list.append(os.path.join("augmented", name))
    return train_list


def split_data(root, split_path, stratified=False, data_config=None, template=None, device="cuda",
               summary=None, seed=0):
    """``MeshInMemoryDataset.split_data`` (data_loading.py:180-218): reuse
    ``data_split.json`` when present, else sort the file names and split
    (stratified 80/10/10 by class letter with sklearn, or the reference's
    ``i % 100`` rule: <= 5 test, <= 10 validation, else train), augment the
    training list when ``augmentation_factor > 0`` (:207-213) and write the
    json."""
    try:
        with open(split_path) as fp:
            d = json.load(fp)
        return d["train"], d["test"], d["val"]
    except FileNotFoundError:
        pass
    data_config = data_config or {}
    data_to_use = find_data_used_from_summary(summary, data_config.get("data_type", "heads"))
    names = sorted(find_filenames(root, data_to_use))
    if stratified:
        from sklearn.model_selection import train_test_split
        y = [n[0] for n in names]
        train, test, _, test_y = train_test_split(names, y, stratify=y, test_size=0.2)
        test, val, _, _ = train_test_split(test, test_y, stratify=test_y, test_size=0.5)
    else:
        train, test, val = [], [], []
        for i, f in enumerate(names):
            (test if i % 100 <= 5 else val if i % 100 <= 10 else train).append(f)
    if int(data_config.get("augmentation_factor", 0) or 0) > 0:
        train = augment_train_list(root, train, data_config, template, device, summary,
                                   os.path.dirname(split_path), seed)
    with open(split_path, "w") as fp:
        json.dump({"train": train, "test": test, "val": val}, fp)
    return train, test, val


def labels_of(name):
    """Class label from the file name (data_loading.py:265-266): first letter
    ('b' paediatric folded into 'n'); 'aug' in the path marks augmentation."""
    base = name.split("/")[1] if "/" in name else name
    y = base[0]
    return ("n" if y == "b" else y), ("aug" in name)


def compute_mean_and_std(root, train_names, norm_path):
    """``compute_mean_and_std`` (data_loading.py:231-252): load ``norm.pt``
    (weights_only) or compute the per-vertex mean / std (torch, CPU) of the
    training meshes -- augmented ones included -- and save it."""
    try:
        return torch.load(norm_path, weights_only=True)
    except FileNotFoundError:
        verts = torch.stack([load_mesh(os.path.join(root, n)) for n in train_names])
        mean = torch.mean(verts, dim=0)
        std = torch.std(verts, dim=0)
        std = torch.where(std > 0, std, torch.tensor(1e-8))
        norm = {"mean": mean, "std": std}
        torch.save(norm, norm_path)
        return norm


def prepare_split(data_config, template=None, device="cuda", seed=0):
    """The files the data sets are defined by: ``data_split.json`` (with
    augmentation, :func:`split_data`) and ``norm.pt`` in the precomputed
    folder, made once (data-parallel: by rank 0 before the others load).
    Returns (train, test, val, norm, summary)."""
    root = data_config["dataset_path"]
    pre = data_config["precomputed_path"]
    os.makedirs(pre, exist_ok=True)
    summary = get_dataset_summary(data_config, data_config.get("data_type", "heads"))
    train, test, val = split_data(root, os.path.join(pre, "data_split.json"),
                                  data_config.get("stratified_split", False), data_config, template, device,
                                  summary, seed)
    norm = compute_mean_and_std(root, train, os.path.join(pre, "norm.pt"))
    return train, test, val, norm, summary


def load_mesh_dataset(data_config, batch_size, device="cuda", template=None, shard=None, seed=0):
    """``get_data_loaders`` (data_loading.py:23-51) for the resident path:
    train / validation / test :class:`engine.ResidentData` sets (meshes
    normalised on the device with norm.pt, data_loading.py:259-260; train and
    validation shuffled every epoch with drop_last, test in file order) plus
    the normalisation dict and the per-set file names and labels.

    ``shard=(rank, world)`` (data-parallel training): the train and
    validation sets iterate over this rank's contiguous shard only (the whole
    set stays resident; the test set is not sharded)."""
    root = data_config["dataset_path"]
    train, test, val, norm, summary = prepare_split(data_config, template, device, seed)
    sets = {}
    for kind, names, shuffle in (("train", train, True), ("val", val, True), ("test", test, False)):
        if len(names) < batch_size:
            sets[kind] = None
            continue
        meshes = torch.stack([load_mesh(os.path.join(root, n)) for n in names]).to(device)
        rows, n_batches = None, None
        # (a shard smaller than one batch: every rank iterates the whole set;
        # the decision depends on the sizes only, so all ranks agree)
        if shard is not None and kind != "test" and shard[1] > 1 and len(names) // shard[1] >= batch_size:
            from .dist import shard_range, steps_per_epoch
            lo, hi = shard_range(len(names), shard[0], shard[1])
            rows = torch.arange(lo, hi, dtype=torch.int32)
            # shards differ by <= 1 mesh: every rank runs the smallest shard's count
            n_batches = steps_per_epoch(len(names), shard[1], batch_size)
        rd = ResidentData(meshes, bs=batch_size, rows=rows, shuffle=shuffle,
                          norm=norm if data_config.get("normalize_data", True) else None, n_batches=n_batches)
        rd.names = list(names)
        rd.labels = [labels_of(n) for n in names]
        ag = [get_age_and_gender_from_summary(summary, n[:-4]) for n in names]
        rd.ages = [a for a, _ in ag]
        rd.genders = [g for _, g in ag]
        sets[kind] = rd
    return sets["train"], sets["val"], sets["test"], norm
