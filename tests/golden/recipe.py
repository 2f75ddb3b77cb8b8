"""Deterministic inputs shared by the golden generator and the tests.

TEST INFRASTRUCTURE.  The reference's pretrained ``model_00000600.pt`` is not
in the snapshot (``.MISSING_LARGE_BLOBS``), so every golden uses weights
drawn from a frozen NumPy stream instead: xavier-bound uniform matrices and
small NON-zero uniform biases (so bias gradients are exercised).  Parameter
order is the reference ``Model.named_parameters()`` order
(``model.py:103-137``).
"""
import hashlib
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))

IN_CH = 3
OUT_CH = [32, 32, 32, 64]
LATENT = 75
SEQ = 9


def param_shapes(num_vert=67, in_ch=IN_CH, out_ch=OUT_CH, latent=LATENT,
                 seq=SEQ, is_vae=True):
    """(name, shape) in reference ``named_parameters`` order."""
    shapes = []
    for i in range(len(out_ch)):
        cin = in_ch if i == 0 else out_ch[i - 1]
        shapes.append((f"en_layers.{i}.conv.layer.weight", (out_ch[i], seq * cin)))
        shapes.append((f"en_layers.{i}.conv.layer.bias", (out_ch[i],)))
    n = len(out_ch)
    shapes.append((f"en_layers.{n}.weight", (latent, num_vert * out_ch[-1])))
    shapes.append((f"en_layers.{n}.bias", (latent,)))
    if is_vae:
        shapes.append((f"en_layers.{n + 1}.weight", (latent, num_vert * out_ch[-1])))
        shapes.append((f"en_layers.{n + 1}.bias", (latent,)))
    shapes.append(("de_layers.0.weight", (num_vert * out_ch[-1], latent)))
    shapes.append(("de_layers.0.bias", (num_vert * out_ch[-1],)))
    for idx in range(len(out_ch)):
        if idx == 0:
            cin, cout = out_ch[-1], out_ch[-1]
        else:
            cin, cout = out_ch[-idx], out_ch[-idx - 1]
        shapes.append((f"de_layers.{idx + 1}.conv.layer.weight", (cout, seq * cin)))
        shapes.append((f"de_layers.{idx + 1}.conv.layer.bias", (cout,)))
    shapes.append((f"de_layers.{len(out_ch) + 1}.layer.weight", (in_ch, seq * out_ch[0])))
    shapes.append((f"de_layers.{len(out_ch) + 1}.layer.bias", (in_ch,)))
    return shapes


def golden_weights(shapes=None, seed=0):
    """Ordered dict name -> float32 ndarray from RandomState(seed)."""
    shapes = shapes if shapes is not None else param_shapes()
    rs = np.random.RandomState(seed)
    out = {}
    for name, shp in shapes:
        if name.endswith("bias"):
            out[name] = rs.uniform(-0.05, 0.05, size=shp).astype(np.float32)
        else:
            fan_out, fan_in = shp
            a = np.sqrt(6.0 / (fan_in + fan_out))
            out[name] = rs.uniform(-a, a, size=shp).astype(np.float32)
    return out


def weights_sha256(weights):
    h = hashlib.sha256()
    for k, v in weights.items():
        h.update(k.encode())
        h.update(np.ascontiguousarray(v, np.float32).tobytes())
    return h.hexdigest()


def train_eps(step, batch=16, latent=LATENT):
    """Injected VAE noise for golden train step ``step`` (replaces
    ``torch.randn_like`` at ``model.py:187``)."""
    return np.random.RandomState(1000 + step).randn(batch, latent).astype(np.float32)


def train_key_index(step):
    """Injected swap region for golden train step ``step`` (replaces
    ``random.choice`` at ``swap_batch_transform.py:26``)."""
    return (3 + 5 * step) % 15


def load_topology():
    return dict(np.load(os.path.join(HERE, "topology_craniofacial.npz")))


def load_meshes():
    return dict(np.load(os.path.join(HERE, "demo_meshes.npz")))


def normalized_meshes(n=None):
    m = load_meshes()
    v = (m["verts"] - m["norm_mean"][None]) / m["norm_std"][None]
    v = v.astype(np.float32)
    return v if n is None else v[:n]


def sha256(arr):
    return hashlib.sha256(np.ascontiguousarray(arr).tobytes()).hexdigest()


def sample_idx(n, k=64, seed=7):
    rs = np.random.RandomState(seed)
    return np.sort(rs.choice(n, size=min(k, n), replace=False))
