"""Diagnostics of the bf16 kernels (GPU): fraction of outputs equal to the
fp64 reference of the same bf16 inputs rounded to bf16, and max ulp error."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests", "golden")]
import cfsd_loader  # noqa: E402
import recipe  # noqa: E402
from oracle import cfsd_oracle as O  # noqa: E402

cfsd_loader.load()
from craniofacialsd_vae_amd import ops, topology  # noqa: E402

BF = torch.bfloat16
npz = recipe.load_topology()
ot = O.Topology(npz)
dt = topology.DeviceTopology.from_npz(npz, device="cuda")


def gather(x, sp):
    idx = torch.as_tensor(sp, dtype=torch.long)
    return torch.index_select(x, 1, idx.reshape(-1)).view(x.shape[0], idx.shape[0], -1)


def ulps(got_bf, ref64):
    r = ref64.to(BF)
    a = got_bf.cpu().view(torch.int16).int()
    b = r.view(torch.int16).int()
    d = (a - b).abs()
    return float((d == 0).float().mean()), int(d.max())


g = torch.Generator().manual_seed(0)
for lv, act in ((0, 1), (1, 1), (0, 0)):
    sp = ot.spirals[lv]
    x = torch.randn(4, sp.shape[0], 32, generator=g).to(BF)
    w = (torch.randn(32, 288, generator=g) * 0.1).to(BF)
    b = torch.randn(32, generator=g) * 0.1
    ref = gather(x.double(), sp) @ w.double().T + b.double()
    if act:
        ref = torch.nn.functional.elu(ref)
    out = torch.empty(4, sp.shape[0], 32, dtype=BF, device="cuda")
    ops.spiral_conv_fwd_x(x.cuda(), dt.spiral[lv], w.float().cuda(), w.cuda(), b.cuda(), act, out)
    print("fwd_b16 level", lv, "act", act, "exact frac, max ulp:", ulps(out, ref))
    out32 = torch.empty(4, sp.shape[0], 32, device="cuda")
    ops.spiral_conv_fwd_x(x.cuda(), dt.spiral[lv], w.float().cuda(), w.cuda(), b.cuda(), act, out32)
    print("   fp32 out max abs err", float((out32.cpu().double() - ref).abs().max()), "max |ref|", float(ref.abs().max()))
# E0
sp0 = ot.spirals[0]
sel = np.asarray(ot.down[0][1])[np.argsort(ot.down[0][0])]
x = torch.randn(4, sp0.shape[0], 3, generator=g)
w0 = torch.randn(32, 27, generator=g) * 0.1
b0 = torch.randn(32, generator=g) * 0.1
ref = torch.nn.functional.elu(gather(x.double(), sp0[sel]) @ w0.double().T + b0.double())
y = torch.empty(4, len(sel), 32, dtype=BF, device="cuda")
ops.spiral_conv_fwd_x(x.cuda(), dt.enc_rows[0], w0.cuda(), None, b0.cuda(), 1, y)
print("E0 in3 bf16 out exact frac, max ulp:", ulps(y, ref))
# Dout
h = torch.randn(4, sp0.shape[0], 32, generator=g).to(BF)
w5 = torch.randn(3, 288, generator=g) * 0.1
b5 = torch.randn(3, generator=g) * 0.1
ref = gather(h.double(), sp0) @ w5.double().T + b5.double()
o = torch.empty(4, sp0.shape[0], 3, device="cuda")
ops.spiral_conv_fwd_x(h.cuda(), dt.spiral[0], w5.cuda(), None, b5.cuda(), 0, o)
print("Dout out3 fp32 max abs err", float((o.cpu().double() - ref).abs().max()), "max |ref|", float(ref.abs().max()))

# ---- layer-by-layer: engine (bf16 mode) vs the bf16-emulating oracle, C2 step 0
from craniofacialsd_vae_amd import engine as E  # noqa: E402
import torch.nn.functional as F  # noqa: E402
w = recipe.golden_weights()
eng = E.SDVAEEngine(dt, E.ModelSpec(), device="cuda", precision="bf16")
eng.load_state_dict({k: torch.from_numpy(v) for k, v in w.items()})
P = O.make_params(w)
meshes = recipe.normalized_meshes(4)
key, eps = recipe.train_key_index(0), torch.from_numpy(recipe.train_eps(0))
x16 = torch.from_numpy(O.swap_features(meshes, ot.region_features, key))
b = eng.set_batch(x16.cuda(), key_index=key, eps=eps.cuda())
eng.forward(b, train=True)
torch.cuda.synchronize()
q = O._q
with torch.no_grad():
    h = x16
    ref_enc = []
    for i in range(4):
        low = i in (0, 1) and h.shape[-1] >= 16
        h = O.elu(O.spiral_conv(h, ot.spirals[i], O._w(P, f"en_layers.{i}.conv.layer.weight", low),
                                P[f"en_layers.{i}.conv.layer.bias"]))
        h = O.pool(h, ot.down[i])
        if i + 1 in (0, 1) and i + 1 < 4:
            h = q(h)
        ref_enc.append(h)
    for i in range(4):
        d = (b.enc_out[i].float().cpu() - ref_enc[i]).abs()
        print(f"enc_out[{i}] max abs {float(d.max()):.3e} mean {float(d.mean()):.3e} max|ref| {float(ref_enc[i].abs().max()):.3f}")
    rec, z, mu, lv = O.forward(P, x16, ot, eps=eps, lp={0, 1})
    print("mu max abs", float((b.mulv[:, 75:].cpu() - mu).abs().max()), "logvar", float((b.mulv[:, :75].cpu() - lv).abs().max()),
          "z", float((b.z.cpu() - z).abs().max()))
    hh = F.linear(b.z.cpu(), P["de_layers.0.weight"], P["de_layers.0.bias"]).view(-1, 67, 64)
    print("h max abs", float((b.h.cpu() - hh).abs().max()))
    for i in range(1, 5):
        lv_ = 4 - i
        hu = O.pool(hh, ot.up[lv_])
        if lv_ in (0, 1):
            hu = q(hu)
        du = (b.dec_up[i - 1].float().cpu() - hu).abs()
        hh = O.elu(O.spiral_conv(hu, ot.spirals[lv_], O._w(P, f"de_layers.{i}.conv.layer.weight", lv_ in (0, 1)),
                                 P[f"de_layers.{i}.conv.layer.bias"]))
        if lv_ in (0, 1):
            hh = q(hh)
        do = (b.dec_out[i - 1].float().cpu() - hh).abs()
        print(f"dec[{i - 1}] level {lv_}: up max {float(du.max()):.3e} out max {float(do.max()):.3e} mean {float(do.mean()):.3e} max|ref| {float(hh.abs().max()):.3f}")
        # feed the ENGINE's tensor forward to isolate per-layer error
        hh = b.dec_out[i - 1].float().cpu()
    out = O.spiral_conv(hh, ot.spirals[0], P["de_layers.5.layer.weight"], P["de_layers.5.layer.bias"])
    print("out (from engine dec_out[3]) max abs", float((b.out.cpu() - out).abs().max()))
    print("out vs emulation end-to-end: max per-vertex L1", float((b.out.cpu() - rec).abs().sum(-1).max()))
