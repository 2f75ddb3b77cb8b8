"""Drop-in replacement for the reference ``model.py`` module API.

Same class names, constructor signatures, attributes, ``__repr__`` and
``state_dict`` keys as the reference (``model.py:11-188``):

* ``SpiralConv(in_channels, out_channels, indices, dim=1)``
* ``Pool(x, trans, dim=1)``
* ``SpiralEnblock(in_channels, out_channels, indices).forward(x, down_transform)``
* ``SpiralDeblock(in_channels, out_channels, indices).forward(x, up_transform)``
* ``Model(in_channels, out_channels, latent_size, spiral_indices,
  down_transform, up_transform, pre_z_sigmoid=False, is_vae=False)``

The arithmetic runs in libcfsd (HIP, gfx950) through ``torch.autograd.Function``
wrappers; index tables are converted once per (tensor, device) and cached.
There is no CPU path: these modules require device tensors.  For training
throughput use :class:`craniofacialsd_vae_amd.engine.SDVAEEngine` (flat
parameters, hipGraph-captured step); both produce the same numbers.
"""
import weakref

import numpy as np
import torch
import torch.nn as nn

from . import ops, topology
from .ops import ACT_ELU, ACT_NONE

# ------------------------------------------------------------------ plan caches
_SPIRAL_PLANS = {}
_POOL_PLANS = {}


def _cache_get(cache, key_obj, device, build):
    key = (id(key_obj), str(device))
    hit = cache.get(key)
    if hit is not None and hit[0]() is key_obj:
        return hit[1]
    plan = build()
    try:
        ref = weakref.ref(key_obj)
    except TypeError:  # pragma: no cover
        ref = (lambda o=key_obj: o)
    cache[key] = (ref, plan)
    return plan


class _SpiralPlan:
    def __init__(self, idx_np, vsrc, device):
        self.rows, self.seq = idx_np.shape
        self.vsrc = vsrc
        self.idx = torch.from_numpy(topology._i32(idx_np)).to(device)
        self.inv = tuple(torch.from_numpy(a).to(device) for a in topology.inverse_spiral(idx_np, vsrc))


def spiral_plan(indices, device, vsrc=None, rows=None):
    """Device tables for a spiral index tensor (optionally a row subset)."""
    def build():
        idx = indices.detach().cpu().numpy().astype(np.int64)
        sub = idx if rows is None else idx[rows]
        return _SpiralPlan(sub, vsrc or idx.shape[0], device)
    if rows is None:
        return _cache_get(_SPIRAL_PLANS, indices, device, build)
    key_holder = _selection_plan_holder(indices, rows)
    return _cache_get(_SPIRAL_PLANS, key_holder, device, build)


class _Holder:
    pass


_SEL_HOLDERS = {}


def _selection_plan_holder(indices, rows):
    key = (id(indices), rows.tobytes())
    h = _SEL_HOLDERS.get(key)
    if h is None:
        h = _SEL_HOLDERS[key] = _Holder()
    return h


class _PoolPlan:
    def __init__(self, trans, device):
        t = trans.detach().cpu()
        if not t.is_sparse:
            raise TypeError("Pool expects a torch sparse COO transform (as in transforms.pkl)")
        idx = t._indices().numpy()
        val = t._values().numpy()
        self.m, self.n = int(t.shape[0]), int(t.shape[1])
        csr = topology.csr_from_coo(idx[0], idx[1], val, self.m)
        self.uniform = topology.uniform_rows(csr[0])
        self.csr = tuple(torch.from_numpy(a).to(device) for a in csr)
        self.csrT = tuple(torch.from_numpy(a).to(device)
                          for a in topology.csr_transpose_from_coo(idx[0], idx[1], val, self.n))
        self.selection = topology.selection_rows(idx[0], idx[1], val, self.m)


def pool_plan(trans, device):
    return _cache_get(_POOL_PLANS, trans, device, lambda: _PoolPlan(trans, device))


# ------------------------------------------------------------------ autograd ops
class _SpiralConvFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, plan, act):
        x = x.contiguous()
        w = weight.contiguous()
        y = ops.spiral_conv_fwd(x, plan.idx, w, bias.contiguous() if bias is not None else None, act)
        ctx.plan, ctx.act = plan, act
        ctx.save_for_backward(x, w, y)
        ctx.has_bias = bias is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, y = ctx.saved_tensors
        plan = ctx.plan
        dy = dy.contiguous()
        dpre = ops.elu_bwd(dy, y) if ctx.act == ACT_ELU else dy
        dx = dw = db = None
        need_w = ctx.needs_input_grad[1] or (ctx.has_bias and ctx.needs_input_grad[2])
        if need_w:  # fused dX + dW/db (cfsd_spiral_conv_bwd)
            dw = torch.empty_like(w)
            db = torch.empty(w.shape[0], dtype=w.dtype, device=w.device)
            dx = torch.empty_like(x) if ctx.needs_input_grad[0] else None
            ops.spiral_conv_bwd(x, plan.idx, dpre, plan.inv, w, dw, db, dx=dx)
        elif ctx.needs_input_grad[0]:
            dx = ops.spiral_conv_bwd_data(dpre, plan.inv, w, x.shape[1])
        return dx, dw, (db if ctx.has_bias else None), None, None


class _PoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, plan):
        ctx.plan = plan
        return ops.spmm(plan.csr, x.contiguous(), plan.m, uniform=plan.uniform)

    @staticmethod
    def backward(ctx, dy):
        return ops.spmm(ctx.plan.csrT, dy.contiguous(), ctx.plan.n), None


class _LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias):
        x2 = x.reshape(-1, x.shape[-1]).contiguous()
        y = ops.linear_fwd(x2, weight.contiguous(), bias.contiguous() if bias is not None else None)
        ctx.save_for_backward(x2, weight)
        ctx.in_shape = x.shape
        ctx.has_bias = bias is not None
        return y.view(*x.shape[:-1], weight.shape[0])

    @staticmethod
    def backward(ctx, dy):
        x2, w = ctx.saved_tensors
        dy2 = dy.reshape(-1, w.shape[0]).contiguous()
        dx = torch.empty_like(x2) if ctx.needs_input_grad[0] else None
        dw = torch.empty_like(w) if ctx.needs_input_grad[1] else None
        db = torch.empty(w.shape[0], device=w.device) if ctx.has_bias and ctx.needs_input_grad[2] else None
        ops.linear_bwd(x2, w.contiguous(), dy2, dx=dx, dw=dw, db=db)
        return (dx.view(ctx.in_shape) if dx is not None else None), dw, db


def _as_batched(x):
    if x.dim() == 2:
        return x.unsqueeze(0), True
    if x.dim() == 3:
        return x, False
    raise RuntimeError(f"x.dim() is expected to be 2 or 3, but received {x.dim()}")


def _check_device(x):
    if not x.is_cuda:
        raise RuntimeError("craniofacialsd_vae_amd runs on the GPU only (libcfsd); got a CPU tensor")


# ------------------------------------------------------------------ modules
class SpiralConv(nn.Module):
    """``SpiralConv`` (reference ``model.py:11-47``)."""

    def __init__(self, in_channels, out_channels, indices, dim=1):
        super().__init__()
        self.dim = dim
        self.indices = indices
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.seq_length = indices.size(1)
        self.layer = nn.Linear(in_channels * self.seq_length, out_channels)
        self.reset_parameters()

    def reset_parameters(self):
        torch.nn.init.xavier_uniform_(self.layer.weight)
        torch.nn.init.constant_(self.layer.bias, 0)

    def _conv(self, x, act, rows=None, vsrc=None):
        xb, squeeze = _as_batched(x)
        _check_device(xb)
        if self.dim != 1 and not squeeze:
            raise RuntimeError("only dim=1 (vertex dimension) is supported, as in the reference")
        plan = spiral_plan(self.indices, xb.device, vsrc=xb.shape[1] if rows is not None else None,
                           rows=rows)
        if plan.vsrc != xb.shape[1]:
            raise RuntimeError(f"input has {xb.shape[1]} vertices, spiral indexes {plan.vsrc}")
        y = _SpiralConvFn.apply(xb, self.layer.weight, self.layer.bias, plan, act)
        return y.squeeze(0) if squeeze else y

    def forward(self, x):
        return self._conv(x, ACT_NONE)

    def __repr__(self):
        return '{}({}, {}, seq_length={})'.format(self.__class__.__name__, self.in_channels,
                                                  self.out_channels, self.seq_length)


def Pool(x, trans, dim=1):
    """``Pool`` (reference ``model.py:50-55``): sparse down/up-sample."""
    if dim != 1:
        raise RuntimeError("only dim=1 (vertex dimension) is supported, as in the reference")
    xb, squeeze = _as_batched(x)
    _check_device(xb)
    plan = pool_plan(trans, xb.device)
    y = _PoolFn.apply(xb, plan)
    return y.squeeze(0) if squeeze else y


class SpiralEnblock(nn.Module):
    """``SpiralEnblock`` (reference ``model.py:58-70``): conv -> ELU -> Pool(down).
    A 0/1 selection ``down_transform`` folds into evaluating the conv at the
    kept vertices only (bit-identical, 4x less work)."""

    def __init__(self, in_channels, out_channels, indices):
        super().__init__()
        self.conv = SpiralConv(in_channels, out_channels, indices)
        self.reset_parameters()

    def reset_parameters(self):
        self.conv.reset_parameters()

    def forward(self, x, down_transform):
        xb, squeeze = _as_batched(x)
        _check_device(xb)
        plan = pool_plan(down_transform, xb.device)
        if plan.selection is not None:
            out = self.conv._conv(xb, ACT_ELU, rows=plan.selection, vsrc=xb.shape[1])
        else:
            out = Pool(self.conv._conv(xb, ACT_ELU), down_transform)
        return out.squeeze(0) if squeeze else out


class SpiralDeblock(nn.Module):
    """``SpiralDeblock`` (reference ``model.py:73-85``): Pool(up) -> conv -> ELU."""

    def __init__(self, in_channels, out_channels, indices):
        super().__init__()
        self.conv = SpiralConv(in_channels, out_channels, indices)
        self.reset_parameters()

    def reset_parameters(self):
        self.conv.reset_parameters()

    def forward(self, x, up_transform):
        out = Pool(x, up_transform)
        return self.conv._conv(out, ACT_ELU)


class _Linear(nn.Linear):
    """``nn.Linear`` whose arithmetic runs in libcfsd (same parameters/keys)."""

    def forward(self, x):
        _check_device(x)
        return _LinearFn.apply(x, self.weight, self.bias)


class Model(nn.Module):
    """``Model`` (reference ``model.py:88-188``)."""

    def __init__(self, in_channels, out_channels, latent_size, spiral_indices, down_transform,
                 up_transform, pre_z_sigmoid=False, is_vae=False):
        super().__init__()
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.latent_size = latent_size
        self.spiral_indices = spiral_indices
        self.down_transform = down_transform
        self.up_transform = up_transform
        self.num_vert = self.down_transform[-1].size(0)
        self.pre_z_sigmoid = pre_z_sigmoid
        self.is_vae = is_vae

        self.en_layers = nn.ModuleList()
        for idx in range(len(out_channels)):
            cin = in_channels if idx == 0 else out_channels[idx - 1]
            self.en_layers.append(SpiralEnblock(cin, out_channels[idx], self.spiral_indices[idx]))
        self.en_layers.append(_Linear(self.num_vert * out_channels[-1], latent_size))
        if self.is_vae:
            self.en_layers.append(_Linear(self.num_vert * out_channels[-1], latent_size))

        self.de_layers = nn.ModuleList()
        self.de_layers.append(_Linear(latent_size, self.num_vert * out_channels[-1]))
        for idx in range(len(out_channels)):
            if idx == 0:
                cin, cout = out_channels[-idx - 1], out_channels[-idx - 1]
            else:
                cin, cout = out_channels[-idx], out_channels[-idx - 1]
            self.de_layers.append(SpiralDeblock(cin, cout, self.spiral_indices[-idx - 1]))
        self.de_layers.append(SpiralConv(out_channels[0], in_channels, self.spiral_indices[0]))
        self.reset_parameters()

    def reset_parameters(self):
        for name, param in self.named_parameters():
            if 'bias' in name:
                nn.init.constant_(param, 0)
            else:
                nn.init.xavier_uniform_(param)

    def encode(self, x):
        n_linear_layers = 2 if self.is_vae else 1
        for i, layer in enumerate(self.en_layers):
            if i < len(self.en_layers) - n_linear_layers:
                x = layer(x, self.down_transform[i])
        x = x.reshape(-1, self.en_layers[-1].weight.size(1))
        mu = self.en_layers[-1](x)
        if self.is_vae:
            logvar = self.en_layers[-2](x)
        else:
            mu = torch.sigmoid(mu) if self.pre_z_sigmoid else mu
            logvar = None
        return mu, logvar

    def decode(self, x):
        num_layers = len(self.de_layers)
        num_features = num_layers - 2
        for i, layer in enumerate(self.de_layers):
            if i == 0:
                x = layer(x)
                x = x.view(-1, self.num_vert, self.out_channels[-1])
            elif i != num_layers - 1:
                x = layer(x, self.up_transform[num_features - i])
            else:
                x = layer(x)
        return x

    def forward(self, x, eps=None):
        mu, logvar = self.encode(x)
        if self.is_vae and self.training:
            z = self._reparameterize(mu, logvar, eps)
        else:
            z = mu
        out = self.decode(z)
        return out, z, mu, logvar

    @staticmethod
    def _reparameterize(mu, logvar, eps=None):
        """``model.py:184-188``; ``eps`` may be injected (parity tests)."""
        std = torch.exp(0.5 * logvar)
        if eps is None:
            eps = torch.randn_like(std)
        return mu + eps * std
