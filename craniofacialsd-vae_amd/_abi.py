"""ctypes binding of ``libcfsd.so`` (the C ABI declared in ``include/cfsd.h``).

The library is built in-tree (``csrc/Makefile``, ``__graft_entry__.build()``)
and this module refuses to run without it: there is no CPU or PyTorch
fallback for any kernel.
"""
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("CFSD_LIB_PATH") or os.path.join(_HERE, "libcfsd.so")

_lib = None

_P = ctypes.c_void_p
_I = ctypes.c_int
_F = ctypes.c_float
_Z = ctypes.c_size_t
_U64 = ctypes.c_ulonglong

# name -> (restype, argtypes); must match include/cfsd.h exactly.
SIGNATURES = {
    "cfsd_version": (_I, []),
    "cfsd_last_error_string": (ctypes.c_char_p, []),
    "cfsd_spiral_conv_workspace": (_Z, [_I, _I, _I, _I, _I, _I]),
    "cfsd_spiral_conv_fwd": (_I, [_P, _P, _P, _P, _P, _P, _Z, _I, _I, _I, _I, _I, _I, _I, _P]),
    "cfsd_spiral_conv_bwd_data": (_I, [_P, _P, _P, _P, _P, _P, _P, _P, _Z, _I, _I, _I, _I, _I, _I,
                                       _P]),
    "cfsd_spiral_conv_bwd_weight": (_I, [_P, _P, _P, _P, _P, _P, _Z, _I, _I, _I, _I, _I, _I, _P]),
    "cfsd_spiral_conv_bwd_weight_workspace": (_Z, [_I, _I, _I, _I, _I]),
    "cfsd_spiral_conv_bwd": (_I, [_P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _Z, _I, _I, _I,
                                  _I, _I, _I, _P]),
    "cfsd_spiral_conv_bwd_workspace": (_Z, [_I, _I, _I, _I, _I, _I]),
    "cfsd_spiral_conv_bwd_paired": (_I, [_I, _I, _I, _I, _I, _I]),
    "cfsd_spiral_conv_bwd_rowsub": (_I, [_P, _P, _P, _P, _I, _P, _P, _P, _P, _P, _P, _Z, _I, _I, _I,
                                         _I, _I, _I, _P]),
    "cfsd_spiral_conv_bwd_rowsub_x": (_I, [_P, _I, _P, _P, _P, _I, _P, _P, _P, _P, _P, _P, _Z, _I, _I, _I,
                                           _I, _I, _I, _P]),
    "cfsd_spiral_conv_bwd_rowsub_workspace": (_Z, [_I, _I, _I, _I, _I, _I]),
    "cfsd_spiral_conv_bwd_flat_pair": (_I, [_P, _P, _P, _P, _I, _P, _P, _P, _P, _P, _P, _Z, _I, _I, _I, _I,
                                            _I, _I, _P]),
    "cfsd_spiral_conv_bwd_flat_pair_workspace": (_Z, [_I, _I, _I, _I, _I]),
    "cfsd_spiral_conv_bwd_flat_pair_bf16": (_I, [_P, _P, _P, _P, _I, _P, _P, _P, _P, _Z, _I, _I, _I, _I, _I, _I,
                                                 _P]),
    "cfsd_spiral_conv_bwd_rowsub_pair_bf16": (_I, [_P, _P, _P, _P, _I, _P, _P, _P, _P, _Z, _I, _I, _I, _I, _I,
                                                   _I, _P]),
    "cfsd_spiral_conv_bwd_data_rowsub": (_I, [_P, _P, _I, _P, _P, _P, _I, _P, _Z, _I, _I, _I, _I, _I, _I,
                                              _P]),
    "cfsd_spiral_conv_bwd_data_rowsub_workspace": (_Z, [_I, _I, _I, _I]),
    "cfsd_linear_bwd_split_parts": (_I, [_I]),
    "cfsd_bottleneck_bwd_exchange_floats": (_Z, [_I, _I, _I, _I]),
    "cfsd_linear_bwd_split": (_I, [_P, _P, _P, _P, _P, _P, _I, _I, _I, _P]),
    "cfsd_latent_bwd_parts": (_I, [_P, _P, _P, _P, _I, _P, _P, _I, _I, _I, _I, _I, _P]),
    "cfsd_spiral_gather": (_I, [_P, _P, _P, _I, _I, _I, _I, _I, _P]),
    "cfsd_spmm_csr_sched": (_I, [_P, _P, _P, _P, _P, _I, _P, _P, _I, _I, _I, _I, _I, _P]),
    "cfsd_spmm_csr": (_I, [_P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _P]),
    "cfsd_swap_features": (_I, [_P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _P]),
    "cfsd_swap_features_x": (_I, [_P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _P]),
    "cfsd_spiral_conv_fwd_up_supported": (_I, [_I, _I, _I, _I, _I]),
    "cfsd_spiral_conv_fwd_up": (_I, [_P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _P]),
    "cfsd_gather_meshes": (_I, [_P, _P, _P, _I, _I, _I, _I, _I, _P]),
    "cfsd_normalize": (_I, [_P, _P, _P, _P, _I, _I, _I, _P]),
    "cfsd_spectral_blend": (_I, [_P, _P, _P, _P, _I, _I, _I, _I, _P]),
    "cfsd_linear_workspace": (_Z, [_I, _I, _I]),
    "cfsd_linear_fwd": (_I, [_P, _P, _P, _P, _P, _Z, _I, _I, _I, _P]),
    "cfsd_linear_bwd": (_I, [_P, _P, _P, _P, _P, _P, _P, _P, _Z, _I, _I, _I, _I, _P]),
    "cfsd_recon_lap_blocks": (_I, [_I, _I]),
    "cfsd_recon_lap_fwd": (_I, [_P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _P]),
    "cfsd_recon_lap_bwd": (_I, [_P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _F, _F, _P]),
    "cfsd_recon_lap_bwd_finalize": (_I, [_P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _F, _F, _P, _I, _P, _P,
                                         _P, _F, _F, _P]),
    "cfsd_recon_lap_fwd_x": (_I, [_P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _P]),
    "cfsd_recon_lap_bwd_x": (_I, [_P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _F, _F, _I, _P]),
    "cfsd_recon_lap_bwd_finalize_x": (_I, [_P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _F, _F, _P, _I, _P, _P,
                                           _P, _F, _F, _I, _P]),
    "cfsd_latent_fwd": (_I, [_P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _F, _F, _F, _F, _P]),
    "cfsd_latent_linear_fwd_supported": (_I, [_I, _I, _I]),
    "cfsd_latent_linear_fwd": (_I, [_P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _F, _F, _F, _F,
                                    _P, _P, _P, _I, _P]),
    "cfsd_latent_bwd": (_I, [_P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _P]),
    "cfsd_loss_finalize": (_I, [_P, _I, _P, _P, _P, _I, _I, _I, _F, _F, _F, _P]),
    "cfsd_adam": (_I, [_P, _P, _P, _P, _P, _Z, _F, _F, _F, _F, _F, _P, _P]),
    "cfsd_adam_scaled": (_I, [_P, _P, _P, _P, _P, _Z, _F, _F, _F, _F, _F, _F, _P, _P]),
    "cfsd_spiral_conv_fwd_in_swap": (_I, [_P, _P, _P, _P, _I, _I, _I, _P, _I, _P, _P, _P, _P, _I, _I, _I, _I, _I,
                                          _I, _P]),
    "cfsd_bottleneck_bwd": (_I, [_P, _P, _P, _P, _I, _I, _P, _P, _P, _P, _P, _I, _P, _P, _P, _P, _I, _I, _I,
                                 _P, _P, _P, _P, _P, _P, _I, _I, _I, _P, _I, _I, _P]),
    "cfsd_spiral_conv_fwd_x": (_I, [_P, _I, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _P]),
    "cfsd_spiral_conv_bwd_data_x": (_I, [_P, _I, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _P]),
    "cfsd_spiral_conv_bwd_data_flat": (_I, [_P, _I, _P, _I, _P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _P]),
    "cfsd_spiral_conv_bwd_weight_x_workspace": (_Z, [_I, _I, _I, _I, _I]),
    "cfsd_spiral_conv_bwd_weight_x": (_I, [_P, _I, _P, _P, _I, _P, _P, _P, _Z, _I, _I, _I, _I, _I, _I, _P]),
    "cfsd_spiral_conv_bwd_x": (_I, [_P, _I, _P, _P, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _Z, _I, _I, _I,
                                    _I, _I, _I, _P]),
    "cfsd_spiral_conv_bwd_out_flat": (_I, [_P, _I, _P, _P, _I, _P, _I, _P, _P, _P, _P, _P, _P, _Z, _I, _I, _I,
                                           _I, _I, _I, _P]),
    "cfsd_spmm_csr_x": (_I, [_P, _P, _P, _P, _I, _P, _P, _I, _I, _I, _I, _I, _P]),
    "cfsd_spmm_uniform": (_I, [_I, _P, _P, _P, _I, _P, _P, _I, _I, _I, _I, _I, _P]),
    "cfsd_spmm_sched_csr": (_I, [_P, _P, _P, _P, _P, _I, _P, _P, _I, _I, _I, _I, _I, _P]),
    "cfsd_cast": (_I, [_P, _I, _P, _I, _Z, _P]),
    "cfsd_step_begin": (_I, [_P, _U64, _P, _I, _P, _I, _P, _I, _I, _P, _I, _I, _P, _P]),
    "cfsd_dw_reduce_batch": (_I, [_P, _I, _P]),
    "cfsd_dw_reduce_batch_adam": (_I, [_P, _I, _P, _P, _P, _P, _P, _Z, _F, _F, _F, _F, _F, _P, _P]),
    "cfsd_scale": (_I, [_P, _Z, _F, _P]),
    "cfsd_elu_bwd": (_I, [_P, _P, _P, _Z, _P]),
    "cfsd_vertex_errors": (_I, [_P, _P, _P, _P, _P, _P, _P, _I, _I, _F, _P]),
}


class DwSlabs(ctypes.Structure):
    """``cfsd_dw_slabs`` (include/cfsd.h): one deferred weight-gradient slab set."""
    _fields_ = [("workspace", _P), ("dw", _P), ("db", _P), ("batch", _I), ("vsrc", _I),
                ("rows", _I), ("cin", _I), ("cout", _I), ("fused", _I)]


class CfsdError(RuntimeError):
    pass


def load(path=LIB_PATH):
    """Load libcfsd.so (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise CfsdError(
            f"{path} not found: build the HIP extension first "
            "(python -c 'import __graft_entry__ as g; g.build()' or make -C csrc)")
    lib = ctypes.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def lib():
    return _lib if _lib is not None else load()


def check(rc, what=""):
    if rc != 0:
        msg = lib().cfsd_last_error_string().decode(errors="replace")
        raise CfsdError(f"{what or 'cfsd'} failed (rc={rc}): {msg}")


def ptr(t):
    """Device pointer of a CUDA(HIP) tensor, or None."""
    if t is None:
        return None
    if not t.is_cuda:
        raise CfsdError("cfsd kernels take device tensors only")
    return ctypes.c_void_p(t.data_ptr())


def stream_ptr(stream=None):
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


_trace = None  # list of (name, args, start_event, end_event) while tracing


class trace_launches:
    """Context manager recording every libcfsd launch with a HIP event pair on
    the launch stream (per-kernel device time of an eager step; measurement
    only -- the product path never enables it)."""

    def __enter__(self):
        global _trace
        self.records = []
        _trace = self.records
        return self.records

    def __exit__(self, *exc):
        global _trace
        _trace = None
        return False


def call(name, *args):
    if _trace is None:
        check(getattr(lib(), name)(*args), name)
        return
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    check(getattr(lib(), name)(*args), name)
    e1.record()
    _trace.append((name, args, e0, e1))
