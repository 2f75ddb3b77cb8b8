"""MI355X-native spiral-convolution mesh-VAE training path (CraniofacialSD-VAE).

Kernels: ``libcfsd.so`` (HIP, gfx950) behind the C ABI of ``include/cfsd.h``.
Host: this package (PyTorch-ROCm for device memory, streams and
``torch.distributed``).  Import through ``cfsd_loader.load()`` (the directory
name contains a hyphen).
"""
from . import _abi  # noqa: F401

__version__ = "0.1.0"
