"""Per-wave phase timing of the coarse slot-group forward (s_memrealtime,
100 MHz): where the microseconds of a small conv launch go.  Debug hook
cfsd_debug_set_stamps (not part of include/cfsd.h)."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import cfsd_loader  # noqa: E402

cfsd_loader.load()
from craniofacialsd_vae_amd import _abi  # noqa: E402
import kbench  # noqa: E402

lib = _abi.lib()
lib.cfsd_debug_set_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
FLAGS = int(os.environ.get('KB_DBG', '0'))
lib.cfsd_debug_set_stamps.restype = None
buf = torch.zeros(1 << 20, dtype=torch.int64, device="cuda")
cases, _, _ = kbench.build_cases(sys.argv[1:])
for name in sys.argv[1:]:
    fn = cases[name]
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    for rep in range(2):
        buf.zero_()
        lib.cfsd_debug_set_stamps(ctypes.c_void_p(buf.data_ptr()), FLAGS)
        torch.cuda._sleep(1000000)
        fn()
        torch.cuda.synchronize()
        lib.cfsd_debug_set_stamps(None, 0)
        st = buf.view(-1, 8).cpu().numpy()
        if os.environ.get("KB_PT"):  # persistent kernel: start, first loads landed, sum mfma, sum barrier, end, tiles
            st = st[st[:, 0] != 0][:, :6].astype(np.float64)
            t0 = st[:, 0].min()
            print(f"{name} rep{rep}: waves {len(st)} span {(st[:, 4].max() - t0) / 100:.2f} us | start spread "
                  f"{(st[:, 0].max() - t0) / 100:.2f} | first loads {(st[:, 1] - st[:, 0]).mean() / 100:.2f} | tiles/wg "
                  f"{st[:, 5].mean():.2f} | per tile: mfma+lds {(st[:, 2] / st[:, 5]).mean() / 100:.2f} barrier "
                  f"{(st[:, 3] / st[:, 5]).mean() / 100:.2f} | loop total {(st[:, 4] - st[:, 1]).mean() / 100:.2f} "
                  f"-> per tile {((st[:, 4] - st[:, 1]) / st[:, 5]).mean() / 100:.2f}", flush=True)
            continue
        st = st[st[:, 0] != 0][:, :6].astype(np.float64) / 100.0  # us
        t0 = st[:, 0].min()
        st -= t0
        d = np.diff(st, axis=1)
        print(f"{name} rep{rep}: waves {len(st)} span {st[:, 5].max():.2f} us | start spread {st[:, 0].max():.2f} "
              f"(median {np.median(st[:, 0]):.2f}) | idx+issue {d[:, 0].mean():.2f} wait-loads {d[:, 1].mean():.2f} "
              f"(max {d[:, 1].max():.2f}) mfma+lds {d[:, 2].mean():.2f} barrier {d[:, 3].mean():.2f} "
              f"epilogue {d[:, 4].mean():.2f} | last wave end {st[:, 5].max():.2f} first end {st[:, 5].min():.2f}",
              flush=True)
