"""The step roofline prices every launch that does required work.

bench.py's ``step_roofline`` divides the ideal time of each launch of one
eager train step (max(flop / peak, algorithmic bytes / HBM), from its ABI
arguments by ``bench.launch_cost``) by the measured time.  A launch kind the
pricing does not know would be counted as zero required work, so this test
traces one eager step (fp32 and bf16) and requires every launch to be priced
or to be one of the named bookkeeping launches (``bench.BOOKKEEPING``).
Reference work being priced: model.py:27-55 (convs, Pool), 146-188
(Linears, latent head), model_manager.py:282-316 (losses, Adam).
"""
import os
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_every_work_launch_is_priced(precision):
    import bench
    from craniofacialsd_vae_amd import _abi
    dev = torch.device("cuda", 0)
    r = bench.Runner(1, 0, dev, 16, False, "craniofacial", precision)
    r.eager_step()
    torch.cuda.synchronize()
    with _abi.trace_launches() as rec:
        r.eager_step()
    torch.cuda.synchronize()
    flop = byte = 0.0
    unpriced = []
    for name, args, _, _ in rec:
        fl, by, _ = bench.launch_cost(name, args)
        flop += fl
        byte += by
        if fl == 0 and by == 0 and name not in bench.BOOKKEEPING:
            unpriced.append(name)
    assert not unpriced, f"launches priced at zero that do required work: {sorted(set(unpriced))}"
    # fp32 step: 3 x (conv flops of every layer) - E0's dx, Enblock row subsets
    # applied, + the Linears: 24.6-24.8 GFLOP (1.826 GFLOP/mesh
    # counts full-resolution Enblocks)
    assert 24.0e9 < flop < 25.5e9, flop
    assert byte > 4.0e8, byte
    sr = bench.step_roofline(r, 1.0)
    assert sr["unpriced_work_launches"] == []
    assert abs(sr["required_gflop_per_step"] - flop / 1e9) < 1e-6
