"""build()'s counted-load hazard check.

``gload*_async`` (csrc/cfsd_common.h) issues a gather in inline asm, hidden
from hipcc's waitcnt tracking, and ``vm_wait*`` retires it by count.  A read
of the destination scheduled before that wait uses stale data with no error
(round 5's 6.8e33 gradients).  ``__graft_entry__.check_async_isa`` compiles
every kernel to gfx950 ISA and fails the build on such a read; here a planted
hazard must fail it and the same kernel with the wait in place must pass.
The gather these loads implement is the spiral ``index_select`` of
``model.py:34``.  CPU only (hipcc cross-compiles).
"""
import os
import shutil

import pytest

import __graft_entry__ as G

PLANTED = r'''
#include "cfsd_common.h"
using namespace cfsd;
__global__ void gather_kernel(const float* __restrict__ x, const int* __restrict__ idx, float* __restrict__ y) {
  f32x4 a, b, c, d;
  const int r = idx[threadIdx.x];
  gload4_async(a, x + 16L * r);
  gload4_async(b, x + 16L * r + 4);
  gload4_async(c, x + 16L * r + 8);
  gload4_async(d, x + 16L * r + 12);
  %s
  vm_wait4<0>(a, b, c, d);
  st4(y + 16 * threadIdx.x, a + b + c + d);
}
'''


@pytest.mark.skipif(not os.path.exists(G.HIPCC), reason="hipcc not installed")
@pytest.mark.parametrize("planted", [False, True])
def test_check_async_catches_planted_hazard(tmp_path, planted):
    # the planted read: a's first element stored BEFORE vm_wait4 retires it
    src = tmp_path / "planted.hip"
    src.write_text(PLANTED % ("y[16 * blockDim.x + threadIdx.x] = a.x;" if planted else ""))
    work = tmp_path / "asm"
    if planted:
        with pytest.raises(RuntimeError, match="potential hazard"):
            G.check_async_isa([str(src)], str(work), include=G.CSRC)
        assert not (work / "planted.ok").exists()
    else:
        res = G.check_async_isa([str(src)], str(work), include=G.CSRC)
        assert res[0][1] == 0 and (work / "planted.ok").exists()
        assert G.check_async_isa([str(src)], str(work), include=G.CSRC)[0][2] == "cached"
    shutil.rmtree(work, ignore_errors=True)


def test_check_async_covers_every_makefile_source():
    names = {os.path.basename(s) for s in G._sources()}
    assert {"spiral_conv.hip", "spiral_conv_coarse.hip", "spiral_conv_vm32.hip"} <= names
    assert all(os.path.exists(s) for s in G._sources())
