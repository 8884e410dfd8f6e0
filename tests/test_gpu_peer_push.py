"""k_peer_push (csrc/kernels/copy_kernels.hip) numerics on one MI355X: the
source-GPU push kernel of the xGMI peer plane, run with both pointers in local
HBM (a one-GPU box has no peer); unaligned tails take the generic path. The
destination must equal the source byte for byte."""
from __future__ import annotations

import pytest
import torch

from ogkm._native import lib

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("nbytes", [4096, 3 * (1 << 20) + 4096, 64 << 20, (1 << 20) + 12])
def test_peer_push_local_numerics(gpu_rt, nbytes):
    src = torch.randint(0, 256, (nbytes,), dtype=torch.uint8, device="cuda")
    dst = torch.zeros(nbytes + 64, dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream()
    lib.peer_push(0, s.cuda_stream, dst.data_ptr(), src.data_ptr(), nbytes)
    torch.cuda.synchronize()
    assert torch.equal(dst[:nbytes], src)
    assert int(dst[nbytes:].max()) == 0          # nothing written past the end


def test_peer_engine_masks_reported(gpu_rt):
    """Host-direction SDMA masks are non-empty on the box; a single GPU has no
    peer pairs (mask 0)."""
    assert lib.copy_engine_mask(0, -1) != 0 and lib.copy_engine_mask(-1, 0) != 0
    assert lib.copy_engine_mask(0, 0) == 0
