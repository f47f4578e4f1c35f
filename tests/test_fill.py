"""The synthetic input generator of SURVEY §8(d) (rfec_fill_xorshift,
bench / test inputs): the host jump-ahead equals stepping the oracle's
xorshift64* (CPU), and the device fill equals the oracle's sequential fill,
also for a slice that starts mid-stream (GPU)."""
import ctypes as C

import numpy as np
import pytest

SEED = 0x52415A4F52464543


def test_jump_ahead_matches_sequential(product, oracle1000):
    s = C.c_uint64(SEED ^ 4)
    seq = []
    for _ in range(3001):
        seq.append(s.value)
        oracle1000.lib.oracle_xs_next(C.byref(s))
    for n in (0, 1, 2, 149, 150, 1500, 3000):
        assert product.lib.rfec_xorshift_jump(SEED ^ 4, n) == seq[n], n


def test_fill_rejects_bad_geometry(product):
    assert product.lib.rfec_fill_xorshift(None, 2, 0, 1, 10, 1200, 1200, None) == -1
    assert product.lib.rfec_fill_xorshift(C.c_void_p(16), 2, 0, 1, 10, 1200, 1100, None) == -1


@pytest.mark.gpu
@pytest.mark.parametrize("k,S,stride,cfg", [(10, 1200, 1200, 2), (32, 256, 256, 5), (10, 1000, 1008, 6),
                                            (3, 13, 16, 9)])
def test_device_fill_matches_oracle(product, oracle1000, k, S, stride, cfg):
    import torch

    G, g0 = 300, 1700
    ref_all, _ = oracle1000.fill_groups(cfg, g0 + G, k, S, stride=stride)
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev).cuda_stream
    for lo, n in ((0, G), (g0, G), (g0 + 7, 1)):
        buf = torch.full((n, k, stride), 0x5A, dtype=torch.uint8, device=dev)
        product.fill_xorshift(buf.data_ptr(), cfg, lo, n, k, S, stride, st)
        assert np.array_equal(buf.cpu().numpy(), ref_all[lo:lo + n]), (lo, n)
