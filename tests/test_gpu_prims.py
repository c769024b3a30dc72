"""The library's single-pass exclusive scan (greedy.hip scan_1p: lane-contiguous 16-byte loads, a one-barrier
multi-quarter block scan, a decoupled look-back across 8192-int tiles; one workgroup with a running carry up to
64 Ki ints), called through aos_debug_scan on device arrays, vs numpy's cumsum: sizes around every tile and
path boundary, 16-byte aligned and unaligned arrays, zero_in."""
import numpy as np
import pytest

import aos_gpu

pytestmark = pytest.mark.gpu

SIZES = [0, 1, 3, 4, 5, 4095, 4096, 4097, 16383, 16384, 16385, 65535, 65536, 65537, 65538, 8191, 8192, 8193,
         3 * 8192 + 5, 517 * 8192 - 1, 2_113_541, 5_283_840]


@pytest.fixture(scope="module")
def ctx():
    c = aos_gpu.Ctx(aos_gpu.default_params())
    yield c
    c.close()


@pytest.mark.parametrize("n", SIZES)
@pytest.mark.parametrize("shift", [0, 1])
def test_scan_vs_numpy(ctx, n, shift):
    import torch
    rng = np.random.default_rng(n + 7 * shift)
    x = rng.integers(0, 50, size=n, dtype=np.int32)
    # shift = 1: both arrays start one int past a 16-byte boundary (the scalar-access form)
    buf_in = torch.zeros(n + 8, dtype=torch.int32, device="cuda")
    buf_out = torch.full((n + 9,), -1, dtype=torch.int32, device="cuda")
    buf_in[shift:shift + n] = torch.from_numpy(x)
    ctx.debug_scan(buf_in.data_ptr() + 4 * shift, buf_out.data_ptr() + 4 * shift, n, zero_in=bool(n % 2))
    out = buf_out[shift:shift + n + 1].cpu().numpy()
    want = np.zeros(n + 1, np.int64)
    want[1:] = np.cumsum(x, dtype=np.int64)
    assert np.array_equal(out.astype(np.int64), want)
    assert int(buf_out[shift + n + 1]) == -1 and (shift == 0 or int(buf_out[0]) == -1)   # nothing written outside
    rest = buf_in[shift:shift + n].cpu().numpy()
    assert np.array_equal(rest, np.zeros(n, np.int32) if n % 2 else x)
