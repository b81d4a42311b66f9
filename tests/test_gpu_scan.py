"""The single-pass exclusive scan (scan.hip: decoupled look-back, tile = blockIdx.x (in-order dispatch), epoch-tagged state) that every
deterministic compaction of the step runs on (the march's sample bases, the progressive rounds' chunk lists, the loss
compaction, the scatter's bucket x block slots), against numpy's cumsum: exact for ragged sizes around the 4096-element
tile, look-back windows longer than one wave (> 64 tiles), counts near the u32 range, aligned and unaligned buffers,
and repeated launches on one state (the epoch re-arm); no bounded-wait give-ups."""
import ctypes as C

import numpy as np
import pytest

from gpu_util import dev, host

pytestmark = pytest.mark.gpu


def _scan(t, a, reps=1, offset=0):
    from neus2_amd._lib import check, lib
    n = a.size
    x = dev(t, np.concatenate([np.zeros(offset, np.uint32), a]))
    y = t.zeros(n + offset, dtype=t.int32, device="cuda")
    fails = C.c_uint32(0)
    stream = C.c_void_p(t.cuda.current_stream().cuda_stream)
    check(lib().neus_debug_exclusive_scan(stream, C.c_void_p(x.data_ptr() + 4 * offset), C.c_void_p(y.data_ptr() + 4 * offset), C.c_uint32(n),
                                          C.c_int(reps), C.byref(fails)))
    return host(y, np.uint32)[offset:], fails.value


@pytest.mark.parametrize("n", [1, 17, 4095, 4096, 4097, 1 << 18, (1 << 18) + 3, 64 * 4096 + 1, 1_000_003, 3_000_000])
def test_exclusive_scan_matches_cumsum(torch_cuda, n):
    rng = np.random.default_rng(n)
    a = rng.integers(0, 40, n, dtype=np.uint32)
    a[rng.random(n) < 0.3] = 0
    ref = (np.cumsum(a, dtype=np.uint64) - a).astype(np.uint32)
    got, fails = _scan(torch_cuda, a, reps=3)
    assert fails == 0
    np.testing.assert_array_equal(got, ref)


def test_exclusive_scan_unaligned_and_wrapping(torch_cuda):
    rng = np.random.default_rng(7)
    n = 300_001
    a = rng.integers(0, 1 << 16, n, dtype=np.uint32)
    a[0] = 0xFFFFFFF0  # the u32 sums wrap as the reference's u32 counters would
    ref = (np.cumsum(a, dtype=np.uint64) - a).astype(np.uint32)
    got, fails = _scan(torch_cuda, a, reps=2, offset=1)
    assert fails == 0
    np.testing.assert_array_equal(got, ref)
