"""Device health of the training step (VERDICT r3 "close the hang"; ADVICE r3 "make a scan give-up visible"):
* the look-back scan's bounded wait really gives up and counts it (neus_debug_scan_giveup: the first tile never runs);
* a raised health bit (march t precondition, scan give-up) makes Testbed::train fail with an error instead of training
  on corrupted sampling / compaction bases (neus_debug_inject_health);
* the stale-LDS corruption of round 3 (k_march_write slots past n_kept): with every CU's LDS filled with garbage (a
  negative-t pattern) before the write kernel, the progressive round-0 list, the numsteps and the coordinates equal the
  oracle's march (the cap is hit: n_kept < requested), and a progressive training run equals the one-pass run bitwise."""
import ctypes as C
import os

import numpy as np
import pytest

from gpu_util import dev, host, ptr

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BATCH = 4096
GARBAGE = 0xBF800000  # -1.0f: a stale LDS t would be negative (step_until's guarded precondition)


def _lib():
    from neus2_amd._lib import check, lib
    return lib(), check


def _testbed(sc, batch=BATCH):
    from neus2_amd import pyngp
    tb = pyngp.Testbed(pyngp.TestbedMode.Nerf)
    tb.set_dataset(sc["images"], sc["focal"], sc["principal"], sc["xforms"], 1)
    tb.reload_network_from_file(os.path.join(ROOT, "configs", "nerf", "base.json"), batch_size=batch)
    return tb


@pytest.fixture(scope="module")
def scene(torch_cuda):
    from neus2_amd import scenes
    return scenes.small_scene(n_views=8, width=64, height=48)


def test_scan_giveup_is_counted(torch_cuda):
    t = torch_cuda
    lib, check = _lib()
    n = 3 * 4096 + 5
    x = np.ones(n, np.uint32)
    out = t.zeros(n, dtype=t.int32, device="cuda")
    fails = C.c_uint32()
    check(lib.neus_debug_scan_giveup(None, ptr(dev(t, x)), ptr(out), C.c_uint32(n), C.byref(fails)))
    assert fails.value > 0
    got = host(out, np.uint32)
    # a tile that gave up takes a prefix of 0 from the missing tile: the scan is wrong, which is why it must be reported
    assert not np.array_equal(got[4096:], np.arange(4096, n, dtype=np.uint32))


@pytest.mark.parametrize("flag,word", [(1, "non-finite or negative t"), (2, "look-back scan gave up")])
def test_health_bit_fails_training(scene, flag, word):
    from neus2_amd._lib import NeusError
    lib, check = _lib()
    tb = _testbed(scene)
    tb.train_steps(17)  # the step-16 readback is pending (clean)
    assert tb.stats()["health_flags"] == 0
    check(lib.neus_debug_inject_health(tb.handle, C.c_uint32(flag)))
    assert tb.stats()["health_flags"] & flag
    # step 32 reads back step 16 (clean), step 48 reads back step 32 (after the injection): the train call fails there
    with pytest.raises(NeusError, match=word):
        tb.train_steps(40)
    assert tb.training_step < 17 + 40


def test_round0_list_with_stale_lds_matches_oracle(scene, torch_cuda):
    """The training step's progressive sampling (march + scan + write with the round-0 list) on a trained state, the
    cap hit, garbage in every CU's LDS before the write kernel: numsteps, coordinates and the round-0 list equal the
    oracle's march (the list = the first min(n, e1) sample slots of every kept ray, in ray order)."""
    import oracle as O
    t = torch_cuda
    lib, check = _lib()
    tb = _testbed(scene)
    tb.train_steps(40)
    st = tb.stats()
    rs, ri = tb.get_rng()[:2]
    _, bf = tb.get_density_grid()
    ds = O.Dataset(scene["images"], scene["focal"], scene["principal"], scene["xforms"])
    n_rays = 4096
    for max_s, e1 in ((30000, 32), (4096 * 16, 8)):
        rays = t.zeros((n_rays, 6), dtype=t.float32, device="cuda")
        ns = t.zeros((n_rays, 2), dtype=t.int32, device="cuda")
        co = t.zeros((max_s, 7), dtype=t.float32, device="cuda")
        lst = t.full((max_s,), -1, dtype=t.int32, device="cuda")
        cnt = (C.c_uint32 * 3)()
        ll = C.c_uint32()
        check(lib.neus_debug_sample_rays_round0(tb.handle, None, C.c_uint32(n_rays), C.c_uint32(st["n_rays_total"]), C.c_uint64(rs),
                                                C.c_uint64(ri), C.c_uint32(max_s), ptr(dev(t, bf)), ptr(rays), ptr(ns), ptr(co), cnt,
                                                C.c_uint32(e1), ptr(lst), C.byref(ll), C.c_uint32(GARBAGE)))
        r_rays, r_ns, r_co, r_cnt, r_nr = O.generate_samples(ds, bf, n_rays, st["n_rays_total"], rs, ri, max_s)
        np.testing.assert_array_equal(host(ns, np.uint32), r_ns)
        nk = int(cnt[1])
        assert nk == int(r_ns[:, 0].sum()) and cnt[0] == r_cnt
        if max_s == 30000:
            assert r_cnt > nk, "the cap was not hit: the test does not exercise the slots past n_kept"
        np.testing.assert_array_equal(host(co, np.uint32)[:nk], r_co.view(np.uint32)[:nk])
        expect = np.concatenate([np.arange(b, b + min(n, e1), dtype=np.uint32) for n, b in r_ns if n > 0])
        assert ll.value == expect.size
        np.testing.assert_array_equal(host(lst, np.uint32)[: ll.value], expect)


def test_progressive_training_with_stale_lds_bit_identical(scene):
    """Forced-progressive and one-pass training (same init) with every step's march write preceded by an LDS garbage
    fill: per-ray counts every step, then parameters and the occupancy grid bitwise equal; the cap was hit."""
    lib, check = _lib()
    tbs = []
    for mode in (2, 0):
        tb = _testbed(scene)
        tb.set_progressive_inference(mode, (32, 64, 96))
        check(lib.neus_debug_set_lds_fill(tb.handle, C.c_uint32(GARBAGE)))
        tbs.append(tb)
    a, b = tbs
    capped = 0
    for _ in range(24):
        a.train_steps(1)
        b.train_steps(1)
        na, ca, sa = a.ray_counts(1 << 18)
        nb, cb, sb = b.ray_counts(1 << 18)
        np.testing.assert_array_equal(sa, sb)
        np.testing.assert_array_equal(ca, cb)
        s = b.stats()
        capped += s["measured_batch_size_before_compaction"] > s["evaluated_samples_last"]
    assert capped > 0
    assert a.stats()["progressive_steps"] == 24 and b.stats()["progressive_steps"] == 0
    np.testing.assert_array_equal(a.get_params().view(np.uint32), b.get_params().view(np.uint32))
    np.testing.assert_array_equal(a.get_density_grid()[0].view(np.uint32), b.get_density_grid()[0].view(np.uint32))
    assert a.stats()["health_flags"] == 0 and b.stats()["health_flags"] == 0
