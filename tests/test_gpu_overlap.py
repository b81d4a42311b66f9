"""Work issued beside the backward must not change a bit (round 6):
* the next step's ray sampling (the lookahead) with a data-parallel group: the step's counters are all-reduced right
  after the loss (StepState::compacted_global), so the sampling no longer waits for the whole exchange;
* the optimizer in pieces beside the grid scatter (NEUS_ADAM_OVERLAP=1): the MLP blocks after the weight-gradient
  reduction, each grid level group after its accumulation launch.
Each is compared bitwise with the same training without it. Reference: testbed_nerf.cu:3723-4001 (the step),
adam.h:51-160 (elementwise Adam)."""
import contextlib
import os
import sys
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

BATCH = 4096


@contextlib.contextmanager
def _env(**kv):
    old = {k: os.environ.get(k) for k in kv}
    os.environ.update({k: str(v) for k, v in kv.items()})
    try:
        yield
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def _testbed(sc, fixed_rays=0, batch=BATCH):
    from neus2_amd import pyngp
    tb = pyngp.Testbed(pyngp.TestbedMode.Nerf)
    tb.set_dataset(sc["images"], sc["focal"], sc["principal"], sc["xforms"], 1)
    tb.reload_network_from_file(os.path.join(ROOT, "configs", "nerf", "base.json"), batch_size=batch, fixed_rays_per_batch=fixed_rays)
    return tb


def _parallel(*fns):
    errs = []

    def run(f):
        try:
            f()
        except Exception as e:  # noqa: BLE001 - re-raised below
            errs.append(e)

    ts = [threading.Thread(target=run, args=(f,)) for f in fns]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=300)
    assert not any(t.is_alive() for t in ts), "a rank did not finish"
    if errs:
        raise errs[0]


def _same(a, b):
    np.testing.assert_array_equal(a.get_params().view(np.uint32), b.get_params().view(np.uint32))
    np.testing.assert_array_equal(a.get_gradients().view(np.uint32), b.get_gradients().view(np.uint32))
    np.testing.assert_array_equal(a.get_ema_params().view(np.uint32), b.get_ema_params().view(np.uint32))
    np.testing.assert_array_equal(a.get_density_grid()[0].view(np.uint32), b.get_density_grid()[0].view(np.uint32))
    sa, sb = a.stats(), b.stats()
    for k in ("training_step", "rays_per_batch", "measured_batch_size", "n_rays_total", "loss"):
        assert sa[k] == sb[k], (k, sa[k], sb[k])


@pytest.fixture(scope="module")
def scene(torch_cuda):
    from neus2_amd import scenes
    return scenes.small_scene(n_views=8, width=64, height=48)


def test_adam_overlap_bitwise(scene):
    """300 steps in one call (the progressive level changes, the occupancy updates and their cadence change at step 256,
    the lookahead) with the optimizer split beside the scatter and without: bitwise the same parameters, gradients, EMA
    weights, occupancy grid and counters."""
    with _env(NEUS_ADAM_OVERLAP=1):
        a = _testbed(scene)
    with _env(NEUS_ADAM_OVERLAP=0):
        b = _testbed(scene)
    a.train_steps(300)
    b.train_steps(300)
    assert a.stats()["adam_split_steps"] == 300 and b.stats()["adam_split_steps"] == 0
    assert a.stats()["lookahead_steps"] > 0
    _same(a, b)


def test_dp_lookahead_bitwise(scene):
    """Two ranks (in-process group, host-staged collectives) with the lookahead on - it now runs beside the backward at
    any world size - against two ranks with it off (NEUS_LOOKAHEAD=0): 40 steps in one call each, bitwise the same on
    every rank; the lookahead ran."""
    from neus2_amd import pyngp
    R = 2048
    ga = pyngp.LocalGroup(2)
    a = [_testbed(scene, R) for _ in range(2)]
    with _env(NEUS_LOOKAHEAD=0):
        gb = pyngp.LocalGroup(2)
        b = [_testbed(scene, R) for _ in range(2)]
    for r in range(2):
        ga.join(a[r], r)
        gb.join(b[r], r)
    _parallel(lambda: a[0].train_steps(40), lambda: a[1].train_steps(40))
    _parallel(lambda: b[0].train_steps(40), lambda: b[1].train_steps(40))
    assert a[0].stats()["lookahead_steps"] > 0 and a[1].stats()["lookahead_steps"] > 0
    assert b[0].stats()["lookahead_steps"] == 0
    for x in (a[1], b[0], b[1]):
        _same(a[0], x)
    del ga, gb


def test_rccl_world1_lookahead_bitwise(scene):
    """A world-1 RCCL communicator (collectives forced on) now takes the lookahead too, its counters all-reduced on the
    communication stream before the sampling starts: bitwise the testbed without a communicator."""
    from neus2_amd import pyngp
    R = 2048
    plain = _testbed(scene, R)
    comm = _testbed(scene, R)
    comm.init_data_parallel(0, 1, pyngp.nccl_unique_id(), force_collectives=True)
    plain.train_steps(40)
    comm.train_steps(40)
    assert comm.stats()["lookahead_steps"] > 0
    _same(plain, comm)


def test_dp_adam_overlap_bitwise(scene):
    """Data parallel with the optimizer in pieces, each behind its range's all-reduce on the exchange stream (the MLP blocks,
    then every grid level group, the rest after the last collective), against the one Adam launch after the exchange:
    two world-2 groups, 40 steps, bitwise the same on every rank."""
    from neus2_amd import pyngp
    R = 2048
    with _env(NEUS_ADAM_OVERLAP=1):
        ga = pyngp.LocalGroup(2)
        a = [_testbed(scene, R) for _ in range(2)]
    with _env(NEUS_ADAM_OVERLAP=0):
        gb = pyngp.LocalGroup(2)
        b = [_testbed(scene, R) for _ in range(2)]
    for r in range(2):
        ga.join(a[r], r)
        gb.join(b[r], r)
    _parallel(lambda: a[0].train_steps(40), lambda: a[1].train_steps(40))
    _parallel(lambda: b[0].train_steps(40), lambda: b[1].train_steps(40))
    assert a[0].stats()["adam_split_steps"] == 40 and b[0].stats()["adam_split_steps"] == 0
    for x in (a[1], b[0], b[1]):
        _same(a[0], x)
    del ga, gb


def test_compaction_cut_bitwise(torch_cuda):
    """The compaction cut (march.hip k_prog_cut): with fixed rays per batch, the progressive rounds after round 0 skip the
    rays whose compaction base is already past the batch, and round 0 itself runs the rays below the previous step's cut first
    (the split sort), the rest only when the cut is not reached there. At the bench's shape (Config S, base.json, R = Nc =
    2^18 fixed) with progressive inference forced on from step 0, 600 steps in one call with the cut and without
    (NEUS_PROG_CUT=0): bitwise the same parameters, gradients, EMA weights, occupancy grid and - the last step of a call never
    cuts - the same counters; the cut ran and evaluated fewer samples. (On small scenes round 0 rarely reaches the batch
    before the last kept ray, so there is little to skip; scripts/fingerprint_bench_shape.py checks 900 steps with the auto
    rule.)"""
    from neus2_amd import pyngp, scenes
    sc = scenes.sphere_scene(49, 1600, 1200, principal=(823.2 / 1600, 619.1 / 1200))
    n = 1 << 18

    def tb_():
        tb = pyngp.Testbed(pyngp.TestbedMode.Nerf)
        tb.set_dataset(sc["images"], sc["focal"], sc["principal"], sc["xforms"], 1)
        tb.reload_network_from_file(os.path.join(ROOT, "configs", "nerf", "base.json"), batch_size=n, fixed_rays_per_batch=n)
        tb.set_progressive_inference(2)
        return tb
    res = {}
    for cut in (1, 0):
        with _env(NEUS_PROG_CUT=cut):
            tb = tb_()
        tb.train_steps(600)
        res[cut] = (tb.stats(), tb.get_params(), tb.get_gradients(), tb.get_ema_params(), tb.get_density_grid()[0])
        del tb
    sa, sb = res[1][0], res[0][0]
    assert sa["cut_steps"] > 400 and sb["cut_steps"] == 0, (sa["cut_steps"], sb["cut_steps"])
    assert sa["evaluated_samples_total"] < 0.9 * sb["evaluated_samples_total"], (sa["evaluated_samples_total"], sb["evaluated_samples_total"])
    for k in ("training_step", "rays_per_batch", "measured_batch_size", "measured_batch_size_before_compaction", "n_rays_total",
              "n_rays_with_samples", "progressive_steps", "loss"):
        assert sa[k] == sb[k], (k, sa[k], sb[k])
    for x, y in zip(res[1][1:], res[0][1:]):
        np.testing.assert_array_equal(x.view(np.uint32), y.view(np.uint32))
