"""Work issued beside the backward must not change a bit (round 6):
* the next step's ray sampling (the lookahead) with a data-parallel group: the step's counters are all-reduced right
  after the loss (StepState::compacted_global), so the sampling no longer waits for the whole exchange;
* the optimizer in pieces beside the grid scatter (NEUS_ADAM_OVERLAP=1): the MLP blocks after the weight-gradient
  reduction, each grid level group after its accumulation launch;
* the compaction cut and the march cut (the march of a cut step limited to the slots below the cut's estimate, with its
  witness and the host's re-run of a step whose witness failed).
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


def _bench_shape_runs(configs, steps, call=None):
    """Config S at the bench's shape (base.json, R = Nc = 2^18 fixed, progressive inference forced on), one testbed per
    environment in `configs`, each trained `steps` steps in one call: (stats, params, grads, EMA, occupancy grid)."""
    from neus2_amd import pyngp, scenes
    sc = scenes.sphere_scene(49, 1600, 1200, principal=(823.2 / 1600, 619.1 / 1200))
    n = 1 << 18
    res = []
    for env in configs:
        with _env(**env):
            tb = pyngp.Testbed(pyngp.TestbedMode.Nerf)
            tb.set_dataset(sc["images"], sc["focal"], sc["principal"], sc["xforms"], 1)
            tb.reload_network_from_file(os.path.join(ROOT, "configs", "nerf", "base.json"), batch_size=n, fixed_rays_per_batch=n)
            tb.set_progressive_inference(2)
            for k in range(0, steps, call or steps):
                tb.train_steps(min(call or steps, steps - k))
            res.append((tb.stats(), tb.get_params(), tb.get_gradients(), tb.get_ema_params(), tb.get_density_grid()[0]))
        del tb
    return res


STAT_KEYS = ("training_step", "rays_per_batch", "measured_batch_size", "measured_batch_size_before_compaction", "n_rays_total",
             "n_rays_with_samples", "progressive_steps", "loss")


def _same_run(a, b):
    for k in STAT_KEYS:
        assert a[0][k] == b[0][k], (k, a[0][k], b[0][k])
    for x, y in zip(a[1:], b[1:]):
        np.testing.assert_array_equal(x.view(np.uint32), y.view(np.uint32))


def test_march_cut_bitwise(torch_cuda):
    """The march cut (testbed.cpp march_cut_for): a cut step generates and marches only the ray slots below
    the compaction cut's estimate. At the bench's shape, 600 steps in one call with it (the default), without it
    (NEUS_MARCH_CUT=0) and with neither it nor the compaction cut (NEUS_PROG_CUT=0): bitwise the same parameters,
    gradients, EMA weights, occupancy grid and last-step counters; the march was cut on most steps; a failed witness
    (the re-run path) is counted."""
    a, b, c = _bench_shape_runs([{"NEUS_MARCH_CUT": 1}, {"NEUS_MARCH_CUT": 0}, {"NEUS_PROG_CUT": 0, "NEUS_MARCH_CUT": 0}], 600)
    assert a[0]["march_cut_steps"] > 300 and b[0]["march_cut_steps"] == 0, (a[0]["march_cut_steps"], b[0]["march_cut_steps"])
    assert a[0]["cut_steps"] > 400 and c[0]["cut_steps"] == 0
    _same_run(a, b)
    _same_run(a, c)


def test_march_cut_rerun_bitwise(torch_cuda):
    """The re-run path of the march cut: with the test hook NEUS_DBG_MARCH_CUT_DIV=8 the cut march covers an eighth of the
    estimate, so its slots often do not fill the batch (witness a) and the step after a cut one often has contributing rays
    past the marched count's bound (witness b, which first recounts the step before in full). Every such step is run again
    with the full march, nothing of its first run applied: 300 steps bitwise those without the march cut."""
    a, b = _bench_shape_runs([{"NEUS_MARCH_CUT": 1, "NEUS_DBG_MARCH_CUT_DIV": 8}, {"NEUS_MARCH_CUT": 0}], 300)
    assert a[0]["march_cut_reruns"] > 10, a[0]["march_cut_reruns"]
    _same_run(a, b)
    # the same in train calls of 23 steps (the re-runs land next to call ends, loss readbacks and occupancy updates)
    c, = _bench_shape_runs([{"NEUS_MARCH_CUT": 1, "NEUS_DBG_MARCH_CUT_DIV": 8}], 300, call=23)
    assert c[0]["march_cut_reruns"] > 10
    _same_run(c, b)


def test_dp_march_cut_rerun_bitwise(scene):
    """Two ranks (in-process group) with the march cut and the re-run hook (NEUS_DBG_MARCH_CUT_DIV=8, progressive inference
    forced on): a failed witness on either rank is all-reduced with the step's counters, so both ranks withhold the step and
    run it again together. 60 steps, bitwise two ranks without the march cut, on every rank."""
    from neus2_amd import pyngp
    R = 2048

    def group(env):
        with _env(**env):
            g = pyngp.LocalGroup(2)
            tbs = [_testbed(scene, R) for _ in range(2)]
        for r in range(2):
            tbs[r].set_progressive_inference(2)
            g.join(tbs[r], r)
        _parallel(lambda: tbs[0].train_steps(60), lambda: tbs[1].train_steps(60))
        return g, tbs
    ga, a = group({"NEUS_MARCH_CUT": 1, "NEUS_DBG_MARCH_CUT_DIV": 8})
    gb, b = group({"NEUS_MARCH_CUT": 0})
    sa = [t.stats() for t in a]
    assert sa[0]["march_cut_steps"] > 0 and sa[0]["march_cut_reruns"] == sa[1]["march_cut_reruns"], sa
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
        with _env(NEUS_PROG_CUT=cut, NEUS_MARCH_CUT=0):
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
