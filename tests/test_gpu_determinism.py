"""Determinism of the whole training step at the bench's shape.

The step is meant to be bitwise reproducible: every compaction is a scan, the grid gradient is summed in int64 fixed
point, the weight-gradient and variance sums are split-ordered, and the orders that atomics do fix (the spatial ray
sort's LDS cursors, k_ray_sort_place; the progressive rounds' list appends, k_loss_scan_chunk) only permute independent
work items. Three ways that could fail are probed at once, from one initialisation on Config S (49 x 1600x1200 views),
base.json, R = Nc = 2^18 fixed - the bench's step, with the auto rule running the progressive rounds, the spatial ray
order with its atomic within-cell order, and the region scatter's split heavy buckets:
* reference: one testbed trained alone;
* LDS garbage: every CU's LDS filled with a pattern (its complement on odd steps) before every kernel of every step
  (neus_debug_set_lds_fill_all): a kernel that read LDS it had not written in its own launch would change the result;
* concurrency: two testbeds trained at the same time from two host threads on the same GPU (the situation of round 4's
  r04d run, whose two-rank test found 5,096 parameters differing), so the atomics' orders and the CU sharing differ.
After 800 + 16 steps all four hold bitwise the same parameters, gradients, EMA weights and occupancy grid.
Round 5 found what broke the concurrent case: with kernels of two testbeds of one process co-resident on
a SIMD, a packed-fp32 instruction's upper-half result was read stale in lanes 48-63 (k_loss_grad's dL/doutput column 7;
6-8 of 12 concurrent pairs differing, 0 of 12 once no object uses packed fp32: profiles/r05i_*, r05j_*). The library is
built without packed fp32 since; this test passed with that build (profiles/r05j_pytest_determinism.log)."""
import ctypes as C
import os
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N = 1 << 18
PREPARE, STEPS = 800, 16


def _testbed(sc):
    from neus2_amd import pyngp
    tb = pyngp.Testbed(pyngp.TestbedMode.Nerf)
    tb.set_dataset(sc["images"], sc["focal"], sc["principal"], sc["xforms"], 1)
    tb.reload_network_from_file(os.path.join(ROOT, "configs", "nerf", "base.json"), batch_size=N, fixed_rays_per_batch=N)
    return tb


def _state(tb):
    grid, bf = tb.get_density_grid()
    return {"params": tb.get_params(), "grads": tb.get_gradients(), "ema": tb.get_ema_params(), "grid": grid, "bitfield": bf}


def test_bench_step_bitwise_under_lds_garbage_and_concurrency(torch_cuda):
    from neus2_amd import scenes
    from neus2_amd._lib import check, lib
    assert os.environ.get("NEUS_RAY_SORT", "1") != "0"
    sc = scenes.sphere_scene(49, 1600, 1200, principal=(823.2 / 1600, 619.1 / 1200))
    ref = _testbed(sc)
    ref.train_steps(PREPARE)
    p0 = ref.stats()["progressive_steps"]
    ref.train_steps(STEPS)
    st = ref.stats()
    assert st["progressive_steps"] - p0 == STEPS, "the auto rule did not run the progressive rounds (no ray sort either)"
    parts = np.zeros(st["valid_level"] + 1, np.uint32)
    check(lib().neus_debug_scatter_parts(ref.handle, C.c_void_p(parts.ctypes.data)))
    assert parts.max() > 1, "no split scatter bucket"
    want = _state(ref)
    del ref

    garbage = _testbed(sc)
    check(lib().neus_debug_set_lds_fill_all(garbage.handle, C.c_uint32(0xBF800000)))
    garbage.train_steps(PREPARE + STEPS)
    got = _state(garbage)
    for k, v in want.items():
        np.testing.assert_array_equal(got[k].view(np.uint8), v.view(np.uint8), err_msg=f"LDS garbage: {k}")
    del garbage

    pair = [_testbed(sc), _testbed(sc)]
    errs = []

    def run(tb):
        try:
            tb.train_steps(PREPARE + STEPS)
        except Exception as e:  # noqa: BLE001 - re-raised below
            errs.append(e)

    ts = [threading.Thread(target=run, args=(tb,)) for tb in pair]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=300)
    assert not any(t.is_alive() for t in ts) and not errs, errs
    for i, tb in enumerate(pair):
        got = _state(tb)
        for k, v in want.items():
            np.testing.assert_array_equal(got[k].view(np.uint8), v.view(np.uint8), err_msg=f"concurrent testbed {i}: {k}")


def test_lookahead_sampling_bitwise(torch_cuda):
    """The next step's ray sampling issued beside the current step's backward (the default; NEUS_LOOKAHEAD=0 turns it
    off, testbed.cpp la_go) gives the step the same samples: from one initialisation, 300 steps in one call (occupancy
    updates and loss readbacks, where the lookahead pauses, included) end with bitwise equal parameters, EMA weights,
    occupancy grid and per-ray counts, with and without it."""
    from neus2_amd import pyngp, scenes
    sc = scenes.sphere_scene(16, 400, 300, principal=(0.51, 0.52))
    out = {}
    for la in ("0", "1"):
        os.environ["NEUS_LOOKAHEAD"] = la
        try:
            tb = pyngp.Testbed(pyngp.TestbedMode.Nerf)
            tb.set_dataset(sc["images"], sc["focal"], sc["principal"], sc["xforms"], 1)
            tb.reload_network_from_file(os.path.join(ROOT, "configs", "nerf", "base.json"), batch_size=1 << 16)
            tb.train_steps(300)
            grid, bf = tb.get_density_grid()
            out[la] = {"params": tb.get_params(), "ema": tb.get_ema_params(), "grid": grid, "bitfield": bf,
                       "counts": np.concatenate(tb.ray_counts(1 << 16)[:2]), "step": tb.stats()["training_step"]}
            del tb
        finally:
            os.environ.pop("NEUS_LOOKAHEAD", None)
    assert out["0"]["step"] == out["1"]["step"] == 300
    for k in ("params", "ema", "grid", "bitfield", "counts"):
        np.testing.assert_array_equal(out["0"][k], out["1"][k], err_msg=k)
