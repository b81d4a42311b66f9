"""The product's data-parallel path as separate processes: two rank processes on one
MI355X (tests/dp_worker.py), each a Testbed attached to the cross-process host-staged group (hostgroup.h), whose
collectives are staged on the communication stream by host functions gated by the same events as the RCCL collectives
(the overlapped exchange's concurrency runs). Checked: after 16 steps both processes hold bitwise the parameters,
gradients, EMA weights and occupancy grid of each other and of the in-process two-rank group (NeusLocalGroup, which
reduces in the same rank order); the rank-setting check; a health failure injected on one rank stops both ranks on the
same step (the health words are all-reduced with the loss sums and raised at a step boundary)."""
import os
import socket
import subprocess
import sys
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BATCH = 4096
R = 2048
STEPS = 16


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _parallel(*fns):
    errs = [None] * len(fns)

    def run(i, f):
        try:
            f()
        except Exception as e:  # noqa: BLE001 - returned to the caller
            errs[i] = e

    ts = [threading.Thread(target=run, args=(i, f)) for i, f in enumerate(fns)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=300)
    assert not any(t.is_alive() for t in ts), "a rank did not finish"
    return errs


@pytest.fixture(scope="module")
def scene(torch_cuda):
    from neus2_amd import scenes
    return scenes.small_scene(n_views=8, width=64, height=48)


def _testbed(sc):
    from neus2_amd import pyngp
    tb = pyngp.Testbed(pyngp.TestbedMode.Nerf)
    tb.set_dataset(sc["images"], sc["focal"], sc["principal"], sc["xforms"], 1)
    tb.reload_network_from_file(os.path.join(ROOT, "configs", "nerf", "base.json"), batch_size=BATCH, fixed_rays_per_batch=R)
    return tb


def test_two_processes_match_each_other_and_the_local_group(scene, tmp_path):
    from neus2_amd import pyngp
    port = _free_port()
    outs = [str(tmp_path / f"rank{r}.npz") for r in range(2)]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    procs = [subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "dp_worker.py"), str(r), "2", str(port), str(STEPS), str(R),
                               "1", outs[r]], env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True) for r in range(2)]
    logs = []
    for p in procs:
        try:
            o, _ = p.communicate(timeout=240)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        logs.append(o)
    assert all(p.returncode == 0 for p in procs), logs
    a, b = (np.load(o) for o in outs)
    # the in-process two-rank group from the same init, on this process
    group = pyngp.LocalGroup(2)
    tbs = [_testbed(scene) for _ in range(2)]
    for r, tb in enumerate(tbs):
        group.join(tb, r)
    errs = _parallel(lambda: tbs[0].train_steps(STEPS), lambda: tbs[1].train_steps(STEPS))
    assert not any(errs), errs
    ref = {"params": tbs[0].get_params(), "grads": tbs[0].get_gradients(), "ema": tbs[0].get_ema_params(), "grid": tbs[0].get_density_grid()[0]}
    for k, v in ref.items():
        np.testing.assert_array_equal(a[k].view(np.uint32), b[k].view(np.uint32), err_msg=k)
        np.testing.assert_array_equal(a[k].view(np.uint32), v.view(np.uint32), err_msg=k)
    np.testing.assert_array_equal(a["bitfield"], b["bitfield"])
    np.testing.assert_array_equal(a["stats"], b["stats"])
    st = tbs[0].stats()
    assert int(a["stats"][3]) == STEPS * 2 * R == st["n_rays_total"]
    assert float(a["loss"]) == float(b["loss"]) == st["loss"]
    assert int(a["host_group"]) == 1 and int(a["coll_calls"]) > 0 and int(a["coll_bytes"]) == int(b["coll_bytes"])
    del tbs, group


def test_mismatched_exchange_setting_fails_on_every_rank(scene):
    """the overlapped and grouped exchanges issue different collective sequences, so ranks with different
    settings would deadlock; the first step checks the setting across ranks and every rank fails with a message."""
    from neus2_amd import pyngp
    group = pyngp.LocalGroup(2)
    tbs = [_testbed(scene) for _ in range(2)]
    for r, tb in enumerate(tbs):
        group.join(tb, r)
    tbs[1].set_exchange_overlap(False)
    errs = _parallel(lambda: tbs[0].train_steps(2), lambda: tbs[1].train_steps(2))
    for e in errs:
        assert e is not None and "exchange overlap" in str(e), errs
    assert tbs[0].stats()["training_step"] == tbs[1].stats()["training_step"] == 0
    del tbs, group


def test_health_failure_on_one_rank_stops_every_rank(scene):
    """a device health bit raised on rank 1 only (neus_debug_inject_health) is all-reduced with the
    loss sums, so both ranks raise at the same step boundary (no rank left blocking in a collective, no step half
    applied: the training step counts agree)."""
    import ctypes as C
    from neus2_amd import pyngp
    from neus2_amd._lib import check, lib
    group = pyngp.LocalGroup(2)
    tbs = [_testbed(scene) for _ in range(2)]
    for r, tb in enumerate(tbs):
        group.join(tb, r)
    errs = _parallel(lambda: tbs[0].train_steps(3), lambda: tbs[1].train_steps(3))
    assert not any(errs), errs
    check(lib().neus_debug_inject_health(tbs[1].handle, C.c_uint32(1)))
    errs = _parallel(lambda: tbs[0].train_steps(40), lambda: tbs[1].train_steps(40))
    assert errs[0] is not None and "another rank" in str(errs[0]), errs
    assert errs[1] is not None and "health check failed" in str(errs[1]) and "another rank" not in str(errs[1]), errs
    s0, s1 = tbs[0].stats(), tbs[1].stats()
    assert s0["training_step"] == s1["training_step"] and s0["training_step"] % 16 == 0, (s0["training_step"], s1["training_step"])
    assert s0["training_aborted"] and s1["training_aborted"] and s1["health_flags"] & 1
    del tbs, group


def test_health_failure_on_every_rank_names_its_cause(scene):
    """the health words are summed over the ranks. The same march fault (STEP_FAIL_MARCH_T = 1) on both ranks
    sums to 2, which read as a bit set would have named the look-back scan; both ranks must report the march."""
    import ctypes as C
    from neus2_amd import pyngp
    from neus2_amd._lib import check, lib
    group = pyngp.LocalGroup(2)
    tbs = [_testbed(scene) for _ in range(2)]
    for r, tb in enumerate(tbs):
        group.join(tb, r)
    errs = _parallel(lambda: tbs[0].train_steps(3), lambda: tbs[1].train_steps(3))
    assert not any(errs), errs
    for tb in tbs:
        check(lib().neus_debug_inject_health(tb.handle, C.c_uint32(1)))
    errs = _parallel(lambda: tbs[0].train_steps(40), lambda: tbs[1].train_steps(40))
    for e in errs:
        assert e is not None and "non-finite or negative t" in str(e) and "look-back scan" not in str(e), errs
    s0, s1 = tbs[0].stats(), tbs[1].stats()
    assert s0["training_step"] == s1["training_step"], (s0["training_step"], s1["training_step"])
    assert s0["health_flags"] == s1["health_flags"] == 1, (s0["health_flags"], s1["health_flags"])
    del tbs, group
