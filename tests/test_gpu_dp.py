"""The product's data-parallel step with two ranks in one process on one MI355X.

neus_local_group gives the testbeds the RCCL path's collectives with host-staged buffers, so the whole
train_step runs as it does on 8 GPUs: the sharded occupancy update with its max all-reduce, the gradient /
counter / loss / DeltaNetwork all-reduces (collectives 1-3), then the replicated optimizer. Checked here:
* the sharded occupancy update is bit-identical to the single-GPU update (max is exact);
* the all-reduced gradient of a step equals the oracle's sum of the two ranks' gradients (oracle/cpu_step.py
  with rank/world: global ray index r*R + i, loss over world*R rays, eikonal over world*Nc);
* after free-running steps both ranks hold bitwise-identical parameters and the same counters / rays per batch;
* a dynamic frame (global-movement phase) keeps the DeltaNetwork parameters identical across ranks."""
import ctypes as C
import os
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BATCH = 4096
G3 = 128 ** 3


def _record(test, **metrics):
    import json
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "parity_metrics.jsonl"), "a") as f:
        f.write(json.dumps({"test": test, **{k: float(v) for k, v in metrics.items()}}) + "\n")


def _parallel(*fns):
    """Runs one callable per rank in its own thread (the collectives block until every rank arrives)."""
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


def _testbed(sc, fixed_rays=0):
    from neus2_amd import pyngp
    tb = pyngp.Testbed(pyngp.TestbedMode.Nerf)
    tb.set_dataset(sc["images"], sc["focal"], sc["principal"], sc["xforms"], 1)
    tb.reload_network_from_file(os.path.join(ROOT, "configs", "nerf", "base.json"), batch_size=BATCH, fixed_rays_per_batch=fixed_rays)
    return tb


def _ranks(sc, world=2, fixed_rays=0):
    from neus2_amd import pyngp
    group = pyngp.LocalGroup(world)
    tbs = [_testbed(sc, fixed_rays) for _ in range(world)]
    for r, tb in enumerate(tbs):
        group.join(tb, r)
    return group, tbs


@pytest.fixture(scope="module")
def scene(torch_cuda):
    from neus2_amd import scenes
    return scenes.small_scene(n_views=8, width=64, height=48)


def _occ(tb, n_u, n_nu):
    from neus2_amd._lib import check, lib
    check(lib().neus_occ_update(tb.handle, None, C.c_uint32(n_u), C.c_uint32(n_nu)))


def test_dp_sharded_occupancy_matches_single(scene):
    """Each rank evaluates half of the density-grid samples; after the max all-reduce every rank's grid and
    bitfield equal the single-GPU update bit for bit: the step-0 update (128^3 uniform samples) and a
    quarter-uniform + quarter-occupancy-biased update on perturbed parameters."""
    single = _testbed(scene)
    group, (a, b) = _ranks(scene)
    _occ(single, G3, 0)
    _parallel(lambda: _occ(a, G3, 0), lambda: _occ(b, G3, 0))
    g1, b1 = single.get_density_grid()
    for tb in (a, b):
        g, bf = tb.get_density_grid()
        np.testing.assert_array_equal(g, g1)
        np.testing.assert_array_equal(bf, b1)
    rng = np.random.default_rng(5)
    p = single.get_params().copy()
    lay = single.layout()
    p[lay["grid_offset"]:lay["variance_offset"]] += rng.uniform(-0.05, 0.05, lay["variance_offset"] - lay["grid_offset"]).astype(np.float32)
    for tb in (single, a, b):
        tb.set_params(p)
    _occ(single, G3 // 4, G3 // 4)
    _parallel(lambda: _occ(a, G3 // 4, G3 // 4), lambda: _occ(b, G3 // 4, G3 // 4))
    g1, b1 = single.get_density_grid()
    assert np.unpackbits(b1[: G3 // 8]).mean() > 0.001
    for tb in (a, b):
        g, bf = tb.get_density_grid()
        np.testing.assert_array_equal(g, g1)
        np.testing.assert_array_equal(bf, b1)
    assert a.get_rng()[2] == single.get_rng()[2]
    del group


def _blocks(lay):
    return {"density": (0, lay["n_density"]), "rgb": (lay["n_density"], lay["n_matrix"]),
            "grid": (lay["grid_offset"], lay["variance_offset"]), "variance": (lay["variance_offset"], lay["variance_offset"] + 1)}


def _perturbed(tb, seed=5):
    """Parameters that make every gradient block nonzero at step 0: geometric init leaves W0's encoding columns at 0
    (so no grid gradient at all); draw them ~N(0, 0.3) and the grid ~U(-0.1, 0.1) (as test_gpu_configs)."""
    rng = np.random.default_rng(seed)
    lay = tb.layout()
    p = tb.get_params().copy()
    W, din, L = 64, lay["density_input_width"], lay["n_levels"]
    w0 = p[: W * din].reshape(W, din)
    w0[:, 3:3 + 2 * L] = rng.normal(0, 0.3, (W, 2 * L))
    p[: W * din] = w0.reshape(-1)
    p[lay["grid_offset"]:lay["variance_offset"]] = rng.uniform(-0.1, 0.1, lay["variance_offset"] - lay["grid_offset"])
    return p


def test_dp_step_gradient_matches_oracle_and_ranks_stay_identical(scene):
    """World 2, R = 2048 rays per rank (fixed), from perturbed parameters (every block, the grid included, has a
    nonzero gradient): the all-reduced gradient of the first step against the oracle's rank-0 + rank-1 gradients on
    the same occupancy grid (the device's, injected: the march is then bit-exact), per parameter block cosine >= 0.999
    and rel-L2 <= 2e-2 (the device sums fp16 contributions in a different order; the fp16 network noise can move a
    transmittance cut-off, i.e. a few compacted samples). Then 11 more free-running steps after which both ranks'
    parameters, EMA weights, counters and occupancy grids are bitwise identical and n_rays_total counts the global
    rays."""
    import oracle as O
    from cpu_step import CpuTrainer
    R = 2048
    group, (a, b) = _ranks(scene, fixed_rays=R)
    lay = a.layout()
    p0 = _perturbed(a)
    a.set_params(p0)
    b.set_params(p0)
    _parallel(lambda: a.train_steps(1), lambda: b.train_steps(1))
    ga, gb = a.get_gradients(), b.get_gradients()
    np.testing.assert_array_equal(ga, gb)
    grid, bf = a.get_density_grid()
    cfg = O.make_cfg(per_level_scale=a._net_cfg.per_level_scale)
    ds = O.Dataset(scene["images"], scene["focal"], scene["principal"], scene["xforms"])
    gref = np.zeros(p0.size, np.float64)
    comp = 0
    for r in range(2):
        tr = CpuTrainer(cfg, ds, p0, batch=BATCH, rays_per_batch=R, fixed_rays=True, rank=r, world=2)
        tr.density_grid[:] = grid
        tr.bitfield[:] = bf
        gref += tr.grads(skip_occupancy=True)
        comp += tr.last["compacted"]
    res = {}
    for name, (lo, hi) in _blocks(lay).items():
        x, y = ga[lo:hi].astype(np.float64), gref[lo:hi]
        res[name] = (x @ y / max(np.linalg.norm(x) * np.linalg.norm(y), 1e-30), np.linalg.norm(x - y) / max(np.linalg.norm(y), 1e-30))
    _record("dp_world2_grad", compacted_gpu=a.stats()["measured_batch_size"] * 2, compacted_oracle=comp,
            **{f"cos_{k}": v[0] for k, v in res.items()}, **{f"rel_{k}": v[1] for k, v in res.items()})
    for name, (cos, rel) in res.items():
        lo, hi = _blocks(lay)[name]
        assert np.any(gref[lo:hi]) and np.any(ga[lo:hi]), name  # every block carries a gradient here
        assert cos >= 0.999 and rel <= 2e-2, (name, cos, rel)
    assert abs(a.stats()["measured_batch_size"] - comp / 2) <= 0.01 * comp / 2
    _parallel(lambda: a.train_steps(11), lambda: b.train_steps(11))
    np.testing.assert_array_equal(a.get_params(), b.get_params())
    np.testing.assert_array_equal(a.get_ema_params(), b.get_ema_params())
    sa, sb = a.stats(), b.stats()
    for k in ("training_step", "rays_per_batch", "measured_batch_size", "n_rays_total", "loss"):
        assert sa[k] == sb[k], k
    assert sa["n_rays_total"] == 12 * 2 * R
    np.testing.assert_array_equal(a.get_density_grid()[0], b.get_density_grid()[0])
    del group


def test_dp_overlapped_exchange_bitwise(scene):
    """The overlapped gradient exchange (MLP blocks after the weight-gradient reduction, the grid levels in three
    groups as the scatter finishes them) against the one grouped exchange after the backward: two world-2 groups from
    the same init train 20 steps (crossing progressive-level changes and occupancy updates); every rank of both groups
    holds bitwise the same parameters, gradients and EMA weights, and the overlapped ranks issued more (split)
    collective calls for the same bytes."""
    R = 2048
    ga, (a0, a1) = _ranks(scene, fixed_rays=R)
    gb, (b0, b1) = _ranks(scene, fixed_rays=R)
    for tb in (b0, b1):
        tb.set_exchange_overlap(False)
    _parallel(lambda: a0.train_steps(20), lambda: a1.train_steps(20))
    _parallel(lambda: b0.train_steps(20), lambda: b1.train_steps(20))
    for x in (a1, b0, b1):
        np.testing.assert_array_equal(a0.get_params().view(np.uint32), x.get_params().view(np.uint32))
        np.testing.assert_array_equal(a0.get_gradients().view(np.uint32), x.get_gradients().view(np.uint32))
        np.testing.assert_array_equal(a0.get_ema_params().view(np.uint32), x.get_ema_params().view(np.uint32))
    # the exchange skips the grid range past the progressive valid level: it must be zero on every rank (the scatter's
    # sc_zero_from invariant the reduced range relies on, testbed.cpp collective 1)
    import oracle as O
    lay = a0.layout()
    off, _, _, _ = O.grid_tables(O.make_cfg(per_level_scale=a0._net_cfg.per_level_scale))
    act = a0.stats()["valid_level"] + 1
    assert act < lay["n_levels"]
    for x in (a0, a1):
        tail = x.get_gradients()[lay["grid_offset"] + 2 * int(off[act]): lay["variance_offset"]]
        assert tail.size > 0 and not np.any(tail)
    ia, ib = a0.data_parallel_info(), b0.data_parallel_info()
    assert ia["allreduce_bytes"] == ib["allreduce_bytes"]
    assert ia["collective_calls"] > ib["collective_calls"]
    del ga, gb


def test_rccl_world1_matches_no_communicator(scene):
    """The RCCL path of the data-parallel step with a world-1 communicator (neus_nccl_unique_id ->
    neus_testbed_init_data_parallel(0, 1, id): ncclCommInitRank, and the grouped ncclAllReduce calls of every step
    forced on although one rank would skip them): 12 steps are bitwise identical to the testbed without a
    communicator (a one-rank all-reduce is the identity). The default overlapped exchange runs its all-reduces on the
    communication stream, joined by events; the non-overlapped grouped exchange is checked the same way."""
    from neus2_amd import pyngp
    R = 2048
    plain = _testbed(scene, fixed_rays=R)
    comm = _testbed(scene, fixed_rays=R)
    comm.init_data_parallel(0, 1, pyngp.nccl_unique_id(), force_collectives=True)
    plain.train_steps(12)
    comm.train_steps(12)
    np.testing.assert_array_equal(plain.get_params(), comm.get_params())
    np.testing.assert_array_equal(plain.get_gradients(), comm.get_gradients())
    np.testing.assert_array_equal(plain.get_density_grid()[0], comm.get_density_grid()[0])
    sp, sc = plain.stats(), comm.stats()
    for k in ("training_step", "rays_per_batch", "measured_batch_size", "n_rays_total", "loss"):
        assert sp[k] == sc[k], k
    assert comm.data_parallel_info()["collective_calls"] > 0
    grouped = _testbed(scene, fixed_rays=R)
    grouped.init_data_parallel(0, 1, pyngp.nccl_unique_id(), force_collectives=True)
    grouped.set_exchange_overlap(False)
    grouped.train_steps(12)
    np.testing.assert_array_equal(plain.get_params(), grouped.get_params())


def test_dp_dynamic_frame_movement_identical(torch_cuda):
    """A dynamic frame on two ranks: the global-movement phase (DeltaNetwork only) and the finetuning steps after
    it all-reduce the DeltaNetwork gradient partials, so the learned movement and the canonical parameters stay
    bitwise identical across ranks (without the exchange each rank would learn its own movement)."""
    from neus2_amd import pyngp, scenes
    frames = scenes.dynamic_scene(n_frames=2, shift=(0.02, 0.0, 0.0))
    group = pyngp.LocalGroup(2)
    tbs = []
    for r in range(2):
        tb = pyngp.Testbed(pyngp.TestbedMode.Nerf)
        tb.set_dataset_frames(frames)
        tb.reload_network_from_file(os.path.join(ROOT, "configs", "nerf", "base.json"), batch_size=BATCH)
        group.join(tb, r)
        tbs.append(tb)
    a, b = tbs
    _parallel(lambda: a.train_steps(100), lambda: b.train_steps(100))
    _parallel(lambda: a.training_network_next_frame(), lambda: b.training_network_next_frame())
    _parallel(lambda: a.train_steps(60), lambda: b.train_steps(60))
    la, lb = a.get_movement()[1], b.get_movement()[1]
    np.testing.assert_array_equal(la, lb)
    assert la[0] != 0.0
    np.testing.assert_array_equal(a.get_params(), b.get_params())
    del group
