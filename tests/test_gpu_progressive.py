"""Progressive (cut-off-aware) inference of the training step (march.hip k_chunk_first / k_loss_scan_chunk): the
network evaluated in rounds of per-ray sample chunks, a ray's next chunk only while its transmittance is >= 1e-4.
The composited samples, the recurrence and therefore every output must be bit-identical to the one-pass step
(testbed_nerf.cu:3802-3811 infers every kept sample): two testbeds from the same init, one forced progressive, one
forced one-pass, trained side by side and compared bitwise (parameters, optimizer state, occupancy grid, per-ray
counts, loss). The variance parameter is raised so the initial sphere is opaque and rays end mid-march (checked).
The progressive testbed runs the rounds in the spatial ray order (k_ray_sort_place, one list eighth per XCD) unless
NEUS_RAY_SORT=0 at its creation; both orders are compared with the one-pass step."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _pair(chunk_ends, steps=12, batch=4096):
    import os
    from neus2_amd import pyngp, scenes
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sc = scenes.small_scene(n_views=8, width=64, height=48)
    tbs = []
    for mode in (0, 2):
        tb = pyngp.Testbed(pyngp.TestbedMode.Nerf)
        tb.set_dataset(sc["images"], sc["focal"], sc["principal"], sc["xforms"], 1)
        tb.reload_network_from_file(os.path.join(root, "configs", "nerf", "base.json"), batch_size=batch)
        lay = tb.layout()
        p = tb.get_params()
        p[lay["variance_offset"]] = 0.9  # inv_s = exp(9): a sharp surface from step 0
        tb.set_params(p)
        tb.set_progressive_inference(mode, chunk_ends)
        tbs.append(tb)
    a, b = tbs
    cut = 0
    for _ in range(steps):
        a.train_steps(1)
        b.train_steps(1)
        na, ca, sa = a.ray_counts(1 << 18)
        nb, cb, sb = b.ray_counts(1 << 18)
        np.testing.assert_array_equal(ca, cb)
        np.testing.assert_array_equal(sa, sb)
        cut += int(((ca < na) & (na > chunk_ends[0])).sum())
    return a, b, cut


@pytest.mark.parametrize("chunk_ends", [(32, 80), (16, 48, 112), (1, 2, 5, 9)])
def test_progressive_inference_bit_identical(torch_cuda, chunk_ends):
    a, b, cut = _pair(chunk_ends)
    assert cut > 0, "no ray was cut mid-march: the test does not exercise the later rounds"
    np.testing.assert_array_equal(a.get_params().view(np.uint32), b.get_params().view(np.uint32))
    ga, bfa = a.get_density_grid()
    gb, bfb = b.get_density_grid()
    np.testing.assert_array_equal(ga.view(np.uint32), gb.view(np.uint32))
    np.testing.assert_array_equal(bfa, bfb)
    oa, ob = a.get_optimizer_state(), b.get_optimizer_state()
    for k in ("m1", "m2", "param_steps", "ema"):
        np.testing.assert_array_equal(np.asarray(oa[k]).view(np.uint8), np.asarray(ob[k]).view(np.uint8))
    sa, sb = a.stats(), b.stats()
    for k in ("loss", "measured_batch_size", "measured_batch_size_before_compaction"):
        assert sa[k] == sb[k], (k, sa[k], sb[k])


def test_progressive_slot_order_bit_identical(torch_cuda, monkeypatch):
    """The rounds in ray-slot order (NEUS_RAY_SORT=0, no XCD eighths): the same bitwise equality."""
    monkeypatch.setenv("NEUS_RAY_SORT", "0")
    a, b, cut = _pair((32, 80), steps=8)
    assert cut > 0
    np.testing.assert_array_equal(a.get_params().view(np.uint32), b.get_params().view(np.uint32))
