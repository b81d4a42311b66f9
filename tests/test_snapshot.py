"""Snapshot format (Testbed::save_snapshot / load_snapshot, testbed.cu:3144-3254): the msgpack object the
reference writes, built from a testbed's state and decoded back. CPU: the host encoder/decoder on a stand-in
testbed (no device). GPU (test_gpu_parity.py::test_snapshot_round_trip): train, save, load into a fresh
testbed, identical parameters / grid / counters and identical renders."""
import os

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class _FakeTestbed:
    """The state accessors build_snapshot reads, with fixed values."""

    def __init__(self, n_params=1000):
        from neus2_amd import config
        rng = np.random.default_rng(3)
        self._cfg_dict = config.load_json(os.path.join(ROOT, "configs", "nerf", "base.json"))
        self._params = rng.standard_normal(n_params).astype(np.float32)
        self._grid = np.abs(rng.standard_normal(128 ** 3)).astype(np.float32)
        self._images = [np.zeros((6, 8, 4), np.uint8)] * 3
        self._dataset_meta = {"xforms": [np.eye(4)[:3]] * 3, "focal": [[10.0, 10.0]] * 3,
                              "principal": [[0.5, 0.5]] * 3, "aabb_scale": 1.0}
        self._scale, self._offset = 0.5, np.full(3, 0.5, np.float32)

    def stats(self):
        return {"training_step": 123, "rays_per_batch": 4096, "measured_batch_size": 5000,
                "measured_batch_size_before_compaction": 9000, "loss": 0.25}

    def get_ema_params(self):
        return self._params

    def get_params(self):
        return self._params * 0

    def get_half_params(self, inference=False):
        return (self._params if inference else self._params * 0).astype(np.float16)

    def get_optimizer_state(self):
        n = self._params.size
        return {"current_step": 123, "learning_rate": 1e-3, "learning_rate_factor": 0.5,
                "m1": np.linspace(-1, 1, n).astype(np.float32), "m2": np.linspace(0, 2, n).astype(np.float32),
                "param_steps": np.arange(n, dtype=np.uint32), "ema": self._params.astype(np.float16)}

    def get_density_grid(self):
        return self._grid, None

    def get_movement(self):
        R = np.array([[0, -1, 0], [1, 0, 0], [0, 0, 1]], np.float32)
        return np.concatenate([R, np.array([[0.1], [0.2], [0.3]], np.float32)], 1), np.arange(12, dtype=np.float32) / 16


def test_snapshot_layout_and_round_trip(tmp_path):
    from neus2_amd import snapshot
    tb = _FakeTestbed()
    cfg = snapshot.build_snapshot(tb)
    p = tmp_path / "s.msgpack"
    p.write_bytes(snapshot.pack(cfg))
    back = snapshot.read_snapshot(str(p))
    s = back["snapshot"]
    # keys the reference writes (testbed.cu:3146-3172, trainer.h:284-286, nerf_network.h:1202-1245)
    for k in ("n_params", "params_binary", "rotation", "transition", "local_rotation", "local_transition",
              "density_grid_size", "density_grid_binary", "training_step", "loss"):
        assert k in s, k
    assert set(s["nerf"]["rgb"]) == {"rays_per_batch", "measured_batch_size", "measured_batch_size_before_compaction"}
    assert isinstance(s["params_binary"], bytes) and len(s["params_binary"]) == 2 * tb._params.size
    assert len(s["rotation"]) == 2 * 12 and len(s["transition"]) == 2 * 4
    assert len(s["local_rotation"]) == 2 * 8 and len(s["local_transition"]) == 2 * 4
    assert len(s["density_grid_binary"]) == 2 * 128 ** 3 and s["density_grid_size"] == 128
    assert back["encoding"] == tb._cfg_dict["encoding"] and back["network"] == tb._cfg_dict["network"]
    f = snapshot.restore_fields(back)
    np.testing.assert_array_equal(f["params"], tb._params.astype(np.float16).astype(np.float32))
    np.testing.assert_array_equal(f["grid"], tb._grid.astype(np.float16).astype(np.float32))
    g, l = tb.get_movement()
    np.testing.assert_array_equal(f["global_Rt"], g.astype(np.float16).astype(np.float32))
    np.testing.assert_array_equal(f["local"], l.astype(np.float16).astype(np.float32))
    assert (f["training_step"], f["rays_per_batch"], f["measured_batch_size"],
            f["measured_batch_size_before_compaction"]) == (123, 4096, 5000, 9000)
    assert f["loss"] == 0.25 and "snapshot" not in f["network"]


def test_snapshot_errors(tmp_path):
    from neus2_amd import snapshot
    p = tmp_path / "n.msgpack"
    p.write_bytes(snapshot.pack({"network": {}}))
    with pytest.raises(RuntimeError, match="does not contain a snapshot"):
        snapshot.read_snapshot(str(p))
    cfg = snapshot.build_snapshot(_FakeTestbed())
    cfg["snapshot"]["density_grid_size"] = 64
    with pytest.raises(RuntimeError, match="Incompatible grid size"):
        snapshot.restore_fields(cfg)
    cfg["snapshot"]["density_grid_size"] = 128
    cfg["snapshot"]["density_grid_binary"] = bytes(2 * 128 ** 3 * 2)
    with pytest.raises(RuntimeError, match="cascades"):
        snapshot.restore_fields(cfg)
    cfg["snapshot"]["density_grid_binary"] = b""  # an untrained model's empty grid is valid
    assert snapshot.restore_fields(cfg)["grid"].size == 0



def test_snapshot_optimizer_state_layout():
    """include_optimizer_state: snapshot.optimizer = Ema::serialize {nested: ExponentialDecay {nested: Adam
    {current_step, base_learning_rate, first/second_moments_binary (f32), param_steps_binary (u32)}, learning_rate,
    learning_rate_factor}, weights_ema_binary (fp16)} (ema.h:182-187, exponential_decay.h:128-134, adam.h:424-432),
    decoded back exactly; without it there is no optimizer key."""
    from neus2_amd import snapshot
    tb = _FakeTestbed()
    assert "optimizer" not in snapshot.build_snapshot(tb)["snapshot"]
    cfg = snapshot.unpack(snapshot.pack(snapshot.build_snapshot(tb, include_optimizer_state=True)))
    o = cfg["snapshot"]["optimizer"]
    adam = o["nested"]["nested"]
    assert set(adam) == {"current_step", "base_learning_rate", "first_moments_binary", "second_moments_binary", "param_steps_binary"}
    assert o["nested"]["learning_rate"] == 1e-3 and o["nested"]["learning_rate_factor"] == 0.5
    assert adam["current_step"] == 123 and abs(adam["base_learning_rate"] - 5e-4) < 1e-12
    n = tb._params.size
    assert len(adam["first_moments_binary"]) == 4 * n and len(adam["param_steps_binary"]) == 4 * n
    assert len(o["weights_ema_binary"]) == 2 * n
    f = snapshot.restore_fields(cfg)["optimizer"]
    ref = tb.get_optimizer_state()
    for k in ("m1", "m2", "param_steps", "ema"):
        np.testing.assert_array_equal(f[k], ref[k])
    assert (f["current_step"], f["learning_rate_factor"]) == (123, 0.5)


def test_snapshot_dataset_schema():
    """snapshot.nerf.dataset follows NerfDataset to_json (json_binding.h:131-159): every key from_json reads with
    .at() (json_binding.h:161-201) is present, per image under metadata[i], and xforms[i] is a TrainingXForm
    {start, end} of 3x4 rows."""
    from neus2_amd import snapshot
    tb = _FakeTestbed()
    tb._aabb = (np.full(3, -0.5, np.float32), np.full(3, 1.5, np.float32))
    tb._from_na = False
    ds = snapshot.build_snapshot(tb)["snapshot"]["nerf"]["dataset"]
    for k in snapshot.DATASET_REQUIRED_KEYS:
        assert k in ds, k
    assert ds["n_images"] == 3 and len(ds["metadata"]) == 3 and len(ds["xforms"]) == 3
    for m in ds["metadata"]:
        for k in snapshot.METADATA_REQUIRED_KEYS:
            assert k in m, k
        assert m["resolution"] == [8, 6] and m["focal_length"] == [10.0, 10.0] and m["principal_point"] == [0.5, 0.5]
        assert m["rolling_shutter"] == [0.0, 0.0, 0.0, 0.0] and m["camera_distortion"] is None
    for x in ds["xforms"]:
        assert np.asarray(x["start"]).shape == (3, 4) and x["start"] == x["end"]
    assert ds["render_aabb"] == {"min": [-0.5] * 3, "max": [1.5] * 3}
    assert ds["up"] == [0.0, 1.0, 0.0] and ds["envmap_resolution"] == [0, 0]
    assert ds["scale"] == 0.5 and ds["offset"] == [0.5] * 3 and ds["aabb_scale"] == 1
    assert ds["from_mitsuba"] is False and ds["from_na"] is False
    # msgpack round trip keeps the structure (null distortion, nested lists)
    back = snapshot.unpack(snapshot.pack({"d": ds}))["d"]
    assert back == ds
