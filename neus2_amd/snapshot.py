"""Snapshot save / load in the reference's msgpack format.

The file is the network config JSON with a "snapshot" object, serialised with msgpack; binary blobs are
msgpack `bin` (nlohmann::json::binary_t). Fields, in the reference's order of writing:

  Testbed::save_snapshot             testbed.cu:3144-3178
    snapshot = Trainer::serialize    trainer.h:281-293   n_params, params_binary (fp16 inference params)
                                                         [, optimizer] (include_optimizer_state: Ema / ExpDecay / Adam)
    rotation / transition            nerf_network.h:1179-1205  accumulated global movement, fp16 [12] / [4]
                                                         (3x3 row-major + 3 zero pad / xyz + 1 zero pad)
    local_rotation / local_transition nerf_network.h:1243-1247 DeltaNetwork params, fp16 [8] / [4]
    density_grid_size = 128, density_grid_binary (fp16), nerf.aabb_scale, training_step, loss,
    nerf.rgb.{rays_per_batch, measured_batch_size, measured_batch_size_before_compaction}, nerf.dataset

  Testbed::load_snapshot             testbed.cu:3197-3254: reset_network from the file's own config, counters,
    density grid (fp16 -> fp32, then update_density_grid_mean_and_bitfield), training_step, loss,
    Trainer::deserialize (params), global and local movement.

The inference params the reference serialises (m_params_inference) are the EMA weights when the EMA optimizer
is active (base.json), so params_binary = fp16(EMA weights); after a load both the training and the inference
weights are the loaded ones (Trainer::set_params, trainer.h:72-109), as in the reference.
"""
from __future__ import annotations

import copy

import numpy as np

try:
    import msgpack
except ImportError as e:  # pragma: no cover - msgpack ships in the image
    raise ImportError("neus2_amd.snapshot needs the msgpack package") from e

NERF_GRIDSIZE = 128


def _f16_bytes(a) -> bytes:
    return np.ascontiguousarray(np.asarray(a, np.float32).astype(np.float16)).tobytes()


def _f16_array(b) -> np.ndarray:
    return np.frombuffer(bytes(b), np.float16).astype(np.float32)


# NerfDataset::from_json (json_binding.h:161-201) reads these keys with .at(); the per-image ones live under
# metadata[i] and xforms[i] (TrainingXForm start / end).
DATASET_REQUIRED_KEYS = ("n_images", "xforms", "render_aabb", "up", "offset", "envmap_resolution", "scale", "aabb_scale",
                         "from_mitsuba", "from_na")
METADATA_REQUIRED_KEYS = ("resolution", "focal_length", "principal_point", "rolling_shutter", "camera_distortion")


def dataset_json(tb) -> dict:
    """NerfDataset to_json (json_binding.h:131-159): per-image metadata (focal length in pixels, camera
    distortion - none, so null -, normalised principal point, rolling shutter, resolution), per-image TrainingXForm
    {start, end} 3x4 row lists, render_aabb {min, max}, up, offset, envmap_resolution, scale, aabb_scale and the
    loader flags. No pixels (the reference does not serialise them either)."""
    imgs = tb._images or []
    meta = getattr(tb, "_dataset_meta", None) or {}
    xforms = [np.asarray(x, np.float32).reshape(3, 4).tolist() for x in meta.get("xforms", [])]
    focal = [[float(v) for v in np.broadcast_to(np.asarray(f, np.float32), (2,))] for f in meta.get("focal", [])]
    principal = [[float(v) for v in np.asarray(p, np.float32).reshape(2)] for p in meta.get("principal", [])]
    metadata = [{
        "focal_length": focal[i],
        "camera_distortion": None,
        "principal_point": principal[i],
        "rolling_shutter": [0.0, 0.0, 0.0, 0.0],
        "resolution": [int(im.shape[1]), int(im.shape[0])],
    } for i, im in enumerate(imgs)]
    amin, amax = getattr(tb, "_aabb", (np.zeros(3), np.ones(3)))
    return {
        "n_images": len(imgs),
        "metadata": metadata,
        "xforms": [{"start": x, "end": x} for x in xforms],
        "render_aabb": {"min": [float(v) for v in amin], "max": [float(v) for v in amax]},
        "up": [0.0, 1.0, 0.0],
        "offset": [float(x) for x in np.asarray(getattr(tb, "_offset", np.zeros(3)), np.float32)],
        "envmap_resolution": [0, 0],
        "scale": float(getattr(tb, "_scale", 1.0)),
        "aabb_scale": int(meta.get("aabb_scale", 1)),
        "from_mitsuba": False,
        "from_na": bool(getattr(tb, "_from_na", False)),
        "is_hdr": False,
        "wants_importance_sampling": True,
    }


def build_snapshot(tb, include_optimizer_state: bool = False) -> dict:
    """The m_network_config object save_snapshot writes (testbed.cu:3144-3178)."""
    if tb._cfg_dict is None:
        raise RuntimeError("save_snapshot: no network loaded (reload_network_from_file first)")
    cfg = copy.deepcopy(tb._cfg_dict)
    cfg.pop("snapshot", None)
    st = tb.stats()
    # m_params_inference: the fp16 EMA weights once training has stepped, the fp16 training weights before
    params = tb.get_half_params(inference=st["training_step"] > 0)
    grid, _ = tb.get_density_grid()
    g, l = tb.get_movement()
    rot = np.zeros(12, np.float32); rot[:9] = g[:, :3].reshape(-1)
    tr = np.zeros(4, np.float32); tr[:3] = g[:, 3]
    ds = dataset_json(tb)
    snap = {
        "n_params": int(params.size),
        "params_binary": _f16_bytes(params),
        "rotation": _f16_bytes(rot),
        "transition": _f16_bytes(tr),
        "local_rotation": _f16_bytes(l[4:12]),
        "local_transition": _f16_bytes(l[0:4]),
        "density_grid_size": NERF_GRIDSIZE,
        "density_grid_binary": _f16_bytes(grid),
        "nerf": {
            "aabb_scale": ds["aabb_scale"],
            "rgb": {
                "rays_per_batch": int(st["rays_per_batch"]),
                "measured_batch_size": int(st["measured_batch_size"]),
                "measured_batch_size_before_compaction": int(st["measured_batch_size_before_compaction"]),
            },
            "dataset": ds,
        },
        "training_step": int(st["training_step"]),
        "loss": float(st["loss"]),
    }
    if include_optimizer_state:
        snap["optimizer"] = optimizer_json(tb.get_optimizer_state())
    cfg["snapshot"] = snap
    return cfg


def optimizer_json(o: dict) -> dict:
    """Ema::serialize { nested: ExponentialDecay::serialize { nested: Adam::serialize, learning_rate,
    learning_rate_factor }, weights_ema_binary } (ema.h:182-187, exponential_decay.h:128-134, adam.h:424-432)."""
    adam = {
        "current_step": int(o["current_step"]),
        "base_learning_rate": float(o["learning_rate"]) * float(o["learning_rate_factor"]),
        "first_moments_binary": np.ascontiguousarray(o["m1"], np.float32).tobytes(),
        "second_moments_binary": np.ascontiguousarray(o["m2"], np.float32).tobytes(),
        "param_steps_binary": np.ascontiguousarray(o["param_steps"], np.uint32).tobytes(),
    }
    return {"nested": {"nested": adam, "learning_rate": float(o["learning_rate"]),
                       "learning_rate_factor": float(o["learning_rate_factor"])},
            "weights_ema_binary": np.ascontiguousarray(o["ema"], np.float16).tobytes()}


def optimizer_state(j: dict) -> dict:
    """The inverse of optimizer_json (Ema / ExponentialDecay / Adam deserialize; param_steps optional)."""
    dec = j["nested"]
    adam = dec["nested"]
    steps = np.frombuffer(bytes(adam["param_steps_binary"]), np.uint32).copy() if "param_steps_binary" in adam else None
    return {"current_step": int(adam["current_step"]), "learning_rate": float(dec["learning_rate"]),
            "learning_rate_factor": float(dec.get("learning_rate_factor", 1.0)),
            "m1": np.frombuffer(bytes(adam["first_moments_binary"]), np.float32).copy(),
            "m2": np.frombuffer(bytes(adam["second_moments_binary"]), np.float32).copy(),
            "param_steps": steps, "ema": np.frombuffer(bytes(j["weights_ema_binary"]), np.float16).copy()}


def pack(cfg: dict) -> bytes:
    return msgpack.packb(cfg, use_bin_type=True)


def unpack(data: bytes) -> dict:
    return msgpack.unpackb(data, raw=False, strict_map_key=False)


def save_snapshot(tb, path: str, include_optimizer_state: bool = False) -> None:
    """Testbed::save_snapshot (testbed.cu:3144-3178)."""
    with open(path, "wb") as f:
        f.write(pack(build_snapshot(tb, include_optimizer_state)))


def read_snapshot(path: str) -> dict:
    """load_network_config (testbed.cu:144-162) for a .msgpack file, with the 'snapshot' check of
    load_snapshot (testbed.cu:3199-3201)."""
    with open(path, "rb") as f:
        cfg = unpack(f.read())
    if not isinstance(cfg, dict) or "snapshot" not in cfg:
        raise RuntimeError(f"File '{path}' does not contain a snapshot.")
    return cfg


def restore_fields(cfg: dict) -> dict:
    """Host-side decode of a snapshot object into the arrays / counters load_snapshot applies."""
    snap = cfg["snapshot"]
    if int(snap["density_grid_size"]) != NERF_GRIDSIZE:
        raise RuntimeError("Incompatible grid size.")
    grid = _f16_array(snap["density_grid_binary"]) if "density_grid_binary" in snap else np.zeros(0, np.float32)
    if grid.size not in (0, NERF_GRIDSIZE ** 3):
        # size 0 = never populated (untrained model); more than one cascade is not built here (testbed.cu:3239-3244)
        raise RuntimeError("Incompatible number of grid cascades.")
    rgb = snap.get("nerf", {}).get("rgb", {})
    out = {
        "network": {k: v for k, v in cfg.items() if k != "snapshot"},
        "params": _f16_array(snap["params_binary"]),
        "n_params": int(snap.get("n_params", 0)),
        "grid": grid,
        "training_step": int(snap["training_step"]),
        "loss": float(snap["loss"]),
        "rays_per_batch": int(rgb.get("rays_per_batch", 1 << 12)),
        "measured_batch_size": int(rgb.get("measured_batch_size", 0)),
        "measured_batch_size_before_compaction": int(rgb.get("measured_batch_size_before_compaction", 0)),
        "global_Rt": None, "local": None,
        "optimizer": optimizer_state(snap["optimizer"]) if "optimizer" in snap else None,
    }
    if "rotation" in snap and "transition" in snap:
        rot, tr = _f16_array(snap["rotation"]), _f16_array(snap["transition"])
        out["global_Rt"] = np.concatenate([rot[:9].reshape(3, 3), tr[:3].reshape(3, 1)], 1)
    if "local_rotation" in snap and "local_transition" in snap:
        out["local"] = np.concatenate([_f16_array(snap["local_transition"])[:4], _f16_array(snap["local_rotation"])[:8]])
    return out


def apply_snapshot(tb, cfg: dict) -> None:
    """Testbed::load_snapshot (testbed.cu:3197-3254) on a loaded config object."""
    from ._lib import C, NeusRestoreState, check, lib

    f = restore_fields(cfg)
    tb.reload_network_from_json(f["network"], batch_size=(tb._net_cfg.batch_size if tb._net_cfg is not None else None))
    n = tb.layout()["n_params"]
    if f["params"].size != n or (f["n_params"] and f["n_params"] != n):
        raise RuntimeError(f"snapshot has {f['params'].size} params, the network from its config has {n}")
    tb.set_params(f["params"])
    if f["grid"].size:
        tb.set_density_grid(f["grid"])
    st = NeusRestoreState()
    st.training_step = f["training_step"]
    st.rays_per_batch = f["rays_per_batch"]
    st.measured_batch_size = f["measured_batch_size"]
    st.measured_batch_size_before_compaction = f["measured_batch_size_before_compaction"]
    st.loss = f["loss"]
    st.rebuild_bitfield = 1 if f["grid"].size else 0
    check(lib().neus_testbed_restore_state(tb.handle, C.byref(st)))
    if f["global_Rt"] is not None or f["local"] is not None:
        tb.set_movement(f["global_Rt"], f["local"])
    if f["optimizer"] is not None:  # Trainer::deserialize -> m_optimizer->deserialize (trainer.h:296-305)
        tb.set_optimizer_state(f["optimizer"])


def load_snapshot(tb, path: str) -> None:
    apply_snapshot(tb, read_snapshot(path))
