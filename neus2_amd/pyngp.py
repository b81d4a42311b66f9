"""Python mirror of the reference's pybind11 `pyngp` module (src/python_api.cu:216-600) for the
NeuS2 training path, implemented over the C-ABI of libneus2_hip.so (include/neus2_hip.h).

Drop-in surface used by the reference drivers (scripts/run.py):
    testbed = pyngp.Testbed(pyngp.TestbedMode.Nerf)
    testbed.load_training_data("transforms.json")
    testbed.reload_network_from_file("configs/nerf/base.json")
    while testbed.frame(): ...   # one Testbed::train step per frame while shall_train
    testbed.training_step, testbed.loss, testbed.ek_loss, testbed.mask_loss

The transforms.json parser restates ngp::load_nerf (src/nerf_loader.cu:197-751) for the
fields the NeuS2 path uses; images are decoded with PIL into RGBA8.
"""
from __future__ import annotations

import ctypes as C
import enum
import glob
import json
import math
import os

import numpy as np

from . import config as _config
from . import _lib
from ._lib import NeusError, NeusImage, NeusNetLayout, NeusTrainStats, check, lib


class TestbedMode(enum.IntEnum):
    Nerf = 0
    Sdf = 1
    Image = 2
    Volume = 3


NERF_SCALE = 0.33  # nerf_loader.h:31


def mesh_vertex_normals(V, F):
    """compute_mesh_1ring (marching_cubes.cu:331-366, 699-705): per vertex, the sum of the (area-weighted)
    normals of its faces, normalised as compute_marching_cubes_mesh does (python_api.cu:115-118)."""
    N = np.zeros_like(V, dtype=np.float32)
    if len(F):
        P = V[F.astype(np.int64)]
        n = np.cross(P[:, 1] - P[:, 0], P[:, 2] - P[:, 0]).astype(np.float32)
        for k in range(3):
            np.add.at(N, F[:, k].astype(np.int64), n)
    ln = np.linalg.norm(N, axis=1, keepdims=True)
    return np.divide(N, ln, out=np.zeros_like(N), where=ln > 0)


def save_mesh(filename, V, N, Cc, F, scale=1.0, offset=(0.0, 0.0, 0.0)):
    """save_mesh (marching_cubes.cu:826-960) for .ply / .obj without texture unwrapping."""
    P = (np.asarray(V, np.float32) - np.asarray(offset, np.float32)) / np.float32(scale)
    F = np.asarray(F, np.int64)
    ext = os.path.splitext(filename)[1].lower()
    with open(filename, "w") as f:
        if ext == ".ply":
            f.write("ply\nformat ascii 1.0\ncomment output from neus2_amd\nelement vertex %d\n"
                    "property float x\nproperty float y\nproperty float z\nproperty float nx\nproperty float ny\nproperty float nz\n"
                    "property uchar red\nproperty uchar green\nproperty uchar blue\nelement face %d\n"
                    "property list uchar int vertex_index\nend_header\n" % (len(P), len(F)))
            c8 = np.clip(np.asarray(Cc, np.float32) * 255.0, 0, 255).astype(np.uint8)
            for p, n, c in zip(P, N, c8):
                f.write("%0.5f %0.5f %0.5f %0.3f %0.3f %0.3f %d %d %d\n" % (p[0], p[1], p[2], n[0], n[1], n[2], c[0], c[1], c[2]))
            for a, b, c in F:
                f.write("3 %d %d %d\n" % (c, b, a))
        else:
            for p, c in zip(P, np.clip(Cc, 0, 1)):
                f.write("v %0.5f %0.5f %0.5f %0.3f %0.3f %0.3f\n" % (p[0], p[1], p[2], c[0], c[1], c[2]))
            for n in N:
                f.write("vn %0.5f %0.5f %0.5f\n" % (n[0], n[1], n[2]))
            for a, b, c in F:
                f.write("f %d//%d %d//%d %d//%d\n" % (c + 1, c + 1, b + 1, b + 1, a + 1, a + 1))


def srgb_to_linear(img):
    """scripts/common.py:136-138"""
    limit = 0.04045
    return np.where(img > limit, np.power((img + 0.055) / 1.055, 2.4), img / 12.92)


def linear_to_srgb(img):
    """scripts/common.py:140-142"""
    limit = 0.0031308
    return np.where(img > limit, 1.055 * (np.maximum(img, 0) ** (1.0 / 2.4)) - 0.055, 12.92 * img)


def mse2psnr(x):
    """scripts/common.py:46"""
    return -10. * np.log(x) / np.log(10.)


def reference_image_linear(rgba8):
    """read_image (common.py:144-158) of an 8-bit RGBA image: sRGB -> linear, alpha premultiplied."""
    img = np.asarray(rgba8, np.float32) / 255.0
    if img.shape[-1] == 4:
        img[..., :3] = srgb_to_linear(img[..., :3]) * img[..., 3:4]
    else:
        img = srgb_to_linear(img)
    return img


def eval_psnr(image, rgba8, background_color=(0.0, 0.0, 0.0, 0.0)):
    """render_img_training_view's metric (render_utils.py:252-359): the reference image composited on
    the background in sRGB space, then PSNR of clip(srgb(pred)) vs clip(srgb(gt)) over rgb."""
    ref = reference_image_linear(rgba8)
    bg = np.asarray(background_color, np.float32)
    if ref.shape[2] == 4:
        a = ref[..., 3:4]
        ref[..., :3] = np.divide(ref[..., :3], a, out=np.zeros_like(ref[..., :3]), where=a != 0)
        ref[..., :3] = linear_to_srgb(ref[..., :3])
        ref[..., :3] *= a
        ref += (1.0 - a) * bg
        ref[..., :3] = srgb_to_linear(ref[..., :3])
    A = np.clip(linear_to_srgb(image[..., :3]), 0.0, 1.0)
    R = np.clip(linear_to_srgb(ref[..., :3]), 0.0, 1.0)
    mse = float(np.mean((A - R) ** 2))
    return mse2psnr(mse), mse


def fov_to_focal_length(resolution, degrees):
    return 0.5 * resolution / math.tan(0.5 * degrees * math.pi / 180.0)


def nerf_matrix_to_ngp(m, scale, offset, from_na):
    """NerfDataset::nerf_matrix_to_ngp (nerf_loader.h:112-134)."""
    r = np.array(m, np.float32)[:3, :4].copy()
    r[:, 1] *= -1
    r[:, 2] *= -1
    r[:, 3] = r[:, 3] * np.float32(scale) + np.asarray(offset, np.float32)
    if from_na:
        r[:, 1] *= -1
        r[:, 2] *= -1
    else:
        r = r[[1, 2, 0], :]
    return r


def load_transforms(path):
    """ngp::load_nerf (nerf_loader.cu:197-751) subset: from_na/scale/offset/aabb_scale, per-frame
    intrinsic_matrix or fl_x/fl_y/camera_angle_x, cx/cy; RGBA PNG images (alpha premultiplied on
    the device by read_rgba)."""
    from PIL import Image
    with open(path) as f:
        js = json.load(f)
    base = os.path.dirname(path)
    scale = float(js.get("scale", NERF_SCALE))
    offset = js.get("offset", [0.5, 0.5, 0.5])
    if not isinstance(offset, list):
        offset = [offset] * 3
    offset = np.array(offset, np.float32)
    from_na = "from_na" in js
    aabb_scale = int(js.get("aabb_scale", 1))
    if "aabb" in js:
        a = np.array(js["aabb"], np.float32)
        length = max(1e-6, float(np.max(np.abs(a[1] - a[0]))))
        scale = 1.0 / length
        offset = (a[1] + a[0]) * 0.5 * -scale + 0.5
    images, focal, principal, xforms = [], [], [], []
    for fr in js["frames"]:
        p = os.path.join(base, fr["file_path"])
        if not os.path.splitext(p)[1]:
            p = p + ".png"
        img = np.asarray(Image.open(p).convert("RGBA"), np.uint8)
        h, w = img.shape[:2]
        pp = np.array([0.5, 0.5], np.float32)
        if "cx" in js:
            pp[0] = float(js["cx"]) / float(js["w"])
        if "cy" in js:
            pp[1] = float(js["cy"]) / float(js["h"])

        def read_fl(res, axis):
            if axis + "_fov" in fr:
                return fov_to_focal_length(res, float(fr[axis + "_fov"]))
            if "fl_" + axis in js:
                return float(js["fl_" + axis])
            if "camera_angle_" + axis in js:
                return fov_to_focal_length(res, float(js["camera_angle_" + axis]) * 180 / math.pi)
            return 0.0

        fx, fy = read_fl(w, "x"), read_fl(h, "y")
        if fx != 0:
            fl = [fx, fy if fy != 0 else fx]
        elif fy != 0:
            fl = [fy, fy]
        elif "intrinsic_matrix" in fr:
            K = fr["intrinsic_matrix"]
            fl = [float(K[0][0]), float(K[1][1])]
            pp = np.array([float(K[0][2]) / float(js["w"]), float(K[1][2]) / float(js["h"])], np.float32)
        else:
            raise RuntimeError("Couldn't read fov.")
        m = fr.get("transform_matrix_start", fr.get("transform_matrix"))
        xforms.append(nerf_matrix_to_ngp(m, scale, offset, from_na))
        images.append(img)
        focal.append(fl)
        principal.append(pp)
    return dict(images=images, focal=np.array(focal, np.float32), principal=np.array(principal, np.float32),
                xforms=np.stack(xforms).astype(np.float32), aabb_scale=aabb_scale, scale=scale, offset=offset)


def geometric_init_weights(n_levels, width=64, seed=1337, path_hint=True):
    """Density-MLP geometric initialisation (my_tcnn/scripts/geometry_init_save_weights.py:291-331).
    The reference loads utils/mlp_weights*.txt (nerf_network.h:787-813); that file is used when present,
    otherwise the same recipe is generated deterministically: W0[:, :3] ~ N(0, sqrt(2)/sqrt(W)),
    W0[:, 3:] = 0, W1 ~ N(sqrt(pi)/sqrt(W), 1e-5)."""
    din = _config.density_input_width(n_levels)
    if path_hint:
        fname = {32: "utils/mlp_weights_hidden_layer_num_1_hidden_size_32.txt", 48: "utils/mlp_weights.txt"}.get(din)
        if fname and os.path.exists(fname):
            return np.loadtxt(fname, dtype=np.float32)[: width * din + 16 * width]
    rng = np.random.default_rng(seed)
    w0 = np.zeros((width, din), np.float32)
    w0[:, :3] = rng.normal(0.0, math.sqrt(2) / math.sqrt(width), size=(width, 3))
    w1 = rng.normal(math.sqrt(math.pi) / math.sqrt(width), 1e-5, size=(16, width)).astype(np.float32)
    return np.concatenate([w0.reshape(-1), w1.reshape(-1)]).astype(np.float32)


def _images_array(imgs, focal, principal, xforms):
    """NeusImage records over host RGBA8 arrays (the arrays must outlive the C call)."""
    arr = (NeusImage * len(imgs))()
    for i, im in enumerate(imgs):
        arr[i].width = im.shape[1]
        arr[i].height = im.shape[0]
        arr[i].rgba8 = im.ctypes.data
        arr[i].focal[:] = [float(v) for v in np.asarray(focal[i]).reshape(2)]
        arr[i].principal[:] = [float(v) for v in np.asarray(principal[i]).reshape(2)]
        arr[i].xform[:] = [float(v) for v in np.asarray(xforms[i], np.float32).reshape(12)]
    return arr


class _Training:
    def __init__(self, tb):
        self._tb = tb

    @property
    def n_images_for_training(self):
        return self._tb._n_images

    @property
    def counters_rgb(self):
        return self._tb.stats()


class _Nerf:
    def __init__(self, tb):
        self.training = _Training(tb)
        self.rendering_min_transmittance = 0.01  # testbed.h: Nerf::rendering_min_transmittance


# neus_testbed_kernel_times order (include/neus2_hip.h NEUS_N_PHASES)
PHASES = ["occupancy", "sample", "inference", "loss", "train_encode", "mlp_train", "wgrad", "grid_scatter", "allreduce",
          "optimizer"]


class Testbed:
    """pyngp.Testbed (python_api.cu:216-600), NeuS2 training subset."""

    def __init__(self, mode: TestbedMode = TestbedMode.Nerf, device: int = 0):
        if mode != TestbedMode.Nerf:
            raise NeusError("only TestbedMode.Nerf (NeuS2) is implemented on the gfx950 path")
        h = C.c_void_p()
        check(lib().neus_testbed_create(C.c_int(device), C.byref(h)))
        self._h = h
        self._n_images = 0
        self._images = None
        self._net_cfg = None
        self._cfg_dict = None
        self.shall_train = True
        self.nerf = _Nerf(self)
        # render state (testbed.h: m_snap_to_pixel_centers, m_background_color, camera)
        self.snap_to_pixel_centers = False
        self.background_color = [0.0, 0.0, 0.0, 0.0]
        self._render_view = None
        self.max_training_steps = None

    def __del__(self):
        try:
            if getattr(self, "_h", None):
                lib().neus_testbed_destroy(self._h)
                self._h = None
        except Exception:
            pass

    # ------------------------------------------------------------------ data
    def load_training_data(self, path: str):
        """Testbed::load_training_data (testbed.cu:93) -> load_nerf (testbed_nerf.cu:2964):
        a transforms.json file, or a directory whose sorted *.json files are frames (first used)."""
        if os.path.isdir(path):
            files = sorted(f for f in glob.glob(os.path.join(path, "*.json")) if "downsample" not in os.path.basename(f))
            if not files:
                raise NeusError(f"no json files in {path}")
        else:
            files = [path]
        d = load_transforms(files[0])
        self.set_dataset(d["images"], d["focal"], d["principal"], d["xforms"], d["aabb_scale"])
        self._scale, self._offset = float(d["scale"]), np.asarray(d["offset"], np.float32)
        self._frames = files  # all_json_paths (testbed_nerf.cu:2967-2994): one transforms file per time frame

    def set_dataset_frames(self, frames):
        """A dynamic sequence given in memory: a list of dicts (images, focal, principal, xforms[, aabb_scale]),
        one per time frame; frame 0 is loaded (the in-memory twin of a directory of per-frame json files)."""
        f0 = frames[0]
        self.set_dataset(f0["images"], f0["focal"], f0["principal"], f0["xforms"], f0.get("aabb_scale", 1))
        self._frames = list(frames)

    # ------------------------------------------------------------------ dynamic scenes
    @property
    def all_training_time_frame(self):
        return len(getattr(self, "_frames", None) or [None])

    @property
    def current_training_time_frame(self):
        return self.frame_state()["frame"]

    def _hyper(self, key, default):
        return (self._cfg_dict or {}).get("hyperparams", {}).get(key, default)

    @property
    def first_frame_max_training_step(self):
        return int(self._hyper("first_frame_max_training_step", 2000))

    @property
    def next_frame_max_training_step(self):
        return int(self._hyper("next_frame_max_training_step", 1000))

    def frame_state(self):
        o = (C.c_uint32 * 4)()
        check(lib().neus_testbed_frame_state(self._h, o))
        return {"frame": o[0], "canonical_step": o[1], "train_canonical": bool(o[2]), "train_delta": bool(o[3])}

    def training_network_next_frame(self):
        """Testbed::training_network_next_frame (testbed.cu:2001-2082): False on the last frame, else loads the next
        frame (load_nerf(frame), testbed_nerf.cu:3096-3113) and restarts training on it with the global-movement
        phase first."""
        k = self.current_training_time_frame
        if k >= self.all_training_time_frame - 1:
            return False
        nxt = self._frames[k + 1]
        d = load_transforms(nxt) if isinstance(nxt, str) else nxt
        imgs = [np.ascontiguousarray(im, np.uint8) for im in d["images"]]
        arr = _images_array(imgs, d["focal"], d["principal"], d["xforms"])
        check(lib().neus_testbed_next_frame(self._h, C.c_uint32(len(imgs)), arr))
        self._images = imgs
        self._n_images = len(imgs)
        return True

    def get_movement(self):
        """(accumulated 3x4 [R | t] of the rays, DeltaNetwork params transition[4] | rotation 6D[8])."""
        g, l = (C.c_float * 12)(), (C.c_float * 12)()
        check(lib().neus_testbed_get_movement(self._h, g, l))
        g = np.array(g, np.float32)
        return np.concatenate([g[:9].reshape(3, 3), g[9:].reshape(3, 1)], 1), np.array(l, np.float32)

    def set_movement(self, global_Rt=None, local=None):
        g = None if global_Rt is None else np.concatenate([np.asarray(global_Rt, np.float32)[:, :3].reshape(-1),
                                                          np.asarray(global_Rt, np.float32)[:, 3]]).astype(np.float32)
        l = None if local is None else np.ascontiguousarray(local, np.float32)
        check(lib().neus_testbed_set_movement(self._h, C.c_void_p(g.ctypes.data) if g is not None else None,
                                              C.c_void_p(l.ctypes.data) if l is not None else None))

    def set_dataset(self, images, focal, principal, xforms, aabb_scale=1):
        imgs = [np.ascontiguousarray(im, np.uint8) for im in images]
        arr = _images_array(imgs, focal, principal, xforms)
        self._frames = None
        check(lib().neus_testbed_set_dataset(self._h, C.c_uint32(len(imgs)), arr, C.c_float(aabb_scale)))
        self._images = imgs
        self._n_images = len(imgs)
        self._dataset_meta = {"xforms": list(xforms), "focal": list(focal), "principal": list(principal),
                              "aabb_scale": float(aabb_scale)}
        s = int(aabb_scale)
        infl = 0.5 * min(1 << 7, s)
        self._aabb = (np.full(3, 0.5 - infl, np.float32), np.full(3, 0.5 + infl, np.float32))
        self._scale, self._offset = 1.0, np.zeros(3, np.float32)

    # ------------------------------------------------------------------ network
    def reload_network_from_file(self, path: str = "", batch_size=None, fixed_rays_per_batch=0):
        """Testbed::reload_network_from_file (testbed.cu:164) -> reset_network (testbed.cu:2084)."""
        cfg = _config.load_json(path)
        self.reload_network_from_json(cfg, batch_size=batch_size, fixed_rays_per_batch=fixed_rays_per_batch)

    def reload_network_from_json(self, cfg, batch_size=None, fixed_rays_per_batch=0, geometric_init=None):
        if isinstance(cfg, str):
            cfg = _config.parse_json_text(cfg)
        c = _config.network_config(cfg, batch_size=batch_size, fixed_rays_per_batch=fixed_rays_per_batch)
        geo = geometric_init if geometric_init is not None else geometric_init_weights(c.n_levels, c.n_neurons)
        geo = np.ascontiguousarray(geo, np.float32)
        check(lib().neus_testbed_reload_network(self._h, C.byref(c), C.c_void_p(geo.ctypes.data)))
        c.per_level_scale = self.layout()["per_level_scale"]
        self._net_cfg = c
        self._cfg_dict = cfg
        self._geo = geo

    def save_snapshot(self, path: str, include_optimizer_state: bool = False):
        """Testbed::save_snapshot (testbed.cu:3144-3178; python_api.cu:370): msgpack network config + snapshot."""
        from . import snapshot
        snapshot.save_snapshot(self, path, include_optimizer_state)

    def load_snapshot(self, path: str):
        """Testbed::load_snapshot (testbed.cu:3197-3254; python_api.cu:371). Needs a dataset loaded first
        (the reference's snapshot-only render path, load_nerf from the stored metadata, is not built)."""
        from . import snapshot
        if not self._n_images:
            raise NeusError("load_snapshot: load the training data first (set_dataset / load_training_data)")
        snapshot.load_snapshot(self, path)

    def layout(self):
        l = NeusNetLayout()
        check(lib().neus_testbed_layout(self._h, C.byref(l)))
        return {k: getattr(l, k) for k, _ in l._fields_}

    # ------------------------------------------------------------------ training
    def frame(self):
        """Testbed::frame (testbed.cu:1722-1783) without GUI or rendering: one training step
        (train_and_render -> train(m_training_batch_size)) while shall_train; a static scene stops
        at hyperparams.first_frame_max_training_step (testbed.cu:1752-1758). Returns False when done."""
        if not self.shall_train:
            return False
        if self.max_training_steps is not None:
            if self.training_step >= int(self.max_training_steps):
                self.shall_train = False
                return False
        elif self._cfg_dict is not None:
            # testbed.cu:1749-1756: a frame's step budget reached -> next frame (or stop after the last one)
            k = self.current_training_time_frame
            limit = self.first_frame_max_training_step if k == 0 else self.next_frame_max_training_step
            if self.training_step >= limit and not self.training_network_next_frame():
                self.shall_train = False
                return False
        self.train_steps(1)
        return True

    # ------------------------------------------------------------------ rendering
    def set_camera_to_training_view(self, view: int):
        """Testbed::set_camera_to_training_view (testbed.cu:264-270): camera, focal length and screen
        centre of training image `view`."""
        if not 0 <= int(view) < self._n_images:
            raise NeusError(f"training view {view} out of range (0..{self._n_images - 1})")
        self._render_view = int(view)

    def reset_camera(self):
        """Testbed::reset_camera (testbed.cu:272-285); only the training-view camera is supported for
        rendering, so this clears it."""
        self._render_view = None

    def render(self, width: int = 1920, height: int = 1080, spp: int = 1, linear: bool = True, use_ema: bool = True):
        """Testbed::render_to_cpu (python_api.cu:123-169) for the NeuS Shade mode: `spp` frames of
        NerfTracer::trace accumulated in linear colour, returned as float32 [height, width, 4] with
        premultiplied alpha. The background colour is composited as tonemap_kernel
        (render_buffer.cu:474-500) does; linear=False returns sRGB."""
        if self._render_view is None:
            raise NeusError("render: call set_camera_to_training_view(view) first")
        rq = _lib.NeusRenderRequest()
        rq.width, rq.height, rq.spp = int(width), int(height), int(spp)
        rq.training_view = self._render_view
        rq.snap_to_pixel_centers = int(bool(self.snap_to_pixel_centers))
        rq.min_transmittance = float(self.nerf.rendering_min_transmittance)
        rq.use_ema = int(bool(use_ema))
        out = np.empty((int(height), int(width), 4), np.float32)
        it = C.c_uint32()
        check(lib().neus_testbed_render(self._h, C.byref(rq), C.c_void_p(out.ctypes.data), C.byref(it)))
        self.last_render_iterations = it.value
        bg = np.asarray(self.background_color, np.float32)
        if bg[3] != 0:
            bgl = np.where(bg[:3] <= 0.04045, bg[:3] / 12.92, ((bg[:3] + 0.055) / 1.055) ** 2.4)
            out[..., :3] += bgl * (1 - out[..., 3:4]) * bg[3]
        if not linear:
            out[..., :3] = linear_to_srgb(out[..., :3])
        return out

    # ------------------------------------------------------------------ meshes
    def compute_marching_cubes_mesh(self, resolution=(256, 256, 256), aabb=None, thresh=None, density_grid=None):
        """Testbed::compute_marching_cubes_mesh (python_api.cu:99-121): dict V (vertices), N (normalised
        1-ring normals), C (vertex colours), F (faces). `aabb` = (min, max); None = the render aabb.
        thresh None = m_mesh.thresh = 0 (the SDF level set). `density_grid` (torch cuda tensor of
        res[2] x res[1] x res[0] floats) skips the network and meshes that grid as given."""
        res = (C.c_int32 * 3)(*[int(r) for r in np.broadcast_to(np.asarray(resolution), 3)])
        amin, amax = self._aabb if aabb is None else (np.asarray(aabb[0], np.float32), np.asarray(aabb[1], np.float32))
        cmin, cmax = (C.c_float * 3)(*map(float, amin)), (C.c_float * 3)(*map(float, amax))
        thresh = 0.0 if thresh is None else float(thresh)
        nv, nt = C.c_uint32(), C.c_uint32()
        dptr = C.c_void_p(density_grid.data_ptr()) if density_grid is not None else None
        check(lib().neus_testbed_marching_cubes(self._h, res, cmin, cmax, C.c_float(thresh), dptr, C.byref(nv), C.byref(nt)))
        V = np.zeros((nv.value, 3), np.float32)
        F = np.zeros((nt.value, 3), np.uint32)
        check(lib().neus_testbed_get_mesh(self._h, C.c_void_p(V.ctypes.data), C.c_void_p(F.ctypes.data)))
        N = mesh_vertex_normals(V, F)
        Cc = np.zeros_like(V)
        if density_grid is None and nv.value:
            check(lib().neus_testbed_mesh_vertex_colors(self._h, C.c_void_p(Cc.ctypes.data)))
        return {"V": V, "N": N, "C": Cc, "F": F.astype(np.int32)}

    def get_sdf_on_grid(self, resolution, aabb=None):
        """Testbed::get_density_on_grid (testbed_nerf.cu:4096-4139) for NeuS: raw SDF of the inference (EMA)
        weights at x / res * (aabb.max - aabb.min) + aabb.min; float32 [res_z, res_y, res_x]."""
        r = [int(v) for v in np.broadcast_to(np.asarray(resolution), 3)]
        res = (C.c_int32 * 3)(*r)
        amin, amax = self._aabb if aabb is None else (np.asarray(aabb[0], np.float32), np.asarray(aabb[1], np.float32))
        cmin, cmax = (C.c_float * 3)(*map(float, amin)), (C.c_float * 3)(*map(float, amax))
        out = np.zeros((r[2], r[1], r[0]), np.float32)
        check(lib().neus_testbed_sdf_on_grid(self._h, res, cmin, cmax, C.c_void_p(out.ctypes.data)))
        return out

    def compute_and_save_marching_cubes_mesh(self, filename, resolution=(256, 256, 256), aabb=None, thresh=None, unwrap_it=False):
        """Testbed::compute_and_save_marching_cubes_mesh (testbed.cu:308-317) -> save_mesh
        (marching_cubes.cu:826-960): .ply (ascii, with normals and 8-bit colours) or .obj, vertices mapped back
        to the dataset's coordinates as (v - offset) / scale."""
        if unwrap_it:
            raise NeusError("unwrap_it (texture atlas export) is not supported")
        m = self.compute_marching_cubes_mesh(resolution, aabb, thresh)
        save_mesh(filename, m["V"], m["N"], m["C"], m["F"], self._scale, self._offset)
        return m

    def train(self, batch_size: int | None = None):
        """Testbed::train(batch_size) (testbed.cu:2640-2736): ONE training step targeting `batch_size`
        compacted samples. The device workspace is sized at reload_network_* time for the configured
        batch; a different batch_size raises (call reload_network_from_json with batch_size=...)."""
        if batch_size is not None and self._net_cfg is not None and int(batch_size) != int(self._net_cfg.batch_size):
            raise NeusError(f"train({batch_size}): the network was configured for batch_size={self._net_cfg.batch_size}")
        self.train_steps(1)

    def train_steps(self, n_steps: int = 1):
        """n consecutive Testbed::train steps in one call (no host synchronisation in between)."""
        check(lib().neus_testbed_train(self._h, C.c_uint32(n_steps)))

    def stats(self):
        s = NeusTrainStats()
        check(lib().neus_testbed_get_stats(self._h, C.byref(s)))
        return {k: getattr(s, k) for k, _ in s._fields_}

    @property
    def training_step(self):
        return self.stats()["training_step"]

    @property
    def loss(self):
        return self.stats()["loss"]

    @property
    def ek_loss(self):
        return self.stats()["ek_loss"]

    @property
    def mask_loss(self):
        return self.stats()["mask_loss"]

    def set_profiling(self, on=True):
        check(lib().neus_testbed_set_profiling(self._h, C.c_int(1 if on else 0)))

    def time_kernel(self, kernel, iters=5):
        """(mean ms per launch, work units per launch) of one hot-path kernel replayed on the current
        training state (neus_testbed_time_kernel; ids in include/neus2_hip.h)."""
        ms = C.c_float()
        units = C.c_uint32()
        check(lib().neus_testbed_time_kernel(self._h, C.c_int(kernel), C.c_int(iters), C.byref(ms), C.byref(units)))
        return float(ms.value), int(units.value)

    def phase_times(self):
        """Mean ms per profiled step for each of PHASES, plus (n_steps, mean Npre, mean Ntrain)."""
        n = len(PHASES)
        a = (C.c_float * (n + 3))()
        check(lib().neus_testbed_kernel_times(self._h, a))
        return dict(zip(PHASES, list(a)[:n])), dict(steps=int(a[n]), npre=float(a[n + 1]), ntrain=float(a[n + 2]))

    # ------------------------------------------------------------------ state access
    def get_params(self):
        n = self.layout()["n_params"]
        out = np.zeros(n, np.float32)
        check(lib().neus_testbed_get_params(self._h, C.c_void_p(out.ctypes.data), C.c_uint64(n)))
        return out

    def set_params(self, p):
        p = np.ascontiguousarray(p, np.float32)
        check(lib().neus_testbed_set_params(self._h, C.c_void_p(p.ctypes.data), C.c_uint64(p.size)))

    def get_gradients(self):
        n = self.layout()["n_params"]
        out = np.zeros(n, np.float32)
        check(lib().neus_testbed_get_gradients(self._h, C.c_void_p(out.ctypes.data), C.c_uint64(n)))
        return out

    def get_ema_params(self):
        n = self.layout()["n_params"]
        out = np.zeros(n, np.float32)
        check(lib().neus_testbed_get_ema_params(self._h, C.c_void_p(out.ctypes.data), C.c_uint64(n)))
        return out

    def get_half_params(self, inference: bool = False):
        """The fp16 parameter copy the kernels read: training weights, or the inference (EMA) weights."""
        n = self.layout()["n_params"]
        out = np.zeros(n, np.uint16)
        check(lib().neus_testbed_get_half_params(self._h, C.c_int(1 if inference else 0), C.c_void_p(out.ctypes.data), C.c_uint64(n)))
        return out.view(np.float16)

    def get_density_grid(self):
        g = np.zeros(128 ** 3, np.float32)
        bf = np.zeros(128 ** 3 // 8 * 8, np.uint8)
        check(lib().neus_testbed_get_density_grid(self._h, C.c_void_p(g.ctypes.data), C.c_void_p(bf.ctypes.data)))
        return g, bf

    def set_density_grid(self, grid=None, bitfield=None):
        g = None if grid is None else np.ascontiguousarray(grid, np.float32)
        b = None if bitfield is None else np.ascontiguousarray(bitfield, np.uint8)
        check(lib().neus_testbed_set_density_grid(self._h, C.c_void_p(g.ctypes.data if g is not None else 0),
                                                  C.c_void_p(b.ctypes.data if b is not None else 0)))

    def get_rng(self):
        o = (C.c_uint64 * 4)()
        check(lib().neus_testbed_get_rng(self._h, o))
        return list(o)

    def ray_counts(self, n=None):
        """(requested samples, composited samples, compacted samples) per ray of the last step."""
        n = int(self.stats()["rays_per_batch"] if n is None else n)
        a, b, c = np.zeros(n, np.uint32), np.zeros(n, np.uint32), np.zeros(2 * n, np.uint32)
        check(lib().neus_testbed_ray_counts(self._h, C.c_uint32(n), C.c_void_p(a.ctypes.data), C.c_void_p(b.ctypes.data),
                                            C.c_void_p(c.ctypes.data)))
        return a, b, c.reshape(n, 2)[:, 0].copy()

    def synchronize(self):
        check(lib().neus_testbed_synchronize(self._h))

    def init_data_parallel(self, rank, world, unique_id: bytes):
        buf = (C.c_uint8 * 128).from_buffer_copy(unique_id)
        check(lib().neus_testbed_init_data_parallel(self._h, C.c_int(rank), C.c_int(world), buf))

    @property
    def handle(self):
        return self._h


class LocalGroup:
    """In-process data-parallel group (neus_local_group_create): `world` testbeds, each trained from its own host
    thread, exchange through host staging with the RCCL path's collectives (several ranks on one device)."""

    def __init__(self, world: int):
        self._h = C.c_void_p()
        check(lib().neus_local_group_create(C.c_int(world), C.byref(self._h)))
        self.world = world

    def join(self, tb, rank: int):
        check(lib().neus_testbed_init_local_group(tb.handle, self._h, C.c_int(rank)))

    def __del__(self):
        if getattr(self, "_h", None):
            lib().neus_local_group_destroy(self._h)
            self._h = None


def nccl_unique_id() -> bytes:
    buf = (C.c_uint8 * 128)()
    check(lib().neus_nccl_unique_id(buf))
    return bytes(buf)
