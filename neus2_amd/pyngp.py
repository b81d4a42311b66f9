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


class ColorSpace(enum.IntEnum):
    """EColorSpace (common.h; python_api.cu:278-281)."""
    Linear = 0
    SRGB = 1


class TonemapCurve(enum.IntEnum):
    """ETonemapCurve (common.h; python_api.cu:283-288)."""
    Identity = 0
    ACES = 1
    Hable = 2
    Reinhard = 3


class BoundingBox:
    """ngp::BoundingBox (bounding_box.cuh; python_api.cu:296-315): min / max corners; the default box is inside-out
    (empty), which compute_*marching_cubes_mesh read as "use the render aabb"."""

    def __init__(self, min=None, max=None):  # noqa: A002 - the reference's argument names
        self.min = np.full(3, np.inf, np.float32) if min is None else np.asarray(min, np.float32).reshape(3).copy()
        self.max = np.full(3, -np.inf, np.float32) if max is None else np.asarray(max, np.float32).reshape(3).copy()

    def is_empty(self):
        return bool(np.any(self.max < self.min))

    def center(self):
        return 0.5 * (self.max + self.min)

    def diag(self):
        return self.max - self.min

    def contains(self, p):
        p = np.asarray(p, np.float32)
        return bool(np.all(p >= self.min) and np.all(p <= self.max))

    def inflate(self, amount):
        self.min -= np.float32(amount)
        self.max += np.float32(amount)

    def enlarge(self, other):
        if isinstance(other, BoundingBox):
            self.min = np.minimum(self.min, other.min)
            self.max = np.maximum(self.max, other.max)
        else:
            p = np.asarray(other, np.float32)
            self.min = np.minimum(self.min, p)
            self.max = np.maximum(self.max, p)

    def intersection(self, other):
        return BoundingBox(np.maximum(self.min, other.min), np.minimum(self.max, other.max))

    def intersects(self, other):
        return not self.intersection(other).is_empty()

    def get_vertices(self):
        return np.array([[(self.max if i & 1 else self.min)[0], (self.max if i & 2 else self.min)[1],
                          (self.max if i & 4 else self.min)[2]] for i in range(8)], np.float32)

    def __repr__(self):
        return f"BoundingBox(min={self.min.tolist()}, max={self.max.tolist()})"


def _aabb_pair(aabb):
    """None, an empty BoundingBox -> None (the render aabb); a BoundingBox or (min, max) -> float32 corners."""
    if aabb is None:
        return None
    if isinstance(aabb, BoundingBox):
        return None if aabb.is_empty() else (aabb.min.copy(), aabb.max.copy())
    return np.asarray(aabb[0], np.float32), np.asarray(aabb[1], np.float32)


def tonemap_curve(x, curve):
    """tonemap(Array3f, ETonemapCurve) (render_buffer.cu:254-312), float32."""
    x = np.asarray(x, np.float32)
    curve = TonemapCurve(curve)
    if curve == TonemapCurve.Identity:
        return x
    x = np.maximum(x, np.float32(0))
    f = np.float32
    if curve == TonemapCurve.ACES:
        k0, k1, k2, k3, k4, k5 = f(0.6) * f(0.6) * f(2.51), f(0.6) * f(0.03), f(0), f(0.6) * f(0.6) * f(2.43), f(0.6) * f(0.59), f(0.14)
    elif curve == TonemapCurve.Hable:
        A, B, Cc, D, E, F = f(0.15), f(0.50), f(0.10), f(0.20), f(0.02), f(0.30)
        k0, k1, k2, k3, k4, k5 = A * F - A * E, Cc * B * F - B * E, f(0), A * F, B * F, D * F * F
        W = f(11.2)
        white_scale = (k3 * (W * W) + k4 * W + k5) / (k0 * (W * W) + k1 * W + k2)
        k0, k1, k2, k3, k4 = f(4) * k0 * white_scale, f(2) * k1 * white_scale, k2 * white_scale, f(4) * k3, f(2) * k4
    else:  # Reinhard
        Y = x[..., 0:1] * f(0.2126) + x[..., 1:2] * f(0.7152) + x[..., 2:3] * f(0.0722)
        return (x * (f(1) / (Y + f(1)))).astype(np.float32)
    sq = x * x
    return ((sq * k0 + k1 * x + k2) / (k3 * sq + k4 * x + k5)).astype(np.float32)


def tonemap_image(rgba, exposure=0.0, background_color=(0.0, 0.0, 0.0, 0.0), color_space=ColorSpace.Linear,
                  curve=TonemapCurve.Identity, to_srgb=False):
    """tonemap_kernel (render_buffer.cu:474-500) on the linear accumulation buffer (H x W x 4, float32): the sRGB
    background composited behind it (converted to linear unless the colour space is SRGB; alpha += weight), then
    tonemap(col, exposure, curve, color_space, output) (render_buffer.cu:314-334): SRGB colour space -> linear,
    x 2^exposure, the curve, linear -> sRGB when to_srgb (render(linear=False)). No clamp (no DLSS)."""
    out = np.array(rgba, np.float32, copy=True)
    bg = np.asarray(background_color, np.float32).reshape(4).copy()
    if ColorSpace(color_space) != ColorSpace.SRGB:
        bg[:3] = srgb_to_linear(bg[:3]).astype(np.float32)
    weight = (np.float32(1) - out[..., 3:4]) * bg[3]
    out[..., :3] += bg[:3] * weight
    out[..., 3:4] += weight
    col = out[..., :3]
    if ColorSpace(color_space) == ColorSpace.SRGB:
        col = srgb_to_linear(col).astype(np.float32)
    col = col * np.float32(2.0) ** np.float32(exposure)
    col = tonemap_curve(col, curve)
    if to_srgb:
        col = linear_to_srgb(col).astype(np.float32)
    out[..., :3] = col
    return out


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


def ngp_matrix_to_nerf(m, scale, offset, from_na):
    """NerfDataset::ngp_matrix_to_nerf (nerf_loader.h:135-155): the inverse of nerf_matrix_to_ngp."""
    r = np.array(m, np.float32)[:3, :4].copy()
    if from_na:
        r[:, 1] *= -1
        r[:, 2] *= -1
    else:
        r = r[[2, 0, 1], :]
    r[:, 1] *= -1
    r[:, 2] *= -1
    r[:, 3] = (r[:, 3] - np.asarray(offset, np.float32)) / np.float32(scale)
    return r


def prepare_image(img, alpha=None, mask=None, white_transparent=False, black_transparent=False):
    """ngp::load_nerf's training-image preparation (neus_prepare_image_rgba8): alpha image, dynamic mask (hot-pink
    key), white / black transparency. Returns (prepared h x w x 4 uint8 copy, mask colour key or 0)."""
    out = np.ascontiguousarray(img, np.uint8).copy()
    h, w = out.shape[:2]
    a = None if alpha is None else np.ascontiguousarray(alpha, np.uint8)
    m = None if mask is None else np.ascontiguousarray(mask, np.uint8)
    for x in (a, m):
        if x is not None and x.shape[:2] != (h, w):
            raise RuntimeError("prepare_image: alpha / mask resolution differs from the image")
    key = C.c_uint32(0)
    flags = (1 if white_transparent else 0) | (2 if black_transparent else 0)
    check(lib().neus_prepare_image_rgba8(C.c_void_p(out.ctypes.data), C.c_uint32(w), C.c_uint32(h),
                                         C.c_void_p(a.ctypes.data) if a is not None else None,
                                         C.c_void_p(m.ctypes.data) if m is not None else None, C.c_uint32(flags), C.byref(key)))
    return out, int(key.value)


def load_transforms(path):
    """ngp::load_nerf (nerf_loader.cu:197-751) subset: from_na/scale/offset/aabb_scale, per-frame
    intrinsic_matrix or fl_x/fl_y/camera_angle_x, cx/cy; RGBA PNG images (alpha premultiplied on
    the device by read_rgba), with the reference's image preparation (neus_prepare_image_rgba8): separate alpha
    images, dynamic masks (the hot-pink key) and white_transparent / black_transparent."""
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
    white_t, black_t = bool(js.get("white_transparent", False)), bool(js.get("black_transparent", False))
    flags = white_t or black_t
    # depth maps (nerf_loader.cu:321-393, 599-612): frames' `depth_path` 16-bit images, loaded when the dataset sets
    # `integer_depth_scale` > 0 and `enable_depth_loading` is not false; metres = value x integer_depth_scale x scale
    # (set_training_image(..., depth_scale * result.scale), copy_depth :91-99)
    enable_depth = bool(js.get("enable_depth_loading", True))
    int_depth_scale = float(js.get("integer_depth_scale", -1.0))
    images, focal, principal, xforms, mask_colors, depths = [], [], [], [], [], []
    for fr in js["frames"]:
        fp = fr["file_path"]
        p = os.path.join(base, fp)
        name = os.path.basename(p)
        if "." not in name:  # path.extension() == "" -> png (exr is not supported here)
            p = p + ".png"
            name += ".png"
            if not os.path.exists(p):
                raise RuntimeError("Could not find image file: " + p)
        ext = name[name.rfind(".") + 1:]
        img = np.ascontiguousarray(np.asarray(Image.open(p).convert("RGBA"), np.uint8)).copy()
        h, w = img.shape[:2]
        # alpha image `<file_path>.alpha.<ext>` and dynamic mask `dynamic_mask_<basename>.png` (nerf_loader.cu:550-590)
        alpha = mask = None
        apath = os.path.join(base, fp + ".alpha." + ext)
        if os.path.exists(apath):
            alpha = np.ascontiguousarray(np.asarray(Image.open(apath).convert("RGBA"), np.uint8))
            if alpha.shape[:2] != (h, w):
                raise RuntimeError("Alpha image has wrong resolution: " + apath)
        mpath = os.path.join(os.path.dirname(p), "dynamic_mask_" + name[: name.rfind(".")] + ".png")
        if os.path.exists(mpath):
            mask = np.ascontiguousarray(np.asarray(Image.open(mpath).convert("RGBA"), np.uint8))
            if mask.shape[:2] != (h, w):
                raise RuntimeError("Mask image has wrong resolution: " + mpath)
        key = 0
        if alpha is not None or mask is not None or flags:
            img, key = prepare_image(img, alpha, mask, white_t, black_t)
        mask_colors.append(key)
        depth = None
        if enable_depth and int_depth_scale > 0 and "depth_path" in fr:
            dpath = os.path.join(base, str(fr["depth_path"]))
            if os.path.exists(dpath):
                d16 = read_depth_u16(dpath)
                if d16.shape != (h, w):
                    raise RuntimeError("Depth image has wrong resolution: " + dpath)
                depth = (d16.astype(np.float32) * np.float32(int_depth_scale * scale)).astype(np.float32)
        depths.append(depth)
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
                xforms=np.stack(xforms).astype(np.float32), aabb_scale=aabb_scale, scale=scale, offset=offset, from_na=from_na,
                mask_colors=mask_colors, white_transparent=white_t, black_transparent=black_t, depths=depths)


def read_depth_u16(path):
    """stbi_load_16(path, ..., 1) as nerf_loader.cu:603 calls it: one 16-bit channel; 8-bit images are widened by
    x 257, colour images reduced to stbi's luma (77 r + 150 g + 29 b) >> 8 (stbi__compute_y_16)."""
    from PIL import Image
    im = Image.open(path)
    if im.mode in ("I;16", "I;16B", "I;16L", "I"):
        a = np.asarray(im).astype(np.int64)
        if a.ndim == 3:
            a = a[..., 0]
        return np.clip(a, 0, 65535).astype(np.uint16)
    if im.mode in ("L", "P", "1"):
        return (np.asarray(im.convert("L"), np.uint16) * 257).astype(np.uint16)
    rgb = np.asarray(im.convert("RGB"), np.uint32) * 257
    return ((rgb[..., 0] * 77 + rgb[..., 1] * 150 + rgb[..., 2] * 29) >> 8).astype(np.uint16)


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


def _opt_property(field, conv=float):
    """A Testbed::Nerf(::Training) member that lives in the device dataset (NeusTrainingOptions)."""

    def get(self):
        return conv(getattr(self._tb._get_options(), field))

    def put(self, v):
        o = self._tb._get_options()
        setattr(o, field, conv(v))
        self._tb._set_options(o)

    return property(get, put)


class _Dataset:
    """Testbed::Nerf::Training::dataset (NerfDataset, python_api.cu:517-531), read-only view."""

    def __init__(self, tb):
        self._tb = tb

    @property
    def n_images(self):
        return self._tb._n_images

    @property
    def scale(self):
        return float(self._tb._scale)

    @property
    def offset(self):
        return np.asarray(self._tb._offset, np.float32).copy()

    @property
    def aabb_scale(self):
        return int((self._tb._dataset_meta or {}).get("aabb_scale", 1))

    @property
    def from_na(self):
        return bool(self._tb._from_na)

    @property
    def render_aabb(self):
        return BoundingBox(*self._tb._aabb)

    @property
    def has_depth(self):
        return any(d is not None for d in (getattr(self._tb, "_depths", None) or []))

    def depth(self, image):
        """The depth map of a training image (scene units) or None."""
        return self._tb._depths[image]

    @property
    def transforms(self):
        return [np.asarray(x, np.float32).reshape(3, 4).copy() for x in (self._tb._dataset_meta or {}).get("xforms", [])]


class _Training:
    """Testbed::Nerf::Training (python_api.cu:533-578), the members the NeuS2 path reads."""

    random_bg_color = _opt_property("random_bg_color", bool)
    linear_colors = _opt_property("linear_colors", bool)
    near_distance = _opt_property("near_distance", float)
    # nerf.training.depth_supervision_lambda (python_api.cu:555; default 0, testbed.h:649). The reference's loss kernel
    # computes the depth term (testbed_nerf.cu:1697-1698, 1836) but never adds it to dL/dalpha or any output, so in
    # zbqq/neus2 it does not change training; stored and passed to the device step, which keeps those semantics.
    depth_supervision_lambda = _opt_property("depth_supervision_lambda", float)

    def __init__(self, tb):
        self._tb = tb
        self.dataset = _Dataset(tb)

    @property
    def n_images_for_training(self):
        return self._tb._n_images

    @property
    def counters_rgb(self):
        return self._tb.stats()

    @property
    def transforms(self):
        return self.dataset.transforms

    @property
    def snap_to_pixel_centers(self):
        return False

    @snap_to_pixel_centers.setter
    def snap_to_pixel_centers(self, v):
        if v:
            raise NeusError("nerf.training.snap_to_pixel_centers: training rays use random sub-pixel positions on the gfx950 path")


class _Nerf:
    """Testbed::Nerf (python_api.cu:482-493)."""

    cone_angle_constant = _opt_property("cone_angle_constant", float)

    def __init__(self, tb):
        self._tb = tb
        self.training = _Training(tb)
        self.rendering_min_transmittance = 0.01  # testbed.h: Nerf::rendering_min_transmittance
        # stored for script compatibility; the NeuS path has no camera distortion and no sharpening pass
        self.sharpen = 0.0
        self.render_with_camera_distortion = False
        self.visualize_cameras = False


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
        self._dataset_meta = None
        self._scale, self._offset, self._from_na = 1.0, np.zeros(3, np.float32), False
        self._aabb = (np.zeros(3, np.float32), np.ones(3, np.float32))
        self.nerf = _Nerf(self)
        # render state (testbed.h: m_snap_to_pixel_centers, m_background_color, m_exposure, m_color_space, camera)
        self.snap_to_pixel_centers = False
        self._background_color = np.zeros(4, np.float32)
        self.exposure = 0.0
        self._color_space = ColorSpace.Linear
        self.tonemap_curve = TonemapCurve.Identity
        self.render_mode = "Shade"
        self.max_training_steps = None
        self.reset_camera()

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
        for i, dep in enumerate(d.get("depths") or []):
            if dep is not None:
                self.set_depth(i, dep)
        self._scale, self._offset, self._from_na = float(d["scale"]), np.asarray(d["offset"], np.float32), bool(d["from_na"])
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
        d, imgs = self._frame_data(k + 1)
        arr = _images_array(imgs, d["focal"], d["principal"], d["xforms"])
        check(lib().neus_testbed_next_frame(self._h, C.c_uint32(len(imgs)), arr))
        self._images = imgs
        self._n_images = len(imgs)
        self._dataset_meta = dict(self._dataset_meta or {}, xforms=list(d["xforms"]), focal=list(d["focal"]), principal=list(d["principal"]))
        return True

    def _frame_data(self, k):
        f = self._frames[k]
        d = load_transforms(f) if isinstance(f, str) else f
        imgs = [np.ascontiguousarray(im, np.uint8) for im in d["images"]]
        return d, imgs

    def change_to_frame(self, frame_idx: int):
        """Testbed::change_to_frame (testbed.cu:1939-1985): frame `frame_idx`'s images, training step 0, a fresh
        optimizer; the network, the movement and the phase flags stay (run_dynamic.py loads a snapshot next)."""
        k = int(frame_idx)
        if not 0 <= k < self.all_training_time_frame or not getattr(self, "_frames", None):
            raise NeusError(f"change_to_frame({k}): the dataset has {self.all_training_time_frame} frame(s)")
        d, imgs = self._frame_data(k)
        arr = _images_array(imgs, d["focal"], d["principal"], d["xforms"])
        check(lib().neus_testbed_change_frame(self._h, C.c_uint32(k), C.c_uint32(len(imgs)), arr))
        self._images = imgs
        self._n_images = len(imgs)
        self._dataset_meta = dict(self._dataset_meta or {}, xforms=list(d["xforms"]), focal=list(d["focal"]), principal=list(d["principal"]))

    def prepare_for_test(self):
        """Testbed::prepare_for_test (testbed.cu:1987-1999): render / mesh through the DeltaNetwork iff the current
        frame is not 0 and the movement is being trained. Returns the flag."""
        u = C.c_int()
        check(lib().neus_testbed_prepare_for_test(self._h, C.byref(u)))
        return bool(u.value)

    def saved_transform(self):
        """(R 3x3, t 3) that save_transform writes: this frame's movement composed with the accumulated one."""
        o = (C.c_float * 12)()
        check(lib().neus_testbed_saved_transform(self._h, o))
        a = np.array(o, np.float32)
        return a[:9].reshape(3, 3), a[9:]

    def save_transform(self, path: str):
        """Testbed::save_transform (testbed.cu:3118-3141): three rows of the rotation and the translation, "%f"."""
        R, t = self.saved_transform()
        with open(path, "w") as f:
            for r in R:
                f.write("%f %f %f\n" % (r[0], r[1], r[2]))
            f.write("%f %f %f\n\n" % (t[0], t[1], t[2]))

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

    def set_depth(self, image, depth):
        """NerfDataset::set_training_image's depth (nerf_loader.cu:753-790): a float depth map (scene units) of training
        image `image` at its resolution, kept with the dataset (metadata[img].depth). The reference's training step does
        not use it (see _Training.depth_supervision_lambda)."""
        h, w = self._images[image].shape[:2]
        d = np.ascontiguousarray(depth, np.float32)
        if d.shape != (h, w):
            raise NeusError(f"depth map of image {image} must be {h} x {w}, got {d.shape}")
        self._depths[image] = d

    def set_dataset(self, images, focal, principal, xforms, aabb_scale=1):
        imgs = [np.ascontiguousarray(im, np.uint8) for im in images]
        arr = _images_array(imgs, focal, principal, xforms)
        self._frames = None
        check(lib().neus_testbed_set_dataset(self._h, C.c_uint32(len(imgs)), arr, C.c_float(aabb_scale)))
        self._images = imgs
        self._depths = [None] * len(imgs)
        self._n_images = len(imgs)
        self._dataset_meta = {"xforms": list(xforms), "focal": list(focal), "principal": list(principal),
                              "aabb_scale": float(aabb_scale)}
        s = int(aabb_scale)
        infl = 0.5 * min(1 << 7, s)
        self._aabb = (np.full(3, 0.5 - infl, np.float32), np.full(3, 0.5 + infl, np.float32))
        self._scale, self._offset, self._from_na = 1.0, np.zeros(3, np.float32), False

    def set_progressive_inference(self, mode, chunk_ends=None):
        """Training-step inference in rounds of per-ray sample chunks, skipping the samples past the T < 1e-4 cut
        (bit-identical to one pass; an option of this implementation). mode: 0 off, 1 auto (default), 2 always;
        chunk_ends: the increasing round boundaries (default 32, 64, 96)."""
        e = None if chunk_ends is None else np.ascontiguousarray(chunk_ends, np.uint32)
        check(lib().neus_testbed_set_progressive_inference(self._h, C.c_int(int(mode)),
                                                           None if e is None else C.c_void_p(e.ctypes.data),
                                                           C.c_uint32(0 if e is None else len(e))))

    # ------------------------------------------------------------------ options (device dataset)
    def _get_options(self):
        o = _lib.NeusTrainingOptions()
        check(lib().neus_testbed_get_training_options(self._h, C.byref(o)))
        return o

    def _set_options(self, o):
        check(lib().neus_testbed_set_training_options(self._h, C.byref(o)))

    @property
    def background_color(self):
        """m_background_color (sRGB rgba): composited by render() (tonemap_kernel) and, without
        nerf.training.random_bg_color, the training background (testbed_nerf.cu:1642-1645)."""
        return self._background_color.copy()

    @background_color.setter
    def background_color(self, v):
        self._background_color = np.asarray(v, np.float32).reshape(4).copy()
        o = self._get_options()
        o.background_color[:] = [float(x) for x in self._background_color[:3]]
        self._set_options(o)

    @property
    def color_space(self):
        """m_color_space: the loss targets (testbed_nerf.cu:1657-1671) and render's tonemap input space."""
        return self._color_space

    @color_space.setter
    def color_space(self, v):
        self._color_space = ColorSpace(int(v))
        o = self._get_options()
        o.color_space = int(self._color_space)
        self._set_options(o)

    # ------------------------------------------------------------------ GUI (not part of the training path)
    def want_repl(self):
        return False

    def init_window(self, width, height, hidden=False):
        raise NeusError("init_window: the GLFW/ImGui viewer is not part of the gfx950 training path; use render()")

    def destroy_window(self):
        pass

    def reset_accumulation(self):
        pass

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

    def n_params(self):
        """Testbed::n_params: trainable parameters of the NeuS network (MLPs + hash grid + variance)."""
        return int(self.layout()["n_params"])

    def n_encoding_params(self):
        """Testbed::n_encoding_params: hash-grid parameters."""
        return int(self.layout()["n_grid_params"])

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
        st = self.stats()
        if st["training_aborted"]:
            # testbed_nerf.cu:3542-3548 (0 compacted samples: "Aborting training"), or a non-finite loss
            import warnings
            warnings.warn("NeuS training generated 0 samples or a non-finite loss; aborting training")
            self.shall_train = False
        return True

    # ------------------------------------------------------------------ camera (testbed.cu:238-285, 1830-1844, 2738-2746)
    def reset_camera(self):
        """Testbed::reset_camera (testbed.cu:272-285): fov_axis 1, fov 50.625 deg, zoom 1, screen centre 0.5, the
        default camera looking down -z from (0.5, 0.5, 2.0)."""
        self.fov_axis = 1
        self.fov = 50.625
        self.zoom = 1.0
        self._screen_center = np.array([0.5, 0.5], np.float32)
        cam = np.array([[1, 0, 0, 0.5], [0, -1, 0, 0.5], [0, 0, -1, 0.5]], np.float32)
        cam[:, 3] -= np.float32(1.5) * cam[:, 2]
        self._camera = cam
        self._render_view = None

    @property
    def fov(self):
        """Testbed::fov: focal_length_to_fov(1, relative focal length[fov_axis]) in degrees."""
        return float(2.0 * math.atan(0.5 / float(self._rel_focal[int(self.fov_axis)])) * 180.0 / math.pi)

    @fov.setter
    def fov(self, deg):
        self._rel_focal = np.full(2, fov_to_focal_length(1, float(deg)), np.float32)
        self._render_view = None

    @property
    def fov_xy(self):
        return np.array([2.0 * math.atan(0.5 / float(f)) * 180.0 / math.pi for f in self._rel_focal], np.float32)

    @fov_xy.setter
    def fov_xy(self, v):
        self._rel_focal = np.array([fov_to_focal_length(1, float(x)) for x in np.asarray(v).reshape(2)], np.float32)
        self._render_view = None

    @property
    def screen_center(self):
        return self._screen_center.copy()

    @screen_center.setter
    def screen_center(self, v):
        self._screen_center = np.asarray(v, np.float32).reshape(2).copy()
        self._render_view = None

    @property
    def camera_matrix(self):
        """m_camera: camera-to-world 3x4 in the ngp convention."""
        return self._camera.copy()

    @camera_matrix.setter
    def camera_matrix(self, m):
        self._camera = np.asarray(m, np.float32).reshape(3, 4).copy()
        self._render_view = None

    def set_nerf_camera_matrix(self, cam):
        """Testbed::set_nerf_camera_matrix (testbed.cu:238-240): m_camera = dataset.nerf_matrix_to_ngp(cam), a 3x4
        (or 4x4) NeRF camera-to-world matrix in the dataset's original coordinates."""
        self._camera = nerf_matrix_to_ngp(np.asarray(cam, np.float32)[:3, :4], self._scale, self._offset, self._from_na)
        self._render_view = None

    def set_camera_to_training_view(self, view: int):
        """Testbed::set_camera_to_training_view (testbed.cu:264-270): the camera, relative focal length
        (focal / resolution[fov_axis]) and screen centre (1 - principal point) of training image `view`."""
        if not 0 <= int(view) < self._n_images:
            raise NeusError(f"training view {view} out of range (0..{self._n_images - 1})")
        v = int(view)
        meta = self._dataset_meta
        im = self._images[v]
        res = np.array([im.shape[1], im.shape[0]], np.float32)
        self._camera = np.asarray(meta["xforms"][v], np.float32).reshape(3, 4).copy()
        self._rel_focal = (np.asarray(meta["focal"][v], np.float32).reshape(2) / res[int(self.fov_axis)]).astype(np.float32)
        self._screen_center = (np.float32(1.0) - np.asarray(meta["principal"][v], np.float32).reshape(2)).astype(np.float32)
        # the device computes this camera from its own copy of the view (bit-identical to the oracle's render)
        self._render_view = v if int(self.fov_axis) == 1 else None

    # ------------------------------------------------------------------ rendering
    def _render_request(self, width, height, spp, use_ema):
        rq = _lib.NeusRenderRequest()
        rq.width, rq.height, rq.spp = int(width), int(height), int(spp)
        if self._render_view is not None and float(self.zoom) == 1.0:
            rq.training_view = self._render_view
        else:
            # calc_focal_length = relative focal * resolution[fov_axis] * zoom; render_screen_center
            rq.training_view = -1
            rq.xform[:] = [float(x) for x in self._camera.reshape(12)]
            z = np.float32(self.zoom)
            fl = self._rel_focal * np.float32((int(width), int(height))[int(self.fov_axis)]) * z
            rq.focal[:] = [float(x) for x in fl]
            sc = (np.float32(0.5) - self._screen_center) * z + np.float32(0.5)
            rq.screen_center[:] = [float(x) for x in sc]
        rq.snap_to_pixel_centers = int(bool(self.snap_to_pixel_centers))
        rq.min_transmittance = float(self.nerf.rendering_min_transmittance)
        rq.use_ema = int(bool(use_ema))
        return rq

    def render_accumulation(self, width: int = 1920, height: int = 1080, spp: int = 1, use_ema: bool = True):
        """The linear accumulation buffer of `spp` NerfTracer::trace frames (render_buffer.cu:217-260): float32
        [height, width, 4], premultiplied alpha, before tonemap_kernel."""
        if not self._n_images:
            raise NeusError("render: load the training data first")
        rq = self._render_request(width, height, spp, use_ema)
        out = np.empty((int(height), int(width), 4), np.float32)
        it = C.c_uint32()
        check(lib().neus_testbed_render(self._h, C.byref(rq), C.c_void_p(out.ctypes.data), C.byref(it)))
        self.last_render_iterations = it.value
        return out

    def render(self, width: int = 1920, height: int = 1080, spp: int = 1, linear: bool = True, start_t: float = -1.0,
               end_t: float = -1.0, fps: float = 30.0, shutter_fraction: float = 1.0, use_ema: bool = True):
        """Testbed::render_to_cpu (python_api.cu:123-169) for the NeuS Shade mode: `spp` frames accumulated in linear
        colour from the current camera (set_camera_to_training_view / set_nerf_camera_matrix / camera_matrix with
        fov, fov_axis, zoom, screen_center), then tonemap_kernel (render_buffer.cu:474-500): background_color
        composited, exposure, tonemap_curve, sRGB output when linear=False. Camera paths (start_t >= 0) are not
        supported."""
        if start_t >= 0.0:
            raise NeusError("render: camera paths (start_t/end_t) are not supported; set the camera per frame")
        acc = self.render_accumulation(width, height, spp, use_ema)
        return tonemap_image(acc, self.exposure, self._background_color, self._color_space, self.tonemap_curve, to_srgb=not linear)

    # ------------------------------------------------------------------ meshes
    def compute_marching_cubes_mesh(self, resolution=(256, 256, 256), aabb=None, thresh=None, density_grid=None):
        """Testbed::compute_marching_cubes_mesh (python_api.cu:99-121): dict V (vertices), N (normalised
        1-ring normals), C (vertex colours), F (faces). `aabb`: a BoundingBox or (min, max); None or an empty
        (inside-out) box = the render aabb.
        thresh None = m_mesh.thresh = 0 (the SDF level set). `density_grid` (torch cuda tensor of
        res[2] x res[1] x res[0] floats) skips the network and meshes that grid as given."""
        res = (C.c_int32 * 3)(*[int(r) for r in np.broadcast_to(np.asarray(resolution), 3)])
        pair = _aabb_pair(aabb)
        amin, amax = self._aabb if pair is None else pair
        cmin, cmax = (C.c_float * 3)(*map(float, amin)), (C.c_float * 3)(*map(float, amax))
        thresh = 0.0 if thresh is None or float(thresh) >= 3.0e38 else float(thresh)  # float max = m_mesh.thresh (0)
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
        pair = _aabb_pair(aabb)
        amin, amax = self._aabb if pair is None else pair
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

    def infer_timing(self, steps):
        """Trains `steps` steps with the step's own pre-compaction network launches timed (hipEvents around each
        k_nerf_infer launch: the one pass or the progressive rounds): dict of summed launch ms, launches, steps and the
        samples those launches evaluated (neus_testbed_set_infer_timing)."""
        s0 = self.stats()["evaluated_samples_total"]
        check(lib().neus_testbed_set_infer_timing(self._h, C.c_int(1)))
        try:
            self.train_steps(steps)
            self.synchronize()
            ms, n, k = C.c_double(), C.c_uint64(), C.c_uint64()
            check(lib().neus_testbed_infer_timing(self._h, C.byref(ms), C.byref(n), C.byref(k)))
        finally:
            check(lib().neus_testbed_set_infer_timing(self._h, C.c_int(0)))
        return {"ms": float(ms.value), "launches": int(n.value), "steps": int(k.value),
                "evaluated": int(self.stats()["evaluated_samples_total"] - s0)}

    def set_exchange_timing(self, on=True):
        """Data-parallel exchange timing (neus_testbed_set_exchange_timing): per step, how long the join before the
        optimizer waits for the collectives (exposed) and the exchange's whole window; totals restart here."""
        check(lib().neus_testbed_set_exchange_timing(self._h, C.c_int(1 if on else 0)))

    def exchange_timing(self):
        """dict of exposed_ms / span_ms totals and the steps they cover since set_exchange_timing(True)."""
        e, sp, k = C.c_double(), C.c_double(), C.c_uint64()
        check(lib().neus_testbed_exchange_timing(self._h, C.byref(e), C.byref(sp), C.byref(k)))
        return {"exposed_ms": float(e.value), "span_ms": float(sp.value), "steps": int(k.value)}

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

    def get_optimizer_state(self):
        """Ema(ExponentialDecay(Adam)) state (neus_testbed_get_optimizer_state): dict of current_step,
        learning_rate, learning_rate_factor, m1, m2 (f32), param_steps (u32), ema (fp16 EMA weights)."""
        n = self.layout()["n_params"]
        st = _lib.NeusOptimizerState()
        m1, m2 = np.zeros(n, np.float32), np.zeros(n, np.float32)
        steps, ema = np.zeros(n, np.uint32), np.zeros(n, np.uint16)
        check(lib().neus_testbed_get_optimizer_state(self._h, C.byref(st), C.c_void_p(m1.ctypes.data), C.c_void_p(m2.ctypes.data),
                                                     C.c_void_p(steps.ctypes.data), C.c_void_p(ema.ctypes.data)))
        return {"current_step": int(st.current_step), "learning_rate": float(st.learning_rate),
                "learning_rate_factor": float(st.learning_rate_factor), "m1": m1, "m2": m2, "param_steps": steps,
                "ema": ema.view(np.float16)}

    def set_optimizer_state(self, state):
        n = self.layout()["n_params"]
        st = _lib.NeusOptimizerState()
        st.n_params, st.current_step = n, int(state["current_step"])
        st.learning_rate, st.learning_rate_factor = float(state.get("learning_rate", 0.0)), float(state.get("learning_rate_factor", 1.0))
        m1 = np.ascontiguousarray(state["m1"], np.float32)
        m2 = np.ascontiguousarray(state["m2"], np.float32)
        ema = np.ascontiguousarray(np.asarray(state["ema"], np.float16)).view(np.uint16)
        steps = state.get("param_steps")
        steps = None if steps is None else np.ascontiguousarray(steps, np.uint32)
        if m1.size != n or m2.size != n or ema.size != n or (steps is not None and steps.size != n):
            raise NeusError("set_optimizer_state: array sizes do not match the network's parameter count")
        check(lib().neus_testbed_set_optimizer_state(self._h, C.byref(st), C.c_void_p(m1.ctypes.data), C.c_void_p(m2.ctypes.data),
                                                     C.c_void_p(steps.ctypes.data) if steps is not None else None,
                                                     C.c_void_p(ema.ctypes.data)))

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

    def init_data_parallel(self, rank, world, unique_id: bytes, force_collectives=False):
        """RCCL data parallelism over ray batches (one rank per GPU). force_collectives: create the communicator and
        issue the step's collectives at world 1 as well (tests of the RCCL path on one GPU)."""
        buf = (C.c_uint8 * 128).from_buffer_copy(unique_id)
        check(lib().neus_testbed_init_data_parallel_ex(self._h, C.c_int(rank), C.c_int(world), buf,
                                                       C.c_uint32(1 if force_collectives else 0)))

    def set_exchange_overlap(self, on=True):
        """Overlapped gradient exchange of the data-parallel step (default on; off: one exchange after the backward)."""
        check(lib().neus_testbed_set_exchange_overlap(self._h, C.c_int(1 if on else 0)))

    def data_parallel_info(self):
        from ._lib import NeusDataParallelInfo
        o = NeusDataParallelInfo()
        check(lib().neus_testbed_data_parallel_info(self._h, C.byref(o)))
        return {k: getattr(o, k) for k, _ in o._fields_}

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


class HostGroup:
    """Cross-process data-parallel group (neus_host_group_create): one per rank process; rank 0 listens on host:port, the
    others connect. The testbed's collectives are staged on its communication stream through pinned host memory and
    exchanged over TCP (several ranks on one GPU, where RCCL refuses duplicate devices). Keep it alive while training.
    token: the per-job value every rank passes alike (rank 0 drops connections with another one; draw it at random and
    hand it to the ranks with the port)."""

    def __init__(self, rank: int, world: int, host: str = "127.0.0.1", port: int = 29533, token: int = 0):
        self._h = C.c_void_p()
        check(lib().neus_host_group_create(C.c_int(rank), C.c_int(world), host.encode(), C.c_int(port), C.c_uint64(token),
                                           C.byref(self._h)))
        self.rank, self.world = rank, world

    def join(self, tb):
        check(lib().neus_testbed_init_host_group(tb.handle, self._h))

    def __del__(self):
        if getattr(self, "_h", None):
            lib().neus_host_group_destroy(self._h)
            self._h = None


def nccl_unique_id() -> bytes:
    buf = (C.c_uint8 * 128)()
    check(lib().neus_nccl_unique_id(buf))
    return bytes(buf)
