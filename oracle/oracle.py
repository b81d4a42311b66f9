"""ctypes wrapper of the CPU oracle (liboracle) — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this
module. It restates the reference NeuS2 training step on the CPU (see
neus_oracle.cpp for the per-function reference citations).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "libneus_oracle.so")
_lib = None


class OrNetCfg(C.Structure):
    _fields_ = [
        ("n_levels", C.c_uint32), ("log2_hashmap_size", C.c_uint32), ("base_resolution", C.c_uint32),
        ("per_level_scale", C.c_float), ("width", C.c_uint32), ("n_density_hidden", C.c_uint32),
        ("n_rgb_hidden", C.c_uint32), ("density_in", C.c_uint32), ("rgb_in", C.c_uint32), ("sdf_bias", C.c_float),
    ]


class OrDataset(C.Structure):
    _fields_ = [
        ("n_images", C.c_uint32), ("pixels", C.c_void_p), ("pixel_offsets", C.c_void_p),
        ("resolution", C.c_void_p), ("focal", C.c_void_p), ("principal", C.c_void_p), ("xform", C.c_void_p),
        ("aabb_min", C.c_float * 3), ("aabb_max", C.c_float * 3), ("cone_angle", C.c_float),
        ("motion_R", C.c_float * 9), ("motion_t", C.c_float * 3), ("motion_on", C.c_uint32),
        ("fixed_bg", C.c_uint32), ("bg_color", C.c_float * 3), ("target_mode", C.c_uint32),
    ]


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB):
            build()
        _lib = C.CDLL(_LIB)
        _lib.or_grid_tables.restype = C.c_uint32
        _lib.or_net_n_params.restype = C.c_uint32
        _lib.or_generate_samples.restype = C.c_uint32
        _lib.or_compute_loss.restype = C.c_uint32
        _lib.or_det_expf.restype = C.c_float
        _lib.or_det_expf.argtypes = [C.c_float]
        _lib.or_num_threads.restype = C.c_int
        _lib.or_pcg32.argtypes = [C.c_uint64, C.c_uint64, C.c_int64, C.c_uint32, C.c_void_p]
    return _lib


def P(a):
    """Raw pointer to a numpy buffer. The caller must hold a reference to `a` for the duration of the call."""
    return C.c_void_p(a.ctypes.data) if a is not None else C.c_void_p(0)


def f32(x):
    return np.ascontiguousarray(x, dtype=np.float32)


def make_cfg(n_levels=14, log2_hashmap_size=19, base_resolution=16, per_level_scale=None, top_resolution=2048.0,
             aabb_scale=1, width=64, n_density_hidden=1, n_rgb_hidden=2, sdf_bias=-0.1):
    """Derives per_level_scale exactly as Testbed::reset_network (testbed.cu:2175-2187), in float32."""
    if per_level_scale is None:
        if n_levels > 1:
            v = np.float32(top_resolution) * np.float32(aabb_scale) / np.float32(base_resolution)
            per_level_scale = float(np.exp(np.log(np.float32(v), dtype=np.float32) / np.float32(n_levels - 1), dtype=np.float32))
        else:
            per_level_scale = 2.0
    density_in = ((3 + 2 * n_levels) + 15) // 16 * 16
    c = OrNetCfg(n_levels, log2_hashmap_size, base_resolution, per_level_scale, width, n_density_hidden, n_rgb_hidden,
                 density_in, 48, sdf_bias)
    return c


def layout(cfg):
    out = np.zeros(7, np.uint32)
    lib().or_net_layout(C.byref(cfg), P(out))
    keys = ["n_density", "n_rgb", "grid_off", "n_grid_params", "var_off", "n_params", "n_matrix"]
    return {k: int(v) for k, v in zip(keys, out)}


def grid_tables(cfg):
    L = cfg.n_levels
    off = np.zeros(L + 1, np.uint32)
    res = np.zeros(L, np.uint32)
    sc = np.zeros(L, np.float32)
    n = lib().or_grid_tables(C.byref(cfg), P(off), P(res), P(sc))
    return off, res, sc, n


def geometric_init(cfg, seed=1337):
    lay = layout(cfg)
    out = np.zeros(lay["n_density"], np.float32)
    lib().or_geometric_init(C.byref(cfg), C.c_uint64(seed), P(out))
    return out


def init_params(cfg, seed=1337, geo=True):
    lay = layout(cfg)
    params = np.zeros(lay["n_params"], np.float32)
    g = geometric_init(cfg) if geo else None
    lib().or_init_params(C.byref(cfg), C.c_uint32(seed), P(g), P(params))
    return params


def pcg32(seed, seq=1, advance=0, n=4):
    out = np.zeros(n, np.uint32)
    lib().or_pcg32(seed, seq, advance, n, P(out))
    return out


def grid_forward(cfg, params, pos, valid_level, want_dydx=True):
    pos = f32(pos)
    n = pos.shape[0]
    L = cfg.n_levels
    enc = np.zeros((n, 2 * L), np.float32)
    dydx = np.zeros((n, 2 * L, 3), np.float32) if want_dydx else None
    params = f32(params)
    lib().or_grid_forward(C.byref(cfg), P(params), C.c_uint32(n), P(pos), C.c_uint32(valid_level), P(enc), P(dydx))
    return enc, dydx


def network_forward(cfg, params, coords, valid_level):
    coords = f32(coords)
    n = coords.shape[0]
    out = np.zeros((n, 16), np.uint16)
    params = f32(params)
    lib().or_network_forward(C.byref(cfg), P(params), C.c_uint32(n), P(coords), C.c_uint32(valid_level), P(out))
    return out


def network_backward(cfg, params, coords, valid_level, dL_dout_u16, indeed_batch_size):
    coords = f32(coords)
    n = coords.shape[0]
    grads = np.zeros(layout(cfg)["n_params"], np.float32)
    d = np.ascontiguousarray(dL_dout_u16, np.uint16)
    params = f32(params)
    lib().or_network_backward(C.byref(cfg), P(params), C.c_uint32(n), P(coords), C.c_uint32(valid_level), P(d),
                              C.c_uint32(indeed_batch_size), P(grads))
    return grads


def network_backward_pos(cfg, params, coords, valid_level, dL_dout_u16, indeed_batch_size):
    """network_backward plus dL/d(position) [n, 4] (the DeltaNetwork's input gradient)."""
    coords = f32(coords)
    n = coords.shape[0]
    grads = np.zeros(layout(cfg)["n_params"], np.float32)
    dpos = np.zeros((n, 4), np.float32)
    d = np.ascontiguousarray(dL_dout_u16, np.uint16)
    params = f32(params)
    lib().or_network_backward_pos(C.byref(cfg), P(params), C.c_uint32(n), P(coords), C.c_uint32(valid_level), P(d),
                                  C.c_uint32(indeed_batch_size), P(grads), P(dpos))
    return grads, dpos


class Dataset:
    """Host-side dataset view shared by oracle calls (RGBA8 images + ngp cameras)."""

    def __init__(self, images, focal, principal, xform, aabb_min=(0, 0, 0), aabb_max=(1, 1, 1), cone_angle=0.0):
        self.images = [np.ascontiguousarray(im, np.uint8) for im in images]
        self.res = np.array([[im.shape[1], im.shape[0]] for im in self.images], np.int32)
        self.pixels = np.concatenate([im.reshape(-1, 4).view(np.uint32).reshape(-1) for im in self.images])
        sizes = [im.shape[0] * im.shape[1] for im in self.images]
        self.offsets = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.uint64)
        self.focal = f32(focal).reshape(-1, 2)
        self.principal = f32(principal).reshape(-1, 2)
        self.xform = f32(xform).reshape(-1, 12)
        self.c = OrDataset()
        self.c.n_images = len(self.images)
        self.c.pixels = self.pixels.ctypes.data
        self.c.pixel_offsets = self.offsets.ctypes.data
        self.c.resolution = self.res.ctypes.data
        self.c.focal = self.focal.ctypes.data
        self.c.principal = self.principal.ctypes.data
        self.c.xform = self.xform.ctypes.data
        self.c.aabb_min[:] = list(aabb_min)
        self.c.aabb_max[:] = list(aabb_max)
        self.c.cone_angle = cone_angle
        self.set_motion(None)

    def set_motion(self, Rt):
        """Accumulated global movement of the rays (3x4 [R | t]); None = identity (static scene / frame 0)."""
        if Rt is None:
            self.c.motion_R[:] = [1, 0, 0, 0, 1, 0, 0, 0, 1]
            self.c.motion_t[:] = [0, 0, 0]
            self.c.motion_on = 0
        else:
            Rt = np.asarray(Rt, np.float32)
            self.c.motion_R[:] = [float(v) for v in Rt[:, :3].reshape(-1)]
            self.c.motion_t[:] = [float(v) for v in Rt[:, 3]]
            self.c.motion_on = 1

    def set_target(self, background=None, mode=0):
        """Loss targets (testbed_nerf.cu:1642-1671): background None = random per ray (random_bg_color), else a
        fixed sRGB colour; mode 0 color_space Linear, 1 color_space SRGB, 2 linear_colors."""
        self.c.fixed_bg = 0 if background is None else 1
        self.c.bg_color[:] = [0.0, 0.0, 0.0] if background is None else [float(v) for v in list(background)[:3]]
        self.c.target_mode = int(mode)


def generate_samples(ds, bitfield, n_rays, n_rays_total, rng_state, rng_inc, max_samples, ray_offset=0, n_rays_global=None):
    n_rays_global = n_rays if n_rays_global is None else n_rays_global
    rays = np.zeros((n_rays, 6), np.float32)
    numsteps = np.zeros((n_rays, 2), np.uint32)
    coords = np.zeros((max_samples, 7), np.float32)
    nr = C.c_uint32(0)
    bitfield = np.ascontiguousarray(bitfield, np.uint8)
    counter = lib().or_generate_samples(C.byref(ds.c), P(bitfield), C.c_uint32(n_rays),
                                        C.c_uint32(ray_offset), C.c_uint32(n_rays_global), C.c_uint32(n_rays_total),
                                        C.c_uint64(rng_state), C.c_uint64(rng_inc), C.c_uint32(max_samples),
                                        P(rays), P(numsteps), P(coords), C.byref(nr))
    return rays, numsteps, coords, int(counter), int(nr.value)


def compute_loss(ds, n_rays, n_rays_total, rng_state, rng_inc, max_compacted, rays, numsteps, coords, net_out,
                 loss_scale=128.0, mean_density=0.0, ek_w=0.01, mask_w=0.0, cos_anneal=1.0, ray_offset=0, n_rays_global=None):
    n_rays_global = n_rays if n_rays_global is None else n_rays_global
    numsteps = np.ascontiguousarray(numsteps, np.uint32).copy()
    coords_out = np.zeros((max_compacted, 7), np.float32)
    dout = np.zeros((max_compacted, 16), np.uint16)
    loss = np.zeros(n_rays, np.float32)
    ek = np.zeros(n_rays, np.float32)
    mask = np.zeros(n_rays, np.float32)
    rays, coords, net_out = f32(rays), f32(coords), np.ascontiguousarray(net_out, np.uint16)
    counter = lib().or_compute_loss(C.byref(ds.c), C.c_uint32(n_rays), C.c_uint32(ray_offset), C.c_uint32(n_rays_global),
                                    C.c_uint32(n_rays_total), C.c_uint64(rng_state), C.c_uint64(rng_inc), C.c_uint32(max_compacted),
                                    P(rays), P(numsteps), P(coords), P(net_out),
                                    C.c_float(loss_scale), C.c_float(mean_density), C.c_float(ek_w), C.c_float(mask_w),
                                    C.c_float(cos_anneal), P(coords_out), P(dout), P(loss), P(ek), P(mask))
    return dict(numsteps=numsteps, coords=coords_out, dL_dout=dout, loss=loss, ek=ek, mask=mask, counter=int(counter))


def ray_target(ds, ray_idx_global, n_rays_global, n_rays_total, rng_state, rng_inc):
    t = np.zeros(3, np.float32)
    b = np.zeros(3, np.float32)
    lib().or_ray_target(C.byref(ds.c), C.c_uint32(ray_idx_global), C.c_uint32(n_rays_global), C.c_uint32(n_rays_total),
                        C.c_uint64(rng_state), C.c_uint64(rng_inc), P(t), P(b))
    return t, b


def fill_rollover(n_elements, n_in, coords, dout):
    lib().or_fill_rollover(C.c_uint32(n_elements), C.c_uint32(n_in), P(coords), P(dout))


def adam_ema_step(weights, grads, m1, m2, steps, ema_tmp, ema_out, n_matrix, optimizer_step, lr=1e-3, beta1=0.9,
                  beta2=0.99, eps=1e-15, l2=1e-6, loss_scale=128.0, ema_decay=0.95):
    grads = f32(grads)
    lib().or_adam_ema_step(C.c_uint32(weights.size), C.c_uint32(n_matrix), C.c_float(loss_scale), C.c_float(lr),
                           C.c_float(beta1), C.c_float(beta2), C.c_float(eps), C.c_float(l2), C.c_uint32(optimizer_step),
                           C.c_float(ema_decay), P(weights), P(grads), P(m1), P(m2), P(steps), P(ema_tmp), P(ema_out))


def density_grid_update(cfg, params, valid_level, n_uniform, n_nonuniform, ema_step, rng_state, rng_inc, density_grid,
                        bitfield, decay=0.95, aabb_min=(0, 0, 0), aabb_max=(1, 1, 1)):
    st = C.c_uint64(rng_state)
    mean = C.c_float(0)
    params, amin, amax = f32(params), f32(aabb_min), f32(aabb_max)  # keep the buffers alive across the call
    lib().or_density_grid_update(C.byref(cfg), P(params), C.c_uint32(valid_level), P(amin), P(amax),
                                 C.c_uint32(n_uniform), C.c_uint32(n_nonuniform), C.c_uint32(ema_step), C.c_float(decay),
                                 C.byref(st), C.c_uint64(rng_inc), P(density_grid), P(bitfield), C.byref(mean))
    return int(st.value), float(mean.value)


def det_expf(x):
    return lib().or_det_expf(float(x))


def prepare_image(img, alpha=None, mask=None, white_transparent=False, black_transparent=False):
    """ngp::load_nerf's image preparation (nerf_loader.cu:550-590 + convert_rgba32 :59-81); returns (rgba, mask_color)."""
    out = np.ascontiguousarray(img, np.uint8).copy()
    h, w = out.shape[:2]
    a = None if alpha is None else np.ascontiguousarray(alpha, np.uint8)
    m = None if mask is None else np.ascontiguousarray(mask, np.uint8)
    lib().or_prepare_image_rgba8.restype = C.c_uint32
    key = lib().or_prepare_image_rgba8(P(out), C.c_uint32(w), C.c_uint32(h), P(a) if a is not None else None,
                                       P(m) if m is not None else None, C.c_int(int(white_transparent)), C.c_int(int(black_transparent)))
    return out, int(key)


def num_threads():
    return lib().or_num_threads()


SUM_ORDERS = {"index": 0, "reversed": 1, "pairwise": 2, "blocked": 3}


def set_sum_order(order):
    """Order in which the layer products are summed: "index" (the default), "reversed", "pairwise" (recursive halves) or
    "blocked" (blocks of 8, then the block sums); True / False mean reversed / index. Test-only: the alternative orders
    measure how much the fp32 accumulation order alone moves a step (the noise floor of the fp16 network)."""
    if isinstance(order, bool):
        order = "reversed" if order else "index"
    lib().or_set_sum_order(C.c_int(SUM_ORDERS[order] if isinstance(order, str) else int(order)))


GRID_GRAD_MODES = {"exact": 0, "ref_operand": 1, "ref_half": 2}


def set_grid_grad_mode(mode):
    """Semantics of the hash-grid gradient sum (neus_oracle.cpp, or_set_grid_grad_mode). "exact" (the default): corner
    contributions summed unrounded in double. "ref_operand": each contribution rounded to fp16 as the reference's
    atomicAdd(__half2) operand (grid.h:418-421), summed in double. "ref_half": operand and accumulator in fp16
    (grad_t = __half, grid.h:1433), adds in thread-schedule order like the reference's atomics (not reproducible).
    Test-only: bounds how far the reference's own fp16 gradient path sits from the exact sum."""
    lib().or_set_grid_grad_mode(C.c_int(GRID_GRAD_MODES[mode] if isinstance(mode, str) else int(mode)))


class OrRenderCamera(C.Structure):
    _fields_ = [("xform", C.c_float * 12), ("focal", C.c_float * 2), ("screen_center", C.c_float * 2),
                ("width", C.c_uint32), ("height", C.c_uint32)]


def render(cfg, params, valid_level, ds, bitfield, xform, focal, screen_center, width, height, spp=1, snap=True,
           min_transmittance=1e-4, cos_anneal=1.0):
    """CPU restatement of Testbed::render_to_cpu (Shade mode): float32 [H, W, 4] linear premultiplied."""
    cam = OrRenderCamera()
    cam.xform[:] = [float(v) for v in np.asarray(xform, np.float32).reshape(12)]
    cam.focal[:] = [float(v) for v in np.asarray(focal).reshape(2)]
    cam.screen_center[:] = [float(v) for v in np.asarray(screen_center).reshape(2)]
    cam.width, cam.height = int(width), int(height)
    out = np.zeros((int(height), int(width), 4), np.float32)
    it = C.c_uint32()
    params = f32(params)
    bitfield = np.ascontiguousarray(bitfield, np.uint8)
    lib().or_render(C.byref(cfg), P(params), C.c_uint32(valid_level), C.byref(ds.c), P(bitfield), C.byref(cam),
                    C.c_uint32(spp), C.c_int(int(bool(snap))), C.c_float(min_transmittance), C.c_float(cos_anneal), P(out), C.byref(it))
    return out, int(it.value)


def ld_random_val(index, seed):
    lib().or_ld_random_val_export.restype = C.c_float
    return float(lib().or_ld_random_val_export(C.c_uint32(index), C.c_uint32(seed)))


def ld_random_val_2d(index, seed):
    o = np.zeros(2, np.float32)
    lib().or_ld_random_val_2d_export(C.c_uint32(index), C.c_uint32(seed), P(o))
    return o


def sobol(index, dim):
    lib().or_sobol_export.restype = C.c_uint32
    return int(lib().or_sobol_export(C.c_uint32(index), C.c_uint32(dim)))


def marching_cubes(density, thresh, aabb_min=(0, 0, 0), aabb_max=(1, 1, 1), table=None):
    """or_marching_cubes: density [rz][ry][rx] float32 -> V float32 [n, 3], F uint32 [m, 3]."""
    import mc_table
    d = np.ascontiguousarray(density, np.float32)
    rz, ry, rx = d.shape
    tab = np.ascontiguousarray(mc_table.build_table() if table is None else table, np.int8)
    amin, amax = f32(aabb_min), f32(aabb_max)
    f = lib().or_marching_cubes
    f.restype = C.c_uint64
    nt = C.c_uint64()
    nv = f(P(d), C.c_uint32(rx), C.c_uint32(ry), C.c_uint32(rz), C.c_float(thresh), P(amin), P(amax), P(tab), None, None, C.byref(nt))
    V = np.zeros((nv, 3), np.float32)
    F = np.zeros((nt.value, 3), np.uint32)
    f(P(d), C.c_uint32(rx), C.c_uint32(ry), C.c_uint32(rz), C.c_float(thresh), P(amin), P(amax), P(tab), P(V), P(F), C.byref(nt))
    return V, F
