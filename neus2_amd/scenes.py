"""Synthetic scenes: an analytic Lambertian sphere rendered to RGBA8 views with
ngp-convention cameras, plus the analytic occupancy shell. Used for config 1, "Config S"
(DTU-shaped, 49 x 1600x1200) and the throughput benchmark (no datasets are reachable here)."""
from __future__ import annotations

import numpy as np

CENTER = np.array([0.5, 0.5, 0.5], np.float64)
RADIUS = 0.25
ALBEDO = np.array([0.8, 0.6, 0.4])
LIGHT = np.array([1.0, 1.0, 1.0]) / np.sqrt(3.0)


def look_at(pos, target):
    """camera-to-world 3x4 (columns: right, down, forward, position) in the ngp convention where
    a pixel ray is R @ ((x - cx) * W / fx, (y - cy) * H / fy, 1) (testbed_nerf.cu:1351-1372)."""
    pos = np.asarray(pos, np.float64)
    f = np.asarray(target, np.float64) - pos
    f /= np.linalg.norm(f)
    down = np.array([0.0, 1.0, 0.0])
    down = down - f * np.dot(down, f)
    if np.linalg.norm(down) < 1e-6:
        down = np.array([0.0, 0.0, 1.0]) - f * f[2]
    down /= np.linalg.norm(down)
    right = np.cross(down, f)
    M = np.zeros((3, 4))
    M[:, 0], M[:, 1], M[:, 2], M[:, 3] = right, down, f, pos
    return M


def render_sphere(M, width, height, focal, principal, center=None):
    """Ray-sphere intersection per pixel centre; premultiplied RGBA8 (alpha = coverage)."""
    CENTER = globals()["CENTER"] if center is None else np.asarray(center, np.float64)
    xs = (np.arange(width) + 0.5) / width
    ys = (np.arange(height) + 0.5) / height
    X, Y = np.meshgrid(xs, ys)
    d = np.stack([(X - principal[0]) * width / focal[0], (Y - principal[1]) * height / focal[1], np.ones_like(X)], -1)
    d = d @ M[:, :3].T
    d /= np.linalg.norm(d, axis=-1, keepdims=True)
    o = M[:, 3]
    oc = o - CENTER
    b = d @ oc
    c = oc @ oc - RADIUS ** 2
    disc = b * b - c
    hit = disc > 0
    t = -b - np.sqrt(np.maximum(disc, 0.0))
    hit &= t > 0
    p = o + t[..., None] * d
    n = (p - CENTER) / RADIUS
    shade = np.clip(n @ LIGHT, 0.0, 1.0) * 0.85 + 0.15
    lin = shade[..., None] * ALBEDO
    srgb = np.where(lin <= 0.0031308, 12.92 * lin, 1.055 * np.power(np.maximum(lin, 1e-12), 1 / 2.4) - 0.055)
    rgba = np.zeros((height, width, 4), np.uint8)
    rgba[..., :3] = np.where(hit[..., None], np.clip(np.round(srgb * 255), 0, 255), 0).astype(np.uint8)
    rgba[..., 3] = np.where(hit, 255, 0).astype(np.uint8)
    return rgba


def sphere_scene(n_views=49, width=1600, height=1200, focal=(2892.0, 2892.0), principal=(823.2 / 1600, 619.1 / 1200),
                 distance=2.0, elevation_deg=20.0):
    """Config S: cameras on a ring around the sphere centre."""
    images, xforms = [], []
    for k in range(n_views):
        th = 2 * np.pi * k / n_views
        el = np.deg2rad(elevation_deg * np.sin(3 * th))
        pos = CENTER + distance * np.array([np.sin(th) * np.cos(el), -np.sin(el), -np.cos(th) * np.cos(el)])
        M = look_at(pos, CENTER)
        xforms.append(M.astype(np.float32))
        images.append(render_sphere(M, width, height, focal, principal))
    n = len(images)
    return dict(images=images, xforms=np.stack(xforms), focal=np.tile(np.float32(focal), (n, 1)),
                principal=np.tile(np.float32(principal), (n, 1)), aabb_scale=1)


def dynamic_scene(n_frames=3, shift=(0.01, 0.0, 0.0), n_views=8, width=64, height=48, focal=60.0, distance=1.6):
    """Config 4: the sphere translated by `shift` per frame, fixed cameras on a ring;
    one dataset dict per frame (set_dataset_frames)."""
    frames = []
    for f in range(n_frames):
        c = CENTER + np.asarray(shift, np.float64) * f
        images, xforms = [], []
        for k in range(n_views):
            th = 2 * np.pi * k / n_views
            el = np.deg2rad(20.0 * np.sin(3 * th))
            pos = CENTER + distance * np.array([np.sin(th) * np.cos(el), -np.sin(el), -np.cos(th) * np.cos(el)])
            M = look_at(pos, CENTER)
            xforms.append(M.astype(np.float32))
            images.append(render_sphere(M, width, height, (focal, focal), (0.5, 0.5), center=c))
        frames.append(dict(images=images, xforms=np.stack(xforms), focal=np.tile(np.float32([focal, focal]), (n_views, 1)),
                           principal=np.tile(np.float32([0.5, 0.5]), (n_views, 1)), aabb_scale=1))
    return frames


def config1_scene():
    """Config 1: one 64x64 view from (0.5, 0.5, -1.5) looking +z, focal 64 px."""
    M = np.zeros((3, 4), np.float32)
    M[:, :3] = np.eye(3)
    M[:, 3] = (0.5, 0.5, -1.5)
    img = render_sphere(M.astype(np.float64), 64, 64, (64.0, 64.0), (0.5, 0.5))
    return dict(images=[img], xforms=M[None], focal=np.float32([[64.0, 64.0]]), principal=np.float32([[0.5, 0.5]]), aabb_scale=1)


def small_scene(n_views=8, width=64, height=48, seed_focal=60.0):
    """Tiny DTU-shaped scene for parity tests (8 views, 64x48)."""
    return sphere_scene(n_views, width, height, (seed_focal, seed_focal), (0.5, 0.5), distance=1.6)


def _morton_expand(v):
    v = v.astype(np.uint64)
    v = (v * 0x00010001) & 0xFF0000FF
    v = (v * 0x00000101) & 0x0F00F00F
    v = (v * 0x00000011) & 0xC30C30C3
    v = (v * 0x00000005) & 0x49249249
    return v


def shell_bitfield(thickness=2.0 / 128, radius=RADIUS, center=CENTER):
    """Occupancy bitfield (8 mips, max-pooled like bitfield_max_pool) of the cells whose centre
    satisfies | |p - c| - r | < thickness. Mip 0 covers [0,1]^3."""
    G = 128
    idx = np.arange(G, dtype=np.float64)
    cx = (idx + 0.5) / G
    X, Y, Z = np.meshgrid(cx, cx, cx, indexing="ij")
    dist = np.sqrt((X - center[0]) ** 2 + (Y - center[1]) ** 2 + (Z - center[2]) ** 2)
    occ = np.abs(dist - radius) < thickness
    return bitfield_from_occupancy(occ)


def bitfield_from_occupancy(occ):
    G = 128
    ii = np.arange(G)
    X, Y, Z = np.meshgrid(ii, ii, ii, indexing="ij")
    m = (_morton_expand(X) | (_morton_expand(Y) << 1) | (_morton_expand(Z) << 2)).astype(np.int64)
    flat = np.zeros(G ** 3, bool)
    flat[m.reshape(-1)] = occ.reshape(-1)
    bf = np.zeros(G ** 3 // 8 * 8, np.uint8)
    lvl0 = np.packbits(flat.reshape(-1, 8), axis=1, bitorder="little").reshape(-1)
    bf[: G ** 3 // 8] = lvl0
    nbytes = G ** 3 // 8
    # bitfield_max_pool (testbed_nerf.cu:774-795)
    i = np.arange(G ** 3 // 64)
    inv = lambda x: _morton_invert(x)
    for level in range(1, 8):
        prev = bf[nbytes * (level - 1): nbytes * level]
        bits = (prev.reshape(-1, 8) > 0).astype(np.uint8)
        byte = np.packbits(bits, axis=1, bitorder="little").reshape(-1)
        x = inv(i) + 16
        y = inv(i >> 1) + 16
        z = inv(i >> 2) + 16
        dst = (_morton_expand(x) | (_morton_expand(y) << 1) | (_morton_expand(z) << 2)).astype(np.int64)
        nxt = bf[nbytes * level: nbytes * (level + 1)]
        nxt[dst] |= byte
    return bf


def _morton_invert(x):
    x = x.astype(np.uint64) & 0x49249249
    x = (x | (x >> 2)) & 0xc30c30c3
    x = (x | (x >> 4)) & 0x0f00f00f
    x = (x | (x >> 8)) & 0xff0000ff
    x = (x | (x >> 16)) & 0x0000ffff
    return x


def write_transforms(scene, directory, scale=0.33, offset=(0.5, 0.5, 0.5), name="transforms.json"):
    """Writes a scene (images, focal, principal, ngp xforms) as the reference's dataset format: RGBA PNGs plus a
    transforms.json with fl_x / fl_y / cx / cy / w / h and NeRF camera-to-world matrices (ngp_matrix_to_nerf of the
    ngp cameras, so load_transforms recovers them up to float rounding)."""
    import json
    import os
    from PIL import Image
    from .pyngp import ngp_matrix_to_nerf
    os.makedirs(directory, exist_ok=True)
    h, w = scene["images"][0].shape[:2]
    frames = []
    sub = "images" if name == "transforms.json" else os.path.splitext(name)[0]
    for i, im in enumerate(scene["images"]):
        fn = f"{sub}/{i:03d}.png"
        os.makedirs(os.path.join(directory, sub), exist_ok=True)
        Image.fromarray(np.asarray(im, np.uint8), "RGBA").save(os.path.join(directory, fn))
        m = np.eye(4, dtype=np.float64)
        m[:3, :4] = ngp_matrix_to_nerf(scene["xforms"][i], scale, offset, False)
        frames.append({"file_path": fn, "transform_matrix": m.tolist()})
    f0, p0 = np.asarray(scene["focal"][0], np.float64), np.asarray(scene["principal"][0], np.float64)
    import math
    js = {"w": w, "h": h, "fl_x": float(f0[0]), "fl_y": float(f0[1]), "cx": float(p0[0] * w), "cy": float(p0[1] * h),
          "camera_angle_x": 2.0 * math.atan(0.5 * w / float(f0[0])),
          "scale": float(scale), "offset": [float(v) for v in np.broadcast_to(offset, 3)], "aabb_scale": 1, "frames": frames}
    path = os.path.join(directory, name)
    with open(path, "w") as f:
        json.dump(js, f, indent=1)
    return path
