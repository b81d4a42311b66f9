"""transforms.json image preparation: separate alpha images, dynamic masks and
white / black transparency, through the product loader (pyngp.load_transforms -> neus_prepare_image_rgba8, host
code) against the oracle's restatement of ngp::load_nerf (nerf_loader.cu:59-81, 550-590), bit-exact, on small PNG
fixtures written here. CPU only: the preparation is host code (the device only reads the prepared RGBA8)."""
import json
import os

import numpy as np
import pytest

pytest.importorskip("PIL")


def _png(path, arr):
    from PIL import Image
    Image.fromarray(np.ascontiguousarray(arr, np.uint8), "RGBA").save(path)


def _scene(tmp_path, white=False, black=False, alpha_frames=(), mask_frames=(), n=3, w=20, h=12, seed=0):
    rng = np.random.default_rng(seed)
    os.makedirs(tmp_path / "images", exist_ok=True)
    frames, raw = [], []
    for i in range(n):
        img = rng.integers(0, 256, (h, w, 4), dtype=np.uint8)
        img[0, :4, :3] = 255  # pure white pixels
        img[1, :4, :3] = 0    # pure black pixels
        img[2, 0] = (0xFF, 0x00, 0xFF, 0x00)  # a pixel already equal to the hot-pink key
        name = f"images/{i:03d}"
        # frame 0 names its file without an extension (the loader appends .png)
        fp = name if i == 0 else name + ".png"
        _png(tmp_path / (name + ".png"), img)
        alpha = mask = None
        if i in alpha_frames:
            alpha = rng.integers(0, 256, (h, w, 4), dtype=np.uint8)
            _png(tmp_path / (fp + ".alpha.png"), alpha)
        if i in mask_frames:
            mask = np.zeros((h, w, 4), np.uint8)
            mask[rng.random((h, w)) < 0.3, 0] = rng.integers(1, 256)
            mask[..., 3] = 255
            _png(tmp_path / "images" / f"dynamic_mask_{i:03d}.png", mask)
        raw.append((img, alpha, mask))
        c2w = np.eye(4)
        c2w[:3, 3] = (0.5, 0.5, -1.0 - 0.1 * i)
        frames.append({"file_path": fp, "transform_matrix": c2w.tolist()})
    js = {"camera_angle_x": 0.8, "scale": 0.5, "offset": [0.5, 0.5, 0.5], "aabb_scale": 1, "frames": frames}
    if white:
        js["white_transparent"] = True
    if black:
        js["black_transparent"] = True
    with open(tmp_path / "transforms.json", "w") as f:
        json.dump(js, f)
    return raw


@pytest.mark.parametrize("white,black", [(False, False), (True, False), (False, True), (True, True)])
def test_load_transforms_prepares_images_as_reference(tmp_path, white, black):
    import oracle as O
    from neus2_amd import pyngp
    raw = _scene(tmp_path, white, black, alpha_frames=(0, 2), mask_frames=(1, 2))
    ds = pyngp.load_transforms(str(tmp_path / "transforms.json"))
    assert len(ds["images"]) == 3
    for i, (img, alpha, mask) in enumerate(raw):
        ref, key = O.prepare_image(img, alpha, mask, white, black)
        np.testing.assert_array_equal(ds["images"][i], ref)
        assert ds["mask_colors"][i] == key == (0x00FF00FF if mask is not None else 0)
    # spot checks of the semantics themselves
    img0, a0, _ = raw[0]
    got0 = ds["images"][0]
    lin = np.where(a0[..., 0] / 255.0 <= 0.04045, a0[..., 0] / 255.0 / 12.92, ((a0[..., 0] / 255.0 + 0.055) / 1.055) ** 2.4)
    # (rows 0-1 hold the pure white / black pixels the transparency flags may clear; row 2 the hot-pink pixel)
    assert np.abs(got0[3:, :, 3].astype(np.int32) - np.floor(255 * lin[3:]).astype(np.int32)).max() <= 1
    img1, _, m1 = raw[1]
    got1 = ds["images"][1].view(np.uint32)[..., 0]
    assert np.all(got1[m1[..., 0] != 0] == 0x00FF00FF)
    if white:
        sel = (img1[..., :3] == 255).all(-1) & (m1[..., 0] == 0)
        assert sel.any() and np.all(ds["images"][1][sel, 3] == 0)


def test_mask_and_alpha_resolution_checked(tmp_path):
    from neus2_amd import pyngp
    _scene(tmp_path, mask_frames=(0,))
    from PIL import Image
    Image.fromarray(np.zeros((5, 5, 4), np.uint8), "RGBA").save(tmp_path / "images" / "dynamic_mask_000.png")
    with pytest.raises(RuntimeError, match="Mask image has wrong resolution"):
        pyngp.load_transforms(str(tmp_path / "transforms.json"))


def test_plain_dataset_unchanged(tmp_path):
    """No alpha / mask files, no transparency flags: the images load untouched and carry no mask key."""
    from neus2_amd import pyngp
    raw = _scene(tmp_path)
    ds = pyngp.load_transforms(str(tmp_path / "transforms.json"))
    for i, (img, _, _) in enumerate(raw):
        np.testing.assert_array_equal(ds["images"][i], img)
        assert ds["mask_colors"][i] == 0


def _depth_scene(tmp_path, scale_int=1e-3, enable=None, n=3, w=20, h=12, seed=5, missing=(), wrong=()):
    """Frames with `depth_path` 16-bit PNGs (nerf_loader.cu:599-612); frame indices in `missing` name a file that does
    not exist, those in `wrong` one of the wrong resolution."""
    from PIL import Image
    _scene(tmp_path, n=n, w=w, h=h)
    js = json.load(open(tmp_path / "transforms.json"))
    rng = np.random.default_rng(seed)
    raw = []
    for i, fr in enumerate(js["frames"]):
        d = rng.integers(0, 65536, (h, w), dtype=np.uint16)
        if i in wrong:
            d = d[:-1]
        name = f"depth/{i:03d}.png"
        os.makedirs(tmp_path / "depth", exist_ok=True)
        if i not in missing:
            Image.fromarray(d).save(tmp_path / name)
        fr["depth_path"] = name
        raw.append(d)
    if scale_int is not None:
        js["integer_depth_scale"] = scale_int
    if enable is not None:
        js["enable_depth_loading"] = enable
    with open(tmp_path / "transforms.json", "w") as f:
        json.dump(js, f)
    return raw, js["scale"]


def test_depth_maps_loaded_as_reference(tmp_path):
    """depth = uint16 x integer_depth_scale x scale (set_training_image(..., depth_scale * result.scale), copy_depth
    nerf_loader.cu:91-99, 736); a frame whose depth file does not exist has none (the reference skips it)."""
    from neus2_amd import pyngp
    raw, scale = _depth_scene(tmp_path, scale_int=2.5e-4, missing=(1,))
    ds = pyngp.load_transforms(str(tmp_path / "transforms.json"))
    assert ds["depths"][1] is None
    for i in (0, 2):
        expect = raw[i].astype(np.float32) * np.float32(2.5e-4 * scale)
        np.testing.assert_array_equal(ds["depths"][i], expect)
        assert ds["depths"][i].dtype == np.float32


@pytest.mark.parametrize("scale_int,enable", [(None, None), (-1.0, None), (1e-3, False)])
def test_depth_loading_gated(tmp_path, scale_int, enable):
    """No `integer_depth_scale` (default -1), a non-positive one, or enable_depth_loading false: no depth is loaded
    (nerf_loader.cu:321-339, 392-393, 599)."""
    from neus2_amd import pyngp
    _depth_scene(tmp_path, scale_int=scale_int, enable=enable)
    ds = pyngp.load_transforms(str(tmp_path / "transforms.json"))
    assert all(d is None for d in ds["depths"])


def test_depth_resolution_checked(tmp_path):
    from neus2_amd import pyngp
    _depth_scene(tmp_path, wrong=(2,))
    with pytest.raises(RuntimeError, match="Depth image has wrong resolution"):
        pyngp.load_transforms(str(tmp_path / "transforms.json"))


def test_read_depth_u16_formats(tmp_path):
    """stbi_load_16(..., 1): 16-bit grey as is, 8-bit grey widened x 257, colour reduced to stbi's 16-bit luma."""
    from PIL import Image
    from neus2_amd import pyngp
    g8 = np.arange(60, dtype=np.uint8).reshape(6, 10)
    Image.fromarray(g8, "L").save(tmp_path / "g8.png")
    np.testing.assert_array_equal(pyngp.read_depth_u16(str(tmp_path / "g8.png")), g8.astype(np.uint16) * 257)
    rgb = np.stack([g8, g8[::-1], g8 // 2], -1)
    Image.fromarray(rgb, "RGB").save(tmp_path / "rgb.png")
    r, g, b = [rgb[..., k].astype(np.uint32) * 257 for k in range(3)]
    np.testing.assert_array_equal(pyngp.read_depth_u16(str(tmp_path / "rgb.png")), ((r * 77 + g * 150 + b * 29) >> 8).astype(np.uint16))
