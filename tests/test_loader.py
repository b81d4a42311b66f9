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
