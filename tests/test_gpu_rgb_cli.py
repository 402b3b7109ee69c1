"""GPU tests of SURVEY.md §8(f) rows 2 and 4: the RGB -> luma conversion the reference's
callers run before detect (image 0.24.6 to_luma8, src/main.rs:58), on the device, and the
command-line counterpart of src/main.rs.  Grey inputs are pinned by the golden fixture
(the reference's media image is grey, r = g = b); colour inputs are checked against the
oracle's restatement of image's formula (parity unpinned: no reference output exists)."""
import os
import subprocess
import sys

import numpy as np
import pytest

import workloads
from feature_detector_fast_amd import Config, NonMaximalSuppression, fast_hip
from oracle import oracle

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")


def _grey_as_rgb(img):
    return np.repeat(img[..., None], 3, axis=2)


def test_rgb_grey_input_reproduces_goldens(golden):
    img, off, maxt = golden
    rgb = _grey_as_rgb(img)
    assert np.array_equal(fast_hip.detect_rgb_array(rgb, Config(16, 9, NonMaximalSuppression.Off)), off)
    assert np.array_equal(
        fast_hip.detect_rgb_array(rgb, Config(16, 9, NonMaximalSuppression.MaxThreshold)), maxt)


@pytest.mark.parametrize("w,h", [(300, 200), (97, 41), (1920, 1080), (7, 7), (33, 13)])
@pytest.mark.parametrize("nms", [0, 1, 2])
def test_rgb_colour_matches_oracle(w, h, nms):
    rng = np.random.default_rng(w * 31 + h + nms)
    grey = workloads.s1_frame(nms, w, h)
    tint = rng.integers(0, 40, (h, w, 3), dtype=np.uint8)
    rgb = np.clip(_grey_as_rgb(grey).astype(np.int32) + tint - 20, 0, 255).astype(np.uint8)
    want = oracle.detect(oracle.rgb_to_luma(rgb), 16, 9, nms)
    got = fast_hip.detect_rgb_array(rgb, Config(16, 9, NonMaximalSuppression(nms)))
    assert np.array_equal(got, want)


def test_rgb_strided_rows():
    rng = np.random.default_rng(1)
    big = rng.integers(0, 256, (60, 90, 3), dtype=np.uint8)
    view = big[5:55, 7:80]                       # row stride 270 bytes, width 73
    want = oracle.detect(oracle.rgb_to_luma(np.ascontiguousarray(view)), 10, 9, 0)
    assert np.array_equal(fast_hip.detect_rgb_array(view, Config(10, 9, NonMaximalSuppression.Off)), want)


@pytest.mark.parametrize("f,h,w", [(3, 1080, 1920), (2, 37, 53), (5, 7, 9)])
def test_rgb_to_luma_device_bit_exact(f, h, w):
    import torch

    rng = np.random.default_rng(f + h + w)
    rgb = rng.integers(0, 256, (f, h, w, 3), dtype=np.uint8)
    d_rgb = torch.from_numpy(rgb).cuda()
    d_out = torch.full((f, h, w), 7, dtype=torch.uint8, device="cuda")
    fast_hip.rgb_to_luma(d_rgb, d_out)
    torch.cuda.synchronize()
    got = d_out.cpu().numpy()
    for k in range(f):
        assert np.array_equal(got[k], oracle.rgb_to_luma(rgb[k])), k


def _run_cli(tmp_path, *args):
    out_png = str(tmp_path / "out.png")
    res = subprocess.run([sys.executable, "-m", "feature_detector_fast_amd",
                          os.path.join(GOLD, "screenshot315_grey.pgm"), out_png, *args],
                         capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert res.returncode == 0, res.stdout + res.stderr
    return out_png, res.stdout


@pytest.mark.parametrize("nms,fixture", [("off", "kp_t16_n9_off.txt"),
                                         ("max_threshold", "kp_t16_n9_maxt.txt")])
def test_cli_reproduces_golden_txt_and_overlay(tmp_path, nms, fixture):
    from PIL import Image

    out_png, stdout = _run_cli(tmp_path, "16", "9", nms)
    want = workloads.read_points(os.path.join(GOLD, fixture))
    got = workloads.read_points(out_png.replace(".png", ".txt"))
    assert np.array_equal(got, want)
    assert f"found {len(want)} keypoints" in stdout
    ov = np.asarray(Image.open(out_png).convert("RGB"))
    red = np.argwhere((ov[..., 0] == 255) & (ov[..., 1] == 0) & (ov[..., 2] == 0))
    assert sorted(map(tuple, red[:, ::-1].tolist())) == sorted(map(tuple, want.tolist()))


def test_cli_default_nms_is_sum_absolute(tmp_path):
    """src/main.rs:41-49: without the 5th argument the code picks SumAbsolute."""
    out_png, _ = _run_cli(tmp_path)
    got = workloads.read_points(out_png.replace(".png", ".txt"))
    img = workloads.read_pgm(os.path.join(GOLD, "screenshot315_grey.pgm"))
    assert np.array_equal(got, oracle.detect(img, 16, 9, 2))


@pytest.mark.parametrize("nms", [0, 1, 2])
@pytest.mark.parametrize("geometry", [0, 1])
def test_rgb_device_batch_fused(nms, geometry):
    """fdf_detect_device_rgb (luma converted inside the detector's row and window loads)
    equals fdf_rgb_to_luma_device + fdf_detect_device on a batch of colour frames -- random
    colours, a colour-tinted S1 frame, odd sizes, the last frame read exactly -- and the oracle
    on two frames; with the batch's own geometry and with the tall bands."""
    import torch

    rng = np.random.default_rng(31 + nms)
    H, W = 301, 517
    frames = []
    for i in range(6):
        if i % 2:
            g = workloads.s1_frame(i, W, H).astype(np.int32)
            tint = rng.integers(-40, 41, 3)
            frames.append(np.clip(g[..., None] + tint, 0, 255).astype(np.uint8))
        else:
            frames.append(rng.integers(0, 256, (H, W, 3), dtype=np.uint8))
    rgb = torch.from_numpy(np.stack(frames)).cuda()
    grey = torch.empty((6, H, W), dtype=torch.uint8, device="cuda")
    cfg = Config(12, 9, NonMaximalSuppression(nms))
    cap = 6 * H * W
    out_a = torch.empty((cap, 2), dtype=torch.int32, device="cuda")
    out_b = torch.empty((cap, 2), dtype=torch.int32, device="cuda")
    offs_a = torch.zeros(7, dtype=torch.int64, device="cuda")
    offs_b = torch.zeros(7, dtype=torch.int64, device="cuda")
    ctx = fast_hip.context(0)
    ctx.set_geometry(geometry)
    try:
        fast_hip.detect_device_rgb(rgb, cfg, out_a, offs_a)
        fast_hip.rgb_to_luma(rgb, grey)
        fast_hip.detect_device(grey, cfg, out_b, offs_b)
        torch.cuda.synchronize()
    finally:
        ctx.set_geometry(0)
    assert torch.equal(offs_a, offs_b)
    n = int(offs_a[-1])
    assert torch.equal(out_a[:n], out_b[:n])
    o = offs_a.cpu().numpy()
    for f in (1, 5):
        want = oracle.detect(oracle.rgb_to_luma(frames[f]), 12, 9, nms)
        assert np.array_equal(out_a[o[f]:o[f + 1]].cpu().numpy().astype(np.uint32), want), f
