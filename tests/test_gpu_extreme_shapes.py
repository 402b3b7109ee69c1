"""Frames far from the benchmark's shapes, on the device and the host path: 8K UHD, rows of
tens of thousands of pixels (the bitmap row is then most of a band's LDS: bands of 1-3 rows,
one sub-band, the score list's 20-bit positions past their range), and frames a few pixels
wide and tens of thousands of rows tall (one strip with mostly halo lanes).  The reference
takes any image of h >= 7, w >= 7 (src/fast_simd.rs:307-330); every list here equals the CPU
checker's over the whole frame (oracle.avx2_detect_batch, the AVX2 port pinned to the scalar
oracle by tests/test_oracle.py)."""
import numpy as np
import pytest

import workloads
from feature_detector_fast_amd import Config, NonMaximalSuppression, fast_hip
from oracle import oracle

pytestmark = pytest.mark.gpu

SHAPES = [
    ("s1", 7680, 4320),     # 8K UHD
    ("s3", 16384, 40),      # wide: 2 KB bitmap rows
    ("s3", 40000, 12),
    ("s3", 65535, 9),       # the widest row a 16-bit x holds
    ("s3", 7, 20000),       # one centre column
    ("s3", 16, 16384),
    ("s1", 33, 9000),
]


def _frame(kind, w, h):
    if kind == "s1":
        return np.ascontiguousarray(workloads.s1_frame(3, w, h))
    return workloads.s3_frame(w * 7 + h, w, h)


def _want(img, t, n, nms):
    pts, offs = oracle.avx2_detect_batch(img[None], t, n, nms)
    assert int(offs[-1]) == len(pts)
    if img.size <= 1 << 20:      # small enough for the scalar oracle itself
        assert np.array_equal(oracle.detect(img, t, n, nms), pts)
    return pts


@pytest.mark.parametrize("kind,w,h", SHAPES)
@pytest.mark.parametrize("nms", [0, 1, 2])
def test_extreme_shapes_device(kind, w, h, nms):
    import torch

    img = _frame(kind, w, h)
    t, n = (16, 9) if kind == "s1" else (40, 9)
    want = _want(img, t, n, nms)
    frames = torch.from_numpy(img).cuda().unsqueeze(0).contiguous()
    out = torch.empty((max(len(want), 1) + 64, 2), dtype=torch.int32, device="cuda")
    offs = torch.zeros(2, dtype=torch.int64, device="cuda")
    fast_hip.detect_device(frames, Config(t, n, NonMaximalSuppression(nms)), out, offs)
    torch.cuda.synchronize()
    k = int(offs[1].item())
    assert k == len(want), (w, h, nms, k, len(want))
    assert np.array_equal(out[:k].cpu().numpy().astype(np.uint32), want)


@pytest.mark.parametrize("kind,w,h", SHAPES)
def test_extreme_shapes_host(kind, w, h):
    img = _frame(kind, w, h)
    for nms in (0, 1, 2):
        t, n = (16, 9) if kind == "s1" else (40, 9)
        got = fast_hip.detect_array(img, Config(t, n, NonMaximalSuppression(nms)))
        assert np.array_equal(got, _want(img, t, n, nms)), (w, h, nms)


def test_8k_config5_settings():
    """8K at config 5's settings (t=8 n=12 SAD): dense bands, every NMS tier."""
    img = _frame("s1", 7680, 4320)
    for nms in (2, 1):
        got = fast_hip.detect_array(img, Config(8, 12, NonMaximalSuppression(nms)))
        assert np.array_equal(got, _want(img, 8, 12, nms)), nms
