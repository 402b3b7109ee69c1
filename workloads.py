"""Synthetic frame generators for tests and bench.py, integer-only and
reproducible.  Nothing here reads /root/reference: S1 tiles the committed golden fixture.

S1 "tiled media": the 300x200 grey fixture tiled to W x H; frame i rolled by
    (dx, dy) = ((37 i) % 300, (53 i) % 200):  out[y][x] = g[(y + dy) % 200][(x + dx) % 300].
S2 "blocks+noise": SplitMix64 24x24 blocks plus 3-bit noise, seed = frame index.
S3 "uniform": uniform u8 from numpy's PCG64 (a stress case: ~28% keypoints at t=16 n=9).
"""
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tests", "golden")


def read_pgm(path):
    with open(path, "rb") as f:
        data = f.read()
    parts = data.split(maxsplit=4)
    assert parts[0] == b"P5" and parts[3] == b"255"
    w, h = int(parts[1]), int(parts[2])
    px = np.frombuffer(parts[4][: w * h], dtype=np.uint8)
    return px.reshape(h, w).copy()


def read_points(path):
    pts = np.loadtxt(path, dtype=np.uint32, ndmin=2)
    return pts.reshape(-1, 2)


def golden_image():
    return read_pgm(os.path.join(GOLDEN, "screenshot315_grey.pgm"))


def s1_roll(i):
    return (37 * i) % 300, (53 * i) % 200


def s1_frame(i, w=1920, h=1080, base=None):
    g = golden_image() if base is None else base
    dx, dy = s1_roll(i)
    ys = (np.arange(h) + dy) % g.shape[0]
    xs = (np.arange(w) + dx) % g.shape[1]
    return g[ys[:, None], xs[None, :]]


def s1_frames_torch(first, count, w=1920, h=1080, device="cuda"):
    """S1 frames [first, first+count) built on the GPU (no host copy of the batch)."""
    import torch

    g = torch.from_numpy(golden_image()).to(device)
    out = torch.empty((count, h, w), dtype=torch.uint8, device=device)
    ar_y = torch.arange(h, device=device)
    ar_x = torch.arange(w, device=device)
    for k in range(count):
        dx, dy = s1_roll(first + k)
        out[k] = g[((ar_y + dy) % g.shape[0])[:, None], ((ar_x + dx) % g.shape[1])[None, :]]
    return out


_GOLDEN_GAMMA = np.uint64(0x9E3779B97F4A7C15)


def _mix(z):
    z = z.astype(np.uint64)
    z ^= z >> np.uint64(30)
    z *= np.uint64(0xBF58476D1CE4E5B9)
    z ^= z >> np.uint64(27)
    z *= np.uint64(0x94D049BB133111EB)
    z ^= z >> np.uint64(31)
    return z


def _sm(seed, k):
    with np.errstate(over="ignore"):
        return _mix(np.uint64(seed) + (k.astype(np.uint64) + np.uint64(1)) * _GOLDEN_GAMMA)


def s2_frame(seed, w=1920, h=1080):
    bw = -(-w // 24)
    bh = -(-h // 24)
    blocks = (_sm(seed, np.arange(bh * bw, dtype=np.uint64)) >> np.uint64(56)).reshape(bh, bw)
    idx = np.arange(h * w, dtype=np.uint64)
    noise = (_sm(np.uint64(seed) ^ np.uint64(0xA5A5A5A5), idx) >> np.uint64(61)).reshape(h, w)
    ys = np.arange(h) // 24
    xs = np.arange(w) // 24
    base = blocks[ys[:, None], xs[None, :]]
    return np.minimum(base + noise, 255).astype(np.uint8)


def s3_frame(seed, w=1920, h=1080):
    return np.random.Generator(np.random.PCG64(seed)).integers(0, 256, (h, w), dtype=np.uint8)
