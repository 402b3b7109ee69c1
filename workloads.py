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


# ---- inputs given by file (the reference's INPUT_FILE, tests/compare.rs:24-33) ---------------

# PIL modes whose conversion to RGB8 is the same as image 0.24's to_rgb8 (8-bit channels:
# grey is replicated, alpha dropped, a palette looked up).  16-bit and float images are scaled
# by image 0.24 and clipped by PIL's convert('RGB'), so they are refused rather than detected
# on different luma.
_RGB8_MODES = ("1", "L", "LA", "P", "PA", "RGB", "RGBA", "RGBX")


def load_rgb(path):
    """An image file as RGB8 (H, W, 3), as `image::open(..).to_rgb8()` (tests/compare.rs:29-31).
    PNG / PGM / anything PIL reads with 8-bit channels; a grey file becomes r = g = b."""
    from PIL import Image

    with Image.open(path) as im:
        if im.mode not in _RGB8_MODES:
            raise ValueError(f"{path}: PIL mode {im.mode!r} is not an 8-bit-per-channel image; "
                             "its conversion to RGB8 would differ from image 0.24's to_rgb8")
        return np.asarray(im.convert("RGB")).copy()


def luma8(rgb):
    """image 0.24.6 to_luma8 on Rgb<u8>: (2126 r + 7152 g + 722 b) / 10000, integer."""
    r, g, b = (rgb[..., k].astype(np.uint32) for k in range(3))
    return ((2126 * r + 7152 * g + 722 * b) // 10000).astype(np.uint8)


def input_image(path):
    """(grey, rgb) of an INPUT_FILE: `DynamicImage::ImageRgb8(rgb).to_luma8()` (compare.rs:33)."""
    rgb = load_rgb(path)
    return luma8(rgb), rgb


# Rust's std DefaultHasher (SipHash-1-3, keys 0, 0) over the byte stream `Hash` writes: a slice
# writes its length as a usize (8 bytes LE), then u8 elements as raw bytes, Point {x, y} as two
# u32 (LE).  tests/compare.rs:5-20 hashes the RGB bytes and the max-t keypoints this way.
_M64 = (1 << 64) - 1


def _rotl(x, b):
    return ((x << b) | (x >> (64 - b))) & _M64


def siphash(data, c_rounds=1, d_rounds=3, k0=0, k1=0):
    v0 = k0 ^ 0x736F6D6570736575
    v1 = k1 ^ 0x646F72616E646F6D
    v2 = k0 ^ 0x6C7967656E657261
    v3 = k1 ^ 0x7465646279746573

    def rnd(v0, v1, v2, v3):
        v0 = (v0 + v1) & _M64; v1 = _rotl(v1, 13); v1 ^= v0; v0 = _rotl(v0, 32)
        v2 = (v2 + v3) & _M64; v3 = _rotl(v3, 16); v3 ^= v2
        v0 = (v0 + v3) & _M64; v3 = _rotl(v3, 21); v3 ^= v0
        v2 = (v2 + v1) & _M64; v1 = _rotl(v1, 17); v1 ^= v2; v2 = _rotl(v2, 32)
        return v0, v1, v2, v3

    data = bytes(data)
    n = len(data)
    tail = n & ~7
    words = np.frombuffer(data[:tail], dtype="<u8").tolist() if tail else []
    last = int.from_bytes(data[tail:] + bytes(8 - (n - tail)), "little") & ((1 << 56) - 1)
    words.append(last | ((n & 0xFF) << 56))
    for i, m in enumerate(words):
        v3 ^= m
        for _ in range(c_rounds):
            v0, v1, v2, v3 = rnd(v0, v1, v2, v3)
        v0 ^= m
    v2 ^= 0xFF
    for _ in range(d_rounds):
        v0, v1, v2, v3 = rnd(v0, v1, v2, v3)
    return v0 ^ v1 ^ v2 ^ v3


def rust_hash_bytes(buf):
    """`DefaultHasher` of a &[u8] (compare.rs:13-20 hash_slice_u8)."""
    b = bytes(buf) if isinstance(buf, (bytes, bytearray)) else \
        np.ascontiguousarray(buf, dtype=np.uint8).tobytes()
    return siphash(len(b).to_bytes(8, "little") + b)


def rust_hash_points(points):
    """`DefaultHasher` of a &[Point] (compare.rs:5-12 hash_result)."""
    p = np.ascontiguousarray(np.asarray(points, dtype="<u4").reshape(-1, 2))
    return siphash(p.shape[0].to_bytes(8, "little") + p.tobytes())


# compare.rs:83-89: on the reference's own test image (RGB bytes hashing to REF_IMAGE_HASH) the
# max-t t=16 n=9 keypoints must hash to REF_MAXT_HASH
REF_IMAGE_HASH = 0x8444A9356505ECAB
REF_MAXT_HASH = 0x8BF9CD0F9CA9EBEC


def kernel_source_sha16():
    """sha256 (16 hex digits) of the detector's sources: the kernels, the host layer and the
    C ABI header.  Profiles stamped with it (profiles/pmc_traffic.json) are stale once the
    sources change."""
    import hashlib

    root = os.path.dirname(os.path.abspath(__file__))
    csrc = os.path.join(root, "feature_detector_fast_amd", "csrc")
    h = hashlib.sha256()
    files = sorted(f for f in os.listdir(csrc) if f.endswith((".h", ".hip", ".cpp")))
    for f in files + ["../../include/fdf.h"]:
        with open(os.path.normpath(os.path.join(csrc, f)), "rb") as fh:
            h.update(f.encode() + b"\0" + fh.read())
    return h.hexdigest()[:16]
