"""CPU tests of the checker itself: the scalar oracle (oracle/fast_oracle.c) must reproduce
the reference's golden vectors and unit-test KATs before anything is compared against it;
the AVX2 port (the CPU baseline) must agree with the oracle; and the algebraic
reformulations the HIP kernels rely on are verified here in numpy on the same ground."""
import numpy as np
import pytest

import workloads
from oracle import oracle

CIRCLE = ((0, -3), (1, -3), (2, -2), (3, -1), (3, 0), (3, 1), (2, 2), (1, 3),
          (0, 3), (-1, 3), (-2, 2), (-3, 1), (-3, 0), (-3, -1), (-2, -2), (-1, -3))


# --- golden vectors (tests/golden/, decoded from the reference's media/ overlays) ---------

def test_golden_nms_off(golden):
    img, off, _ = golden
    assert np.array_equal(oracle.detect(img, 16, 9, 0), off)
    assert len(off) == 309


def test_golden_max_threshold(golden):
    img, _, maxt = golden
    assert np.array_equal(oracle.detect(img, 16, 9, 1), maxt)
    assert len(maxt) == 131


@pytest.mark.parametrize("t,n,nms,count", [(16, 9, 2, 135), (16, 12, 2, 80), (32, 12, 2, 16),
                                           (16, 12, 1, 77), (8, 12, 2, 318)])
def test_survey_cross_check_counts(golden, t, n, nms, count):
    """Counts measured by the survey's independent restatement."""
    assert len(oracle.detect(golden[0], t, n, nms)) == count


# --- KATs from the reference's unit tests -------------------------------------------------

HAND_RING = [37, 37, 39, 39, 37, 42, 43, 16, 14, 13, 15, 16, 15, 38, 37, 38]


def test_47_115_score_kat():
    """src/fast_simd.rs:919-948: centre 17 with this ring, n=9 -> max-t score 20."""
    assert oracle.score_max_threshold(17, HAND_RING, 9) == 20
    assert oracle.is_corner(17, HAND_RING, 16, 9)


def test_47_115_hand_detect():
    """src/fast_simd.rs:950-1022: the 128x128 sample image has a keypoint at (64, 64)."""
    img = np.zeros((128, 128), dtype=np.uint8)
    img[64, 64] = 17
    for (dx, dy), v in zip(CIRCLE, HAND_RING):
        img[64 + dy, 64 + dx] = v
    assert [64, 64] in oracle.detect(img, 16, 9, 0).tolist()


def _consecutive(z, k):
    """src/opencv_compat.rs:311-325 (the helper under test there)."""
    n = len(z)
    for s in range(n):
        run = 0
        for i in range(n):
            if not z[(s + i) % n]:
                break
            run += 1
        if run >= k:
            return True
    return False


def test_consecutive_kats():
    """src/opencv_compat.rs:327-345 verbatim vectors."""
    assert not _consecutive([0, 0, 0, 1], 3)
    assert not _consecutive([1, 0, 0, 1], 3)
    assert _consecutive([1, 0, 1, 1], 2)
    assert _consecutive([0, 1, 1, 1], 3)
    assert _consecutive([1, 0, 1, 1], 3)
    assert _consecutive([1, 1, 0, 1], 3)
    assert _consecutive([1, 1, 1, 0], 3)
    assert not _consecutive([1, 0, 0, 0, 1, 0, 0, 1, 0, 0, 1, 0, 0, 1], 3)
    assert _consecutive([1, 0, 0, 0, 1, 0, 0, 1, 0, 0, 1, 1, 1, 1], 4)


def test_oracle_corner_matches_cyclic_helper():
    """The oracle's run test equals the KAT helper on random rings (n = 9..16)."""
    rng = np.random.default_rng(0)
    for _ in range(3000):
        ring = rng.integers(0, 256, 16).tolist()
        c = int(rng.integers(0, 256))
        t = int(rng.integers(0, 80))
        n = int(rng.integers(9, 17))
        bright = [p > c + t for p in ring]
        dark = [p < c - t for p in ring]
        want = _consecutive(bright, n) or _consecutive(dark, n)
        assert oracle.is_corner(c, ring, t, n) == want


def test_sad_score_against_formula():
    """src/fast_simd.rs:1185-1236 (test_score_function_3), on 20k random triples (the GPU's
    fdf_score_points gets 1M+ cases against the oracle in tests/test_gpu_scored.py)."""
    rng = np.random.default_rng(0)
    for _ in range(20000):
        ring = rng.integers(0, 256, 16)
        c = int(rng.integers(0, 256))
        t = int(rng.integers(0, 256))
        light = sum(int(c - p - t) for p in ring if c - p > t)
        dark = sum(int(p - c - t) for p in ring if p - c > t)
        assert oracle.score_sum_abs(c, ring.tolist(), t) == max(light, dark)


# --- the kernels' algebra, checked on the CPU -------------------------------------------

def test_max_threshold_equals_arc_strength():
    """fast_band_kernel scores a keypoint as its arc strength (max_k min_w p - c, or the dark
    mirror), which equals the reference's min(|eh|, |el|) whenever 9 <= n (windows intersect)."""
    rng = np.random.default_rng(1)
    checked = 0
    while checked < 4000:
        ring = rng.integers(0, 256, 16)
        c = int(rng.integers(0, 256))
        t = int(rng.integers(0, 60))
        n = int(rng.integers(9, 17))
        if not oracle.is_corner(c, ring.tolist(), t, n):
            continue
        dark = any(all(ring[(k + i) % 16] < c - t for i in range(n)) for k in range(16))
        q = 255 - ring if dark else ring
        cq = 255 - c if dark else c
        best = max(min(q[(k + i) % 16] for i in range(n)) for k in range(16))
        assert best - cq == oracle.score_max_threshold(c, ring.tolist(), n)
        checked += 1


def _lerp(a, b, r):
    return (a.astype(np.int32) + b.astype(np.int32) + r) >> 1


def test_lerp_byte_comparisons_exact():
    """The pre-filter's v_lerp_u8 comparisons equal X - c > t and X - c < -t for all
    (c, X, t < 255) -- the constants are the ones lerp_consts() computes."""
    c = np.arange(256)[:, None]
    x = np.arange(256)[None, :]
    for t in range(255):
        ob, od = t & 1, (t + 1) & 1
        kb = 128 - ((t + ob) >> 1)
        kd = 255 - ((254 - t + od) >> 1)
        bright = _lerp(_lerp(x, 255 - c, ob), np.full((256, 256), kb), 0) >= 128
        not_dark = _lerp(_lerp(x, 255 - c, od), np.full((256, 256), kd), 0) >= 128
        assert np.array_equal(bright, x > c + t), t
        assert np.array_equal(~not_dark, x < c - t), t


def _prefilter(ring, c, t, n):
    card = [ring[0], ring[4], ring[8], ring[12]]
    b = [p > c + t for p in card]
    d = [p < c - t for p in card]
    if n < 12:
        return ((b[0] or b[2]) and (b[1] or b[3])) or ((d[0] or d[2]) and (d[1] or d[3]))
    return sum(b) >= 3 or sum(d) >= 3


def test_prefilter_is_necessary():
    """Every keypoint passes the (reformulated) cardinal pre-filter of src/fast_simd.rs:441-509."""
    rng = np.random.default_rng(2)
    for _ in range(20000):
        ring = rng.integers(0, 256, 16).tolist()
        c = int(rng.integers(0, 256))
        t = int(rng.integers(0, 60))
        n = int(rng.integers(9, 17))
        if oracle.is_corner(c, ring, t, n):
            assert _prefilter(ring, c, t, n)


# --- error semantics ---------------------------------------------------------------------

@pytest.mark.parametrize("w,h,n,expect", [
    (10, 2, 9, ("err", oracle.ERR_SIZE)), (0, 0, 9, ("err", oracle.ERR_SIZE)),
    (0, 3, 9, ("empty",)), (100, 6, 9, ("empty",)), (5, 7, 9, ("err", oracle.ERR_SIZE)),
    (6, 7, 9, ("empty",)), (7, 7, 9, ("ok",)), (10, 10, 8, ("err", oracle.ERR_COUNT)),
    (10, 10, 17, ("err", oracle.ERR_COUNT))])
def test_reference_size_rules(w, h, n, expect):
    status, empty = oracle.check(w, h, n, 0)
    if expect[0] == "err":
        assert status == expect[1]
    else:
        assert status == 0 and empty == (expect[0] == "empty")


# --- the AVX2 port (CPU baseline) agrees with the oracle ---------------------------------

@pytest.mark.parametrize("nms", [0, 1, 2])
def test_avx2_port_matches_oracle(golden, nms):
    rng = np.random.default_rng(10 + nms)
    imgs = [golden[0], rng.integers(0, 256, (37, 91), dtype=np.uint8),
            workloads.s2_frame(1, 200, 120), workloads.s1_frame(2, 333, 77)]
    for img in imgs:
        for t, n in ((16, 9), (8, 12), (30, 16), (0, 10)):
            assert np.array_equal(oracle.avx2_detect(img, t, n, nms),
                                  oracle.detect(img, t, n, nms)), (img.shape, t, n, nms)


@pytest.mark.parametrize("nms", [0, 1, 2])
def test_avx2_batch_checker_matches_oracle(nms):
    """The whole-batch checker bench.py and the batch parity tests use (the AVX2 port over a
    thread pool) equals the scalar oracle frame by frame, in frame order, on the bench's own
    shapes: S1 1080p t=16 n=9 and S1 4K t=8 n=12 (configs 4 and 5), plus dense noise."""
    cases = [(np.stack([workloads.s1_frame(i) for i in (0, 211, 422)]), 16, 9),
             (np.stack([workloads.s3_frame(i, 300, 200) for i in range(5)]), 16, 9),
             (workloads.s1_frame(5, 3840, 2160)[None], 8, 12)]
    for frames, t, n in cases:
        pts, offs = oracle.avx2_detect_batch(frames, t, n, nms, threads=3)
        assert offs[0] == 0 and offs[-1] == len(pts)
        for f in range(frames.shape[0]):
            want = oracle.detect(frames[f], t, n, nms)
            assert np.array_equal(pts[offs[f]:offs[f + 1]], want), (frames.shape, f, nms)


# --- synthetic workload generators (SURVEY.md §8d counts) --------------------------------

def test_s1_1080p_counts():
    img = workloads.s1_frame(0)
    assert img.shape == (1080, 1920)
    assert len(oracle.detect(img, 16, 9, 0)) == 10346
    assert len(oracle.detect(img, 16, 9, 1)) == 4332


def test_s2_1080p_counts():
    img = workloads.s2_frame(0)
    assert len(oracle.detect(img, 16, 9, 0)) == 30877
    assert len(oracle.detect(img, 16, 9, 1)) == 5426
    assert len(oracle.detect(img, 16, 12, 0)) == 0


def _lane_segment_test(c, ring, t, n, rng=None):
    """numpy restatement of fdf_common.h lane_segment_test_packed: bytes packed 4 per word
    (byte j of word m = pixel 4j + m), lerp SWAR compares (only bit 7 of each byte is a flag;
    the other bits are filled with noise here, as the lerps leave them), each polarity's flags
    gathered by masked bitop3 selects (gather_ring; the dark side inverted in the tables), the
    two rings joined into one word by v_perm (bright bits 0-15, dark 16-31), then the run test
    of both rings at once with packed 16-bit rotations (runs16x2)."""
    ob, od = t & 1, (t + 1) & 1
    kb = 128 - ((t + ob) >> 1)
    kd = 255 - ((254 - t + od) >> 1)
    ring = np.asarray(ring)
    M = 0xffffffff

    def word_flags(r, k):
        fl = [0, 0, 0, 0]
        for m in range(4):
            for j in range(4):
                v = _lerp(_lerp(np.array(ring[4 * j + m]), np.array(255 - c), r), np.array(k), 0)
                noise = int(rng.integers(0, 128)) if rng is not None else 0
                fl[m] |= ((int(v) & 0x80) | noise) << (8 * j)
        return fl

    def sel(s, a, b):
        return ((s & a) | (~s & b)) & M

    def gather_ring(f, inv):
        g = (lambda x: ~x & M) if inv else (lambda x: x)
        tt = g(f[3]) & 0x80808080
        tt = sel(0x40404040, g(f[2] >> 1), tt)
        tt = sel(0x20202020, g(f[1] >> 2), tt)
        tt = sel(0x10101010, g(f[0] >> 3), tt)
        return (tt | (tt << 4)) & M

    def rot16x2(m, sh):
        r = lambda v: ((v >> sh) | (v << (16 - sh))) & 0xffff
        return r(m & 0xffff) | (r(m >> 16) << 16)

    def runs16x2(m):
        for sh in [1, 2, 4] + ([n - 8] if n > 8 else []):
            m = m & (rot16x2(m, sh))
        return m

    rings = _perm(gather_ring(word_flags(od, kd), True), gather_ring(word_flags(ob, kb), False),
                  0x07050301)
    m = runs16x2(rings)
    return (m & 0xffff) != 0, m > 0xffff


def test_lane_segment_test_matches_oracle():
    """The sweep kernel's per-lane segment test equals the reference's run test."""
    rng = np.random.default_rng(5)
    for k in range(4000):
        c = int(rng.integers(0, 256))
        t = int(rng.integers(0, 255))
        n = int(rng.integers(9, 17))
        if k % 2:   # bias towards corners: a long arc of one polarity
            ring = rng.integers(0, 256, 16)
            s0, ln = int(rng.integers(0, 16)), int(rng.integers(n - 1, 17))
            hi = rng.integers(min(c + t + 1, 255), 256, ln) if rng.integers(2) else rng.integers(0, max(c - t, 1), ln)
            for q in range(ln):
                ring[(s0 + q) % 16] = hi[q]
        else:
            ring = rng.integers(0, 256, 16)
        b, d = _lane_segment_test(c, ring.tolist(), t, n, rng)
        bright = [p > c + t for p in ring]
        dark = [p < c - t for p in ring]
        assert b == _consecutive(bright, n) and d == _consecutive(dark, n), (c, t, n, ring)


def _perm(hi, lo, sel):
    """v_perm_b32: byte k of the result = byte sel_k of {hi:lo} (0-3 lo, 4-7 hi), 0x0c -> 0."""
    src = [(lo >> (8 * i)) & 0xff for i in range(4)] + [(hi >> (8 * i)) & 0xff for i in range(4)]
    out = 0
    for k in range(4):
        s = (sel >> (8 * k)) & 0xff
        out |= (src[s] if s < 8 else 0) << (8 * k)
    return out


def test_sweep_gather_windows_pack_the_circle():
    """fdf_sweep.hip issue_batch + pack_ring: 7 row windows (4 B from x-1 at y+-3, 8 B from
    x-2 at y+-2, 8 B from x-3 at y-1..y+1) permuted into the 4 compare words, byte j of
    word m = circle pixel 4j + m, and the centre."""
    rng = np.random.default_rng(7)
    img = rng.integers(0, 256, (20, 24), dtype=np.uint8)
    flat = img.reshape(-1).astype(np.int64)
    W = img.shape[1]

    def word(o):
        return int(sum(int(flat[o + i]) << (8 * i) for i in range(4)))

    for y in range(3, 17):
        for x in range(3, 21):
            o = (y - 3) * W + x
            a0, a6 = word(o - 1), word(o - 1 + 6 * W)
            a1 = (word(o - 2 + W), word(o - 2 + W + 4))
            a2 = (word(o - 3 + 2 * W), word(o - 3 + 2 * W + 4))
            a3 = (word(o - 3 + 3 * W), word(o - 3 + 3 * W + 4))
            a4 = (word(o - 3 + 4 * W), word(o - 3 + 4 * W + 4))
            a5 = (word(o - 2 + 5 * W), word(o - 2 + 5 * W + 4))
            w = [_perm(a3[1], a0, 0x0c0c0601) | _perm(a3[0], a6, 0x04010c0c),
                 _perm(a4[1], a0, 0x0c0c0602) | _perm(a2[0], a6, 0x04000c0c),
                 _perm(a1[1], a1[0], 0x000c0c04) | _perm(a5[1], a5[0], 0x0c00040c),
                 _perm(a6, a2[1], 0x0c0c0602) | _perm(a0, a4[0], 0x04000c0c)]
            for i, (dx, dy) in enumerate(CIRCLE):
                assert (w[i & 3] >> (8 * (i >> 2))) & 0xff == img[y + dy, x + dx], (x, y, i)
            assert a3[0] >> 24 == img[y, x]


def test_luma_restatement():
    """fdf_oracle_rgb_to_luma == image 0.24.6's integer formula; identity on grey pixels
    (the reference's media image is grey, r = g = b, so its detections are pinned)."""
    rng = np.random.default_rng(3)
    rgb = rng.integers(0, 256, (17, 23, 3), dtype=np.uint8)
    r, g, b = (rgb[..., k].astype(np.uint32) for k in range(3))
    want = ((2126 * r + 7152 * g + 722 * b) // 10000).astype(np.uint8)
    assert np.array_equal(oracle.rgb_to_luma(rgb), want)
    v = np.arange(256, dtype=np.uint8)
    assert np.array_equal(oracle.rgb_to_luma(np.stack([v, v, v], -1)[None]), v[None])


def test_cli_helpers_without_gpu(tmp_path):
    """cli.py host helpers: the overlay luma equals the restated formula, keypoint pixels go
    red except at x <= 0 / y <= 0 (draw_plus_sized), and the .txt format is "x y" lines."""
    from feature_detector_fast_amd import cli

    rng = np.random.default_rng(4)
    rgb = rng.integers(0, 256, (9, 11, 3), dtype=np.uint8)
    assert np.array_equal(cli.luma8(rgb), oracle.rgb_to_luma(rgb))
    grey = oracle.rgb_to_luma(rgb)
    pts = np.array([[3, 4], [0, 5], [10, 8]], dtype=np.uint32)
    ov = cli.overlay(grey, pts)
    assert tuple(ov[4, 3]) == (255, 0, 0) and tuple(ov[8, 10]) == (255, 0, 0)
    assert tuple(ov[5, 0]) == (grey[5, 0],) * 3
    f = tmp_path / "k.txt"
    cli.write_keypoints(pts, str(f))
    assert f.read_text() == "3 4\n0 5\n10 8\n"
    assert np.array_equal(workloads.read_points(str(f)), pts)
    assert cli.main(["--help"]) == 0


def _sad_u8(a, b, acc):
    """v_sad_u8: acc + sum over the 4 bytes of |a.byte - b.byte| (uint32 arrays)."""
    tot = acc.astype(np.int64)
    for k in range(4):
        tot += np.abs(((a >> (8 * k)) & 0xFF).astype(np.int64) - ((b >> (8 * k)) & 0xFF).astype(np.int64))
    return tot.astype(np.uint32)


def test_sad_score_packed_identity():
    """fdf_common.h score_sum_abs_packed: the SAD score from 12 v_sad_u8 on the packed ring
    equals the reference's SAD score (src/opencv_compat.rs:278-299) for random rings, all t,
    including the saturating ends (c + t > 255, c < t)."""
    rng = np.random.default_rng(5)
    m = 200000
    ring = rng.integers(0, 256, (m, 16)).astype(np.int64)
    c = rng.integers(0, 256, m).astype(np.int64)
    near = rng.integers(0, 2, m).astype(bool)          # half the rings close to the centre
    ring[near] = np.clip(c[near, None] + rng.integers(-30, 31, (near.sum(), 16)), 0, 255)
    t = rng.integers(0, 256, m).astype(np.int64)
    w = [np.zeros(m, dtype=np.uint32) for _ in range(4)]
    for i in range(16):                                 # byte j of w[k] = pixel 4j + k
        w[i & 3] |= (ring[:, i].astype(np.uint32) << np.uint32(8 * (i >> 2)))
    U = np.minimum(c + t, 255).astype(np.uint32)
    L = np.where(c > t, c - t, 0).astype(np.uint32)
    su = sl = sp = np.zeros(m, dtype=np.uint32)
    for k in range(4):
        su = _sad_u8(w[k], U * np.uint32(0x01010101), su)
        sl = _sad_u8(w[k], L * np.uint32(0x01010101), sl)
        sp = _sad_u8(w[k], np.zeros(m, dtype=np.uint32), sp)
    su, sl, sp = su.astype(np.int64), sl.astype(np.int64), sp.astype(np.int64)
    got = np.maximum((su + sp - 16 * U) >> 1, (sl + 16 * L - sp) >> 1)
    sb = np.maximum(ring - (c + t)[:, None], 0).sum(1)
    sd = np.maximum((c - t)[:, None] - ring, 0).sum(1)
    assert np.array_equal(got, np.maximum(sb, sd))
    for k in range(0, m, 20000):                        # and the literal oracle, sampled
        assert got[k] == oracle.score_sum_abs(int(c[k]), ring[k].tolist(), int(t[k]))


def test_rowdiv_multiply_high_division():
    """fdf_common.h RowDiv / udiv: q = hi32(x * m) with m = 0xffffffff // d + 1 (= ceil(2^32 / d)),
    then q -= (q * d > x), equals x // d for every x < 2^24 and d >= 2 (d = 1: m = 0 -> x).
    Exhaustive over x < 4d + 10 for d < 5000 (all remainders), random x < 2^24 and large d."""
    rng = np.random.default_rng(11)
    divisors = list(range(1, 5000)) + rng.integers(5000, 1 << 20, 500).tolist() + [65535, 65536, 1 << 20]
    for d in divisors:
        x = np.concatenate([np.arange(0, min(1 << 24, 4 * d + 10), dtype=np.uint64),
                            rng.integers(0, 1 << 24, 2000, dtype=np.uint64),
                            np.array([(1 << 24) - 1], dtype=np.uint64)])
        m = (0xffffffff // d + 1) if d >= 2 else 0
        if m == 0:
            q = x
        else:
            q = (x * np.uint64(m)) >> np.uint64(32)
            q = q - ((q * np.uint64(d)) > x).astype(np.uint64)
        assert np.array_equal(q, x // np.uint64(d)), d


def test_byte_broadcast_and_partial_entry_mask():
    """fdf_common.h bcast_byte (v_perm selector 0: byte 0 of the low source in all four bytes)
    equals c * 0x01010101; the issue's partial FIFO entry keeps the bits above batch lane 63's
    selected bit, which equals clearing below the (64 - excl)-th set bit (the old select)."""
    for c in range(256):
        perm = sum(c << (8 * k) for k in range(4))
        assert perm == c * 0x01010101
    rng = np.random.default_rng(12)

    def select_bit(m, j):                 # position of the j-th set bit (fdf_sweep_impl.h)
        return [b for b in range(16) if (m >> b) & 1][j]

    for _ in range(20000):
        m = int(rng.integers(1, 1 << 16))
        k = bin(m).count("1")
        taken = int(rng.integers(1, k)) if k > 1 else 0   # bits of the entry in this batch
        if taken == 0:
            continue
        last = select_bit(m, taken - 1)                    # batch lane 63's bit
        new = m & ((~0 << (last + 1)) & 0xffffffff)
        old = m & ((~0 << select_bit(m, taken)) & 0xffffffff)
        assert new == old


def test_rust_default_hasher():
    """workloads.siphash: SipHash-2-4's published vectors (key 00..0f; messages of 0 and 15
    bytes), so the SipHash-1-3 of Rust's DefaultHasher (tests/compare.rs:5-20 hash guard)
    runs the same code with fewer rounds; and the byte stream `Hash` writes for &[u8] and
    &[Point] (length as a LE usize, then the elements)."""
    k0 = int.from_bytes(bytes(range(8)), "little")
    k1 = int.from_bytes(bytes(range(8, 16)), "little")
    assert workloads.siphash(b"", 2, 4, k0, k1) == 0x726FDB47DD0E0E31
    assert workloads.siphash(bytes(range(15)), 2, 4, k0, k1) == 0xA129CA6149BE45E5
    pts = np.array([[3, 4], [70000, 5]], dtype=np.uint32)
    stream = (2).to_bytes(8, "little") + b"".join(int(v).to_bytes(4, "little") for v in pts.reshape(-1))
    assert workloads.rust_hash_points(pts) == workloads.siphash(stream)
    assert workloads.rust_hash_bytes(b"\x01\x02") == workloads.siphash((2).to_bytes(8, "little") + b"\x01\x02")


def test_input_image_is_compare_rs_luma(tmp_path):
    """An INPUT_FILE goes through to_rgb8 and to_luma8 as tests/compare.rs:29-33 does: the
    golden grey fixture written as PNG comes back unchanged (r = g = b), and a colour PNG
    gives image 0.24.6's integer luma."""
    from PIL import Image

    g = workloads.golden_image()
    p = tmp_path / "grey.png"
    Image.fromarray(g).save(p)
    grey, rgb = workloads.input_image(str(p))
    assert np.array_equal(grey, g) and rgb.shape == g.shape + (3,)
    rng = np.random.default_rng(5)
    col = rng.integers(0, 256, (20, 30, 3), dtype=np.uint8)
    p2 = tmp_path / "col.png"
    Image.fromarray(col).save(p2)
    grey2, _ = workloads.input_image(str(p2))
    assert np.array_equal(grey2, oracle.rgb_to_luma(col))


def test_load_rgb_rejects_wide_modes(tmp_path):
    """a 16-bit PNG is not silently clipped to 8 bits (image 0.24's to_rgb8
    scales it); load_rgb refuses modes other than 8-bit channels."""
    from PIL import Image

    p = tmp_path / "wide.png"
    Image.fromarray(np.arange(64 * 48, dtype=np.uint16).reshape(48, 64) * 20, mode="I;16").save(p)
    with pytest.raises(ValueError, match="8-bit"):
        workloads.load_rgb(str(p))
    q = tmp_path / "grey.png"
    Image.fromarray(np.arange(64 * 48, dtype=np.uint8).reshape(48, 64)).save(q)
    rgb = workloads.load_rgb(str(q))
    assert rgb.shape == (48, 64, 3) and np.array_equal(rgb[..., 0], rgb[..., 2])


def test_three_of_four_prefilter_tables():
    """fdf_sweep_impl.h, n >= 12: the 3-of-4 cardinal pre-filter as six v_bitop3 on the raw
    flag words (and3 | maj3 & w for bright; maj3 | or3 & w for not-dark, inversions in the
    tables) equals the reference's formula (src/fast_simd.rs:441-509) bit for bit."""
    M = 0xffffffff

    def lut3(f):
        return sum(1 << i for i in range(8) if f((i >> 2) & 1, (i >> 1) & 1, i & 1))

    def bitop3(a, b, c, lut):
        out = 0
        for bit in range(32):
            i = (((a >> bit) & 1) << 2) | (((b >> bit) & 1) << 1) | ((c >> bit) & 1)
            out |= ((lut >> i) & 1) << bit
        return out

    k_maj = lut3(lambda a, b, c: (1 - a + b + c) >= 2)
    k_and = lut3(lambda a, b, c: (not a) and b and c)
    k_or = lut3(lambda a, b, c: (not a) or b or c)
    k_join = lut3(lambda a, b, c: a or (b and not c))
    rng = np.random.default_rng(11)
    for _ in range(300):
        vn_nd, vs_b, h_b, hndw, vn_b, vs_nd, h_nd, hbw = (int(v) for v in rng.integers(0, 1 << 32, 8))
        bn, bs, be, bw = ~vn_nd & M, vs_b, h_b, ~hndw & M
        dn, ds, de, dw = ~vn_b & M, vs_nd, h_nd, ~hbw & M
        br_ref = (bn & bs & (be | bw)) | (be & bw & (bn | bs))
        nd_ref = (dn & ds) | (de & dw) | ((dn | ds) & (de | dw))
        m1 = bitop3(vn_nd, vs_b, h_b, k_maj)
        t1 = bitop3(vn_nd, vs_b, h_b, k_and)
        br = bitop3(t1, m1, hndw, k_join)
        m2 = bitop3(vn_b, vs_nd, h_nd, k_maj)
        o2 = bitop3(vn_b, vs_nd, h_nd, k_or)
        nd = bitop3(m2, o2, hbw, k_join)
        assert br == br_ref and nd == nd_ref
