"""fdf_detect on a frame in pinned host memory: the detector reads it in place over PCIe (no
copy before the launch; fdf_ctx_set_upload_chunks, include/fdf.h).

The buffer is reused across calls with different contents -- an L2 line cached from the
previous call's frame would show as a wrong list (the launch's system-scope acquire must make
the host's writes visible) -- at an aligned and an odd offset inside the allocation, and every list
equals the CPU oracle (oracle/fast_oracle.c, pinned to the reference's goldens; the image
contract is src/fast_simd.rs:307-330).  The two-call pattern keeps the frame for
fdf_fetch_last's scores; a result that fit asks for fdf_detect_scored instead."""
import ctypes
import json
import os

import numpy as np
import pytest

import workloads
from feature_detector_fast_amd import _native
from oracle import oracle

pytestmark = pytest.mark.gpu


def _pinned(nbytes):
    import torch

    return torch.empty(nbytes, dtype=torch.uint8).pin_memory()


def _detect(lib, ctx, ptr, w, h, t, n, nms, cap=None):
    cfg = _native.FdfConfig(t, n, nms)
    cap = w * h if cap is None else cap
    out = np.zeros((max(cap, 1), 2), dtype=np.uint32)
    got = ctypes.c_size_t(0)
    rc = lib.fdf_detect(ctx.handle, ctypes.c_void_p(ptr), w, h, w, ctypes.byref(cfg),
                        out.ctypes.data if cap else None, cap, ctypes.byref(got))
    return rc, out[: min(got.value, cap)], got.value


@pytest.mark.parametrize("offset", [0, 4096 + 13])
def test_in_place_frames_alternate(offset):
    W, H = 1920, 1080
    frames = [workloads.s1_frame(31), workloads.s3_frame(12), workloads.s2_frame(9),
              workloads.s1_frame(77)]
    buf = _pinned(W * H + 8192)
    view = buf.numpy()
    lib = _native.load()
    ctx = _native.Context(0)
    try:
        for rep in range(2):
            for i, f in enumerate(frames):
                nms = (i + rep) % 3
                view[offset: offset + W * H] = f.reshape(-1)
                rc, got, _ = _detect(lib, ctx, buf.data_ptr() + offset, W, H, 16, 9, nms)
                _native.check(rc, "fdf_detect")
                assert np.array_equal(got, oracle.detect(f, 16, 9, nms)), (rep, i, nms)
        # the same frames through one copy (chunks = 1) give the same lists
        ctx.set_upload_chunks(1)
        view[offset: offset + W * H] = frames[1].reshape(-1)
        rc, got, _ = _detect(lib, ctx, buf.data_ptr() + offset, W, H, 16, 9, 1)
        _native.check(rc, "fdf_detect")
        assert np.array_equal(got, oracle.detect(frames[1], 16, 9, 1))
    finally:
        ctx.close()


def test_in_place_small_and_ragged_frames():
    lib = _native.load()
    ctx = _native.Context(0)
    try:
        for (w, h) in [(7, 7), (33, 20), (641, 479), (1000, 7)]:
            img = workloads.s3_frame(5)[:h, :w].copy()
            buf = _pinned(w * h)
            buf.numpy()[:] = img.reshape(-1)
            for nms in (0, 1, 2):
                rc, got, _ = _detect(lib, ctx, buf.data_ptr(), w, h, 16, 9, nms)
                _native.check(rc, "fdf_detect")
                assert np.array_equal(got, oracle.detect(img, 16, 9, nms)), (w, h, nms)
    finally:
        ctx.close()


def test_in_place_two_call_pattern_keeps_scores():
    """cap 0 -> FDF_ERR_CAPACITY; fdf_fetch_last then returns the points and their scores (the
    frame was copied for it).  A result that fit has no retained frame: scores -> FDF_ERR_ARG,
    points still fine."""
    W, H = 640, 480
    img = workloads.s1_frame(1, W, H)
    want, want_sc = oracle.detect(img, 16, 9, 1, with_scores=True)
    buf = _pinned(W * H)
    buf.numpy()[:] = img.reshape(-1)
    lib = _native.load()
    ctx = _native.Context(0)
    try:
        rc, _, n = _detect(lib, ctx, buf.data_ptr(), W, H, 16, 9, 1, cap=0)
        assert rc == _native.FDF_ERR_CAPACITY and n == len(want)
        buf.numpy()[:] = 0          # the caller may reuse its buffer after the call
        out = np.zeros((n, 2), dtype=np.uint32)
        sc = np.zeros(n, dtype=np.uint16)
        got = ctypes.c_size_t(0)
        _native.check(lib.fdf_fetch_last(ctx.handle, out.ctypes.data, sc.ctypes.data, n,
                                         ctypes.byref(got)), "fdf_fetch_last")
        assert np.array_equal(out, want) and np.array_equal(sc, want_sc)

        buf.numpy()[:] = img.reshape(-1)
        rc, pts, n = _detect(lib, ctx, buf.data_ptr(), W, H, 16, 9, 1)
        _native.check(rc, "fdf_detect")
        assert np.array_equal(pts, want)
        assert lib.fdf_fetch_last(ctx.handle, out.ctypes.data, sc.ctypes.data, n,
                                  ctypes.byref(got)) == _native.FDF_ERR_ARG
        out[:] = 0
        _native.check(lib.fdf_fetch_last(ctx.handle, out.ctypes.data, None, n,
                                         ctypes.byref(got)), "fdf_fetch_last")
        assert np.array_equal(out, want)
    finally:
        ctx.close()


def _hip():
    """The HIP runtime already in the process (the one libfdf.so and torch use), never a
    second copy."""
    import os

    _native.load()
    hip = ctypes.CDLL("libamdhip64.so.7", mode=os.RTLD_NOLOAD | os.RTLD_NOW)
    for fn in ("hipHostMalloc", "hipHostFree"):
        getattr(hip, fn).restype = ctypes.c_int
    return hip


def test_in_place_coherent_pinned_is_copied():
    """Fine-grained (coherent) pinned memory is copied, not read in place; the lists equal the
    oracle across frames written into the same buffer."""
    W, H = 1280, 720
    frames = [workloads.s1_frame(3, W, H), workloads.s3_frame(7)[:H, :W].copy(),
              workloads.s1_frame(40, W, H)]
    hip = _hip()
    ptr = ctypes.c_void_p()
    assert hip.hipHostMalloc(ctypes.byref(ptr), ctypes.c_size_t(W * H),
                             ctypes.c_uint(0x40000000)) == 0
    view = np.ctypeslib.as_array(ctypes.cast(ptr, ctypes.POINTER(ctypes.c_uint8)), (W * H,))
    lib = _native.load()
    ctx = _native.Context(0)
    try:
        for rep in range(2):
            for i, f in enumerate(frames):
                nms = (i + rep) % 3
                view[:] = f.reshape(-1)
                rc, got, _ = _detect(lib, ctx, ptr.value, W, H, 16, 9, nms)
                _native.check(rc, "fdf_detect")
                assert np.array_equal(got, oracle.detect(f, 16, 9, nms)), (rep, i, nms)
    finally:
        ctx.close()
        assert hip.hipHostFree(ptr) == 0


@pytest.mark.parametrize("case", ["registered", "shorter0", "shorter4"])
def test_in_place_host_registered_ranges(case):
    """Memory the caller registered with hipHostRegister: a whole frame is read in place
    ("registered"); a registered range shorter than the frame is copied, not read past its
    end, by the single copy and by the chunked upload ("shorter0" / "shorter4"; ADVICE r04,
    r05).  The cases register and unregister ranges of their own numpy memory, so they run in
    a child process (tests/_host_register_cases.py): that memory is never
    handed back to this session's allocator and its later pageable copies."""
    import subprocess
    import sys

    script = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_host_register_cases.py")
    r = subprocess.run([sys.executable, "-u", script, case], capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["ok"] and res["case"] == case and res["calls"] >= 3, res

