"""Padded frame strides and concurrent direct-output grids.

fdf_detect_device / fdf_detect_batch / fdf_detect_device_rgb take a frame stride that may be
larger than one frame (include/fdf.h): frame f starts at f * stride and the bytes between
frames belong to nobody.  The kernel reads rows through a buffer resource of W*H + 15 bytes
per frame (the windows of the last lane may run up to 15 bytes past a frame's end) and the
batch's last frame exactly (fdf_sweep_impl.h, RowSource).  These tests fill every gap byte
with 0xFF -- a value that would create keypoints next to dark pixels if it were ever read as a
pixel -- and check each frame against the CPU oracle (oracle/fast_oracle.c, pinned to the
reference's goldens; the image contract is src/fast_simd.rs:307-330).

The concurrency tests run direct-output grids (small batches whose bands write their points
after a decoupled look-back, no compaction launch) from two contexts at once on one GPU, so
that together they hold more workgroups than the chip has slots: a band's number is its
workgroup's start ticket, so its look-back never waits on a band that has not started."""
import ctypes
import threading

import numpy as np
import pytest

import workloads
from feature_detector_fast_amd import Config, NonMaximalSuppression, _native, fast_hip
from oracle import oracle

pytestmark = pytest.mark.gpu

GAPS = [13, 4096]


def _frames(w, h):
    if (w, h) == (1920, 1080):
        return [workloads.s1_frame(5), workloads.s3_frame(11), workloads.s1_frame(17)]
    return [workloads.s1_frame(2, w, h), workloads.s3_frame(4, w, h), workloads.s2_frame(6, w, h)]


def _padded(frames, stride, px=1):
    """The frames at `stride`-byte spacing, gap bytes 0xFF; the buffer ends at the last
    frame's last byte (so the exact last-frame path is what keeps reads inside it)."""
    fb = frames[0].size
    buf = np.full((len(frames) - 1) * stride + fb, 0xFF, dtype=np.uint8)
    for f, fr in enumerate(frames):
        buf[f * stride: f * stride + fb] = fr.reshape(-1)
    return buf


def _check(frames, pts, offs, t, n, nms):
    for f, img in enumerate(frames):
        want = oracle.detect(img, t, n, nms)
        assert np.array_equal(pts[offs[f]:offs[f + 1]], want), f


@pytest.mark.parametrize("gap", GAPS)
@pytest.mark.parametrize("shape", [(1920, 1080), (333, 177)])
@pytest.mark.parametrize("t,n,nms", [(16, 9, 0), (16, 9, 1), (16, 9, 2), (8, 12, 2)])
def test_device_padded_stride(gap, shape, t, n, nms):
    import torch

    w, h = shape
    frames = _frames(w, h)
    stride = w * h + gap
    buf = torch.from_numpy(_padded(frames, stride)).cuda()
    F = len(frames)
    cap = F * w * h // 4 + 64
    out = torch.full((cap, 2), -1, dtype=torch.int32, device="cuda")
    offs = torch.zeros(F + 1, dtype=torch.int64, device="cuda")
    ctx = fast_hip.context(0)
    cfg = _native.FdfConfig(t, n, nms)
    stream = torch.cuda.current_stream()
    rc = _native.load().fdf_detect_device(ctx.handle, buf.data_ptr(), F, w, h, stride,
                                          ctypes.byref(cfg), out.data_ptr(), cap,
                                          offs.data_ptr(), ctypes.c_void_p(stream.cuda_stream))
    _native.check(rc, "fdf_detect_device")
    torch.cuda.synchronize()
    o = offs.cpu().numpy()
    assert o[-1] <= cap
    _check(frames, out[: o[-1]].cpu().numpy().astype(np.uint32), o, t, n, nms)


@pytest.mark.parametrize("gap", GAPS)
@pytest.mark.parametrize("nms", [0, 1, 2])
def test_host_batch_padded_stride(gap, nms):
    w, h = 1920, 1080
    frames = _frames(w, h)
    stride = w * h + gap
    buf = _padded(frames, stride)
    lib = _native.load()
    ctx = fast_hip.context(0)
    cfg = _native.FdfConfig(16, 9, nms)
    F = len(frames)
    offs = np.zeros(F + 1, dtype=np.uint64)
    n = ctypes.c_size_t(0)
    with ctx.lock:
        rc = lib.fdf_detect_batch(ctx.handle, buf.ctypes.data, F, w, h, stride, ctypes.byref(cfg),
                                  None, 0, offs.ctypes.data, ctypes.byref(n))
        assert rc in (_native.FDF_OK, _native.FDF_ERR_CAPACITY)
        pts = np.zeros((max(n.value, 1), 2), dtype=np.uint32)
        _native.check(lib.fdf_fetch_last(ctx.handle, pts.ctypes.data, None, n.value,
                                         ctypes.byref(n)), "fdf_fetch_last")
    _check(frames, pts[: n.value], offs, 16, 9, nms)


@pytest.mark.parametrize("gap", GAPS)
@pytest.mark.parametrize("nms", [0, 1])
def test_device_rgb_padded_stride(gap, nms):
    """The fused RGB detector: frames of 3 * w * h bytes at a padded stride (grey repeated per
    channel, so the luma is the grey frame and the oracle's list applies)."""
    import torch

    w, h = 1920, 1080
    frames = _frames(w, h)
    rgb = [np.repeat(fr[:, :, None], 3, axis=2) for fr in frames]
    stride = 3 * w * h + gap
    buf = torch.from_numpy(_padded(rgb, stride)).cuda()
    F = len(frames)
    cap = F * w * h // 4
    out = torch.full((cap, 2), -1, dtype=torch.int32, device="cuda")
    offs = torch.zeros(F + 1, dtype=torch.int64, device="cuda")
    ctx = fast_hip.context(0)
    cfg = _native.FdfConfig(16, 9, nms)
    stream = torch.cuda.current_stream()
    rc = _native.load().fdf_detect_device_rgb(ctx.handle, buf.data_ptr(), F, w, h, stride,
                                              ctypes.byref(cfg), out.data_ptr(), cap,
                                              offs.data_ptr(), ctypes.c_void_p(stream.cuda_stream))
    _native.check(rc, "fdf_detect_device_rgb")
    torch.cuda.synchronize()
    o = offs.cpu().numpy()
    _check(frames, out[: o[-1]].cpu().numpy().astype(np.uint32), o, 16, 9, nms)


def test_stride_below_frame_is_rejected():
    import torch

    w, h = 64, 48
    buf = torch.zeros(2 * w * h, dtype=torch.uint8, device="cuda")
    out = torch.zeros((16, 2), dtype=torch.int32, device="cuda")
    offs = torch.zeros(3, dtype=torch.int64, device="cuda")
    cfg = _native.FdfConfig(16, 9, 0)
    rc = _native.load().fdf_detect_device(fast_hip.context(0).handle, buf.data_ptr(), 2, w, h,
                                          w * h - 1, ctypes.byref(cfg), out.data_ptr(), 16,
                                          offs.data_ptr(), None)
    assert rc == _native.FDF_ERR_ARG


@pytest.mark.parametrize("nms", [0, 1])
def test_concurrent_direct_grids_host(nms):
    """detector_batch over two contexts of one GPU, 32 1080p frames -- each
    shard is a ~1 000-workgroup direct grid, the two together more than the chip holds at
    once.  Every frame equals the oracle, on every repetition."""
    host = [(workloads.s1_frame, workloads.s3_frame)[i % 4 == 3](i) for i in range(32)]
    frames = np.stack(host)
    cfg = Config(16, 9, NonMaximalSuppression(nms))
    want = [oracle.detect(f, 16, 9, nms) for f in host]
    for _ in range(3):
        pts, offs = fast_hip.detector_batch(frames, cfg, devices=[0, 0])
        for f in range(len(host)):
            assert np.array_equal(pts[offs[f]:offs[f + 1]], want[f]), f


def test_concurrent_direct_grids_device():
    """Two threads, two contexts, two streams: device-path direct grids (8 frames each)
    launched back to back and at the same time, 20 times; every result equals the first run
    of its thread and frames 0 and 7 equal the oracle."""
    import torch

    results, errors = {}, []
    hosts = {k: [workloads.s1_frame(8 * k + i) if i % 3 else workloads.s3_frame(8 * k + i)
                 for i in range(8)] for k in range(2)}

    def worker(k):
        try:
            ctx = _native.Context(0)
            lib = _native.load()
            stream = torch.cuda.Stream()
            frames = torch.from_numpy(np.stack(hosts[k])).cuda()
            F, H, W = frames.shape
            out = torch.empty((F * 700_000, 2), dtype=torch.int32, device="cuda")
            offs = torch.zeros(F + 1, dtype=torch.int64, device="cuda")
            cfg = _native.FdfConfig(16, 9, 1)
            ctx.set_timing(True)
            runs = []
            for _ in range(20):
                rc = lib.fdf_detect_device(ctx.handle, frames.data_ptr(), F, W, H, W * H,
                                           ctypes.byref(cfg), out.data_ptr(), out.shape[0],
                                           offs.data_ptr(), ctypes.c_void_p(stream.cuda_stream))
                _native.check(rc, "fdf_detect_device")
                stream.synchronize()
                o = offs.cpu().numpy().copy()
                runs.append((o, out[: o[-1]].cpu().numpy().astype(np.uint32)))
            _, comp = ctx.timing_samples()
            ctx.close()
            results[k] = (runs, comp)
        except Exception as e:      # noqa: BLE001 -- reported by the main thread
            errors.append(e)

    ths = [threading.Thread(target=worker, args=(k,)) for k in range(2)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    assert not errors, errors
    for k in range(2):
        runs, comp = results[k]
        assert np.all(comp == 0.0), "expected direct-output grids (no compaction launch)"
        o0, p0 = runs[0]
        for o, p in runs[1:]:
            assert np.array_equal(o, o0) and np.array_equal(p, p0)
        for f in (0, 7):
            assert np.array_equal(p0[o0[f]:o0[f + 1]], oracle.detect(hosts[k][f], 16, 9, 1)), (k, f)


@pytest.mark.parametrize("chunks", [4, 2, 16, 1, 0])
def test_host_overlapped_upload(chunks):
    """fdf_detect's overlapped upload (fdf_ctx_set_upload_chunks): the frame goes up in row
    chunks while the detector runs, each band waiting for the chunk of its last row.  Frames
    alternate between contents (a band reading a row before its chunk landed, or a stale
    cached line of the previous frame, would show as a wrong list), with packed and padded
    row strides; every list equals the oracle.  chunks = 1 is the one-copy path."""
    ctx = fast_hip.context(0)
    frames = [workloads.s1_frame(31), workloads.s3_frame(12), workloads.s2_frame(9),
              workloads.s1_frame(77)]
    want = {(i, nms): oracle.detect(f, 16, 9, nms) for i, f in enumerate(frames) for nms in (0, 1)}
    ctx.set_upload_chunks(chunks)
    try:
        for rep in range(2):
            for i, f in enumerate(frames):
                nms = (i + rep) % 2
                img = f
                if (i + rep) % 3 == 2:          # a padded row stride (hipMemcpy2DAsync chunks)
                    padded = np.full((f.shape[0], f.shape[1] + 40), 0xFF, dtype=np.uint8)
                    padded[:, : f.shape[1]] = f
                    img = padded[:, : f.shape[1]]
                got = fast_hip.detect_array(img, Config(16, 9, NonMaximalSuppression(nms)))
                assert np.array_equal(got, want[(i, nms)]), (rep, i, nms)
        # the flag handshake worked: no band's chunk wait ran out and fell back to a second
        # detection from one copy, and no look-back was rebuilt
        assert ctx.recoveries() == (0, 0), ctx.recoveries()
    finally:
        ctx.set_upload_chunks(0)


def test_context_setter_bounds():
    """fdf_ctx_set_band_rows rejects heights past the automatic range (256; the
    LDS layout arithmetic would overflow far beyond it) and fdf_ctx_set_upload_chunks more
    than 16 chunks, with FDF_ERR_ARG and the context unchanged."""
    ctx = _native.Context(0)
    try:
        for bad in (257, 1 << 30, 0xFFFFFFFF):
            with pytest.raises(_native.FdfError) as e:
                ctx.set_band_rows(bad)
            assert e.value.status == _native.FDF_ERR_ARG
        with pytest.raises(_native.FdfError) as e:
            ctx.set_upload_chunks(17)
        assert e.value.status == _native.FDF_ERR_ARG
        ctx.set_band_rows(256)
        import torch

        img = workloads.s1_frame(3)
        frames = torch.from_numpy(img[None].copy()).cuda()
        out = torch.empty((200_000, 2), dtype=torch.int32, device="cuda")
        offs = torch.zeros(2, dtype=torch.int64, device="cuda")
        fast_hip.detect_device(frames, Config(16, 9, NonMaximalSuppression.MaxThreshold), out,
                               offs, ctx=ctx)
        torch.cuda.synchronize()
        got = out[: int(offs[1])].cpu().numpy().astype(np.uint32)
        assert np.array_equal(got, oracle.detect(img, 16, 9, 1))
    finally:
        ctx.close()
