"""Host-API behaviour of the C ABI on the GPU: the two-call capacity pattern runs the
detection once (fdf_fetch_last), device work on different streams is ordered, the output
buffer grows by compacting again, the geometry override, per-launch timing samples, and the
multi-device batch (fdf_detect_batch_multi) -- every result checked against the oracle."""
import ctypes

import numpy as np
import pytest

import workloads
from feature_detector_fast_amd import Config, NonMaximalSuppression, _native, fast_hip
from oracle import oracle

pytestmark = pytest.mark.gpu


def test_capacity_retry_runs_one_detection():
    """A result larger than the first capacity guess (S3: ~28% keypoints) is copied out of
    the context with fdf_fetch_last: one detector launch per call (fdf_ctx_set_timing)."""
    img = workloads.s3_frame(4)[:400, :600].copy()
    cfg = Config(16, 9, NonMaximalSuppression.Off)
    assert len(oracle.detect(img, 16, 9, 0)) > fast_hip.capacity_guess(img.size)
    ctx = fast_hip.context(0)
    ctx.set_timing(True)
    try:
        got = fast_hip.detect_array(img, cfg)
        calls, _, _ = ctx.timing()
    finally:
        ctx.set_timing(False)
    assert calls == 1
    assert np.array_equal(got, oracle.detect(img, 16, 9, 0))


def test_fetch_last_c_abi():
    """fdf_detect with cap 0 -> FDF_ERR_CAPACITY + n; fdf_fetch_last with a short buffer ->
    the first cap points and FDF_ERR_CAPACITY again; then the whole list and its scores."""
    img = workloads.s1_frame(1, 640, 480)
    want, want_sc = oracle.detect(img, 16, 9, 1, with_scores=True)
    lib = _native.load()
    ctx = fast_hip.context(0)
    cfg = _native.FdfConfig(16, 9, 1)
    n = ctypes.c_size_t(0)
    with ctx.lock:
        ctx.set_timing(True)
        rc = lib.fdf_detect(ctx.handle, img.ctypes.data, 640, 480, 640, ctypes.byref(cfg), None,
                            0, ctypes.byref(n))
        assert rc == _native.FDF_ERR_CAPACITY and n.value == len(want)
        part = np.zeros((10, 2), dtype=np.uint32)
        rc = lib.fdf_fetch_last(ctx.handle, part.ctypes.data, None, 10, ctypes.byref(n))
        assert rc == _native.FDF_ERR_CAPACITY and n.value == len(want)
        assert np.array_equal(part, want[:10])
        out = np.zeros((n.value, 2), dtype=np.uint32)
        sc = np.zeros(n.value, dtype=np.uint16)
        rc = lib.fdf_fetch_last(ctx.handle, out.ctypes.data, sc.ctypes.data, n.value,
                                ctypes.byref(n))
        calls, _, _ = ctx.timing()
        ctx.set_timing(False)
    assert rc == _native.FDF_OK and calls == 1
    assert np.array_equal(out, want) and np.array_equal(sc, want_sc)


def test_fetch_last_needs_a_result():
    lib = _native.load()
    c = _native.Context(0)
    n = ctypes.c_size_t(0)
    assert lib.fdf_fetch_last(c.handle, None, None, 0, ctypes.byref(n)) == _native.FDF_ERR_ARG
    c.close()


def test_output_grows_by_compacting_again():
    """A batch whose total exceeds the context's output buffer: the buffer grows and only the
    compaction runs again (one detector launch), the result equals the oracle."""
    frames = np.stack([workloads.s3_frame(10 + i)[:300, :400] for i in range(6)])
    c = _native.Context(0)
    c.lock = __import__("threading").Lock()
    lib = _native.load()
    cfg = _native.FdfConfig(12, 9, 0)
    offs = np.zeros(7, dtype=np.uint64)
    n = ctypes.c_size_t(0)
    c.set_timing(True)
    out = np.zeros((6 * 300 * 400, 2), dtype=np.uint32)
    rc = lib.fdf_detect_batch(c.handle, frames.ctypes.data, 6, 400, 300, 400 * 300,
                              ctypes.byref(cfg), out.ctypes.data, out.shape[0],
                              offs.ctypes.data, ctypes.byref(n))
    calls, _, _ = c.timing()
    c.close()
    assert rc == _native.FDF_OK and calls == 1
    assert n.value > fast_hip.capacity_guess(frames.size)
    for f in range(6):
        assert np.array_equal(out[offs[f]:offs[f + 1]], oracle.detect(frames[f], 12, 9, 0)), f


def test_device_then_host_call_without_sync():
    """fdf_detect_device on torch's stream, then a host call on the context's own stream,
    with no synchronisation between them: the host call waits on the device for the first
    call's use of the shared workspace, and both results are exact."""
    import torch

    frames = workloads.s1_frames_torch(0, 64)
    cfg = Config(16, 9, NonMaximalSuppression.MaxThreshold)
    out = torch.empty((64 * 20000, 2), dtype=torch.int32, device="cuda")
    offs = torch.zeros(65, dtype=torch.int64, device="cuda")
    img = workloads.s3_frame(3)[:500, :700].copy()
    fast_hip.detect_device(frames, cfg, out, offs)
    got = fast_hip.detect_array(img, cfg)           # no torch.cuda.synchronize() before
    torch.cuda.synchronize()
    assert np.array_equal(got, oracle.detect(img, 16, 9, 1))
    o = offs.cpu().numpy()
    for f in (0, 31, 63):
        want = oracle.detect(frames[f].cpu().numpy(), 16, 9, 1)
        assert np.array_equal(out[o[f]:o[f + 1]].cpu().numpy().astype(np.uint32), want), f


def test_ticket_out_of_step_is_reported_once():
    """A direct-output launch whose start tickets run past its grid (the device counter and
    the host's base out of step, forced with fdf_ctx_test_skew_tickets) touches no band
    memory outside the grid (fdf_sweep_impl.h fast_sweep_kernel) and is reported: a host call
    returns FDF_ERR_DEVICE; an asynchronous device call reports it at the context's next
    device call, exactly once; both contexts are correct again afterwards (the counter is
    re-zeroed).  Also the pending-error path of ADVICE r05: a host call in between that sees
    the device call's error word first keeps it for the next device call."""
    import torch

    lib = _native.load()
    img = workloads.s1_frame(2)
    want = oracle.detect(img, 16, 9, 1)
    cfg = Config(16, 9, NonMaximalSuppression.MaxThreshold)
    ccfg = _native.FdfConfig(16, 9, 1)
    c = _native.Context(0)
    try:
        out = np.zeros((len(want) + 16, 2), dtype=np.uint32)
        n = ctypes.c_size_t(0)
        # (a context's first launch zeroes the counter and the host count: skew after it)
        rc = lib.fdf_detect(c.handle, img.ctypes.data, 1920, 1080, 1920, ctypes.byref(ccfg),
                            out.ctypes.data, out.shape[0], ctypes.byref(n))
        assert rc == _native.FDF_OK and np.array_equal(out[: n.value], want)
        # host call: the skewed launch is an error of that call
        _native.check(lib.fdf_ctx_test_skew_tickets(c.handle, 5))
        rc = lib.fdf_detect(c.handle, img.ctypes.data, 1920, 1080, 1920, ctypes.byref(ccfg),
                            out.ctypes.data, out.shape[0], ctypes.byref(n))
        assert rc == _native.FDF_ERR_DEVICE
        rc = lib.fdf_detect(c.handle, img.ctypes.data, 1920, 1080, 1920, ctypes.byref(ccfg),
                            out.ctypes.data, out.shape[0], ctypes.byref(n))
        assert rc == _native.FDF_OK and np.array_equal(out[: n.value], want)
        # device calls: the skewed launch returns OK (asynchronous), the next device call
        # reports it -- after a host call in between -- once
        one = torch.from_numpy(img).cuda().unsqueeze(0).contiguous()
        d_out = torch.empty((len(want) + 16, 2), dtype=torch.int32, device="cuda")
        d_offs = torch.zeros(2, dtype=torch.int64, device="cuda")
        _native.check(lib.fdf_ctx_test_skew_tickets(c.handle, 7))
        fast_hip.detect_device(one, cfg, d_out, d_offs, ctx=c)
        torch.cuda.synchronize()
        rc = lib.fdf_detect(c.handle, img.ctypes.data, 1920, 1080, 1920, ctypes.byref(ccfg),
                            out.ctypes.data, out.shape[0], ctypes.byref(n))
        assert rc == _native.FDF_OK and np.array_equal(out[: n.value], want)
        with pytest.raises(_native.FdfError):
            fast_hip.detect_device(one, cfg, d_out, d_offs, ctx=c)
        fast_hip.detect_device(one, cfg, d_out, d_offs, ctx=c)
        torch.cuda.synchronize()
        o = d_offs.cpu().numpy()
        assert o[1] == len(want)
        assert np.array_equal(d_out[: o[1]].cpu().numpy().astype(np.uint32), want)
    finally:
        c.close()


@pytest.mark.parametrize("nframes", [1, 2, 3])
def test_dense_frames_default_geometry(nframes):
    """the one-round geometry a single frame or a few get by default (short
    latency bands, direct output, 4x slots) on dense noise frames, where bands take the
    bitmap-slot and NMS-spill paths: every mode equals the oracle."""
    frames = [workloads.s3_frame(70 + i) for i in range(nframes)]
    for nms in (0, 1, 2):
        pts, offs = fast_hip.detector_batch(np.stack(frames), Config(8, 9, NonMaximalSuppression(nms)))
        for f, img in enumerate(frames):
            assert np.array_equal(pts[offs[f]:offs[f + 1]], oracle.detect(img, 8, 9, nms)), (nms, f)


def test_geometry_override_same_result():
    img = workloads.s1_frame(6, 800, 600)
    cfg = Config(16, 9, NonMaximalSuppression.SumAbsolute)
    base = fast_hip.detect_array(img, cfg)
    ctx = fast_hip.context(0)
    ctx.set_geometry(1)
    try:
        tall = fast_hip.detect_array(img, cfg)
    finally:
        ctx.set_geometry(0)
    assert np.array_equal(base, tall)
    assert np.array_equal(base, oracle.detect(img, 16, 9, 2))


def test_timing_samples():
    """Per-call kernel durations from the dispatch-stamped events: an 8-frame batch writes
    its points directly (no compaction launch: 0 ms), a 64-frame batch runs both kernels."""
    import torch

    ctx = fast_hip.context(0)
    for F, direct in ((8, True), (64, False)):
        frames = workloads.s1_frames_torch(0, F)
        out = torch.empty((F * 20000, 2), dtype=torch.int32, device="cuda")
        offs = torch.zeros(F + 1, dtype=torch.int64, device="cuda")
        ctx.set_timing(True)
        for _ in range(5):
            fast_hip.detect_device(frames, Config(16, 9, NonMaximalSuppression.Off), out, offs)
        det, com = ctx.timing_samples()
        calls, d_tot, c_tot = ctx.timing()
        ctx.set_timing(False)
        assert calls == 5 and det.shape == (5,) and np.all(det > 0)
        assert np.all(com == 0) if direct else np.all(com > 0)
        assert abs(float(det.sum()) - d_tot) < 1e-3 * max(d_tot, 1.0)
        assert abs(float(com.sum()) - c_tot) < 1e-3 * max(c_tot, 1.0)


@pytest.mark.parametrize("devices", [[0, 0], [0, 0, 0]])
def test_multi_device_batch(devices):
    """Frames sharded over several contexts (all on device 0 on a 1-GPU box) give the
    single-context result, frame for frame, and equal the oracle."""
    frames = np.stack([workloads.s1_frame(i, 960, 540) for i in range(7)] +
                      [workloads.s3_frame(40)[:540, :960]])
    cfg = Config(16, 9, NonMaximalSuppression.MaxThreshold)
    pts1, offs1 = fast_hip.detector_batch(frames, cfg)
    ptsm, offsm = fast_hip.detector_batch(frames, cfg, devices=devices)
    assert np.array_equal(offs1, offsm)
    assert np.array_equal(pts1, ptsm)
    for f in range(frames.shape[0]):
        assert np.array_equal(ptsm[offsm[f]:offsm[f + 1]], oracle.detect(frames[f], 16, 9, 1)), f


def test_multi_device_more_contexts_than_frames():
    frames = np.stack([workloads.s1_frame(i, 320, 240) for i in range(2)])
    cfg = Config(16, 9, NonMaximalSuppression.Off)
    pts, offs = fast_hip.detector_batch(frames, cfg, devices=[0, 0, 0, 0])
    for f in range(2):
        assert np.array_equal(pts[offs[f]:offs[f + 1]], oracle.detect(frames[f], 16, 9, 0))


def test_multi_device_rejects_repeated_context():
    lib = _native.load()
    ctx = fast_hip.context(0)
    handles = (ctypes.c_void_p * 2)(ctx.handle.value, ctx.handle.value)
    frames = np.zeros((2, 20, 20), dtype=np.uint8)
    n = ctypes.c_size_t(0)
    cfg = _native.FdfConfig(16, 9, 0)
    rc = lib.fdf_detect_batch_multi(handles, 2, frames.ctypes.data, 2, 20, 20, 400,
                                    ctypes.byref(cfg), None, 0, None, ctypes.byref(n))
    assert rc == _native.FDF_ERR_ARG


def _multi(lib, handles, frames, cfg, out, offs, n):
    f, h, w = frames.shape
    return lib.fdf_detect_batch_multi(handles, len(handles), frames.ctypes.data, f, w, h, h * w,
                                      ctypes.byref(cfg), out.ctypes.data if out is not None else None,
                                      0 if out is None else out.shape[0],
                                      offs.ctypes.data, ctypes.byref(n))


def test_multi_device_reversed_orders_do_not_deadlock():
    """Two threads run fdf_detect_batch_multi over the same two contexts listed in opposite
    orders: the contexts are locked in one global order, so both finish, and
    each result equals the oracle in its own shard order."""
    import threading

    lib = _native.load()
    a, b = _native.Context(0), _native.Context(0)
    frames = np.stack([workloads.s1_frame(i, 320, 240) for i in range(4)])
    want = [oracle.detect(frames[f], 16, 9, 1) for f in range(4)]
    cfg = _native.FdfConfig(16, 9, 1)
    errors = []

    def run(order):
        handles = (ctypes.c_void_p * 2)(*[c.handle.value for c in order])
        for _ in range(20):
            out = np.zeros((4 * 320 * 240 // 8, 2), dtype=np.uint32)
            offs = np.zeros(5, dtype=np.uint64)
            n = ctypes.c_size_t(0)
            rc = _multi(lib, handles, frames, cfg, out, offs, n)
            if rc != _native.FDF_OK:
                errors.append(rc)
                return
            for f in range(4):
                if not np.array_equal(out[offs[f]:offs[f + 1]], want[f]):
                    errors.append(("frame", f))
                    return

    ts = [threading.Thread(target=run, args=(o,)) for o in ((a, b), (b, a))]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=90)
    alive = any(t.is_alive() for t in ts)
    assert not alive, "fdf_detect_batch_multi deadlocked"
    a.close()
    b.close()
    assert not errors, errors


def test_fetch_last_multi_checks_the_call():
    """fdf_fetch_last_multi joins only the shards of one fdf_detect_batch_multi call in its
    order: a reordered array, or a host call on one context in between, is FDF_ERR_ARG
    (ADVICE r02); the matching array gets the oracle's lists."""
    lib = _native.load()
    a, b = _native.Context(0), _native.Context(0)
    frames = np.stack([workloads.s1_frame(i, 320, 240) for i in range(3)])
    cfg = _native.FdfConfig(16, 9, 0)
    ab = (ctypes.c_void_p * 2)(a.handle.value, b.handle.value)
    ba = (ctypes.c_void_p * 2)(b.handle.value, a.handle.value)
    offs = np.zeros(4, dtype=np.uint64)
    n = ctypes.c_size_t(0)
    assert _multi(lib, ab, frames, cfg, None, offs, n) == _native.FDF_ERR_CAPACITY
    total = n.value
    out = np.zeros((total, 2), dtype=np.uint32)
    assert lib.fdf_fetch_last_multi(ba, 2, out.ctypes.data, total, ctypes.byref(n)) == _native.FDF_ERR_ARG
    assert lib.fdf_fetch_last_multi(ab, 2, out.ctypes.data, total, ctypes.byref(n)) == _native.FDF_OK
    want = np.concatenate([oracle.detect(frames[f], 16, 9, 0) for f in range(3)])
    assert n.value == total and np.array_equal(out, want)
    img = frames[0].copy()
    one = np.zeros((10000, 2), dtype=np.uint32)
    assert lib.fdf_detect(a.handle, img.ctypes.data, 320, 240, 320, ctypes.byref(cfg),
                          one.ctypes.data, 10000, ctypes.byref(n)) == _native.FDF_OK
    assert lib.fdf_fetch_last_multi(ab, 2, out.ctypes.data, total, ctypes.byref(n)) == _native.FDF_ERR_ARG
    a.close()
    b.close()


def test_scores_do_not_break_a_concurrent_two_call():
    """keypoint_scores / score_rings take the context lock that holds detect_array's two-call
    pattern together: dense detections (fetched with fdf_fetch_last) running
    beside score calls on the same context stay exact."""
    import threading

    img = workloads.s3_frame(5)[:300, :400].copy()
    cfg = Config(16, 9, NonMaximalSuppression.Off)
    want = oracle.detect(img, 16, 9, 0)
    assert len(want) > fast_hip.capacity_guess(img.size)
    pts = want[:500]
    scfg = Config(16, 9, NonMaximalSuppression.MaxThreshold)
    want_sc = fast_hip.keypoint_scores(img, pts, scfg)
    errors = []

    def detect():
        try:
            for _ in range(15):
                if not np.array_equal(fast_hip.detect_array(img, cfg), want):
                    errors.append("detect")
        except Exception as e:          # noqa: BLE001 -- reported below
            errors.append(repr(e))

    def score():
        try:
            for _ in range(15):
                if not np.array_equal(fast_hip.keypoint_scores(img, pts, scfg), want_sc):
                    errors.append("scores")
                fast_hip.score_rings(np.zeros(64, np.uint8), np.zeros((64, 16), np.uint8),
                                     NonMaximalSuppression.SumAbsolute, threshold=3)
        except Exception as e:          # noqa: BLE001
            errors.append(repr(e))

    ts = [threading.Thread(target=detect), threading.Thread(target=score)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
    assert not any(t.is_alive() for t in ts)
    assert not errors, errors[:3]
