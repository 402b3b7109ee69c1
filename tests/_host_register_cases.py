"""Child process of tests/test_gpu_host_inplace.py: the cases that hipHostRegister and
hipHostUnregister ranges of the test's own (numpy) memory.

They run in a process of their own, not in the pytest session: every unexplained
hipErrorIllegalAddress of rounds 5-6 surfaced at the first sizeable runtime-managed host copy
(a staged SDMA D2H, or an H2D from pageable memory the runtime pins on the fly) in the test
files that run right after these cases -- in the same process, where freed numpy blocks that
had been registered and unregistered are reused for the next tests' pageable copies
(DESIGN.md §7.7).  The library itself never registers memory; it only reads a range its
caller registered in place (fdf_api.cpp run_host).

usage: python tests/_host_register_cases.py {registered|shorter0|shorter4}
Prints one JSON line and exits 0 on success; a failed check raises (exit 1)."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import workloads  # noqa: E402
from feature_detector_fast_amd import _native  # noqa: E402
from oracle import oracle  # noqa: E402


def _detect(lib, ctx, ptr, w, h, t, n, nms):
    cfg = _native.FdfConfig(t, n, nms)
    out = np.zeros((w * h, 2), dtype=np.uint32)
    got = ctypes.c_size_t(0)
    rc = lib.fdf_detect(ctx.handle, ctypes.c_void_p(ptr), w, h, w, ctypes.byref(cfg),
                        out.ctypes.data, w * h, ctypes.byref(got))
    return rc, out[: min(got.value, w * h)]


def _hip():
    """The HIP runtime already in the process (the one libfdf.so uses), never a second copy."""
    _native.load()
    hip = ctypes.CDLL("libamdhip64.so.7", mode=os.RTLD_NOLOAD | os.RTLD_NOW)
    for fn in ("hipHostRegister", "hipHostUnregister"):
        getattr(hip, fn).restype = ctypes.c_int
    return hip


def registered():
    """Memory registered with hipHostRegister is read in place; the lists equal the oracle
    across frames written into the same buffer."""
    W, H = 1280, 720
    frames = [workloads.s1_frame(3, W, H), workloads.s3_frame(7)[:H, :W].copy(),
              workloads.s1_frame(40, W, H)]
    hip = _hip()
    keep = np.zeros(W * H + 4096, dtype=np.uint8)
    base = keep.ctypes.data + (-keep.ctypes.data) % 4096   # page-aligned start
    view = np.ctypeslib.as_array(ctypes.cast(base, ctypes.POINTER(ctypes.c_uint8)), (W * H,))
    assert hip.hipHostRegister(ctypes.c_void_p(base), ctypes.c_size_t(W * H),
                               ctypes.c_uint(0)) == 0
    lib = _native.load()
    ctx = _native.Context(0)
    calls = 0
    try:
        for rep in range(2):
            for i, f in enumerate(frames):
                nms = (i + rep) % 3
                view[:] = f.reshape(-1)
                rc, got = _detect(lib, ctx, base, W, H, 16, 9, nms)
                _native.check(rc, "fdf_detect")
                assert np.array_equal(got, oracle.detect(f, 16, 9, nms)), (rep, i, nms)
                calls += 1
    finally:
        ctx.close()
        assert hip.hipHostUnregister(ctypes.c_void_p(base)) == 0
    return {"calls": calls}


def shorter(chunks):
    """a frame whose first bytes sit in a hipHostRegister'ed range that ends before
    the frame does is copied, not read in place (reading it in place would read past the
    registration over PCIe).  ADVICE r05: the overlapped chunked upload (chunks = 4) stages
    such a frame as well, so no chunk copy is rejected and no fallback is counted."""
    W, H = 1280, 720
    img = workloads.s1_frame(11, W, H)
    hip = _hip()
    keep = np.zeros(W * H + 4096, dtype=np.uint8)
    base = keep.ctypes.data + (-keep.ctypes.data) % 4096
    view = np.ctypeslib.as_array(ctypes.cast(base, ctypes.POINTER(ctypes.c_uint8)), (W * H,))
    view[:] = img.reshape(-1)
    half = (W * H // 2) & ~4095                       # whole pages, half the frame
    assert hip.hipHostRegister(ctypes.c_void_p(base), ctypes.c_size_t(half), ctypes.c_uint(0)) == 0
    lib = _native.load()
    ctx = _native.Context(0)
    ctx.set_upload_chunks(chunks)
    try:
        for nms in (0, 1, 2):
            rc, got = _detect(lib, ctx, base, W, H, 16, 9, nms)
            _native.check(rc, "fdf_detect")
            assert np.array_equal(got, oracle.detect(img, 16, 9, nms)), nms
        rec = ctx.recoveries()
        assert rec == (0, 0), rec
    finally:
        ctx.close()
        assert hip.hipHostUnregister(ctypes.c_void_p(base)) == 0
    return {"calls": 3, "recoveries": list(rec)}


CASES = {"registered": registered, "shorter0": lambda: shorter(0), "shorter4": lambda: shorter(4)}


def main(argv):
    if len(argv) != 2 or argv[1] not in CASES:
        print("usage: _host_register_cases.py {%s}" % "|".join(CASES), file=sys.stderr)
        return 2
    res = CASES[argv[1]]()
    print(json.dumps({"case": argv[1], "ok": True, **res}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv))
