"""ctypes binding of the C ABI in include/fdf.h (libfdf.so, built in-tree by ``make``).

There is no fallback: if the shared library is missing or no HIP device is visible the
calls raise :class:`FdfError` -- the HIP kernels are the only implementation.
"""
import ctypes
import importlib.util
import os
import sys

_HERE = os.path.dirname(os.path.abspath(__file__))
# FDF_LIB_PATH: another build of the same library (A/B timing of two kernel versions,
# tools/build_rev.sh); the default is the in-tree build.
LIB_PATH = os.environ.get("FDF_LIB_PATH") or os.path.join(_HERE, "libfdf.so")

# include/fdf.h enum fdf_status
FDF_OK = 0
FDF_ERR_COUNT = 1
FDF_ERR_SIZE = 2
FDF_ERR_CAPACITY = 3
FDF_ERR_NMS = 4
FDF_ERR_DEVICE = 5
FDF_ERR_ARG = 6
FDF_ERR_ALLOC = 7
FDF_ERR_BUSY = 8
FDF_ERR_DROPPED = 9
# enum fdf_pipe_flags
FDF_PIPE_RGB = 1
FDF_PIPE_SCORES = 2

# Every symbol include/fdf.h declares (tests/test_abi.py checks the .so exports them all).
EXPORTED_SYMBOLS = (
    "fdf_abi_version", "fdf_status_string", "fdf_device_count", "fdf_validate",
    "fdf_ctx_create", "fdf_ctx_destroy", "fdf_ctx_stream", "fdf_ctx_set_timing",
    "fdf_ctx_timing", "fdf_detect", "fdf_detect_rgb", "fdf_rgb_to_luma_device",
    "fdf_detect_batch", "fdf_detect_device", "fdf_score_points", "fdf_detect_scored",
    "fdf_detect_batch_scored", "fdf_score_device", "fdf_pipeline_create",
    "fdf_pipeline_destroy", "fdf_pipeline_acquire", "fdf_pipeline_submit", "fdf_pipeline_push",
    "fdf_pipeline_collect", "fdf_ctx_set_geometry", "fdf_ctx_timing_samples", "fdf_fetch_last",
    "fdf_detect_batch_multi", "fdf_fetch_last_multi", "fdf_ctx_workspace_bytes",
    "fdf_detect_device_rgb", "fdf_circle", "fdf_calculate_offsets", "fdf_score_rings",
    "fdf_score_rings_device", "fdf_ctx_set_band_rows", "fdf_ctx_set_upload_chunks",
    "fdf_ctx_recoveries", "fdf_ctx_test_skew_tickets",
)


class FdfConfig(ctypes.Structure):
    _fields_ = [("threshold", ctypes.c_uint8), ("count", ctypes.c_uint8), ("nms", ctypes.c_uint8)]


class FdfPoint(ctypes.Structure):
    _fields_ = [("x", ctypes.c_uint32), ("y", ctypes.c_uint32)]


class FdfError(RuntimeError):
    """A non-OK fdf_status; ``.status`` holds the code."""

    def __init__(self, status, where=""):
        self.status = status
        msg = status_string(status) if _lib is not None else f"status {status}"
        super().__init__(f"{where}: {msg}" if where else msg)


_lib = None


def _share_torch_runtime():
    """Map PyTorch's bundled HIP runtime before libfdf.so when torch is installed.

    torch ships its own libamdhip64.so (SONAME libamdhip64.so.7).  If libfdf.so were loaded
    first it would map /opt/rocm's copy, and a later ``import torch`` would map a second HIP
    runtime into the process, which then fails to initialise.  With torch's copy mapped
    first, libfdf.so's NEEDED libamdhip64.so.7 binds to it, so device pointers and streams
    are shared with torch.  Without torch, /opt/rocm's runtime is used."""
    if "torch" in sys.modules:
        return
    spec = importlib.util.find_spec("torch")
    if spec is None or spec.origin is None:
        return
    path = os.path.join(os.path.dirname(spec.origin), "lib", "libamdhip64.so")
    if os.path.exists(path):
        ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)


def load():
    """Load libfdf.so once and declare the prototypes.  Raises if it is not built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise FdfError(FDF_ERR_DEVICE, f"{LIB_PATH} is not built (run `make` or __graft_entry__.build())")
    _share_torch_runtime()
    lib = ctypes.CDLL(LIB_PATH)
    u8p = ctypes.POINTER(ctypes.c_uint8)
    vp = ctypes.c_void_p
    sz = ctypes.c_size_t
    u32 = ctypes.c_uint32
    u64 = ctypes.c_uint64
    cfgp = ctypes.POINTER(FdfConfig)
    lib.fdf_abi_version.restype = ctypes.c_int
    lib.fdf_status_string.restype = ctypes.c_char_p
    lib.fdf_status_string.argtypes = [ctypes.c_int]
    lib.fdf_device_count.restype = ctypes.c_int
    lib.fdf_validate.restype = ctypes.c_int
    lib.fdf_validate.argtypes = [u32, u32, cfgp, ctypes.POINTER(ctypes.c_int)]
    lib.fdf_ctx_create.restype = ctypes.c_int
    lib.fdf_ctx_create.argtypes = [ctypes.c_int, ctypes.POINTER(vp)]
    lib.fdf_ctx_destroy.restype = None
    lib.fdf_ctx_destroy.argtypes = [vp]
    lib.fdf_ctx_stream.restype = vp
    lib.fdf_ctx_stream.argtypes = [vp]
    lib.fdf_ctx_set_timing.restype = ctypes.c_int
    lib.fdf_ctx_set_timing.argtypes = [vp, ctypes.c_int]
    lib.fdf_ctx_timing.restype = ctypes.c_int
    lib.fdf_ctx_timing.argtypes = [vp, ctypes.POINTER(u32), ctypes.POINTER(ctypes.c_float),
                                   ctypes.POINTER(ctypes.c_float)]
    lib.fdf_detect.restype = ctypes.c_int
    lib.fdf_detect.argtypes = [vp, vp, u32, u32, sz, cfgp, vp, sz, ctypes.POINTER(sz)]
    lib.fdf_detect_rgb.restype = ctypes.c_int
    lib.fdf_detect_rgb.argtypes = [vp, vp, u32, u32, sz, cfgp, vp, sz, ctypes.POINTER(sz)]
    lib.fdf_rgb_to_luma_device.restype = ctypes.c_int
    lib.fdf_rgb_to_luma_device.argtypes = [vp, vp, u32, u32, u32, ctypes.c_uint64, vp, vp]
    lib.fdf_detect_batch.restype = ctypes.c_int
    lib.fdf_detect_batch.argtypes = [vp, vp, u32, u32, u32, sz, cfgp, vp, sz, vp,
                                     ctypes.POINTER(sz)]
    lib.fdf_detect_device.restype = ctypes.c_int
    lib.fdf_detect_device.argtypes = [vp, vp, u32, u32, u32, u64, cfgp, vp, u64, vp, vp]
    lib.fdf_detect_device_rgb.restype = ctypes.c_int
    lib.fdf_detect_device_rgb.argtypes = [vp, vp, u32, u32, u32, u64, cfgp, vp, u64, vp, vp]
    i32p = ctypes.POINTER(ctypes.c_int32)
    lib.fdf_circle.restype = None
    lib.fdf_circle.argtypes = [i32p, i32p]
    lib.fdf_calculate_offsets.restype = None
    lib.fdf_calculate_offsets.argtypes = [u32, i32p]
    lib.fdf_score_rings.restype = ctypes.c_int
    lib.fdf_score_rings.argtypes = [vp, vp, vp, sz, cfgp, vp]
    lib.fdf_score_rings_device.restype = ctypes.c_int
    lib.fdf_score_rings_device.argtypes = [vp, vp, vp, u64, cfgp, vp, vp]
    lib.fdf_score_points.restype = ctypes.c_int
    lib.fdf_score_points.argtypes = [vp, vp, u32, u32, sz, cfgp, vp, sz, vp]
    lib.fdf_detect_scored.restype = ctypes.c_int
    lib.fdf_detect_scored.argtypes = [vp, vp, u32, u32, sz, cfgp, vp, vp, sz, ctypes.POINTER(sz)]
    lib.fdf_detect_batch_scored.restype = ctypes.c_int
    lib.fdf_detect_batch_scored.argtypes = [vp, vp, u32, u32, u32, sz, cfgp, vp, vp, sz, vp,
                                            ctypes.POINTER(sz)]
    lib.fdf_score_device.restype = ctypes.c_int
    lib.fdf_score_device.argtypes = [vp, vp, u32, u32, u32, u64, cfgp, vp, u64, vp, vp, vp]
    lib.fdf_pipeline_create.restype = ctypes.c_int
    lib.fdf_pipeline_create.argtypes = [ctypes.c_int, u32, u32, u32, u32, u64, u32, cfgp,
                                        ctypes.POINTER(vp)]
    lib.fdf_pipeline_destroy.restype = None
    lib.fdf_pipeline_destroy.argtypes = [vp]
    lib.fdf_pipeline_acquire.restype = ctypes.c_int
    lib.fdf_pipeline_acquire.argtypes = [vp, ctypes.POINTER(vp), ctypes.POINTER(u64)]
    lib.fdf_pipeline_submit.restype = ctypes.c_int
    lib.fdf_pipeline_submit.argtypes = [vp, u64, u32]
    lib.fdf_pipeline_push.restype = ctypes.c_int
    lib.fdf_pipeline_push.argtypes = [vp, vp, u32, sz, ctypes.POINTER(u64)]
    lib.fdf_pipeline_collect.restype = ctypes.c_int
    lib.fdf_pipeline_collect.argtypes = [vp, u64, vp, vp, sz, vp, ctypes.POINTER(sz)]
    lib.fdf_ctx_workspace_bytes.restype = ctypes.c_int
    lib.fdf_ctx_workspace_bytes.argtypes = [vp, ctypes.POINTER(u64)]
    lib.fdf_ctx_test_skew_tickets.restype = ctypes.c_int
    lib.fdf_ctx_test_skew_tickets.argtypes = [vp, u32]
    lib.fdf_ctx_set_geometry.restype = ctypes.c_int
    lib.fdf_ctx_set_geometry.argtypes = [vp, u32]
    lib.fdf_ctx_set_band_rows.restype = ctypes.c_int
    lib.fdf_ctx_set_band_rows.argtypes = [vp, u32]
    lib.fdf_ctx_set_upload_chunks.restype = ctypes.c_int
    lib.fdf_ctx_set_upload_chunks.argtypes = [vp, u32]
    lib.fdf_ctx_recoveries.restype = ctypes.c_int
    lib.fdf_ctx_recoveries.argtypes = [vp, ctypes.POINTER(u64), ctypes.POINTER(u64)]
    lib.fdf_ctx_timing_samples.restype = ctypes.c_int
    lib.fdf_ctx_timing_samples.argtypes = [vp, vp, vp, u32, ctypes.POINTER(u32)]
    lib.fdf_fetch_last.restype = ctypes.c_int
    lib.fdf_fetch_last.argtypes = [vp, vp, vp, sz, ctypes.POINTER(sz)]
    lib.fdf_detect_batch_multi.restype = ctypes.c_int
    lib.fdf_detect_batch_multi.argtypes = [vp, u32, vp, u32, u32, u32, sz, cfgp, vp, sz, vp,
                                           ctypes.POINTER(sz)]
    lib.fdf_fetch_last_multi.restype = ctypes.c_int
    lib.fdf_fetch_last_multi.argtypes = [vp, u32, vp, sz, ctypes.POINTER(sz)]
    del u8p
    _lib = lib
    return lib


def status_string(status):
    return load().fdf_status_string(int(status)).decode()


def check(status, where=""):
    if status != FDF_OK:
        raise FdfError(status, where)


class Context:
    """One device + one HIP stream (fdf_ctx_create / fdf_ctx_destroy)."""

    def __init__(self, device=0):
        lib = load()
        handle = ctypes.c_void_p()
        check(lib.fdf_ctx_create(int(device), ctypes.byref(handle)), "fdf_ctx_create")
        self._lib = lib
        self.handle = handle
        self.device = int(device)

    @property
    def stream(self):
        return self._lib.fdf_ctx_stream(self.handle)

    def set_timing(self, enable=True, every=1):
        """Record the detector and compaction kernel durations of every `every`-th call
        (dispatch-timestamped HIP events; fdf_ctx_set_timing)."""
        check(self._lib.fdf_ctx_set_timing(self.handle, max(1, int(every)) if enable else 0))

    def timing(self):
        """(calls, detector_ms_total, compaction_ms_total) since timing was enabled."""
        n, a, b = ctypes.c_uint32(), ctypes.c_float(), ctypes.c_float()
        check(self._lib.fdf_ctx_timing(self.handle, ctypes.byref(n), ctypes.byref(a),
                                       ctypes.byref(b)))
        return n.value, a.value, b.value

    def timing_samples(self):
        """Per-call (detector_ms, compaction_ms) arrays since timing was enabled."""
        import numpy as np

        n = ctypes.c_uint32()
        check(self._lib.fdf_ctx_timing_samples(self.handle, None, None, 0, ctypes.byref(n)))
        det = np.zeros(n.value, dtype=np.float32)
        com = np.zeros(n.value, dtype=np.float32)
        if n.value:
            check(self._lib.fdf_ctx_timing_samples(self.handle, det.ctypes.data, com.ctypes.data,
                                                   n.value, ctypes.byref(n)))
        return det, com

    def workspace_bytes(self):
        """Device bytes held by the context's workspace (fdf_ctx_workspace_bytes)."""
        v = ctypes.c_uint64()
        check(self._lib.fdf_ctx_workspace_bytes(self.handle, ctypes.byref(v)))
        return v.value

    def set_geometry(self, min_tasks=0):
        """Band geometry override (fdf_ctx_set_geometry): min_tasks=1 gives small jobs the
        tall bands of large batches (tests); 0 restores the default."""
        check(self._lib.fdf_ctx_set_geometry(self.handle, int(min_tasks)))

    def set_band_rows(self, rows=0):
        """Band height override (fdf_ctx_set_band_rows): bands of ``rows`` centre rows for
        every later detection (same keypoints, other NMS tiers); 0 = automatic."""
        check(self._lib.fdf_ctx_set_band_rows(self.handle, int(rows)))

    def set_upload_chunks(self, chunks=0):
        """fdf_detect's overlapped upload (fdf_ctx_set_upload_chunks): the frame in
        ``chunks`` row chunks while the detector runs; 1 = one copy first; 0 = default."""
        check(self._lib.fdf_ctx_set_upload_chunks(self.handle, int(chunks)))

    def recoveries(self):
        """(upload_fallbacks, lookback_recoveries) the host calls made on their own
        (fdf_ctx_recoveries): both 0 in a healthy run."""
        a, b = ctypes.c_uint64(), ctypes.c_uint64()
        check(self._lib.fdf_ctx_recoveries(self.handle, ctypes.byref(a), ctypes.byref(b)))
        return a.value, b.value

    def close(self):
        if self.handle:
            self._lib.fdf_ctx_destroy(self.handle)
            self.handle = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
