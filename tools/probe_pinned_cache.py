"""Probe: does memory the HIP runtime pins on its own (for a device-to-host copy into pageable
memory) look like caller-pinned memory to hipPointerGetAttributes -- and so to the library's
in-place / direct-output checks (fdf_api.cpp run_host)?

No kernel here touches memory it does not own; every step only queries attributes or runs
ordinary copies and one fdf_detect.  Prints one JSON object per probe."""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from feature_detector_fast_amd import _native  # noqa: E402
import workloads  # noqa: E402


class Attr(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int), ("device", ctypes.c_int),
                ("devicePointer", ctypes.c_void_p), ("hostPointer", ctypes.c_void_p),
                ("isManaged", ctypes.c_int), ("allocationFlags", ctypes.c_uint)]


def main():
    torch.cuda.init()
    _native.load()
    hip = ctypes.CDLL("libamdhip64.so.7", mode=os.RTLD_NOLOAD | os.RTLD_NOW)
    for fn in ("hipPointerGetAttributes", "hipGetLastError", "hipHostRegister",
               "hipHostUnregister", "hipHostGetFlags"):
        getattr(hip, fn).restype = ctypes.c_int

    def attr(p):
        a = Attr()
        rc = hip.hipPointerGetAttributes(ctypes.byref(a), ctypes.c_void_p(p))
        hip.hipGetLastError()
        fl = ctypes.c_uint(0)
        rf = hip.hipHostGetFlags(ctypes.byref(fl), ctypes.c_void_p(p))
        hip.hipGetLastError()
        return {"rc": rc, "type": a.type, "dev": a.devicePointer or 0,
                "dev_eq_host": (a.devicePointer or 0) == p, "flags": a.allocationFlags,
                "hostGetFlags_rc": rf, "hostGetFlags": fl.value}

    out = []
    # 1. torch pageable destinations of D2H copies, by size
    keep = []
    for size in (24, 4096, 60000, 65536, 70000, 1 << 20, 8 << 20):
        d = (torch.arange(size, device="cuda") % 251).to(torch.uint8)
        h = torch.empty(size, dtype=torch.uint8)
        p = h.data_ptr()
        before = attr(p)
        h.copy_(d)
        torch.cuda.synchronize()
        rec = {"probe": "torch_d2h", "size": size, "before": before, "after": attr(p),
               "after_mid": attr(p + size // 2), "after_last": attr(p + size - 1)}
        out.append(rec)
        print(json.dumps(rec), flush=True)
        keep.append((h, d))
    # 2. does the state outlive the tensor?  free, reallocate the same size, look again
    sizes = [t[0].numel() for t in keep]
    ptrs = [t[0].data_ptr() for t in keep]
    keep.clear()
    again = []
    for size, p in zip(sizes, ptrs):
        a = np.empty(size, dtype=np.uint8)
        again.append(a)
        rec = {"probe": "realloc_numpy", "size": size, "old_ptr_attr": attr(p),
               "new_same_addr": a.ctypes.data == p, "new_attr": attr(a.ctypes.data)}
        out.append(rec)
        print(json.dumps(rec), flush=True)
    # 3. numpy destination (torch.from_numpy) of a 1080p-sized D2H copy, then fdf_detect on
    # it: does the library read this pageable frame in place (scores -> FDF_ERR_ARG)?
    W, H = 1920, 1080
    img = workloads.s1_frame(7)
    frame = np.empty(W * H, dtype=np.uint8)
    torch.from_numpy(frame).copy_(torch.from_numpy(img.reshape(-1)).cuda())
    torch.cuda.synchronize()
    fa = attr(frame.ctypes.data)
    lib = _native.load()
    ctx = _native.Context(0)
    cfg = _native.FdfConfig(16, 9, 1)
    pts = np.zeros((W * H, 2), dtype=np.uint32)
    got = ctypes.c_size_t(0)
    rc = lib.fdf_detect(ctx.handle, ctypes.c_void_p(frame.ctypes.data), W, H, W,
                        ctypes.byref(cfg), pts.ctypes.data, W * H, ctypes.byref(got))
    sc = np.zeros(max(got.value, 1), dtype=np.uint16)
    g2 = ctypes.c_size_t(0)
    rs = lib.fdf_fetch_last(ctx.handle, pts.ctypes.data, sc.ctypes.data, got.value,
                            ctypes.byref(g2))
    rec = {"probe": "fdf_detect_on_d2h_destination", "frame_attr": fa, "detect_rc": rc,
           "n": got.value, "scores_rc": rs,
           "read_in_place": rs == _native.FDF_ERR_ARG}
    out.append(rec)
    print(json.dumps(rec), flush=True)
    ctx.close()
    # 4. hipHostRegister / Unregister over a range the runtime pinned for a copy
    buf = np.empty(4 << 20, dtype=np.uint8)
    torch.from_numpy(buf).copy_(torch.zeros(4 << 20, dtype=torch.uint8, device="cuda"))
    torch.cuda.synchronize()
    base = buf.ctypes.data + (-buf.ctypes.data) % 4096
    r0 = attr(base)
    rr = hip.hipHostRegister(ctypes.c_void_p(base), ctypes.c_size_t(1 << 20), ctypes.c_uint(0))
    hip.hipGetLastError()
    r1 = attr(base)
    ru = hip.hipHostUnregister(ctypes.c_void_p(base))
    hip.hipGetLastError()
    r2 = attr(base)
    rec = {"probe": "register_over_runtime_pinned", "before": r0, "register_rc": rr,
           "registered": r1, "unregister_rc": ru, "after_unregister": r2}
    out.append(rec)
    print(json.dumps(rec), flush=True)
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/probe_pinned_cache.json", "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
