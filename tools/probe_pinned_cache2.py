"""Probe: does the HIP runtime keep a caller's pageable buffer locked (pinned, GPU-mapped)
after a host-to-device copy from it has finished -- and after the buffer is freed?

Queries only (hsa_amd_pointer_info on host addresses); every copy is an ordinary torch copy
from memory the probe owns.  Prints one JSON object per probe.  Round 6, DESIGN.md §7.7."""
import ctypes
import gc
import json
import mmap
import os
import sys

import numpy as np
import torch

HSA_TYPES = {0: "unknown", 1: "hsa", 2: "locked", 3: "graphics", 4: "ipc", 5: "reserved",
             6: "vmem"}


class PtrInfo(ctypes.Structure):
    _fields_ = [("size", ctypes.c_uint32), ("type", ctypes.c_int),
                ("agentBaseAddress", ctypes.c_void_p), ("hostBaseAddress", ctypes.c_void_p),
                ("sizeInBytes", ctypes.c_size_t), ("userData", ctypes.c_void_p),
                ("agentOwner", ctypes.c_uint64), ("global_flags", ctypes.c_uint32),
                ("pad", ctypes.c_uint32 * 16)]


def main():
    torch.cuda.init()
    torch.zeros(1, device="cuda")
    hsa = ctypes.CDLL("libhsa-runtime64.so.1", mode=os.RTLD_NOLOAD | os.RTLD_NOW)
    hsa.hsa_amd_pointer_info.restype = ctypes.c_int
    hsa.hsa_amd_pointer_info.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.c_void_p, ctypes.c_void_p]

    def info(p):
        i = PtrInfo()
        i.size = 56
        rc = hsa.hsa_amd_pointer_info(ctypes.c_void_p(p), ctypes.byref(i), None, None, None)
        return {"rc": rc, "type": HSA_TYPES.get(i.type, i.type),
                "host_base": i.hostBaseAddress or 0, "bytes": i.sizeInBytes}

    out = []

    def emit(rec):
        out.append(rec)
        print(json.dumps(rec), flush=True)

    # positive control: memory locked with hipHostRegister reads as "locked"
    hip = ctypes.CDLL("libamdhip64.so.7", mode=os.RTLD_NOLOAD | os.RTLD_NOW)
    hip.hipHostRegister.restype = ctypes.c_int
    hip.hipHostUnregister.restype = ctypes.c_int
    ctl = np.zeros(1 << 20, dtype=np.uint8)
    rr = hip.hipHostRegister(ctypes.c_void_p(ctl.ctypes.data), ctypes.c_size_t(ctl.size),
                             ctypes.c_uint(0))
    emit({"probe": "control_hipHostRegister", "register_rc": rr, "info": info(ctl.ctypes.data)})
    hip.hipHostUnregister(ctypes.c_void_p(ctl.ctypes.data))
    emit({"probe": "control_after_unregister", "info": info(ctl.ctypes.data)})
    # (no transfer ever runs after something was freed: a transfer at a reused address is
    # the hazard itself)
    # 1. pageable destination of a large device-to-host copy
    d = torch.full((16 << 20,), 5, dtype=torch.uint8, device="cuda")
    h = np.empty(16 << 20, dtype=np.uint8)
    torch.from_numpy(h).copy_(d)
    torch.cuda.synchronize()
    emit({"probe": "d2h_destination_16MB", "info": info(h.ctypes.data)})
    # 2. pageable numpy sources of host-to-device copies, by size: locked after the copy?
    keep = []
    for size in (73544, 1 << 20, 4147200, 16 << 20, 64 << 20):
        a = np.full(size, 7, dtype=np.uint8)
        p = a.ctypes.data
        before = info(p)
        dd = torch.from_numpy(a).cuda()
        torch.cuda.synchronize()
        emit({"probe": "h2d_source", "size": size, "before": before, "after_copy": info(p),
              "after_copy_mid": info(p + size // 2)})
        keep.append((a, dd, p, size))
    # 3. an mmap'd source the probe unmaps itself
    m = mmap.mmap(-1, 8 << 20)
    buf = np.frombuffer(m, dtype=np.uint8)
    buf[:] = 3
    addr = buf.ctypes.data
    dm = torch.from_numpy(buf).cuda()
    torch.cuda.synchronize()
    emit({"probe": "mmap_source_after_copy", "info": info(addr)})
    # 4. queries only from here on: the freed / unmapped addresses
    ptrs = [(p, size) for _, _, p, size in keep]
    keep.clear()
    del buf, dm, h, d
    gc.collect()
    m.close()
    emit({"probe": "mmap_source_after_munmap", "info": info(addr)})
    for p, size in ptrs:
        emit({"probe": "freed_h2d_source", "size": size, "info": info(p)})
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/probe_pinned_cache2.json", "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    sys.exit(main())
