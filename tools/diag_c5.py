"""Diagnostic: bench.py's config-5 leg on its own and after the 1080p legs of bench.main on
the same lanes, with the keypoint total of a fresh context beside it.
    python tools/diag_c5.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import bench
    import workloads
    from feature_detector_fast_amd import Config, NonMaximalSuppression as N, fast_hip
    from oracle import oracle

    dev = torch.device("cuda", 0)
    lanes = fast_hip.Lanes(3, 0)
    res = {}

    def c5(tag):
        r = bench.config5_4k(fast_hip, Config, N, workloads, lanes, dev, oracle.detect, settle=1.0)
        res[tag] = {"kp": r["keypoints_per_step"], "ms": r["kernel_ms_avg"],
                    "single_ms": r["single_lane"]["kernel_ms_avg"], "parity": r["parity"]}
        print(tag, json.dumps(res[tag]), flush=True)

    batch = workloads.s1_frames_torch(0, 128, 3840, 2160, device=dev)
    out = torch.empty((128 * 120_000, 2), dtype=torch.int32, device=dev)
    offs = torch.zeros(129, dtype=torch.int64, device=dev)
    torch.cuda.synchronize()
    fast_hip.detect_device(batch, Config(8, 12, N.SumAbsolute), out, offs)
    torch.cuda.synchronize()
    res["fresh_total"] = int(offs[-1])
    print("fresh_total", res["fresh_total"], flush=True)
    del batch, out, offs
    c5("isolated")
    copies = bench.make_batch(workloads, 0, 512, 1920, 1080, dev, min_bytes=1 << 29)
    bufs = bench.LaneBufs(3, 512 * 200_000, 512, dev)
    for nms in (1, 0, 2):
        bench.timed_steps(fast_hip, lanes, bufs, copies, Config(16, 9, N(nms)), 50, 10, 1, settle=1.0)
    c5("after_1080p")
    print(json.dumps(res))


if __name__ == "__main__":
    main()
