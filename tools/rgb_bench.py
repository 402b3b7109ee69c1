"""The RGB extras of bench.py alone: 256 device-resident 1080p RGB8 frames, two-pass (luma
kernel + grey detector) against fused (fdf_detect_device_rgb)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    import bench
    import workloads
    from feature_detector_fast_amd import Config, NonMaximalSuppression, fast_hip

    frames = workloads.s1_frames_torch(0, 256)
    out = torch.empty((256 * 20000, 2), dtype=torch.int32, device="cuda")
    offs = torch.zeros(257, dtype=torch.int64, device="cuda")
    for nms in (1, 0):
        cfg = Config(16, 9, NonMaximalSuppression(nms))
        r = bench.rgb_path(fast_hip, cfg, frames, out, offs, torch.cuda.current_stream(), steps=20)
        print(json.dumps({"nms": nms, **r}))


if __name__ == "__main__":
    main()
