"""Command-line counterpart of the reference's binary (src/main.rs), on the MI355X detector.

    python -m feature_detector_fast_amd <input> [output(default: /tmp/output.png)]
        [threshold(default: 16)] [count(default: 9)]
        [non_maximal_suppression: off|sum_absolute|max_threshold (default: sum_absolute)]

As src/main.rs:17-84: the image is opened as RGB8 and converted with image 0.24.6's
to_luma8 (here on the device, fdf_detect_rgb); the keypoints are written one per line as
"x y" to the output name with ".png" replaced by ".txt" (write_keypoints, :4-15), and an
overlay -- the grey image as RGB with each keypoint's pixel set to red, as
util::draw_plus_sized(.., RED, 1) does (src/util.rs:62-81) -- to the output name.  (The
reference's usage text says the NMS default is max_threshold; its code uses
sum_absolute, which is what is reproduced.)
"""
import sys
import time

import numpy as np

from . import fast_hip
from .types import Config, NonMaximalSuppression

USAGE = ("python -m feature_detector_fast_amd <input> [output(default; /tmp/output.png)] "
         "[threshold(default: 16)] [count(default:9)] "
         "[non_maximal_suppression:off|sum_absolute|max_threshold (default: max_threshold)]\n"
         " arguments required left to right.")

NMS_ARGS = {"off": NonMaximalSuppression.Off,
            "sum_absolute": NonMaximalSuppression.SumAbsolute,
            "max_threshold": NonMaximalSuppression.MaxThreshold}


def luma8(rgb):
    """image 0.24.6 to_luma8 on Rgb<u8>: (2126 r + 7152 g + 722 b) / 10000 (for the overlay;
    detection converts on the device)."""
    r, g, b = (rgb[..., k].astype(np.uint32) for k in range(3))
    return ((2126 * r + 7152 * g + 722 * b) // 10000).astype(np.uint8)


def write_keypoints(points, filename):
    """src/main.rs:4-15: one "x y" line per keypoint."""
    with open(filename, "w") as f:
        for x, y in points:
            f.write(f"{int(x)} {int(y)}\n")


def overlay(grey, points):
    """The grey image as RGB with every keypoint pixel red: draw_plus_sized with size 1
    draws only the centre, and skips pixels with x <= 0 or y <= 0 (src/util.rs:62-81)."""
    rgb = np.repeat(grey[..., None], 3, axis=2)
    h, w = grey.shape
    for x, y in points:
        x, y = int(x), int(y)
        if 0 < x < w and 0 < y < h:
            rgb[y, x] = (255, 0, 0)
    return rgb


def _parse_u8(text, what):
    try:
        v = int(text)
    except ValueError:
        v = -1
    if not 0 <= v <= 255:
        raise SystemExit(f"failed to parse {what}")
    return v


def main(argv=None):
    args = sys.argv[1:] if argv is None else list(argv)
    if not args or (len(args) == 1 and args[0] == "--help"):
        print(USAGE)
        return 0
    from PIL import Image

    input_file = args[0]
    output_image = args[1] if len(args) > 1 else "/tmp/output.png"
    output_txt = output_image.replace(".png", ".txt")
    threshold = _parse_u8(args[2] if len(args) > 2 else "16", "threshold")
    count = _parse_u8(args[3] if len(args) > 3 else "9", "count")
    nms_arg = args[4] if len(args) > 4 else "sum_absolute"
    if nms_arg not in NMS_ARGS:
        raise SystemExit("unknown non maximal, support: off, sum_absolute, max_threshold")
    try:
        rgb = np.asarray(Image.open(input_file).convert("RGB"))
    except OSError as e:
        raise SystemExit(f"could not load image at {input_file!r}: {e}")

    config = Config(threshold, count, NMS_ARGS[nms_arg])
    start = time.perf_counter()
    points = fast_hip.detect_rgb_array(rgb, config)
    elapsed = time.perf_counter() - start
    print(f"Took: {elapsed * 1e3:.3f}ms, found {len(points)} keypoints")

    Image.fromarray(overlay(luma8(rgb), points)).save(output_image)
    write_keypoints(points, output_txt)
    return 0


if __name__ == "__main__":
    sys.exit(main())
