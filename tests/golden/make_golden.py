"""Regenerate the golden fixtures under tests/golden/ from the reference's media/ PNGs.

Runs only where /root/reference exists (the build container); the outputs are committed so
tests never read the reference at run time.  What it extracts:

* ``screenshot315_grey.pgm`` -- the 300x200 grey input ``media/Screenshot315_torch_grey.png``.
  The PNG is RGB with r == g == b, so ``to_luma8`` (tests/compare.rs:33) is the R channel.
* ``kp_t16_n9_off.txt`` / ``kp_t16_n9_maxt.txt`` -- keypoint lists in the reference CLI's
  ``x y\\n`` format (src/main.rs:4-15), decoded from the overlay PNGs.  Every keypoint is
  drawn as exactly one (255,0,0) pixel (src/util.rs:62-81 with size 1, src/main.rs:76);
  every other pixel equals the grey input.  The Rust overlays and the OpenCV 3.2 overlays
  decode to identical lists, which this script asserts.
"""
import os
import sys

import numpy as np
from PIL import Image

REF_MEDIA = "/root/reference/media"
HERE = os.path.dirname(os.path.abspath(__file__))


def load_rgb(name):
    return np.asarray(Image.open(os.path.join(REF_MEDIA, name)).convert("RGB"))


def decode_overlay(grey, overlay):
    red = (overlay[..., 0] == 255) & (overlay[..., 1] == 0) & (overlay[..., 2] == 0)
    rest = ~red
    assert np.array_equal(overlay[..., 0][rest], grey[rest]), "non-marker pixel differs"
    ys, xs = np.nonzero(red)  # np.nonzero is raster order: y ascending, then x
    return list(zip(xs.tolist(), ys.tolist()))


def write_pgm(path, img):
    h, w = img.shape
    with open(path, "wb") as f:
        f.write(b"P5\n%d %d\n255\n" % (w, h))
        f.write(np.ascontiguousarray(img, dtype=np.uint8).tobytes())


def write_points(path, pts):
    with open(path, "w") as f:
        for x, y in pts:
            f.write(f"{x} {y}\n")


def main():
    if not os.path.isdir(REF_MEDIA):
        sys.exit("reference media not present; fixtures are already committed")
    rgb = load_rgb("Screenshot315_torch_grey.png")
    assert (rgb[..., 0] == rgb[..., 1]).all() and (rgb[..., 1] == rgb[..., 2]).all()
    grey = rgb[..., 0].copy()
    write_pgm(os.path.join(HERE, "screenshot315_grey.pgm"), grey)

    pairs = {
        "kp_t16_n9_off.txt": ("with_rust_threshold_16_consecutive_9.png",
                              "with_opencv_threshold_16_type_9_16.png"),
        "kp_t16_n9_maxt.txt": ("with_rust_threshold_16_consecutive_9.png_nonmax.png",
                               "with_opencv_threshold_16_type_9_16_nonmax.png"),
    }
    for out, (rust_png, cv_png) in pairs.items():
        rust = decode_overlay(grey, load_rgb(rust_png))
        cv = decode_overlay(grey, load_rgb(cv_png))
        assert rust == cv, f"{rust_png} and {cv_png} disagree"
        write_points(os.path.join(HERE, out), rust)
        print(out, len(rust))


if __name__ == "__main__":
    main()
