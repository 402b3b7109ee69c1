"""MI355X-native drop-in for the hot path of iwanders/feature_detector_fast.

Mirrors the reference crate API (src/lib.rs:9-64) over the C ABI of include/fdf.h:

    reference                                   here
    Point {x, y}                (lib.rs:17-20)  Point
    NonMaximalSuppression       (lib.rs:26-36)  NonMaximalSuppression
    Config {threshold, count,   (lib.rs:40-52)  Config
            non_maximal_supression}
    Config::detect(&img)        (lib.rs:56-58)  Config.detect(img)
    detect(&img, &config)       (lib.rs:62-64)  detect(img, config)
    fast_simd::detector         (fast_simd.rs:847)  fast_hip.detector(img, config)

Images are 8-bit grayscale: a 2-D numpy uint8 array (H, W) or a :class:`GrayImage`.
Where the reference panics (count outside [9, 16], degenerate sizes) these raise
:class:`FdfError`.  Every call runs on the HIP kernels; there is no CPU fallback.
"""
from ._native import FdfError  # noqa: F401
from .types import Config, GrayImage, NonMaximalSuppression, Point  # noqa: F401
from . import fast_hip  # noqa: F401


def detect(img, config):
    """Perform FAST keypoint detection (src/lib.rs:62-64)."""
    return fast_hip.detector(img, config)


__all__ = ["Config", "GrayImage", "NonMaximalSuppression", "Point", "FdfError", "detect",
           "fast_hip"]
