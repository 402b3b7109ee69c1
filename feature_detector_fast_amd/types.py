"""Value types of the reference crate (src/lib.rs:15-52)."""
import enum
from dataclasses import dataclass

import numpy as np


@dataclass(frozen=True, order=True)
class Point:
    """A feature point at an image position (src/lib.rs:17-20); ordering = (x, y) fields."""

    x: int
    y: int


class NonMaximalSuppression(enum.IntEnum):
    """src/lib.rs:26-36."""

    Off = 0
    MaxThreshold = 1
    SumAbsolute = 2


@dataclass(frozen=True)
class Config:
    """Detector configuration (src/lib.rs:40-52).  ``non_maximal_supression`` keeps the
    reference's spelling."""

    threshold: int
    count: int
    non_maximal_supression: NonMaximalSuppression = NonMaximalSuppression.Off

    def detect(self, img):
        """src/lib.rs:56-58."""
        from . import fast_hip

        return fast_hip.detector(img, self)


class GrayImage:
    """Minimal stand-in for image::GrayImage: row-major u8 pixels, stride == width."""

    def __init__(self, width, height, raw=None):
        self._w = int(width)
        self._h = int(height)
        if raw is None:
            raw = np.zeros(self._w * self._h, dtype=np.uint8)
        arr = np.frombuffer(bytes(raw), dtype=np.uint8) if not isinstance(raw, np.ndarray) else raw
        if arr.size != self._w * self._h:
            raise ValueError("raw buffer size does not match width * height")
        self._px = np.ascontiguousarray(arr.reshape(self._h, self._w), dtype=np.uint8)

    @classmethod
    def from_array(cls, arr):
        arr = np.asarray(arr)
        return cls(arr.shape[1], arr.shape[0], arr.reshape(-1))

    def width(self):
        return self._w

    def height(self):
        return self._h

    def dimensions(self):
        return (self._w, self._h)

    def as_raw(self):
        return self._px.reshape(-1)

    def array(self):
        return self._px

    def put_pixel(self, x, y, value):
        self._px[y, x] = value

    def get_pixel(self, x, y):
        return int(self._px[y, x])
