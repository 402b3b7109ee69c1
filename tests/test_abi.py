"""CPU tests of the C-ABI library: it loads, exports every symbol include/fdf.h declares,
validates configurations exactly like the reference's panics, and fails loudly (never a
silent CPU fallback) when no HIP device is present."""
import ctypes
import os
import re

import numpy as np
import pytest

from feature_detector_fast_amd import Config, FdfError, NonMaximalSuppression, fast_hip
from feature_detector_fast_amd import _native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    text = open(os.path.join(ROOT, "include", "fdf.h")).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\*?\s+\*?(fdf_\w+)\(", text, re.M)))


def test_header_symbols_are_exported():
    lib = _native.load()
    syms = declared_symbols()
    assert len(syms) == len(_native.EXPORTED_SYMBOLS)
    assert sorted(_native.EXPORTED_SYMBOLS) == syms
    for name in syms:
        assert hasattr(lib, name), name


def test_abi_version_and_status_strings():
    lib = _native.load()
    assert lib.fdf_abi_version() == 6
    for code in range(8):
        assert lib.fdf_status_string(code)
    assert _native.status_string(_native.FDF_ERR_COUNT).startswith("count")


def _validate(w, h, t, n, nms):
    lib = _native.load()
    empty = ctypes.c_int(-1)
    cfg = _native.FdfConfig(t, n, nms)
    rc = lib.fdf_validate(w, h, ctypes.byref(cfg), ctypes.byref(empty))
    return rc, empty.value


@pytest.mark.parametrize("w,h,n,nms,rc,empty", [
    (1920, 1080, 9, 0, 0, 0), (1920, 1080, 16, 2, 0, 0), (1920, 1080, 8, 0, 1, -1),
    (1920, 1080, 17, 1, 1, -1), (1920, 1080, 9, 3, 4, -1), (10, 2, 9, 0, 2, 0),
    (0, 5, 9, 0, 0, 1), (5, 7, 9, 0, 2, 0), (6, 9, 9, 0, 0, 1), (7, 7, 9, 0, 0, 0)])
def test_validate_mirrors_reference_rules(w, h, n, nms, rc, empty):
    got_rc, got_empty = _validate(w, h, 16, n, nms)
    assert got_rc == rc
    if empty >= 0:
        assert got_empty == empty


def test_validate_agrees_with_oracle():
    from oracle import oracle

    for h in range(0, 10):
        for w in (0, 3, 5, 6, 7, 20):
            for n in (8, 9, 16, 17):
                o_rc, o_empty = oracle.check(w, h, n, 0)
                rc, empty = _validate(w, h, 16, n, 0)
                assert (o_rc < 0) == (rc != 0), (w, h, n)
                if rc == 0:
                    assert bool(empty) == o_empty


def test_no_device_fails_loudly():
    if _native.load().fdf_device_count() > 0:
        pytest.skip("a HIP device is present")
    with pytest.raises(FdfError) as e:
        fast_hip.detect_array(np.zeros((20, 20), np.uint8), Config(16, 9))
    assert e.value.status == _native.FDF_ERR_DEVICE


def test_python_config_validation():
    with pytest.raises(ValueError):
        fast_hip._to_c_config(Config(300, 9))
    with pytest.raises(TypeError):
        fast_hip._to_c_config((16, 9, 0))
    assert fast_hip.calculate_offsets(100)[0] == -300
    assert fast_hip.circle()[fast_hip.EAST] == (3, 0)
    assert int(NonMaximalSuppression.SumAbsolute) == 2
