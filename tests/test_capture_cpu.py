"""Native V4L2 capture (csrc/host/v4l2.cpp): the YUYV/UYVY -> BGR conversion against
the float BT.601 limited-range formula, and the capture path's failure modes on a
machine without a camera. Parity with OpenCV's own conversion is unpinned (cv2 is
not importable); the reference reads its camera at /root/reference/sem_seg_server.py:144-148."""
import os

import numpy as np
import pytest

from semantic_segmentation_server_amd.ops.native import host
from semantic_segmentation_server_amd.runtime.sources import V4L2Source, make_source


def _ref_bgr(y, u, v):
    c = np.maximum(y.astype(np.float64) - 16, 0)
    d = u.astype(np.float64) - 128
    e = v.astype(np.float64) - 128
    r = 1.164 * c + 1.596 * e
    g = 1.164 * c - 0.391 * d - 0.813 * e
    b = 1.164 * c + 2.018 * d
    return np.clip(np.stack([b, g, r], -1), 0, 255)


@pytest.mark.parametrize("uyvy", [False, True])
def test_yuv422_to_bgr_matches_bt601(uyvy):
    rng = np.random.default_rng(3)
    H, W = 7, 10
    y = rng.integers(0, 256, (H, W), dtype=np.uint8)
    u = rng.integers(0, 256, (H, W // 2), dtype=np.uint8)
    v = rng.integers(0, 256, (H, W // 2), dtype=np.uint8)
    packed = np.empty((H, 2 * W), np.uint8)
    if uyvy:
        packed[:, 0::4], packed[:, 1::4], packed[:, 2::4], packed[:, 3::4] = u, y[:, 0::2], v, y[:, 1::2]
    else:
        packed[:, 0::4], packed[:, 1::4], packed[:, 2::4], packed[:, 3::4] = y[:, 0::2], u, y[:, 1::2], v
    out = host().yuv422_to_bgr(packed, uyvy)
    ref = _ref_bgr(y, np.repeat(u, 2, axis=1), np.repeat(v, 2, axis=1))
    assert out.shape == (H, W, 3) and out.dtype == np.uint8
    assert np.abs(out.astype(np.float64) - ref).max() <= 1.0  # 20-bit fixed point vs float


def test_yuv422_rejects_odd_width():
    with pytest.raises(ValueError):
        host().yuv422_to_bgr(np.zeros((2, 6), np.uint8))


def test_missing_camera_raises():
    dev = "/dev/video-ssa-missing"
    assert not os.path.exists(dev)
    with pytest.raises(RuntimeError, match="open"):
        host().V4L2Capture(dev, 640, 480)
    with pytest.raises(RuntimeError):
        V4L2Source(0, device=dev)


def test_non_capture_device_raises():
    # /dev/null opens but answers no V4L2 ioctl
    with pytest.raises(RuntimeError, match="QUERYCAP"):
        host().V4L2Capture("/dev/null", 640, 480)


def test_make_source_camera_uses_native_capture(monkeypatch):
    monkeypatch.delenv("SSA_CAPTURE", raising=False)
    if os.path.exists("/dev/video1"):
        pytest.skip("a camera is attached")
    with pytest.raises(RuntimeError):
        make_source("camera", camera_idx=1)
