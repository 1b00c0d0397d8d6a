"""CPU restatement of the reference's episode transforms (TEST INFRASTRUCTURE ONLY: imported by
tests/ as the checker of csrc/preprocess.hip; never by the product path).

  * transform.py:110-167 ``Resize``: ``find_new_hw`` (longer side -> S, the other scaled by
    int(), both floored to a multiple of 8), cv2.resize INTER_LINEAR of the fp32 image, top-left
    placement on an S x S canvas (0, or mean*255 with ``padding: avg``), the label by
    INTER_NEAREST on an S x S canvas of 255;
  * transform.py:59-84 ``ToTensor`` (HWC -> CHW, /255 in fp32) and :87-107 ``Normalize``;
  * dataset.py:222-228 / 261-266 the episode label remap (chosen class -> 1, 255 kept, else 0);
  * transform.py ``RandomHorizontalFlip`` / ``RandomVerticalFlip`` (cv2.flip) before the resize.

cv2 is not installed in this image, so the cv2.resize arithmetic is restated from OpenCV's
published resize.cpp (float path: per-destination-column taps fx = (float)((dx + 0.5) * scale
- 0.5), sx = floor(fx), clamped at both edges with fx = 0; a horizontal pass of two products
and a sum per source row, then the same vertical blend, all fp32; INTER_NEAREST:
min(floor(dx * scale), src - 1)).  Parity against cv2 itself is therefore UNPINNED; the HIP
kernels are pinned bit-exactly against this restatement.
"""
from __future__ import annotations

import numpy as np


def find_new_hw(h: int, w: int, S: int):
    """transform.py:117-135."""
    if h >= w:
        new_h, new_w = S, int(w * (S * 1.0 / h))
    else:
        new_h, new_w = int(h * (S * 1.0 / w)), S
    if new_h % 8 != 0:
        new_h = int(new_h / 8) * 8
    if new_w % 8 != 0:
        new_w = int(new_w / 8) * 8
    return new_h, new_w


def _linear_taps(dst: int, src: int):
    scale = 1.0 / (dst / src)
    d = np.arange(dst, dtype=np.float64)
    f = ((d + 0.5) * scale - 0.5).astype(np.float32)
    s = np.floor(f).astype(np.int64)
    f = (f - s.astype(np.float32)).astype(np.float32)
    lo = s < 0
    s[lo], f[lo] = 0, np.float32(0)
    hi = s >= src - 1
    s[hi], f[hi] = src - 1, np.float32(0)
    return s, np.minimum(s + 1, src - 1), (np.float32(1) - f).astype(np.float32), f


def cv2_resize_linear_f32(img: np.ndarray, new_w: int, new_h: int) -> np.ndarray:
    """cv2.resize(img fp32 HxWxC, (new_w, new_h), INTER_LINEAR)."""
    img = img.astype(np.float32)
    H, W = img.shape[:2]
    x0, x1, wx0, wx1 = _linear_taps(new_w, W)
    y0, y1, wy0, wy1 = _linear_taps(new_h, H)
    rows = img[:, x0] * wx0[None, :, None] + img[:, x1] * wx1[None, :, None]     # [H, new_w, C] fp32
    return (rows[y0] * wy0[:, None, None] + rows[y1] * wy1[:, None, None]).astype(np.float32)


def cv2_resize_nearest(a: np.ndarray, new_w: int, new_h: int) -> np.ndarray:
    """cv2.resize(a, (new_w, new_h), INTER_NEAREST)."""
    H, W = a.shape[:2]
    ys = np.minimum(np.floor(np.arange(new_h) * (1.0 / (new_h / H))).astype(np.int64), H - 1)
    xs = np.minimum(np.floor(np.arange(new_w) * (1.0 / (new_w / W))).astype(np.int64), W - 1)
    return a[ys][:, xs]


def remap_label(label: np.ndarray, class_chosen: int) -> np.ndarray:
    """dataset.py:222-228: 255 -> 255, class_chosen -> 1, everything else 0."""
    out = np.zeros_like(label)
    out[label == 255] = 255
    out[label == class_chosen] = 1
    return out


def val_transform(image: np.ndarray, label: np.ndarray | None, S: int, mean, std, padding=None,
                  flip_h: bool = False, flip_v: bool = False):
    """[flips] -> Resize(S, padding) -> ToTensor -> Normalize.  image HxWx3 (uint8 or fp32 RGB),
    label HxW (already remapped) -> (fp32 [3,S,S], int64 [S,S])."""
    image = np.float32(image)
    if flip_h:
        image, label = image[:, ::-1], (label[:, ::-1] if label is not None else None)
    if flip_v:
        image, label = image[::-1], (label[::-1] if label is not None else None)
    nh, nw = find_new_hw(image.shape[0], image.shape[1], S)
    canvas = np.zeros((S, S, 3))
    if padding:
        canvas[:, :, :] = np.asarray(padding, np.float64)[None, None, :]
    canvas[:nh, :nw, :] = cv2_resize_linear_f32(np.ascontiguousarray(image), nw, nh)
    t = canvas.transpose(2, 0, 1).astype(np.float32) / np.float32(255)
    for c in range(3):
        t[c] = (t[c] - np.float32(mean[c])) / np.float32(std[c])
    lab = None
    if label is not None:
        lh, lw = find_new_hw(label.shape[0], label.shape[1], S)
        lab = np.full((S, S), 255.0)
        lab[:lh, :lw] = cv2_resize_nearest(np.ascontiguousarray(label).astype(np.float32), lw, lh)
        lab = lab.astype(np.int64)
    return t.astype(np.float32), lab
