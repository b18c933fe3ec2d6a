"""Image metrics.

mape8   — the reference's metric, restated from Graphing/mape.py:10-21:
          sum(|gt/255 - p/255| / ((gt + 0.01)/255)) / (H*W*3) on 8-bit RGB.
mape_f  — the per-pixel float MAPE of BASELINE.md's parity gate:
          mean |a - f| / (a + 0.01/255) over pixels x channels.
"""
from __future__ import annotations

import numpy as np


def mape8(gt8: np.ndarray, p8: np.ndarray) -> float:
    gt = np.asarray(gt8, np.float64)[..., :3]
    p = np.asarray(p8, np.float64)[..., :3]
    score = np.sum(np.abs(gt / 255 - p / 255) / ((gt + 0.01) / 255))
    return float(score / gt.size)


def mape_f(ref: np.ndarray, test: np.ndarray) -> float:
    a = np.asarray(ref, np.float64)
    f = np.asarray(test, np.float64)
    return float(np.mean(np.abs(a - f) / (a + 0.01 / 255.0)))


def argb_to_rgb8(argb: np.ndarray) -> np.ndarray:
    a = np.asarray(argb, np.uint32)
    return np.stack([(a >> 16) & 255, (a >> 8) & 255, a & 255], axis=-1).astype(np.uint8)
