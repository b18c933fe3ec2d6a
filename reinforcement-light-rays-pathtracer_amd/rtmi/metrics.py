"""Image metrics.

mape8   — the reference's metric, restated from Graphing/mape.py:10-21:
          sum(|gt/255 - p/255| / ((gt + 0.01)/255)) / (H*W*3) on 8-bit RGB.
python -m rtmi.metrics GROUND_TRUTH PREDICTION
        — the reference's CLI (Graphing/mape.py:24-33): prints mape8 of two image files
          (PNG/BMP, read as 8-bit RGB) rounded to 4 places.
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


def read_rgb8(path: str) -> np.ndarray:
    """An image file as H x W x 3 uint8 (scipy.misc.imread(mode='RGB') of mape.py:13-14)."""
    from PIL import Image

    with Image.open(path) as im:
        return np.asarray(im.convert("RGB"), np.uint8)


def mape_files(ground_truth: str, prediction: str) -> float:
    return round(mape8(read_rgb8(ground_truth), read_rgb8(prediction)), 4)


def main(argv=None) -> int:
    import sys

    args = sys.argv[1:] if argv is None else argv
    if len(args) != 2:
        print("Two file paths to images must be given. Terminating.")
        return 1
    print(mape_files(args[0], args[1]))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
