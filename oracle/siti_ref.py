"""numpy P.910 SI/TI reference ("the numpy reference" of BASELINE.json north_star).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, never by the product.

The reference repository has no SI/TI implementation;
its hooks are util/SRC_analysis.py:120-147 (analyse_src) and
util/complexity_classification.py:50-69 (get_difficulty).  This module is the
written spec "PP-SITI-1" (identical to oracle/siti_oracle.c):

* luma only, raw code values at native bit depth;
* Sobel 3x3, Gx = [[-1,0,1],[-2,0,2],[-1,0,1]], Gy = Gx^T, "valid" region
  (the 1-px border is dropped);
* SI_n = population std (ddof=0) of hypot(Gx, Gy);
* TI_n = population std of Y_n - Y_{n-1} over the full frame, n >= 1
  (TI_0 = NaN);
* SI = max_n SI_n, TI = max_n TI_n.

Parity unpinned against the reference (no implementation exists); pinned by
known-answer tests (tests/test_oracle_siti.py) and a scipy.ndimage cross-check.
"""
import numpy as np

SOBEL_X = np.array([[-1, 0, 1], [-2, 0, 2], [-1, 0, 1]], dtype=np.int64)
SOBEL_Y = SOBEL_X.T.copy()


def sobel_valid(y):
    """Gx, Gy on the valid region of one luma frame (int64 arrays)."""
    y = np.asarray(y, dtype=np.int64)
    h, w = y.shape
    gx = np.zeros((h - 2, w - 2), dtype=np.int64)
    gy = np.zeros((h - 2, w - 2), dtype=np.int64)
    for dy in range(3):
        for dx in range(3):
            win = y[dy:dy + h - 2, dx:dx + w - 2]
            if SOBEL_X[dy, dx]:
                gx += SOBEL_X[dy, dx] * win
            if SOBEL_Y[dy, dx]:
                gy += SOBEL_Y[dy, dx] * win
    return gx, gy


def si_frame(y):
    gx, gy = sobel_valid(y)
    mag = np.sqrt((gx * gx + gy * gy).astype(np.float64))
    return float(np.std(mag))


def ti_frame(y, prev):
    d = np.asarray(y, dtype=np.int64) - np.asarray(prev, dtype=np.int64)
    return float(np.std(d.astype(np.float64)))


def siti(frames, prev=None, bitdepth=None, normalize=False):
    """Per-frame (si, ti) arrays for a [N, H, W] luma stack.

    ``prev`` is the frame preceding frames[0] (a 1-frame halo when a long SRC
    is split across workers), else TI_0 is NaN.  ``normalize`` (with
    ``bitdepth``): both divided by 2^(bitdepth-8), the optional 8-bit-scale
    normalisation of SURVEY.md 8a-13 (PP_SITI_NORMALIZE).
    """
    frames = np.asarray(frames)
    n = frames.shape[0]
    si = np.empty(n, dtype=np.float64)
    ti = np.empty(n, dtype=np.float64)
    for i in range(n):
        si[i] = si_frame(frames[i])
        p = frames[i - 1] if i else prev
        ti[i] = ti_frame(frames[i], p) if p is not None else np.nan
    if normalize:
        k = 1.0 / (1 << (int(bitdepth) - 8))
        si, ti = si * k, ti * k
    return si, ti


def siti_summary(si, ti):
    """(SI, TI) = max over frames; NaN TI entries are ignored."""
    ti = np.asarray(ti, dtype=np.float64)
    valid = ti[~np.isnan(ti)]
    return float(np.max(si)), (float(np.max(valid)) if valid.size else float("nan"))
