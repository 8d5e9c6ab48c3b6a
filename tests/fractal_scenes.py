"""Synthetic planes that drive every branch of the thesis's macroblock gate
(encode_one_macroblock / encode_block_8, ZL/src/block_enc.c:508-1675).

The current picture is a smooth texture (so its co-located reference block
stays highly correlated: chun >= 0.9) shifted by a small motion, with per-8x8
offset steps planted on top: a horizontal step makes the 8x8 fail and its
8x4 pair match (partition 1), a vertical step the 4x8 pair (partition 2), a
checkerboard forces four 4x4; steps in enough quadrants push the 16x16 rms
over tol_16^2 * 256 so the macroblock splits.  Flat and saturated macroblocks
give the gate its 0/0 (NaN chun) and clipped cases."""
import numpy as np


def _smooth(h, w, scale, rng):
    c = rng.normal(128, 60, ((h + 8) // scale + 2, (w + 8) // scale + 2))
    y, x = np.arange(h + 8) / scale, np.arange(w + 8) / scale
    y0, x0 = np.floor(y).astype(int), np.floor(x).astype(int)
    fy, fx = (y - y0)[:, None], (x - x0)[None, :]
    return (c[y0][:, x0] * (1 - fy) * (1 - fx) + c[y0 + 1][:, x0] * fy * (1 - fx) +
            c[y0][:, x0 + 1] * (1 - fy) * fx + c[y0 + 1][:, x0 + 1] * fy * fx)


def gate_scene(w, h, seed, n_views=1, scale=8):
    """-> (org, [ref views]) uint8 h x w; w, h multiples of 16"""
    rng = np.random.default_rng(seed)
    big = _smooth(h, w, scale, rng)
    ref = big[4:4 + h, 4:4 + w]
    dx, dy = rng.integers(-1, 2, 2)
    cur = big[4 + dy:4 + dy + h, 4 + dx:4 + dx + w].copy()
    # per-8x8 planted steps
    step = np.zeros((h, w))
    for by in range(0, h, 8):
        for bx in range(0, w, 8):
            kind = rng.choice(4, p=[0.4, 0.2, 0.2, 0.2])
            d = rng.choice([3.0, 8.0, 20.0, 30.0])
            blk = step[by:by + 8, bx:bx + 8]
            if kind == 1:
                blk[:4] += d
                blk[4:] -= d
            elif kind == 2:
                blk[:, :4] += d
                blk[:, 4:] -= d
            elif kind == 3:
                blk[:4, :4] += d
                blk[4:, 4:] += d
                blk[:4, 4:] -= d
                blk[4:, :4] -= d
    cur += step
    cur += rng.normal(0, 1, (h, w)) * rng.choice([0.0, 1.0, 2.0])
    org = np.clip(np.rint(cur), 0, 255).astype(np.uint8)
    # a flat macroblock (sR = 0: the gate's correlation is 0/0) and a
    # saturated one
    mbs = [(x, y) for y in range(0, h, 16) for x in range(0, w, 16)]
    i, j = rng.choice(len(mbs), 2, replace=False)
    x, y = mbs[i]
    org[y:y + 16, x:x + 16] = 77
    x, y = mbs[j]
    org[y:y + 16, x:x + 16] = np.clip(org[y:y + 16, x:x + 16].astype(np.int32) * 3 - 200, 0, 255).astype(np.uint8)
    refs = [np.clip(np.rint(ref), 0, 255).astype(np.uint8)]
    for k in range(1, n_views):
        # other views: the same texture seen with a small disparity and noise
        ox = int(rng.integers(-2, 3))
        v = big[4:4 + h, 4 + ox:4 + ox + w] + rng.normal(0, 2.0 * k, (h, w))
        refs.append(np.clip(np.rint(v), 0, 255).astype(np.uint8))
    return np.ascontiguousarray(org), [np.ascontiguousarray(r) for r in refs]
