"""Seeded synthetic YUV 4:2:0 8-bit sequences for ME parity tests and the bench.

SURVEY.md §8(d) "Synthetic inputs": luma is a box-filtered uniform-noise
texture translated by a per-frame global motion vector plus N(0, sigma) noise;
chroma is flat 128.  The "adversarial" variant moves every 16x16 macroblock by
its own random vector within +-R, which defeats JM's early-exit SAD.

Pure numpy, deterministic for a given (seed, size, frames).  The same bytes
are written to a .yuv file for JM (oracle/_ref/lencod) and fed to the HIP path,
so both see identical input.
"""
from __future__ import annotations

import numpy as np


def _texture(rng: np.random.Generator, h: int, w: int, box: int = 5) -> np.ndarray:
    t = rng.uniform(0.0, 255.0, size=(h + box, w + box))
    # separable box filter (integral image): spatially correlated texture
    c = np.cumsum(np.cumsum(t, axis=0), axis=1)
    c = np.pad(c, ((1, 0), (1, 0)))
    s = c[box:, box:] - c[:-box, box:] - c[box:, :-box] + c[:-box, :-box]
    s = s[:h, :w] / (box * box)
    # stretch contrast back toward the full 8-bit range
    s = (s - s.mean()) * 3.0 + 128.0
    return s


def luma_sequence(width: int, height: int, frames: int, seed: int = 1234,
                  gmv: tuple[int, int] = (5, 3), noise_sigma: float = 2.0,
                  adversarial: bool = False, adv_range: int = 32) -> np.ndarray:
    """Return uint8 [frames, height, width] luma planes."""
    rng = np.random.default_rng(seed)
    mx, my = gmv
    margin = max(abs(mx), abs(my)) * frames + adv_range + 8
    tex = _texture(rng, height + 2 * margin, width + 2 * margin)
    out = np.empty((frames, height, width), dtype=np.uint8)
    for t in range(frames):
        ox, oy = margin + t * mx, margin + t * my
        f = tex[oy:oy + height, ox:ox + width].copy()
        if adversarial and t > 0:
            for by in range(0, height, 16):
                for bx in range(0, width, 16):
                    dx, dy = rng.integers(-adv_range, adv_range + 1, size=2)
                    sy, sx = oy + by + dy, ox + bx + dx
                    hh, ww = min(16, height - by), min(16, width - bx)
                    f[by:by + hh, bx:bx + ww] = tex[sy:sy + hh, sx:sx + ww]
        f = f + rng.normal(0.0, noise_sigma, size=f.shape)
        out[t] = np.clip(np.rint(f), 0, 255).astype(np.uint8)
    return out


def write_yuv420(path: str, luma: np.ndarray) -> None:
    """Write planar I420 (chroma = 128) for JM's InputFile."""
    f, h, w = luma.shape
    chroma = np.full((h // 2, w // 2), 128, dtype=np.uint8).tobytes()
    with open(path, "wb") as fp:
        for t in range(f):
            fp.write(luma[t].tobytes())
            fp.write(chroma)
            fp.write(chroma)


def read_yuv420_luma(path: str, width: int, height: int, frames: int | None = None) -> np.ndarray:
    fsize = width * height * 3 // 2
    data = np.fromfile(path, dtype=np.uint8)
    n = data.size // fsize if frames is None else frames
    out = np.empty((n, height, width), dtype=np.uint8)
    for t in range(n):
        out[t] = data[t * fsize:t * fsize + width * height].reshape(height, width)
    return out


def luma_sequence_hbd(width: int, height: int, frames: int, bits: int, seed: int = 1234,
                      gmv: tuple[int, int] = (5, 3), adversarial: bool = False) -> np.ndarray:
    """uint16 [frames, height, width] luma at `bits` (9..14): the 8-bit clip scaled
    by 2^(bits-8) plus seeded low-order noise that only a high-bit-depth search sees."""
    luma = luma_sequence(width, height, frames, seed=seed, gmv=gmv, adversarial=adversarial).astype(np.int32)
    sh = bits - 8
    rng = np.random.default_rng(seed + 0x10B17)
    return np.clip((luma << sh) + rng.integers(0, 1 << sh, size=luma.shape), 0, (1 << bits) - 1).astype(np.uint16)


def write_yuv420_16(path: str, luma: np.ndarray, bits: int) -> None:
    """Planar I420 with 16-bit little-endian samples (JM reads two bytes per
    sample above 8 bits); chroma mid-grey."""
    f, h, w = luma.shape
    grey = np.full((h // 2, w // 2), 1 << (bits - 1), np.uint16).astype("<u2").tobytes()
    with open(path, "wb") as fp:
        for t in range(f):
            fp.write(luma[t].astype("<u2").tobytes())
            fp.write(grey)
            fp.write(grey)
