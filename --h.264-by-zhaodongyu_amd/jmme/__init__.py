"""jmme -- MI355X-native JM 18.5 integer-pel motion estimation (host side).

Mirrors the JM 18.5 lencod ME interface (encoder.cfg keys, get_mem2Dpel frame
buffers, the IntPelME search contract) over the C ABI of libjmme.so
(include/jmme.h).  See DESIGN.md.
"""
from ._lib import (BLK_CHECK00, BLOCK_REQ, BLOCK_RES, DISTBLK_MAX, EPZS_BOUNDS, EPZS_REQ, EPZS_RES,  # noqa: F401
                   FAST_FULL_SEARCH,
                   FRACTAL_MB, FRACTAL_NODE, FRACTAL_REQ, FRACTAL_RES, FULL_SEARCH, MB_REQ, NSLOT, QUANT4x4_PARAMS, RESID4x4_REQ,
                   RESID4x4_RES,
                   SP_CHECK0, SP_TEST8x8, SUBPEL_REQ, TRANSFORM_OPS, JmmeError)
from .engine import MotionEstimator, config_from_cfg, slot_of, spiral  # noqa: F401
