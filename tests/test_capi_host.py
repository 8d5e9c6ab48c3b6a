"""Host-side checks of libjmme.so that need no GPU: the library loads, exports
every symbol include/jmme.h declares, and its host-computable tables (spiral
order, mvbits, slot geometry, .cfg parsing, max_mvd) equal JM's.
"""
import ctypes
import os
import re

import numpy as np
import pytest

import oracle_lib as ol
from conftest import REPO


def _declared_functions():
    text = open(os.path.join(REPO, "include", "jmme.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    names = re.findall(r"\b(jmme_[a-z0-9_]+)\s*\(", text)
    return sorted(set(names))


def test_library_exports_every_declared_symbol(built_lib):
    names = _declared_functions()
    assert len(names) >= 15
    missing = [n for n in names if not hasattr(built_lib, n)]
    assert not missing, missing


def test_spiral_order_matches_jm(built_lib):
    for R in (0, 1, 2, 7, 16, 32, 44, 64):
        ref = ol.spiral(R).astype(np.int32)          # JM's own loop (oracle restatement)
        for i, (x, y) in enumerate(ref):
            assert built_lib.jmme_spiral_index(int(x), int(y)) == i
        ox, oy = ctypes.c_int(), ctypes.c_int()
        for i in range(0, len(ref), max(1, len(ref) // 997)):
            built_lib.jmme_spiral_offset(i, ctypes.byref(ox), ctypes.byref(oy))
            assert (ox.value, oy.value) == tuple(ref[i])


@pytest.mark.parametrize("R", [4, 16, 32, 64])
def test_mvbits_matches_jm_table(built_lib, R):
    max_mvd, table = ol.mvbits_table(R)
    for v in range(-max_mvd, max_mvd + 1):
        assert built_lib.jmme_mvbits(v) == table[max_mvd + v], v


def test_slot_geometry():
    from jmme import slot_of
    # JM block_size (macroblock.h:58) and BlockSAD indexing (me_fullfast.c:640)
    sizes = {1: (4, 4), 2: (4, 2), 3: (2, 4), 4: (2, 2), 5: (2, 1), 6: (1, 2), 7: (1, 1)}
    seen = set()
    for bt, (w, h) in sizes.items():
        for by in range(0, 4, h):
            for bx in range(0, 4, w):
                s = slot_of(bt, bx, by)
                assert 0 <= s < 41 and s not in seen
                seen.add(s)
    assert len(seen) == 41
    assert slot_of(2, 0, 1) == -1 and slot_of(8, 0, 0) == -1


CFG_TEXT = """
# a JM-style encoder.cfg (syntax of JM/bin/encoder_baseline.cfg)
SourceWidth           = 1920   # Source frame width
SourceHeight          = 1080
SearchMode            = 0      # -1 FS, 0 FFS
SearchRange           = 16
RDOptimization        =  1  # rd-optimized mode decision
InputFile             = "foreman_part_qcif.yuv"   # strings are skipped
LambdaWeightPSlice    =  0.68
RestrictSearchRange   =  2
"""


def test_config_parse_file_and_overrides(tmp_path):
    from jmme import config_from_cfg
    p = tmp_path / "enc.cfg"
    p.write_text(CFG_TEXT)
    c = config_from_cfg(str(p), {"SearchMode": -1, "SearchRange": 32, "DisableSubpelME": 1})
    d = c.as_dict()
    assert d["SourceWidth"] == 1920 and d["SourceHeight"] == 1080
    assert d["SearchMode"] == -1 and d["SearchRange"] == 32      # -p wins over the file
    assert d["RDOptimization"] == 1 and d["DisableSubpelME"] == 1 and d["RestrictSearchRange"] == 2


def test_config_rejects_malformed_value(tmp_path):
    from jmme import config_from_cfg, JmmeError
    p = tmp_path / "bad.cfg"
    p.write_text("SearchRange = abc\n")
    with pytest.raises(JmmeError):
        config_from_cfg(str(p))


@pytest.mark.parametrize("R", [7, 16, 32, 64])
def test_max_mvd_matches_jm(built_lib, R):
    from jmme import config_from_cfg
    c = config_from_cfg(None, {"SearchRange": R})
    assert built_lib.jmme_max_mvd(ctypes.byref(c)) == ol.mvbits_table(R)[0]


def test_max_mvd_matches_captured_runs():
    import golden_io as g
    from jmme import config_from_cfg
    for name in g.cases():
        m = g.manifest()[name]
        c = g.Case(name)
        cfg = config_from_cfg(None, {"SearchRange": m["cfg_overrides"]["SearchRange"]})
        from jmme import _lib
        assert _lib.lib().jmme_max_mvd(ctypes.byref(cfg)) == int(c.r["max_mvd"][0])
