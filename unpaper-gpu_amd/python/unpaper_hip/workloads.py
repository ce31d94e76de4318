"""The BASELINE.json configurations as (geometry, options) pairs, shared by
bench.py, the GPU tests and the golden-hash generators.

C2/C3/C5: GRAY8 A4@300dpi pages (2480x3508), the reference defaults
          (lib/options.c == uphip_options_init).
C4:       RGB24 600dpi double-page scans (9920x7016, synth.h synth_rgb_channel):
          --layout double (sheet_stages.c:232-279 points/masks per half),
          --interpolate linear (deskew rotate bilinear), and a border wipe
          (--border 60,60,60,60: sheet_stages.c wipe stage, apply_border).
"""
import ctypes as C

from . import ctypes_abi as A

A4_W, A4_H = 2480, 3508
C4_W, C4_H = 9920, 7016
C4_BORDER = 60


def default_options(lib):
    o = A.Options()
    lib.uphip_options_init(C.byref(o))
    return o


def c4_options(opts):
    """Apply the C4 switches to a default option block (in place)."""
    opts.layout = A.LAYOUT_DOUBLE
    opts.interpolate_type = A.INTERP_LINEAR
    opts.border = A.Border(C4_BORDER, C4_BORDER, C4_BORDER, C4_BORDER)
    return opts
