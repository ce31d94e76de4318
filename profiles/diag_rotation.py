#!/usr/bin/env python3
"""Diagnostic: how many rotation-detection lines of synthetic A4 pages leave
the shared-band path for the direct walk (UPHIP_DIAG_ROTATION=1 makes the
op-level detect_rotation print the count).  Needs a GPU and the tuning
build (make lib DIAG=1; UNPAPER_HIP_LIB=unpaper-gpu_amd/lib_diag/libunpaper_hip.so)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "unpaper-gpu_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
os.environ["UPHIP_DIAG_ROTATION"] = "1"

from oracle_py import Oracle  # noqa: E402
from unpaper_hip import ctypes_abi as A  # noqa: E402
from unpaper_hip.device import Backend  # noqa: E402
from unpaper_hip.hostimage import HostImage  # noqa: E402
from unpaper_hip.pipeline import synth_page_host  # noqa: E402

hip, oracle = Backend(), Oracle()
opts = oracle.default_options()
for p in range(4):
    h = HostImage.from_array(synth_page_host(2480, 3508, p), A.FMT_GRAY8)
    n, masks = oracle.detect_masks(h, opts.mask_detection_parameters, [A.Point(1240, 1754)])
    r = hip.detect_rotation(hip.upload(h), masks[0], opts.deskew_parameters)
    print("page", p, "mask", masks[0].tuple(), "rotation", r, flush=True)

# the same count inside the batch pipeline (after the filters and mask scan)
from unpaper_hip.pipeline import Batch  # noqa: E402
b = Batch(opts, 16, 2480, 3508, A.FMT_GRAY8)
for p in range(16):
    b.set_input(p, 0, HostImage.from_array(synth_page_host(2480, 3508, p), A.FMT_GRAY8))
b.run(16)
b.wait()
for p in range(4):
    rep = b.report(p)
    print("batch sheet", p, "mask", rep.masks[0].tuple(), "rotation", rep.rotation[0], flush=True)
b.close()
