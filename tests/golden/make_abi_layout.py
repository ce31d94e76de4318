#!/usr/bin/env python3
"""Generate tests/golden/abi_layout.json: sizeof / offsetof of every field of
the reference's value types, measured by compiling a C probe against the
reference headers themselves (imageprocess/{primitives,image,filters,masks,
deskew,interpolate}.h, constants.h — they need no FFmpeg headers).

TEST INFRASTRUCTURE: runs in the build container, where /root/reference
exists; the probe source is generated here and compiled into a temporary
directory, nothing of the reference is copied.  tests/test_abi.py checks the
library's uphip_abi_sizeof / uphip_abi_offsetof against the committed JSON.

usage: python3 tests/golden/make_abi_layout.py [--reference /root/reference]
"""
import argparse
import json
import os
import subprocess
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))

# reference type -> (HIP peer type, fields).  BlackfilterParameters holds an
# exclusions POINTER in the reference (filters.h:27-28) and an inline array in
# the peer (the batch carries it to the device by value); only the fields
# before it are layout-shared.
TYPES = {
    "Point": ("UphipPoint", ["x", "y"]),
    "Delta": ("UphipDelta", ["horizontal", "vertical"]),
    "Direction": ("UphipDirection", ["horizontal", "vertical"]),
    "Edges": ("UphipEdges", ["left", "top", "right", "bottom"]),
    "Pixel": ("UphipPixel", ["r", "g", "b"]),
    "Rectangle": ("UphipRectangle", ["vertex[0].x", "vertex[0].y", "vertex[1].x",
                                     "vertex[1].y"]),
    "RectangleSize": ("UphipRectangleSize", ["width", "height"]),
    "Image": ("UphipImage", ["frame", "background", "abs_black_threshold"]),
    "Border": ("UphipBorder", ["left", "top", "right", "bottom"]),
    "Wipes": ("UphipWipes", ["count", "areas", "areas[99]"]),
    "BlurfilterParameters": ("UphipBlurfilterParameters",
                             ["scan_size", "scan_step", "intensity"]),
    "GrayfilterParameters": ("UphipGrayfilterParameters",
                             ["scan_size", "scan_step", "abs_threshold"]),
    "BlackfilterParameters": ("UphipBlackfilterParameters",
                              ["scan_size", "scan_step", "scan_depth.horizontal",
                               "scan_depth.vertical", "scan_direction", "abs_threshold",
                               "intensity", "exclusions_count", "exclusions"]),
    "MaskDetectionParameters": ("UphipMaskDetectionParameters",
                                ["scan_size", "scan_step", "scan_depth.horizontal",
                                 "scan_depth.vertical", "scan_direction",
                                 "scan_threshold.horizontal", "scan_threshold.vertical",
                                 "minimum_width", "maximum_width", "minimum_height",
                                 "maximum_height"]),
    "MaskAlignmentParameters": ("UphipMaskAlignmentParameters", ["alignment", "margin"]),
    "BorderScanParameters": ("UphipBorderScanParameters",
                             ["scan_size", "scan_step", "scan_threshold.horizontal",
                              "scan_threshold.vertical", "scan_direction"]),
    "DeskewParameters": ("UphipDeskewParameters",
                         ["deskewScanRangeRad", "deskewScanStepRad", "deskewScanDeviationRad",
                          "deskewScanSize", "deskewScanDepth", "scan_edges"]),
}
ENUMS = {"Interpolation": "UphipInterpolation", "Layout": "UphipLayout"}
HEADERS = ["imageprocess/primitives.h", "imageprocess/image.h", "imageprocess/filters.h",
           "imageprocess/masks.h", "imageprocess/deskew.h", "imageprocess/interpolate.h",
           "constants.h"]


def probe_source():
    lines = ["#include <stddef.h>", "#include <stdio.h>"]
    lines += ['#include "%s"' % h for h in HEADERS]
    lines += ["int main(void) {", '  printf("{\\n");']
    items = []
    for t, (_, fields) in TYPES.items():
        items.append('  printf("\\"%s\\": {\\"sizeof\\": %%zu", sizeof(%s));' % (t, t))
        for f in fields:
            items.append('  printf(", \\"%s\\": %%zu", offsetof(%s, %s));' % (f, t, f))
        items.append('  printf("},\\n");')
    for e in ENUMS:
        items.append('  printf("\\"%s\\": {\\"sizeof\\": %%zu},\\n", sizeof(%s));' % (e, e))
    items.append('  printf("\\"MAX_MASKS\\": {\\"value\\": %d},\\n", (int)MAX_MASKS);')
    items.append('  printf("\\"MAX_POINTS\\": {\\"value\\": %d}\\n", (int)MAX_POINTS);')
    lines += items + ['  printf("}\\n");', "  return 0;", "}"]
    return "\n".join(lines) + "\n"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    args = ap.parse_args()
    with tempfile.TemporaryDirectory() as d:
        src = os.path.join(d, "probe.c")
        exe = os.path.join(d, "probe")
        with open(src, "w") as f:
            f.write(probe_source())
        subprocess.check_call(["gcc", "-std=gnu11", "-I", args.reference, src, "-o", exe])
        layout = json.loads(subprocess.check_output([exe]).decode())
    doc = {"generator": "tests/golden/make_abi_layout.py (gcc, x86-64, reference headers: %s)"
                        % ", ".join(HEADERS),
           "peers": {t: p for t, (p, _) in TYPES.items()},
           "enum_peers": ENUMS,
           "layout": layout}
    with open(os.path.join(HERE, "abi_layout.json"), "w") as f:
        json.dump(doc, f, indent=1)
        f.write("\n")
    print("wrote %d types" % len(layout))


if __name__ == "__main__":
    main()
