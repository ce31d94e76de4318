"""Copy the reference's own test data into tests/golden/reference/.

Run once in the build container (where /root/reference exists); the result is
committed because the GPU box has no /root/reference.  Source images are copied
byte for byte; the PBM/PPM goldens are re-encoded losslessly as PNG (same
pixels, ~10x smaller).  Provenance: ErrorTzy/unpaper-gpu tests/source_images/
and tests/golden_images/ (GPL-2.0, see the .license files there).
"""
import os
import shutil
import sys

from PIL import Image

REF = "/root/reference/tests"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "reference")

SOURCES = ["imgsrc001.png", "imgsrc002.png", "imgsrc003.png", "imgsrc004.png",
           "imgsrc005.png", "imgsrc006.png", "imgsrcE001.png", "imgsrcE002.png",
           "imgsrcE003.png"]
GOLDENS = ["goldenA1.pbm", "goldenC1.pbm", "goldenC2.pbm", "goldenC1.ppm",
           "goldenE1-01.pbm", "goldenE1-02.pbm", "goldenE1-03.pbm",
           "goldenE1-04.pbm", "goldenE1-05.pbm", "goldenE1-06.pbm", "goldenF.pbm"]


def main():
    if not os.path.isdir(REF):
        sys.exit("reference tree not present")
    os.makedirs(OUT, exist_ok=True)
    for s in SOURCES:
        shutil.copyfile(os.path.join(REF, "source_images", s), os.path.join(OUT, s))
    for g in GOLDENS:
        im = Image.open(os.path.join(REF, "golden_images", g))
        im.load()
        stem, ext = os.path.splitext(g)
        im.save(os.path.join(OUT, stem + ext.replace(".", "_") + ".png"), optimize=True)


if __name__ == "__main__":
    main()
