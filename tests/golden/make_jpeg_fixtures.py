"""Small JPEG fixtures for the host decoder's sanitizer run (tests/c/sanitize_main.c):
PIL-encoded files of the kinds the decoder takes (gray, 4:2:0 with restart
markers, 4:4:4 with optimised tables, progressive).
Run from the repository root: python tests/golden/make_jpeg_fixtures.py"""
import os

import numpy as np
from PIL import Image

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "jpeg")


def content(w, h, seed):
    rng = np.random.default_rng(seed)
    g = np.full((h, w), 255, np.uint8)
    g[h // 4:3 * h // 4, w // 5:4 * w // 5] = rng.integers(0, 256, (3 * h // 4 - h // 4,
                                                                  4 * w // 5 - w // 5))
    return g


def main():
    os.makedirs(OUT, exist_ok=True)
    g = content(96, 72, 1)
    rgb = np.stack([g, np.roll(g, 5, 1), 255 - g], 2)
    Image.fromarray(g).save(os.path.join(OUT, "gray.jpg"), "JPEG", quality=90)
    Image.fromarray(rgb).save(os.path.join(OUT, "rgb420_rst.jpg"), "JPEG", quality=85,
                              subsampling=2, restart_marker_blocks=2)
    Image.fromarray(rgb).save(os.path.join(OUT, "rgb444_opt.jpg"), "JPEG", quality=95,
                              subsampling=0, optimize=True)
    Image.fromarray(rgb).save(os.path.join(OUT, "progressive.jpg"), "JPEG", quality=80,
                              progressive=True)


if __name__ == "__main__":
    main()
