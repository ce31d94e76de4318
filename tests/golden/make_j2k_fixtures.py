"""Small JPEG 2000 fixtures: files written by PIL's OpenJPEG encoder (the
decoder nvImageCodec's JPEG2000 path is pinned against here, nvImageCodec
itself being absent) covering the codestream features the decoder takes, with
OpenJPEG's decode of each (PIL) as the expected pixels (<name>.npy).  Used by
tests/test_j2k.py and the host decoder's sanitizer run (tests/c/sanitize_main.c).
Run from the repository root: python tests/golden/make_j2k_fixtures.py"""
import os

import numpy as np
from PIL import Image

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "j2k")

# name -> (rgb?, PIL save options)
CASES = {
    "gray.jp2": (False, {}),
    "rgb_mct.jp2": (True, {"mct": 1}),
    "rgb_nomct.jp2": (True, {"mct": 0, "num_resolutions": 3}),
    "tiled_rpcl.j2k": (False, {"tile_size": (32, 32), "progression": "RPCL",
                               "precinct_size": (16, 16), "codeblock_size": (16, 16),
                               "no_jp2": True}),
    "offset_tiles.jp2": (True, {"offset": (5, 3), "tile_offset": (2, 1), "tile_size": (40, 40),
                                "mct": 1}),
    "lossy_layers.jp2": (False, {"irreversible": True, "quality_mode": "rates",
                                 "quality_layers": [40, 10, 2], "progression": "CPRL"}),
    "lossy_rgb.jp2": (True, {"irreversible": True, "mct": 1, "progression": "PCRL"}),
    "plt.jp2": (False, {"plt": True, "progression": "RLCP", "codeblock_size": (32, 16)}),
}


def content(w, h, seed):
    rng = np.random.default_rng(seed)
    g = np.full((h, w), 255, np.uint8)
    g[h // 4:3 * h // 4, w // 5:4 * w // 5] = rng.integers(0, 256, (3 * h // 4 - h // 4,
                                                                  4 * w // 5 - w // 5))
    y, x = np.mgrid[0:h, 0:w]
    g[: h // 4] = ((x + 2 * y) * 3 % 256)[: h // 4]
    return g


def main():
    os.makedirs(OUT, exist_ok=True)
    g = content(77, 61, 3)
    rgb = np.stack([g, np.roll(g, 5, 1), 255 - g], 2)
    for name, (colour, kw) in CASES.items():
        path = os.path.join(OUT, name)
        Image.fromarray(rgb if colour else g).save(path, "JPEG2000", **kw)
        np.save(os.path.join(OUT, name.rsplit(".", 1)[0] + ".npy"), np.asarray(Image.open(path)))


if __name__ == "__main__":
    main()
