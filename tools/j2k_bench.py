"""JPEG 2000 decode timing on one GPU: synthetic A4 pages (BASELINE's page
generator) saved by PIL (OpenJPEG) losslessly, decoded with uphip_jp2_decode
(host: headers and packet headers; device: code-blocks, wavelet, colour);
checked against PIL's decode.  usage: python tools/j2k_bench.py [pages] [rgb]"""
import ctypes as C
import io
import os
import sys
import time

import numpy as np
from PIL import Image

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "unpaper-gpu_amd", "python"))
from unpaper_hip import ctypes_abi as A  # noqa: E402
from unpaper_hip.device import load_library  # noqa: E402
from unpaper_hip.pipeline import DeviceBuffer, synth_page_host  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    rgb = len(sys.argv) > 2 and sys.argv[2] == "rgb"
    L = load_library()
    assert L.uphip_try_init() == 0
    W, H = 2480, 3508
    files, refs = [], []
    for i in range(n):
        g = synth_page_host(W, H, 7 + i)
        a = np.stack([g, np.roll(g, 5, 1), np.maximum(g, 30)], 2) if rgb else g
        b = io.BytesIO()
        Image.fromarray(a).save(b, "JPEG2000", **({"mct": 1} if rgb else {}))
        files.append(b.getvalue())
        refs.append(a)
    row = W * (3 if rgb else 1)
    pitch = (row + 255) // 256 * 256
    d = DeviceBuffer(pitch * H)
    info = A.PnmInfo()
    host = np.zeros((H, pitch), np.uint8)
    # warm-up + check
    assert L.uphip_jp2_decode(files[0], len(files[0]), d.ptr, pitch, C.byref(info)) == 0, L.uphip_last_error()
    assert L.uphip_memcpy_dtoh(host.ctypes.data, d.ptr, pitch * H) == 0
    check = not os.environ.get("J2K_NOCHECK")  # timing-only variants of the tuning build
    assert not check or (host[:, :row].reshape(refs[0].shape) == refs[0]).all(), "decode differs"
    t = time.perf_counter()
    for f in files:
        assert L.uphip_jp2_decode(f, len(f), d.ptr, pitch, C.byref(info)) == 0
    dt = (time.perf_counter() - t) / n
    coef = np.zeros(W * H * (3 if rgb else 1), np.uint32)
    t = time.perf_counter()
    L.uphip_jp2_entropy_decode(files[0], len(files[0]), coef.ctypes.data, coef.nbytes, C.byref(info))
    dh = time.perf_counter() - t
    print("jp2 %s A4 lossless: file %.2f MB, uphip_jp2_decode %.1f ms/page (host headers + device "
          "code-blocks/wavelet), host code-block decode %.0f ms/page" %
          ("RGB" if rgb else "gray", sum(len(f) for f in files) / n / 1e6, dt * 1e3, dh * 1e3), flush=True)
    # encode: the decoded page back to a lossless file (device transforms and
    # code-blocks, host packets); the file must equal PIL's packets
    from unpaper_hip.pipeline import jp2_encode
    fmt = A.FMT_RGB24 if rgb else A.FMT_GRAY8
    f0 = jp2_encode(d.ptr, pitch, W, H, fmt)
    back = np.asarray(Image.open(io.BytesIO(f0)))
    assert not check or (back == refs[-1]).all(), "encode does not round-trip"
    body = lambda f: f[f.index(b"\xff\x93") + 2:]
    same = body(f0) == body(files[-1])
    t = time.perf_counter()
    for _ in range(n):
        jp2_encode(d.ptr, pitch, W, H, fmt)
    de = (time.perf_counter() - t) / n
    print("jp2 encode %.1f ms/page (%.2f MB), packets %s OpenJPEG's" %
          (de * 1e3, len(f0) / 1e6, "equal to" if same else "DIFFERENT from"), flush=True)
    d.close()


if __name__ == "__main__":
    main()
