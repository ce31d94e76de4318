"""Debug: batch JPEG encode of a q100 noise page (expected to overflow the batch buffer)."""
import io, sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "unpaper-gpu_amd", "python"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "oracle"))
import numpy as np
from PIL import Image
import ctypes as C
from unpaper_hip import ctypes_abi as A
from unpaper_hip.pipeline import Batch, jpeg_encode
from unpaper_hip.hostimage import HostImage
from unpaper_hip.device import load_library
L = load_library()
o = A.Options(); L.uphip_options_init(C.byref(o)); o.disable = A.NO_PROCESSING
for (w, h) in ((640, 480), (200, 160)):
    rng = np.random.default_rng(5)
    noise = rng.integers(0, 256, (h, w)).astype(np.uint8)
    b = Batch(o, 2, w, h, A.FMT_GRAY8)
    b.set_input(0, 0, HostImage.from_array(noise, A.FMT_GRAY8))
    b.set_input(1, 0, HostImage.from_array(noise, A.FMT_GRAY8))
    b.run(2); b.encode_jpeg(100, 0); b.wait()
    sizes = (C.c_int64 * 2)()
    tot = L.uphip_batch_jpeg_sizes(b.handle, sizes, 2)
    pil = io.BytesIO(); Image.fromarray(noise).save(pil, "JPEG", quality=100)
    src = b.jpeg_page(0)
    single = jpeg_encode(*src, 100, 0)
    print(w, h, "sizes", list(sizes), "total", tot, "pil", len(pil.getvalue()), "single", len(single),
          "single==pil", single == pil.getvalue(), flush=True)
    files = b.jpeg_files(2)
    print("  batch files", [None if f is None else len(f) for f in files],
          [None if f is None else f == pil.getvalue() for f in files], flush=True)
    b.close()
# the sheets themselves
for (w, h) in ((640, 480), (200, 160)):
    rng = np.random.default_rng(5)
    noise = rng.integers(0, 256, (h, w)).astype(np.uint8)
    b = Batch(o, 2, w, h, A.FMT_GRAY8)
    b.set_input(0, 0, HostImage.from_array(noise, A.FMT_GRAY8))
    b.set_input(1, 0, HostImage.from_array(noise, A.FMT_GRAY8))
    b.run(2); b.wait()
    for s in range(2):
        out = b.output(s)
        g = out.data[:, :w]
        print(w, h, "sheet", s, "equal", np.array_equal(g, noise), "mean", g.mean(), "diff px",
              int(np.count_nonzero(g != noise)), flush=True)
    r = b.report(0)
    print("  report", r.mask_count, r.width, r.height, r.flags, flush=True)
    b.close()
