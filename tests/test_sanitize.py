"""Host code under AddressSanitizer + UBSan: the oracle's full
sheet pipeline in every input format and layout, and the product library's
PNM codec on good and malformed files (tests/c/sanitize_main.c, `make
sanitize`).  CPU only."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_host_code_is_sanitizer_clean():
    p = subprocess.run(["make", "-s", "sanitize"], cwd=ROOT, capture_output=True, text=True,
                       timeout=600)
    out = p.stdout + p.stderr
    assert p.returncode == 0, out[-4000:]
    assert "sanitize: 0 failures" in out
    assert "AddressSanitizer" not in out and "runtime error" not in out
