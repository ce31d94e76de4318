"""A plain C caller of the vtable (tests/c/backend_ops.c): the 20 ops through
uphip_backend() — what the reference's C stages do after
image_backend_select() — each compared with the oracle in all five formats."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "c", "_build", "backend_ops")


def _ensure_built():
    if not os.path.exists(EXE):
        subprocess.check_call(["make", "-s", "ctest"], cwd=ROOT)


def test_c_caller_links_and_reports_missing_device():
    """CPU: the program links against libunpaper_hip.so + the oracle and, with
    no HIP device, fails loudly (exit 2) instead of falling back."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present (see the gpu test)")
    _ensure_built()
    p = subprocess.run([EXE], capture_output=True, text=True, timeout=60)
    assert p.returncode == 2 and "no HIP device" in p.stderr


@pytest.mark.gpu
def test_c_caller_all_ops_match_oracle():
    _ensure_built()
    p = subprocess.run([EXE], capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:] + p.stdout[-1000:]
    assert "0 mismatches" in p.stdout and "20 ops x 5 formats" in p.stdout
