"""A plain C caller of the vtable (tests/c/backend_ops.c): the 20 ops through
uphip_backend() — what the reference's C stages do after
image_backend_select() — each compared with the oracle in all five formats."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "c", "_build", "backend_ops")
ADAPTER = os.path.join(ROOT, "tests", "c", "_build", "adapter_ops")
REFERENCE_HEADERS = "/root/reference/imageprocess/image.h"


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


def _adapter():
    """integration/backend_hip.c compiled against the reference's own headers
    (make adapter); prebuilt here, where the reference tree is, and carried to
    the GPU box with the tree."""
    if os.path.isfile(REFERENCE_HEADERS):
        subprocess.check_call(["make", "-s", "adapter"], cwd=ROOT)
    if not os.path.exists(ADAPTER):
        pytest.fail("tests/c/_build/adapter_ops is not built (run build() where the reference is)")
    return ADAPTER


def test_adapter_compiles_against_reference_headers():
    """CPU: the adapter builds on the reference's Image and value types (the
    layout static asserts hold) and, with no device, fails loudly (exit 2)."""
    import torch
    if not os.path.isfile(REFERENCE_HEADERS):
        pytest.skip("no reference tree here")
    exe = _adapter()
    if torch.cuda.is_available():
        return
    p = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    assert p.returncode == 2 and "no HIP device" in p.stderr


@pytest.mark.gpu
def test_adapter_all_ops_on_reference_types_match_oracle():
    exe = _adapter()
    p = subprocess.run([exe], capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:] + p.stdout[-1000:]
    assert "0 mismatches" in p.stdout and "x 5 formats" in p.stdout
