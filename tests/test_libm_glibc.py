"""The device's restatement of glibc sinf/cosf/powf(x, 2) (csrc/libm_glibc.h),
used by the batch path's rotation select for more than two deskew edges
(deskew.c:219-240 and :260-261), against this host's glibc bit for bit.

CPU: the same header compiled for the host (tests/c/libm_check.cpp) over
every 61st float of the checked ranges.  The exhaustive run (`libm_check
full`, every float: 0 mismatches) is recorded in profiles/r04/libm_check_full.txt.
GPU: the device evaluation (uphip_check_libm) over the same strided inputs."""
import ctypes as C
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHECK = os.path.join(ROOT, "tests", "c", "_build", "libm_check")


def test_host_restatement_matches_glibc():
    subprocess.check_call(["make", "-s", "libm_check"], cwd=ROOT)
    r = subprocess.run([CHECK, "stride", "61"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    lines = dict(l.split(":", 1) for l in r.stdout.strip().splitlines())
    for fn in ("sinf", "cosf", "powf2"):
        assert lines[fn].strip().endswith(" 0 mismatches"), r.stdout


@pytest.mark.gpu
def test_device_matches_glibc(hip):
    L = hip.lib
    counts = (C.c_uint64 * 4)()
    assert L.uphip_check_libm(61, counts) == 0
    assert counts[3] > 60_000_000
    assert (counts[0], counts[1], counts[2]) == (0, 0, 0), list(counts)
