"""Host-side logic of the host-resident path that needs no GPU."""
import os
import subprocess

import pytest

from tests.conftest import ROOT

SRC = os.path.join(ROOT, "tests", "cpp", "copypool_stress.cc")
INC = os.path.join(ROOT, "rdc_amd", "csrc")


def _build(tmp_path, extra):
    exe = str(tmp_path / "copypool_stress")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-pthread", "-I", INC] + extra + [SRC, "-o", exe])
    return exe


def test_copypool_back_to_back_runs(tmp_path):
    """rdc_copypool.h: 200k short Run() calls with jobs on the caller's stack;
    every item runs exactly once and no pool thread runs a stale job (the
    host path's pageable <-> pinned copies; a late-waking thread used to
    claim the next call's items with the previous call's destroyed job)."""
    exe = _build(tmp_path, [])
    out = subprocess.run([exe, "200000"], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    assert '"bad": 0' in out.stdout


def test_copypool_under_address_sanitizer(tmp_path):
    """The same under AddressSanitizer (host code only): a stale job pointer is
    a use-after-free of the previous call's freed job."""
    try:
        exe = _build(tmp_path, ["-fsanitize=address", "-fno-omit-frame-pointer", "-g"])
    except subprocess.CalledProcessError:
        pytest.skip("no AddressSanitizer in this toolchain")
    out = subprocess.run([exe, "50000"], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0 and "ERROR: AddressSanitizer" not in out.stderr, out.stderr[-3000:]


def test_parallel_copy_covers_every_byte(tmp_path):
    """rdc_copypool.h ParallelCopy, the host path's pageable <-> pinned copy
    (streaming stores into pinned slots, memcpy out): every byte of sizes
    around the part boundaries arrives and nothing outside the range is
    written.  Cutting a copy by the floor of bytes / parts rounded up to
    4 KiB used to drop the last bytes % parts bytes (e.g. 4 x 256 KiB + 3 B)."""
    src = os.path.join(ROOT, "tests", "cpp", "hostcopy_check.cc")
    exe = str(tmp_path / "hostcopy_check")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-pthread", "-I", INC, src, "-o", exe])
    out = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]
    assert '"bad": 0' in out.stdout
