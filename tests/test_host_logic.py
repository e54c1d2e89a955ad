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
