"""Register and scratch budgets of the built gfx950 kernels (CPU test: reads the
code objects inside rdc_amd/librdc_amd.so, no GPU).

Round 4 found two silent regressions only a profile would have shown:
k_mesh copied its 1.2 KiB argument block into per-lane scratch (1180 B/lane,
`mesh_body` not inlined) and the int8 / uint8 folds took 256 VGPRs (one wave
per SIMD).  Every collective kernel must stay free of scratch and below 256
VGPRs, so that a waiting launch's grid clamp (rdc_plan.cpp ResidentGrid) and
its occupancy stay what the planner assumes.  (The opt-in host-exchange
service variant spilled its polling arrays until it polled four ranks at a
time.)
"""
import os
import re
import shutil
import struct
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "rdc_amd", "librdc_amd.so")
READELF = shutil.which("llvm-readelf") or "/opt/rocm/lib/llvm/bin/llvm-readelf"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def kernel_metadata(path):
    """{kernel symbol: (private_segment_fixed_size, vgpr_count)} over every
    gfx950 code object of every offload bundle in the library."""
    data = open(path, "rb").read()
    out = {}
    pos = 0
    while True:
        i = data.find(MAGIC, pos)
        if i < 0:
            break
        (n,) = struct.unpack_from("<Q", data, i + 24)
        off = i + 32
        for _ in range(n):
            eo, es, ts = struct.unpack_from("<QQQ", data, off)
            triple = data[off + 24: off + 24 + ts].decode()
            off += 24 + ts
            if "gfx950" not in triple or es == 0:
                continue
            with tempfile.NamedTemporaryFile(suffix=".co", delete=False) as f:
                f.write(data[i + eo: i + eo + es])
                co = f.name
            try:
                notes = subprocess.run([READELF, "--notes", co], capture_output=True, text=True, timeout=60).stdout
            finally:
                os.unlink(co)
            for blk in notes.split("  - .agpr_count")[1:]:
                name = re.search(r"\.name:\s+(\S+)", blk).group(1)
                priv = int(re.search(r"\.private_segment_fixed_size:\s+(\d+)", blk).group(1))
                vgpr = int(re.search(r"\.vgpr_count:\s+(\d+)", blk).group(1))
                out[name] = (priv, vgpr)
        pos = i + len(MAGIC)
    return out


@pytest.fixture(scope="module")
def kernels():
    if not os.path.exists(LIB):
        pytest.skip("librdc_amd.so not built")
    if not os.path.exists(READELF):
        pytest.skip("llvm-readelf not available")
    k = kernel_metadata(LIB)
    assert k, "no gfx950 kernels found in " + LIB
    return k


def test_every_kernel_family_is_present(kernels):
    names = " ".join(kernels)
    for fam in ("k_reduce", "k_mesh", "k_ring", "k_oneshot", "k_tree", "k_svc", "k_bcast", "k_allgather",
                "k_copy", "k_push", "k_pack", "k_fill"):
        assert fam in names, fam


def test_no_kernel_uses_scratch(kernels):
    bad = {k: v for k, v in kernels.items() if v[0] != 0}
    assert not bad, bad


def test_collective_kernels_keep_two_waves_per_simd(kernels):
    """k_mesh / k_ring / k_oneshot / k_tree below 256 VGPRs (256 = one wave per
    SIMD with 256-thread blocks)."""
    coll = {k: v for k, v in kernels.items() if re.search(r"k_(mesh|ring|oneshot|tree)I", k)}
    assert len(coll) >= 4 * 10, len(coll)  # 4 ops x 10 element types, several widths each
    bad = {k: v for k, v in coll.items() if v[1] >= 256}
    assert not bad, bad
