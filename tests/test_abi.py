"""CPU-only checks of the drop-in boundary: the C-ABI library builds for
gfx950, loads, and exports every symbol include/pardis.h declares.  No
compute call is made here (no GPU in this container)."""
import ctypes
import os
import re

import pytest

from conftest import REPO

HEADER = os.path.join(REPO, "include", "pardis.h")


def declared_symbols():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"^\w[\w\s\*]*?\b(pd_\w+)\s*\(", txt, re.M)))


@pytest.fixture(scope="module")
def lib():
    from pypardis_amd import build
    path = build.build(verbose=False)
    return ctypes.CDLL(path)


def test_header_declares_entry_points():
    syms = declared_symbols()
    for s in ["pd_cluster", "pd_train", "pd_kd_moments", "pd_kd_counts", "pd_kd_split",
              "pd_bbox", "pd_halo_members", "pd_ctx_create", "pd_last_error"]:
        assert s in syms


def test_library_exports_every_declared_symbol(lib):
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing


def test_python_binding_covers_header():
    from pypardis_amd import _native
    assert sorted(_native.EXPORTS) == declared_symbols()


def test_abi_version_and_error_string(lib):
    lib.pd_abi_version.restype = ctypes.c_int32
    lib.pd_last_error.restype = ctypes.c_char_p
    assert lib.pd_abi_version() == 3
    assert isinstance(lib.pd_last_error(), bytes)


def test_kernels_are_gfx950_code_objects(lib, tmp_path):
    """The fat binary carries exactly one device target: gfx950."""
    import subprocess
    so = os.path.join(REPO, "pypardis_amd", "libpardis.so")
    out = tmp_path / "fat.bin"
    subprocess.check_call(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", so, str(out)])
    triples = set(re.findall(rb"hipv4-amdgcn-amd-amdhsa--(gfx\w+)", out.read_bytes()))
    assert triples == {b"gfx950"}


def test_product_never_imports_oracle():
    pkg = os.path.join(REPO, "pypardis_amd")
    for root, _, files in os.walk(pkg):
        for f in files:
            if f.endswith(".py"):
                src = open(os.path.join(root, f)).read()
                assert not re.search(r"^\s*(import|from)\s+oracle\b", src, re.M), f
                if f != "synth.py":   # synth imports sklearn only for the C0 demo data
                    assert not re.search(r"^\s*(import|from)\s+sklearn\b", src, re.M), f
