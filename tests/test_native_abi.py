"""The C-ABI library (libfmt.so) loads and exports every entry point include/fmt.h declares (CPU).

No compute call is made without a GPU; fmt_open must fail cleanly (FMT_E_DEVICE), never crash.
"""
import ctypes
import os
import re
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "fmt.h")


def _declared_functions():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"^(?:int|void|const char\*)\s+(fmt_\w+)\(", text, re.M)))


@pytest.fixture(scope="module")
def libfmt():
    from fluidframework_amd import native

    if not os.path.exists(native.LIB_PATH):
        subprocess.run(["make", "-s", "-C", os.path.join(REPO, "fluidframework_amd", "csrc")], check=True)
    return native


def test_header_declares_the_boundary():
    fns = _declared_functions()
    assert "fmt_mt_run" in fns and "fmt_map_run" in fns and len(fns) >= 15


def test_library_exports_every_declared_symbol(libfmt):
    lib = ctypes.CDLL(libfmt.LIB_PATH)
    missing = [f for f in _declared_functions() if not hasattr(lib, f)]
    assert not missing, missing
    assert sorted(libfmt.EXPORTED_SYMBOLS) == _declared_functions()


def test_library_is_built_for_gfx950_only(libfmt):
    data = open(libfmt.LIB_PATH, "rb").read()
    targets = set(re.findall(rb"hipv4-amdgcn-amd-amdhsa--(gfx[0-9a-z]+)", data))
    assert targets == {b"gfx950"}, targets


def test_capacity_query_without_device(libfmt):
    leaves, chars, props = libfmt.capacity()
    assert leaves >= 512 and chars >= 2048 and props >= 32


@pytest.mark.skipif(os.path.exists("/dev/kfd") and os.access("/dev/kfd", os.R_OK), reason="a GPU is present")
def test_open_without_gpu_fails_loudly(libfmt):
    with pytest.raises(libfmt.EngineUnavailable):
        libfmt.Engine(0)
