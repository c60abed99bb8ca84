"""The C-ABI library loads (no GPU needed) and exports exactly the symbols include/nrse_hip.h
declares; the ctypes table covers every declaration."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "nrse_hip.h")
PKG = os.path.join(ROOT, "noise-robust-speech-embedding_amd")


def declared():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?(?:\w+\s+)*\w+\*?\s+\*?(nrse_\w+)\s*\(", text, flags=re.M)))


@pytest.fixture(scope="module")
def lib():
    from nrse_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        subprocess.run(["make", "-j8"], cwd=os.path.join(PKG, "csrc"), check=True)
    return _lib


def test_header_declares_the_ctypes_table(lib):
    names = declared()
    assert len(names) >= 30, names
    assert names == lib.exported_symbols(), set(names) ^ set(lib.exported_symbols())


def test_library_exports_every_declared_symbol(lib):
    L = lib.lib()
    for name in declared():
        assert hasattr(L, name), name
    assert L.nrse_abi_version() == 9


def test_nm_dynamic_symbols(lib):
    out = subprocess.run(["nm", "-D", "--defined-only", lib.LIB_PATH], capture_output=True, text=True, check=True)
    exported = set(re.findall(r"\b(nrse_\w+)\b", out.stdout))
    assert set(declared()) <= exported
