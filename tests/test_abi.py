"""The C-ABI library loads (no GPU needed) and exports exactly the symbols include/nrse_hip.h
declares; the ctypes table covers every declaration; the ABI 10 struct_size handshake refuses a
params struct of another layout before reading it (no GPU call is reached)."""
import ctypes
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
    version = int(re.search(r"#define NRSE_ABI_VERSION (\d+)", open(HEADER).read()).group(1))
    assert L.nrse_abi_version() == version == lib.ABI_VERSION == 11


def test_retired_mxfp6_forms_are_gone(lib):
    """ABI 11 retired ABI 8-10's MXFP6 correction planes (slower than fp8 at the same accuracy,
    profiles/r05_mx6_ab.txt): neither the dtype nor its producers remain."""
    text = open(HEADER).read()
    assert "NRSE_MX6 =" not in text and not hasattr(lib, "MX6")
    out = subprocess.run(["nm", "-D", "--defined-only", lib.LIB_PATH], capture_output=True, text=True, check=True)
    assert "mx6" not in out.stdout


def test_nm_dynamic_symbols(lib):
    out = subprocess.run(["nm", "-D", "--defined-only", lib.LIB_PATH], capture_output=True, text=True, check=True)
    exported = set(re.findall(r"\b(nrse_\w+)\b", out.stdout))
    assert set(declared()) <= exported


PARAMS = {  # ctypes struct -> (entry point, workspace query or None)
    "GemmParams": ("nrse_gemm", "nrse_gemm_colsum_workspace"),
    "LnFwdParams": ("nrse_layernorm_fwd", None),
    "LnBwdParams": ("nrse_layernorm_bwd", "nrse_layernorm_bwd_workspace"),
    "AttnFwdParams": ("nrse_attn_fwd", None),
    "AttnBwdParams": ("nrse_attn_bwd", "nrse_attn_bwd_workspace"),
    "Conv0Params": ("nrse_conv0_fwd", "nrse_conv0_bwd_workspace"),
    "AdamWParams": ("nrse_adamw", None),
}


def test_params_structs_lead_with_their_size(lib):
    """Every params struct the header declares starts with uint32_t struct_size, and the binding
    stamps it with its own sizeof."""
    text = open(HEADER).read()
    for cname in ("nrse_gemm_params", "nrse_ln_fwd_params", "nrse_ln_bwd_params", "nrse_attn_fwd_params",
                  "nrse_attn_bwd_params", "nrse_conv0_params", "nrse_adamw_params"):
        body = text[:text.index("} " + cname + ";")]
        body = body[body.rindex("typedef struct {"):]
        first = re.sub(r"/\*.*?\*/", "", body, flags=re.S).split("{", 1)[1].strip().split(";")[0]
        assert first == "uint32_t struct_size", (cname, first)
    for cls in PARAMS:
        p = getattr(lib, cls)()
        assert p.struct_size == ctypes.sizeof(type(p)) and type(p)._fields_[0][0] == "struct_size"


@pytest.mark.parametrize("cls", sorted(PARAMS))
@pytest.mark.parametrize("delta", [-8, 8, None])
def test_mismatched_struct_is_refused(lib, cls, delta):
    """A caller built against another header passes a shorter (older ABI) or longer struct, or an
    older one whose first field is a pointer: refused with NRSE_ERR_ARG (-1) and a message naming
    struct_size, before any other field is read -- here every other field is garbage."""
    L = lib.lib()
    T = getattr(lib, cls)
    buf = (ctypes.c_ubyte * (ctypes.sizeof(T) + 64))(*([0xA5] * (ctypes.sizeof(T) + 64)))
    p = T.from_buffer(buf)
    if delta is None:
        p.struct_size = 0x5A5A0000   # the low half of a pointer in the old layout's first slot
    else:
        p.struct_size = ctypes.sizeof(T) + delta
    entry, ws = PARAMS[cls]
    fn = getattr(L, entry)
    rc = fn(ctypes.byref(p), None) if entry != "nrse_conv0_bwd_workspace" else fn(ctypes.byref(p))
    assert rc == -1, (entry, rc)
    assert "struct_size" in L.nrse_last_error().decode(), L.nrse_last_error()
    if ws is not None:
        assert getattr(L, ws)(ctypes.byref(p)) == -1, ws
