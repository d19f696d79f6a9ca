"""The C-ABI libraries load and export every symbol their headers declare (no GPU calls)."""
from __future__ import annotations

import ctypes as C
import re

import pytest

from cuda_raytracing_amd import _abi
from conftest import REPO


def declared(header: str) -> list[str]:
    text = (REPO / "include" / header).read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    names = re.findall(r"\b(rt_[a-z0-9_]+)\s*\(", text)
    return sorted(set(names))


def test_render_header_symbols():
    lib = C.CDLL(str(_abi.HIP_LIB))
    names = [n for n in declared("rt_render.h") if n != "rt_render_cpu"]
    assert "rt_render" in names and "rt_context_render" in names
    for n in names:
        assert hasattr(lib, n), n
    assert lib.rt_abi_version() == 6


def test_host_header_symbols():
    lib = C.CDLL(str(_abi.HOST_LIB))
    for n in declared("rt_host.h"):
        assert hasattr(lib, n), n


def test_oracle_symbol():
    lib = C.CDLL(str(_abi.ORACLE_LIB))
    assert hasattr(lib, "rt_render_cpu")


def test_struct_layouts():
    # the ctypes mirrors match the compiled C structs
    L = _abi.host_lib()
    L.rt_abi_struct_sizes.restype = C.c_int
    out = (C.c_uint32 * 8)()
    assert L.rt_abi_struct_sizes(out, 8) == 8
    mirrors = [_abi.Scene, _abi.Camera, _abi.Params, _abi.Stats, _abi.Settings]
    assert [C.sizeof(m) for m in mirrors] == list(out)[:5]
    assert list(out)[5:] == [120, 24, 32]


def test_status_strings():
    lib = _abi.hip_lib()
    assert lib.rt_status_string(0) == b"ok"
    assert lib.rt_status_string(-2) == b"malformed scene"


def test_product_path_never_loads_oracle():
    # the render entry points live in librt_hip.so: no product source may call or load the oracle
    srcs = [REPO / "cuda_raytracing_amd" / "__init__.py"]
    srcs += [f for f in (REPO / "cuda_raytracing_amd" / "csrc").rglob("*") if f.is_file()]
    for f in srcs:
        t = f.read_text()
        assert "rt_render_cpu" not in t and "liboracle" not in t and "oracle_lib" not in t, f


def test_build_stamp_refuses_a_stale_library(tmp_path, monkeypatch):
    # the libraries record the sources they were built from; a tree whose sources differ is refused loudly
    lib = C.CDLL(str(_abi.HIP_LIB))
    _abi.check_build_stamp(lib, "rt_hip", _abi.HIP_LIB)        # this tree: accepted
    lib.rt_hip_build_files.restype = C.c_char_p
    files = lib.rt_hip_build_files().decode().split()
    assert "cuda_raytracing_amd/csrc/device/rt_body.h" in files and "cuda_raytracing_amd/csrc/rt_capi.cpp" in files
    for name in files:
        dst = tmp_path / name
        dst.parent.mkdir(parents=True, exist_ok=True)
        dst.write_bytes((REPO / name).read_bytes())
    (tmp_path / "cuda_raytracing_amd/csrc/device/rt_body.h").write_bytes(
        (REPO / "cuda_raytracing_amd/csrc/device/rt_body.h").read_bytes() + b"// edited after the build\n")
    monkeypatch.setattr(_abi, "REPO_DIR", tmp_path)
    with pytest.raises(RuntimeError, match="stale library"):
        _abi.check_build_stamp(lib, "rt_hip", _abi.HIP_LIB)
