"""CPU: the C-ABI libraries load and export every symbol their headers declare; struct layouts and
defaults agree between the headers, the ctypes mirror and the library.  No compute call is made."""
import ctypes as C
import os
import re

import dxrpathtracer_amd._abi as A

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared(header):
    txt = open(os.path.join(REPO, "include", header)).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(dxrpt_\w+)\s*\(", txt)))


def test_libdxrpt_exports_every_declared_function():
    L = A.lib()
    names = _declared("dxrpt.h")
    assert "dxrpt_render" in names and "dxrpt_build_bvh" in names
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing
    assert set(names) == set(A.DXRPT_SYMBOLS)


def test_libdxrpt_host_exports_every_declared_function():
    H = A.host()
    names = _declared("dxrpt_host.h")
    missing = [n for n in names if not hasattr(H, n)]
    assert not missing, missing
    assert set(names) == set(A.DXRPT_HOST_SYMBOLS)


def test_abi_version_and_defaults():
    L = A.lib()
    assert L.dxrpt_abi_version() == 2
    s = A.AppSettings()
    L.dxrpt_default_settings(C.byref(s))
    py = A.default_settings()
    assert bytes(s) == bytes(py)
    # AppSettings.cpp:95-208
    assert (s.SqrtNumSamples, s.MaxPathLength, s.MaxAnyHitPathLength) == (4, 3, 1)
    assert s.ApplyMultiscatteringEnergyCompensation == 1 and s.EnableIndirectSpecular == 0


def test_struct_sizes_match_reference_layouts():
    # SharedTypes.h / Model.h / DXRPathTracer.cpp:145-165 / AppSettings.h:97-128
    assert C.sizeof(A.MeshVertex) == 64
    assert C.sizeof(A.GeometryInfo) == 16
    assert C.sizeof(A.Material) == 24
    assert C.sizeof(A.SpotLight) == 48
    assert C.sizeof(A.RayTraceConstants) == 156
    assert C.sizeof(A.AppSettings) == 124
    assert A.RayTraceConstants.CurrSampleIdx.offset == 124
    assert A.RayTraceConstants.TotalNumPixels.offset == 128


def test_create_without_device_fails_cleanly():
    # no GPU in the build container: dxrpt_create must return an error code, never crash
    import torch
    if torch.cuda.is_available():
        return
    L = A.lib()
    ctx = C.c_void_p()
    rc = L.dxrpt_create(0, C.byref(ctx))
    assert rc != 0 and not ctx.value


def test_oracle_is_not_linked_by_the_product():
    for lib in ("libdxrpt.so", "libdxrpt_host.so"):
        data = open(os.path.join(A.LIB_DIR, lib), "rb").read()
        assert b"oracle_" not in data, lib


def test_option_ids_match_header():
    # every DXRPT_OPT_* id of include/dxrpt.h has the same value in the Python binding
    import re
    hdr = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "dxrpt.h")).read()
    ids = {m.group(1): int(m.group(2)) for m in re.finditer(r"#define DXRPT_OPT_(\w+)\s+(\d+)u", hdr)}
    assert len(ids) >= 29
    for name, v in ids.items():
        assert getattr(A, "OPT_" + name) == v, name
