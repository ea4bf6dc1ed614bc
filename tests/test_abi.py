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
    assert L.dxrpt_abi_version() == A.ABI_VERSION == 4
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


def test_option_ids_match_the_header():
    # every DXRPT_OPT_* of include/dxrpt.h is mirrored with the same id; retired ids are neither
    txt = open(os.path.join(REPO, "include", "dxrpt.h")).read()
    hdr = {m.group(1): int(m.group(2)) for m in re.finditer(r"#define DXRPT_OPT_(\w+) (\d+)u", txt)}
    py = {k[4:]: v for k, v in vars(A).items() if k.startswith("OPT_")}
    assert hdr == py
    assert not set(hdr.values()) & set(A.RETIRED_OPTIONS)
    # the retired ids are listed once in the header (DXRPT_RETIRED_OPTIONS, which the library's
    # dxrpt_set_option uses); the Python mirror must be that list
    m = re.search(r"#define DXRPT_RETIRED_OPTIONS \{([^}]*)\}", txt)
    assert m, "DXRPT_RETIRED_OPTIONS missing from include/dxrpt.h"
    assert tuple(int(v.strip().rstrip("u")) for v in m.group(1).split(",")) == A.RETIRED_OPTIONS
    kinds = {m.group(1): int(m.group(2)) for m in re.finditer(r"#define DXRPT_K_(\w+) (\d+)", txt)}
    assert kinds["COUNT"] == A.K_COUNT == len(A.KERNEL_NAMES)
    assert (kinds["PATH"], kinds["PATH_HEAD"], kinds["PATH_TAIL"]) == (A.K_PATH, A.K_PATH_HEAD, A.K_PATH_TAIL)


def test_stats_and_tile_layouts_match_the_header(tmp_path):
    # the ctypes mirrors of dxrpt_stats / dxrpt_tile / dxrpt_bvh_info against the C compiler's layout of
    # include/dxrpt.h (gcc, host only)
    import subprocess
    src = tmp_path / "layout.c"
    src.write_text("""#include <stdio.h>
#include <stddef.h>
#include "dxrpt.h"
int main(void) {
  printf("%zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu\\n", sizeof(dxrpt_stats), offsetof(dxrpt_stats, kernel_ms),
         offsetof(dxrpt_stats, schedule), offsetof(dxrpt_stats, tail_occupancy),
         offsetof(dxrpt_stats, radiance_hits), offsetof(dxrpt_stats, census_depth1), sizeof(dxrpt_tile),
         sizeof(dxrpt_bvh_info), offsetof(dxrpt_bvh_info, phase_ms), offsetof(dxrpt_bvh_info, binary_depth_cap),
         offsetof(dxrpt_bvh_info, ref_budget_pct), offsetof(dxrpt_stats, packed_textures));
  return 0;
}
""")
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", os.path.join(REPO, "include"), str(src), "-o", str(exe)], check=True)
    got = [int(v) for v in subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split()]
    want = [C.sizeof(A.Stats), A.Stats.kernel_ms.offset, A.Stats.schedule.offset, A.Stats.tail_occupancy.offset,
            A.Stats.radiance_hits.offset, A.Stats.census_depth1.offset, C.sizeof(A.Tile), C.sizeof(A.BvhInfo),
            A.BvhInfo.phase_ms.offset, A.BvhInfo.binary_depth_cap.offset, A.BvhInfo.ref_budget_pct.offset,
            A.Stats.packed_textures.offset]
    assert got == want
