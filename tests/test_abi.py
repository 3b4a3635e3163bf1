"""C-ABI checks that need no GPU: the HIP library loads, exports every entry point declared in
include/sightpy_rt.h, the ctypes binding declares the same set, the table records have the C
layout (a gcc-compiled probe of the header against the numpy dtypes), and without a visible GPU the
backend fails loudly instead of falling back to the CPU."""
import ctypes
import re
import subprocess

import numpy as np
import pytest

from conftest import ROOT

HEADER = ROOT / "include" / "sightpy_rt.h"
LIB = ROOT / "python-raytracer_amd" / "sightpy" / "libsightpy_hip.so"


def header_functions():
    text = re.sub(r"/\*.*?\*/|//[^\n]*", "", HEADER.read_text(), flags=re.S)
    return sorted(set(re.findall(r"\b(srt_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_the_entry_points():
    fns = header_functions()
    assert {"srt_create", "srt_upload_scene", "srt_render", "srt_trace", "srt_nearest",
            "srt_intersect_collider", "srt_primary_rays", "srt_last_error"} <= set(fns)


def test_library_exports_every_header_symbol():
    if not LIB.exists():
        pytest.skip("libsightpy_hip.so not built (run __graft_entry__.build())")
    lib = ctypes.CDLL(str(LIB))
    missing = [f for f in header_functions() if not hasattr(lib, f)]
    assert not missing, missing
    nm = subprocess.run(["nm", "-D", "--defined-only", str(LIB)], capture_output=True, text=True).stdout
    exported = set(re.findall(r"\bT (srt_[a-z0-9_]+)\b", nm))
    assert set(header_functions()) <= exported


def test_binding_covers_the_header():
    from sightpy import _native as N

    assert set(N.SIGNATURES) == set(header_functions())


def test_abi_version_and_no_gpu_behaviour():
    if not LIB.exists():
        pytest.skip("libsightpy_hip.so not built")
    from sightpy import _native as N

    lib = N.load_library()
    assert lib.srt_abi_version() == N.ABI_VERSION
    n = ctypes.c_int(-1)
    rc = lib.srt_device_count(ctypes.byref(n))
    if rc == 0 and n.value > 0:
        pytest.skip("a GPU is visible")
    import sightpy._backend as B

    saved = dict(B._STATE)
    try:
        B._STATE.update(lib=None, ctx=None)
        with pytest.raises(N.BackendUnavailable):
            B.context()
    finally:
        B._STATE.update(saved)


PROBE = r"""
#include <stdio.h>
#include <stddef.h>
#include "sightpy_rt.h"
#define S(T) printf(#T " %zu\n", sizeof(T));
#define O(T, f) printf(#T "." #f " %zu\n", offsetof(T, f));
int main(void) {
  S(srt_collider) S(srt_material) S(srt_texture) S(srt_light) S(srt_scene_desc) S(srt_camera)
  S(srt_render_args) S(srt_stats) S(srt_trace_args) S(srt_mt_state) S(srt_children)
  O(srt_children, diffuse_reflections)
  O(srt_collider, p) O(srt_material, p) O(srt_texture, lut) O(srt_stats, total_rays)
  O(srt_render_args, out_hit_id) O(srt_render_args, seed) O(srt_camera, xs)
  return 0;
}
"""


def test_struct_layout_matches_binding(tmp_path):
    from sightpy import _native as N

    src = tmp_path / "probe.c"
    src.write_text(PROBE)
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-std=c11", "-I", str(HEADER.parent), "-o", str(exe), str(src)], check=True)
    vals = dict(line.rsplit(" ", 1) for line in subprocess.run([str(exe)], capture_output=True, text=True,
                                                               check=True).stdout.splitlines())
    vals = {k: int(v) for k, v in vals.items()}
    assert vals["srt_collider"] == N.COLLIDER_DTYPE.itemsize
    assert vals["srt_material"] == N.MATERIAL_DTYPE.itemsize
    assert vals["srt_texture"] == N.TEXTURE_DTYPE.itemsize
    assert vals["srt_light"] == N.LIGHT_DTYPE.itemsize
    assert vals["srt_collider.p"] == N.COLLIDER_DTYPE.fields["p"][1]
    assert vals["srt_material.p"] == N.MATERIAL_DTYPE.fields["p"][1]
    assert vals["srt_texture.lut"] == N.TEXTURE_DTYPE.fields["lut"][1]
    for name, cls in (("srt_scene_desc", N.SceneDesc), ("srt_camera", N.CameraDesc),
                      ("srt_render_args", N.RenderArgs), ("srt_stats", N.Stats), ("srt_trace_args", N.TraceArgs),
                      ("srt_children", N.Children)):
        assert vals[name] == ctypes.sizeof(cls), name
    assert vals["srt_children.diffuse_reflections"] == N.Children.diffuse_reflections.offset
    assert vals["srt_stats.total_rays"] == N.Stats.total_rays.offset
    assert vals["srt_render_args.out_hit_id"] == N.RenderArgs.out_hit_id.offset
    assert vals["srt_render_args.seed"] == N.RenderArgs.seed.offset
    assert vals["srt_mt_state"] == ctypes.sizeof(N.MtState)
    assert vals["srt_camera.xs"] == N.CameraDesc.xs.offset
