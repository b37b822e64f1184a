"""C-ABI boundary checks on CPU: the library loads, exports every symbol the public headers
declare, the ctypes mirror matches the C layouts, and device entry points fail loudly without a
GPU (no CPU fallback)."""
import ctypes as C
import os
import re
import subprocess

import pytest

from conftest import ROOT


def _declared(header):
    src = open(os.path.join(ROOT, "include", header)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return set(re.findall(r"\b(rt_[a-z0-9_]+)\s*\(", src))


def test_library_exports_every_declared_symbol(rt):
    lib = rt.lib()
    declared = _declared("rt_api.h") | _declared("rt_scene.h")
    assert declared, "no declarations parsed"
    missing = [s for s in sorted(declared) if not hasattr(lib, s)]
    assert not missing, missing
    assert declared == set(rt._abi.EXPORTED_SYMBOLS), declared ^ set(rt._abi.EXPORTED_SYMBOLS)


def test_struct_layouts_match_c(rt, tmp_path):
    """Compile the public headers with gcc and compare sizes/offsets with the ctypes mirror."""
    prog = tmp_path / "layout.c"
    prog.write_text(r'''
#include <stdio.h>
#include <stddef.h>
#include "rt_api.h"
#include "rt_scene.h"
#define P(T) printf(#T " %zu\n", sizeof(T))
#define O(T, f) printf(#T "." #f " %zu\n", offsetof(T, f))
int main(void) {
  P(Camera); P(Light); P(Uniforms); P(Material); P(rt_packed_float4x3); P(rt_submesh_desc); P(rt_mesh_desc);
  P(rt_scene_desc); P(rt_opts); P(rt_tile_set); P(rt_stats); P(rt_material_override);
  O(Light, position); O(Light, coneAngle); O(Light, direction); O(Uniforms, camera); O(Uniforms, previousCamera);
  O(Uniforms, debugTextureMode); O(Uniforms, motionSamplingHighThresholdPixels); O(Material, textureFlags);
  O(rt_mesh_desc, transform); O(rt_mesh_desc, joint_count); O(rt_submesh_desc, material); O(rt_stats, kernel_ms);
  O(rt_stats, iterations); O(rt_stats, total_kernel_ms); O(rt_stats, total_finish_launches); O(rt_stats, trace_nodes_lds); O(rt_stats, total_finish_dev_launches);
  return 0;
}''')
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), str(prog), "-o", str(exe)], check=True)
    out = dict(line.rsplit(" ", 1) for line in subprocess.check_output([str(exe)]).decode().splitlines())
    A = rt._abi
    sizes = {"Camera": A.Camera, "Light": A.Light, "Uniforms": A.Uniforms, "Material": A.Material,
             "rt_packed_float4x3": A.PackedFloat4x3, "rt_submesh_desc": A.SubmeshDesc, "rt_mesh_desc": A.MeshDesc,
             "rt_scene_desc": A.SceneDesc, "rt_opts": A.Opts, "rt_tile_set": A.TileSet, "rt_stats": A.Stats,
             "rt_material_override": A.MaterialOverride}
    for name, cls in sizes.items():
        assert int(out[name]) == C.sizeof(cls), name
    # ShaderTypes.h layout
    assert int(out["Camera"]) == 64 and int(out["Light"]) == 128
    assert int(out["Uniforms"]) == 208 and int(out["Material"]) == 64
    offs = {"Light.position": A.Light.position.offset, "Light.coneAngle": A.Light.coneAngle.offset,
            "Light.direction": A.Light.direction.offset, "Uniforms.camera": A.Uniforms.camera.offset,
            "Uniforms.previousCamera": A.Uniforms.previousCamera.offset,
            "Uniforms.debugTextureMode": A.Uniforms.debugTextureMode.offset,
            "Uniforms.motionSamplingHighThresholdPixels": A.Uniforms.motionSamplingHighThresholdPixels.offset,
            "Material.textureFlags": A.Material.textureFlags.offset, "rt_mesh_desc.transform": A.MeshDesc.transform.offset,
            "rt_mesh_desc.joint_count": A.MeshDesc.joint_count.offset,
            "rt_submesh_desc.material": A.SubmeshDesc.material.offset, "rt_stats.kernel_ms": A.Stats.kernel_ms.offset,
            "rt_stats.iterations": A.Stats.iterations.offset,
            "rt_stats.total_kernel_ms": A.Stats.total_kernel_ms.offset,
            "rt_stats.total_finish_launches": A.Stats.total_finish_launches.offset,
            "rt_stats.trace_nodes_lds": A.Stats.trace_nodes_lds.offset,
            "rt_stats.total_finish_dev_launches": A.Stats.total_finish_dev_launches.offset}
    for k, v in offs.items():
        assert int(out[k]) == v, k
    assert offs["Light.position"] == 16 and offs["Light.direction"] == 112 and offs["Uniforms.camera"] == 32


def test_version_and_no_cpu_fallback(rt):
    assert "gfx950" in rt.version()
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present: covered by -m gpu tests")
    opts = rt._abi.Opts()
    ctx = C.c_void_p()
    st = rt.lib().rt_create(C.byref(opts), C.byref(ctx))
    assert st == rt._abi.RT_ERR_NO_DEVICE and not ctx.value
    with pytest.raises(rt.RTError):
        rt.Renderer(rt.Scene.preset("c1"), 8, 8)


def test_null_arguments_return_status(rt):
    lib = rt.lib()
    assert lib.rt_scene_upload(None, None) == rt._abi.RT_ERR_INVALID_ARG
    assert lib.rt_render_frame(None, None, None) == rt._abi.RT_ERR_INVALID_ARG
    assert lib.rt_get_stats(None, None) == rt._abi.RT_ERR_INVALID_ARG
    assert lib.rt_last_error(None)  # message set, no crash


def test_tile_count(rt):
    ts = rt._abi.TileSet(64, 0, 1, 0)
    assert rt.lib().rt_tile_count(1920, 1080, C.byref(ts)) == 30 * 17
    total = 0
    for r in range(8):
        ts = rt._abi.TileSet(64, r, 8, 0)
        total += rt.lib().rt_tile_count(1920, 1080, C.byref(ts))
    assert total == 30 * 17
