"""ctypes mirror of the C-ABI structs (include/rt_types.h, rt_api.h, rt_scene.h).

Layouts follow MetalRaytracing/ShaderTypes.h:80-145 exactly (float3 = 16 bytes); the sizes and
offsets are asserted against the compiled library in tests/test_abi.py.
"""
import ctypes as C

c_float3 = C.c_float * 4  # x, y, z, pad (simd vector_float3: 16 bytes)


class Float3(C.Structure):
    _fields_ = [("x", C.c_float), ("y", C.c_float), ("z", C.c_float), ("_pad", C.c_float)]

    def tolist(self):
        return [self.x, self.y, self.z]


def f3(x, y, z):
    return Float3(float(x), float(y), float(z), 0.0)


class Camera(C.Structure):  # ShaderTypes.h:80-85
    _fields_ = [("position", Float3), ("right", Float3), ("up", Float3), ("forward", Float3)]


class Light(C.Structure):  # ShaderTypes.h:95-106
    _fields_ = [
        ("type", C.c_int32),
        ("_pad0", C.c_int32 * 3),
        ("position", Float3),
        ("color", Float3),
        ("forward", Float3),
        ("right", Float3),
        ("up", Float3),
        ("coneAngle", C.c_float),
        ("_pad1", C.c_float * 3),
        ("direction", Float3),
    ]


class Uniforms(C.Structure):  # ShaderTypes.h:108-130
    _fields_ = [
        ("width", C.c_int32),
        ("height", C.c_int32),
        ("blocksWide", C.c_int32),
        ("frameIndex", C.c_uint32),
        ("lightCount", C.c_int32),
        ("samplesPerPixel", C.c_int32),
        ("maxBounces", C.c_int32),
        ("_pad0", C.c_int32),
        ("camera", Camera),
        ("previousCamera", Camera),
        ("debugTextureMode", C.c_int32),
        ("accumulationWeight", C.c_float),
        ("enableDenoiseGBuffer", C.c_int32),
        ("shadingMode", C.c_int32),
        ("enableMotionAdaptiveAccumulation", C.c_int32),
        ("motionAccumulationMinWeight", C.c_float),
        ("motionAccumulationLowThresholdPixels", C.c_float),
        ("motionAccumulationHighThresholdPixels", C.c_float),
        ("enableMotionAdaptiveSampling", C.c_int32),
        ("motionSamplingMaxExtraSamples", C.c_int32),
        ("motionSamplingLowThresholdPixels", C.c_float),
        ("motionSamplingHighThresholdPixels", C.c_float),
    ]


class Material(C.Structure):  # ShaderTypes.h:137-145
    _fields_ = [
        ("baseColor", Float3),
        ("specular", Float3),
        ("emission", Float3),
        ("specularExponent", C.c_float),
        ("refractionIndex", C.c_float),
        ("opacity", C.c_float),
        ("textureFlags", C.c_uint32),
    ]


class PackedFloat4x3(C.Structure):
    _fields_ = [("columns", (C.c_float * 3) * 4)]


class TextureDesc(C.Structure):  # rt_texture_desc
    _fields_ = [("rgba8", C.c_void_p), ("width", C.c_uint32), ("height", C.c_uint32)]


TEXTURE_SLOTS = {"baseColor": 0, "normal": 1, "roughness": 2, "metallic": 3, "ao": 4, "emission": 5, "opacity": 6}


class SubmeshDesc(C.Structure):
    _fields_ = [
        ("indices", C.POINTER(C.c_uint32)),
        ("index_count", C.c_uint32),
        ("_pad", C.c_uint32),
        ("material", Material),
        ("textures", C.c_int32 * 8),
    ]


class MeshDesc(C.Structure):
    _fields_ = [
        ("positions", C.POINTER(Float3)),
        ("normals", C.POINTER(Float3)),
        ("uvs", C.c_void_p),
        ("joint_indices", C.POINTER(C.c_uint16)),
        ("joint_weights", C.POINTER(C.c_float)),
        ("vertex_count", C.c_uint32),
        ("submesh_count", C.c_uint32),
        ("submeshes", C.POINTER(SubmeshDesc)),
        ("transform", PackedFloat4x3),
        ("joint_count", C.c_uint32),
        ("_pad", C.c_uint32),
    ]


class SceneDesc(C.Structure):
    _fields_ = [
        ("mesh_count", C.c_uint32),
        ("light_count", C.c_uint32),
        ("meshes", C.POINTER(MeshDesc)),
        ("lights", C.POINTER(Light)),
        ("texture_count", C.c_uint32),
        ("_pad", C.c_uint32),
        ("textures", C.POINTER(TextureDesc)),
    ]


class Opts(C.Structure):
    _fields_ = [("device", C.c_int32), ("pipeline", C.c_int32), ("tail_paths", C.c_int32), ("sort_bins", C.c_int32),
                ("frames_in_flight", C.c_int32), ("reserved", C.c_int32 * 3)]


class PresentOpts(C.Structure):  # rt_present_opts
    _fields_ = [("out_width", C.c_int32), ("out_height", C.c_int32), ("scaler", C.c_int32), ("encode", C.c_int32),
                ("denoise_passes", C.c_int32), ("reserved", C.c_int32 * 3)]


SCALERS = {"none": 0, "spatial": 1, "temporal": 2, "denoised": 3}


class TileSet(C.Structure):
    _fields_ = [("tile_size", C.c_int32), ("rank", C.c_int32), ("nranks", C.c_int32), ("_pad", C.c_int32)]


class Stats(C.Structure):
    _fields_ = [
        ("closest_rays", C.c_uint64),
        ("shadow_rays", C.c_uint64),
        ("node_visits", C.c_uint64),
        ("tri_tests", C.c_uint64),
        ("paths", C.c_uint64),
        ("bvh_nodes", C.c_uint64),
        ("triangles", C.c_uint64),
        ("device_bytes", C.c_uint64),
        ("last_frame_ms", C.c_float),
        ("kernel_ms", C.c_float * 7),
        ("pipeline", C.c_int32),
        ("iterations", C.c_int32),
        ("trace_rays", C.c_uint64),
        ("trace_nodes", C.c_uint64),
        ("trace_tris", C.c_uint64),
        ("trace_launches", C.c_int32),
        ("trace_ms", C.c_float),
        ("trace_closest_rays", C.c_uint64),
        ("finish_launches", C.c_int32),
        ("frames_in_flight", C.c_int32),
        ("frames_total", C.c_uint64),
        ("total_closest_rays", C.c_uint64),
        ("total_shadow_rays", C.c_uint64),
        ("total_paths", C.c_uint64),
        ("total_frame_ms", C.c_double),
        ("total_kernel_ms", C.c_double * 7),
        ("total_trace_rays", C.c_uint64),
        ("total_trace_closest_rays", C.c_uint64),
        ("total_trace_ms", C.c_double),
        ("total_trace_launches", C.c_uint64),
        ("total_finish_launches", C.c_uint64),
        ("node_visits_lds", C.c_uint64),
        ("trace_nodes_lds", C.c_uint64),
        ("trace_dev_ms", C.c_float),
        ("trace_dev_launches", C.c_int32),
        ("finish_dev_ms", C.c_float),
        ("finish_dev_launches", C.c_int32),
        ("total_trace_dev_ms", C.c_double),
        ("total_trace_dev_launches", C.c_uint64),
        ("total_finish_dev_ms", C.c_double),
        ("total_finish_dev_launches", C.c_uint64),
        ("total_graph_replays", C.c_uint64),
        ("total_graph_captures", C.c_uint64),
        ("total_graph_fallbacks", C.c_uint64),
        ("total_graph_eager", C.c_uint64),
        ("total_auto_rebuilds", C.c_uint64),
        ("bvh_cost_built", C.c_float),
        ("bvh_cost_refit", C.c_float),
    ]


class MaterialOverride(C.Structure):  # Model.swift:11-27
    _fields_ = [
        ("has_base_color", C.c_int32),
        ("base_color", C.c_float * 3),
        ("has_refraction_index", C.c_int32),
        ("refraction_index", C.c_float),
        ("has_opacity", C.c_int32),
        ("opacity", C.c_float),
    ]


class Tuning(C.Structure):
    """rt_tuning (include/rt_api.h): the wavefront kernels' scheduling parameters, 0 = default."""
    _fields_ = [(n, C.c_int32) for n in ("trace_chunk", "finish_chunk", "refill_min", "shade_min", "shade_min_drained",
                                         "team", "finish_grid_pct", "trace_grid_pct", "shade_blocks", "host_rounds",
                                         "log", "device_bvh", "refit_rebuild_pct")] + [("reserved", C.c_int32 * 3)]


# enums (ShaderTypes.h)
LightTypeUnused, LightTypeSunlight, LightTypeSpotlight, LightTypePointlight, LightTypeAreaLight = range(5)
ShadingModePBR, ShadingModeLegacy = 0, 1
(DebugTextureModeNone, DebugTextureModeBaseColor, DebugTextureModeNormal, DebugTextureModeRoughness,
 DebugTextureModeMetallic, DebugTextureModeAO, DebugTextureModeEmission, DebugTextureModeMotion) = range(8)

RT_OK = 0
RT_ERR_INVALID_ARG = 1
RT_ERR_HIP = 2
RT_ERR_IO = 3
RT_ERR_OUT_OF_MEMORY = 4
RT_ERR_STATE = 5
RT_ERR_UNSUPPORTED = 6
RT_ERR_NO_DEVICE = 7
RT_PIPELINE_MEGAKERNEL = 0
RT_PIPELINE_WAVEFRONT = 1

# Every symbol include/rt_api.h and include/rt_scene.h declare (checked by tests/test_abi.py).
EXPORTED_SYMBOLS = [
    # rt_api.h
    "rt_create", "rt_destroy", "rt_last_error", "rt_set_stream", "rt_scene_upload", "rt_bvh_build",
    "rt_bvh_build_device", "rt_bvh_refit", "rt_set_instance_transforms", "rt_skin", "rt_resize", "rt_render_frame", "rt_wait",
    "rt_read_radiance", "rt_read_radiance_half", "rt_read_aux", "rt_tile_count", "rt_pack_tiles", "rt_unpack_tiles",
    "rt_pack_tiles_on", "rt_unpack_tiles_on", "rt_present", "rt_write_png",
    "rt_pack_tiles_host", "rt_unpack_tiles_host",
    "rt_set_counting", "rt_set_device_spans", "rt_set_graphs", "rt_get_stats", "rt_set_tuning", "rt_get_tuning",
    "rt_version", "rt_debug_trace_host",
    # rt_scene.h
    "rt_material_override_glass", "rt_scene_new", "rt_scene_free", "rt_scene_last_error",
    "rt_scene_add_obj", "rt_scene_add_usd", "rt_scene_add_procedural", "rt_scene_set_lights", "rt_scene_set_light_intensity",
    "rt_scene_preset", "rt_scene_get_desc", "rt_scene_triangle_count", "rt_scene_joint_matrices",
    "rt_scene_add_texture", "rt_scene_load_texture", "rt_scene_bind_texture", "rt_decode_png",
    "rt_camera_default", "rt_camera_orbit", "rt_uniforms_default", "rt_random_offsets",
]


# entry points a library built from an older revision may lack without losing any compute path
OPTIONAL = {"rt_set_device_spans"}


def declare(lib):
    """Attach argtypes/restype to every exported function."""
    P = C.POINTER
    vp = C.c_void_p
    st = C.c_int32
    sig = {
        "rt_create": (st, [P(Opts), P(vp)]),
        "rt_destroy": (st, [vp]),
        "rt_last_error": (C.c_char_p, [vp]),
        "rt_set_stream": (st, [vp, vp]),
        "rt_scene_upload": (st, [vp, P(SceneDesc)]),
        "rt_bvh_build": (st, [vp]),
        "rt_bvh_build_device": (st, [vp]),
        "rt_bvh_refit": (st, [vp]),
        "rt_set_instance_transforms": (st, [vp, P(PackedFloat4x3), C.c_uint32]),
        "rt_skin": (st, [vp, C.c_uint32, P(C.c_float), C.c_uint32]),
        "rt_resize": (st, [vp, C.c_int32, C.c_int32, P(C.c_uint32)]),
        "rt_render_frame": (st, [vp, P(Uniforms), P(TileSet)]),
        "rt_wait": (st, [vp]),
        "rt_read_radiance": (st, [vp, P(C.c_float)]),
        "rt_read_radiance_half": (st, [vp, P(C.c_uint16)]),
        "rt_read_aux": (st, [vp, P(C.c_float), P(C.c_float), P(C.c_float)]),
        "rt_tile_count": (C.c_int32, [C.c_int32, C.c_int32, P(TileSet)]),
        "rt_pack_tiles": (st, [vp, P(TileSet), vp]),
        "rt_unpack_tiles": (st, [vp, P(TileSet), vp]),
        "rt_pack_tiles_on": (st, [vp, P(TileSet), vp, vp]),
        "rt_present": (st, [vp, P(PresentOpts), vp]),
        "rt_write_png": (st, [C.c_char_p, vp, C.c_uint32, C.c_uint32]),
        "rt_unpack_tiles_on": (st, [vp, P(TileSet), vp, vp]),
        "rt_pack_tiles_host": (st, [C.c_int32, C.c_int32, P(TileSet), P(C.c_float), P(C.c_float)]),
        "rt_unpack_tiles_host": (st, [C.c_int32, C.c_int32, P(TileSet), P(C.c_float), P(C.c_float)]),
        "rt_set_counting": (st, [vp, C.c_int32]),
        "rt_set_device_spans": (st, [vp, C.c_int32]),
        "rt_set_graphs": (st, [vp, C.c_int32]),
        "rt_get_stats": (st, [vp, P(Stats)]),
        "rt_set_tuning": (st, [vp, P(Tuning)]),
        "rt_get_tuning": (st, [vp, P(Tuning)]),
        "rt_version": (C.c_char_p, []),
        "rt_debug_trace_host": (st, [P(SceneDesc), P(C.c_float), P(C.c_float), C.c_uint32, C.c_int32, P(C.c_float),
                                     P(C.c_uint32), P(C.c_float), P(C.c_float), P(C.c_uint32), P(C.c_uint32)]),
        "rt_material_override_glass": (None, [P(MaterialOverride)]),
        "rt_scene_new": (st, [P(vp)]),
        "rt_scene_free": (st, [vp]),
        "rt_scene_last_error": (C.c_char_p, [vp]),
        "rt_scene_add_obj": (st, [vp, C.c_char_p, P(C.c_float), P(C.c_float), C.c_float, P(MaterialOverride)]),
        "rt_scene_add_usd": (st, [vp, C.c_char_p, P(C.c_float), P(C.c_float), C.c_float, P(MaterialOverride)]),
        "rt_scene_add_procedural": (st, [vp, C.c_char_p, C.c_char_p, P(C.c_float), P(C.c_float), C.c_float,
                                         P(MaterialOverride)]),
        "rt_scene_set_lights": (st, [vp, P(Light), C.c_uint32]),
        "rt_scene_set_light_intensity": (st, [vp, C.c_float]),
        "rt_scene_preset": (st, [C.c_char_p, C.c_char_p, P(vp), P(C.c_int32)]),
        "rt_scene_get_desc": (st, [vp, P(SceneDesc)]),
        "rt_scene_add_texture": (st, [vp, vp, C.c_uint32, C.c_uint32, P(C.c_uint32)]),
        "rt_scene_load_texture": (st, [vp, C.c_char_p, P(C.c_uint32)]),
        "rt_scene_bind_texture": (st, [vp, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32]),
        "rt_decode_png": (st, [vp, C.c_size_t, vp, P(C.c_uint32), P(C.c_uint32), C.c_char_p, C.c_size_t]),
        "rt_scene_triangle_count": (C.c_uint64, [vp]),
        "rt_scene_joint_matrices": (st, [vp, C.c_uint32, C.c_double, P(C.c_float), C.c_uint32, P(C.c_uint32)]),
        "rt_camera_default": (None, [C.c_int32, C.c_int32, P(Camera)]),
        "rt_camera_orbit": (None, [C.c_int32, C.c_int32, P(C.c_float), C.c_float, C.c_float, C.c_float, C.c_float,
                                   P(Camera)]),
        "rt_uniforms_default": (None, [C.c_int32, C.c_int32, C.c_int32, P(Uniforms)]),
        "rt_random_offsets": (None, [C.c_uint64, C.c_int32, C.c_int32, P(C.c_uint32)]),
    }
    for name, (res, args) in sig.items():
        if name in OPTIONAL and not hasattr(lib, name):
            continue   # measurement hook absent from an older library (A/B runs); compute entry points are required
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib
