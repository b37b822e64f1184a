"""metal4-raytracing_amd — MI355X-native path tracer for the raytracingKernel hot path.

Python host mirror of the reference's Swift interface for this path, over the C-ABI
library librt_hip.so (include/rt_api.h, include/rt_scene.h):

    Scene      ~ MetalRaytracing/Scene.swift + AppScene.swift (models, lights, orbit camera)
    Renderer   ~ MetalRaytracing/Renderer.swift (knobs with didSet -> frameIndex = 0,
                 updateUniforms, draw, accumulation ping-pong)

The compute path is the HIP library; there is no CPU fallback: importing this package on a
machine without the built library raises, and Renderer() raises without a HIP device.
Load it with importlib.import_module("metal4-raytracing_amd") (the directory name has a dash).
"""
import ctypes as C
import os

import numpy as np

from . import _abi
from ._abi import (TEXTURE_SLOTS, Tuning, Camera, Float3, Light, MaterialOverride, PackedFloat4x3, SceneDesc, Stats, TextureDesc,
                   TileSet, Uniforms,
                   f3)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "librt_hip.so")
ASSET_DIR_DEFAULT = os.environ.get("RT_ASSET_DIR", os.path.join(os.path.dirname(_HERE), "assets"))

_lib = None


class RTError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"rt status {code}: {msg}")
        self.code = code


def lib():
    """The loaded librt_hip.so (raises if it was not built — no fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} is missing: run __graft_entry__.build() (make -C metal4-raytracing_amd)")
        # torch bundles its own libamdhip64.so.7 (same soname as /opt/rocm's). Load torch first so
        # the process holds ONE HIP runtime; torch.distributed / tensors then share it with us.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        _lib = _abi.declare(C.CDLL(LIB_PATH))
    return _lib


def _check(st, ctx=None, scene=None):
    if st != 0:
        if scene is not None:
            msg = lib().rt_scene_last_error(scene)
        else:
            msg = lib().rt_last_error(ctx)
        raise RTError(st, (msg or b"").decode())


def version():
    return lib().rt_version().decode()


def uniforms_default(width, height, light_count=2):
    u = Uniforms()
    lib().rt_uniforms_default(width, height, light_count, C.byref(u))
    return u


def decode_png(data):
    """PNG bytes -> (H, W, 4) uint8 RGBA (row 0 = top), the library's texture decoder."""
    buf = (C.c_uint8 * len(data)).from_buffer_copy(data)
    w, h = C.c_uint32(0), C.c_uint32(0)
    err = C.create_string_buffer(256)
    st = lib().rt_decode_png(buf, len(data), None, C.byref(w), C.byref(h), err, 256)
    if st != 0:
        raise RTError(st, err.value.decode())
    out = np.empty((h.value, w.value, 4), dtype=np.uint8)
    st = lib().rt_decode_png(buf, len(data), out.ctypes.data, C.byref(w), C.byref(h), err, 256)
    if st != 0:
        raise RTError(st, err.value.decode())
    return out


def write_png(path, rgba8):
    """(H, W, 4) uint8 rows top-down -> an RGBA PNG file (e.g. Renderer.present())."""
    a = np.ascontiguousarray(rgba8, dtype=np.uint8)
    assert a.ndim == 3 and a.shape[2] == 4, a.shape
    _check(lib().rt_write_png(str(path).encode(), a.ctypes.data, a.shape[1], a.shape[0]))


def camera_default(width, height):
    c = Camera()
    lib().rt_camera_default(width, height, C.byref(c))
    return c


def random_offsets(seed, width, height):
    """splitmix64(seed) % 2^20 per pixel, row-major (Renderer.swift:719-738, seeded)."""
    out = np.empty(width * height, dtype=np.uint32)
    lib().rt_random_offsets(seed, width, height, out.ctypes.data_as(C.POINTER(C.c_uint32)))
    return out


def debug_trace_host(scene, origins, dirs, tmax=None, any_hit=False):
    """Test hook: trace rays through the library's own BVH + traversal code on the host.
    Returns dict(t, id, u, v, nodes, tris) arrays."""
    o = np.ascontiguousarray(origins, np.float32).reshape(-1, 3)
    d = np.ascontiguousarray(dirs, np.float32).reshape(-1, 3)
    n = o.shape[0]
    rays = np.ascontiguousarray(np.concatenate([o, d], axis=1), np.float32)
    tm = None if tmax is None else np.ascontiguousarray(np.broadcast_to(tmax, (n,)), np.float32)
    out = dict(t=np.empty(n, np.float32), id=np.empty(n, np.uint32), u=np.empty(n, np.float32),
               v=np.empty(n, np.float32), nodes=np.empty(n, np.uint32), tris=np.empty(n, np.uint32))
    FP, UP = C.POINTER(C.c_float), C.POINTER(C.c_uint32)
    d_ = scene.desc()
    _check(lib().rt_debug_trace_host(C.byref(d_), rays.ctypes.data_as(FP), tm.ctypes.data_as(FP) if tm is not None else None,
                                     n, 1 if any_hit else 0, out["t"].ctypes.data_as(FP), out["id"].ctypes.data_as(UP),
                                     out["u"].ctypes.data_as(FP), out["v"].ctypes.data_as(FP),
                                     out["nodes"].ctypes.data_as(UP), out["tris"].ctypes.data_as(UP)))
    return out


def glass_override():
    o = MaterialOverride()
    lib().rt_material_override_glass(C.byref(o))
    return o


class Scene:
    """Host scene (Scene.swift / AppScene.swift / Model.swift OBJ path)."""

    def __init__(self, handle=None):
        if handle is None:
            h = C.c_void_p()
            _check(lib().rt_scene_new(C.byref(h)))
            handle = h
        self._h = handle
        self.synthetic = False

    @classmethod
    def preset(cls, name, asset_dir=None):
        h = C.c_void_p()
        synth = C.c_int32(0)
        st = lib().rt_scene_preset(name.encode(), (asset_dir or ASSET_DIR_DEFAULT).encode(), C.byref(h),
                                   C.byref(synth))
        if st != 0:
            msg = lib().rt_scene_last_error(h) if h.value else lib().rt_last_error(None)
            if h.value:
                lib().rt_scene_free(h)
            raise RTError(st, (msg or b"").decode())
        s = cls(h)
        s.synthetic = bool(synth.value)
        return s

    def add_model(self, obj_path, position, rotation=(0, 0, 0), scale=1.0, material_override=None):
        """Model(name:position:rotation:scale:materialOverride:) for an OBJ file."""
        p = (C.c_float * 3)(*position)
        r = (C.c_float * 3)(*rotation)
        _check(lib().rt_scene_add_obj(self._h, obj_path.encode(), p, r, scale,
                                      C.byref(material_override) if material_override else None), scene=self._h)

    def add_usd(self, usd_path, position, rotation=(0, 0, 0), scale=1.0, material_override=None):
        """Model(name:...) for a .usdz / .usda / .usdc asset (Model.swift:87-184)."""
        p = (C.c_float * 3)(*position)
        r = (C.c_float * 3)(*rotation)
        _check(lib().rt_scene_add_usd(self._h, usd_path.encode(), p, r, scale,
                                      C.byref(material_override) if material_override else None), scene=self._h)

    def add_procedural(self, kind, position, rotation=(0, 0, 0), scale=1.0, material_override=None, mtl_path=None):
        p = (C.c_float * 3)(*position)
        r = (C.c_float * 3)(*rotation)
        _check(lib().rt_scene_add_procedural(self._h, kind.encode(), mtl_path.encode() if mtl_path else None, p, r,
                                             scale, C.byref(material_override) if material_override else None),
               scene=self._h)

    def add_texture(self, rgba8):
        """Adds an (H, W, 4) uint8 texture (row 0 = top); returns its id."""
        a = np.ascontiguousarray(rgba8, dtype=np.uint8)
        assert a.ndim == 3 and a.shape[2] == 4, a.shape
        tid = C.c_uint32(0)
        _check(lib().rt_scene_add_texture(self._h, a.ctypes.data, a.shape[1], a.shape[0], C.byref(tid)), scene=self._h)
        return tid.value

    def load_texture(self, png_path):
        """Decodes a PNG file into the scene's textures (MTKTextureLoader stand-in); returns its id."""
        tid = C.c_uint32(0)
        _check(lib().rt_scene_load_texture(self._h, png_path.encode(), C.byref(tid)), scene=self._h)
        return tid.value

    def bind_texture(self, mesh_index, submesh_index, slot, texture_id):
        """slot: 'baseColor' | 'normal' | 'roughness' | 'metallic' | 'ao' | 'emission' | 'opacity'
        (or its index).  Sets the material's textureFlags bit (and baseColor = 1 for baseColor)."""
        k = TEXTURE_SLOTS[slot] if isinstance(slot, str) else int(slot)
        _check(lib().rt_scene_bind_texture(self._h, mesh_index, submesh_index, k, texture_id), scene=self._h)

    def set_lights(self, lights):
        arr = (Light * len(lights))(*lights)
        _check(lib().rt_scene_set_lights(self._h, arr, len(lights)), scene=self._h)

    def set_light_intensity(self, intensity):
        _check(lib().rt_scene_set_light_intensity(self._h, intensity), scene=self._h)

    def desc(self):
        d = SceneDesc()
        _check(lib().rt_scene_get_desc(self._h, C.byref(d)), scene=self._h)
        return d

    @property
    def triangle_count(self):
        return int(lib().rt_scene_triangle_count(self._h))

    @property
    def light_count(self):
        return int(self.desc().light_count)

    def joint_matrices(self, mesh_index, time_seconds, capacity=256):
        out = np.zeros((capacity, 16), dtype=np.float32)
        n = C.c_uint32(0)
        _check(lib().rt_scene_joint_matrices(self._h, mesh_index, time_seconds,
                                             out.ctypes.data_as(C.POINTER(C.c_float)), capacity, C.byref(n)),
               scene=self._h)
        return out[: n.value].copy()

    def close(self):
        if self._h:
            lib().rt_scene_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


_KNOBS = {
    # Renderer.swift:52-192 property -> (Uniforms field, default)
    "samplesPerPixel": ("samplesPerPixel", 2),
    "maxBounces": ("maxBounces", 2),
    "accumulationWeight": ("accumulationWeight", 0.9),
    "useMotionAdaptiveAccumulation": ("enableMotionAdaptiveAccumulation", True),
    "motionAccumulationMinWeight": ("motionAccumulationMinWeight", 0.1),
    "motionAccumulationLowThresholdPixels": ("motionAccumulationLowThresholdPixels", 0.5),
    "motionAccumulationHighThresholdPixels": ("motionAccumulationHighThresholdPixels", 4.0),
    "useMotionAdaptiveSampling": ("enableMotionAdaptiveSampling", True),
    "motionSamplingMaxExtraSamples": ("motionSamplingMaxExtraSamples", 2),
    "motionSamplingLowThresholdPixels": ("motionSamplingLowThresholdPixels", 1.0),
    "motionSamplingHighThresholdPixels": ("motionSamplingHighThresholdPixels", 6.0),
    "debugTextureMode": ("debugTextureMode", 0),
    "shadingMode": ("shadingMode", 0),
    "useTemporalDenoiser": ("enableDenoiseGBuffer", False),
}


# Legacy environment names of the rt_tuning fields (and of three rt_opts / rt_set_graphs settings),
# read by tuning_from_env for the test and bench harnesses only: the library itself reads none.
_TUNING_ENV = {"RT_CHUNK": "trace_chunk", "RT_FCHUNK": "finish_chunk", "RT_REFILL_MIN": "refill_min",
               "RT_SHADE_MIN": "shade_min", "RT_SHADE_MIN_X": "shade_min_drained", "RT_TEAM": "team",
               "RT_FINISH_FRAC": "finish_grid_pct", "RT_TRACE_FRAC": "trace_grid_pct", "RT_SHADE_BLOCKS": "shade_blocks",
               "RT_WF_HOST": "host_rounds", "RT_WF_LOG": "log", "RT_DEVICE_BVH": "device_bvh"}


def tuning_from_env(environ=None):
    """Harness convenience (bench.py, the tests' child processes): the rt_tuning fields named by the
    legacy RT_* environment variables (RT_TEAM: 0 = off, as before; RT_DEVICE_BVH=lbvh), plus
    'tail_paths' (RT_TAIL_RAYS), 'frames_in_flight' (RT_FRAMES_IN_FLIGHT) and 'graphs' (RT_GRAPH).
    The library reads no environment variable: a caller sets these with Renderer(tuning=...) /
    rt_set_tuning, rt_opts and rt_set_graphs."""
    env = os.environ if environ is None else environ
    out = {}
    for name, field in _TUNING_ENV.items():
        v = env.get(name)
        if v is None or v == "":
            continue
        if field == "team":
            out[field] = 1 if int(v) in (0, 1) else int(v)
        elif field == "device_bvh":
            out[field] = 1 if v == "lbvh" else 0
        else:
            out[field] = int(v)
    for name, key in (("RT_TAIL_RAYS", "tail_paths"), ("RT_FRAMES_IN_FLIGHT", "frames_in_flight"), ("RT_GRAPH", "graphs")):
        if env.get(name):
            out[key] = int(env[name])
    return out


def _tuning_struct(fields):
    t = Tuning()
    for k, v in fields.items():
        if not hasattr(t, k) or k == "reserved":
            raise KeyError(f"unknown rt_tuning field {k!r}")
        setattr(t, k, int(v))
    return t


class Renderer:
    """Renderer.swift for the hot path: owns a device context, the uniforms and the frame index.

    Setting any knob resets frameIndex to 0 (the reference's didSet { frameIndex = 0 }).
    draw() = updateUniforms + raytracingKernel dispatch + accumulation swap.
    """

    def __init__(self, scene, width, height, device=0, pipeline="wavefront", seed=1, stream=None, tail_paths=0,
                 sort_bins=0, bvh="sah", frames_in_flight=0, tuning=None):
        object.__setattr__(self, "_ctx", None)
        self.scene = scene
        self.width, self.height = int(width), int(height)
        opts = _abi.Opts()
        opts.device = device
        opts.pipeline = {"megakernel": 0, "wavefront": 1}[pipeline]
        opts.tail_paths = int(tail_paths)
        opts.sort_bins = int(sort_bins)   # 0 = default hit sort, < 0 = none
        opts.frames_in_flight = int(frames_in_flight)   # 0 = default (one per HIP hardware queue: 4, or 8 with GPU_MAX_HW_QUEUES >= 8; within a 96 GB budget, >= 2), 1 = one frame at a time
        ctx = C.c_void_p()
        _check(lib().rt_create(C.byref(opts), C.byref(ctx)))
        object.__setattr__(self, "_ctx", ctx)
        if stream is not None:
            _check(lib().rt_set_stream(ctx, C.c_void_p(stream)), ctx)
        if tuning:
            self.set_tuning(**tuning)
        d = scene.desc()
        self.light_count = int(d.light_count)
        _check(lib().rt_scene_upload(ctx, C.byref(d)), ctx)
        self.bvh_builder = bvh   # "sah": host binned-SAH build; "lbvh": on-device build
        _check((lib().rt_bvh_build_device if bvh == "lbvh" else lib().rt_bvh_build)(ctx), ctx)
        self.random = random_offsets(seed, self.width, self.height)
        _check(lib().rt_resize(ctx, self.width, self.height, self.random.ctypes.data_as(C.POINTER(C.c_uint32))), ctx)
        self.camera = camera_default(self.width, self.height)
        self.previousCamera = None
        self.frameIndex = 0
        self._knobs = {k: v for k, (_, v) in _KNOBS.items()}

    def __getattr__(self, name):
        knobs = self.__dict__.get("_knobs")
        if knobs is not None and name in knobs:
            return knobs[name]
        raise AttributeError(name)

    def __setattr__(self, name, value):
        if name in _KNOBS and "_knobs" in self.__dict__:
            self._knobs[name] = value
            self.__dict__["frameIndex"] = 0  # didSet { frameIndex = 0 }
            return
        object.__setattr__(self, name, value)

    # --- Renderer.updateUniforms (Renderer.swift:608-664) ---
    def uniforms(self):
        u = uniforms_default(self.width, self.height, self.light_count)
        for k, (field, _) in _KNOBS.items():
            v = self._knobs[k]
            setattr(u, field, int(v) if isinstance(v, bool) else v)
        u.camera = self.camera
        u.previousCamera = self.previousCamera if self.previousCamera is not None else self.camera
        u.frameIndex = self.frameIndex
        return u

    def draw(self, tiles=None):
        u = self.uniforms()
        ts = None
        if tiles is not None:
            ts = TileSet(tiles[0], tiles[1], tiles[2], 0)
        _check(lib().rt_render_frame(self._ctx, C.byref(u), C.byref(ts) if ts else None), self._ctx)
        self.__dict__["frameIndex"] = self.frameIndex + 1
        self.previousCamera = self.camera
        return u

    def set_tuning(self, **fields):
        """rt_set_tuning: the wavefront kernels' scheduling parameters (rt_tuning fields; omitted = default)."""
        _check(lib().rt_set_tuning(self._ctx, C.byref(_tuning_struct(fields))), self._ctx)

    def tuning(self):
        """rt_get_tuning: the parameters in effect, defaults resolved."""
        t = Tuning()
        _check(lib().rt_get_tuning(self._ctx, C.byref(t)), self._ctx)
        return {n: getattr(t, n) for n, _ in Tuning._fields_ if n != "reserved"}

    def wait(self):
        _check(lib().rt_wait(self._ctx), self._ctx)

    def set_counting(self, on):
        _check(lib().rt_set_counting(self._ctx, 1 if on else 0), self._ctx)

    def set_device_spans(self, on):
        """Device-clock launch spans in the stats (rt_set_device_spans; measurement only)."""
        _check(lib().rt_set_device_spans(self._ctx, 1 if on else 0), self._ctx)

    def set_graphs(self, on):
        """Frames captured as HIP graphs and replayed (default) or enqueued launch by launch
        (rt_set_graphs); frames enqueued eagerly always record their per-stage times."""
        _check(lib().rt_set_graphs(self._ctx, 1 if on else 0), self._ctx)

    def stats(self):
        s = Stats()
        _check(lib().rt_get_stats(self._ctx, C.byref(s)), self._ctx)
        return s

    def radiance(self):
        out = np.empty((self.height, self.width, 4), dtype=np.float32)
        _check(lib().rt_read_radiance(self._ctx, out.ctypes.data_as(C.POINTER(C.c_float))), self._ctx)
        return out

    def radiance_half(self):
        """rt_read_radiance_half: the radiance as RGBA16F (the reference's accumulation format,
        Renderer.swift:685), rounded to nearest even on the device; (H, W, 4) float16."""
        out = np.empty((self.height, self.width, 4), dtype=np.float16)
        _check(lib().rt_read_radiance_half(self._ctx, out.ctypes.data_as(C.POINTER(C.c_uint16))), self._ctx)
        return out

    def aux(self, gbuffer=False):
        depth = np.empty((self.height, self.width), dtype=np.float32)
        motion = np.empty((self.height, self.width, 2), dtype=np.float32)
        gb = np.empty((4, self.height, self.width, 4), dtype=np.float32) if gbuffer else None
        FP = C.POINTER(C.c_float)
        _check(lib().rt_read_aux(self._ctx, depth.ctypes.data_as(FP), motion.ctypes.data_as(FP),
                                 gb.ctypes.data_as(FP) if gb is not None else None), self._ctx)
        return depth, motion, gb

    def set_instance_transforms(self, mats):
        """mats: (n, 4, 3) packed column-major object->world (updateInstanceDescriptors)."""
        arr = np.ascontiguousarray(mats, dtype=np.float32).reshape(-1, 12)
        _check(lib().rt_set_instance_transforms(self._ctx, arr.ctypes.data_as(C.POINTER(PackedFloat4x3)),
                                                arr.shape[0]), self._ctx)

    def skin(self, mesh_index, joints):
        j = np.ascontiguousarray(joints, dtype=np.float32)
        _check(lib().rt_skin(self._ctx, mesh_index, j.ctypes.data_as(C.POINTER(C.c_float)), j.shape[0]), self._ctx)

    def refit(self):
        _check(lib().rt_bvh_refit(self._ctx), self._ctx)

    def rebuild(self, device=None):
        """Full BVH rebuild from the current geometry (Renderer.swift:1252-1277); on the GPU when
        device is True (default: the builder this renderer was created with)."""
        dev = (self.bvh_builder == "lbvh") if device is None else device
        _check((lib().rt_bvh_build_device if dev else lib().rt_bvh_build)(self._ctx), self._ctx)

    def present(self, width=None, height=None, scaler="none", srgb=True, denoise_passes=0):
        """Display image of the newest frame (FramePresenter + Shaders.metal): resampled to
        width x height ('none' = nearest, 'spatial' = bilinear, 'temporal' = reprojected history
        through the motion vectors, 'denoised' = G-buffer-guided a-trous filter then 'temporal';
        needs useTemporalDenoiser), tone-mapped c / (1 + c), 8-bit sRGB (or linear) RGBA rows
        top-down."""
        o = _abi.PresentOpts()
        o.out_width = int(width or 0)
        o.out_height = int(height or 0)
        o.scaler = _abi.SCALERS[scaler]
        o.encode = 0 if srgb else 1
        o.denoise_passes = int(denoise_passes)
        out = np.empty((height or self.height, width or self.width, 4), dtype=np.uint8)
        _check(lib().rt_present(self._ctx, C.byref(o), out.ctypes.data), self._ctx)
        return out

    def resize(self, width, height, seed=1):
        """mtkView(_:drawableSizeWillChange:) (Renderer.swift:1505-1511): new targets and random
        offsets, frameIndex = 0.  Frames in flight finish first."""
        self.width, self.height = int(width), int(height)
        self.random = random_offsets(seed, self.width, self.height)
        _check(lib().rt_resize(self._ctx, self.width, self.height, self.random.ctypes.data_as(C.POINTER(C.c_uint32))),
               self._ctx)
        self.camera = camera_default(self.width, self.height)
        self.previousCamera = None
        self.frameIndex = 0

    def upload(self, desc):
        """Re-uploads a scene description (rt_scene_upload) and rebuilds the BVH."""
        _check(lib().rt_scene_upload(self._ctx, C.byref(desc)), self._ctx)
        self.rebuild()

    def tile_count(self, tile_size, rank, nranks):
        ts = TileSet(tile_size, rank, nranks, 0)
        return int(lib().rt_tile_count(self.width, self.height, C.byref(ts)))

    def pack_tiles(self, tile_size, rank, nranks, device_ptr, stream=None):
        """Packs this rank's tiles of the newest frame (after it, on `stream`: a HIP stream handle, 0 =
        HIP's null stream, i.e. torch's default stream; None = the renderer's stream); no host wait."""
        ts = TileSet(tile_size, rank, nranks, 0)
        if stream is None:
            _check(lib().rt_pack_tiles(self._ctx, C.byref(ts), C.c_void_p(device_ptr)), self._ctx)
        else:
            _check(lib().rt_pack_tiles_on(self._ctx, C.byref(ts), C.c_void_p(device_ptr), C.c_void_p(stream)),
                   self._ctx)

    def unpack_tiles(self, tile_size, rank, nranks, device_ptr, stream=None):
        ts = TileSet(tile_size, rank, nranks, 0)
        if stream is None:
            _check(lib().rt_unpack_tiles(self._ctx, C.byref(ts), C.c_void_p(device_ptr)), self._ctx)
        else:
            _check(lib().rt_unpack_tiles_on(self._ctx, C.byref(ts), C.c_void_p(device_ptr), C.c_void_p(stream)),
                   self._ctx)

    def set_stream(self, stream_handle):
        _check(lib().rt_set_stream(self._ctx, C.c_void_p(stream_handle) if stream_handle else None), self._ctx)

    def close(self):
        ctx = self.__dict__.get("_ctx")
        if ctx:
            lib().rt_destroy(ctx)
            object.__setattr__(self, "_ctx", None)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
