"""Python handle on the CPU oracle (oracle/rt_oracle.c).  TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module, and
only as the checker / CPU baseline.  The product path (metal4-raytracing_amd) never loads it.
"""
import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# RT_ORACLE_LIB selects another build of the same source (e.g. _build/librt_oracle_native.so)
LIB_PATH = os.environ.get("RT_ORACLE_LIB") or os.path.join(_HERE, "_build", "librt_oracle.so")
_lib = None


def _abi():
    import importlib
    return importlib.import_module("metal4-raytracing_amd")._abi


class Frame(C.Structure):
    _fields_ = [
        ("uniforms", C.c_void_p),
        ("random", C.POINTER(C.c_uint32)),
        ("accum_in", C.POINTER(C.c_float)),
        ("accum_out", C.POINTER(C.c_float)),
        ("depth", C.POINTER(C.c_float)),
        ("motion", C.POINTER(C.c_float)),
        ("gbuffer", C.POINTER(C.c_float)),
        ("row_start", C.c_int32),
        ("row_step", C.c_int32),
        ("threads", C.c_int32),
        ("tile_size", C.c_int32),
        ("rank", C.c_int32),
        ("nranks", C.c_int32),
        ("closest_rays", C.c_uint64),
        ("shadow_rays", C.c_uint64),
        ("paths", C.c_uint64),
    ]


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def _cpu_key():
    """A short key of this host's CPU (model + feature flags): a -march=native build is only ever
    loaded on a CPU with the same key (the tree travels between machines)."""
    import hashlib
    text = ""
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith(("model name", "flags")):
                text += ln
                if ln.startswith("flags"):
                    break
    except OSError:
        pass
    return hashlib.sha1(text.encode()).hexdigest()[:12]


def build_native():
    """Builds the -march=native variant for this machine's CPU (CPU baseline); returns its path or
    None."""
    path = os.path.join(_HERE, "_build", "librt_oracle_native_%s.so" % _cpu_key())
    try:
        subprocess.run(["make", "-s", "-C", _HERE, "native", "NATIVE=" + os.path.relpath(path, _HERE)], check=True,
                       capture_output=True, timeout=120)
    except (OSError, subprocess.SubprocessError):
        return None
    return path if os.path.exists(path) else None


def use_library(path):
    """Selects the oracle build to load (before the first call into it)."""
    global LIB_PATH
    if _lib is not None and path != LIB_PATH:
        raise RuntimeError("oracle library already loaded from " + LIB_PATH)
    LIB_PATH = path


def default_threads():
    """Worker threads for oracle renders: the CPUs this process may run on, capped at 16 (the CPU
    share of one GPU on the GPU boxes, whose nproc counts the whole machine)."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    return max(1, min(n, 16))


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        A = _abi()
        vp = C.c_void_p
        FP = C.POINTER(C.c_float)
        L.rt_oracle_scene_create.argtypes = [C.POINTER(A.SceneDesc), C.POINTER(vp)]
        L.rt_oracle_scene_create.restype = C.c_int
        L.rt_oracle_scene_destroy.argtypes = [vp]
        L.rt_oracle_scene_destroy.restype = None
        L.rt_oracle_scene_triangles.argtypes = [vp]
        L.rt_oracle_scene_triangles.restype = C.c_uint32
        L.rt_oracle_render.argtypes = [vp, C.POINTER(Frame)]
        L.rt_oracle_render.restype = C.c_int
        L.rt_oracle_halton.argtypes = [C.c_int32, C.c_int32]
        L.rt_oracle_halton.restype = C.c_float
        L.rt_oracle_sincos.argtypes = [C.c_float, FP, FP]
        L.rt_oracle_sincos.restype = None
        L.rt_oracle_pow5.argtypes = [C.c_float]
        L.rt_oracle_pow5.restype = C.c_float
        for name in ("rt_oracle_intersect", "rt_oracle_intersect_bruteforce"):
            f = getattr(L, name)
            f.argtypes = [vp, FP, FP, C.c_float, C.c_float, C.c_int, FP, C.POINTER(C.c_uint32), FP, FP]
            f.restype = C.c_int
        L.rt_oracle_skin.argtypes = [vp, vp, vp, vp, vp, vp, vp, C.c_uint32]
        L.rt_oracle_skin.restype = None
        L.rt_oracle_scene_set_previous.argtypes = [vp, C.c_uint32, vp, vp]
        L.rt_oracle_scene_set_previous.restype = C.c_int
        L.rt_oracle_tex_sample.argtypes = [vp, C.c_int32, C.c_float, C.c_float, C.c_int32, FP]
        L.rt_oracle_tex_sample.restype = C.c_int
        _lib = L
    return _lib


def halton(i, d):
    return float(lib().rt_oracle_halton(i, d))


def sincos(x):
    s, c = C.c_float(), C.c_float()
    lib().rt_oracle_sincos(x, C.byref(s), C.byref(c))
    return s.value, c.value


def pow5(x):
    return float(lib().rt_oracle_pow5(x))


class OracleScene:
    def __init__(self, desc):
        h = C.c_void_p()
        if lib().rt_oracle_scene_create(C.byref(desc), C.byref(h)) != 0:
            raise RuntimeError("oracle scene create failed")
        self._h = h
        self._desc = desc  # keep the arrays it points at alive via the caller's scene

    @property
    def triangles(self):
        return int(lib().rt_oracle_scene_triangles(self._h))

    def tex_sample(self, tex, u, v, srgb=False):
        out = (C.c_float * 4)()
        if lib().rt_oracle_tex_sample(self._h, tex, u, v, 1 if srgb else 0, out) != 0:
            raise ValueError("bad texture")
        return np.array(list(out), dtype=np.float32)

    def intersect(self, o, d, tmin=0.0, tmax=float("inf"), any_hit=False, brute=False):
        fo = (C.c_float * 3)(*o)
        fd = (C.c_float * 3)(*d)
        t, u, v = C.c_float(), C.c_float(), C.c_float()
        i = C.c_uint32()
        fn = lib().rt_oracle_intersect_bruteforce if brute else lib().rt_oracle_intersect
        hit = fn(self._h, fo, fd, tmin, tmax, 1 if any_hit else 0, C.byref(t), C.byref(i), C.byref(u), C.byref(v))
        if not hit:
            return None
        return (t.value, i.value, u.value, v.value)

    def set_previous(self, mesh, prev_positions=None, prev_transform=None):
        """Motion-vector history of one mesh: positions (n,4) f32 before the last skinning tick
        and/or the previous (4,3) packed transform. The arrays must outlive the scene."""
        pp = None if prev_positions is None else prev_positions.ctypes.data
        pt = None if prev_transform is None else np.ascontiguousarray(prev_transform, np.float32).ctypes.data
        if lib().rt_oracle_scene_set_previous(self._h, mesh, pp, pt) != 0:
            raise RuntimeError("set_previous failed")

    def render(self, uniforms, random, accum_in=None, motion_in=None, gbuffer=False, row_start=0, row_step=1,
               threads=None, tiles=None):
        """Render one frame (rows row_start + k * row_step; tiles = (tile_size, rank, nranks): only that
        rank's tiles); returns dict(radiance HxWx4, depth, motion, gbuffer, counts).  Pixels not
        rendered stay zero (motion: the motion_in value)."""
        W, H = uniforms.width, uniforms.height
        accum_out = np.zeros((H, W, 4), np.float32)
        depth = np.zeros((H, W), np.float32)
        motion = np.zeros((H, W, 2), np.float32) if motion_in is None else np.array(motion_in, np.float32, copy=True)
        gb = np.zeros((4, H, W, 4), np.float32) if gbuffer else None
        rnd = np.ascontiguousarray(random, dtype=np.uint32)
        FP = C.POINTER(C.c_float)
        ain = np.ascontiguousarray(accum_in, np.float32) if accum_in is not None else None
        f = Frame()
        f.uniforms = C.cast(C.pointer(uniforms), C.c_void_p)
        f.random = rnd.ctypes.data_as(C.POINTER(C.c_uint32))
        f.accum_in = ain.ctypes.data_as(FP) if ain is not None else None
        f.accum_out = accum_out.ctypes.data_as(FP)
        f.depth = depth.ctypes.data_as(FP)
        f.motion = motion.ctypes.data_as(FP)
        f.gbuffer = gb.ctypes.data_as(FP) if gb is not None else None
        f.row_start = row_start
        f.row_step = row_step
        f.threads = threads or default_threads()
        if tiles is not None:
            f.tile_size, f.rank, f.nranks = tiles
        st = lib().rt_oracle_render(self._h, C.byref(f))
        if st != 0:
            raise RuntimeError(f"oracle render failed: {st}")
        return dict(radiance=accum_out, depth=depth, motion=motion, gbuffer=gb, closest_rays=f.closest_rays,
                    shadow_rays=f.shadow_rays, paths=f.paths)

    def close(self):
        if self._h:
            lib().rt_oracle_scene_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def skin(rest_pos, rest_nrm, jidx, jw, joints):
    """Skinning.metal:7-49 on host arrays: rest_pos/rest_nrm (n,4) f32, jidx (n,4) u16, jw (n,4) f32,
    joints (J,16) column-major."""
    rp = np.ascontiguousarray(rest_pos, np.float32)
    rn = np.ascontiguousarray(rest_nrm, np.float32)
    ji = np.ascontiguousarray(jidx, np.uint16)
    w = np.ascontiguousarray(jw, np.float32)
    J = np.ascontiguousarray(joints, np.float32)
    op = np.zeros_like(rp)
    on = np.zeros_like(rn)
    lib().rt_oracle_skin(rp.ctypes.data, rn.ctypes.data, ji.ctypes.data, w.ctypes.data, J.ctypes.data, op.ctypes.data,
                         on.ctypes.data, rp.shape[0])
    return op, on
