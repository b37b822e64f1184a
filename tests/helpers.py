"""Shared helpers for the parity tests (tolerances and comparison)."""
import os
import numpy as np

# North-star parity bar (BASELINE.json): per-pixel relative L2 of RGB radiance <= 1e-4.
REL_L2_TOL = 1e-4


def rel_l2_per_pixel(a, b):
    """Per-pixel ||a-b|| / max(||b||, 1e-6) over RGB."""
    a = np.asarray(a, np.float64)[..., :3]
    b = np.asarray(b, np.float64)[..., :3]
    num = np.linalg.norm(a - b, axis=-1)
    den = np.maximum(np.linalg.norm(b, axis=-1), 1e-6)
    return num / den


def parity_report(gpu, ref):
    e = rel_l2_per_pixel(gpu, ref)
    exact = np.mean(np.all(np.asarray(gpu)[..., :3] == np.asarray(ref)[..., :3], axis=-1))
    return dict(max_rel=float(e.max()), n_bad=int((e > REL_L2_TOL).sum()), frac_bitwise=float(exact))


# Pipeline variants of the GPU tests: the per-pixel megakernel, and the wavefront pipeline with
# the default finish threshold (small frames run almost entirely in the persistent finish
# kernel), with no finish kernel at all (every bounce through extend / shade / connect) and
# with a small threshold (bulk rounds, then finish).  "wavefront-bulk-sort" and the mixed variant
# also sort hits by BVH leaf bin between extend and shade (off by default).
PIPELINES = ["megakernel", "wavefront", "wavefront-bulk", "wavefront-mixed", "wavefront-bulk-sort"]
_VARIANTS = {"megakernel": ("megakernel", 0, 0), "wavefront": ("wavefront", 0, 0),
             "wavefront-bulk": ("wavefront", 1, 0), "wavefront-mixed": ("wavefront", 2048, 4096),
             "wavefront-bulk-sort": ("wavefront", 1, 2048)}


def make_renderer(rt, scene, W, H, pipeline="wavefront", **kw):
    """A Renderer of the given test pipeline variant.  The legacy RT_* variables of the test's own
    environment (the env-variant tests' child processes set them) are applied through rt_set_tuning /
    rt_set_graphs: the library reads no environment."""
    pl, tail, sort_bins = _VARIANTS[pipeline]
    env = rt.tuning_from_env()
    graphs = env.pop("graphs", None)
    env_tail = env.pop("tail_paths", None)
    fif = env.pop("frames_in_flight", None)
    if fif is not None:
        kw.setdefault("frames_in_flight", fif)
    R = rt.Renderer(scene, W, H, pipeline=pl, tail_paths=tail or env_tail or 0, sort_bins=sort_bins, tuning=env, **kw)
    if graphs is not None:
        R.set_graphs(bool(graphs))
    return R


# ---- the textured test scene (tests/test_gpu_textures.py, tests/golden tex case) -------------------
def procedural_textures(seed=1):
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:64, 0:64]
    base = np.zeros((64, 64, 4), np.uint8)
    chk = ((xx // 8 + yy // 8) % 2).astype(np.uint8)
    base[..., 0] = 40 + 200 * chk
    base[..., 1] = rng.integers(30, 220, size=(64, 64))
    base[..., 2] = 255 - 180 * chk
    base[..., 3] = 255
    # bumps: tangent-space normals from a height field
    hx = np.cos(xx / 64.0 * 2 * np.pi * 3) * 0.6
    hy = np.sin(yy / 64.0 * 2 * np.pi * 2) * 0.6
    n = np.stack([hx, hy, np.ones_like(hx)], axis=-1)
    n /= np.linalg.norm(n, axis=-1, keepdims=True)
    normal = np.concatenate([((n * 0.5 + 0.5) * 255).round().astype(np.uint8), np.full((64, 64, 1), 255, np.uint8)],
                            axis=-1)
    rough = np.repeat(((xx * 4) % 256).astype(np.uint8)[..., None], 4, axis=-1)
    metal = np.repeat((255 * ((yy // 4) % 2)).astype(np.uint8)[..., None], 4, axis=-1)
    emis = np.zeros((32, 32, 4), np.uint8)
    emis[::5, ::7, :3] = rng.integers(100, 256, size=emis[::5, ::7, :3].shape)
    emis[..., 3] = 255
    opac = np.full((16, 16, 4), 255, np.uint8)
    opac[4:12, 4:12, 0] = 40
    return dict(base=base, normal=normal, rough=rough, metal=metal, emis=emis, opac=opac)


def textured_scene(rt, assets):
    """c1 (floor with UVs, two spheres without, back wall) + the train (UVs, 6 submeshes)."""
    sc = rt.Scene.preset("c1", assets)
    sc.add_model(os.path.join(assets, "train.obj"), (-0.3, 0.0, 0.4), scale=0.5)
    T = {k: sc.add_texture(v) for k, v in procedural_textures().items()}
    sc.bind_texture(0, 0, "baseColor", T["base"])        # floor
    sc.bind_texture(0, 0, "roughness", T["rough"])
    sc.bind_texture(0, 0, "normal", T["normal"])
    sc.bind_texture(1, 0, "baseColor", T["base"])        # sphere without UVs: samples (0, 1)
    sc.bind_texture(1, 0, "metallic", T["metal"])
    sc.bind_texture(4, 0, "normal", T["normal"])         # train submeshes
    sc.bind_texture(4, 0, "metallic", T["metal"])
    sc.bind_texture(4, 1, "emission", T["emis"])
    sc.bind_texture(4, 2, "opacity", T["opac"])
    sc.bind_texture(4, 3, "roughness", T["rough"])
    sc.bind_texture(4, 4, "baseColor", T["base"])
    sc.bind_texture(4, 5, "baseColor", T["base"])
    sc.bind_texture(4, 5, "normal", T["normal"])
    sc.bind_texture(4, 5, "ao", T["rough"])              # AO: bound, never sampled (ENABLE_AO 0)
    return sc


# ---- light types (Scene.swift:161-208): the reference's factories, with the values Scene.init uses
# or has commented out (Scene.swift:82-90): area light1 and light2, spot light3, sunLight, pointLight
LIGHT_TYPES = {"sun": 1, "spot": 2, "point": 3, "area": 4}


def make_light(rt, kind):
    L = rt.Light()
    f3 = rt.f3
    if kind == "area":            # Scene.setupLight (light1)
        L.type, L.position, L.forward = 4, f3(0.0, 1.98, 0.0), f3(0.0, -1.0, 0.0)
        L.right, L.up, L.color = f3(0.25, 0.0, 0.0), f3(0.0, 0.0, 0.25), f3(4.0, 4.0, 4.0)
    elif kind == "area2":         # light2 (built, unused by the reference scene)
        L.type, L.position, L.forward = 4, f3(2.0, 1.98, 3.0), f3(0.0, -0.5, 0.0)
        L.right, L.up, L.color = f3(0.1, 0.0, 0.0), f3(0.0, 0.0, 0.1), f3(4.0, 4.0, 4.0)
    elif kind == "spot":          # light3
        L.type, L.position, L.direction = 2, f3(2.0, 1.0, 4.0), f3(-1.5, -0.5, -1.5)
        L.coneAngle, L.color = 25.0 / 180.0 * 3.14159265358979323846, f3(4.0, 4.0, 4.0)
    elif kind == "sun":           # Light.sunLight(direction: [-1, -2, 0], color: [1, 1, 1])
        L.type, L.direction, L.color = 1, f3(-1.0, -2.0, 0.0), f3(1.0, 1.0, 1.0)
    elif kind == "point":         # Light.pointLight(position: [1, 1, 1], color: [1, 1, 1])
        L.type, L.position, L.color = 3, f3(1.0, 1.0, 1.0), f3(1.0, 1.0, 1.0)
    else:
        raise ValueError(kind)
    return L


def lights_scene(rt, assets, kinds):
    """The c1 scene lit by the given lights (lightCount = len(kinds), Raytracing.metal:588-647)."""
    sc = rt.Scene.preset("c1", assets)
    sc.set_lights([make_light(rt, k) for k in kinds])
    return sc


# ---- a triangle soup: closest-hit order against triangle ids (tests/test_gpu_parity.py) -----------
def write_triangle_soup(path, n=4000, seed=5):
    """An OBJ of n random, overlapping, roughly camera-facing triangles in a thin slab: BVH leaves
    hold several triangles a ray crosses, in slot orders and with ids unrelated to their depth, so
    a closest-hit search that accepted a triangle beyond a closer hit already found whenever its id
    is smaller (round 4's second-triangle bound) keeps a farther one."""
    import os
    rng = np.random.default_rng(seed)
    c = rng.uniform([-0.5, -0.5, -0.15], [0.5, 0.5, 0.15], size=(n, 3))
    off = rng.normal(size=(n, 3, 3)) * np.array([0.08, 0.08, 0.02])
    v = (c[:, None, :] + off).reshape(-1, 3)
    with open(path, "w") as fh:
        fh.write("mtllib soup.mtl\nusemtl None\n")
        fh.writelines("v %.6f %.6f %.6f\n" % tuple(p) for p in v)
        fh.writelines("f %d %d %d\n" % (3 * k + 1, 3 * k + 2, 3 * k + 3) for k in range(n))
    with open(os.path.join(os.path.dirname(path), "soup.mtl"), "w") as fh:
        fh.write("newmtl None\nKd 0.6 0.7 0.5\nd 1\n")


def write_tie_scene(path, n=600, grid=24, seed=7):
    """An OBJ whose closest hits tie exactly (equal t -> the smaller triangle id).
    Part 1: n random triangles in a thin slab, written three times over the SAME vertex indices:
    first under material Red, then Blue, then Green with the vertex order rotated (v1, v2, v0).
    The Red and Blue copies are bit-identical world-space triangles (every ray hits both at the same
    t, u, v), so only the id tie-break decides which material a hit shades -- the Red copy, whose
    ids are smaller; a traversal (or a team member's merge) that lets the later copy win shows
    blue.  The rotated Green copy ties up to the last bit of t.  Part 2: a grid x grid quad mesh
    (two triangles per quad, shared edges and vertices) in front of the slab, for hits on shared
    edges."""
    import os
    rng = np.random.default_rng(seed)
    c = rng.uniform([-0.5, -0.5, -0.1], [0.5, 0.5, 0.1], size=(n, 3))
    off = rng.normal(size=(n, 3, 3)) * np.array([0.07, 0.07, 0.02])
    v = (c[:, None, :] + off).reshape(-1, 3)
    lines = ["mtllib ties.mtl\n"]
    lines += ["v %.6f %.6f %.6f\n" % tuple(p) for p in v]
    for mat, rot in (("Red", False), ("Blue", False), ("Green", True)):
        lines.append("usemtl %s\n" % mat)
        for k in range(n):
            a, b, cc = 3 * k + 1, 3 * k + 2, 3 * k + 3
            lines.append("f %d %d %d\n" % ((b, cc, a) if rot else (a, b, cc)))
    base = 3 * n
    xs, ys = np.linspace(-0.6, 0.0, grid + 1), np.linspace(-0.6, 0.6, grid + 1)   # the left half
    for y in ys:
        for x in xs:
            lines.append("v %.6f %.6f %.6f\n" % (x, y, 0.25 + 0.05 * x))
    lines.append("usemtl Grid\n")
    for j in range(grid):
        for i in range(grid):
            p00 = base + j * (grid + 1) + i + 1
            p10, p01, p11 = p00 + 1, p00 + grid + 1, p00 + grid + 2
            if (i + j) % 3 == 0:
                continue   # holes: rays reach the slab behind
            lines.append("f %d %d %d\n" % (p00, p10, p11))
            lines.append("f %d %d %d\n" % (p00, p11, p01))
    with open(path, "w") as fh:
        fh.writelines(lines)
    with open(os.path.join(os.path.dirname(path), "ties.mtl"), "w") as fh:
        fh.write("newmtl Red\nKd 0.9 0.15 0.1\nd 1\nnewmtl Blue\nKd 0.1 0.2 0.9\nd 1\n"
                 "newmtl Green\nKd 0.1 0.8 0.2\nd 1\nnewmtl Grid\nKd 0.7 0.7 0.7\nd 1\n")


def traversal_scene(rt, assets, kind, tmpdir):
    """The C1 room with the triangle soup ('soup') or the exact-tie scene ('ties') in front."""
    import os
    scene = rt.Scene.preset("c1", assets)
    if kind == "soup":
        write_triangle_soup(os.path.join(tmpdir, "soup.obj"))
        scene.add_model(os.path.join(tmpdir, "soup.obj"), (0.0, 1.0, 0.0), scale=3.0)
    else:
        write_tie_scene(os.path.join(tmpdir, "ties.obj"))
        scene.add_model(os.path.join(tmpdir, "ties.obj"), (0.0, 1.0, 0.5), rotation=(0.0, 0.3, 0.0), scale=3.0)
    return scene
