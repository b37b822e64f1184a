"""Texture ingest and the texture sampler's specification (SubMesh.swift:69-241,
Raytracing.metal:399-504), on the CPU:

* the library's PNG decoder (the MTKTextureLoader stand-in) against images this test encodes
  itself: every colour type, bit depths 1-16, all five row filters, Adam7 interlacing, tRNS;
  and, when the reference snapshot is present, its three PNG assets decode with their stated
  sizes;
* texture binding (textureFlags bit per slot, baseColor -> 1 for the base color map,
  SubMesh.swift:120-124) through the host scene API and through MTL map statements;
* the oracle's bilinear LOD-0 repeat sampler against a numpy restatement of the same formula.

The reference's own textures are only ever bound through USDZ materials (the OBJ assets carry no
active map_* statements), so the sampled values are "parity unpinned" against Metal's hardware
filter; the GPU tests pin the HIP path to this oracle bit for bit."""
import os
import struct
import zlib

import numpy as np
import pytest

REF_ASSETS = "/root/reference/AssetResources"


# ---------------------------------------------------------------- a small PNG encoder (test side)
def _chunk(t, body):
    return struct.pack(">I", len(body)) + t + body + struct.pack(">I", zlib.crc32(t + body) & 0xffffffff)


def _filter_rows(raw_rows, bpp, rng):
    """raw_rows: list of bytes rows; each row gets a random filter type 0-4."""
    out = bytearray()
    prev = bytes(len(raw_rows[0])) if raw_rows else b""
    for row in raw_rows:
        ft = int(rng.integers(0, 5))
        f = bytearray(len(row))
        for i in range(len(row)):
            a = row[i - bpp] if i >= bpp else 0
            b = prev[i]
            c = prev[i - bpp] if i >= bpp else 0
            if ft == 0:
                p = 0
            elif ft == 1:
                p = a
            elif ft == 2:
                p = b
            elif ft == 3:
                p = (a + b) >> 1
            else:
                pp = a + b - c
                pa, pb, pc = abs(pp - a), abs(pp - b), abs(pp - c)
                p = a if (pa <= pb and pa <= pc) else (b if pb <= pc else c)
            f[i] = (row[i] - p) & 0xff
        out += bytes([ft]) + bytes(f)
        prev = row
    return bytes(out)


def _pack_row(samples, depth):
    """samples: 1-D int array of channel samples for one row."""
    if depth == 8:
        return bytes(samples.astype(np.uint8))
    if depth == 16:
        return bytes(samples.astype(">u2").tobytes())
    bits = "".join(format(int(s), "0%db" % depth) for s in samples)
    bits += "0" * (-len(bits) % 8)
    return bytes(int(bits[i:i + 8], 2) for i in range(0, len(bits), 8))


def encode_png(samples, ctype, depth, rng, interlace=False, plte=None, trns=None):
    """samples: (H, W, C) ints in the PNG's sample range."""
    h, w, ch = samples.shape
    bpp = max(1, ch * depth // 8)
    ihdr = struct.pack(">IIBBBBB", w, h, depth, ctype, 0, 0, 1 if interlace else 0)
    if interlace:
        data = b""
        for x0, y0, dx, dy in [(0, 0, 8, 8), (4, 0, 8, 8), (0, 4, 4, 8), (2, 0, 4, 4), (0, 2, 2, 4), (1, 0, 2, 2),
                               (0, 1, 1, 2)]:
            sub = samples[y0::dy, x0::dx]
            if sub.shape[0] == 0 or sub.shape[1] == 0:
                continue
            data += _filter_rows([_pack_row(r.reshape(-1), depth) for r in sub], bpp, rng)
    else:
        data = _filter_rows([_pack_row(r.reshape(-1), depth) for r in samples], bpp, rng)
    png = b"\x89PNG\r\n\x1a\n" + _chunk(b"IHDR", ihdr)
    if plte is not None:
        png += _chunk(b"PLTE", bytes(plte.astype(np.uint8).reshape(-1)))
    if trns is not None:
        png += _chunk(b"tRNS", trns)
    png += _chunk(b"tEXt", b"Comment\x00test")   # ancillary chunk: skipped
    # split the image data over two IDAT chunks
    z = zlib.compress(data, 6)
    png += _chunk(b"IDAT", z[: len(z) // 2]) + _chunk(b"IDAT", z[len(z) // 2:]) + _chunk(b"IEND", b"")
    return png


def _to8(v, depth):
    if depth == 8:
        return v
    if depth == 16:
        return (v * 255 + 32767) // 65535
    return v * 255 // ((1 << depth) - 1)


@pytest.mark.parametrize("ctype,depth", [(0, 1), (0, 2), (0, 4), (0, 8), (0, 16), (2, 8), (2, 16), (3, 1), (3, 4),
                                         (3, 8), (4, 8), (4, 16), (6, 8), (6, 16)])
@pytest.mark.parametrize("interlace", [False, True])
def test_png_decode(rt, ctype, depth, interlace):
    rng = np.random.default_rng(ctype * 100 + depth + (7 if interlace else 0))
    h, w = 11, 13
    ch = {0: 1, 2: 3, 3: 1, 4: 2, 6: 4}[ctype]
    top = (1 << depth) - 1
    plte = trns = None
    if ctype == 3:
        n = min(top + 1, 20)
        samples = rng.integers(0, n, size=(h, w, 1))
        plte = rng.integers(0, 256, size=(n, 3))
        trns = bytes(rng.integers(0, 256, size=n // 2).astype(np.uint8))
    else:
        samples = rng.integers(0, top + 1, size=(h, w, ch))
    png = encode_png(samples, ctype, depth, rng, interlace, plte, trns)
    out = rt.decode_png(png)
    assert out.shape == (h, w, 4) and out.dtype == np.uint8
    if ctype == 3:
        idx = samples[..., 0]
        exp = np.zeros((h, w, 4), np.int64)
        exp[..., :3] = plte[idx]
        alpha = np.full(len(plte), 255)
        alpha[: len(trns)] = np.frombuffer(trns, np.uint8)
        exp[..., 3] = alpha[idx]
    else:
        s8 = _to8(samples.astype(np.int64), depth)
        exp = np.zeros((h, w, 4), np.int64)
        if ctype in (0, 4):
            exp[..., :3] = s8[..., :1]
            exp[..., 3] = s8[..., 1] if ctype == 4 else 255
        elif ctype == 2:
            exp[..., :3] = s8
            exp[..., 3] = 255
        else:
            exp[...] = s8
    assert np.array_equal(out, exp)


def test_png_transparency_key_and_errors(rt):
    rng = np.random.default_rng(3)
    samples = rng.integers(0, 4, size=(5, 6, 3)) * 60
    key = samples[2, 3]
    png = encode_png(samples, 2, 8, rng, trns=struct.pack(">HHH", *[int(k) for k in key]))
    out = rt.decode_png(png)
    hit = np.all(samples == key, axis=2)
    assert np.all(out[hit, 3] == 0) and np.all(out[~hit, 3] == 255)
    with pytest.raises(rt.RTError):
        rt.decode_png(b"not a png at all")
    bad = bytearray(png)
    bad[40] ^= 0xff   # corrupt a chunk: CRC mismatch
    with pytest.raises(rt.RTError):
        rt.decode_png(bytes(bad))


@pytest.mark.skipif(not os.path.isdir(REF_ASSETS), reason="reference snapshot absent")
@pytest.mark.parametrize("name,size", [("uv_test/uv_test.png", (1024, 1024)), ("coatball/tex_metallic.png", (4096, 4096)),
                                       ("coatball/tex_ao.png", (4096, 4096))])
def test_reference_pngs_decode(rt, name, size):
    with open(os.path.join(REF_ASSETS, name), "rb") as f:
        img = rt.decode_png(f.read())
    assert img.shape[:2] == size
    assert img.std() > 0   # not a blank image


# ---------------------------------------------------------------- binding + sampler spec
def _checker(h, w, seed):
    rng = np.random.default_rng(seed)
    return rng.integers(0, 256, size=(h, w, 4), dtype=np.uint8)


def test_bind_texture_flags(rt, assets):
    sc = rt.Scene.preset("c1", assets)
    d0 = sc.desc()
    tid = sc.add_texture(_checker(4, 6, 1))
    nid = sc.add_texture(_checker(3, 3, 2))
    sc.bind_texture(0, 0, "baseColor", tid)
    sc.bind_texture(0, 0, "normal", nid)
    sc.bind_texture(1, 0, "metallic", tid)
    d = sc.desc()
    assert d.texture_count == 2
    assert (d.textures[0].width, d.textures[0].height) == (6, 4)
    m0 = d.meshes[0].submeshes[0]
    assert m0.material.textureFlags == 0b11
    assert (m0.material.baseColor.x, m0.material.baseColor.y, m0.material.baseColor.z) == (1.0, 1.0, 1.0)
    assert m0.textures[0] == tid and m0.textures[1] == nid
    m1 = d.meshes[1].submeshes[0]
    assert m1.material.textureFlags == 0b1000 and m1.textures[3] == tid
    # metallic map leaves baseColor alone
    assert m1.material.baseColor.x == d0.meshes[1].submeshes[0].material.baseColor.x
    with pytest.raises(rt.RTError):
        sc.bind_texture(0, 0, 7, tid)
    with pytest.raises(rt.RTError):
        sc.bind_texture(0, 0, "baseColor", 99)
    with pytest.raises(rt.RTError):
        sc.bind_texture(99, 0, "baseColor", tid)


def test_mtl_maps_bind(rt, tmp_path):
    rng = np.random.default_rng(5)
    (tmp_path / "tex").mkdir()
    img = rng.integers(0, 256, size=(8, 8, 3))
    (tmp_path / "tex" / "base.png").write_bytes(encode_png(img, 2, 8, rng))
    (tmp_path / "rough.png").write_bytes(encode_png(img[..., :1], 0, 8, rng))
    (tmp_path / "m.mtl").write_text("newmtl A\nKd 0.5 0.5 0.5\nmap_Kd -bm 1.0 tex/base.png\nmap_Pr rough.png\n"
                                    "map_Pm missing.png\n")
    (tmp_path / "q.obj").write_text("mtllib m.mtl\nv 0 0 0\nv 1 0 0\nv 1 1 0\nvt 0 0\nvt 1 0\nvt 1 1\nvn 0 0 1\n"
                                    "usemtl A\nf 1/1/1 2/2/1 3/3/1\n")
    sc = rt.Scene()
    sc.add_model(str(tmp_path / "q.obj"), (0, 0, 0))
    d = sc.desc()
    sm = d.meshes[0].submeshes[0]
    # base color + roughness bound, the missing metallic map stays unbound (SubMesh.swift:100-107)
    assert sm.material.textureFlags == 0b101
    assert sm.material.baseColor.x == 1.0
    assert d.texture_count == 2
    t = d.textures[sm.textures[0]]
    got = np.ctypeslib.as_array(rt.C.cast(t.rgba8, rt.C.POINTER(rt.C.c_uint8)), shape=(8, 8, 4))
    assert np.array_equal(got[..., :3], img) and np.all(got[..., 3] == 255)


def _np_srgb_lut():
    v = np.arange(256, dtype=np.float64) / 255.0
    lin = v.astype(np.float32)
    srgb = np.where(v <= 0.04045, v / 12.92, ((v + 0.055) / 1.055) ** 2.4).astype(np.float32)
    return lin, srgb


def _np_sample(img, u, v, srgb):
    """The sampler specification in numpy float32, same operation order as the oracle."""
    lin, sl = _np_srgb_lut()
    h, w = img.shape[:2]
    f = np.float32
    x = f(u) * f(w) - f(0.5)
    y = f(v) * f(h) - f(0.5)
    x = x if abs(x) < 1e9 else f(0)
    y = y if abs(y) < 1e9 else f(0)
    fx, fy = np.floor(x), np.floor(y)
    ax, ay = f(x - fx), f(y - fy)
    bx, by = f(f(1) - ax), f(f(1) - ay)
    x0, y0 = int(fx) % w, int(fy) % h
    x1, y1 = (x0 + 1) % w, (y0 + 1) % h
    out = np.zeros(4, np.float32)
    for c in range(4):
        L = sl if (srgb and c < 3) else lin
        c00, c10, c01, c11 = (L[img[y0, x0, c]], L[img[y0, x1, c]], L[img[y1, x0, c]], L[img[y1, x1, c]])
        out[c] = f(f(f(c00 * bx) + f(c10 * ax)) * by) + f(f(f(c01 * bx) + f(c11 * ax)) * ay)
    return out


def test_oracle_sampler_spec(rt, orc, assets):
    sc = rt.Scene.preset("c1", assets)
    imgs = [_checker(5, 7, 11), _checker(1, 1, 12), _checker(16, 3, 13)]
    ids = [sc.add_texture(im) for im in imgs]
    desc = sc.desc()
    o = orc.OracleScene(desc)
    rng = np.random.default_rng(0)
    uvs = list(rng.uniform(-3.0, 4.0, size=(200, 2))) + [(0.0, 0.0), (1.0, 1.0), (0.5 / 7, 0.5 / 5), (-1e-7, 1.0),
                                                          (float("nan"), 0.25), (1e12, -1e12)]
    for tid, im in zip(ids, imgs):
        for (u, v) in uvs:
            for srgb in (False, True):
                exp = _np_sample(im, np.float32(u), np.float32(v), srgb)
                got = o.tex_sample(tid, float(np.float32(u)), float(np.float32(v)), srgb)
                assert np.array_equal(got, exp), (tid, u, v, srgb, got, exp)
    # a texel centre returns the texel exactly (linear)
    im = imgs[0]
    got = o.tex_sample(ids[0], (2 + 0.5) / 7, (3 + 0.5) / 5, False)
    assert np.array_equal(got, (im[3, 2] / np.float32(255)).astype(np.float32))


def test_write_png_roundtrip(rt, tmp_path):
    img = _checker(9, 17, 21)
    p = tmp_path / "o.png"
    rt.write_png(p, img)
    assert np.array_equal(rt.decode_png(p.read_bytes()), img)
