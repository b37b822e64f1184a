"""GPU parity of the display output (FramePresenter.swift:103-238,
Shaders.metal:39-52): rt_present resamples the newest radiance (nearest / bilinear / temporal
reprojection through the motion vectors and depth), tone-maps color / (1 + color) and encodes
8-bit sRGB or linear rows top-down.  The kernel is byte work on float inputs with a fixed
operation order, so a numpy float32 restatement (below) reproduces its bytes exactly; the
radiance, depth and motion it reads are the library's own (pinned elsewhere against the oracle).
MetalFX's scalers are unpublished, so the spatial / temporal / denoised modes are parity unpinned
against the reference and pinned here against this restatement; the denoised mode is also checked
to bring a 1-spp frame closer to a converged one."""
import os

import numpy as np
import pytest

from helpers import make_renderer

pytestmark = pytest.mark.gpu
f32 = np.float32


def _thresholds():
    s = (np.arange(255, dtype=np.float64) + 0.5) / 255.0
    return np.where(s <= 0.04045, s / 12.92, ((s + 0.055) / 1.055) ** 2.4).astype(np.float32)


def _encode(c, srgb):
    with np.errstate(invalid="ignore", divide="ignore"):
        v = np.where(c > 0, c / (f32(1) + c), f32(0)).astype(np.float32)
    if srgb:
        return np.searchsorted(_thresholds(), v, side="right").astype(np.uint8)
    return np.minimum(np.floor(v * f32(255) + f32(0.5)), f32(255)).astype(np.uint8)


def _clamped(img, x, y):
    h, w = img.shape[:2]
    return img[np.clip(y, 0, h - 1), np.clip(x, 0, w - 1)]


def _bilinear(img, x, y):
    fx, fy = np.floor(x), np.floor(y)
    ax, ay = (x - fx).astype(f32), (y - fy).astype(f32)
    bx, by = f32(1) - ax, f32(1) - ay
    x0 = np.clip(fx, -2, img.shape[1] + 2).astype(np.int64)
    y0 = np.clip(fy, -2, img.shape[0] + 2).astype(np.int64)
    c00, c10 = _clamped(img, x0, y0), _clamped(img, x0 + 1, y0)
    c01, c11 = _clamped(img, x0, y0 + 1), _clamped(img, x0 + 1, y0 + 1)
    ax, ay, bx, by = ax[..., None], ay[..., None], bx[..., None], by[..., None]
    return (c00 * bx + c10 * ax) * by + (c01 * bx + c11 * ax) * ay


def present_np(acc, depth, motion, ow, oh, scaler, srgb, hist=None, hdepth=None, use_hist=False):
    """Returns (display rows top-down uint8 (oh, ow, 4), new history, new history depth); arrays in
    render row order (row 0 = bottom) like the library's targets."""
    h, w = acc.shape[:2]
    oy, ox = np.meshgrid(np.arange(oh), np.arange(ow), indexing="ij")   # render-order output rows
    oxf, oyf = ox.astype(f32), oy.astype(f32)
    nh = nd = None
    if scaler == "none":
        tx = np.minimum((((oxf + f32(0.5)) / f32(ow)) * f32(w)).astype(np.int64), w - 1)
        ty = np.minimum((((oyf + f32(0.5)) / f32(oh)) * f32(h)).astype(np.int64), h - 1)
        c = acc[ty, tx]
    else:
        sx, sy = f32(w) / f32(ow), f32(h) / f32(oh)
        px = (oxf + f32(0.5)) * sx - f32(0.5)
        py = (oyf + f32(0.5)) * sy - f32(0.5)
        c = _bilinear(acc, px, py).astype(f32)
        if scaler == "temporal":
            nx = np.clip(np.floor(px + f32(0.5)).astype(np.int64), 0, w - 1)
            ny = np.clip(np.floor(py + f32(0.5)).astype(np.int64), 0, h - 1)
            mn = acc[ny, nx][..., :3].copy()
            mx = mn.copy()
            for dy in (-1, 0, 1):
                for dx in (-1, 0, 1):
                    q = _clamped(acc, nx + dx, ny + dy)[..., :3]
                    mn, mx = np.minimum(mn, q), np.maximum(mx, q)
            m = motion[ny, nx]
            d = depth[ny, nx]
            qx, qy = px - m[..., 0], py + m[..., 1]
            hx = (qx + f32(0.5)) / sx - f32(0.5)
            hy = (qy + f32(0.5)) / sy - f32(0.5)
            ok = use_hist & (qx >= f32(-0.5)) & (qx <= f32(w) - f32(0.5)) & (qy >= f32(-0.5)) & (qy <= f32(h) - f32(0.5))
            with np.errstate(invalid="ignore"):
                hnx = np.clip(np.nan_to_num(np.floor(hx + f32(0.5)), nan=0, posinf=ow, neginf=-1), 0, ow - 1).astype(np.int64)
                hny = np.clip(np.nan_to_num(np.floor(hy + f32(0.5)), nan=0, posinf=oh, neginf=-1), 0, oh - 1).astype(np.int64)
            if use_hist:
                hd = hdepth[hny, hnx]
                ok = ok & (np.abs(hd - d) <= f32(0.1) * np.maximum(d, hd))
                hv = _bilinear(hist, np.nan_to_num(hx), np.nan_to_num(hy)).astype(f32)[..., :3]
                hv = np.minimum(np.maximum(hv, mn), mx)
                blend = hv + (c[..., :3] - hv) * f32(0.1)
                c = c.copy()
                c[..., :3] = np.where(ok[..., None], blend, c[..., :3])
            nh = np.concatenate([c[..., :3], np.ones(c.shape[:2] + (1,), f32)], axis=-1).astype(f32)
            nd = d.astype(f32)
    out = np.empty((oh, ow, 4), np.uint8)
    out[..., :3] = _encode(c[..., :3].astype(f32), srgb)
    out[..., 3] = 255
    return out[::-1], nh, nd


def denoise_np(acc, depth, gb, passes=3):
    """RT_SCALER_DENOISED's render-size filter (rt_present.hip denoise_prep_k / denoise_atrous_k):
    demodulate by diffuse + specular albedo, `passes` a-trous passes weighted by the B3 spline,
    max(0, n.n')^16 and 1 / (1 + (dz / (0.05 step z))^2), background only with background,
    remodulate.  Same operation order as the kernels."""
    h, w = acc.shape[:2]
    hit = gb[2][..., 3] > f32(0.5)
    a = gb[0][..., :3] + gb[1][..., :3]
    a = np.where(hit[..., None] & (a > f32(1e-3)), a, f32(1)).astype(f32)
    src = acc.astype(f32).copy()
    src[..., :3] = acc[..., :3] / a
    guide = np.zeros((h, w, 4), f32)
    guide[..., 3] = -1
    guide[hit, :3] = gb[2][hit, :3] * f32(2) - f32(1)
    guide[hit, 3] = depth[hit]
    kern = np.array([0.0625, 0.25, 0.375, 0.25, 0.0625], f32)
    ys, xs = np.meshgrid(np.arange(h), np.arange(w), indexing="ij")
    p = guide
    pb = p[..., 3] < 0
    for k in range(passes):
        step = 1 << k
        zs = f32(0.05) * f32(step) * p[..., 3]
        s = np.zeros((h, w, 3), f32)
        sw = np.zeros((h, w), f32)
        for dy in range(-2, 3):
            for dx in range(-2, 3):
                yy, xx = ys + dy * step, xs + dx * step
                inb = (yy >= 0) & (yy < h) & (xx >= 0) & (xx < w)
                yc, xc = np.clip(yy, 0, h - 1), np.clip(xx, 0, w - 1)
                q = guide[yc, xc]
                qb = q[..., 3] < 0
                w0 = kern[dy + 2] * kern[dx + 2]
                t = np.maximum(p[..., 0] * q[..., 0] + p[..., 1] * q[..., 1] + p[..., 2] * q[..., 2], f32(0))
                t = t * t
                t = t * t
                t = t * t
                t = t * t
                with np.errstate(invalid="ignore", divide="ignore", over="ignore"):
                    dz = np.abs(p[..., 3] - q[..., 3]) / zs
                    wv = (w0 * t) / (f32(1) + dz * dz)
                wgt = np.where(pb | qb, w0, wv).astype(f32)
                use = inb & ~(pb ^ qb)
                c = src[yc, xc][..., :3]
                s = np.where(use[..., None], s + c * wgt[..., None], s)
                sw = np.where(use, sw + wgt, sw)
        r = src.copy()
        with np.errstate(invalid="ignore", divide="ignore"):
            r[..., :3] = np.where((sw > 0)[..., None], s / sw[..., None], src[..., :3])
        if k == passes - 1:
            r[..., :3] = r[..., :3] * a
        src = r
    return src


def _renderer(rt, assets, fif=2):
    sc = rt.Scene.preset("c1", assets)
    R = make_renderer(rt, sc, 80, 56, "wavefront", seed=4, frames_in_flight=fif)
    R.samplesPerPixel = 2
    R.maxBounces = 3
    return R


@pytest.mark.parametrize("scaler,size", [("none", (80, 56)), ("none", (120, 90)), ("spatial", (120, 90)),
                                         ("spatial", (53, 37)), ("spatial", (80, 56))])
@pytest.mark.parametrize("srgb", [True, False])
def test_present_matches_restatement(rt, assets, scaler, size, srgb):
    R = _renderer(rt, assets)
    R.draw()
    R.draw()
    got = R.present(size[0], size[1], scaler=scaler, srgb=srgb)
    acc = R.radiance()
    depth, motion, _ = R.aux()
    exp, _, _ = present_np(acc, depth, motion, size[0], size[1], scaler, srgb)
    assert got.shape == (size[1], size[0], 4)
    assert np.array_equal(got, exp), np.argwhere(got != exp)[:5]
    assert len(np.unique(got[..., :3].reshape(-1, 3), axis=0)) > 20


def test_present_temporal_sequence(rt, assets, tmp_path):
    """Five moving-camera frames through the temporal scaler (history, reprojection, clamp,
    depth rejection); every frame's bytes match the restatement; the last is written as PNG."""
    R = _renderer(rt, assets)
    cam0 = R.camera
    ow, oh = 120, 84
    hist = hdepth = None
    for i in range(5):
        c = rt.Camera()
        c.position = type(cam0.position)(cam0.position.x + 0.03 * i, cam0.position.y, cam0.position.z, 0.0)
        c.right, c.up, c.forward = cam0.right, cam0.up, cam0.forward
        R.camera = c
        u = R.draw()
        got = R.present(ow, oh, scaler="temporal")
        acc = R.radiance()
        depth, motion, _ = R.aux()
        use = hist is not None and u.frameIndex > 0
        exp, hist, hdepth = present_np(acc, depth, motion, ow, oh, "temporal", True, hist, hdepth, use)
        assert np.array_equal(got, exp), (i, np.argwhere(got != exp)[:5])
    assert np.abs(motion).max() > 0
    p = os.path.join(tmp_path, "frame.png")
    rt.write_png(p, got)
    with open(p, "rb") as f:
        assert np.array_equal(rt.decode_png(f.read()), got)


def test_present_orientation(rt, assets):
    """Display rows run top-down: the first output row is the last render row (the presenter's
    quad maps texture v = 0 to the bottom of the screen)."""
    R = _renderer(rt, assets, fif=1)
    R.draw()
    got = R.present(scaler="none", srgb=False)
    acc = R.radiance()
    assert np.array_equal(got[0, :, :3], _encode(acc[-1, :, :3], False))
    assert np.array_equal(got[-1, :, :3], _encode(acc[0, :, :3], False))


@pytest.mark.parametrize("passes", [1, 3, 5])
def test_present_denoised_sequence(rt, assets, passes):
    """RT_SCALER_DENOISED over four moving-camera frames (G-buffer on): the G-buffer-guided filter
    and the temporal history match the restatement byte for byte, at a resampled output size."""
    R = _renderer(rt, assets)
    R.useTemporalDenoiser = True
    cam0 = R.camera
    ow, oh = (80, 56) if passes == 3 else (100, 70)
    hist = hdepth = None
    for i in range(4):
        c = rt.Camera()
        c.position = type(cam0.position)(cam0.position.x - 0.02 * i, cam0.position.y, cam0.position.z, 0.0)
        c.right, c.up, c.forward = cam0.right, cam0.up, cam0.forward
        R.camera = c
        u = R.draw()
        got = R.present(ow, oh, scaler="denoised", denoise_passes=passes)
        acc = R.radiance()
        depth, motion, gb = R.aux(gbuffer=True)
        den = denoise_np(acc, depth, gb, passes)
        use = hist is not None and u.frameIndex > 0
        exp, hist, hdepth = present_np(den, depth, motion, ow, oh, "temporal", True, hist, hdepth, use)
        assert np.array_equal(got, exp), (i, np.argwhere(got != exp)[:5])


def test_present_denoised_needs_gbuffer(rt, assets):
    R = _renderer(rt, assets)
    R.draw()
    with pytest.raises(RuntimeError, match="G-buffer"):
        R.present(scaler="denoised")
    R.useTemporalDenoiser = True
    R.draw()
    with pytest.raises(RuntimeError):
        R.present(scaler="denoised", denoise_passes=7)
    assert R.present(scaler="denoised").shape == (56, 80, 4)


def test_present_denoised_reduces_noise(rt, assets):
    """One 1-spp frame: the denoised display is closer to a 64-spp frame's than the raw one."""
    R = _renderer(rt, assets)
    R.useTemporalDenoiser = True
    R.samplesPerPixel = 1
    R.draw()
    raw = R.present(scaler="none", srgb=False).astype(np.float64)
    den = R.present(scaler="denoised", srgb=False).astype(np.float64)
    Q = _renderer(rt, assets)
    Q.samplesPerPixel = 64
    Q.draw()
    ref = Q.present(scaler="none", srgb=False).astype(np.float64)
    e_raw = np.abs(raw - ref)[..., :3].mean()
    e_den = np.abs(den - ref)[..., :3].mean()
    assert e_den < 0.7 * e_raw, (e_den, e_raw)
