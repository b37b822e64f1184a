/*
 * rtbench.c — the C host driver over the C-ABI (SURVEY.md §8b "callers": the shape of
 * Renderer.draw, Renderer.swift:1405-1503, without Swift/Metal).  Plain C11, links
 * metal4-raytracing_amd/librt_hip.so; no torch, no Python.
 *
 *   rtbench [--scene c3g] [--width 1920] [--height 1080] [--spp 4] [--bounces 8] [--frames 16]
 *           [--warmup 2] [--assets DIR] [--png out.png] [--scaler none|spatial|temporal]
 *           [--frames-in-flight N] [--megakernel]
 *
 * Renders `warmup` + `frames` frames back to back (frames in flight), waits once, and prints
 * one line: Grays/s over the timed frames (closest-hit + shadow rays from the library's running
 * totals / host wall time), ms per frame, and the device time of the newest frame.  With --png
 * the newest frame is presented (tone-mapped, sRGB) and written as a PNG.
 */
#define _POSIX_C_SOURCE 199309L
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "rt_api.h"
#include "rt_scene.h"

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

static int check(rt_status st, rt_ctx* ctx, const char* what) {
    if (st != RT_OK) {
        fprintf(stderr, "rtbench: %s failed (%d): %s\n", what, (int)st, rt_last_error(ctx));
        return 1;
    }
    return 0;
}

static void usage(void) {
    fprintf(stderr,
            "usage: rtbench [--scene c3g] [--width W] [--height H] [--spp N] [--bounces N] [--frames N]\n"
            "               [--warmup N] [--assets DIR] [--png FILE] [--scaler none|spatial|temporal]\n"
            "               [--frames-in-flight N] [--megakernel]\n");
}

int main(int argc, char** argv) {
    const char* scene_name = "c3g";
    const char* assets = "assets";
    const char* png = NULL;
    int W = 1920, H = 1080, spp = 4, bounces = 8, frames = 16, warmup = 2, fif = 0, scaler = RT_SCALER_NONE;
    int pipeline = RT_PIPELINE_WAVEFRONT;
    for (int i = 1; i < argc; ++i) {
        const char* a = argv[i];
        const char* v = i + 1 < argc ? argv[i + 1] : NULL;
        if (!strcmp(a, "--help") || !strcmp(a, "-h")) {
            usage();
            return 0;
        } else if (!strcmp(a, "--megakernel")) {
            pipeline = RT_PIPELINE_MEGAKERNEL;
            continue;
        }
        if (!v) {
            usage();
            return 2;
        }
        ++i;
        if (!strcmp(a, "--scene")) scene_name = v;
        else if (!strcmp(a, "--width")) W = atoi(v);
        else if (!strcmp(a, "--height")) H = atoi(v);
        else if (!strcmp(a, "--spp")) spp = atoi(v);
        else if (!strcmp(a, "--bounces")) bounces = atoi(v);
        else if (!strcmp(a, "--frames")) frames = atoi(v);
        else if (!strcmp(a, "--warmup")) warmup = atoi(v);
        else if (!strcmp(a, "--assets")) assets = v;
        else if (!strcmp(a, "--png")) png = v;
        else if (!strcmp(a, "--frames-in-flight")) fif = atoi(v);
        else if (!strcmp(a, "--scaler")) {
            scaler = !strcmp(v, "spatial") ? RT_SCALER_SPATIAL : !strcmp(v, "temporal") ? RT_SCALER_TEMPORAL : RT_SCALER_NONE;
        } else {
            usage();
            return 2;
        }
    }
    if (W <= 0 || H <= 0 || frames <= 0 || warmup < 0) {
        usage();
        return 2;
    }

    /* Scene.init / AppScene / Model.init (Scene.swift:73-169, AppScene.swift:11-28) */
    rt_scene* scene = NULL;
    int32_t synthetic = 0;
    if (rt_scene_preset(scene_name, assets, &scene, &synthetic) != RT_OK) {
        fprintf(stderr, "rtbench: scene %s: %s\n", scene_name, scene ? rt_scene_last_error(scene) : rt_last_error(NULL));
        if (scene) rt_scene_free(scene);
        return 1;
    }
    rt_scene_desc desc;
    rt_scene_get_desc(scene, &desc);

    /* Renderer.init: device, pipeline, buffers, acceleration structures (Renderer.swift:228-606) */
    rt_opts opts;
    memset(&opts, 0, sizeof opts);
    opts.device = 0;
    opts.pipeline = pipeline;
    opts.frames_in_flight = fif;
    rt_ctx* ctx = NULL;
    if (check(rt_create(&opts, &ctx), ctx, "rt_create")) return 1;
    int rc = 1;
    uint32_t* offsets = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)W * H);
    uint8_t* rgba8 = NULL;
    if (!offsets) goto done;
    if (check(rt_scene_upload(ctx, &desc), ctx, "rt_scene_upload") || check(rt_bvh_build(ctx), ctx, "rt_bvh_build"))
        goto done;
    /* createTextures: random offsets + accumulation targets (Renderer.swift:676-804) */
    rt_random_offsets(3, W, H, offsets);
    if (check(rt_resize(ctx, W, H, offsets), ctx, "rt_resize")) goto done;

    /* updateUniforms (Renderer.swift:608-664) + draw (:1405-1503), frames back to back */
    Uniforms u;
    rt_uniforms_default(W, H, (int32_t)desc.light_count, &u);
    u.samplesPerPixel = spp;
    u.maxBounces = bounces;
    uint32_t frame = 0;
    for (int f = 0; f < warmup; ++f, ++frame) {
        u.frameIndex = frame;
        if (check(rt_render_frame(ctx, &u, NULL), ctx, "rt_render_frame")) goto done;
    }
    if (check(rt_wait(ctx), ctx, "rt_wait")) goto done;
    rt_stats s0, s1;
    if (check(rt_get_stats(ctx, &s0), ctx, "rt_get_stats")) goto done;
    const double t0 = now_s();
    for (int f = 0; f < frames; ++f, ++frame) {
        u.frameIndex = frame;
        if (check(rt_render_frame(ctx, &u, NULL), ctx, "rt_render_frame")) goto done;
    }
    if (check(rt_wait(ctx), ctx, "rt_wait")) goto done;
    const double dt = now_s() - t0;
    if (check(rt_get_stats(ctx, &s1), ctx, "rt_get_stats")) goto done;
    const double rays = (double)(s1.total_closest_rays - s0.total_closest_rays) +
                        (double)(s1.total_shadow_rays - s0.total_shadow_rays);
    printf("{\"scene\": \"%s\", \"synthetic\": %d, \"width\": %d, \"height\": %d, \"spp\": %d, \"bounces\": %d, "
           "\"frames\": %d, \"frames_in_flight\": %d, \"grays_per_s\": %.4f, \"ms_per_frame\": %.3f, "
           "\"rays_per_frame\": %.0f, \"last_frame_device_ms\": %.3f, \"triangles\": %llu}\n",
           scene_name, (int)synthetic, W, H, spp, bounces, frames, (int)s1.frames_in_flight, rays / dt / 1e9,
           dt / frames * 1e3, rays / frames, s1.last_frame_ms, (unsigned long long)s1.triangles);

    if (png) {   /* FramePresenter.draw + fragmentShader (FramePresenter.swift:103-238, Shaders.metal:39-52) */
        rgba8 = (uint8_t*)malloc((size_t)W * H * 4);
        rt_present_opts po;
        memset(&po, 0, sizeof po);
        po.scaler = scaler;
        if (!rgba8 || check(rt_present(ctx, &po, rgba8), ctx, "rt_present")) goto done;
        if (rt_write_png(png, rgba8, (uint32_t)W, (uint32_t)H) != RT_OK) {
            fprintf(stderr, "rtbench: cannot write %s\n", png);
            goto done;
        }
    }
    rc = 0;
done:
    free(rgba8);
    free(offsets);
    rt_destroy(ctx);
    rt_scene_free(scene);
    return rc;
}
