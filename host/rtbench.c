/*
 * rtbench.c — the C host driver over the C-ABI (SURVEY.md §8b "callers": the shape of
 * Renderer.draw, Renderer.swift:1405-1503, without Swift/Metal).  Plain C11, links
 * metal4-raytracing_amd/librt_hip.so; no torch, no Python.
 *
 *   rtbench [--scene c3g] [--width 1920] [--height 1080] [--spp 4] [--bounces 8] [--frames 16]
 *           [--warmup 2] [--assets DIR] [--png out.png] [--scaler none|spatial|temporal]
 *           [--frames-in-flight N] [--megakernel] [--ranks N]
 *
 * Renders `warmup` + `frames` frames back to back (frames in flight), waits once, and prints
 * one line: Grays/s over the timed frames (closest-hit + shadow rays from the library's running
 * totals / host wall time), ms per frame, and the device time of the newest frame.  With --png
 * the newest frame is presented (tone-mapped, sRGB) and written as a PNG.
 *
 * --ranks N: the multi-GPU frame split from C.  The launcher starts N child
 * processes of itself (posix_spawn, before anything touches a GPU), one per GPU; rank r renders
 * the 64x64 tiles with tile_id % N == r on device r, packs them (rt_pack_tiles_on) and RCCL's
 * ncclGather collects the packed buffers on rank 0, which unpacks them into its frame
 * (rt_unpack_tiles_on) before presenting.  Rank 0 creates the ncclUniqueId and passes it to the
 * others through a file.  Grays/s = all ranks' rays / the slowest rank's wall time.
 */
#define _POSIX_C_SOURCE 200809L
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>
#include <spawn.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/wait.h>
#include <time.h>
#include <unistd.h>

#include "rt_api.h"
#include "rt_scene.h"

extern char** environ;

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
            "               [--frames-in-flight N] [--megakernel] [--ranks N]\n");
}

#define NCCLC(expr)                                                                         \
    do {                                                                                    \
        ncclResult_t r_ = (expr);                                                           \
        if (r_ != ncclSuccess) {                                                            \
            fprintf(stderr, "rtbench: %s failed: %s\n", #expr, ncclGetErrorString(r_));      \
            goto done;                                                                      \
        }                                                                                   \
    } while (0)
#define HIPCK(expr)                                                                         \
    do {                                                                                    \
        hipError_t e_ = (expr);                                                             \
        if (e_ != hipSuccess) {                                                             \
            fprintf(stderr, "rtbench: %s failed: %s\n", #expr, hipGetErrorString(e_));       \
            goto done;                                                                      \
        }                                                                                   \
    } while (0)

/* The launcher of --ranks N: N children of this program with --rank r --nranks N --id-file F,
 * started before this process touches a GPU; returns the first failing child's status. */
static int launch_ranks(int n, int argc, char** argv) {
    char self[4096];
    ssize_t len = readlink("/proc/self/exe", self, sizeof self - 1);
    if (len <= 0) return 1;
    self[len] = 0;
    char idfile[256], rk[16], nr[16];
    snprintf(idfile, sizeof idfile, "/tmp/rtbench_ncclid_%d", (int)getpid());
    unlink(idfile);
    snprintf(nr, sizeof nr, "%d", n);
    pid_t* pids = (pid_t*)calloc((size_t)n, sizeof(pid_t));
    char** av = (char**)calloc((size_t)argc + 8, sizeof(char*));
    if (!pids || !av) return 1;
    int status = 0;
    for (int r = 0; r < n; ++r) {
        int k = 0;
        av[k++] = self;
        for (int i = 1; i < argc; ++i) {
            if (!strcmp(argv[i], "--ranks")) { ++i; continue; }   /* the children are ranks, not launchers */
            av[k++] = argv[i];
        }
        snprintf(rk, sizeof rk, "%d", r);
        av[k++] = (char*)"--rank";
        av[k++] = rk;
        av[k++] = (char*)"--nranks";
        av[k++] = nr;
        av[k++] = (char*)"--id-file";
        av[k++] = idfile;
        av[k] = NULL;
        if (posix_spawn(&pids[r], self, NULL, NULL, av, environ) != 0) {
            fprintf(stderr, "rtbench: cannot start rank %d\n", r);
            status = 1;
            n = r;
            break;
        }
    }
    for (int r = 0; r < n; ++r) {
        int ws = 0;
        if (waitpid(pids[r], &ws, 0) < 0 || !WIFEXITED(ws) || WEXITSTATUS(ws) != 0) {
            if (!status) status = WIFEXITED(ws) ? WEXITSTATUS(ws) : 1;
            for (int q = 0; q < n; ++q)   /* a failed rank leaves the collectives hanging */
                if (q != r) kill(pids[q], SIGTERM);
        }
    }
    unlink(idfile);
    free(av);
    free(pids);
    return status;
}

int main(int argc, char** argv) {
    const char* scene_name = "c3g";
    const char* assets = "assets";
    const char* png = NULL;
    int W = 1920, H = 1080, spp = 4, bounces = 8, frames = 16, warmup = 2, fif = 0, scaler = RT_SCALER_NONE;
    int pipeline = RT_PIPELINE_WAVEFRONT;
    int ranks = 0, rank = 0, nranks = 0;
    const char* idfile = NULL;
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
        else if (!strcmp(a, "--ranks")) ranks = atoi(v);
        else if (!strcmp(a, "--rank")) rank = atoi(v);
        else if (!strcmp(a, "--nranks")) nranks = atoi(v);
        else if (!strcmp(a, "--id-file")) idfile = v;
        else if (!strcmp(a, "--scaler")) {
            scaler = !strcmp(v, "spatial") ? RT_SCALER_SPATIAL : !strcmp(v, "temporal") ? RT_SCALER_TEMPORAL : RT_SCALER_NONE;
        } else {
            usage();
            return 2;
        }
    }
    if (W <= 0 || H <= 0 || frames <= 0 || warmup < 0 || ranks < 0 || (nranks > 0 && (!idfile || rank < 0 || rank >= nranks))) {
        usage();
        return 2;
    }
    if (ranks > 0) return launch_ranks(ranks, argc, argv);
    const int split = nranks > 0;   /* this process is one rank of a --ranks split */
    if (!split) nranks = 1;
    rt_tile_set tset = {64, rank, nranks, 0};
    ncclComm_t comm = NULL;
    hipStream_t cs = NULL;
    float *d_send = NULL, *d_recv = NULL;
    double* d_red = NULL;
    size_t count = 0;

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
    opts.device = split ? rank : 0;
    opts.pipeline = pipeline;
    opts.frames_in_flight = fif;
    rt_ctx* ctx = NULL;
    if (check(rt_create(&opts, &ctx), ctx, "rt_create")) return 1;
    int rc = 1;
    uint32_t* offsets = NULL;
    uint8_t* rgba8 = NULL;
    if (split) {   /* RCCL communicator over the ranks: rank 0's unique id travels through a file */
        ncclUniqueId id;
        HIPCK(hipSetDevice(rank));
        if (rank == 0) {
            char tmp[300];
            NCCLC(ncclGetUniqueId(&id));
            snprintf(tmp, sizeof tmp, "%s.tmp", idfile);
            FILE* f = fopen(tmp, "wb");
            if (!f || fwrite(&id, sizeof id, 1, f) != 1) { if (f) fclose(f); goto done; }
            fclose(f);
            if (rename(tmp, idfile) != 0) goto done;
        } else {
            int got = 0;
            for (int tries = 0; tries < 1200 && !got; ++tries) {   /* up to 120 s */
                FILE* f = fopen(idfile, "rb");
                if (f) {
                    got = fread(&id, sizeof id, 1, f) == 1;
                    fclose(f);
                }
                if (!got) {
                    struct timespec ts = {0, 100000000};
                    nanosleep(&ts, NULL);
                }
            }
            if (!got) { fprintf(stderr, "rtbench: rank %d: no RCCL id from rank 0\n", rank); goto done; }
        }
        NCCLC(ncclCommInitRank(&comm, nranks, id, rank));
        HIPCK(hipStreamCreate(&cs));
        int max_own = 0;
        for (int r = 0; r < nranks; ++r) {
            rt_tile_set t = {64, r, nranks, 0};
            const int c = rt_tile_count(W, H, &t);
            if (c > max_own) max_own = c;
        }
        count = (size_t)max_own * 64 * 64 * 4;   /* floats per rank (ranks padded to equal size) */
        HIPCK(hipMalloc((void**)&d_send, count * sizeof(float)));
        if (rank == 0) HIPCK(hipMalloc((void**)&d_recv, count * sizeof(float) * (size_t)nranks));
        HIPCK(hipMalloc((void**)&d_red, 4 * sizeof(double)));
    }
    offsets = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)W * H);
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
    rt_stats s0, s1;
    double t0 = 0.0;
    for (int f = 0; f < warmup + frames; ++f, ++frame) {
        if (f == warmup) {   /* the timed region starts with every rank idle */
            if (check(rt_wait(ctx), ctx, "rt_wait") || check(rt_get_stats(ctx, &s0), ctx, "rt_get_stats")) goto done;
            if (split) {
                HIPCK(hipStreamSynchronize(cs));
                NCCLC(ncclAllReduce(d_red, d_red, 1, ncclFloat64, ncclSum, comm, cs));   /* barrier */
                HIPCK(hipStreamSynchronize(cs));
            }
            t0 = now_s();
        }
        u.frameIndex = frame;
        if (check(rt_render_frame(ctx, &u, split ? &tset : NULL), ctx, "rt_render_frame")) goto done;
        if (split) {   /* pack -> ncclGather to rank 0 -> unpack, on one stream, no host wait */
            if (check(rt_pack_tiles_on(ctx, &tset, d_send, cs), ctx, "rt_pack_tiles_on")) goto done;
            NCCLC(ncclGather(d_send, d_recv, count, ncclFloat32, 0, comm, cs));
            if (rank == 0)
                for (int r = 1; r < nranks; ++r) {
                    rt_tile_set t = {64, r, nranks, 0};
                    if (check(rt_unpack_tiles_on(ctx, &t, d_recv + (size_t)r * count, cs), ctx, "rt_unpack_tiles_on"))
                        goto done;
                }
        }
    }
    if (check(rt_wait(ctx), ctx, "rt_wait")) goto done;
    if (split) HIPCK(hipStreamSynchronize(cs));
    double dt = now_s() - t0;
    if (check(rt_get_stats(ctx, &s1), ctx, "rt_get_stats")) goto done;
    double rays = (double)(s1.total_closest_rays - s0.total_closest_rays) +
                  (double)(s1.total_shadow_rays - s0.total_shadow_rays);
    if (split) {   /* all ranks' rays over the slowest rank's wall time */
        double h[2] = {rays, dt};
        HIPCK(hipMemcpy(d_red, h, sizeof h, hipMemcpyHostToDevice));
        NCCLC(ncclAllReduce(d_red, d_red + 2, 1, ncclFloat64, ncclSum, comm, cs));
        NCCLC(ncclAllReduce(d_red + 1, d_red + 3, 1, ncclFloat64, ncclMax, comm, cs));
        HIPCK(hipStreamSynchronize(cs));
        HIPCK(hipMemcpy(h, d_red + 2, sizeof h, hipMemcpyDeviceToHost));
        rays = h[0];
        dt = h[1];
    }
    if (rank == 0)
    printf("{\"scene\": \"%s\", \"synthetic\": %d, \"width\": %d, \"height\": %d, \"spp\": %d, \"bounces\": %d, "
           "\"frames\": %d, \"frames_in_flight\": %d, \"grays_per_s\": %.4f, \"ms_per_frame\": %.3f, "
           "\"rays_per_frame\": %.0f, \"last_frame_device_ms\": %.3f, \"triangles\": %llu, \"ranks\": %d, "
           "\"graph_replays\": %llu, \"graph_captures\": %llu, \"graph_fallbacks\": %llu, \"graph_eager\": %llu}\n",
           scene_name, (int)synthetic, W, H, spp, bounces, frames, (int)s1.frames_in_flight, rays / dt / 1e9,
           dt / frames * 1e3, rays / frames, s1.last_frame_ms, (unsigned long long)s1.triangles, nranks,
           (unsigned long long)s1.total_graph_replays, (unsigned long long)s1.total_graph_captures,
           (unsigned long long)s1.total_graph_fallbacks, (unsigned long long)s1.total_graph_eager);

    if (png && rank == 0) {   /* FramePresenter.draw + fragmentShader (FramePresenter.swift:103-238, Shaders.metal:39-52) */
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
    if (comm) ncclCommDestroy(comm);
    if (d_send) (void)hipFree(d_send);
    if (d_recv) (void)hipFree(d_recv);
    if (d_red) (void)hipFree(d_red);
    if (cs) (void)hipStreamDestroy(cs);
    free(rgba8);
    free(offsets);
    rt_destroy(ctx);
    rt_scene_free(scene);
    return rc;
}
