/*
 * graph_wait_repro.c — the frame-graph shape of the wavefront renderer, reduced to HIP runtime
 * calls (no kernels of ours: memsets stand in for the launches), for the question DESIGN.md §3.4
 * records: can a frame's HIP graph hold the wait for the previous frame (an event recorded on
 * another slot's stream after that slot's graph launch) as a captured external event-wait node?
 *
 * Two "slots" (streams) alternate frames, as frames in flight do (Renderer.swift:1406-1409 keeps
 * up to three command buffers in flight).  Each frame is captured once per slot and replayed:
 *   part 0: memset + external event-record nodes (the timeline events)
 *   the wait for the other slot's `done` event
 *   part 1: memset + external event-record node
 * then `done` is recorded on the slot's stream outside the graph.
 *
 *   graph_wait_repro split      the wait enqueued between two graphs as a plain stream wait (the
 *                                library's design since round 3)
 *   graph_wait_repro captured   the wait captured inside one graph as an external event-wait
 *                                node (hipStreamWaitEvent(..., hipEventWaitExternal) during capture:
 *                                the round-3 design that crashed under the ROCm 7.2 runtime)
 *
 * Prints one line per step to stderr (so a crash names the call it died in) and exits 0 when
 * every frame ran, 3 on a HIP error.
 */
#include <hip/hip_runtime_api.h>
#include <stdio.h>
#include <string.h>

#define CK(expr)                                                                                  \
    do {                                                                                          \
        hipError_t e_ = (expr);                                                                   \
        if (e_ != hipSuccess) {                                                                   \
            fprintf(stderr, "repro: %s -> %s\n", #expr, hipGetErrorString(e_));                   \
            return 3;                                                                             \
        }                                                                                         \
    } while (0)
#define STEP(...)                          \
    do {                                   \
        fprintf(stderr, "repro: " __VA_ARGS__); \
        fputc('\n', stderr);               \
        fflush(stderr);                    \
    } while (0)

enum { kSlots = 2, kFrames = 8, kBytes = 1 << 20 };

typedef struct {
    hipStream_t s;
    hipEvent_t t0, t1, t2, done;     /* timeline events (timing) and the frame's done (no timing) */
    hipGraphExec_t exec[2];
    hipEvent_t exec_wait;            /* captured: the event exec[0] waits on (re-captured when it changes) */
    void* buf;
} Slot;

/* part `part` of a frame on slot `k`, recorded into the stream (capturing or not) */
static int record_part(Slot* S, int part, hipEvent_t wait_on, int capture) {
    const unsigned rf = capture ? hipEventRecordExternal : 0u;
    if (part == 0) {
        CK(hipEventRecordWithFlags(S->t0, S->s, rf));
        CK(hipMemsetAsync(S->buf, 1, kBytes, S->s));
        CK(hipEventRecordWithFlags(S->t1, S->s, rf));
    } else {
        if (wait_on) {
            if (capture) STEP("  hipStreamWaitEvent(external) during capture");
            CK(hipStreamWaitEvent(S->s, wait_on, capture ? hipEventWaitExternal : 0u));
            if (capture) STEP("  returned");
        }
        CK(hipMemsetAsync(S->buf, 2, kBytes, S->s));
        CK(hipEventRecordWithFlags(S->t2, S->s, rf));
    }
    return 0;
}

static int capture(Slot* S, int part, hipEvent_t wait_on, hipGraphExec_t* out) {
    hipGraph_t g = NULL;
    CK(hipStreamBeginCapture(S->s, hipStreamCaptureModeThreadLocal));
    int r = record_part(S, part, wait_on, 1);
    hipError_t ce = hipStreamEndCapture(S->s, &g);
    if (r) return r;
    CK(ce);
    CK(hipGraphInstantiateWithFlags(out, g, 0));
    CK(hipGraphDestroy(g));
    return 0;
}

int main(int argc, char** argv) {
    const int captured = argc > 1 && !strcmp(argv[1], "captured");
    if (argc > 1 && !captured && strcmp(argv[1], "split")) {
        fprintf(stderr, "usage: graph_wait_repro split|captured\n");
        return 2;
    }
    int ver = 0;
    CK(hipRuntimeGetVersion(&ver));
    STEP("HIP runtime %d, mode %s", ver, captured ? "captured" : "split");
    Slot sl[kSlots];
    memset(sl, 0, sizeof sl);
    for (int k = 0; k < kSlots; ++k) {
        CK(hipStreamCreateWithFlags(&sl[k].s, hipStreamNonBlocking));
        CK(hipEventCreate(&sl[k].t0));
        CK(hipEventCreate(&sl[k].t1));
        CK(hipEventCreate(&sl[k].t2));
        CK(hipEventCreateWithFlags(&sl[k].done, hipEventDisableTiming));
        CK(hipMalloc(&sl[k].buf, kBytes));
    }
    for (int f = 0; f < kFrames; ++f) {
        Slot* S = &sl[f % kSlots];
        hipEvent_t prev = f > 0 ? sl[(f - 1) % kSlots].done : NULL;
        if (f >= kSlots) CK(hipEventSynchronize(S->done));   /* the slot's previous frame */
        if (captured) {   /* one graph: part 0, the wait, part 1 */
            if (S->exec[0] && S->exec_wait != prev) {
                CK(hipGraphExecDestroy(S->exec[0]));
                S->exec[0] = NULL;
            }
            if (!S->exec[0]) {
                hipGraph_t g = NULL;
                S->exec_wait = prev;
                STEP("frame %d: capture (wait inside the graph)", f);
                CK(hipStreamBeginCapture(S->s, hipStreamCaptureModeThreadLocal));
                int r = record_part(S, 0, NULL, 1);
                if (!r) {
                    STEP("frame %d: part 1%s", f, prev ? ", after a captured wait on the previous frame's done" : "");
                    r = record_part(S, 1, prev, 1);
                }
                STEP("frame %d: end capture", f);
                hipError_t ce = hipStreamEndCapture(S->s, &g);
                if (r) return r;
                CK(ce);
                STEP("frame %d: instantiate", f);
                CK(hipGraphInstantiateWithFlags(&S->exec[0], g, 0));
                CK(hipGraphDestroy(g));
            }
            STEP("frame %d: launch", f);
            CK(hipGraphLaunch(S->exec[0], S->s));
        } else {          /* two graphs, the wait a plain stream wait between them */
            for (int part = 0; part < 2; ++part)
                if (!S->exec[part]) {
                    STEP("frame %d: capture part %d", f, part);
                    int r = capture(S, part, NULL, &S->exec[part]);
                    if (r) return r;
                }
            STEP("frame %d: launch part 0, wait, launch part 1", f);
            CK(hipGraphLaunch(S->exec[0], S->s));
            if (prev) CK(hipStreamWaitEvent(S->s, prev, 0));
            CK(hipGraphLaunch(S->exec[1], S->s));
        }
        CK(hipEventRecord(S->done, S->s));
    }
    for (int k = 0; k < kSlots; ++k) CK(hipStreamSynchronize(sl[k].s));
    float ms = 0.0f;
    CK(hipEventElapsedTime(&ms, sl[0].t0, sl[0].t2));
    STEP("ok: %d frames, last frame of slot 0 %.3f ms", kFrames, ms);
    for (int k = 0; k < kSlots; ++k) {
        for (int p = 0; p < 2; ++p)
            if (sl[k].exec[p]) CK(hipGraphExecDestroy(sl[k].exec[p]));
        CK(hipFree(sl[k].buf));
        CK(hipStreamDestroy(sl[k].s));
    }
    return 0;
}
