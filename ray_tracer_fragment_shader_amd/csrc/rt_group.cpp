// rt_group.cpp — multi-GPU frames: row bands rendered on every GPU of a group, gathered to rank 0 over
// RCCL (xGMI) and put back in image order there (BASELINE.json configs c4).
//
// The reference renders one frame on one thread (rayTraceScreen, Hw4/MySdlApplication.cpp:1251-1324, called
// by draw() at :1560); it has no distribution.  Pixels are independent (rayTraceRay :1184-1249 reads only the
// scene), so a frame splits by rows: round-robin bands of `band_height` rows (contiguous stripes would be badly
// imbalanced: sky rows are cheap, board rows are not), rank r rendering bands b = r (mod n) densely into its
// slab (rt_rows).  The only data-path exchange is the gather of the slabs to rank 0:
//
//   render stream rs_r[k] (k alternates per frame of a static view: consecutive frames' renders overlap):
//                        wait sent[r][b] -> rt_render_dev(rows of r) into slab[r][b] -> record rendered[r][b]
//   comm stream   cs_r:  wait rendered[r][b] -> ncclSend(slab[r][b] -> rank 0)      -> record sent[r][b]
//   root cs_0:           ncclRecv(gathered[b] + q*slab <- q), q = 1..n-1 (posted at once: they do not wait for
//                        the root's own render); wait the caller stream's earlier work (received[b]) and the
//                        root's render (rendered[b]) -> unshuffle(gathered[b] + root slab[b] -> image)
//                        -> record assembled[b]; the caller's stream waits for assembled[b]
// A process's ranks must switch scenes between the same frames: one-process-per-GPU groups agree on the scene
// (hence the wire formats) with a small all-reduce whenever a rank's scene changes (agree_on_scene).
// Stream priorities: all at the device's default (a high-priority comm stream preempts the renders, setup_rank).
// A one-rank group renders straight into the caller's image on the caller's stream (identity band plan).
//
// What travels: the wire formats.  An achromatic scene (every colour term with R = G = B, rt_scene_achromatic)
// renders R = G = B bit for bit, so the RGBA8 image travels as GRAY8 (1 B/px) and RGBA32F as GRAY32F (4 B/px);
// other scenes send RGB8 (3 B/px; alpha is the constant 255) and RGBA32F.  The root expands them into its images
// in the same kernel that puts the bands in image order (rt_unpack_dev).  At c4 (3840 x 2160 over 8 ranks) the
// root's ingress is 7/8 of 8.3 MB instead of 7/8 of 33.2 MB.
//
// b = frame % n_bufs (3): the slabs and the root's gather buffer are triple-buffered, so frame f's gather overlaps
// the renders of frames f+1 and f+2.  Transports: RCCL (ncclCommInitAll for one process driving n GPUs, ncclCommInitRank
// for one process per GPU) or COPY (hipMemcpyPeerAsync on the root's comm stream; used when contexts share
// a device — RCCL refuses two ranks on one GPU — which is how the n-rank logic is exercised on one GPU).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/rt_api.h"
#include "../../include/rt_diag.h"
#include "rt_internal.hpp"

namespace {

constexpr int kKinds = 2;                      // 0: the RGBA32F image, 1: the RGBA8 image
constexpr int kImageFormat[kKinds] = {RT_PIXEL_RGBA32F, RT_PIXEL_RGBA8};
constexpr int kRing = 64;                      // frames of per-phase timing events kept
// Frame buffers (slabs, the root's gather buffer and their events): frame f uses buffer f % n_bufs.  A buffer is
// rendered into again only once frame f - n_bufs has left it (its send, the root's unpack): with two, a rank's render of
// frame f + 2 waits for frame f's send / unpack, which waits for frame f's render — a chain of one render and one
// exchange per two frames; a third buffer lets it run a frame further ahead (rank 0's pipeline at 8 ranks, one GPU:
// 41 -> 30 us per frame when its streams have hardware queues of their own, tools/c4_gap_probe.py part 6).  RCCL groups
// (one device per rank) use 3; COPY groups (every rank on one device: 3 streams per rank oversubscribe its hardware
// queues, and with 3 buffers the frame time jumped between 0.20 and 1.06 ms run to run, tools/c4_copy_probe.py) use 2.
// RT_GROUP_BUFFERS=2|3 overrides.
constexpr int kBufs = 3;

// Per-phase timing events of one frame on one rank (rt_group_timing): render start / end on the render stream,
// gather start (the rank's render is done) / end on the comm stream, and on the root the assembled image.
struct PhaseEvents {
    hipEvent_t r0 = nullptr, r1 = nullptr, g0 = nullptr, g1 = nullptr, a1 = nullptr;
    bool rec = false, gather_rec = false;
    bool rendered = true;                      // false: an assembling rank 0 (r0 .. r1 is empty, not a render)
};

struct Rank {
    rt_ctx* ctx = nullptr;
    int device = 0;
    int rank = 0;
    // Two render streams and a comm stream (on `device`).  A frame renders on rs[k]: a static view alternates k, so a
    // frame's bands start while the previous frame's last waves drain (a 1/8 band set of the c4 frame is a short
    // launch whose tail is one long wave: 27 us serial, 15 us per frame on two streams, tools/c4_gap_probe.py part 3);
    // a new camera stays on the previous frame's stream (its per-eye preparation rewrites state the other stream's
    // render may still read, which the context would otherwise resolve with a device synchronisation).
    hipStream_t rs[2] = {nullptr, nullptr}, cs = nullptr;
    int last_rs = 1;                           // rs index of the previous frame
    hipEvent_t rendered[kBufs] = {};
    hipEvent_t sent[kBufs] = {};               // on cs (RCCL) or on the root's comm stream (COPY)
    bool sent_rec[kBufs] = {};
    void* slab[kBufs][kKinds] = {};
    size_t slab_cap[kBufs][kKinds] = {};
    ncclComm_t comm = nullptr;
    uint64_t* d_agree = nullptr;               // rt_group_create_rank: the scene agreement's all-reduce buffer
    uint64_t agreed_fp = 0;                    // the scene fingerprint the group last agreed on
    bool agreed = false;
    PhaseEvents ph[kRing];
};

}  // namespace

struct rt_group {
    int n_ranks = 0;                           // ranks of the whole group
    int transport = RT_TRANSPORT_RCCL;
    bool owns_root = false;                    // rank 0 is one of this process's ranks (ranks[0])
    std::vector<Rank> ranks;                   // this process's ranks
    // root only
    void* gathered[kBufs][kKinds] = {};
    size_t gathered_cap[kBufs][kKinds] = {};
    hipEvent_t received[kBufs] = {};
    hipEvent_t assembled[kBufs] = {};
    bool assembled_rec[kBufs] = {};
    int n_bufs = kBufs;                        // RT_GROUP_BUFFERS (A/B): 2
    uint64_t frame = 0;
    int last_band = 0, last_slab_rows = 0;
    // timing (rt_group_timing): frames [t_first, frame) are recorded, the last kRing of them kept
    bool timing = false;
    uint64_t t_first = 0;
    int last_wire[kKinds] = {-1, -1};
    // RT_GATHER_ROOT_WAITS=1 (A/B): the root's receives / peer copies wait for the root's own render first (r03)
    bool root_waits = false;
    uint64_t last_payload = 0;
    // the frame plans (rt_group_plan.cpp) of the local ranks and of rank 0, for the key {W, H, band_height, outputs,
    // achromatic}: recomputed only when the key changes (no host allocation or per-rank loops per frame)
    std::vector<rt_group_plan> plan;           // sized at creation: one per local rank
    rt_group_plan root_plan{};
    int plan_key[5] = {0, 0, 0, 0, 0};
    bool plan_valid = false;
    // the previous frame's camera (a static view alternates the ranks' render streams, Rank::rs)
    rt_camera last_cam{};
    bool last_cam_valid = false;
    int render_streams = 2;                    // RT_GROUP_RENDER_STREAMS (A/B): 1 renders every frame on rs[0]
};

namespace {

#define G_HIP(call)                                                                                   \
    do {                                                                                              \
        hipError_t e_ = (call);                                                                       \
        if (e_ != hipSuccess) return rt_fail(RT_EHIP, std::string(#call) + ": " + hipGetErrorString(e_)); \
    } while (0)

#define G_NCCL(call)                                                                                  \
    do {                                                                                              \
        ncclResult_t r_ = (call);                                                                     \
        if (r_ != ncclSuccess) return rt_fail(RT_EHIP, std::string(#call) + ": " + ncclGetErrorString(r_)); \
    } while (0)

int grow(void** p, size_t* cap, size_t bytes) {
    if (bytes <= *cap) return RT_OK;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
    if (hipMalloc(p, bytes) != hipSuccess) return rt_fail(RT_ENOMEM, "rt_render_multi: hipMalloc of a slab failed");
    *cap = bytes;
    return RT_OK;
}

bool comm_high_priority() {
    const char* e = getenv("RT_GROUP_COMM_PRIORITY");
    return e && atoi(e) == 1;
}

int setup_rank(Rank* r, rt_ctx* ctx, int rank, hipEvent_t* sent_device_events) {
    r->ctx = ctx;
    r->rank = rank;
    r->device = rt_ctx_device(ctx);
    G_HIP(hipSetDevice(r->device));
    // Every stream at the device's lowest (default) priority.  r02-r05 gave the comm stream (RCCL send/recv, the
    // root's unpack) the greatest priority so its kernels would not queue behind the next render grid; measured on
    // MI355X (tools/c4_gap_probe.py part 6, rank 0's pipeline at 8 ranks: bands on two streams, each frame's unpack on
    // the comm stream), a high-priority comm stream runs 120 us per frame against 39 us at normal priority — the
    // renders on the other queues are preempted around every high-priority dispatch.  RT_GROUP_COMM_PRIORITY=1 (A/B)
    // restores it.
    int least = 0, greatest = 0;
    G_HIP(hipDeviceGetStreamPriorityRange(&least, &greatest));
    for (int k = 0; k < 2; ++k) G_HIP(hipStreamCreateWithPriority(&r->rs[k], hipStreamNonBlocking, least));
    G_HIP(hipStreamCreateWithPriority(&r->cs, hipStreamNonBlocking, comm_high_priority() ? greatest : least));
    for (int b = 0; b < kBufs; ++b) {
        G_HIP(hipEventCreateWithFlags(&r->rendered[b], hipEventDisableTiming));
        if (!sent_device_events) G_HIP(hipEventCreateWithFlags(&r->sent[b], hipEventDisableTiming));
        else r->sent[b] = sent_device_events[b];
    }
    return RT_OK;
}

int setup_root_events(rt_group* g) {
    G_HIP(hipSetDevice(g->ranks[0].device));
    for (int b = 0; b < kBufs; ++b) {
        G_HIP(hipEventCreateWithFlags(&g->received[b], hipEventDisableTiming));
        G_HIP(hipEventCreateWithFlags(&g->assembled[b], hipEventDisableTiming));
    }
    return RT_OK;
}

}  // namespace

extern "C" int rt_comm_unique_id(uint8_t* id) {
    if (!id) return rt_fail(RT_EINVAL, "rt_comm_unique_id: null id");
    static_assert(sizeof(ncclUniqueId) == RT_COMM_ID_BYTES, "RCCL unique id size");
    ncclUniqueId u;
    G_NCCL(ncclGetUniqueId(&u));
    memcpy(id, &u, sizeof(u));
    return RT_OK;
}

extern "C" int rt_group_destroy(rt_group* g) {
    if (!g) return RT_OK;
    for (auto& r : g->ranks) {
        (void)hipSetDevice(r.device);
        for (hipStream_t s : r.rs)
            if (s) (void)hipStreamSynchronize(s);
        if (r.cs) (void)hipStreamSynchronize(r.cs);
    }
    for (auto& r : g->ranks) {
        (void)hipSetDevice(r.device);
        if (r.comm) (void)ncclCommDestroy(r.comm);
        if (r.d_agree) (void)hipFree(r.d_agree);
        for (auto& e : r.ph)
            for (hipEvent_t ev : {e.r0, e.r1, e.g0, e.g1, e.a1})
                if (ev) (void)hipEventDestroy(ev);
        for (int b = 0; b < kBufs; ++b) {
            if (r.rendered[b]) (void)hipEventDestroy(r.rendered[b]);
            if (r.sent[b] && g->transport == RT_TRANSPORT_RCCL) (void)hipEventDestroy(r.sent[b]);
            for (int k = 0; k < kKinds; ++k)
                if (r.slab[b][k]) (void)hipFree(r.slab[b][k]);
        }
        for (hipStream_t s : r.rs)
            if (s) (void)hipStreamDestroy(s);
        if (r.cs) (void)hipStreamDestroy(r.cs);
    }
    if (g->owns_root && !g->ranks.empty()) {
        (void)hipSetDevice(g->ranks[0].device);
        for (int b = 0; b < kBufs; ++b) {
            if (g->received[b]) (void)hipEventDestroy(g->received[b]);
            if (g->assembled[b]) (void)hipEventDestroy(g->assembled[b]);
            for (int k = 0; k < kKinds; ++k)
                if (g->gathered[b][k]) (void)hipFree(g->gathered[b][k]);
        }
        if (g->transport == RT_TRANSPORT_COPY)          // COPY: every rank's `sent` events live on the root
            for (auto& r : g->ranks)
                for (int b = 0; b < kBufs; ++b)
                    if (r.sent[b]) (void)hipEventDestroy(r.sent[b]);
    }
    delete g;
    return RT_OK;
}

extern "C" int rt_group_create(rt_ctx* const* ctxs, int n, int transport, rt_group** out) {
    if (!out) return rt_fail(RT_EINVAL, "rt_group_create: null out");
    *out = nullptr;
    if (!ctxs || n <= 0) return rt_fail(RT_EINVAL, "rt_group_create: need at least one context");
    if (transport != RT_TRANSPORT_AUTO && transport != RT_TRANSPORT_RCCL && transport != RT_TRANSPORT_COPY)
        return rt_fail(RT_EINVAL, "rt_group_create: unknown transport");
    std::vector<int> devs(n);
    for (int q = 0; q < n; ++q) {
        if (!ctxs[q]) return rt_fail(RT_EINVAL, "rt_group_create: null context");
        for (int p = 0; p < q; ++p)
            if (ctxs[p] == ctxs[q]) return rt_fail(RT_EINVAL, "rt_group_create: a context appears twice");
        devs[q] = rt_ctx_device(ctxs[q]);
    }
    std::vector<int> sorted = devs;
    std::sort(sorted.begin(), sorted.end());
    const bool distinct = std::adjacent_find(sorted.begin(), sorted.end()) == sorted.end();
    if (transport == RT_TRANSPORT_AUTO) transport = distinct ? RT_TRANSPORT_RCCL : RT_TRANSPORT_COPY;
    if (transport == RT_TRANSPORT_RCCL && !distinct)
        return rt_fail(RT_EINVAL, "rt_group_create: RCCL needs one context per device (use RT_TRANSPORT_COPY)");
    rt_group* g = new rt_group();
    if (const char* e = getenv("RT_GATHER_ROOT_WAITS")) g->root_waits = atoi(e) != 0;
    if (const char* e = getenv("RT_GROUP_RENDER_STREAMS")) g->render_streams = atoi(e) == 1 ? 1 : 2;
    if (const char* e = getenv("RT_GROUP_BUFFERS")) g->n_bufs = atoi(e) == 2 ? 2 : kBufs;
    g->n_ranks = n;
    g->transport = transport;
    if (transport == RT_TRANSPORT_COPY && !getenv("RT_GROUP_BUFFERS")) g->n_bufs = 2;
    g->owns_root = true;
    g->ranks.resize(n);
    g->plan.resize(n);
    int rc = RT_OK;
    // COPY: the root's comm stream records every rank's `sent` events, so they live on the root device.
    std::vector<hipEvent_t> root_sent(kBufs * n, nullptr);
    if (transport == RT_TRANSPORT_COPY) {
        if (hipSetDevice(devs[0]) != hipSuccess) { delete g; return rt_fail(RT_EHIP, "rt_group_create: hipSetDevice"); }
        for (int q = 0; q < n; ++q)
            for (int b = 0; b < kBufs; ++b) {
                if (hipEventCreateWithFlags(&root_sent[kBufs * q + b], hipEventDisableTiming) != hipSuccess)
                    rc = rt_fail(RT_EHIP, "rt_group_create: hipEventCreate failed");
                g->ranks[q].sent[b] = root_sent[kBufs * q + b];    // owned by the group from here on
            }
    }
    for (int q = 0; q < n && rc == RT_OK; ++q)
        rc = setup_rank(&g->ranks[q], ctxs[q], q, transport == RT_TRANSPORT_COPY ? &root_sent[kBufs * q] : nullptr);
    if (rc == RT_OK) rc = setup_root_events(g);
    if (rc == RT_OK && transport == RT_TRANSPORT_RCCL) {
        std::vector<ncclComm_t> comms(n);
        ncclResult_t r = ncclCommInitAll(comms.data(), n, devs.data());
        if (r != ncclSuccess) rc = rt_fail(RT_EHIP, std::string("ncclCommInitAll: ") + ncclGetErrorString(r));
        else
            for (int q = 0; q < n; ++q) g->ranks[q].comm = comms[q];
    }
    if (rc != RT_OK) {
        rt_group_destroy(g);
        return rc;
    }
    *out = g;
    return RT_OK;
}

extern "C" int rt_group_create_rank(rt_ctx* ctx, int n_ranks, int rank, const uint8_t* id, rt_group** out) {
    if (!out) return rt_fail(RT_EINVAL, "rt_group_create_rank: null out");
    *out = nullptr;
    if (!ctx || !id || n_ranks <= 0 || rank < 0 || rank >= n_ranks)
        return rt_fail(RT_EINVAL, "rt_group_create_rank: bad arguments");
    rt_group* g = new rt_group();
    if (const char* e = getenv("RT_GATHER_ROOT_WAITS")) g->root_waits = atoi(e) != 0;
    if (const char* e = getenv("RT_GROUP_RENDER_STREAMS")) g->render_streams = atoi(e) == 1 ? 1 : 2;
    if (const char* e = getenv("RT_GROUP_BUFFERS")) g->n_bufs = atoi(e) == 2 ? 2 : kBufs;
    g->n_ranks = n_ranks;
    g->transport = RT_TRANSPORT_RCCL;
    g->owns_root = rank == 0;
    g->ranks.resize(1);
    g->plan.resize(1);
    int rc = setup_rank(&g->ranks[0], ctx, rank, nullptr);
    if (rc == RT_OK && g->owns_root) rc = setup_root_events(g);
    if (rc == RT_OK) {
        ncclUniqueId u;
        memcpy(&u, id, sizeof(u));
        (void)hipSetDevice(g->ranks[0].device);
        ncclResult_t r = ncclCommInitRank(&g->ranks[0].comm, n_ranks, u, rank);
        if (r != ncclSuccess) rc = rt_fail(RT_EHIP, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
    }
    if (rc != RT_OK) {
        rt_group_destroy(g);
        return rc;
    }
    *out = g;
    return RT_OK;
}

extern "C" int rt_group_info(const rt_group* g, int* n_ranks, int* n_local, int* first_rank, int* transport) {
    if (!g) return rt_fail(RT_EINVAL, "rt_group_info: null group");
    if (n_ranks) *n_ranks = g->n_ranks;
    if (n_local) *n_local = (int)g->ranks.size();
    if (first_rank) *first_rank = g->ranks.empty() ? 0 : g->ranks[0].rank;
    if (transport) *transport = g->transport;
    return RT_OK;
}

extern "C" int rt_group_synchronize(rt_group* g) {
    if (!g) return rt_fail(RT_EINVAL, "rt_group_synchronize: null group");
    for (auto& r : g->ranks) {
        G_HIP(hipSetDevice(r.device));
        for (hipStream_t s : r.rs) G_HIP(hipStreamSynchronize(s));
        G_HIP(hipStreamSynchronize(r.cs));
    }
    return RT_OK;
}

// Timing events of ring slot `slot` for rank r, created on its device on first use.
int phase_events(Rank& r, int slot, bool root, PhaseEvents** out) {
    PhaseEvents& e = r.ph[slot];
    if (!e.r0) {
        G_HIP(hipSetDevice(r.device));
        for (hipEvent_t* ev : {&e.r0, &e.r1, &e.g0, &e.g1}) G_HIP(hipEventCreate(ev));
        if (root) G_HIP(hipEventCreate(&e.a1));
    }
    *out = &e;
    return RT_OK;
}

extern "C" int rt_group_timing(rt_group* g, int enable) {
    if (!g) return rt_fail(RT_EINVAL, "rt_group_timing: null group");
    int rc = rt_group_synchronize(g);
    if (rc) return rc;
    g->timing = enable != 0;
    g->t_first = g->frame;
    for (auto& r : g->ranks)
        for (auto& e : r.ph) e.rec = e.gather_rec = false;
    return RT_OK;
}

extern "C" int rt_group_get_stats(rt_group* g, rt_group_stats* st) {
    if (!g || !st) return rt_fail(RT_EINVAL, "rt_group_get_stats: null argument");
    int rc = rt_group_synchronize(g);
    if (rc) return rc;
    memset(st, 0, sizeof(*st));
    st->frames = (int32_t)(g->frame - g->t_first);
    st->wire_float = g->last_wire[0];
    st->wire_byte = g->last_wire[1];
    st->payload_bytes = g->last_payload;
    double sr = 0, sg = 0, sa = 0, sf = 0;
    int nr = 0, ng = 0, na = 0;
    for (size_t q = 0; q < g->ranks.size(); ++q) {
        Rank& r = g->ranks[q];
        bool any = false;
        G_HIP(hipSetDevice(r.device));
        for (auto& e : r.ph) {
            if (!e.rec) continue;
            any = true;
            // a one-rank group records on the caller's stream, which rt_group_synchronize does not wait for
            G_HIP(hipEventSynchronize(e.r1));
            if (e.gather_rec) G_HIP(hipEventSynchronize(e.g1));
            if (q == 0 && g->owns_root && e.a1) G_HIP(hipEventSynchronize(e.a1));
            float ms = 0.f;
            G_HIP(hipEventElapsedTime(&ms, e.r0, e.r1));
            if (e.rendered) sr += ms, ++nr;
            if (e.gather_rec) {
                G_HIP(hipEventElapsedTime(&ms, e.g0, e.g1));
                sg += ms, ++ng;
            }
            if (q == 0 && g->owns_root && e.a1) {
                G_HIP(hipEventElapsedTime(&ms, e.g1, e.a1));
                sa += ms;
                G_HIP(hipEventElapsedTime(&ms, e.r0, e.a1));
                sf += ms, ++na;
            }
        }
        st->ranks_timed += any ? 1 : 0;
    }
    st->render_ms = nr ? sr / nr : 0.0;
    st->gather_ms = ng ? sg / ng : 0.0;
    st->assemble_ms = na ? sa / na : 0.0;
    st->frame_ms = na ? sf / na : 0.0;
    return RT_OK;
}

// One process per GPU (rt_group_create_rank): each rank picks its wire formats from its own context's scene, so
// the ranks must hold the same scene or the byte counts of ncclSend / ncclRecv disagree (a hang or a torn frame).
// Whenever this rank's scene differs from the one the group last agreed on — every rank changes its scene between
// the same frames (include/rt_api.h, rt_render_multi) — the group all-reduces (max) the ranks' votes
// {h, ~h, a, ~a} of the scene fingerprint h and the achromatic flag a: every rank then sees min = max for both, or
// fails with RT_EINVAL.  The decisions are rt_group_plan.cpp's (rt_group_agree_*), driven without a GPU by the
// CPU tests; this function only adds the collective.
int agree_on_scene(rt_group* g, Rank& r, int achro) {
    (void)g;
    uint64_t gen = 0, h = 0;
    rt_ctx_scene_id(r.ctx, &gen, &h);
    if (!rt_group_agree_due(h, r.agreed ? 1 : 0, r.agreed_fp)) return RT_OK;
    G_HIP(hipSetDevice(r.device));
    if (!r.d_agree && hipMalloc(&r.d_agree, 4 * sizeof(uint64_t)) != hipSuccess)
        return rt_fail(RT_ENOMEM, "rt_render_multi: hipMalloc of the scene agreement buffer failed");
    uint64_t v[4];
    rt_group_agree_vote(h, achro, v);
    // on the comm stream, behind the previous frames' exchanges (collectives run in the same order on every rank)
    G_HIP(hipMemcpyAsync(r.d_agree, v, sizeof(v), hipMemcpyHostToDevice, r.cs));
    G_NCCL(ncclAllReduce(r.d_agree, r.d_agree, 4, ncclUint64, ncclMax, r.comm, r.cs));
    G_HIP(hipMemcpyAsync(v, r.d_agree, sizeof(v), hipMemcpyDeviceToHost, r.cs));
    G_HIP(hipStreamSynchronize(r.cs));
    int rc = rt_group_agree_verdict(v);
    if (rc) return rc;
    r.agreed = true;
    r.agreed_fp = h;
    return RT_OK;
}

extern "C" int rt_render_multi(rt_group* g, const rt_camera* cam, int W, int H, int depth, int band_height,
                               int outputs, float* rgba32f, uint8_t* rgba8, void* stream) {
    if (!g) return rt_fail(RT_EINVAL, "rt_render_multi: null group");
    if (!cam) return rt_fail(RT_EINVAL, "rt_render_multi: null camera");
    if (W <= 0 || H <= 0) return rt_fail(RT_EINVAL, "rt_render_multi: bad image size");
    if (outputs <= 0 || (outputs & ~(RT_OUT_RGBA32F | RT_OUT_RGBA8)))
        return rt_fail(RT_EINVAL, "rt_render_multi: outputs must be a non-empty set of RT_OUT_RGBA32F | RT_OUT_RGBA8");
    // Every rank passes the same `outputs` (it decides what travels); only rank 0's image pointers are used.
    const bool kind_on[kKinds] = {(outputs & RT_OUT_RGBA32F) != 0, (outputs & RT_OUT_RGBA8) != 0};
    void* outs[kKinds] = {rgba32f, rgba8};
    if (g->owns_root && ((kind_on[0] && !rgba32f) || (kind_on[1] && !rgba8)))
        return rt_fail(RT_EINVAL, "rt_render_multi: rank 0 needs a device image for every requested output");
    int rc = RT_OK;
    const int b = (int)(g->frame % (uint64_t)g->n_bufs);
    const int slot = (int)(g->frame % kRing);
    const hipStream_t st = (hipStream_t)stream;
    // Every local rank must hold the same scene: the frame is assembled from their bands, and the wire formats are
    // decided from rank 0's context.  The scene fingerprint (FNV-1a of the flattened record, the value the
    // one-process-per-GPU groups all-reduce below) is compared, not just the achromatic flag.
    const int achro = rt_ctx_achromatic(g->ranks[0].ctx);
    uint64_t gen0 = 0, fp0 = 0;
    rt_ctx_scene_id(g->ranks[0].ctx, &gen0, &fp0);
    for (auto& r : g->ranks) {
        uint64_t gen = 0, fp = 0;
        rt_ctx_scene_id(r.ctx, &gen, &fp);
        if (fp != fp0 || rt_ctx_achromatic(r.ctx) != achro)
            return rt_fail(RT_EINVAL, "rt_render_multi: the ranks' contexts hold different scenes");
    }
    // ... and across the processes of a one-process-per-GPU group
    if (g->n_ranks > 1 && (int)g->ranks.size() < g->n_ranks && (rc = agree_on_scene(g, g->ranks[0], achro)))
        return rc;
    // What every rank sends and where rank 0's receives land: the host-only plan (rt_group_plan.cpp), one per local
    // rank, plus rank 0's (its receive table and payload) — the same plan the CPU tests check across processes.
    const int key[5] = {W, H, band_height, outputs, achro};
    if (!g->plan_valid || memcmp(key, g->plan_key, sizeof(key)) != 0) {
        g->plan_valid = false;
        for (size_t q = 0; q < g->ranks.size(); ++q)
            if ((rc = rt_group_plan_frame(W, H, g->n_ranks, g->ranks[q].rank, band_height, outputs, achro, &g->plan[q])))
                return rc;
        if ((rc = rt_group_plan_frame(W, H, g->n_ranks, 0, band_height, outputs, achro, &g->root_plan))) return rc;
        memcpy(g->plan_key, key, sizeof(key));
        g->plan_valid = true;
    }
    const std::vector<rt_group_plan>& plan = g->plan;
    const rt_group_plan& root_plan = g->root_plan;
    const int hb = root_plan.band_height, slab_rows = root_plan.slab_rows;
    // rank 0 renders bands too (root_renders), or bands go to ranks 1 .. n - 1 (renderers) and it only assembles
    const bool root_renders = root_plan.root_renders != 0;
    const int renderers = root_plan.renderers;
    // (the render call takes a format for an image it does not write too)
    const int wire[kKinds] = {achro ? RT_PIXEL_GRAY32F : RT_PIXEL_RGBA32F, achro ? RT_PIXEL_GRAY8 : RT_PIXEL_RGB8};
    for (int k = 0; k < kKinds; ++k) g->last_wire[k] = root_plan.wire[k];

    // ---- one rank: the band plan is the identity, so the frame is rendered straight into the caller's image
    // on the caller's stream (no slab, no unshuffle, no cross-stream hand-off: each one costs ~30 us) ----
    if (g->n_ranks == 1) {
        Rank& r = g->ranks[0];
        G_HIP(hipSetDevice(r.device));
        PhaseEvents* e = nullptr;
        if (g->timing && (rc = phase_events(r, slot, true, &e))) return rc;
        if (e) G_HIP(hipEventRecord(e->r0, st));
        rc = rt_render_dev(r.ctx, cam, W, H, depth, nullptr, kind_on[0] ? rgba32f : nullptr,
                           kind_on[1] ? rgba8 : nullptr, nullptr, nullptr, st);
        if (rc) return rc;
        if (e) {
            G_HIP(hipSetDevice(r.device));
            G_HIP(hipEventRecord(e->r1, st));
            G_HIP(hipEventRecord(e->g1, st));
            G_HIP(hipEventRecord(e->a1, st));
            e->rec = true;
            e->gather_rec = false;
        }
        g->last_band = hb;
        g->last_slab_rows = slab_rows;
        g->last_payload = 0;
        ++g->frame;
        return RT_OK;
    }

    // ---- buffers (grow-only).  A buffer that must grow may still be in use by frame - n_bufs (a peer copy or an RCCL
    // receive on the root, a send on a rank, the root's unshuffle): wait for the group and the caller's stream
    // first, whatever changed (width, band plan, outputs, wire format). ----
    bool must_grow = false;
    for (size_t q = 0; q < g->ranks.size(); ++q)
        for (int k = 0; k < kKinds; ++k)
            must_grow |= kind_on[k] && plan[q].slab_bytes[k] > g->ranks[q].slab_cap[b][k];
    if (g->owns_root)
        for (int k = 0; k < kKinds; ++k)
            must_grow |= kind_on[k] && root_plan.gather_bytes[k] > g->gathered_cap[b][k];
    if (must_grow && g->frame > 0) {
        rc = rt_group_synchronize(g);
        if (rc) return rc;
        if (g->owns_root) {
            G_HIP(hipSetDevice(g->ranks[0].device));
            G_HIP(hipStreamSynchronize(st));
        }
    }
    g->last_band = hb;
    g->last_slab_rows = slab_rows;
    for (size_t q = 0; q < g->ranks.size(); ++q) {
        Rank& r = g->ranks[q];
        G_HIP(hipSetDevice(r.device));
        for (int k = 0; k < kKinds; ++k)
            if (kind_on[k] && (rc = grow(&r.slab[b][k], &r.slab_cap[b][k], plan[q].slab_bytes[k]))) return rc;
    }
    if (g->owns_root) {
        G_HIP(hipSetDevice(g->ranks[0].device));
        for (int k = 0; k < kKinds; ++k)
            if (kind_on[k] && (rc = grow(&g->gathered[b][k], &g->gathered_cap[b][k], root_plan.gather_bytes[k])))
                return rc;
    }
    PhaseEvents* pe_fixed[8] = {};             // (no allocation per frame for up to 8 local ranks)
    std::vector<PhaseEvents*> pe_more;
    PhaseEvents** pe = pe_fixed;
    if (g->ranks.size() > 8) {
        pe_more.assign(g->ranks.size(), nullptr);
        pe = pe_more.data();
    }
    if (g->timing)
        for (size_t q = 0; q < g->ranks.size(); ++q)
            if ((rc = phase_events(g->ranks[q], slot, q == 0 && g->owns_root, &pe[q]))) return rc;

    // ---- render: every local rank's bands into slab[b], in the wire formats ---------------------------------
    // (rs[k]: the other render stream than the previous frame's for an unchanged camera; RT_GROUP_RENDER_STREAMS=1: one)
    const bool same_view = g->last_cam_valid && memcmp(&g->last_cam, cam, sizeof(rt_camera)) == 0;
    for (size_t q = 0; q < g->ranks.size(); ++q) {
        Rank& r = g->ranks[q];
        const int k = g->render_streams > 1 && same_view ? 1 - r.last_rs : r.last_rs;
        const hipStream_t rs = r.rs[k];
        r.last_rs = k;
        G_HIP(hipSetDevice(r.device));
        if (r.sent_rec[b]) G_HIP(hipStreamWaitEvent(rs, r.sent[b], 0));       // slab[b] has left (frame - n_bufs)
        if (r.rank == 0 && g->assembled_rec[b])                               // the root's slab[b] is read by
            G_HIP(hipStreamWaitEvent(rs, g->assembled[b], 0));                // frame - n_bufs's unshuffle
        if (pe[q]) {
            G_HIP(hipEventRecord(pe[q]->r0, rs));
            pe[q]->rendered = r.rank != 0 || root_renders;
        }
        if (r.rank != 0 || root_renders) {                   // (an assembling rank 0 renders nothing)
            rt_rows rows = {hb, renderers, root_renders ? r.rank : r.rank - 1, 1};
            rc = rt_render_dev_packed(r.ctx, cam, W, H, depth, &rows, wire[0], kind_on[0] ? r.slab[b][0] : nullptr,
                                      wire[1], kind_on[1] ? r.slab[b][1] : nullptr, rs);
            if (rc) return rc;
        }
        G_HIP(hipSetDevice(r.device));
        if (pe[q]) G_HIP(hipEventRecord(pe[q]->r1, rs));
        G_HIP(hipEventRecord(r.rendered[b], rs));
    }
    g->last_cam = *cam;
    g->last_cam_valid = true;

    // ---- gather to rank 0 ------------------------------------------------------------------------------------
    // rank 0's receive from peer q for image k: offset into gathered[b][k] and bytes (= q's send_bytes[k])
    auto recv_of = [&](int q, int k, uint64_t* off, uint64_t* bytes) {
        return rt_group_plan_recv(&root_plan, W, H, q, k, off, bytes);
    };
    g->last_payload = root_plan.payload_bytes;
    if (g->owns_root) {
        Rank& root = g->ranks[0];
        G_HIP(hipSetDevice(root.device));
        if (g->assembled_rec[b]) G_HIP(hipStreamWaitEvent(root.cs, g->assembled[b], 0));   // gathered[b] is free
    }
    if (g->transport == RT_TRANSPORT_RCCL) {
        for (size_t q = 0; q < g->ranks.size(); ++q) {
            Rank& r = g->ranks[q];
            G_HIP(hipSetDevice(r.device));
            // a sender waits for its slab; the root's receives land in gathered[b], which does not depend on the
            // root's own render: they are posted at once (the root's slab is waited for by the unpack below)
            if (r.rank != 0 || g->root_waits) G_HIP(hipStreamWaitEvent(r.cs, r.rendered[b], 0));
            if (pe[q]) G_HIP(hipEventRecord(pe[q]->g0, r.cs));
        }
        G_NCCL(ncclGroupStart());
        for (size_t lq = 0; lq < g->ranks.size(); ++lq) {
            Rank& r = g->ranks[lq];
            for (int k = 0; k < kKinds; ++k) {
                if (!kind_on[k]) continue;
                ncclResult_t e = ncclSuccess;
                if (r.rank != 0) e = ncclSend(r.slab[b][k], plan[lq].send_bytes[k], ncclUint8, 0, r.comm, r.cs);
                if (e != ncclSuccess) {
                    (void)ncclGroupEnd();
                    return rt_fail(RT_EHIP, std::string("ncclSend: ") + ncclGetErrorString(e));
                }
                if (r.rank != 0) continue;
                for (int q = 1; q < g->n_ranks; ++q) {        // the root's own slab is unshuffled in place
                    uint64_t off = 0, bytes = 0;
                    if ((rc = recv_of(q, k, &off, &bytes))) {
                        (void)ncclGroupEnd();
                        return rc;
                    }
                    e = ncclRecv((char*)g->gathered[b][k] + off, bytes, ncclUint8, q, r.comm, r.cs);
                    if (e != ncclSuccess) {
                        (void)ncclGroupEnd();
                        return rt_fail(RT_EHIP, std::string("ncclRecv: ") + ncclGetErrorString(e));
                    }
                }
            }
        }
        G_NCCL(ncclGroupEnd());
        for (size_t q = 0; q < g->ranks.size(); ++q) {
            Rank& r = g->ranks[q];
            G_HIP(hipSetDevice(r.device));
            if (pe[q]) {
                G_HIP(hipEventRecord(pe[q]->g1, r.cs));
                pe[q]->gather_rec = true;
            }
            G_HIP(hipEventRecord(r.sent[b], r.cs));
            r.sent_rec[b] = true;
        }
    } else {
        Rank& root = g->ranks[0];
        G_HIP(hipSetDevice(root.device));
        // the root's gather: from the frame's hand-off to the last peer copy; each copy waits only for its own
        // rank's render (the root's slab is waited for by the unpack below)
        if (g->root_waits) G_HIP(hipStreamWaitEvent(root.cs, root.rendered[b], 0));
        if (pe[0]) G_HIP(hipEventRecord(pe[0]->g0, root.cs));
        for (auto& r : g->ranks) {
            if (r.rank != 0) G_HIP(hipStreamWaitEvent(root.cs, r.rendered[b], 0));
            for (int k = 0; k < kKinds; ++k) {
                if (!kind_on[k] || r.rank == 0) continue;      // the root's own slab is unshuffled in place
                uint64_t off = 0, bytes = 0;
                if ((rc = recv_of(r.rank, k, &off, &bytes))) return rc;
                G_HIP(hipMemcpyPeerAsync((char*)g->gathered[b][k] + off, root.device, r.slab[b][k], r.device, bytes,
                                         root.cs));
            }
            G_HIP(hipEventRecord(r.sent[b], root.cs));
            r.sent_rec[b] = true;
        }
        if (pe[0]) {
            G_HIP(hipEventRecord(pe[0]->g1, root.cs));
            pe[0]->gather_rec = true;
        }
    }

    // ---- assemble on rank 0 (high-priority comm stream), ordered before the caller's stream's later work ----
    // The caller's image is written by this frame's unshuffle: its stream waits for `received` (the previous
    // frame's image may still be read there) before the unshuffle is queued behind it on the comm stream.
    if (g->owns_root) {
        Rank& root = g->ranks[0];
        G_HIP(hipSetDevice(root.device));
        G_HIP(hipEventRecord(g->received[b], st));                   // caller's earlier work on the image
        G_HIP(hipStreamWaitEvent(root.cs, g->received[b], 0));
        if (root_renders) G_HIP(hipStreamWaitEvent(root.cs, root.rendered[b], 0));     // the root's own slab
        for (int k = 0; k < kKinds; ++k) {
            if (!kind_on[k]) continue;
            rc = rt_unpack_dev_ex(g->gathered[b][k], root_renders ? root.slab[b][k] : nullptr, outs[k], W, H, wire[k],
                                  kImageFormat[k], hb, renderers, slab_rows, root.cs);
            if (rc) return rc;
        }
        G_HIP(hipSetDevice(root.device));
        if (pe[0]) G_HIP(hipEventRecord(pe[0]->a1, root.cs));
        G_HIP(hipEventRecord(g->assembled[b], root.cs));
        G_HIP(hipStreamWaitEvent(st, g->assembled[b], 0));
        g->assembled_rec[b] = true;
    }
    for (size_t q = 0; q < g->ranks.size(); ++q)
        if (pe[q]) pe[q]->rec = true;
    ++g->frame;
    return RT_OK;
}
