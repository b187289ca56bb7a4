// rt_group_plan.cpp — the host-side decisions of rt_render_multi (rt_group.cpp) that involve no device: what each
// rank of a row-banded frame sends, what rank 0 receives and where it lands, and the scene agreement of a
// one-process-per-GPU group.  Plain C++ (no HIP), so the CPU tests drive the same code from two gloo processes
// (tests/test_distributed.py) and the sanitizer leg links it.
//
// The reference renders one frame on one thread (rayTraceScreen, Hw4/MySdlApplication.cpp:1251-1324); the whole
// multi-GPU split is this build's.  Pixels are independent (rayTraceRay :1184-1249 reads only the
// scene), so a frame splits into round-robin row bands (rt_band_plan) gathered to rank 0.
#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "../../include/rt_api.h"
#include "../../include/rt_diag.h"
#include "rt_internal.hpp"

namespace {

constexpr int kKinds = 2;                                 // 0: the RGBA32F image, 1: the RGBA8 image

int local_rows(int height, int band, int n_ranks, int rank) {
    rt_rows r = {band, n_ranks, rank, 1};
    int nl = 0;
    return rt_local_rows(height, &r, &nl) == RT_OK ? nl : -1;
}

}  // namespace

extern "C" int rt_group_root_renders(int n_ranks) {
    if (const char* e = getenv("RT_GROUP_ROOT_RENDERS")) return atoi(e) != 0 ? 1 : 0;
    return n_ranks < 4 ? 1 : 0;
}

extern "C" int rt_group_plan_frame(int width, int height, int n_ranks, int rank, int band_height, int outputs,
                                   int achromatic, rt_group_plan* out) {
    if (!out || width <= 0 || height <= 0 || n_ranks <= 0 || rank < 0 || rank >= n_ranks)
        return rt_fail(RT_EINVAL, "rt_group_plan_frame: bad arguments");
    if (outputs <= 0 || (outputs & ~(RT_OUT_RGBA32F | RT_OUT_RGBA8)))
        return rt_fail(RT_EINVAL, "rt_group_plan_frame: outputs must be a non-empty set of RT_OUT_RGBA32F | RT_OUT_RGBA8");
    rt_group_plan p;
    std::memset(&p, 0, sizeof(p));
    // the bands go to the renderers: every rank, or ranks 1 .. n - 1 when rank 0 only assembles
    p.root_renders = n_ranks == 1 ? 1 : rt_group_root_renders(n_ranks);
    p.renderers = p.root_renders ? n_ranks : n_ranks - 1;
    const int rr = p.root_renders ? rank : rank - 1;           // this rank's renderer index, -1: none
    int rc = rt_band_plan(height, p.renderers, band_height, &p.band_height, &p.slab_rows);
    if (rc) return rc;
    p.n_ranks = n_ranks;
    p.rank = rank;
    p.rank_rows = rr >= 0 ? local_rows(height, p.band_height, p.renderers, rr) : 0;
    if (p.rank_rows < 0) return rt_fail(RT_EINVAL, "rt_group_plan_frame: row plan");
    // Wire formats: the narrowest exact one (GRAY for achromatic scenes, whose pixels have R = G = B bit for bit)
    const bool on[kKinds] = {(outputs & RT_OUT_RGBA32F) != 0, (outputs & RT_OUT_RGBA8) != 0};
    const int wire[kKinds] = {achromatic ? RT_PIXEL_GRAY32F : RT_PIXEL_RGBA32F, achromatic ? RT_PIXEL_GRAY8 : RT_PIXEL_RGB8};
    for (int k = 0; k < kKinds; ++k) {
        p.wire[k] = on[k] ? wire[k] : -1;
        if (!on[k]) continue;
        int pb = 0;
        if ((rc = rt_pixel_bytes(wire[k], &pb))) return rc;
        p.elem_bytes[k] = pb;
        const uint64_t slot = (uint64_t)p.slab_rows * width * pb;
        p.slab_bytes[k] = rr >= 0 ? slot : 0;                   // (an assembling rank 0 has no slab)
        // rank 0 unpacks its own slab in place instead of sending it to itself
        p.send_bytes[k] = rank == 0 || n_ranks == 1 ? 0 : (uint64_t)p.rank_rows * width * pb;
        if (rank == 0 && n_ranks > 1) {
            p.gather_bytes[k] = (uint64_t)p.renderers * slot;
            for (int r = p.root_renders ? 1 : 0; r < p.renderers; ++r)
                p.payload_bytes += (uint64_t)local_rows(height, p.band_height, p.renderers, r) * width * pb;
        }
    }
    *out = p;
    return RT_OK;
}

extern "C" int rt_group_plan_recv(const rt_group_plan* p, int width, int height, int peer, int kind, uint64_t* offset,
                                  uint64_t* bytes) {
    if (!p || !offset || !bytes || kind < 0 || kind >= kKinds || peer < 1 || peer >= p->n_ranks || p->rank != 0 ||
        width <= 0 || height <= 0)
        return rt_fail(RT_EINVAL, "rt_group_plan_recv: bad arguments (rank 0's plan, peers 1 .. n_ranks - 1)");
    if (p->wire[kind] < 0) return rt_fail(RT_EINVAL, "rt_group_plan_recv: that image is not requested");
    const int rr = p->root_renders ? peer : peer - 1;         // the peer's renderer index
    const int nl = local_rows(height, p->band_height, p->renderers, rr);
    if (nl < 0) return rt_fail(RT_EINVAL, "rt_group_plan_recv: row plan");
    // the peer's rows land in its renderer's slab-sized slot of rank 0's gather buffer (when rank 0 renders, slot 0
    // stays unused: its rows are read from its own slab by the unpack), which is the layout rt_unpack_dev reads
    *offset = (uint64_t)rr * p->slab_rows * width * p->elem_bytes[kind];
    *bytes = (uint64_t)nl * width * p->elem_bytes[kind];
    return RT_OK;
}

// ---- scene agreement (rt_diag.h) -------------------------------------------------------------------------------
// Each rank picks its wire formats from its own context's scene, so the group must hold one scene: otherwise the
// byte counts of ncclSend / ncclRecv disagree.  A rank votes {h, ~h, a, ~a} (scene fingerprint h, achromatic flag a);
// the element-wise unsigned maximum over the group (ncclAllReduce with ncclMax) has max(h) = ~max(~h) = ~(~min(h)),
// i.e. v[0] == ~v[1] exactly when min(h) == max(h), and likewise for a.

extern "C" int rt_group_agree_due(uint64_t fingerprint, int agreed, uint64_t agreed_fingerprint) {
    // due when this rank's scene differs from the one the group last agreed on (not on every re-upload: a rank that
    // goes X -> Y -> X between two frames holds the agreed scene again and must not enter the all-reduce alone)
    return !agreed || fingerprint != agreed_fingerprint ? 1 : 0;
}

extern "C" void rt_group_agree_vote(uint64_t fingerprint, int achromatic, uint64_t vote[4]) {
    const uint64_t a = achromatic ? 1u : 0u;
    vote[0] = fingerprint;
    vote[1] = ~fingerprint;
    vote[2] = a;
    vote[3] = ~a;
}

extern "C" void rt_group_agree_combine(uint64_t acc[4], const uint64_t other[4]) {
    for (int i = 0; i < 4; ++i) acc[i] = std::max(acc[i], other[i]);
}

extern "C" int rt_group_agree_verdict(const uint64_t reduced[4]) {
    if (reduced[0] != ~reduced[1] || reduced[2] != ~reduced[3])
        return rt_fail(RT_EINVAL, "rt_render_multi: the group's ranks hold different scenes (wire formats would "
                                  "disagree); call rt_set_scene with the same scene on every rank");
    return RT_OK;
}

extern "C" int rt_scene_fingerprint(const rt_scene* scene, uint64_t* out) {
    if (!out) return rt_fail(RT_EINVAL, "rt_scene_fingerprint: null output");
    std::vector<unsigned char> blob;
    int rc = rt_build_dev_scene(scene, &blob);
    if (rc) return rc;
    *out = rt_blob_fingerprint(blob);
    return RT_OK;
}

uint64_t rt_blob_fingerprint(const std::vector<unsigned char>& blob) {
    uint64_t fp = 0xcbf29ce484222325ull;                  // FNV-1a 64 of the flattened record
    for (unsigned char byte : blob) fp = (fp ^ byte) * 0x100000001b3ull;
    return fp;
}
