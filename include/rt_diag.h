/*
 * rt_diag.h — diagnostics exported by librt_amd.so beside the drop-in boundary (rt_api.h).
 *
 * Not part of the reference's interface: these entry points exist so the parity tests can check the
 * device arithmetic the render kernel relies on, operand by operand, against the compiler's IEEE
 * sequences (and, on the host, against binary64 arithmetic as the reference's Point does it,
 * Hw4/MySdlApplication.cpp:174-175).
 */
#ifndef RT_DIAG_H
#define RT_DIAG_H

#include "rt_api.h"

#ifdef __cplusplus
extern "C" {
#endif

/* op 0: for each of n vectors v (3 doubles, device memory) write 9 doubles (device memory):
 *   [0..2] v / |v| and [3] |v| with the compiler's sqrt and division (Point::normalize / length),
 *   [4..7] the same from the render kernel's fast path (unit), [8] its len_fast(v).
 * op 1: for each of n pairs (a, b) write 2 doubles: a / b (the compiler's IEEE division) and the render
 * kernel's division with a shared reciprocal (div_core(a, b, rcp_core(b)), used by the checker).
 * Asynchronous on `stream`.  RT_EINVAL for an unknown op or null buffers. */
int rt_probe_math_dev(int op, const double* in, int n, double* out, void* stream);

/* The scene agreement of a one-process-per-GPU group (rt_render_multi), without its collective, so the CPU tests
 * drive it from several processes.  rt_group_agree_due: 1 when a rank whose scene has `fingerprint` must vote
 * before its next frame (it differs from the last agreed one, or nothing was agreed yet).  rt_group_agree_vote:
 * this rank's vote {h, ~h, a, ~a}.  rt_group_agree_combine: acc = element-wise unsigned max(acc, other) — what the
 * group's ncclAllReduce(ncclMax) computes.  rt_group_agree_verdict: RT_OK when the combined votes of every rank
 * name one scene (fingerprint and achromatic flag), else RT_EINVAL. */
int rt_group_agree_due(uint64_t fingerprint, int agreed, uint64_t agreed_fingerprint);
void rt_group_agree_vote(uint64_t fingerprint, int achromatic, uint64_t vote[4]);
void rt_group_agree_combine(uint64_t acc[4], const uint64_t other[4]);
int rt_group_agree_verdict(const uint64_t reduced[4]);

/* Tile-row dispatch order of later rt_render_dev calls of this context: mode 0 (default) adaptive — the
 * first render of a new (scene, camera, size, row plan, depth) times its 8-row tile rows and later
 * renders dispatch them longest first; mode 1 bottom-to-top.  Images are identical either way (every
 * tile is traced once, by the same code).  RT_EINVAL for another mode. */
int rt_diag_tile_order(rt_ctx* ctx, int mode);

/* Registers per work-item (*vgprs) and private scratch bytes per work-item (*scratch_bytes) of the render
 * kernel instance rt_render_dev launches for `depth` (0..7) and scene kind `variant`: 0 spheres + board,
 * 1 >= 16 spheres (wave-culling variant), 2 meshes or transparent materials, 3 ray trees (whose node stack
 * lives in scratch by design), 4 / 5 the achromatic (one-channel) instances of 0 / 1 (depth <= 3; RT_EINVAL
 * for deeper ones).  Needs a HIP device.  RT_EINVAL for bad arguments. */
int rt_diag_kernel_resources(int depth, int variant, int* vgprs, int* scratch_bytes);

/* Workgroups per CU the HIP runtime allows the render kernel (depth, variant) with lds_bytes of dynamic LDS. */
int rt_diag_kernel_occupancy(int depth, int variant, int lds_bytes, int* blocks_per_cu);

/* How this context's last rt_render_packed / rt_render_packed_async frame reached host memory: *mode 0 the copy
 * kernel on the copy stream, 1 behind the render on the render stream (copy kernel, or hipMemcpyAsync for pageable
 * memory), 2 stored by the render straight into mapped pinned memory, 3 an SDMA engine, -1 no packed frame yet;
 * *writer how an SDMA frame's start is signalled (1 the stream's write-value operation, 2 a one-wave kernel, 0 the
 * engine is not set up).  RT_EINVAL for a null context. */
int rt_diag_copy_path(rt_ctx* ctx, int* mode, int* writer);

#ifdef __cplusplus
}
#endif

#endif /* RT_DIAG_H */
