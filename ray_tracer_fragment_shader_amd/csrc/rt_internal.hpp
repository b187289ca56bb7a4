// rt_internal.hpp — host-side helpers shared by rt_host.cpp and rt_kernel.hip (not part of the ABI).
#pragma once

#include <stdint.h>

#include <string>
#include <vector>

#include "../../include/rt_api.h"
#include "rt_layout.hpp"

// Record `msg` as this thread's rt_last_error() and return `code`.
int rt_fail(int code, const std::string& msg);

// FNV-1a 64 of a flattened scene record (rt_scene_fingerprint; the context's scene_hash).
uint64_t rt_blob_fingerprint(const std::vector<unsigned char>& blob);

// Validate an rt_scene and flatten it into the device record (rt::DevScene followed by the spheres),
// precomputing every derived quantity with the reference's operation order.
int rt_build_dev_scene(const rt_scene* scene, std::vector<unsigned char>* blob);

// rayTraceScreen basis (MySdlApplication.cpp:1270-1277): right = normalize(LD x up),
// up' = normalize(right x LD), LD = look_at - eye.
void rt_camera_basis(const rt_camera* cam, double right[3], double upp[3]);

// Device ordinal of a context (rt_group.cpp).
int rt_ctx_device(const rt_ctx* ctx);

// 1 when the context's uploaded scene is achromatic (rt_scene_achromatic): GRAY pixel formats are exact.
int rt_ctx_achromatic(const rt_ctx* ctx);

// The context's scene generation (changes with every rt_set_scene that uploads a different scene) and a
// fingerprint of the uploaded record (FNV-1a of the flattened scene): rt_group.cpp agrees on the scene — hence
// on the wire formats — across the processes of a group whenever a rank's fingerprint differs from the agreed one.
void rt_ctx_scene_id(const rt_ctx* ctx, uint64_t* gen, uint64_t* fingerprint);

// rt_unshuffle_dev with rank 0's rows read from `rank0_slab` instead of the gathered buffer (the group's root
// unshuffles its own slab in place of sending it to itself); rank0_slab = nullptr: from `gathered`.
int rt_unshuffle_dev_ex(const void* gathered, const void* rank0_slab, void* image, int W, int H, int elem_bytes,
                        int band_height, int n_ranks, int slab_rows, void* stream);

// rt_unpack_dev with rank 0's rows read from `rank0_slab` (as rt_unshuffle_dev_ex).
int rt_unpack_dev_ex(const void* gathered, const void* rank0_slab, void* image, int W, int H, int src_format,
                     int dst_format, int band_height, int n_ranks, int slab_rows, void* stream);

// rt_render_screen's chunk traced in one launch (rt_kernel.hip): ray k of the chunk, window entry j of pixel q
// (pix[q].off <= k < pix[q].off + pix[q].len), is Line(cam, pix[q].sp + 0.5 * jit[pix[q].base + j])
// (ray.set(camera, screenPt + .5 * randomUnit()), MSA:1296); first[b] = the pixel of ray b * kScreenBlock.
// All pointers device-visible; n rays, m pixels.
// done (nullable, device-visible, one word per workgroup of kScreenBlock rays): each workgroup stores `seq` into its
// word after its colours are visible system-wide, so the host can resolve a chunk while it is still being traced.
int rt_trace_screen_dev(rt_ctx* c, const double cam[3], const ScreenPix* pix, const int32_t* first, int m,
                        const double* jit, int n, int depth, double* rgb64f, uint32_t* done, uint32_t seq,
                        void* stream);
constexpr int kScreenMaxRays = 1 << 19;        // rays of one chunk
constexpr int kScreenMaxPix = 4096;            // pixels of one chunk
constexpr int kScreenMaxJit = kScreenMaxPix * 16 + kScreenMaxWindow;   // stream values of one chunk
constexpr int kScreenMaxBlocks = (kScreenMaxRays + kScreenBlock - 1) / kScreenBlock;
// Frees the rt_render_screen buffers kept for `ctx` (rt_ctx_destroy).
void rt_screen_release(const rt_ctx* ctx);
