/*
 * rt_api.h — C ABI of the MI355X-native per-pixel ray tracer.
 *
 * This is the drop-in boundary for the reference's frame hand-off:
 *   draw()            Hw4/MySdlApplication.cpp:1541-1563  (builds lights + camera, calls L5)
 *   rayTraceScreen()  Hw4/MySdlApplication.cpp:1251-1324  (camera basis, per-pixel rays, GL emit)
 *   rayTraceRay()     Hw4/MySdlApplication.cpp:1184-1249  (closest hit, shadows, bounces)
 *   Shape/Triangle/CheckerBoard::intersection  MySdlApplication.cpp:611-823, 1084-1113
 * The reference has no plugin/FFI API: its seam is a C++ call made on the GL thread.
 * This header replaces that call with plain C types: the scene is a flat descriptor built from the
 * same inputs `loadScene` uses (MySdlApplication.cpp:1495-1539), pixels land in caller-owned buffers.
 *
 * Conventions
 *  - All geometry is IEEE binary64, exactly as the reference's `Point` (MySdlApplication.cpp:136-212).
 *  - Pixel (i, j) has j = 0 at the BOTTOM row (gluOrtho2D(0,W,0,H), MySdlApplication.cpp:1383) and is
 *    stored at index j*W + i of a full image.  A row-banded call (rt_rows) stores its rows densely in
 *    local order; rt_unshuffle_dev puts gathered bands back into image order.
 *  - Every entry point returns RT_OK (0) or a negative RT_E* code; rt_last_error() gives the text for
 *    the calling thread.  There is no silent fallback: without a HIP device every render call fails
 *    with RT_EHIP.
 *  - One rt_ctx per (thread, device).  A context owns the device copy of the scene; rt_render_dev is
 *    asynchronous on the caller's stream and does not allocate, so it may be captured in a hipGraph.
 *    A context's renders must be stream-ordered (one stream at a time): a render may update the
 *    context's per-camera data (sphere data for a new eye, the tile-row dispatch order).
 *  - hipGraph capture: a captured render is self-contained (it carries its own per-eye preparation and
 *    uses the identity tile-row order), so renders of other views between replays do not disturb it.
 *    rt_set_scene with a different scene invalidates captured graphs (the scene record may move).
 *  - Multi-GPU: rt_group + rt_render_multi split a frame's rows over GPUs and gather
 *    them to rank 0 over RCCL (one process driving several GPUs, or one process per GPU).
 */
#ifndef RT_API_H
#define RT_API_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RT_ABI_VERSION 7

#define RT_OK            0
#define RT_EINVAL       -1   /* bad argument (null pointer, size, unsupported material, ...) */
#define RT_EHIP         -2   /* HIP runtime error or no device */
#define RT_ENOMEM       -3   /* allocation failed */
#define RT_EUNSUPPORTED -4   /* reference feature outside the GPU path (cylinder/cone stubs) */

#define RT_MAX_SPHERES 1024
#define RT_MAX_LIGHTS  16
#define RT_MAX_MESHES  64
#define RT_MAX_DEPTH   7     /* reference uses MAX_DEPTH = 5 (MySdlApplication.cpp:48) */

#define RT_MESH_TETRAHEDRON 1   /* Tetrahedron(p, edgeSize), MySdlApplication.cpp:863-900 */
#define RT_MESH_CUBE        2   /* Cube(p, edgeSize),        MySdlApplication.cpp:903-950 */

/* Material — MySdlApplication.cpp:272-307 (ambient, diffuse, specular, transparency, refraction). */
typedef struct rt_material {
    double ambient[3];
    double diffuse[3];
    double specular[3];
    double transparency[3];
    double refraction;
} rt_material;

/* Sphere(p, r) — MySdlApplication.cpp:846-860.  `center` is scene-local, exactly the `p` handed to the
 * reference constructor (e.g. convertStringCoordinate("d7")); the world centre is center + scene.position. */
typedef struct rt_sphere {
    double center[3];
    double radius;
} rt_sphere;

/* Light(color, position) — MySdlApplication.cpp:214-232.  World coordinates. */
typedef struct rt_light {
    double color[3];
    double position[3];
} rt_light;

/* A triangle-mesh composite of the reference: a Shape with a bounding sphere of radius
 * sqrt(3)*edge/2 around `position` and triangle sub-objects (tetrahedron: 4 triangles; cube: 6 Quads of
 * 2 triangles), material g_tetrahedronMaterial / g_cubeMaterial.  `position` is scene-local, the `p`
 * handed to the constructor.  g_scene child order: the mesh comes after `after_spheres` spheres (and
 * after every mesh listed before it). */
typedef struct rt_mesh {
    int32_t kind;                /* RT_MESH_TETRAHEDRON or RT_MESH_CUBE */
    int32_t after_spheres;
    double position[3];
    double edge;
} rt_mesh;

/* The reference's g_scene (MySdlApplication.cpp:590) flattened: a bounding sphere at `position` of
 * `radius`, then children in insertion order — the CheckerBoard first when present (initScene2 inserts
 * it first, MySdlApplication.cpp:1442-1443), then spheres and meshes in the order given (see rt_mesh). */
typedef struct rt_scene {
    double position[3];          /* g_scene position, BOARD_POSITION (MySdlApplication.cpp:42) */
    double radius;               /* g_scene radius sqrt(3)*BOARD_HALF_SIZE; <= 0 disables the cull */
    int32_t has_board;           /* CheckerBoard present */
    int32_t n_spheres;           /* <= RT_MAX_SPHERES */
    int32_t n_lights;            /* <= RT_MAX_LIGHTS */
    int32_t reserved0;
    double board_position[3];    /* CheckerBoard(p) argument (scene-local) */
    double board_half_size;      /* BOARD_HALF_SIZE (MySdlApplication.cpp:44) */
    double square_edge_size;     /* SQUARE_EDGE_SIZE (MySdlApplication.cpp:46) */
    double small_number;         /* SMALL_NUMBER (MySdlApplication.cpp:50) */
    double attenuation_factor;   /* ATTENUATION_FACTOR (MySdlApplication.cpp:35) */
    rt_material white_square;    /* g_whiteSquare (MySdlApplication.cpp:583) */
    rt_material black_square;    /* g_blackSquare (MySdlApplication.cpp:585) */
    rt_material sphere_material; /* g_sphereMaterial (MySdlApplication.cpp:586) */
    const rt_sphere* spheres;    /* host pointer, n_spheres entries */
    const rt_light* lights;      /* host pointer, n_lights entries (the per-frame `lights` vector) */
    rt_material tetrahedron_material;  /* g_tetrahedronMaterial (MySdlApplication.cpp:587) */
    rt_material cube_material;         /* g_cubeMaterial (MySdlApplication.cpp:588) */
    int32_t n_meshes;            /* <= RT_MAX_MESHES */
    int32_t reserved1;
    const rt_mesh* meshes;       /* host pointer, n_meshes entries */
} rt_scene;

/* Camera — rayTraceScreen's arguments (MySdlApplication.cpp:1251-1252, called at :1560).
 * Primary ray of pixel (i, j): Line(eye, sp) with
 *   sp = (look_at + (pitch*(double)(i + bottom_x))*right) + (pitch*(double)(j + bottom_y))*up'
 * where right = normalize((look_at-eye) x up), up' = normalize(right x (look_at-eye))
 * (MySdlApplication.cpp:1270-1279).  pitch = 1 is the reference's unit pixel step (:1315, :1321). */
typedef struct rt_camera {
    double eye[3];               /* CAMERA_POSITION (MySdlApplication.cpp:38) */
    double look_at[3];           /* LOOK_AT_VECTOR (MySdlApplication.cpp:39) */
    double up[3];                /* UP_VECTOR (MySdlApplication.cpp:40) */
    double pitch;                /* world units between adjacent pixel centres */
    int32_t bottom_x;            /* -W/2 (C integer division, MySdlApplication.cpp:1560) */
    int32_t bottom_y;            /* -H/2 */
} rt_camera;

/* Row banding for multi-GPU sharding: the image's rows are cut into bands of `band_height` rows and
 * band b goes to rank b % n_ranks.  A call renders only its rank's rows, densely, in increasing order.
 * `frames` > 1 renders that many frames of the same view in one call, frame-major: the rank's rows of
 * frame 0, then of frame 1, ... (each frame banded the same way), so an all-to-all can send frame f's
 * rows to rank f.  NULL rt_rows* (or n_ranks == 1 and frames <= 1) means one full image. */
typedef struct rt_rows {
    int32_t band_height;
    int32_t n_ranks;
    int32_t rank;
    int32_t frames;              /* 0 or 1: one frame */
} rt_rows;

/* Ray counts actually traced (SURVEY.md §8d rule): primary segments, reflected segments (levels 1..B,
 * only after a hit), shadow rays (one per light per hit). */
typedef struct rt_stats {
    uint64_t primary_rays;
    uint64_t reflect_rays;
    uint64_t shadow_rays;
    double kernel_ms;
} rt_stats;

/* Per-ray hit record, the observable part of the reference's Intersection (MySdlApplication.cpp:309-359). */
typedef struct rt_hit {
    double point[3];
    double normal[3];
    double reflected_end[3];     /* reflectedRay().endPoint() = point + r */
    double transmitted_end[3];   /* transmittedRay().endPoint() = point + t (t = 0 on total reflection) */
    int32_t hit;                 /* Intersection::intersects() */
    int32_t material;            /* 0 white square, 1 black square, 2 sphere, 3 tetrahedron, 4 cube, -1 none */
} rt_hit;

typedef struct rt_ctx rt_ctx;

/* ---- library / device ---------------------------------------------------------------------- */
int rt_abi_version(void);
const char* rt_last_error(void);
int rt_device_count(int* count);
int rt_ctx_create(int device, rt_ctx** out);
int rt_ctx_destroy(rt_ctx* ctx);

/* ---- scene (host side; no device needed) --------------------------------------------------- */
/* Fill constants and materials with the reference's globals (MySdlApplication.cpp:31-52, 583-590):
 * empty scene, board present at (0,0,0), no spheres, no lights. */
int rt_scene_init_reference(rt_scene* scene);
/* convertStringCoordinate (MySdlApplication.cpp:1326-1346): "b6" -> board-local point. */
int rt_convert_string_coordinate(const char* square, double out[3]);
/* Light placement used by loadScene (MySdlApplication.cpp:1511):
 * BOARD_POSITION + (0, 3.5*SQUARE_EDGE_SIZE, 0) + convertStringCoordinate(square). */
int rt_light_position_from_square(const char* square, double out[3]);
/* loadScene (MySdlApplication.cpp:1495-1539) over boardMap entries (square -> type; types as the
 * reference enum {LIGHT, TETRAHEDRON, CUBE, SPHERE, CYLINDER, CONE}, MySdlApplication.cpp:16).
 * Duplicate squares keep the last type (boardMap[tmp] = type, :1467), entries are visited in
 * std::map<string> order, the last light wins.  Spheres go to sphere_buf (capacity sphere_cap),
 * tetrahedra and cubes to mesh_buf (capacity mesh_cap) in child order, the light (white,
 * g_lightColor) to *light.  Returns RT_EUNSUPPORTED if a cylinder or cone is present (their reference
 * implementations are stubs: MySdlApplication.cpp:1000-1020, 457-458); everything else is still filled. */
int rt_load_scene(const char* const* squares, const int32_t* types, int n, rt_scene* scene,
                  rt_sphere* sphere_buf, int sphere_cap, rt_mesh* mesh_buf, int mesh_cap, rt_light* light);
/* draw()'s camera (MySdlApplication.cpp:1556-1560) for a W x H window at the given pitch. */
int rt_camera_init_reference(rt_camera* cam, int width, int height, double pitch);
/* Number of rows a rank renders under `rows` (NULL = all rows), over all its frames. */
int rt_local_rows(int height, const rt_rows* rows, int* out);
/* Image row of local row `local_row` under `rows`: frame * height + row within the frame. */
int rt_global_row(int height, const rt_rows* rows, int local_row, int* out);

/* ---- device path ---------------------------------------------------------------------------- */
/* Validate and upload the scene (scene + spheres + lights are copied; caller keeps ownership).
 * A scene identical to the uploaded one (same flattened record) is a no-op: no device work, the per-eye
 * data and tile-row order are kept (rt_render calls this every frame).  A changed scene first waits for
 * all work on the context's device (renders in flight on any stream read the old record), then uploads
 * synchronously. */
int rt_set_scene(rt_ctx* ctx, const rt_scene* scene);

/* Render this rank's rows of a width x height frame with `depth` bounces (rayTraceRay's `depth`).
 * Device pointers, each nullable, each local_rows*width pixels:
 *   rgba32f: float4 (r,g,b,1) unclamped, rgba8: clamp(c,0,1)*255 rounded (RGBA8 = floor(v*255+0.5)),
 *   rgb64f: 3 doubles (the reference's double colour, for bit-exact parity),
 *   raycount: per pixel packed (primary+reflect) | shadow << 16.
 * `stream` is a hipStream_t (NULL = default stream).  Asynchronous; no allocation. */
int rt_render_dev(rt_ctx* ctx, const rt_camera* cam, int width, int height, int depth,
                  const rt_rows* rows, float* rgba32f, uint8_t* rgba8, double* rgb64f,
                  uint32_t* raycount, void* stream);

/* ---- packed pixel formats (ABI 5) --------------------------------------------------------------- */
/* What a frame's bytes look like in a buffer.  Rows are dense (W * bytes per pixel), j = 0 at the bottom.
 * GRAY formats hold the R channel only and are accepted only for an ACHROMATIC scene (rt_scene_achromatic):
 * there R = G = B bit for bit, since every colour term of rayTraceRay (:1223-1226, :1241-1246) is a
 * component-wise product or sum of equal components, so the packed frame expands back to exactly the RGBA
 * frame.  They cut the bytes of a frame over PCIe (rt_render_packed: glDrawPixels(..., GL_LUMINANCE, ...))
 * and over xGMI (rt_render_multi's gather: 1 B/px instead of 4). */
#define RT_PIXEL_RGBA32F 0      /* float4 (r, g, b, 1), 16 B/px (the rgba32f image of rt_render_dev) */
#define RT_PIXEL_GRAY32F 1      /* float r, 4 B/px (achromatic scenes) */
#define RT_PIXEL_RGBA8   2      /* 4 B/px (the rgba8 image of rt_render_dev) */
#define RT_PIXEL_RGB8    3      /* 3 B/px, glDrawPixels(GL_RGB) / PPM order */
#define RT_PIXEL_GRAY8   4      /* 1 B/px: the R byte of RGBA8 (achromatic scenes) */
int rt_pixel_bytes(int format, int* bytes);
/* *out = 1 when the scene is achromatic: every material term the scene's objects use (ambient, diffuse,
 * specular, transparency of the board squares when the board is present, of the sphere material when there
 * are spheres, of the tetrahedron / cube materials when such meshes are present) and every light colour has
 * three equal components (MySdlApplication.cpp:577, 583-588: the app's board, spheres and tetrahedron are; its
 * red cube is not).  Host only.  (The renders use the same test, with no transparent material, to run one-channel
 * kernel instances whose three channels are bitwise equal by construction.) */
int rt_scene_achromatic(const rt_scene* scene, int* out);
/* rt_render_dev with the float image in `float_format` (RT_PIXEL_RGBA32F / GRAY32F) and the byte image in
 * `byte_format` (RT_PIXEL_RGBA8 / RGB8 / GRAY8); each image nullable.  Same rules as rt_render_dev. */
int rt_render_dev_packed(rt_ctx* ctx, const rt_camera* cam, int width, int height, int depth, const rt_rows* rows,
                         int float_format, void* float_pixels, int byte_format, void* byte_pixels, void* stream);
/* Host-buffer frames in one format (draw()'s replacement with fewer PCIe bytes).  rt_render_packed is
 * synchronous (stats nullable, as rt_render): the render and a copy kernel that writes the frame over PCIe
 * into host_pixels, back to back on the context's render stream.  rt_render_packed_async queues the render
 * on the render stream and the frame's device-to-host copy behind it — on an SDMA engine when host_pixels is
 * page-locked (rt_host_alloc; the render stream starts the engine's copy, no CU is taken from the next render),
 * else a copy kernel on the context's copy stream — and returns at once with a ticket: the copy of frame t runs
 * beside the render of frame t+1 (three device buffers: up to two frames may be waited for behind the one being
 * queued); rt_ctx_wait(ctx, t) returns when frame t's pixels are in host_pixels (ticket 0: everything queued).
 * host_pixels must stay valid until then.  RT_COPY_MODE (read at rt_ctx_create) overrides the path for both calls:
 * 0 copy kernel on the copy stream, 1 behind the render, 3 SDMA engine. */
int rt_render_packed(rt_ctx* ctx, const rt_scene* scene, const rt_camera* cam, int width, int height, int depth,
                     int format, void* host_pixels, rt_stats* stats);
int rt_render_packed_async(rt_ctx* ctx, const rt_scene* scene, const rt_camera* cam, int width, int height,
                           int depth, int format, void* host_pixels, uint64_t* ticket);
int rt_ctx_wait(rt_ctx* ctx, uint64_t ticket);
/* Pinned (page-locked) host memory for host-buffer frames (hipHostMalloc / hipHostFree). */
int rt_host_alloc(size_t bytes, void** out);
int rt_host_free(void* p);

/* ---- reference-faithful rayTraceScreen ------------------------------- */
/* rayTraceScreen (MySdlApplication.cpp:1251-1324) exactly as the app runs it: the incremental unit-step
 * screen walk from (bottom_x, bottom_y) (cam->pitch is not used: the reference steps by the unit vectors
 * right and up'), every sample jittered by 0.5 * randomUnit() (:1148-1169, rand() arguments evaluated
 * right to left), up to 16 samples per pixel with the reference's convergence test (:1294-1311), and the
 * average colour carried from pixel to pixel (:1283).  The carry-over and the shared rand() stream make
 * the frame a serial chain; the samples are traced on the GPU in speculative chunks (each pixel's sample
 * count is predicted and a window of stream positions around the prediction is traced; the host resolves the
 * chain in order, with the continuation of the chain already queued, and restarts it where the actual stream
 * position leaves a window), so the result is the reference's, bit for bit.  The context keeps the chunks'
 * buffers between calls (≈ 14 MB of mapped host memory and a stream per buffer set, three sets in the default
 * pipeline; freed by rt_ctx_destroy); concurrent calls on one context are allowed (each beyond the first
 * allocates its own).
 * rand_kind: RT_RAND_GLIBC (glibc rand(), the reference built on Linux) or RT_RAND_MSVC (the MSVC CRT
 * LCG, the reference's own Visual Studio build); seed as given to srand (the app never calls srand: 1).
 * Host outputs, each nullable, width*height pixels, j = 0 bottom: rgb64f (the colour passed to
 * glColor3d, :1312), rgba8 (floor(clamp(c,0,1)*255+0.5)), samples (samples traced per pixel, 2..16);
 * *rand_calls = rand() calls made.  Synchronous. */
#define RT_RAND_GLIBC 0
#define RT_RAND_MSVC  1
int rt_render_screen(rt_ctx* ctx, const rt_scene* scene, const rt_camera* cam, int width, int height,
                     int depth, int rand_kind, uint32_t seed, double* rgb64f, uint8_t* rgba8,
                     uint8_t* samples, uint64_t* rand_calls);

/* Synchronous host-buffer convenience for draw() (MySdlApplication.cpp:1541-1563): uploads `scene` (a
 * no-op when unchanged), renders into device buffers the context keeps between calls, copies back, fills
 * *stats (ray counts summed on the device + kernel time).  Any output pointer may be NULL.  Tile-row order:
 * the first render of a view uses the identity order, the second times its tile rows, later renders
 * of the view dispatch the longest rows first (images are identical either way). */
int rt_render(rt_ctx* ctx, const rt_scene* scene, const rt_camera* cam, int width, int height,
              int depth, const rt_rows* rows, float* rgba32f, uint8_t* rgba8, double* rgb64f,
              rt_stats* stats);

/* Arbitrary rays (Line(start, end)) through the uploaded scene on the device:
 * rt_intersect_dev = g_scene.intersection (MySdlApplication.cpp:724-823) -> rt_hit per ray;
 * rt_trace_rays_dev = rayTraceRay(scene, lights, ray, color, depth) -> 3 doubles per ray. */
int rt_intersect_dev(rt_ctx* ctx, const double* starts, const double* ends, int n, rt_hit* hits,
                     void* stream);
int rt_trace_rays_dev(rt_ctx* ctx, const double* starts, const double* ends, int n, int depth,
                      double* rgb64f, uint32_t* raycount, void* stream);

/* Put gathered bands back into image order: `gathered` holds n_ranks slabs, slab r = rank r's local
 * rows (rt_local_rows rows each, slabs padded to `slab_rows` rows), `image` is height x width.
 * elem_bytes in {1,2,4,8,16,24,32}: bytes per pixel. */
int rt_unshuffle_dev(const void* gathered, void* image, int width, int height, int elem_bytes,
                     int band_height, int n_ranks, int slab_rows, void* stream);
/* rt_unshuffle_dev from packed slabs in src_format into an image in dst_format: equal formats (a plain
 * unshuffle), GRAY8 -> RGBA8, RGB8 -> RGBA8, GRAY32F -> RGBA32F (RT_PIXEL_*). */
int rt_unpack_dev(const void* gathered, void* image, int width, int height, int src_format, int dst_format,
                  int band_height, int n_ranks, int slab_rows, void* stream);

/* ---- multi-GPU: one frame's rows split over GPUs, gathered to rank 0 ---- */
/* A group of ranks: rank r renders the round-robin row bands b = r (mod n_ranks) of every frame into its
 * slab; rt_render_multi gathers the slabs to rank 0 (ncclSend / ncclRecv over xGMI) and puts the rows in
 * image order there (rt_unshuffle_dev).  Slabs and rank 0's gather buffer are double-buffered and every rank
 * renders and sends on the group's own streams, so frame f's gather overlaps frame f+1's render.
 * Each rank renders its context's scene: call rt_set_scene on every context with the same scene. */
#define RT_TRANSPORT_AUTO -1    /* RCCL when the contexts are on distinct devices, else COPY */
#define RT_TRANSPORT_RCCL  0    /* RCCL send/recv (one communicator rank per context) */
#define RT_TRANSPORT_COPY  1    /* hipMemcpyPeerAsync to rank 0 (contexts may share a device) */
#define RT_OUT_RGBA32F 1
#define RT_OUT_RGBA8   2
#define RT_COMM_ID_BYTES 128
typedef struct rt_group rt_group;
/* Bands for n_ranks: band_height 0 = auto (largest height <= 16 that gives every rank the same rows, e.g.
 * 15 for 1080 rows over 8 ranks; else 8).  *slab_rows_out (nullable) = the most rows any rank renders. */
int rt_band_plan(int height, int n_ranks, int band_height, int* band_out, int* slab_rows_out);
/* What one rank of a row-banded frame moves (host only, no device: the plan rt_render_multi follows).
 * kind 0 = the RGBA32F image, 1 = the RGBA8 image (RT_OUT_RGBA32F / RT_OUT_RGBA8). */
typedef struct rt_group_plan {
    int32_t n_ranks, rank;
    int32_t band_height;         /* rt_band_plan */
    int32_t slab_rows;           /* the most rows any rank renders */
    int32_t rank_rows;           /* rows this rank renders (rt_local_rows) */
    int32_t wire[2];             /* RT_PIXEL_* the kind travels in (GRAY for achromatic scenes), -1: not requested */
    int32_t elem_bytes[2];       /* bytes per pixel of wire[k] */
    uint64_t slab_bytes[2];      /* this rank's slab per kind: slab_rows x width x elem_bytes */
    uint64_t send_bytes[2];      /* bytes this rank sends rank 0 per frame (0 on rank 0: its slab is unpacked in place) */
    uint64_t gather_bytes[2];    /* rank 0: its gather buffer per kind (one slab-sized slot per renderer) */
    uint64_t payload_bytes;      /* rank 0: bytes received from the other ranks per frame, all kinds */
    int32_t renderers;           /* ranks that render bands: n_ranks, or n_ranks - 1 when rank 0 only assembles */
    int32_t root_renders;        /* 1: rank 0 renders bands too; 0: bands go to ranks 1 .. n - 1 (rt_group_root_renders) */
} rt_group_plan;
/* The plan of `rank` for a width x height frame (band_height 0 = auto, `outputs` as rt_render_multi, achromatic =
 * rt_scene_achromatic of the group's scene).  The band plan is over the renderers (rt_rows {band_height, renderers,
 * rank - (root_renders ? 0 : 1)}); rank 0 then receives every renderer's slab but its own. */
int rt_group_plan_frame(int width, int height, int n_ranks, int rank, int band_height, int outputs, int achromatic,
                        rt_group_plan* out);
/* Whether rank 0 of an n-rank group renders bands (1) or only receives and assembles the frame (0).  Rank 0 unpacks
 * the whole image (an HBM-bound 33 MB of RGBA8 stores at 4K) and receives every peer's slab besides, so from 4 ranks
 * on its bands go to the others (DESIGN.md §7 has the measurements); RT_GROUP_ROOT_RENDERS=0|1 overrides (every
 * rank of a group must see the same setting). */
int rt_group_root_renders(int n_ranks);
/* Rank 0's receive from `peer` (1 .. n_ranks - 1) for image `kind`: byte offset into rank 0's gather buffer and
 * byte count (equal to that peer's send_bytes[kind]). */
int rt_group_plan_recv(const rt_group_plan* plan, int width, int height, int peer, int kind, uint64_t* offset,
                       uint64_t* bytes);
/* FNV-1a 64 of the scene's flattened device record: what the ranks of a one-process-per-GPU group compare. */
int rt_scene_fingerprint(const rt_scene* scene, uint64_t* out);
/* One process driving n GPUs: ctxs[q] is rank q (ctxs[0] receives the image); distinct contexts, each on
 * its device (ncclCommInitAll over the contexts' devices for RT_TRANSPORT_RCCL). */
int rt_group_create(rt_ctx* const* ctxs, int n, int transport, rt_group** out);
/* One process per GPU (a torchrun-style launch): rank 0 makes the id, the launcher hands the same
 * RT_COMM_ID_BYTES bytes to every rank, each rank passes its own context (ncclCommInitRank). */
int rt_comm_unique_id(uint8_t* id);
int rt_group_create_rank(rt_ctx* ctx, int n_ranks, int rank, const uint8_t* id, rt_group** out);
int rt_group_destroy(rt_group* group);
/* *n_ranks: ranks of the group; *n_local: ranks driven by this process; *first_rank: the first of them;
 * *transport: RT_TRANSPORT_RCCL or RT_TRANSPORT_COPY.  Each pointer nullable. */
int rt_group_info(const rt_group* group, int* n_ranks, int* n_local, int* first_rank, int* transport);
/* One frame over the whole group.  Every rank calls it with the same camera, size, depth, band_height
 * (0 = auto) and `outputs` (RT_OUT_RGBA32F | RT_OUT_RGBA8: the images rank 0 receives).  On rank 0, rgba32f /
 * rgba8 are device images (width x height, j = 0 bottom) on rank 0's device for the requested outputs,
 * assembled in order on `stream` (a hipStream_t of that device; NULL = default stream); other ranks' pointers
 * are ignored.  Asynchronous: rank 0's image is complete when `stream` reaches this call's work.
 * What travels (the wire formats, rt_group_stats): for an achromatic scene (rt_scene_achromatic, decided by
 * each rank from its own context's scene — they are the same scene) GRAY8 for RGBA8 and GRAY32F for RGBA32F,
 * otherwise RGB8 and RGBA32F; rank 0 expands them into its images (rt_unpack_dev), byte for byte the images a
 * single rt_render_dev writes.  Every rank changes its scene (rt_set_scene) between the same frames; in a
 * one-process-per-GPU group the first frame after a rank's scene differs from the one the group last agreed on
 * all-reduces a fingerprint of the scene over the group (blocking, once per scene) and fails with RT_EINVAL on
 * every rank when they differ.  A scene change on some ranks only (the others still holding the agreed scene) is a
 * contract violation: those ranks enter the all-reduce while the others post their sends, and the group HANGS. */
int rt_render_multi(rt_group* group, const rt_camera* cam, int width, int height, int depth, int band_height,
                    int outputs, float* rgba32f, uint8_t* rgba8, void* stream);
/* Wait for the group's own render and gather streams (e.g. before timing on a rank > 0). */
int rt_group_synchronize(rt_group* group);
/* Per-phase timing of rt_render_multi (HIP events on the group's streams), for this process's ranks. */
typedef struct rt_group_stats {
    int32_t frames;              /* frames timed since rt_group_timing(group, 1) (the last <= 64 are averaged) */
    int32_t wire_float;          /* RT_PIXEL_* sent for RT_OUT_RGBA32F, -1: not requested (last frame) */
    int32_t wire_byte;           /* RT_PIXEL_* sent for RT_OUT_RGBA8, -1: not requested (last frame) */
    int32_t ranks_timed;         /* this process's ranks the means are over */
    uint64_t payload_bytes;      /* bytes rank 0 receives from the other ranks per frame (last frame) */
    double render_ms;            /* mean rt_render_dev launch on a rendering rank's render stream */
    double gather_ms;            /* mean send (rank > 0) / receive of every peer's slab (rank 0), from the
                                    point the rank's own render is done (it includes waiting for peers) */
    double assemble_ms;          /* rank 0: unshuffle + expand into the images (0 elsewhere) */
    double frame_ms;             /* rank 0: its render's start to the assembled image (0 elsewhere) */
} rt_group_stats;
/* enable = 1: start recording per-phase events from the next frame on (and clear earlier ones); 0: stop. */
int rt_group_timing(rt_group* group, int enable);
/* Synchronizes the group's streams, then fills *stats from the recorded frames. */
int rt_group_get_stats(rt_group* group, rt_group_stats* stats);

/* ---- output (host) -------------------------------------------------------------------------- */
/* writePpmScreenshot format (Hw4/ppm.cpp:15-25): "P6 W H 255\n" then RGB rows top-down, from an
 * RGBA8 (or RGB8 when channels == 3, GRAY8 when channels == 1) bottom-up image as glReadPixels returns it. */
int rt_write_ppm(const char* path, const uint8_t* pixels, int width, int height, int channels);

#ifdef __cplusplus
}
#endif

#endif /* RT_API_H */
