// rt_host.cpp — host half of the C ABI (include/rt_api.h): scene construction the way the reference
// app builds g_scene, camera, row banding, device-scene flattening, PPM output.  No HIP calls here.
//
// Citations are into /root/reference/Hw4/MySdlApplication.cpp unless a file is named.
#include <algorithm>
#include <array>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <limits>
#include <map>
#include <string>
#include <vector>

#include "../../include/rt_api.h"
#include "rt_internal.hpp"
#include "rt_layout.hpp"

namespace {

thread_local std::string g_last_error;

// Host mirror of the reference Point (:136-212) with the same operation order.
struct HP {
    double x, y, z;
};
inline HP hp(double x, double y, double z) { return HP{x, y, z}; }
inline HP hp(const double* v) { return HP{v[0], v[1], v[2]}; }
inline HP operator+(HP a, HP b) { return hp(a.x + b.x, a.y + b.y, a.z + b.z); }
inline HP operator-(HP a, HP b) { return hp(a.x - b.x, a.y - b.y, a.z - b.z); }
inline HP operator*(double s, HP a) { return hp(s * a.x, s * a.y, s * a.z); }
inline double dot(HP a, HP b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline HP cross(HP a, HP b) { return hp(a.y * b.z - b.y * a.z, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }
inline double length(HP a) { return std::sqrt(a.x * a.x + a.y * a.y + a.z * a.z); }
inline HP normalize(HP a) {
    double l = length(a);
    return hp(a.x / l, a.y / l, a.z / l);
}
inline void put(double* d, HP a) { d[0] = a.x; d[1] = a.y; d[2] = a.z; }

// Reference constants (:31-52).
const double kWhite[3] = {1.0, 1.0, 1.0};
const double kBlack[3] = {0.0, 0.0, 0.0};
const double kRed[3] = {1.0, 0.0, 0.0};
const double kBoardPosition[3] = {0, 0, -160};
const double kBoardEdge = 320.0;
const double kBoardHalf = kBoardEdge / 2;
const unsigned kNumSquares = 8;
const double kSquareEdge = kBoardEdge / kNumSquares;
const double kSmall = .0001;
const double kAttenuation = 100000;
const double kCamera[3] = {0, 100, 200};
const double kLookAt[3] = {0, 0, -160};
const double kUp[3] = {0, 1, 0};

void set_material(rt_material* m, HP a, HP d, HP s, HP t, double r) {
    put(m->ambient, a);
    put(m->diffuse, d);
    put(m->specular, s);
    put(m->transparency, t);
    m->refraction = r;
}

// The kernel divides by a triangle's den with a shared reciprocal (rt_device.hpp div_const) only when
// |den| is in [2^-200, 2^200]: with |A| in [2^-500, 2^500] the IEEE sequence's scale steps are identities.
int32_t const_quotient_ok(double den) {
    return std::fabs(den) >= 0x1p-200 && std::fabs(den) <= 0x1p+200 ? 1 : 0;
}

bool valid_square(const char* sq) { return sq && sq[0] != 0 && sq[1] != 0; }

bool all_zero(const double v[3]) { return v[0] == 0 && v[1] == 0 && v[2] == 0; }

}  // namespace

int rt_fail(int code, const std::string& msg) {
    g_last_error = msg;
    return code;
}

extern "C" int rt_abi_version(void) { return RT_ABI_VERSION; }

extern "C" const char* rt_last_error(void) { return g_last_error.c_str(); }

extern "C" int rt_scene_init_reference(rt_scene* s) {
    if (!s) return rt_fail(RT_EINVAL, "rt_scene_init_reference: null scene");
    memset(s, 0, sizeof(*s));
    put(s->position, hp(kBoardPosition));
    s->radius = std::sqrt((double)3) * kBoardHalf;                              // :590
    s->has_board = 1;
    s->board_half_size = kBoardHalf;
    s->square_edge_size = kSquareEdge;
    s->small_number = kSmall;
    s->attenuation_factor = kAttenuation;
    HP white = hp(kWhite), black = hp(kBlack);
    set_material(&s->white_square, .1 * white, .5 * white, white, black, 1);    // :583
    set_material(&s->black_square, black, .1 * white, black, black, 1);         // :585
    set_material(&s->sphere_material, black, .1 * white, white, black, 1);      // :586
    set_material(&s->tetrahedron_material, black, black, .1 * white, white, 2.0 / 3.0);  // :587
    HP red = hp(kRed);
    set_material(&s->cube_material, .1 * red, .4 * red, red, black, 1);         // :588
    return RT_OK;
}

extern "C" int rt_convert_string_coordinate(const char* sq, double out[3]) {   // :1326-1346
    if (!valid_square(sq) || !out) return rt_fail(RT_EINVAL, "rt_convert_string_coordinate: need 2 chars");
    HP first = hp(-kBoardEdge / 2, 0.0, kBoardEdge / 2);
    HP row = hp(0.0, 0.0, -(double(sq[0] - 'a') + .5) * kSquareEdge);
    HP col = hp((double(sq[1] - '0' - 1) + .5) * kSquareEdge, 0.0, 0.0);
    HP height = hp(0.0, 1.5 * kSquareEdge, 0.0);
    put(out, first + row + col + height);
    return RT_OK;
}

extern "C" int rt_light_position_from_square(const char* sq, double out[3]) {  // :1511
    double c[3];
    int rc = rt_convert_string_coordinate(sq, c);
    if (rc) return rc;
    put(out, hp(kBoardPosition) + hp(0.0, 3.5 * kSquareEdge, 0.0) + hp(c));
    return RT_OK;
}

extern "C" int rt_load_scene(const char* const* squares, const int32_t* types, int n, rt_scene* scene,
                             rt_sphere* sphere_buf, int sphere_cap, rt_mesh* mesh_buf, int mesh_cap, rt_light* light) {
    if (!scene || n < 0 || (n > 0 && (!squares || !types))) return rt_fail(RT_EINVAL, "rt_load_scene: bad args");
    std::map<std::string, int> board_map;                                       // boardMap (:595)
    for (int k = 0; k < n; ++k) {
        if (!valid_square(squares[k])) return rt_fail(RT_EINVAL, "rt_load_scene: bad square");
        if (types[k] < 0 || types[k] > 5) return rt_fail(RT_EINVAL, "rt_load_scene: bad object type");
        board_map[std::string(squares[k])] = types[k];                          // :1467
    }
    rt_scene_init_reference(scene);
    int ns = 0, nm = 0;
    bool unsupported = false;
    double lpos[3] = {0.0, 0.0, 0.0};                                           // g_lightPosition (:573)
    for (const auto& kv : board_map) {                                          // :1503-1538
        const char* sq = kv.first.c_str();
        switch (kv.second) {
            case 0:                                                             // LIGHT (:1510-1513)
                rt_light_position_from_square(sq, lpos);
                break;
            case 1:                                                             // TETRAHEDRON (:1514-1517)
            case 2: {                                                           // CUBE (:1518-1522)
                if (nm >= mesh_cap || !mesh_buf) return rt_fail(RT_EINVAL, "rt_load_scene: mesh_buf too small");
                rt_mesh& m = mesh_buf[nm++];
                m.kind = kv.second == 1 ? RT_MESH_TETRAHEDRON : RT_MESH_CUBE;
                m.after_spheres = ns;
                rt_convert_string_coordinate(sq, m.position);
                m.edge = kSquareEdge;
                break;
            }
            case 3: {                                                           // SPHERE (:1523-1527)
                if (ns >= sphere_cap || !sphere_buf) return rt_fail(RT_EINVAL, "rt_load_scene: sphere_buf too small");
                rt_convert_string_coordinate(sq, sphere_buf[ns].center);
                sphere_buf[ns].radius = kSquareEdge / 2;
                ++ns;
                break;
            }
            default:                                                            // CYLINDER / CONE: stubs
                unsupported = true;
                break;
        }
    }
    scene->n_spheres = ns;
    scene->spheres = sphere_buf;
    scene->n_meshes = nm;
    scene->meshes = mesh_buf;
    if (light) {
        put(light->color, hp(kWhite));                                          // g_lightColor (:577)
        put(light->position, hp(lpos));
        scene->n_lights = 1;                                                    // draw() pushes one light (:1552-1554)
        scene->lights = light;
    }
    if (unsupported)
        return rt_fail(RT_EUNSUPPORTED,
                       "rt_load_scene: cylinder/cone are stubs in the reference (MySdlApplication.cpp:1000-1020, 457-458)");
    return RT_OK;
}

extern "C" int rt_camera_init_reference(rt_camera* cam, int width, int height, double pitch) {
    if (!cam || width <= 0 || height <= 0) return rt_fail(RT_EINVAL, "rt_camera_init_reference: bad args");
    memset(cam, 0, sizeof(*cam));
    put(cam->eye, hp(kCamera));
    put(cam->look_at, hp(kLookAt));
    put(cam->up, hp(kUp));
    cam->bottom_x = -width / 2;                                                 // :1560
    cam->bottom_y = -height / 2;
    cam->pitch = pitch;
    return RT_OK;
}

namespace {

int frames_of(const rt_rows* r) { return (r && r->frames > 1) ? r->frames : 1; }

// Rows of one frame that the rank renders.
int frame_local_rows(int height, const rt_rows* r) {
    if (!r || r->n_ranks <= 1) return height;
    const int hb = r->band_height, G = r->n_ranks;
    const int full_bands = height / hb, tail = height % hb;
    int n = (full_bands / G) * hb;
    if (r->rank < full_bands % G) n += hb;                                      // bands 0..extra-1 of the last round
    if (tail && (full_bands % G) == r->rank) n += tail;                         // the partial last band
    return n;
}

}  // namespace

extern "C" int rt_local_rows(int height, const rt_rows* r, int* out) {
    if (!out || height < 0) return rt_fail(RT_EINVAL, "rt_local_rows: bad args");
    if (r && (r->frames < 0 || r->n_ranks < 1)) return rt_fail(RT_EINVAL, "rt_local_rows: bad frames / ranks");
    if (r && r->n_ranks > 1 && (r->band_height <= 0 || r->rank < 0 || r->rank >= r->n_ranks))
        return rt_fail(RT_EINVAL, "rt_local_rows: bad band geometry");
    if (r && r->n_ranks == 1 && r->rank != 0) return rt_fail(RT_EINVAL, "rt_local_rows: bad rank");
    *out = frame_local_rows(height, r) * frames_of(r);
    return RT_OK;
}

extern "C" int rt_global_row(int height, const rt_rows* r, int local_row, int* out) {
    int nl = 0;
    int rc = rt_local_rows(height, r, &nl);
    if (rc) return rc;
    if (!out || local_row < 0 || local_row >= nl) return rt_fail(RT_EINVAL, "rt_global_row: row out of range");
    const int per = frame_local_rows(height, r);
    const int f = local_row / per, lr = local_row % per;
    int j = lr;
    if (r && r->n_ranks > 1) {
        const int hb = r->band_height;
        j = ((lr / hb) * r->n_ranks + r->rank) * hb + lr % hb;
    }
    *out = f * height + j;
    return RT_OK;
}

// Row bands of the multi-GPU group (rt_group.cpp).
extern "C" int rt_pixel_bytes(int format, int* bytes) {
    if (!bytes) return rt_fail(RT_EINVAL, "rt_pixel_bytes: null pointer");
    switch (format) {
        case RT_PIXEL_RGBA32F: *bytes = 16; return RT_OK;
        case RT_PIXEL_GRAY32F: *bytes = 4; return RT_OK;
        case RT_PIXEL_RGBA8: *bytes = 4; return RT_OK;
        case RT_PIXEL_RGB8: *bytes = 3; return RT_OK;
        case RT_PIXEL_GRAY8: *bytes = 1; return RT_OK;
        default: *bytes = 0; return rt_fail(RT_EINVAL, "rt_pixel_bytes: unknown pixel format");
    }
}

extern "C" int rt_band_plan(int height, int n_ranks, int band_height, int* band_out, int* slab_rows_out) {
    if (height <= 0 || n_ranks <= 0 || band_height < 0 || !band_out)
        return rt_fail(RT_EINVAL, "rt_band_plan: bad arguments");
    int hb = band_height;
    if (hb == 0) {
        // The render's tile height (8 rows): every 8 x 8 tile of a rank's slab is then 8 consecutive image rows, which
        // the per-wave primary cone culling needs (a tile straddling two bands tests every sphere).  Ranks differ by
        // at most one band (c4 at 8 ranks: 272 against 264 rows).  r02-r05 chose the largest height <= 16 giving
        // every rank the same rows (15 for 2160 rows over 8 ranks): its straddling tiles made every rank's band set
        // 10% slower (tools/c4_gap_probe.py part 2: 30.4 -> 27.5 us per 1/8 frame serial).
        hb = 8;
    }
    if (n_ranks == 1) hb = std::max(hb, 1);
    int slab = 0;
    for (int q = 0; q < n_ranks; ++q) {
        rt_rows r = {hb, n_ranks, q, 1};
        int nl = 0;
        int rc = rt_local_rows(height, &r, &nl);
        if (rc) return rc;
        slab = std::max(slab, nl);
    }
    *band_out = hb;
    if (slab_rows_out) *slab_rows_out = slab;
    return RT_OK;
}

void rt_camera_basis(const rt_camera* cam, double right[3], double upp[3]) {
    HP ld = hp(cam->look_at) - hp(cam->eye);                                    // :1270
    HP r = normalize(cross(ld, hp(cam->up)));                                   // :1271-1273
    HP u = normalize(cross(r, ld));                                             // :1276-1277
    put(right, r);
    put(upp, u);
}

int rt_build_dev_scene(const rt_scene* s, std::vector<unsigned char>* blob) {
    if (!s) return rt_fail(RT_EINVAL, "rt_set_scene: null scene");
    if (s->n_spheres < 0 || s->n_spheres > RT_MAX_SPHERES)
        return rt_fail(RT_EINVAL, "rt_set_scene: n_spheres out of range [0, " + std::to_string(RT_MAX_SPHERES) + "]");
    if (s->n_lights < 0 || s->n_lights > RT_MAX_LIGHTS)
        return rt_fail(RT_EINVAL, "rt_set_scene: n_lights out of range [0, " + std::to_string(RT_MAX_LIGHTS) + "]");
    if (s->n_spheres > 0 && !s->spheres) return rt_fail(RT_EINVAL, "rt_set_scene: null spheres");
    if (s->n_lights > 0 && !s->lights) return rt_fail(RT_EINVAL, "rt_set_scene: null lights");
    if (!(s->small_number >= 0) || !(s->square_edge_size != 0))
        return rt_fail(RT_EINVAL, "rt_set_scene: bad constants");
    // The kernel's checker divides by the square size with a shared reciprocal (rt_device.hpp
    // material_of), exact for sizes in this (generous) range.
    if (!(std::fabs(s->square_edge_size) >= 0x1p-400 && std::fabs(s->square_edge_size) <= 0x1p+400))
        return rt_fail(RT_EUNSUPPORTED, "rt_set_scene: square_edge_size outside [2^-400, 2^400]");
    if (s->n_meshes < 0 || s->n_meshes > RT_MAX_MESHES || (s->n_meshes > 0 && !s->meshes))
        return rt_fail(RT_EINVAL, "rt_set_scene: bad meshes");
    int n_tris = 0;
    for (int m = 0; m < s->n_meshes; ++m) {
        const rt_mesh& M = s->meshes[m];
        if (M.kind != RT_MESH_TETRAHEDRON && M.kind != RT_MESH_CUBE) return rt_fail(RT_EINVAL, "rt_set_scene: bad mesh kind");
        if (M.after_spheres < 0 || M.after_spheres > s->n_spheres || (m > 0 && M.after_spheres < s->meshes[m - 1].after_spheres))
            return rt_fail(RT_EINVAL, "rt_set_scene: mesh after_spheres must be non-decreasing in [0, n_spheres]");
        n_tris += M.kind == RT_MESH_TETRAHEDRON ? 4 : 12;
    }
    const rt_material* mats[5] = {&s->white_square, &s->black_square, &s->sphere_material, &s->tetrahedron_material,
                                  &s->cube_material};
    // rayTraceRay (:1230-1247) spawns a transmitted ray when transparency != 0 and |transparency| > eps, a
    // reflected ray when opacity = 1 - transparency != 0.  A material that does both makes every hit on it
    // a branch of a ray tree: such scenes run the trace_tree kernels (depth-first, per-lane node stack);
    // the others follow one continuation per hit.
    bool used[5] = {true, true, s->n_spheres > 0, false, false};
    for (int m = 0; m < s->n_meshes; ++m) used[s->meshes[m].kind == RT_MESH_TETRAHEDRON ? 3 : 4] = true;
    bool any_transparent = false, tree = false;
    rt::DevMat dm[5];
    memset(dm, 0, sizeof(dm));
    for (int m = 0; m < 5; ++m) {
        const rt_material* M = mats[m];
        HP T = hp(M->transparency);
        HP opacity = hp(1.0, 1.0, 1.0) - T;                                     // :1236
        bool zeroT = T.x == 0 && T.y == 0 && T.z == 0;
        bool transmit = !zeroT && length(T) > s->small_number;                  // :1238
        bool reflect = !(opacity.x == 0 && opacity.y == 0 && opacity.z == 0);   // :1243
        if (used[m] && transmit && reflect) tree = true;
        if (used[m] && !zeroT) any_transparent = true;
        for (int q = 0; q < 3; ++q) {
            dm[m].amb[q] = M->ambient[q];
            dm[m].diff[q] = M->diffuse[q];
            dm[m].spec[q] = M->specular[q];
        }
        put(dm[m].w, transmit ? T : opacity);
        put(dm[m].wt, T);
        put(dm[m].wo, opacity);
        dm[m].refr = M->refraction;
        dm[m].transmit = transmit ? 1 : 0;
        dm[m].transparent = zeroT ? 0 : 1;
        dm[m].reflect = reflect ? 1 : 0;
    }

    // (rounded up to 16 B: kernels may copy the whole record into LDS in 4- or 16-byte words)
    const size_t bytes = ((size_t)rt::scene_bytes_for(s->n_spheres, s->n_meshes, n_tris, s->n_lights) + 15) & ~(size_t)15;
    const int np = rt::padded_spheres(s->n_spheres);
    const int ns = rt::sphere_stride(np);            // array stride (rt_layout.hpp)
    blob->assign(bytes, 0);
    rt::DevScene* d = reinterpret_cast<rt::DevScene*>(blob->data());
    rt::DevSphere* sph = reinterpret_cast<rt::DevSphere*>(d + 1);
    rt::DevSpherePrim* prim = reinterpret_cast<rt::DevSpherePrim*>(sph + ns);
    rt::DevSphereF* sphf = reinterpret_cast<rt::DevSphereF*>(prim + ns);
    (void)prim;                                      // per-eye data: filled on the device (rt_prepare_kernel)
    d->n_padded = np;
    d->n_stride = ns;
    d->lds_bytes = rt::lds_bytes_for(s->n_spheres);
    const double inf = std::numeric_limits<double>::infinity();
    d->eye[0] = d->eye[1] = d->eye[2] = std::numeric_limits<double>::quiet_NaN();

    const HP zero = hp(0.0, 0.0, 0.0);
    const HP bc = hp(s->position) + zero;                                       // g_scene: _position + offset (:739)
    put(d->bc, bc);
    d->br2 = s->radius * s->radius;                                             // :750
    d->bound_on = s->radius > 0;                                                // :747 (g_scene is not _amSphere)
    // origins with |o - bc|^2 < (R-1)^2 provably pass the cull (proof at rt_device.hpp bound_pass_dp: |s| >= 1, which
    // clears the reference's |s| < SMALL_NUMBER test only while SMALL_NUMBER < 1 — kept below 0.5 for the rounding)
    d->inner2 = s->radius > 2 && s->small_number < 0.5 ? (s->radius - 1) * (s->radius - 1) : -1.0;
    d->eps = s->small_number;
    d->att = s->attenuation_factor;
    put(d->coff, bc);                                                           // CheckerBoard's positionOffset
    d->half = s->board_half_size;
    d->square = s->square_edge_size;

    d->has_board = 0;
    if (s->has_board) {
        // CheckerBoard(p) -> _boundingSquare = Quad(p, Material(), P1..P4) (:1064-1069) ->
        // Triangle(zero, m, P1,P2,P3), Triangle(zero, m, P1,P3,P4) (:840-841).
        const double h = s->board_half_size;
        const HP P[4] = {hp(-h, 0, -h), hp(h, 0, -h), hp(h, 0, h), hp(-h, 0, h)};
        const int idx[2][3] = {{0, 1, 2}, {0, 2, 3}};
        const HP quad_pos = hp(s->board_position) + bc;                         // Quad: _position + offset
        const HP tri_pos = zero + quad_pos;                                     // Triangle: zero + offset (:640)
        bool degenerate[2];
        for (int t = 0; t < 2; ++t) {
            HP v0 = P[idx[t][0]], v1 = P[idx[t][1]], v2 = P[idx[t][2]];
            HP u = v1 - v0, v = v2 - v0;                                        // :413-414
            HP n = cross(u, v);                                                 // :415
            degenerate[t] = length(n) < s->small_number;                        // :418
            n = normalize(n);                                                   // :422
            double uv = dot(u, v), uu = dot(u, u), vv = dot(v, v);             // :424-426
            double den = uv * uv - uu * vv;                                     // :428
            if (std::fabs(den) < s->small_number) degenerate[t] = true;         // :430
            rt::DevTri& T = d->tri[t];
            put(T.v0, tri_pos + v0);                                            // :641
            put(T.u, u);
            put(T.v, v);
            put(T.n, n);
            T.uv = uv;
            T.uu = uu;
            T.vv = vv;
            T.den = den;
            // den < 0: A > |den| 2^-1070 proves A/den < 0 (nonzero), so the kernel may skip the division.
            // Otherwise disable the shortcut.
            T.thr = (den < 0 && std::fabs(den) >= 1024.0) ? std::ldexp(std::fabs(den), -1070)
                                                          : std::numeric_limits<double>::infinity();
            T.fast = const_quotient_ok(den);
        }
        // The kernel shares the plane step of the two triangles; the reference board always satisfies
        // this (same vertex 0, same normal).  A degenerate board never intersects (:633-637).
        if (!degenerate[0] && !degenerate[1]) {
            if (memcmp(d->tri[0].v0, d->tri[1].v0, sizeof(d->tri[0].v0)) != 0 ||
                memcmp(d->tri[0].n, d->tri[1].n, sizeof(d->tri[0].n)) != 0)
                return rt_fail(RT_EUNSUPPORTED, "rt_set_scene: board triangles do not share a plane");
            d->has_board = 1;
        } else if (degenerate[0] != degenerate[1]) {
            return rt_fail(RT_EUNSUPPORTED, "rt_set_scene: half-degenerate board");
        }
    }
    // Board self-test skip (rt_device.hpp board_skip): with the board normal exactly (0, +-1, 0), a ray that
    // starts at a board hit point q has |n . (v0 - q)| <= 2^-50 (3 |p0.y| + 5 |v0.y| + 1), p0 the origin of
    // the ray that hit; below eps^2 / 2 its m = num / nd (|nd| >= eps) is below eps: a certain miss.
    d->board_skip_y = -1.0;
    d->self_eps2 = 0.25 * s->small_number * s->small_number;
    if (d->has_board && d->tri[0].n[0] == 0.0 && d->tri[0].n[2] == 0.0 && std::fabs(d->tri[0].n[1]) == 1.0 &&
        s->small_number > 0) {
        const double eps2 = s->small_number * s->small_number;
        const double y = (eps2 / 2 / 0x1p-50 - 5 * std::fabs(d->tri[0].v0[1]) - 1) / 3;
        if (y > 0 && std::isfinite(y)) d->board_skip_y = y;
    }
    // Board decided by position (rt_device.hpp board_hit): the reference's CheckerBoard exactly — normal (0, -1, 0),
    // T1 = (P1, P2, P3) with u = (L, 0, 0), v = (L, 0, L), T2 = (P1, P3, P4) with u = (L, 0, L), v = (0, 0, L) — and an
    // integer side L <= 2^12, so uu, uv, vv and den are exact.  Margin delta = L 2^-19, range far = 2^24 L (proof at
    // board_hit).
    d->board_fast = 0;
    d->board_lo = d->board_hi = d->board_out = inf;
    d->board_far = -1.0;
    if (d->has_board) {
        const rt::DevTri &T1 = d->tri[0], &T2 = d->tri[1];
        const double L = 2 * s->board_half_size;
        auto is3 = [](const double* a, double x, double y, double z) { return a[0] == x && a[1] == y && a[2] == z; };
        const bool shape = L >= 1 && L <= 4096 && L == std::floor(L) && is3(T1.n, 0, -1, 0) && is3(T2.n, 0, -1, 0) &&
                           is3(T1.u, L, 0, 0) && is3(T1.v, L, 0, L) && is3(T2.u, L, 0, L) && is3(T2.v, 0, 0, L) &&
                           is3(T1.v0, T2.v0[0], T2.v0[1], T2.v0[2]) && T1.uu == L * L && T1.uv == L * L &&
                           T1.vv == 2 * L * L && T2.uu == 2 * L * L && T2.uv == L * L && T2.vv == L * L &&
                           T1.den == -(L * L * L * L) && T2.den == -(L * L * L * L);
        if (shape) {
            const double delta = std::ldexp(L, -19);
            d->board_fast = 1;
            d->board_lo = delta;
            d->board_hi = L - delta;
            d->board_out = L + delta;
            d->board_far = std::ldexp(L, 24);
        }
    }
    for (int m = 0; m < 5; ++m) d->mat[m] = dm[m];
    d->transparent = any_transparent ? 1 : 0;
    d->tree = tree ? 1 : 0;
    d->hits_inside = 0;                  // set below, once every object's extent is known
    d->hits_lim2 = -1.0;
    d->counters = nullptr;
    d->hits_ok = 0;                      // per eye, rt_prepare_kernel
    d->n_lights = s->n_lights;
    for (int k = 0; k < s->n_lights; ++k) {
        for (int q = 0; q < 3; ++q) {
            d->light[k].pos[q] = s->lights[k].position[q];
            d->light[k].col[q] = s->lights[k].color[q];
        }
    }
    d->n_spheres = s->n_spheres;
    for (int k = 0; k < s->n_spheres; ++k) {
        HP c = hp(s->spheres[k].center) + bc;                                   // sphere: _position + offset
        put(sph[k].c, c);
        sph[k].r2 = s->spheres[k].radius * s->spheres[k].radius;                // :750
        // FP32 filter image (rt_device.hpp sphere_reject32): centre relative to bc, and
        // rm = r2 + 4K sC^2 + K r2 rounded up, sC = max|c_i - bc_i|.
        HP rel = c - bc;
        double sC = std::max(std::fabs(rel.x), std::max(std::fabs(rel.y), std::fabs(rel.z)));
        double K = (double)rt::kFilterK;
        double rm = sph[k].r2 + 4 * K * sC * sC + K * sph[k].r2;
        sphf[k].cx = (float)rel.x;
        sphf[k].cy = (float)rel.y;
        sphf[k].cz = (float)rel.z;
        float rmf = (float)rm;
        if ((double)rmf < rm) rmf = std::nextafter(rmf, std::numeric_limits<float>::infinity());
        sphf[k].rm = rmf;
    }
    for (int k = s->n_spheres; k < ns; ++k) {                                   // padding: never a hit
        sph[k].r2 = -inf;
        sphf[k].rm = -std::numeric_limits<float>::infinity();
    }
    // Shadow-ray cone filter (rt_device.hpp occluded): a shadow ray Line(p, L) lies on a line through the
    // light L, so it can meet sphere k only if |u . v_k| >= cos(phi_k), v_k = unit(C_k - L),
    // sin(phi_k) = r / |C_k - L|.  Stored: f32(v_k) and c_k = cos(phi_k) - 2^-16 rounded down; a light
    // inside or near a sphere (|C - L| <= r (1 + 2^-20) or |C - L| <= 2^-14 (1 + |L| + |C|)) gets c = -inf
    // (always tested), padding spheres c = +inf (never).
    rt::DevSphereLightF* lightf = reinterpret_cast<rt::DevSphereLightF*>(
        reinterpret_cast<rt::DevSphereCone*>(reinterpret_cast<rt::DevSpherePrimF*>(sphf + ns) + ns) + ns);
    for (int i = 0; i < s->n_lights; ++i) {
        const HP L = hp(s->lights[i].position);
        const double aL = std::max(std::fabs(L.x), std::max(std::fabs(L.y), std::fabs(L.z)));
        for (int k = 0; k < ns; ++k) {
            rt::DevSphereLightF& f = lightf[i * ns + k];
            f.vx = f.vy = f.vz = 0.0f;
            if (k >= s->n_spheres) {
                f.c = std::numeric_limits<float>::infinity();
                continue;
            }
            const HP C = hp(sph[k].c[0], sph[k].c[1], sph[k].c[2]);
            const HP v = C - L;
            const double D = length(v), r = std::fabs(s->spheres[k].radius);
            const double aC = std::max(std::fabs(C.x), std::max(std::fabs(C.y), std::fabs(C.z)));
            if (!(D > r * (1.0 + 0x1p-20) && D > 0x1p-14 * (1.0 + aL + aC))) {
                f.c = -std::numeric_limits<float>::infinity();
                continue;
            }
            const double sn = r / D;
            const double c = std::sqrt(std::max(0.0, 1.0 - sn * sn)) - 0x1p-16;
            f.vx = (float)(v.x / D);
            f.vy = (float)(v.y / D);
            f.vz = (float)(v.z / D);
            float cf = (float)c;
            if ((double)cf > c) cf = std::nextafter(cf, -std::numeric_limits<float>::infinity());
            f.c = cf;
        }
    }
    // Meshes (Tetrahedron :863-900, Cube :903-950): Shape(p, m, sqrt(3)*edge/2, false) with Triangle /
    // Quad sub-objects at zero position.  World vertex 0 of a triangle: tetrahedron (zero + (p + bc)) + v0,
    // cube (zero + (zero + (p + bc))) + v0 — the chain of `_position + positionOffset` additions (:739, :640).
    rt::DevMesh* dmesh = reinterpret_cast<rt::DevMesh*>(lightf + (size_t)s->n_lights * ns);
    rt::DevTri* dtri = reinterpret_cast<rt::DevTri*>(dmesh + s->n_meshes);
    d->n_meshes = s->n_meshes;
    d->n_tris = n_tris;
    int t_next = 0;
    for (int m = 0; m < s->n_meshes; ++m) {
        const rt_mesh& M = s->meshes[m];
        rt::DevMesh& DM = dmesh[m];
        const HP mpos = hp(M.position) + bc;                                    // Shape: _position + offset
        const double radius = std::sqrt((double)3) * M.edge / 2;
        put(DM.bc, mpos);
        DM.br2 = radius * radius;
        DM.inner2 = radius > 2 && s->small_number < 0.5 ? (radius - 1) * (radius - 1) : -1.0;   // (as g_scene's)
        DM.tri0 = t_next;
        DM.child = (s->has_board ? 1 : 0) + M.after_spheres + m;
        const double h = M.edge / 2;
        std::vector<std::array<HP, 3>> tris;
        HP tpos;
        if (M.kind == RT_MESH_TETRAHEDRON) {
            DM.mat = 3;
            DM.per_face = 1;
            DM.nfaces = 4;
            tris = {{hp(-h, -h, -h), hp(h, -h, -h), hp(-h, -h, h)},                 // bottom
                    {hp(-h, -h, -h), hp(-h, -h, h), hp(-h, h, -h)},                 // back
                    {hp(-h, -h, -h), hp(-h, h, -h), hp(-h, -h, h)},                 // left
                    {hp(-h, -h, h), hp(h, -h, -h), hp(-h, h, -h)}};                 // front
            tpos = zero + mpos;
        } else {
            DM.mat = 4;
            DM.per_face = 2;
            DM.nfaces = 6;
            const HP q[6][4] = {{hp(-h, h, -h), hp(h, h, -h), hp(h, h, h), hp(-h, h, h)},        // top
                                {hp(-h, -h, -h), hp(h, -h, -h), hp(h, -h, h), hp(-h, -h, h)},    // bottom
                                {hp(-h, -h, -h), hp(-h, h, -h), hp(-h, h, h), hp(-h, -h, h)},    // left
                                {hp(h, -h, -h), hp(h, h, -h), hp(h, h, h), hp(h, -h, h)},        // right
                                {hp(-h, -h, -h), hp(h, -h, -h), hp(h, h, -h), hp(-h, h, -h)},    // back
                                {hp(-h, -h, h), hp(h, -h, h), hp(h, h, h), hp(-h, h, h)}};       // front
            for (int f = 0; f < 6; ++f) {                                       // Quad: T(p1,p2,p3), T(p1,p3,p4)
                tris.push_back({q[f][0], q[f][1], q[f][2]});
                tris.push_back({q[f][0], q[f][2], q[f][3]});
            }
            tpos = zero + (zero + mpos);
        }
        for (const auto& tv : tris) {
            rt::DevTri& T = dtri[t_next++];
            HP u = tv[1] - tv[0], v = tv[2] - tv[0];                            // :413-414
            HP n = cross(u, v);                                                 // :415
            bool degenerate = length(n) < s->small_number;                      // :418
            n = normalize(n);                                                   // :422
            double uv = dot(u, v), uu = dot(u, u), vv = dot(v, v);             // :424-426
            double den = uv * uv - uu * vv;                                     // :428
            if (std::fabs(den) < s->small_number) degenerate = true;            // :430
            put(T.v0, tpos + tv[0]);                                            // :640-641
            put(T.u, u);
            put(T.v, v);
            put(T.n, n);
            T.uv = uv;
            T.uu = uu;
            T.vv = vv;
            T.den = den;
            T.thr = (den < 0 && std::fabs(den) >= 1024.0) ? std::ldexp(std::fabs(den), -1070) : inf;
            T.fast = const_quotient_ok(den);
            T.degenerate = degenerate ? 1.0 : 0.0;
        }
    }
    // Rays that start at a hit point pass g_scene's bounding-sphere cull when every hit point lies within
    // R - 1 of its centre (the kernel's bound_pass shortcut, rt_device.hpp): an upper bound of |q - bc| over
    // the spheres (|C - bc| + r), the board's corners and the meshes' bounding spheres, with a margin far
    // above the rounding of the hit points, lets the kernel skip the test for them (hits_inside).
    if (d->bound_on && d->inner2 > 0) {
        double far = 0.0;
        for (int k = 0; k < s->n_spheres; ++k)
            far = std::max(far, length(hp(sph[k].c[0], sph[k].c[1], sph[k].c[2]) - bc) + std::fabs(s->spheres[k].radius));
        if (d->has_board) {
            const double h = s->board_half_size;
            const HP quad = hp(s->board_position) + bc;
            for (int cx = -1; cx <= 1; cx += 2)
                for (int cz = -1; cz <= 1; cz += 2) far = std::max(far, length(quad + hp(cx * h, 0, cz * h) - bc));
        }
        for (int m = 0; m < s->n_meshes; ++m)
            far = std::max(far, length(hp(dmesh[m].bc[0], dmesh[m].bc[1], dmesh[m].bc[2]) - bc) + std::sqrt(dmesh[m].br2));
        // Hit points carry rounding that grows with their ray's origin o (D = |o - bc|): a sphere hit's
        // |q - C|^2 = r^2 + err(disc), err(disc) <= 2^-49 D^2 (the sqrt keeps it below 2^-50 D^2 / r in |q - C|),
        // and p0 + s u or p0 + m d adds <= 2^-51 (D + |bc| + far).  dev(D) = 2^-44 (D + |bc| + far + 1 + D^2 / rmin)
        // bounds both with room; the shortcut is kept for origins with dev(D) <= slack / 2 (hits_lim2, checked per
        // ray on the device: the camera eye per render, every start of a ray list), and only when that covers the
        // hit points themselves (D = R: the origins of later levels).
        const double Rin = std::sqrt(d->inner2) * (1.0 - 1e-9);
        const double slack = Rin - far - 1e-6 * (1.0 + far);
        double rmin = std::numeric_limits<double>::infinity();
        for (int k = 0; k < s->n_spheres; ++k) rmin = std::min(rmin, std::fabs(s->spheres[k].radius));
        const double absbc = length(bc);
        const double e = 0x1p-44, a = rmin > 0 ? e / rmin : inf, c = e * (absbc + far + 1.0) - slack / 2;
        double dlim = -1.0;                                  // largest D with a D^2 + e D + c <= 0
        if (std::isfinite(far) && std::isfinite(absbc) && slack > 0 && c < 0)
            dlim = std::isfinite(a) ? (-e + std::sqrt(e * e - 4 * a * c)) / (2 * a) : -c / e;
        if (dlim >= Rin) {
            d->hits_inside = 1;
            d->hits_lim2 = dlim * dlim * (1.0 - 1e-9);
        }
    }
    return RT_OK;
}

// R = G = B bit for bit in every frame of the scene: rayTraceRay's colour (:1213-1247) is built from the
// light colours, the material terms and scalar factors by component-wise products and sums only, and every
// decision (hits, shadows, which continuations, :1221, :1230-1247) is the same for the three channels (it
// depends on geometry and on "any component != 0" tests), so equal components in every term that enters the
// sum give equal channels.  Checked: the materials the scene's objects carry and every light colour.
extern "C" int rt_scene_achromatic(const rt_scene* s, int* out) {
    if (!s || !out) return rt_fail(RT_EINVAL, "rt_scene_achromatic: null pointer");
    *out = 0;
    auto grey = [](const double v[3]) { return v[0] == v[1] && v[1] == v[2]; };
    auto grey_mat = [&](const rt_material& m) {
        return grey(m.ambient) && grey(m.diffuse) && grey(m.specular) && grey(m.transparency);
    };
    if (s->n_lights > 0 && !s->lights) return rt_fail(RT_EINVAL, "rt_scene_achromatic: null lights");
    if (s->n_meshes > 0 && !s->meshes) return rt_fail(RT_EINVAL, "rt_scene_achromatic: null meshes");
    bool ok = true;
    if (s->has_board) ok = ok && grey_mat(s->white_square) && grey_mat(s->black_square);
    if (s->n_spheres > 0) ok = ok && grey_mat(s->sphere_material);
    for (int m = 0; m < s->n_meshes && ok; ++m)
        ok = grey_mat(s->meshes[m].kind == RT_MESH_TETRAHEDRON ? s->tetrahedron_material : s->cube_material);
    for (int k = 0; k < s->n_lights && ok; ++k) ok = grey(s->lights[k].color);
    *out = ok ? 1 : 0;
    return RT_OK;
}

extern "C" int rt_write_ppm(const char* path, const uint8_t* px, int W, int H, int channels) {
    // writePpmScreenshot (Hw4/ppm.cpp:15-25): header "P6 W H 255\n", then the bottom-up GL image's rows
    // written top-down (image[3*w*(h-1-i)]).
    if (!path || !px || W <= 0 || H <= 0 || (channels != 1 && channels != 3 && channels != 4))
        return rt_fail(RT_EINVAL, "rt_write_ppm: bad args");
    FILE* f = fopen(path, "wb");
    if (!f) return rt_fail(RT_EINVAL, std::string("rt_write_ppm: cannot open ") + path);
    fprintf(f, "P6 %d %d 255\n", W, H);
    std::vector<unsigned char> row((size_t)W * 3);
    for (int i = 0; i < H; ++i) {
        const uint8_t* src = px + (size_t)(H - 1 - i) * W * channels;
        for (int x = 0; x < W; ++x) {                        // GRAY8 (channels 1): R = G = B
            row[3 * x] = src[channels * x];
            row[3 * x + 1] = src[channels * x + (channels > 1 ? 1 : 0)];
            row[3 * x + 2] = src[channels * x + (channels > 1 ? 2 : 0)];
        }
        if (fwrite(row.data(), 1, row.size(), f) != row.size()) {
            fclose(f);
            return rt_fail(RT_EINVAL, "rt_write_ppm: short write");
        }
    }
    fclose(f);
    return RT_OK;
}
