// rt_device.hpp — FP64 device math and the per-ray tracer of the MI355X path.
//
// Every value that reaches the image is computed with the reference's exact IEEE binary64 operation
// order; the file is compiled with -ffp-contract=off so no a*b+c is fused.
// Citations are into /root/reference/Hw4/MySdlApplication.cpp.
//
// Restatement choices, each bit-identical to the reference (argued at its use):
//  * u = normalize(end - start) is computed once per ray, not once per child (Line::direction :258-263
//    recomputes the same expression on the same inputs);
//  * the closest-hit search keeps (distance, child, point); normal / reflection / material are computed
//    once for the winner (pure functions of the winner's point);
//  * the board's two triangles share vertex 0 and normal, so the plane step (m, p, w) is done once;
//  * shadow rays stop at the first blocker (any-hit): rayTraceRay reads only intersects() and the
//    blocker's transparency (:1221), and the GPU path only accepts opaque materials;
//  * the recursion (:1238-1247) is a loop; with opacity (1,1,1) the colour of level k is
//    local[k] + colour[k+1], so the frame colour is the right-nested sum local[0] + (local[1] + ...);
//  * for primary rays p0 = eye for every pixel, so deltaP = C - eye and dot(deltaP, deltaP) (:740, :750)
//    are computed once per workgroup, with the same operations, instead of once per ray;
// and work-skipping tests that are exact:
//  * FP32 sphere filter: a sphere is skipped only when an FP32 evaluation of the discriminant with a
//    proven error margin shows disc < 0, i.e. the FP64 test would report a miss (sphere_reject32);
//  * board: m = num/nd and s = A/den, t = B/den are divided only when the sign of the operands leaves the
//    quotient's sign test open (board_hit);
//  * bounding sphere: an origin with |o - c|^2 < (R-1)^2 provably passes the cull (bound_pass).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rt_layout.hpp"

namespace rt {

struct d3 {
    double x, y, z;
};

__device__ __forceinline__ d3 mk(double x, double y, double z) { return d3{x, y, z}; }
__device__ __forceinline__ d3 add(d3 a, d3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }     // :196-197
__device__ __forceinline__ d3 sub(d3 a, d3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }     // :199-200
__device__ __forceinline__ d3 scl(double s, d3 a) { return mk(s * a.x, s * a.y, s * a.z); }       // :1118-1131
__device__ __forceinline__ d3 had(d3 a, d3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }     // :192-193
__device__ __forceinline__ double dot(d3 a, d3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }   // :189-190
__device__ __forceinline__ double len(d3 a) { return sqrt(a.x * a.x + a.y * a.y + a.z * a.z); }  // :174
__device__ __forceinline__ d3 divs(d3 a, double l) { return mk(a.x / l, a.y / l, a.z / l); }      // :175
__device__ __forceinline__ d3 ld3(const double* p) { return mk(p[0], p[1], p[2]); }

// Where the kernels read the scene from.  `S`, `sph`, `prim` (header and FP64 exact records) live in
// LDS in the render kernel (or in global memory for the ray-list kernels); the FP32 filter images `sphf`,
// `primf` are always read from global memory with wave-uniform indices, i.e. through the scalar cache
// into SGPR operands.
struct SceneView {
    const DevScene* S;
    const DevSphere* sph;
    const DevSpherePrim* prim;
    const DevSphereF* sphf;
    const DevSpherePrimF* primf;
    int np;                          // padded sphere count (wave-uniform)
    int nl;                          // light count (wave-uniform)
};

// hdr: header copy the kernel reads (LDS or global); g: the global record (for the filter images).
__device__ __forceinline__ SceneView view_of(const DevScene* hdr, const DevScene* g, int np, int nl) {
    SceneView v;
    v.S = hdr;
    v.np = np;
    v.nl = nl;
    v.sph = reinterpret_cast<const DevSphere*>(hdr + 1);
    v.prim = reinterpret_cast<const DevSpherePrim*>(v.sph + np);
    const DevSphere* gsph = reinterpret_cast<const DevSphere*>(g + 1);
    const DevSpherePrim* gprim = reinterpret_cast<const DevSpherePrim*>(gsph + np);
    v.sphf = reinterpret_cast<const DevSphereF*>(gprim + np);
    v.primf = reinterpret_cast<const DevSpherePrimF*>(v.sphf + np);
    return v;
}

// A ray Line(p0, p0 + d) with u = normalize(d), plus its FP32 filter image.
struct Ray {
    d3 p0, d, u;
    float px, py, pz;    // f32(p0 - bound centre)
    float ux, uy, uz;    // f32(u)
    float mP;            // 4K * max|p_i|^2 (the ray's share of the filter margin)
};

__device__ __forceinline__ void set_origin_f32(const DevScene* S, Ray* r) {
    r->px = (float)(r->p0.x - S->bc[0]);
    r->py = (float)(r->p0.y - S->bc[1]);
    r->pz = (float)(r->p0.z - S->bc[2]);
    float sp = fmaxf(fabsf(r->px), fmaxf(fabsf(r->py), fabsf(r->pz)));
    r->mP = 4.0f * kFilterK * sp * sp;
}

__device__ __forceinline__ void set_dir(Ray* r, d3 d, d3 u) {
    r->d = d;
    r->u = u;
    r->ux = (float)u.x;
    r->uy = (float)u.y;
    r->uz = (float)u.z;
}

// ------------------------------------------------------------------------------------------------
// g_scene bounding-sphere cull (:747-758): miss iff disc < 0 or |s| < eps.
// Shortcut: if dd = |bc - p0|^2 < (R-1)^2 the cull passes.  Proof: m = R^2 - dd >= 2R - 1 > 0, so
// disc = uD^2 + m > 0 and s = uD - sqrt(disc) < 0 with |s| = m / (sqrt(uD^2 + m) + uD) >= m / (R + |dP|)
// >= (2R - 1) / (2R - 1) = 1 >> eps (sqrt(uD^2 + m) <= R since uD^2 <= dd); FP64 rounding is ~1e-13.
__device__ __forceinline__ bool bound_pass_dp(const DevScene* S, d3 dP, double dd, d3 u) {
    if (!S->bound_on) return true;
    if (dd < S->inner2) return true;
    double uD = dot(u, dP);
    double disc = uD * uD - dd + S->br2;
    if (disc < 0) return false;
    double s = uD - sqrt(disc);
    return !(fabs(s) < S->eps);
}

__device__ __forceinline__ bool bound_pass(const DevScene* S, d3 p0, d3 u) {
    if (!S->bound_on) return true;
    d3 dP = sub(ld3(S->bc), p0);
    return bound_pass_dp(S, dP, dot(dP, dP), u);
}

// CheckerBoard -> Quad -> Triangle T1 then T2, first hit wins (:1097, :817, :611-707).
// d = end - start (unnormalised, :647).  Returns the hit point in *p.
__device__ __forceinline__ bool board_hit(const DevScene* S, d3 p0, d3 d, d3* p) {
    const DevTri& T = S->tri[0];
    d3 n = ld3(T.n);
    double nd = dot(n, d);                                  // :648
    if (fabs(nd) < S->eps) return false;                    // :651
    d3 v0 = ld3(T.v0);
    double num = dot(n, sub(v0, p0));                       // :657 numerator
    // m = num / nd is <= 0 (hence < eps, a miss at :659) when num == 0 or the signs differ.  NaNs fall
    // through to the division and miss there, as in the reference.
    if (num == 0.0 || ((num < 0.0) != (nd < 0.0))) return false;
    double m = num / nd;                                    // :657 (its denominator recomputed: same value)
    if (m < S->eps) return false;                           // :659
    d3 q = add(p0, scl(m, d));                              // :665
    d3 w = sub(q, v0);                                      // :667
#pragma unroll
    for (int t = 0; t < 2; ++t) {
        const DevTri& Tt = S->tri[t];
        double wu = dot(w, ld3(Tt.u));                      // :670
        double wv = dot(w, ld3(Tt.v));                      // :671
        double A = Tt.uv * wv - Tt.vv * wu;
        double B = Tt.uv * wu - Tt.uu * wv;
        // den < 0 (host-checked, else thr = +inf): A > thr = |den| 2^-1070 makes A/den negative and nonzero,
        // so s >= 0 fails without dividing; likewise B for t.
        if (A > Tt.thr || B > Tt.thr) continue;
        double s = A / Tt.den;                              // :673
        double tt = B / Tt.den;                             // :674
        if (s >= 0 && tt >= 0 && s + tt <= 1) {             // :676
            *p = q;
            return true;
        }
    }
    return false;
}

// FP32 filter: true only if disc = uD^2 - |dP|^2 + r^2 < 0 is certain.
// Error budget (eps32 = 2^-24; S >= |c_i| + |p_i| per component, c, p relative to the bound centre):
// |d(dx)| <= 2 eps32 S; |d(uD)| <= 10.4 eps32 S; |d(uD^2)| <= 36 eps32 S^2; |d(dd)| <= 21 eps32 S^2;
// fma roundings <= 6 eps32 S^2 + eps32 r^2; total < 64 eps32 (S^2 + r^2) = (K/4)(S^2 + r^2).
// The margin folded into rm + mP is 4K(sC^2 + sp^2) + K r^2 >= 2K S^2 + K r^2, so a negative FP32
// value implies a negative exact discriminant.  Inf/NaN compare false and fall through to FP64.
__device__ __forceinline__ bool sphere_reject32(const DevSphereF& f, const Ray& r) {
    float dx = f.cx - r.px, dy = f.cy - r.py, dz = f.cz - r.pz;
    float e = f.rm + r.mP;
    e = fmaf(-dx, dx, e);
    e = fmaf(-dy, dy, e);
    e = fmaf(-dz, dz, e);
    float uD = r.ux * dx;
    uD = fmaf(r.uy, dy, uD);
    uD = fmaf(r.uz, dz, uD);
    return fmaf(uD, uD, e) < 0.0f;
}

// Sphere (:747-772), exact FP64: candidate point if disc >= 0 and s >= eps.
__device__ __forceinline__ bool sphere_hit_dp(d3 dP, double dd, double r2, d3 p0, d3 u, double eps, d3* p) {
    double uD = dot(u, dP);                                 // :749
    double disc = uD * uD - dd + r2;                        // :750
    if (disc < 0) return false;                             // :754
    double s = uD - sqrt(disc);                             // :752
    if (s < eps) return false;                              // covers |s| < eps (:754) and s < eps (:767)
    *p = add(p0, scl(s, u));                                // :762
    return true;
}

__device__ __forceinline__ bool sphere_hit(const DevSphere& sp, d3 p0, d3 u, double eps, d3* p) {
    d3 dP = sub(ld3(sp.c), p0);                             // :740
    return sphere_hit_dp(dP, dot(dP, dP), sp.r2, p0, u, eps, p);
}

// Closest hit of g_scene (:796-821): Euclidean distance |p - p0|, strict <, board (child 0) first.
// kind: -1 miss, 0 board, 1 + k sphere k.
// Spheres go in batches of kChunk: the FP32 filter of the whole batch is evaluated branch-free (records
// in SGPRs), then each lane runs the exact FP64 test only on its own surviving spheres, in increasing k,
// so the strict-< closest-hit order of the reference is unchanged.  Padding spheres never survive.
__device__ __forceinline__ void sphere_batch_closest(const SceneView& V, const Ray& r, int k0, double eps,
                                                     int* kind, double* best, d3* hp) {
    uint32_t pass = 0;
#pragma unroll
    for (int j = 0; j < kChunk; ++j) pass |= (sphere_reject32(V.sphf[k0 + j], r) ? 0u : 1u) << j;
    while (pass) {
        const int k = k0 + __builtin_ctz(pass);
        pass &= pass - 1;
        d3 q;
        if (sphere_hit(V.sph[k], r.p0, r.u, eps, &q)) {
            double dist = len(sub(q, r.p0));                // :811-812
            if (dist < *best || *best < 0.0) {              // :813
                *best = dist;
                *kind = 1 + k;
                *hp = q;
            }
        }
    }
}

__device__ __forceinline__ int closest_hit(const SceneView& V, const Ray& r, d3* hp) {
    const DevScene* S = V.S;
    if (!bound_pass(S, r.p0, r.u)) return -1;
    int kind = -1;
    double best = -1.0;
    if (S->has_board) {
        d3 q;
        if (board_hit(S, r.p0, r.d, &q)) {
            kind = 0;
            best = len(sub(q, r.p0));
            *hp = q;
        }
    }
    const double eps = S->eps;
    for (int k0 = 0; k0 < V.np; k0 += kChunk) sphere_batch_closest(V, r, k0, eps, &kind, &best, hp);
    return kind;
}

// Closest hit of a primary ray Line(eye, sp): deltaP and |deltaP|^2 per sphere were computed for this
// eye by rt_prepare_kernel with the reference's operations (:740, :750).
__device__ __forceinline__ int closest_hit_primary(const SceneView& V, const Ray& r, d3 bdP, double bdd,
                                                   d3* hp) {
    const DevScene* S = V.S;
    if (!bound_pass_dp(S, bdP, bdd, r.u)) return -1;
    int kind = -1;
    double best = -1.0;
    if (S->has_board) {
        d3 q;
        if (board_hit(S, r.p0, r.d, &q)) {
            kind = 0;
            best = len(sub(q, r.p0));
            *hp = q;
        }
    }
    const double eps = S->eps;
    for (int k0 = 0; k0 < V.np; k0 += kChunk) {
        uint32_t pass = 0;
#pragma unroll
        for (int j = 0; j < kChunk; ++j) {
            const DevSpherePrimF& f = V.primf[k0 + j];
            float uD = r.ux * f.dx;
            uD = fmaf(r.uy, f.dy, uD);
            uD = fmaf(r.uz, f.dz, uD);
            pass |= (fmaf(uD, uD, f.c0) < 0.0f ? 0u : 1u) << j;   // < 0: certain disc < 0
        }
        while (pass) {
            const int k = k0 + __builtin_ctz(pass);
            pass &= pass - 1;
            const DevSpherePrim& pp = V.prim[k];
            d3 q;
            if (sphere_hit_dp(ld3(pp.dP), pp.dd, V.sph[k].r2, r.p0, r.u, eps, &q)) {
                double dist = len(sub(q, r.p0));
                if (dist < best || best < 0.0) {
                    best = dist;
                    kind = 1 + k;
                    *hp = q;
                }
            }
        }
    }
    return kind;
}

// Shadow test: intersects() of g_scene.intersection(Line(pt, Lpos)) (:1216-1221), any hit.
__device__ __forceinline__ bool occluded(const SceneView& V, const Ray& r) {
    const DevScene* S = V.S;
    if (!bound_pass(S, r.p0, r.u)) return false;
    const double eps = S->eps;
    for (int k0 = 0; k0 < V.np; k0 += kChunk) {
        uint32_t pass = 0;
#pragma unroll
        for (int j = 0; j < kChunk; ++j) pass |= (sphere_reject32(V.sphf[k0 + j], r) ? 0u : 1u) << j;
        while (pass) {
            const int k = k0 + __builtin_ctz(pass);
            pass &= pass - 1;
            d3 q;
            if (sphere_hit(V.sph[k], r.p0, r.u, eps, &q)) return true;
        }
    }
    if (S->has_board) {
        d3 q;
        if (board_hit(S, r.p0, r.d, &q)) return true;
    }
    return false;
}

// Surface data of a hit: normal, material id, reflected end point p + r (:679-683, :774-778, :1101-1111).
__device__ __forceinline__ void surface(const SceneView& V, int kind, d3 p, d3 u, d3* n, int* mat, d3* pe) {
    const DevScene* S = V.S;
    if (kind == 0) {
        *n = ld3(S->tri[0].n);
        d3 q = add(sub(p, ld3(S->coff)), mk(S->half, 0.0, S->half));
        int squareSum = (int)(q.x / S->square) + (int)(q.z / S->square);
        *mat = (squareSum & 1) == 0 ? 0 : 1;
    } else {
        d3 c = ld3(V.sph[kind - 1].c);
        d3 dp = sub(p, c);                                  // directionP0 (:763)
        *n = divs(dp, len(dp));                             // :774-775
        *mat = 2;
    }
    d3 r = sub(u, scl(2 * dot(u, *n), *n));                 // :682 / :777
    *pe = add(p, r);                                        // Line(p, p + r)
}

// Local illumination of one hit over all lights (:1213-1228).  u = incoming ray direction,
// rdir = reflectedRay().direction().
__device__ __forceinline__ d3 shade(const SceneView& V, d3 p, d3 n, int mat, d3 u, d3 rdir) {
    const DevScene* S = V.S;
    const DevMat& M = S->mat[mat];
    d3 amb = ld3(M.amb), dif = ld3(M.diff), spc = ld3(M.spec);
    double ks = fabs(dot(u, rdir));
    d3 color = mk(0.0, 0.0, 0.0);
    Ray sr;
    sr.p0 = p;
    set_origin_f32(S, &sr);
    for (int i = 0; i < V.nl; ++i) {
        d3 lpos = ld3(S->light[i].pos);
        d3 sd = sub(lpos, p);                               // shadowRay end - start (:1216)
        double dl = len(sd);                                // shadowRay.length()
        d3 sdir = divs(sd, dl);                             // shadowRay.direction()
        set_dir(&sr, sd, sdir);
        if (!occluded(V, sr)) {
            double a = S->att / (S->att + dl * dl);         // attenuation (:1181)
            d3 lC = scl(a, ld3(S->light[i].col));           // :1223
            d3 term = add(add(had(amb, lC), scl(fabs(dot(n, sdir)), had(dif, lC))), scl(ks, had(spc, lC)));
            color = add(color, term);                       // :1224-1226
        }
    }
    return color;
}

// rayTraceRay(g_scene, lights, Line(p0, p1), color, B) with color starting at 0 (:1184-1249), as a loop.
// PRIMARY: p0 is the camera and V.prim/V.primf hold its per-sphere data; (bdP, bdd) = bc - eye, |.|^2.
// seg / shadow count the rays actually traced.
template <int B, bool PRIMARY>
__device__ __forceinline__ d3 trace(const SceneView& V, d3 p0, d3 p1, d3 bdP, double bdd, uint32_t* seg,
                                    uint32_t* shadow) {
    const DevScene* S = V.S;
    d3 local[B + 1];
    int levels = 0;
    Ray r;
    r.p0 = p0;
    d3 d = sub(p1, p0);
    set_dir(&r, d, divs(d, len(d)));
    uint32_t nseg = 0, nsh = 0;
#pragma unroll
    for (int lvl = 0; lvl <= B; ++lvl) {
        local[lvl] = mk(0.0, 0.0, 0.0);
        bool alive = lvl == 0 || levels == lvl;
        if (!__any(alive)) break;                           // the whole wave has missed: early out
        if (alive) {
            ++nseg;
            d3 p;
            int kind;
            if (PRIMARY && lvl == 0) {
                kind = closest_hit_primary(V, r, bdP, bdd, &p);
            } else {
                set_origin_f32(S, &r);
                kind = closest_hit(V, r, &p);
            }
            if (kind >= 0) {
                d3 n, pe;
                int mat;
                surface(V, kind, p, r.u, &n, &mat, &pe);
                d3 rd = sub(pe, p);                         // reflectedRay = Line(p, p + r)
                d3 rdir = divs(rd, len(rd));                // reflectedRay.direction()
                local[lvl] = shade(V, p, n, mat, r.u, rdir);
                nsh += V.nl;
                levels = lvl + 1;
                r.p0 = p;                                   // next level traces the reflected ray
                set_dir(&r, rd, rdir);
            }
        }
    }
    d3 acc = mk(0.0, 0.0, 0.0);
#pragma unroll
    for (int lvl = B; lvl >= 0; --lvl) {
        if (lvl < levels) acc = (lvl == levels - 1) ? local[lvl] : add(local[lvl], acc);
    }
    *seg = nseg;
    *shadow = nsh;
    return acc;
}

}  // namespace rt
