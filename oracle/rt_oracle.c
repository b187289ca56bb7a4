/*
 * rt_oracle.c — CPU restatement of the reference ray tracer.  TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library, and
 * only as the checker / the timed CPU baseline.  The product path (ray_tracer_fragment_shader_amd)
 * never links or calls it.
 *
 * What it restates (all citations into /root/reference/Hw4/MySdlApplication.cpp):
 *   Point ops                  :136-212, operator*(scalar,Point) :1118-1146
 *   Line::direction/length     :258-269
 *   Triangle ctor              :406-433      Triangle::intersection  :611-707
 *   Shape::intersection        :724-823      (bounding sphere, sphere, composite closest hit)
 *   Quad                       :826-843      (2 triangles, first hit wins)
 *   CheckerBoard::intersection :1084-1113
 *   Tetrahedron ctor           :863-900      Cube ctor :903-950 (composite Shapes of Triangles / Quads)
 *   attenuation                :1171-1182    rayTraceRay :1184-1249 (recursive, as the reference)
 *   rayTraceScreen basis       :1270-1279    convertStringCoordinate :1326-1346
 * The structure deliberately follows the reference (recursion, composite walk, closest hit for shadow
 * rays) rather than the GPU kernel's iterative / any-hit form, so the two are independent.
 *
 * Parity pinning: this restatement is checked bit-for-bit against the reference's own rayTraceRay
 * compiled from /root/reference (oracle/Makefile target `ref`, outputs in oracle/_ref/) and against the
 * committed fixtures in tests/golden/ generated from it (tests/golden/make_golden.py).
 *
 * Build: gcc -O2 -ffp-contract=off -fopenmp (see oracle/Makefile).  No FMA contraction, IEEE sqrt/div.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "../include/rt_api.h"

/* ---------------------------------------------------------------- Point (MySdlApplication.cpp:136-212) */
typedef struct { double x, y, z; } P;

static inline P pt(double x, double y, double z) { P p = {x, y, z}; return p; }
static inline P add(P a, P b) { return pt(a.x + b.x, a.y + b.y, a.z + b.z); }          /* :196-197 */
static inline P sub(P a, P b) { return pt(a.x - b.x, a.y - b.y, a.z - b.z); }          /* :199-200 */
static inline P scl(double s, P a) { return pt(s * a.x, s * a.y, s * a.z); }           /* :1118-1131 */
static inline P had(P a, P b) { return pt(a.x * b.x, a.y * b.y, a.z * b.z); }          /* :192-193 */
static inline double dot(P a, P b) { return a.x * b.x + a.y * b.y + a.z * b.z; }       /* :189-190 */
static inline P cross(P a, P b) {                                                     /* :186-187 */
    return pt(a.y * b.z - b.y * a.z, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
static inline double len(P a) { return sqrt(a.x * a.x + a.y * a.y + a.z * a.z); }     /* :174 */
static inline P nrm(P a) { double l = len(a); return pt(a.x / l, a.y / l, a.z / l); }  /* :175 */
static inline int is_zero(P a) { return a.x == 0 && a.y == 0 && a.z == 0; }           /* :173 */
static inline P from3(const double* v) { return pt(v[0], v[1], v[2]); }

/* Line (:234-270): direction = normalize(end - start), length = |end - start|. */
typedef struct { P s, e; } Line;
static inline P line_dir(Line l) { return nrm(sub(l.e, l.s)); }
static inline double line_len(Line l) { return len(sub(l.e, l.s)); }

typedef struct { P amb, diff, spec, transp; double refr; } Mat;

static Mat mat_from(const rt_material* m) {
    Mat r;
    r.amb = from3(m->ambient); r.diff = from3(m->diffuse); r.spec = from3(m->specular);
    r.transp = from3(m->transparency); r.refr = m->refraction;
    return r;
}

/* Intersection (:309-359) — the fields rayTraceRay reads. */
typedef struct {
    int hit;
    P point, normal;
    Mat mat;
    int mat_id;
    Line refl, trans;
} Inter;

/* ---------------------------------------------------------------- Triangle (:380-437, :611-707) */
typedef struct {
    P pos;                    /* RayObject::_position (zero for the board's triangles, :838-841) */
    P v0, v1, v2, u, v, n;
    double uv, uu, vv, den;
    int degenerate;
    Mat mat;
} Tri;

static void tri_init(Tri* t, P pos, Mat m, P p1, P p2, P p3, double eps) {  /* ctor :406-433 */
    t->pos = pos; t->mat = m;
    t->v0 = p1; t->v1 = p2; t->v2 = p3;
    t->u = sub(t->v1, t->v0);
    t->v = sub(t->v2, t->v0);
    t->n = cross(t->u, t->v);
    t->degenerate = len(t->n) < eps;
    t->n = nrm(t->n);
    t->uv = dot(t->u, t->v);
    t->uu = dot(t->u, t->u);
    t->vv = dot(t->v, t->v);
    t->den = t->uv * t->uv - t->uu * t->vv;
    if (fabs(t->den) < eps) t->degenerate = 1;
}

static void tri_intersect(const Tri* t, Line ray, P off, double eps, Inter* in) {  /* :611-707 */
    if (t->degenerate) { in->hit = 0; return; }
    P position = add(t->pos, off);
    P v0 = add(position, t->v0);
    P p0 = ray.s, p1 = ray.e;
    P diffP = sub(p1, p0);
    double ndiffP = dot(t->n, diffP);
    if (fabs(ndiffP) < eps) { in->hit = 0; return; }
    double m = dot(t->n, sub(v0, p0)) / dot(t->n, diffP);
    if (m < eps) { in->hit = 0; return; }
    P p = add(p0, scl(m, diffP));
    P w = sub(p, v0);
    double wu = dot(w, t->u), wv = dot(w, t->v);
    double s = (t->uv * wv - t->vv * wu) / t->den;
    double tt = (t->uv * wu - t->uu * wv) / t->den;
    if (s >= 0 && tt >= 0 && s + tt <= 1) {
        P u = nrm(diffP);
        P r = sub(u, scl(2 * dot(u, t->n), t->n));
        double rr = t->mat.refr;
        P tv = pt(0.0, 0.0, 0.0);
        double cti = dot(u, t->n);
        double modulus = 1 - rr * rr * (1 - cti * cti);
        if (modulus > 0) {
            double ctr = sqrt(modulus);
            tv = sub(scl(rr, u), scl(ctr + rr * cti, t->n));
        }
        in->hit = 1; in->point = p; in->normal = t->n; in->mat = t->mat; in->mat_id = -1;
        in->refl.s = p; in->refl.e = add(p, r);
        in->trans.s = p; in->trans.e = add(p, tv);
    } else {
        in->hit = 0;
    }
}

/* ---------------------------------------------------------------- scene = g_scene (:590) */
typedef struct {
    P pos;            /* Sphere's _position (scene-local) */
    double radius;
    Mat mat;
} Sph;

/* A composite Shape of the reference (Tetrahedron / Cube): bounding sphere, then sub-objects.
 * Tetrahedron sub-objects are Triangles; Cube sub-objects are Quads (2 triangles, first hit wins). */
typedef struct {
    int kind;         /* RT_MESH_TETRAHEDRON / RT_MESH_CUBE */
    P pos;            /* Shape _position (scene-local p) */
    double radius;    /* sqrt(3)*edge/2 */
    int mat_id;       /* 3 tetrahedron, 4 cube */
    int nfaces;
    int ntri[6];      /* 1 (triangle) or 2 (quad) */
    Tri tri[6][2];
} Mesh;

typedef struct { int type; int index; } Child;   /* type: 0 board, 1 sphere, 2 mesh */

typedef struct {
    P position;       /* g_scene _position */
    double radius;    /* g_scene _radius (bounding sphere) */
    double eps, att;
    int has_board;
    P board_p;        /* CheckerBoard(p): the Quad's _position (:1066) */
    Tri board_tri[2]; /* Quad(p, Material(), ...) sub-triangles (:826-843, :1066-1069) */
    double half, square;
    Mat white, black;
    int n_sph;
    Sph* sph;
    int n_lights;
    P lcol[RT_MAX_LIGHTS], lpos[RT_MAX_LIGHTS];
    int n_mesh;
    Mesh* mesh;
    Mat mesh_mat[3];  /* [1] tetrahedron, [2] cube */
    int n_child;
    Child* child;     /* g_scene _subObjects order */
} Scene;

static void mesh_build(Mesh* m, const rt_mesh* d, Mat mat, int mat_id, double eps) {  /* :863-950 */
    P zero = pt(0.0, 0.0, 0.0);
    double h = d->edge / 2;
    m->kind = d->kind;
    m->pos = from3(d->position);
    m->radius = sqrt((double)3) * d->edge / 2;
    m->mat_id = mat_id;
    if (d->kind == RT_MESH_TETRAHEDRON) {
        P v[4][3] = {
            {pt(-h, -h, -h), pt(h, -h, -h), pt(-h, -h, h)},     /* bottom */
            {pt(-h, -h, -h), pt(-h, -h, h), pt(-h, h, -h)},     /* back */
            {pt(-h, -h, -h), pt(-h, h, -h), pt(-h, -h, h)},     /* left */
            {pt(-h, -h, h), pt(h, -h, -h), pt(-h, h, -h)}};     /* front */
        m->nfaces = 4;
        for (int f = 0; f < 4; ++f) {
            m->ntri[f] = 1;
            tri_init(&m->tri[f][0], zero, mat, v[f][0], v[f][1], v[f][2], eps);
        }
    } else {
        P q[6][4] = {
            {pt(-h, h, -h), pt(h, h, -h), pt(h, h, h), pt(-h, h, h)},       /* top */
            {pt(-h, -h, -h), pt(h, -h, -h), pt(h, -h, h), pt(-h, -h, h)},   /* bottom */
            {pt(-h, -h, -h), pt(-h, h, -h), pt(-h, h, h), pt(-h, -h, h)},   /* left */
            {pt(h, -h, -h), pt(h, h, -h), pt(h, h, h), pt(h, -h, h)},       /* right */
            {pt(-h, -h, -h), pt(h, -h, -h), pt(h, h, -h), pt(-h, h, -h)},   /* back */
            {pt(-h, -h, h), pt(h, -h, h), pt(h, h, h), pt(-h, h, h)}};      /* front */
        m->nfaces = 6;
        for (int f = 0; f < 6; ++f) {                           /* Quad(zero, m, p1..p4) (:826-843) */
            m->ntri[f] = 2;
            tri_init(&m->tri[f][0], zero, mat, q[f][0], q[f][1], q[f][2], eps);
            tri_init(&m->tri[f][1], zero, mat, q[f][0], q[f][2], q[f][3], eps);
        }
    }
}

static int scene_build(const rt_scene* d, Scene* s) {
    memset(s, 0, sizeof(*s));
    if (d->n_spheres < 0 || d->n_lights < 0 || d->n_lights > RT_MAX_LIGHTS) return RT_EINVAL;
    s->position = from3(d->position);
    s->radius = d->radius;
    s->eps = d->small_number;
    s->att = d->attenuation_factor;
    s->has_board = d->has_board;
    s->board_p = from3(d->board_position);
    s->half = d->board_half_size;
    s->square = d->square_edge_size;
    s->white = mat_from(&d->white_square);
    s->black = mat_from(&d->black_square);
    {
        double h = s->half;
        Mat def; /* Material() (:291-293) */
        def.amb = pt(0.0, 0.0, 0.0); def.diff = def.amb; def.spec = def.amb; def.transp = def.amb;
        def.refr = 1;
        P p1 = pt(-h, 0, -h), p2 = pt(h, 0, -h), p3 = pt(h, 0, h), p4 = pt(-h, 0, h);
        P zero = pt(0.0, 0.0, 0.0);
        tri_init(&s->board_tri[0], zero, def, p1, p2, p3, s->eps);
        tri_init(&s->board_tri[1], zero, def, p1, p3, p4, s->eps);
    }
    s->n_sph = d->n_spheres;
    s->sph = (Sph*)calloc((size_t)(d->n_spheres > 0 ? d->n_spheres : 1), sizeof(Sph));
    if (!s->sph) return RT_ENOMEM;
    Mat sm = mat_from(&d->sphere_material);
    for (int k = 0; k < d->n_spheres; ++k) {
        s->sph[k].pos = from3(d->spheres[k].center);
        s->sph[k].radius = d->spheres[k].radius;
        s->sph[k].mat = sm;
    }
    s->n_lights = d->n_lights;
    for (int k = 0; k < d->n_lights; ++k) {
        s->lcol[k] = from3(d->lights[k].color);
        s->lpos[k] = from3(d->lights[k].position);
    }
    if (d->n_meshes < 0 || d->n_meshes > RT_MAX_MESHES || (d->n_meshes > 0 && !d->meshes)) return RT_EINVAL;
    s->mesh_mat[1] = mat_from(&d->tetrahedron_material);
    s->mesh_mat[2] = mat_from(&d->cube_material);
    s->n_mesh = d->n_meshes;
    s->mesh = (Mesh*)calloc((size_t)(d->n_meshes > 0 ? d->n_meshes : 1), sizeof(Mesh));
    s->child = (Child*)calloc((size_t)(1 + d->n_spheres + d->n_meshes), sizeof(Child));
    if (!s->mesh || !s->child) return RT_ENOMEM;
    for (int m = 0; m < d->n_meshes; ++m) {
        int kind = d->meshes[m].kind;
        if (kind != RT_MESH_TETRAHEDRON && kind != RT_MESH_CUBE) return RT_EINVAL;
        mesh_build(&s->mesh[m], &d->meshes[m], s->mesh_mat[kind], kind == RT_MESH_TETRAHEDRON ? 3 : 4, s->eps);
    }
    /* g_scene child order: board, then spheres with each mesh inserted after `after_spheres` spheres */
    int nc = 0, m = 0;
    if (s->has_board) { s->child[nc].type = 0; s->child[nc].index = 0; ++nc; }
    for (int k = 0; k <= d->n_spheres; ++k) {
        while (m < d->n_meshes && d->meshes[m].after_spheres <= k) {
            s->child[nc].type = 2; s->child[nc].index = m; ++nc; ++m;
        }
        if (k < d->n_spheres) { s->child[nc].type = 1; s->child[nc].index = k; ++nc; }
    }
    while (m < d->n_meshes) { s->child[nc].type = 2; s->child[nc].index = m; ++nc; ++m; }
    s->n_child = nc;
    return RT_OK;
}

static void scene_free(Scene* s) {
    free(s->sph); s->sph = NULL;
    free(s->mesh); s->mesh = NULL;
    free(s->child); s->child = NULL;
}

/* Quad = Shape(p, m, 0, false, true): no bound test (radius 0), first hit returns (:817). */
static void quad_intersect(const Scene* s, Line ray, P off, Inter* in) {
    P position = add(s->board_p, off);          /* Shape::intersection :739 */
    in->hit = 0;
    double minDistance = -1.0;
    for (int i = 0; i < 2; ++i) {
        Inter tmp;
        tri_intersect(&s->board_tri[i], ray, position, s->eps, &tmp);
        if (tmp.hit) {
            double d = len(sub(tmp.point, ray.s));
            if (d < minDistance || minDistance < 0.0) {
                minDistance = d;
                *in = tmp;
                return;                          /* _canIntersectOnlyOneSubObject */
            }
        }
    }
}

static void board_intersect(const Scene* s, Line ray, P off, Inter* in) {  /* :1084-1113 */
    quad_intersect(s, ray, off, in);
    if (in->hit) {
        P p = add(sub(in->point, off), pt(s->half, 0, s->half));
        int squareSum = (int)(p.x / s->square) + (int)(p.z / s->square);
        if ((squareSum & 1) == 0) { in->mat = s->white; in->mat_id = 0; }
        else { in->mat = s->black; in->mat_id = 1; }
    }
}

static void sphere_intersect(const Sph* sp, Line ray, P off, double eps, Inter* in) {  /* :737-793 */
    P u = line_dir(ray);
    P p0 = ray.s;
    P position = add(sp->pos, off);
    P deltaP = sub(position, p0);
    double uDeltaP = dot(u, deltaP);
    double disc = uDeltaP * uDeltaP - dot(deltaP, deltaP) + sp->radius * sp->radius;
    double s = uDeltaP - sqrt(disc);
    if (disc < 0 || fabs(s) < eps) { in->hit = 0; return; }
    P p = add(p0, scl(s, u));
    P dirP0 = sub(p, position);
    if (s < eps) { in->hit = 0; return; }
    P n = nrm(dirP0);
    P r = sub(u, scl(2 * dot(u, n), n));
    double rr = sp->mat.refr;
    P tv = pt(0.0, 0.0, 0.0);
    double cti = dot(u, n);
    double modulus = 1 - rr * rr * (1 - cti * cti);
    if (modulus > 0) {
        double ctr = sqrt(modulus);
        tv = sub(scl(rr, u), scl(ctr + rr * cti, n));
    }
    in->hit = 1; in->point = p; in->normal = n; in->mat = sp->mat; in->mat_id = 2;
    in->refl.s = p; in->refl.e = add(p, r);
    in->trans.s = p; in->trans.e = add(p, tv);
}

/* Tetrahedron / Cube: Shape::intersection with radius > 0, not a sphere (:736-823): bounding-sphere
 * cull, then the closest sub-object (strict <); a Cube's sub-objects are Quads (first hit, :817). */
static void mesh_intersect(const Mesh* me, Line ray, P off, double eps, Inter* in) {
    P u = line_dir(ray);
    P p0 = ray.s;
    P position = add(me->pos, off);
    P deltaP = sub(position, p0);
    if (me->radius > 0) {
        double uDeltaP = dot(u, deltaP);
        double disc = uDeltaP * uDeltaP - dot(deltaP, deltaP) + me->radius * me->radius;
        double sv = uDeltaP - sqrt(disc);
        if (disc < 0 || fabs(sv) < eps) { in->hit = 0; return; }
    }
    in->hit = 0;
    double minDistance = -1.0;
    for (int f = 0; f < me->nfaces; ++f) {
        Inter tmp;
        tmp.hit = 0;
        if (me->ntri[f] == 1) {
            tri_intersect(&me->tri[f][0], ray, position, eps, &tmp);
        } else {                                   /* Quad(zero, ...): position = zero + offset */
            P qpos = add(pt(0.0, 0.0, 0.0), position);
            for (int t = 0; t < 2 && !tmp.hit; ++t) {
                Inter tt;
                tri_intersect(&me->tri[f][t], ray, qpos, eps, &tt);
                if (tt.hit) tmp = tt;              /* first hit wins */
            }
        }
        if (tmp.hit) {
            double d = len(sub(tmp.point, p0));
            if (d < minDistance || minDistance < 0.0) {
                minDistance = d;
                *in = tmp;
                in->mat_id = me->mat_id;
            }
        }
    }
}

/* g_scene.intersection(ray, Point(0,0,0), inter): bounding sphere then closest child (:724-823). */
static void scene_intersect(const Scene* s, Line ray, Inter* in) {
    P off = pt(0.0, 0.0, 0.0);
    P u = line_dir(ray);
    P p0 = ray.s;
    P position = add(s->position, off);
    P deltaP = sub(position, p0);
    if (s->radius > 0) {
        double uDeltaP = dot(u, deltaP);
        double disc = uDeltaP * uDeltaP - dot(deltaP, deltaP) + s->radius * s->radius;
        double sv = uDeltaP - sqrt(disc);
        if (disc < 0 || fabs(sv) < s->eps) { in->hit = 0; return; }
    }
    in->hit = 0;
    double minDistance = -1.0;
    for (int c = 0; c < s->n_child; ++c) {
        Inter tmp;
        const Child ch = s->child[c];
        if (ch.type == 0) board_intersect(s, ray, position, &tmp);
        else if (ch.type == 1) sphere_intersect(&s->sph[ch.index], ray, position, s->eps, &tmp);
        else mesh_intersect(&s->mesh[ch.index], ray, position, s->eps, &tmp);
        if (tmp.hit) {
            double d = len(sub(tmp.point, p0));
            if (d < minDistance || minDistance < 0.0) {
                minDistance = d;
                *in = tmp;
            }
        }
    }
}

static inline double attenuation(double att, double d) { return att / (att + d * d); }  /* :1171-1182 */

typedef struct { uint32_t seg, shadow; } Count;

/* rayTraceRay (:1184-1249), recursive exactly as the reference. */
static void ray_trace_ray(const Scene* s, Line ray, P* color, unsigned depth, Count* cnt) {
    Inter in;
    cnt->seg++;
    scene_intersect(s, ray, &in);
    if (!in.hit) return;
    P ptv = in.point;
    Mat m = in.mat;
    for (int i = 0; i < s->n_lights; ++i) {
        Line sh; sh.s = ptv; sh.e = s->lpos[i];
        Inter si;
        cnt->shadow++;
        scene_intersect(s, sh, &si);
        if (!si.hit || !is_zero(si.mat.transp)) {
            P lC = scl(attenuation(s->att, line_len(sh)), s->lcol[i]);
            P term = add(add(had(m.amb, lC), scl(fabs(dot(in.normal, line_dir(sh))), had(m.diff, lC))),
                         scl(fabs(dot(line_dir(ray), line_dir(in.refl))), had(m.spec, lC)));
            *color = add(*color, term);
        }
    }
    if (depth > 0) {
        P tc = pt(0.0, 0.0, 0.0), rc = pt(0.0, 0.0, 0.0);
        P transparency = m.transp;
        P opacity = sub(pt(1.0, 1.0, 1.0), transparency);
        if (!is_zero(transparency) && len(transparency) > s->eps) {
            ray_trace_ray(s, in.trans, &tc, depth - 1, cnt);
            *color = add(*color, had(transparency, tc));
        }
        if (!is_zero(opacity)) {
            ray_trace_ray(s, in.refl, &rc, depth - 1, cnt);
            *color = add(*color, had(opacity, rc));
        }
    }
}

/* ---------------------------------------------------------------- exported oracle entry points */

/* rayTraceScreen basis (:1270-1279): right = normalize(LD x up); up' = normalize(right x LD). */
void oracle_camera_basis(const rt_camera* c, double right[3], double upp[3]) {
    P cam = from3(c->eye), look = from3(c->look_at), up = from3(c->up);
    P ld = sub(look, cam);
    P r = nrm(cross(ld, up));
    P u = nrm(cross(r, ld));
    right[0] = r.x; right[1] = r.y; right[2] = r.z;
    upp[0] = u.x; upp[1] = u.y; upp[2] = u.z;
}

/* Screen point of pixel (i, j) — SURVEY.md Appendix B, the parity contract's primary ray. */
static P screen_point(const rt_camera* c, P right, P upp, int i, int j) {
    P look = from3(c->look_at);
    return add(add(look, scl(c->pitch * (double)(i + c->bottom_x), right)),
               scl(c->pitch * (double)(j + c->bottom_y), upp));
}

/* Row banding (rt_api.h rt_rows): rows of one frame owned by the rank, frames stacked frame-major. */
static int frame_rows(int H, const rt_rows* r) {
    if (!r || r->n_ranks <= 1) return H;
    int hb = r->band_height, G = r->n_ranks, n = 0;
    for (int j = 0; j < H; ++j) if ((j / hb) % G == r->rank) ++n;
    return n;
}

static int local_rows(int H, const rt_rows* r) {
    return frame_rows(H, r) * ((r && r->frames > 1) ? r->frames : 1);
}

/* row within its frame of local row lr */
static int global_row(int H, const rt_rows* r, int lr) {
    lr %= frame_rows(H, r);
    if (!r || r->n_ranks <= 1) return lr;
    int hb = r->band_height, G = r->n_ranks;
    int band = lr / hb, within = lr % hb;
    return (band * G + r->rank) * hb + within;
}

int oracle_local_rows(int H, const rt_rows* r) { return local_rows(H, r); }

/* Render rows of a W x H frame: rgb (3 doubles / pixel, local row order), raycount packed as in
 * rt_render_dev.  nthreads <= 0 uses the OpenMP default. */
int oracle_render(const rt_scene* d, const rt_camera* c, int W, int H, int depth, const rt_rows* rows,
                  double* rgb, uint32_t* raycount, int nthreads) {
    if (!d || !c || W <= 0 || H <= 0 || depth < 0) return RT_EINVAL;
    Scene s;
    int rc = scene_build(d, &s);
    if (rc) { scene_free(&s); return rc; }
    double rv[3], uv[3];
    oracle_camera_basis(c, rv, uv);
    P right = from3(rv), upp = from3(uv), cam = from3(c->eye);
    int nl = local_rows(H, rows);
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 1)
#endif
    for (int lr = 0; lr < nl; ++lr) {
        int j = global_row(H, rows, lr);
        for (int i = 0; i < W; ++i) {
            Line ray; ray.s = cam; ray.e = screen_point(c, right, upp, i, j);
            P col = pt(0.0, 0.0, 0.0);
            Count cnt = {0, 0};
            ray_trace_ray(&s, ray, &col, (unsigned)depth, &cnt);
            size_t k = (size_t)lr * W + i;
            if (rgb) { rgb[3 * k] = col.x; rgb[3 * k + 1] = col.y; rgb[3 * k + 2] = col.z; }
            if (raycount) raycount[k] = cnt.seg | (cnt.shadow << 16);
        }
    }
    scene_free(&s);
    return RT_OK;
}

/* rayTraceRay on arbitrary rays. */
int oracle_trace_rays(const rt_scene* d, const double* starts, const double* ends, int n, int depth,
                      double* rgb, uint32_t* raycount, int nthreads) {
    if (!d || !starts || !ends || n < 0 || depth < 0) return RT_EINVAL;
    Scene s;
    int rc = scene_build(d, &s);
    if (rc) { scene_free(&s); return rc; }
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 256)
#endif
    for (int k = 0; k < n; ++k) {
        Line ray; ray.s = from3(starts + 3 * k); ray.e = from3(ends + 3 * k);
        P col = pt(0.0, 0.0, 0.0);
        Count cnt = {0, 0};
        ray_trace_ray(&s, ray, &col, (unsigned)depth, &cnt);
        if (rgb) { rgb[3 * k] = col.x; rgb[3 * k + 1] = col.y; rgb[3 * k + 2] = col.z; }
        if (raycount) raycount[k] = cnt.seg | (cnt.shadow << 16);
    }
    scene_free(&s);
    return RT_OK;
}

/* g_scene.intersection on arbitrary rays. */
int oracle_intersect(const rt_scene* d, const double* starts, const double* ends, int n, rt_hit* hits) {
    if (!d || !starts || !ends || !hits || n < 0) return RT_EINVAL;
    Scene s;
    int rc = scene_build(d, &s);
    if (rc) { scene_free(&s); return rc; }
    for (int k = 0; k < n; ++k) {
        Line ray; ray.s = from3(starts + 3 * k); ray.e = from3(ends + 3 * k);
        Inter in;
        scene_intersect(&s, ray, &in);
        rt_hit* h = &hits[k];
        memset(h, 0, sizeof(*h));
        h->hit = in.hit;
        h->material = in.hit ? in.mat_id : -1;
        if (in.hit) {
            h->point[0] = in.point.x; h->point[1] = in.point.y; h->point[2] = in.point.z;
            h->normal[0] = in.normal.x; h->normal[1] = in.normal.y; h->normal[2] = in.normal.z;
            h->reflected_end[0] = in.refl.e.x; h->reflected_end[1] = in.refl.e.y;
            h->reflected_end[2] = in.refl.e.z;
            h->transmitted_end[0] = in.trans.e.x; h->transmitted_end[1] = in.trans.e.y;
            h->transmitted_end[2] = in.trans.e.z;
        }
    }
    scene_free(&s);
    return RT_OK;
}

/* convertStringCoordinate (:1326-1346) for fixture building. */
void oracle_convert_string_coordinate(const char* sq, double out[3]) {
    const double edge = 320.0, sqe = 320.0 / 8;
    P first = pt(-edge / 2, 0.0, edge / 2);
    P row = pt(0.0, 0.0, -((double)(sq[0] - 'a') + .5) * sqe);
    P col = pt(((double)(sq[1] - '0' - 1) + .5) * sqe, 0.0, 0.0);
    P h = pt(0.0, 1.5 * sqe, 0.0);
    P r = add(add(add(first, row), col), h);
    out[0] = r.x; out[1] = r.y; out[2] = r.z;
}

/* FNV-1a 64 over raw bytes (golden-frame hashes). */
uint64_t oracle_fnv1a64(const void* data, size_t n) {
    const unsigned char* p = (const unsigned char*)data;
    uint64_t h = 1469598103934665603ULL;
    for (size_t i = 0; i < n; ++i) { h ^= p[i]; h *= 1099511628211ULL; }
    return h;
}

/* ---------------------------------------------- reference-faithful rayTraceScreen
 * rayTraceScreen (:1251-1324) as the app runs it: incremental screen walk (screenPt += right per pixel,
 * -= width*right, += up per row), every sample jittered by 0.5 * randomUnit() (:1148-1169), up to
 * SUPER_SAMPLE_NUMBER = 16 samples with the reference's convergence test (:1294-1311), and avgColor
 * carried from pixel to pixel (declared once, :1283).  Serial by construction: the sample count of a
 * pixel depends on its colours and on the carried average, and the rand() stream position of every
 * later sample depends on all earlier counts.
 * rand(): rng_kind 0 = glibc's rand() (TYPE_3 additive feedback generator, RAND_MAX = 2^31 - 1) — what
 * the reference compiled here uses; 1 = the MSVC CRT's LCG (RAND_MAX = 32767) — the reference's own
 * platform (Visual Studio project).  randomUnit's Point(rand, rand, rand) arguments are evaluated right
 * to left (z first) by both g++ and MSVC.  Outputs: rgb = the colour handed to glColor3d (:1312),
 * nsamples = samples traced per pixel, *rand_calls = rand() calls made. */
typedef struct { int kind; uint32_t lcg; int32_t r[34]; int i; } Rng;

static void rng_seed(Rng* g, int kind, uint32_t seed) {
    g->kind = kind;
    g->lcg = seed;
    if (kind == 0) {                                         /* glibc srandom_r, TYPE_3 */
        int32_t r[344];
        r[0] = (int32_t)(seed ? seed : 1);
        for (int i = 1; i < 31; ++i) {
            int64_t v = (16807LL * r[i - 1]) % 2147483647LL;
            r[i] = (int32_t)(v < 0 ? v + 2147483647LL : v);
        }
        for (int i = 31; i < 34; ++i) r[i] = r[i - 31];
        for (int i = 34; i < 344; ++i) r[i] = (int32_t)((uint32_t)r[i - 31] + (uint32_t)r[i - 3]);
        for (int i = 0; i < 34; ++i) g->r[i] = r[310 + i];
        g->i = 0;                                            /* g->r holds r[k .. k+33], oldest first */
    }
}

static int rng_next(Rng* g) {
    if (g->kind == 1) {
        g->lcg = g->lcg * 214013u + 2531011u;
        return (int)((g->lcg >> 16) & 0x7fff);
    }
    int32_t v = (int32_t)((uint32_t)g->r[(g->i + 3) % 34] + (uint32_t)g->r[(g->i + 31) % 34]);
    g->r[g->i] = v;                                          /* replaces r[k], the oldest */
    g->i = (g->i + 1) % 34;
    return (int)((uint32_t)v >> 1);
}

static double rng_max(const Rng* g) { return g->kind == 1 ? 32767.0 : 2147483647.0; }

/* randomUnit (:1148-1169) */
static P random_unit(Rng* g, uint64_t* calls) {
    P v = pt(0.0, 0.0, 0.0);
    const double den = rng_max(g) + 1.0;
    while (is_zero(v)) {
        double z = (double)rng_next(g) / den - .5;          /* arguments evaluated right to left */
        double y = (double)rng_next(g) / den - .5;
        double x = (double)rng_next(g) / den - .5;
        *calls += 3;
        v = pt(x, y, z);
    }
    return nrm(v);
}

int oracle_render_screen(const rt_scene* d, const double eye[3], const double look[3], const double up[3],
                         int bottom_x, int bottom_y, int W, int H, int depth, int rng_kind, uint32_t seed,
                         double* rgb, uint8_t* nsamples, uint64_t* rand_calls) {
    if (!d || !eye || !look || !up || W <= 0 || H <= 0 || depth < 0 || (rng_kind != 0 && rng_kind != 1))
        return RT_EINVAL;
    Scene s;
    int rc = scene_build(d, &s);
    if (rc) { scene_free(&s); return rc; }
    Rng g;
    rng_seed(&g, rng_kind, seed);
    uint64_t calls = 0;
    const double SSN = 16.0;                                 /* SUPER_SAMPLE_NUMBER (:52) */
    P camera = from3(eye), lookAt = from3(look), upv = from3(up);
    P lookDirection = sub(lookAt, camera);                   /* :1270 */
    P right = nrm(cross(lookDirection, upv));                /* :1271-1273 */
    P rightOffset = scl((double)W, right);                   /* :1274 */
    P upn = nrm(cross(right, lookDirection));                /* :1276-1277 */
    P screenPt = add(add(lookAt, scl((double)bottom_x, right)), scl((double)bottom_y, upn));   /* :1279 */
    P avgColor = pt(0.0, 0.0, 0.0);                          /* :1283, never reset */
    for (int j = 0; j < H; j++) {
        for (int i = 0; i < W; i++) {
            double k;
            int n = 0;
            for (k = 0.0; k < SSN; k++) {
                Line ray;
                ray.s = camera;
                ray.e = add(screenPt, scl(.5, random_unit(&g, &calls)));   /* :1296 */
                P color = pt(0.0, 0.0, 0.0);
                Count cnt = {0, 0};
                ray_trace_ray(&s, ray, &color, (unsigned)depth, &cnt);
                ++n;
                P oldWeightedColor = scl(k + 1.0, avgColor);
                avgColor = add(avgColor, color);
                P weightedColor = scl(k, avgColor);
                if (len(sub(weightedColor, oldWeightedColor)) < d->small_number * k * (k + 1)) break;
            }
            avgColor = pt(avgColor.x / k, avgColor.y / k, avgColor.z / k);   /* :1310 */
            size_t px = (size_t)j * W + i;
            if (rgb) { rgb[3 * px] = avgColor.x; rgb[3 * px + 1] = avgColor.y; rgb[3 * px + 2] = avgColor.z; }
            if (nsamples) nsamples[px] = (uint8_t)n;
            screenPt = add(screenPt, right);                 /* :1315 */
        }
        screenPt = sub(screenPt, rightOffset);               /* :1320 */
        screenPt = add(screenPt, upn);                       /* :1321 */
    }
    if (rand_calls) *rand_calls = calls;
    scene_free(&s);
    return RT_OK;
}

/* The rand() generators alone (tests check them against the C library and the published MSVC LCG). */
void oracle_rand_sequence(int rng_kind, uint32_t seed, int n, int32_t* out) {
    Rng g;
    rng_seed(&g, rng_kind, seed);
    for (int i = 0; i < n; ++i) out[i] = rng_next(&g);
}
