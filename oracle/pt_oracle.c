/*
 * pt_oracle.c -- scalar-f32 CPU restatement of the reference WGSL (TEST INFRASTRUCTURE).
 * See pt_oracle.h for scope.  Build: oracle/Makefile (gcc -O2 -ffp-contract=off).
 * Every function cites the WGSL it restates (SH/ = apps/frontend/src/graphics-core/shaders/).
 */
#include "pt_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------ constants
 * SH/PT_1_InitPass.wgsl:193-221 */
#define STRIDE_INSTANCE 33u
#define STRIDE_LIGHT 18u
#define STRIDE_DESCRIPTOR 6u
#define STRIDE_MATERIAL 15u
#define STRIDE_VERTEX 8u
#define STRIDE_BLAS 8u
#define RECONNECTION_DISTANCE 0.1f
#define RECONNECTION_ROUGHNESS 0.5f
#define INF_F 1e11f
#define EPS_F 1e-4f
#define PI_F 3.141592f
#define ENV_C 0.5f
#define LIGHT_DIRECTION 0u
#define LIGHT_POINT 1u
#define LIGHT_RECT 2u
#define LIGHT_ENV 3u
#define LOBE_LAMBERT 0u
#define LOBE_GGX 1u
#define LOBE_LIGHT 3u
#define STACK_MAX 96

/* uniform word indices (SH/PT_1_InitPass.wgsl:5-27) */
enum { U_W = 0, U_H = 1, U_VPINV = 4, U_FRAME = 23, U_OFF_DESC = 24, U_OFF_MAT = 25, U_OFF_LIGHT = 26,
       U_OFF_CDF = 27, U_OFF_INDEX = 28, U_OFF_SUBROOT = 29, U_OFF_BLAS = 30, U_INST_COUNT = 31,
       U_LIGHT_COUNT = 32 };

/* pass-specific epsilons (SURVEY.md §7 "Per-pass epsilon quirks") */
typedef struct pass_eps {
    float det_eps;   /* GetRayTriangleHitDistance |det| threshold */
    float bary_eps;  /* GetBaryCentricWeights |denom| threshold    */
    int final_pass;  /* PT_4 variants of PDF_LIGHT / L_emit (no EPS guard) */
} pass_eps;
static const pass_eps EPS_GBUFFER = {1e-8f, 1e-6f, 0};  /* SH/PT_01_GBufferPass.wgsl:409,468 */
static const pass_eps EPS_INIT = {1e-4f, 1e-8f, 0};     /* SH/PT_1_InitPass.wgsl:528,567 */
static const pass_eps EPS_FINAL = {1e-4f, 1e-8f, 1};    /* SH/PT_4_FinalShadingPass.wgsl:1249,1265 */
static const pass_eps EPS_MCPT = {1e-4f, 1e-8f, 0};     /* SH/TEST_MCPT.wgsl */

/* ------------------------------------------------------------------ f32 vector algebra */
typedef struct { float x, y, z; } v3;
static inline v3 V3(float x, float y, float z) { v3 r = {x, y, z}; return r; }
static inline v3 vadd(v3 a, v3 b) { return V3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 vsub(v3 a, v3 b) { return V3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 vmul(v3 a, v3 b) { return V3(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline v3 vscale(v3 a, float s) { return V3(a.x * s, a.y * s, a.z * s); }
static inline v3 vdivs(v3 a, float s) { return V3(a.x / s, a.y / s, a.z / s); }
static inline v3 vneg(v3 a) { return V3(-a.x, -a.y, -a.z); }
static inline float vdot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static inline v3 vcross(v3 a, v3 b) {
    return V3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
static inline float vlength(v3 a) { return sqrtf(vdot(a, a)); }
static inline v3 vnormalize(v3 a) { return vdivs(a, vlength(a)); }
static inline float fmin_(float a, float b) { return fminf(a, b); }
static inline float fmax_(float a, float b) { return fmaxf(a, b); }
static inline float saturate_(float a) { return fminf(fmaxf(a, 0.0f), 1.0f); }
static inline float mixf(float a, float b, float t) { return a * (1.0f - t) + b * t; }
static inline v3 vmix(v3 a, v3 b, float t) { return V3(mixf(a.x, b.x, t), mixf(a.y, b.y, t), mixf(a.z, b.z, t)); }
static inline float luminance(v3 c) { return c.x * 0.2126f + c.y * 0.7152f + c.z * 0.0722f; }
static inline float f32_of(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static inline uint32_t u32_of(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

/* mat4 (column-major, m[4*col+row]) * vec4, SH/PT_1_InitPass.wgsl:480-484 */
static inline v3 xform_point(const float *m, v3 p) {
    float x = ((m[0] * p.x + m[4] * p.y) + m[8] * p.z) + m[12] * 1.0f;
    float y = ((m[1] * p.x + m[5] * p.y) + m[9] * p.z) + m[13] * 1.0f;
    float z = ((m[2] * p.x + m[6] * p.y) + m[10] * p.z) + m[14] * 1.0f;
    float w = ((m[3] * p.x + m[7] * p.y) + m[11] * p.z) + m[15] * 1.0f;
    return V3(x / w, y / w, z / w);
}
/* transpose(m) * vec4(p,1), then /w (normal transform, SH/PT_1_InitPass.wgsl:395) */
static inline v3 xform_point_transposed(const float *m, v3 p) {
    float x = ((m[0] * p.x + m[1] * p.y) + m[2] * p.z) + m[3] * 1.0f;
    float y = ((m[4] * p.x + m[5] * p.y) + m[6] * p.z) + m[7] * 1.0f;
    float z = ((m[8] * p.x + m[9] * p.y) + m[10] * p.z) + m[11] * 1.0f;
    float w = ((m[12] * p.x + m[13] * p.y) + m[14] * p.z) + m[15] * 1.0f;
    return V3(x / w, y / w, z / w);
}

/* ------------------------------------------------------------------ RNG (PT_1:810-826) */
uint32_t pto_pcg(uint32_t seed) {
    uint32_t state = seed * 747796405u + 2891336453u;
    uint32_t word = ((state >> ((state >> 28u) + 4u)) ^ state) * 277803737u;
    return (word >> 22u) ^ word;
}
float pto_random(uint32_t *seed) {
    uint32_t h = pto_pcg(*seed);
    *seed += 1u;
    return (float)h / 4294967295.0f; /* literal rounds to 2^32 in f32 */
}

/* ------------------------------------------------------------------ scene access */
typedef struct ctx {
    const uint32_t *U, *S, *G, *A;
    pass_eps eps;
    pto_counters *cnt;
} ctx;

typedef struct material {
    v3 albedo;
    float alpha;
    float metalness, roughness, transmission, ior;
} material;

typedef struct surface {
    v3 pos, nrm;
    material mat;
} surface;

typedef struct compact {
    uint32_t valid, inst, mat, prim;
    float bu, bv;
} compact;

typedef struct hit {
    int valid;
    float t;
    compact s;
} hit;

typedef struct ray { v3 o, d; } ray;

typedef struct desc { uint32_t off_vertex, off_index, off_material, off_subroot, off_blas, count_sub; } desc;

static inline const float *inst_model(const ctx *c, uint32_t i) { return (const float *)(c->S + STRIDE_INSTANCE * i); }
static inline const float *inst_inv(const ctx *c, uint32_t i) { return (const float *)(c->S + STRIDE_INSTANCE * i + 16u); }
static inline uint32_t inst_mesh(const ctx *c, uint32_t i) { return c->S[STRIDE_INSTANCE * i + 32u]; }

static inline desc get_desc(const ctx *c, uint32_t mesh) {
    const uint32_t *p = c->S + c->U[U_OFF_DESC] + STRIDE_DESCRIPTOR * mesh;
    desc d = {p[0], p[1], p[2], p[3], p[4], p[5]};
    return d;
}

/* GetMaterial, SH/PT_1_InitPass.wgsl:285-314 (transmissive -> yellow, roughness >= 0.01) */
static material get_material(const ctx *c, const desc *d, uint32_t mid) {
    const uint32_t *p = c->S + c->U[U_OFF_MAT] + d->off_material + STRIDE_MATERIAL * mid;
    material m;
    m.albedo = V3(f32_of(p[0]), f32_of(p[1]), f32_of(p[2]));
    m.alpha = f32_of(p[3]);
    m.metalness = f32_of(p[8]);
    m.roughness = f32_of(p[9]);
    m.transmission = f32_of(p[10]);
    m.ior = f32_of(p[11]);
    if (m.transmission > 0.0f) m.albedo = V3(1.0f, 1.0f, 0.0f);
    m.roughness = fmax_(m.roughness, 0.01f);
    return m;
}

static inline v3 vertex_pos(const ctx *c, const desc *d, uint32_t vid) {
    const uint32_t *p = c->G + d->off_vertex + STRIDE_VERTEX * vid;
    return V3(f32_of(p[0]), f32_of(p[1]), f32_of(p[2]));
}
static inline v3 vertex_nrm(const ctx *c, const desc *d, uint32_t vid) {
    const uint32_t *p = c->G + d->off_vertex + STRIDE_VERTEX * vid;
    return V3(f32_of(p[3]), f32_of(p[4]), f32_of(p[5]));
}
static inline void tri_ids(const ctx *c, const desc *d, uint32_t prim, uint32_t id[3]) {
    const uint32_t *p = c->G + c->U[U_OFF_INDEX] + d->off_index + 3u * prim;
    id[0] = p[0]; id[1] = p[1]; id[2] = p[2];
}

/* GetBlasNode, SH/PT_01_GBufferPass.wgsl:310-322 */
static inline const uint32_t *blas_node(const ctx *c, const desc *d, uint32_t sub, uint32_t node) {
    uint32_t root = c->G[c->U[U_OFF_SUBROOT] + d->off_subroot + sub];
    return c->A + c->U[U_OFF_BLAS] + d->off_blas + root + STRIDE_BLAS * node;
}

/* GetSurface, SH/PT_1_InitPass.wgsl:438-467 (and GetTriangleWorldSpace :390-407) */
static surface get_surface(const ctx *c, compact x) {
    surface s;
    uint32_t mesh = inst_mesh(c, x.inst);
    desc d = get_desc(c, mesh);
    const float *M = inst_model(c, x.inst);
    const float *Mi = inst_inv(c, x.inst);
    uint32_t id[3];
    s.mat = get_material(c, &d, x.mat);
    tri_ids(c, &d, x.prim, id);
    v3 p0 = xform_point(M, vertex_pos(c, &d, id[0]));
    v3 n0 = xform_point_transposed(Mi, vertex_nrm(c, &d, id[0]));
    v3 p1 = xform_point(M, vertex_pos(c, &d, id[1]));
    v3 n1 = xform_point_transposed(Mi, vertex_nrm(c, &d, id[1]));
    v3 p2 = xform_point(M, vertex_pos(c, &d, id[2]));
    v3 n2 = xform_point_transposed(Mi, vertex_nrm(c, &d, id[2]));
    float U = x.bu, V = x.bv, W = 1.0f - U - V;
    s.nrm = vnormalize(vadd(vadd(vscale(n0, U), vscale(n1, V)), vscale(n2, W)));
    s.pos = vadd(vadd(vscale(p0, U), vscale(p1, V)), vscale(p2, W));
    return s;
}

/* ------------------------------------------------------------------ geometry tests */
/* TransformRayWithMat4x4, SH/PT_1_InitPass.wgsl:486-496 */
static ray transform_ray(const float *m, ray r, int normalize_dir) {
    v3 start = xform_point(m, r.o);
    v3 end = xform_point(m, vadd(r.o, r.d));
    v3 dir = vsub(end, start);
    ray out = {start, normalize_dir ? vnormalize(dir) : dir};
    return out;
}

/* GetRayAABBIntersectionRange, SH/PT_1_InitPass.wgsl:498-514; returns 1 and range on hit */
static inline void aabb_range(ray r, const uint32_t *node, float *tmin_out, float *tmax_out) {
    v3 inv = V3(1.0f / r.d.x, 1.0f / r.d.y, 1.0f / r.d.z);
    v3 bmin = V3(f32_of(node[0]), f32_of(node[1]), f32_of(node[2]));
    v3 bmax = V3(f32_of(node[3]), f32_of(node[4]), f32_of(node[5]));
    v3 t1 = vmul(vsub(bmin, r.o), inv);
    v3 t2 = vmul(vsub(bmax, r.o), inv);
    v3 tn = V3(fmin_(t1.x, t2.x), fmin_(t1.y, t2.y), fmin_(t1.z, t2.z));
    v3 tf = V3(fmax_(t1.x, t2.x), fmax_(t1.y, t2.y), fmax_(t1.z, t2.z));
    float t_min = fmax_(tn.x, fmax_(tn.y, tn.z));
    float t_max = fmin_(tf.x, fmin_(tf.y, tf.z));
    if (t_min > t_max) { *tmin_out = 1.0f; *tmax_out = 0.0f; return; }
    *tmin_out = t_min;
    *tmax_out = t_max;
}
/* DoRangesOverlap, SH/PT_1_InitPass.wgsl:475-478 */
static inline int ranges_overlap(float r1x, float r1y, float r2x, float r2y) { return (r1x <= r2y) && (r2x <= r1y); }

/* GetRayTriangleHitDistance, SH/PT_1_InitPass.wgsl:516-547 (det EPS per pass) */
static float ray_triangle(ray r, v3 P0, v3 P1, v3 P2, float det_eps) {
    v3 e1 = vsub(P1, P0);
    v3 e2 = vsub(P2, P0);
    v3 pvec = vcross(r.d, e2);
    float det = vdot(e1, pvec);
    if (fabsf(det) < det_eps) return 1e11f;
    float inv_det = 1.0f / det;
    v3 tvec = vsub(r.o, P0);
    float u = vdot(tvec, pvec) * inv_det;
    if (u < 0.0f || u > 1.0f) return 1e11f;
    v3 qvec = vcross(tvec, e1);
    float v = vdot(r.d, qvec) * inv_det;
    if (v < 0.0f || (u + v) > 1.0f) return 1e11f;
    float t = vdot(e2, qvec) * inv_det;
    if (t <= 1e-4f) return 1e11f;
    return t;
}

/* GetBaryCentricWeights, SH/PT_1_InitPass.wgsl:549-575 -> (w,u,v) */
static void barycentric(v3 P, v3 A, v3 B, v3 C, float eps, float out[3]) {
    v3 v0 = vsub(B, A), v1 = vsub(C, A), v2 = vsub(P, A);
    float d00 = vdot(v0, v0), d01 = vdot(v0, v1), d11 = vdot(v1, v1);
    float d20 = vdot(v2, v0), d21 = vdot(v2, v1);
    float denom = d00 * d11 - d01 * d01;
    if (fabsf(denom) < eps) { out[0] = 1.0f; out[1] = 0.0f; out[2] = 0.0f; return; }
    float inv = 1.0f / denom;
    float u = (d11 * d20 - d01 * d21) * inv;
    float v = (d00 * d21 - d01 * d20) * inv;
    out[0] = 1.0f - u - v;
    out[1] = u;
    out[2] = v;
}

/* TraceRay, SH/PT_1_InitPass.wgsl:605-715 (PT_01:509-621 identical up to epsilons) */
static hit trace_ray(const ctx *c, ray in) {
    hit best;
    memset(&best, 0, sizeof best);
    float vx = 1e-4f, vy = 1e10f; /* RayValidRange */
    uint32_t stack[STACK_MAX];
    const uint32_t ninst = c->U[U_INST_COUNT];
    if (c->cnt) c->cnt->rays++;
    for (uint32_t inst = 0; inst < ninst; ++inst) {
        const uint32_t mesh = inst_mesh(c, inst);
        desc d = get_desc(c, mesh);
        ray local = transform_ray(inst_inv(c, inst), in, 0);
        if (c->cnt) c->cnt->instance_xforms++;
        for (uint32_t sub = 0; sub < d.count_sub; ++sub) {
            float rx, ry;
            aabb_range(local, blas_node(c, &d, sub, 0), &rx, &ry);
            if (c->cnt) c->cnt->aabb_tests++;
            if (!ranges_overlap(vx, vy, rx, ry)) continue;
            int sp = -1;
            stack[++sp] = 0;
            while (sp > -1) {
                uint32_t id = stack[sp--];
                const uint32_t *node = blas_node(c, &d, sub, id);
                int leaf = (node[7] & 0xffff0000u) != 0u;
                if (!leaf) {
                    uint32_t lid = id + 1u, rid = node[6] / 8u;
                    float lx, ly, rrx, rry;
                    aabb_range(local, blas_node(c, &d, sub, lid), &lx, &ly);
                    aabb_range(local, blas_node(c, &d, sub, rid), &rrx, &rry);
                    if (c->cnt) c->cnt->aabb_tests += 2;
                    int lh = ranges_overlap(vx, vy, lx, ly);
                    int rh = ranges_overlap(vx, vy, rrx, rry);
                    if (lh && rh) {
                        if (lx < rrx) { stack[++sp] = rid; stack[++sp] = lid; }
                        else { stack[++sp] = lid; stack[++sp] = rid; }
                    } else if (lh) {
                        stack[++sp] = lid;
                    } else if (rh) {
                        stack[++sp] = rid;
                    }
                    if (sp >= STACK_MAX - 2) abort(); /* reference stack is 96/64 entries */
                    continue;
                }
                uint32_t first = node[6], last = first + (node[7] & 0xffffu);
                for (uint32_t prim = first; prim < last; ++prim) {
                    uint32_t ids[3];
                    tri_ids(c, &d, prim, ids);
                    float t = ray_triangle(local, vertex_pos(c, &d, ids[0]), vertex_pos(c, &d, ids[1]),
                                           vertex_pos(c, &d, ids[2]), c->eps.det_eps);
                    if (c->cnt) c->cnt->tri_tests++;
                    if (vy < t) continue;
                    vy = t;
                    best.valid = 1;
                    best.s.valid = 1;
                    best.s.inst = inst;
                    best.s.mat = sub;
                    best.s.prim = prim;
                }
            }
        }
    }
    if (best.valid) {
        best.t = vy;
        const uint32_t mesh = inst_mesh(c, best.s.inst);
        desc d = get_desc(c, mesh);
        const float *M = inst_model(c, best.s.inst);
        uint32_t ids[3];
        tri_ids(c, &d, best.s.prim, ids);
        v3 A = xform_point(M, vertex_pos(c, &d, ids[0]));
        v3 B = xform_point(M, vertex_pos(c, &d, ids[1]));
        v3 C = xform_point(M, vertex_pos(c, &d, ids[2]));
        v3 P = vadd(in.o, vscale(in.d, best.t));
        float w[3];
        barycentric(P, A, B, C, c->eps.bary_eps, w);
        best.s.bu = w[0];
        best.s.bv = w[1];
        if (c->cnt) c->cnt->hits++;
    }
    return best;
}

/* ------------------------------------------------------------------ lights */
typedef struct light {
    v3 pos, dir, color, U, V;
    uint32_t type;
    float intensity, area;
} light;

typedef struct light_sample {
    v3 dir;
    uint32_t type;
    v3 pos;
    int32_t id;
    v3 Le;
    float pdf;
} light_sample;

static light get_light(const ctx *c, uint32_t id) {
    const uint32_t *p = c->S + c->U[U_OFF_LIGHT] + STRIDE_LIGHT * id;
    light l;
    l.pos = V3(f32_of(p[0]), f32_of(p[1]), f32_of(p[2]));
    l.dir = V3(f32_of(p[3]), f32_of(p[4]), f32_of(p[5]));
    l.color = V3(f32_of(p[6]), f32_of(p[7]), f32_of(p[8]));
    l.U = V3(f32_of(p[9]), f32_of(p[10]), f32_of(p[11]));
    l.V = V3(f32_of(p[12]), f32_of(p[13]), f32_of(p[14]));
    l.type = p[15];
    l.intensity = f32_of(p[16]);
    l.area = f32_of(p[17]);
    return l;
}
static inline float light_cdf(const ctx *c, uint32_t i) { return f32_of(c->S[c->U[U_OFF_CDF] + i]); }

/* ------------------------------------------------------------------ BSDF (PT_1:834-929) */
static float ggx_d(float NdotH, float R) {
    float a = R * R, a2 = a * a;
    float X = NdotH * NdotH * (a2 - 1.0f) + 1.0f;
    float denom = PI_F * X * X;
    return a2 / fmax_(denom, EPS_F);
}
static float geom_shadow(float NdotV, float NdotL, float R) {
    float r = R + 1.0f;
    float K = r * r / 8.0f;
    return 1.0f / ((NdotV * (1.0f - K) + K) * (NdotL * (1.0f - K) + K));
}
/* WGSL pow / sin / cos are implementation-defined (pow is exp2(y*log2(x)) on most
 * WebGPU backends; sin/cos carry an absolute error bound of 2^-11).  Both sides of the
 * parity check use the same fixed f32 definitions below instead of libm, so the oracle
 * and the HIP path agree bit for bit (each is within ~2 ulp of the true function).
 * pow(x, 5): two squarings and a product.
 *
 * PTO_TRANSC selects other admissible WGSL implementations, for the sensitivity study of
 * DESIGN.md §2 only (tests/test_transcendental_sensitivity.py; never the parity oracle):
 *   0  the fixed definitions below (default; what the HIP kernels compute)
 *   1  libm powf / sinf / cosf (correctly rounded or within 1 ulp)
 *   2  a WGSL-admissible backend at its error bounds: pow as exp2(5 * log2 x) (the common
 *      lowering) and sin / cos each off by 2^-11 absolute, the sign hashed from the input
 *   3  mode 2's pow with libm sin / cos;  4  mode 2's sin / cos with libm pow */
#ifndef PTO_TRANSC
#define PTO_TRANSC 0
#endif
#if PTO_TRANSC == 0
static inline float pow5_(float x) {
    float x2 = x * x;
    return (x2 * x2) * x;
}
#elif PTO_TRANSC == 1 || PTO_TRANSC == 4
static inline float pow5_(float x) { return powf(x, 5.0f); }
#else
static inline float pow5_(float x) { return exp2f(5.0f * log2f(x)); }
#endif
/* sin and cos of x >= 0 (the only use: BSDF sampling angles 2*PI_F*u, u in [0,1]).
 * Cody-Waite reduction by pi/4 in three parts (the first exact for the octant counts
 * used), then the classic single-precision minimax polynomials on [-pi/4, pi/4]. */
#if PTO_TRANSC == 1 || PTO_TRANSC == 3
static void sincos_(float x, float *s, float *c) {
    *s = sinf(x);
    *c = cosf(x);
}
#elif PTO_TRANSC == 2 || PTO_TRANSC == 4
static float sincos_err = 0x1p-11f;  /* WGSL's bound; pto_set_sincos_error() scans smaller ones */
void pto_set_sincos_error(float e) { sincos_err = e; }
static void sincos_(float x, float *s, float *c) {
    uint32_t b;
    memcpy(&b, &x, 4);
    const uint32_t h = pto_pcg(b ^ 0x5EEDu);
    *s = sinf(x) + ((h & 1u) ? sincos_err : -sincos_err);
    *c = cosf(x) + ((h & 2u) ? sincos_err : -sincos_err);
}
#else
static void sincos_(float x, float *s, float *c) {
    int j = (int)(x * 1.27323954473516f);
    float y = (float)j;
    if (j & 1) {
        j += 1;
        y += 1.0f;
    }
    j &= 7;
    float z = ((x - y * 0.78515625f) - y * 2.4187564849853515625e-4f) - y * 3.77489497744594108e-8f;
    float zz = z * z;
    float ps = ((-1.9515295891e-4f * zz + 8.3321608736e-3f) * zz - 1.6666654611e-1f) * zz * z + z;
    float pc = ((2.443315711809948e-5f * zz - 1.388731625493765e-3f) * zz + 4.166664568298827e-2f) * zz * zz -
               0.5f * zz + 1.0f;
    if (j == 0) { *s = ps; *c = pc; }
    else if (j == 2) { *s = pc; *c = -ps; }
    else if (j == 4) { *s = -ps; *c = -pc; }
    else { *s = -pc; *c = ps; }
}
#endif
float pto_sin(float x) { float s, c; sincos_(x, &s, &c); return s; }
float pto_cos(float x) { float s, c; sincos_(x, &s, &c); return c; }
float pto_pow5(float x) { return pow5_(x); }

static v3 fresnel(float d, v3 F0) {
    float p = pow5_(1.0f - saturate_(d));
    return V3(F0.x + (1.0f - F0.x) * p, F0.y + (1.0f - F0.y) * p, F0.z + (1.0f - F0.z) * p);
}
static v3 brdf(const surface *X, v3 V, v3 L) {
    v3 N = X->nrm;
    v3 H = vnormalize(vadd(L, V));
    float NdotV = fmax_(vdot(N, V), 0.0f), NdotL = fmax_(vdot(N, L), 0.0f);
    float NdotH = fmax_(vdot(N, H), 0.0f), VdotH = fmax_(vdot(V, H), 0.0f);
    v3 base = X->mat.albedo;
    float metal = X->mat.metalness, R = X->mat.roughness;
    v3 F0 = vmix(V3(0.04f, 0.04f, 0.04f), base, metal);
    float D = ggx_d(NdotH, R);
    float G0 = geom_shadow(NdotV, NdotL, R);
    v3 F = fresnel(VdotH, F0);
    v3 kD = vscale(V3(1.0f - F.x, 1.0f - F.y, 1.0f - F.z), 1.0f - metal);
    v3 diffuse = vmul(vdivs(kD, PI_F), base);
    v3 spec = vscale(vscale(vscale(F, D), G0), 0.25f);
    return vadd(diffuse, spec);
}
static v3 btdf(const surface *X, v3 V, v3 L) {
    v3 albedo = X->mat.albedo;
    float R = X->mat.roughness;
    int same = vdot(V, X->nrm) > 0.0f;
    float n_in = same ? X->mat.ior : 1.0f;
    float n_out = same ? 1.0f : X->mat.ior;
    v3 hv = vadd(vscale(L, n_in), vscale(V, n_out));
    float H_norm = vlength(hv);
    v3 N = same ? X->nrm : vneg(X->nrm);
    v3 H = vnormalize(hv);
    float NdotL = fabsf(vdot(N, L)), NdotV = fabsf(vdot(N, V)), NdotH = fabsf(vdot(N, H));
    float LdotH = fabsf(vdot(L, H)), VdotH = fabsf(vdot(V, H));
    float G0 = geom_shadow(NdotL, NdotV, R);
    float D = ggx_d(NdotH, R);
    float nr = (n_out - n_in) / (n_out + n_in);
    v3 F = fresnel(LdotH, V3(nr * nr, nr * nr, nr * nr));
    float s = n_out * n_out;
    v3 num = vscale(V3(1.0f - F.x, 1.0f - F.y, 1.0f - F.z), s);
    num = vscale(num, LdotH);
    num = vscale(num, VdotH);
    num = vscale(num, G0);
    num = vscale(num, D);
    num = vmul(num, albedo);
    return vdivs(num, fmax_(H_norm * H_norm, EPS_F));
}
static v3 bsdf(const surface *X, v3 V, v3 L) {
    float T = X->mat.transmission;
    v3 N = X->nrm;
    if (vdot(L, N) * vdot(V, N) > 0.0f) return vscale(brdf(X, V, L), 1.0f - T);
    return vscale(btdf(X, V, L), T);
}

/* ------------------------------------------------------------------ sampling (PT_1:577-589,937-1106) */
typedef struct mat3 { v3 T, B, N; } mat3;
static mat3 tbn(v3 N) {
    int same = fabsf(vdot(N, V3(0.0f, 1.0f, 0.0f))) > 0.9999f;
    v3 cv = same ? V3(1.0f, 0.0f, 0.0f) : V3(0.0f, 1.0f, 0.0f);
    mat3 m;
    m.T = vnormalize(vcross(cv, N));
    m.B = vcross(N, m.T);
    m.N = N;
    return m;
}
static inline v3 mat3_mul(mat3 m, v3 v) { return vadd(vadd(vscale(m.T, v.x), vscale(m.B, v.y)), vscale(m.N, v.z)); }
static inline v3 reflect_(v3 I, v3 N) { return vsub(I, vscale(N, 2.0f * vdot(N, I))); }
static inline v3 refract_(v3 I, v3 N, float eta) {
    float d = vdot(N, I);
    float k = 1.0f - eta * eta * (1.0f - d * d);
    if (k < 0.0f) return V3(0.0f, 0.0f, 0.0f);
    return vsub(vscale(I, eta), vscale(N, eta * d + sqrtf(k)));
}
static v3 sample_cosine(uint32_t *seed) {
    float r1 = pto_random(seed), r2 = pto_random(seed);
    float R = sqrtf(r1);
    float phi = 2.0f * PI_F * r2, sp, cp;
    sincos_(phi, &sp, &cp);
    return V3(R * cp, R * sp, sqrtf(1.0f - r1));
}
static v3 sample_ggx(uint32_t *seed, float R) {
    float r1 = pto_random(seed), r2 = pto_random(seed);
    float a = R * R;
    float phi = 2.0f * PI_F * r1;
    float ct = sqrtf((1.0f - r2) / (1.0f + (a * a - 1.0f) * r2));
    float st = sqrtf(1.0f - ct * ct), sp, cp;
    sincos_(phi, &sp, &cp);
    return vnormalize(V3(st * cp, st * sp, ct));
}
static v3 sample_brdf(uint32_t *seed, const surface *X, v3 V, uint32_t *lobe) {
    float metal = X->mat.metalness;
    v3 F0 = vmix(V3(0.04f, 0.04f, 0.04f), X->mat.albedo, metal);
    float p_spec = mixf(luminance(F0), 1.0f, metal);
    mat3 m = tbn(X->nrm);
    int spec = pto_random(seed) < p_spec;
    v3 L;
    if (spec) {
        v3 H = mat3_mul(m, sample_ggx(seed, X->mat.roughness));
        L = reflect_(vneg(V), H);
    } else {
        L = mat3_mul(m, sample_cosine(seed));
    }
    *lobe = spec ? LOBE_GGX : LOBE_LAMBERT;
    return L;
}
static v3 sample_btdf(uint32_t *seed, const surface *X, v3 V, uint32_t *lobe) {
    int same = vdot(V, X->nrm) > 0.0f;
    float n_in = same ? 1.0f : X->mat.ior;
    float n_out = same ? X->mat.ior : 1.0f;
    v3 N = same ? X->nrm : vneg(X->nrm);
    float ratio = n_in / n_out;
    float r = (1.0f - ratio) / (1.0f + ratio);
    float R2 = ratio * ratio;
    float cos_t = fabsf(vdot(V, N));
    float p_refl = fresnel(cos_t, V3(r * r, r * r, r * r)).x;
    if (cos_t * cos_t < (R2 - 1.0f) / R2) p_refl = 1.0f;
    int refl = pto_random(seed) < p_refl;
    mat3 m = tbn(N);
    v3 H = mat3_mul(m, sample_ggx(seed, X->mat.roughness));
    v3 Lr = refract_(vneg(V), H, ratio);
    v3 Ll = reflect_(vneg(V), H);
    *lobe = LOBE_GGX;
    return vnormalize(refl ? Ll : Lr);
}
static v3 sample_bsdf(uint32_t *seed, const surface *X, v3 V, uint32_t *lobe) {
    int transparent = pto_random(seed) < X->mat.transmission;
    if (transparent) return sample_btdf(seed, X, V, lobe);
    return sample_brdf(seed, X, V, lobe);
}

/* ------------------------------------------------------------------ pdfs (PT_1:1114-1245) */
static float pdf_brdf(const surface *X, v3 V, v3 L) {
    float metal = X->mat.metalness, R = X->mat.roughness;
    v3 F0 = vmix(V3(0.04f, 0.04f, 0.04f), X->mat.albedo, metal);
    float p_spec = mixf(luminance(F0), 1.0f, metal);
    v3 N = X->nrm;
    v3 H = vnormalize(vadd(L, V));
    float LdotN = fmax_(vdot(L, N), 0.0f);
    float NdotH = fmax_(vdot(N, H), 0.0f);
    float VdotH = fmax_(vdot(V, H), 0.0f);
    float pdf_s = ggx_d(NdotH, R) / fmax_(4.0f * VdotH, EPS_F);
    float pdf_d = LdotN / PI_F;
    return mixf(pdf_d, pdf_s, p_spec);
}
static float pdf_btdf(const surface *X, v3 V, v3 L) {
    float R = X->mat.roughness;
    int same = vdot(V, X->nrm) > 0.0f;
    float n_in = same ? 1.0f : X->mat.ior;
    float n_out = same ? X->mat.ior : 1.0f;
    float ratio = n_in / n_out;
    v3 N = same ? X->nrm : vneg(X->nrm);
    float r0 = (1.0f - ratio) / (1.0f + ratio);
    float R0 = r0 * r0;
    float cos_t = fabsf(vdot(V, N));
    float p_refl = fresnel(cos_t, V3(R0, R0, R0)).x;
    float sin2 = 1.0f - cos_t * cos_t;
    float R2 = ratio * ratio;
    if (sin2 * R2 > 1.0f) p_refl = 1.0f;
    float p_trans = 1.0f - p_refl;
    float pdf_r = 0.0f;
    if (p_refl > 0.0f) {
        v3 Hr = vnormalize(vadd(V, L));
        float NdotHr = fmax_(0.0f, vdot(N, Hr));
        float VdotHr = fmax_(0.0f, vdot(V, Hr));
        if (VdotHr > 0.0f) pdf_r = ggx_d(NdotHr, R) / (4.0f * VdotHr);
    }
    float pdf_t = 0.0f;
    if (p_trans > 0.0f) {
        v3 Ht = vnormalize(vadd(vscale(V, n_out), vscale(L, n_in)));
        float NdotHt = fmax_(0.0f, vdot(N, Ht));
        float VdotHt = fmax_(0.0f, vdot(V, Ht));
        float LdotHt = fmax_(0.0f, vdot(L, Ht));
        float denom = n_in * LdotHt + n_out * VdotHt;
        if (denom > 0.0f) {
            float J = (n_out * n_out * VdotHt) / (denom * denom);
            pdf_t = ggx_d(NdotHt, R) * fabsf(J);
        }
    }
    return p_refl * pdf_r + p_trans * pdf_t;
}
static float pdf_bsdf(const surface *X, v3 V, v3 L) {
    v3 N = X->nrm;
    if (vdot(L, N) * vdot(V, N) > 0.0f) return pdf_brdf(X, V, L);
    return pdf_btdf(X, V, L);
}

/* DirectionToLight, SH/PT_1_InitPass.wgsl:746-772 */
static v3 direction_to_light(const surface *X, const light_sample *XL) {
    switch (XL->type) {
    case LIGHT_DIRECTION: return vneg(XL->dir);
    case LIGHT_POINT:
    case LIGHT_RECT: return vnormalize(vsub(XL->pos, X->pos));
    case LIGHT_ENV: return vneg(XL->dir);
    default: return V3(0.0f, 0.0f, 0.0f);
    }
}

/* PDF_LIGHT, SH/PT_1_InitPass.wgsl:1220-1245 (PT_4:1249 drops the EPS guard) */
static float pdf_light(const ctx *c, const surface *X, v3 V, const light_sample *XL) {
    if (XL->type == LIGHT_ENV) {
        v3 L = direction_to_light(X, XL);
        return pdf_bsdf(X, V, L);
    }
    light ls = get_light(c, (uint32_t)XL->id);
    float before = (XL->id == 0) ? 0.0f : light_cdf(c, (uint32_t)XL->id - 1u);
    float choose = light_cdf(c, (uint32_t)XL->id) - before;
    float pdf_point = 1.0f;
    if (XL->type == LIGHT_RECT) {
        v3 r = vsub(XL->pos, X->pos);
        v3 L = vnormalize(r);
        float denom = ls.area * fabsf(vdot(ls.dir, L));
        pdf_point = vdot(r, r) / (c->eps.final_pass ? denom : fmax_(denom, EPS_F));
    }
    return choose * pdf_point;
}

/* SampleNEE, SH/PT_1_InitPass.wgsl:970-1025 */
static light_sample sample_nee(const ctx *c, uint32_t *seed, const surface *X, v3 V) {
    light_sample s;
    memset(&s, 0, sizeof s);
    float P = pto_random(seed);
    uint32_t L = 0, R = c->U[U_LIGHT_COUNT] - 1u, M = (L + R) >> 1;
    while (L < R) {
        if (P < light_cdf(c, M)) R = M;
        else L = M + 1u;
        M = (L + R) >> 1;
    }
    s.id = (int32_t)M;
    light ls = get_light(c, M);
    s.type = ls.type;
    s.Le = vscale(ls.color, ls.intensity);
    switch (ls.type) {
    case LIGHT_DIRECTION:
        s.pos = vsub(X->pos, vscale(ls.dir, INF_F));
        s.dir = ls.dir;
        break;
    case LIGHT_POINT:
        s.pos = ls.pos;
        s.dir = vnormalize(vsub(X->pos, ls.pos));
        break;
    case LIGHT_RECT: {
        float ru = pto_random(seed) * 2.0f - 1.0f;
        float rv = pto_random(seed) * 2.0f - 1.0f;
        v3 off = vadd(vscale(ls.U, ru), vscale(ls.V, rv));
        s.pos = vadd(ls.pos, off);
        s.dir = vnormalize(vsub(X->pos, s.pos));
        break;
    }
    default: break;
    }
    s.pdf = pdf_light(c, X, V, &s);
    return s;
}

/* L_emit, SH/PT_1_InitPass.wgsl:1253-1260 (PT_4:1265: no EPS guard) */
static v3 l_emit(const ctx *c, const light_sample *XL, const surface *X) {
    v3 r = vsub(XL->pos, X->pos);
    float rr = vdot(r, r);
    float att = (XL->type == LIGHT_POINT) ? 1.0f / (c->eps.final_pass ? rr : fmax_(rr, EPS_F)) : 1.0f;
    return vscale(XL->Le, att);
}

/* GetMaterialFromHit + Visibility, SH/PT_1_InitPass.wgsl:316-322,774-802 */
static float visibility(const ctx *c, v3 start, v3 end) {
    float T = 1.0f;
    float dist = vlength(vsub(end, start));
    v3 dir = vdivs(vsub(end, start), dist);
    ray r = {start, dir};
    float remain = dist;
    for (int it = 0; it < 5; ++it) {
        hit h = trace_ray(c, r);
        if (!h.valid || h.t > remain) return T;
        desc d = get_desc(c, inst_mesh(c, h.s.inst));
        material m = get_material(c, &d, h.s.mat);
        if (m.transmission == 0.0f) return 0.0f;
        T *= m.transmission;
        remain -= h.t;
        surface s = get_surface(c, h.s);
        r.o = s.pos;
    }
    return 0.0f;
}

/* CreateEnvLight, SH/PT_1_InitPass.wgsl:717-730 */
static light_sample create_env_light(const surface *X, v3 V, v3 L) {
    light_sample s;
    memset(&s, 0, sizeof s);
    s.pos = vadd(X->pos, vscale(L, INF_F));
    s.type = LIGHT_ENV;
    s.dir = vneg(L);
    s.id = -1;
    s.Le = V3(ENV_C, ENV_C, ENV_C);
    s.pdf = pdf_bsdf(X, V, L);
    return s;
}

/* ------------------------------------------------------------------ camera */
static ray camera_ray(const ctx *c, uint32_t x, uint32_t y) { /* GenerateRayFromThreadID, PT_01:496-507 */
    const float *vpinv = (const float *)(c->U + U_VPINV);
    float u = ((float)x + 0.5f) / (float)c->U[U_W];
    float v = ((float)y + 0.5f) / (float)c->U[U_H];
    ray clip = {V3(2.0f * u - 1.0f, 2.0f * v - 1.0f, 0.0f), V3(0.0f, 0.0f, 1.0f)};
    return transform_ray(vpinv, clip, 1);
}
static v3 get_x0(const ctx *c, uint32_t x, uint32_t y) { /* Get_X0, PT_1:732-738 */
    const float *vpinv = (const float *)(c->U + U_VPINV);
    float u = ((float)x + 0.5f) / (float)c->U[U_W];
    float v = ((float)y + 0.5f) / (float)c->U[U_H];
    return xform_point(vpinv, V3(2.0f * u - 1.0f, 2.0f * v - 1.0f, 0.0f));
}
static inline uint32_t init_seed(const ctx *c, uint32_t x, uint32_t y) { /* PT_1:823-826 */
    return pto_pcg(x * 1973u + y * 9277u + c->U[U_FRAME] * 26699u);
}

/* G-buffer texel encode / decode, PT_01:643-653, PT_1:409-436 */
static inline void encode_compact(compact s, uint32_t *out4) {
    out4[0] = (s.valid << 31) | (s.inst << 16) | s.mat;
    out4[1] = s.prim;
    out4[2] = u32_of(s.bu);
    out4[3] = u32_of(s.bv);
}
static inline compact decode_compact(const uint32_t *in4) {
    compact s;
    s.valid = (in4[0] & 0x80000000u) != 0u;
    s.inst = (in4[0] & 0x7fff0000u) >> 16;
    s.mat = in4[0] & 0x0000ffffu;
    s.prim = in4[1];
    s.bu = f32_of(in4[2]);
    s.bv = f32_of(in4[3]);
    return s;
}

static void ctx_init(ctx *c, const pto_inputs *in, pass_eps eps, pto_counters *cnt) {
    c->U = in->uniform;
    c->S = in->scene;
    c->G = in->geometry;
    c->A = in->accel;
    c->eps = eps;
    c->cnt = cnt;
}

/* ================================================================== PT_01 G-buffer */
void pto_gbuffer(const pto_inputs *in, int x0, int y0, int x1, int y1, uint32_t *gbuffer, pto_counters *cnt) {
    ctx c;
    ctx_init(&c, in, EPS_GBUFFER, cnt);
    const uint32_t W = c.U[U_W];
    for (int y = y0; y < y1; ++y)
        for (int x = x0; x < x1; ++x) {
            ray r = camera_ray(&c, (uint32_t)x, (uint32_t)y);
            hit h = trace_ray(&c, r);
            compact s = h.s;
            s.valid = (uint32_t)h.valid;
            encode_compact(s, gbuffer + 4u * ((uint32_t)y * W + (uint32_t)x));
        }
}

/* ================================================================== PT_1 init pass */
typedef struct path_state {
    v3 pos[4];          /* Path.Surface[k].Position, k = 0..3                 */
    float rough[4];     /* Path.Surface[k].Material.Roughness (k >= 1)        */
    uint32_t lobe[4];   /* Path.Lobe[k] as set after SampleBSDF at vertex k   */
    uint32_t nee_seed[4], bsdf_seed[4]; /* Path.rSeed[k+1] before NEE / BSDF at k */
    compact cs[4];      /* CSurface[k]                                        */
} path_state;

/* CompressPath + SafeReconnectionIndex, PT_1:1262-1353, on the candidate chosen by
 * UpdateReservoir. Candidate = (vertex i, NEE or env).  The snapshot Path it stands for
 * has Surface[0..i] = the chain's, Lobe[1..i-1] set (and Lobe[i] for env),
 * rSeed[2..i] = BSDF seeds of vertices 1..i-1, rSeed[i+1] = NEE seed (NEE) or BSDF seed
 * (env) of vertex i, zero elsewhere. */
static void compress_path(const path_state *ps, int i, int is_env, const light_sample *XL, uint32_t *out,
                          int rcnext) {
    uint32_t lobe[8] = {0}, seed[8] = {0};
    for (int k = 1; k < i; ++k) { lobe[k] = ps->lobe[k]; seed[k + 1] = ps->bsdf_seed[k]; }
    if (is_env) { lobe[i] = ps->lobe[i]; seed[i + 1] = ps->bsdf_seed[i]; }
    else seed[i + 1] = ps->nee_seed[i];
    const uint32_t length = (uint32_t)i + 1u;
    uint32_t k = 0;
    for (uint32_t kk = 2; kk < length; ++kk) {
        float ra = lobe[kk - 1] == LOBE_LAMBERT ? 1.0f : ps->rough[kk - 1];
        float rb = lobe[kk] == LOBE_LAMBERT ? 1.0f : ps->rough[kk];
        int rough = fmin_(ra, rb) >= RECONNECTION_ROUGHNESS;
        int far = vlength(vsub(ps->pos[kk - 1], ps->pos[kk])) >= RECONNECTION_DISTANCE;
        if (far && rough) { k = kk; break; }
    }
    if (k == 0) {
        int rough = ps->rough[length - 1] >= RECONNECTION_ROUGHNESS;
        int dirl = XL->type == LIGHT_DIRECTION || XL->type == LIGHT_ENV;
        int far = dirl || vlength(vsub(ps->pos[length - 1], XL->pos)) >= RECONNECTION_DISTANCE;
        if (far && rough) k = length;
    }
    memset(out, 0, 4u * PTO_RESERVOIR_WORDS);
    out[0] = seed[2]; out[1] = seed[3]; out[2] = seed[4]; out[3] = seed[5];
    out[4] = u32_of(XL->dir.x); out[5] = u32_of(XL->dir.y); out[6] = u32_of(XL->dir.z);
    out[7] = XL->type;
    out[8] = u32_of(XL->pos.x); out[9] = u32_of(XL->pos.y); out[10] = u32_of(XL->pos.z);
    out[11] = (uint32_t)XL->id;
    out[12] = u32_of(XL->Le.x); out[13] = u32_of(XL->Le.y); out[14] = u32_of(XL->Le.z);
    out[15] = u32_of(XL->pdf);
    out[20] = k;
    out[23] = length;
    if (k != 0) {
        int is_light = (k == length);
        out[22] = is_light ? LOBE_LIGHT : lobe[k];
        out[21] = lobe[k - 1];
        if (!is_light) encode_compact(ps->cs[k], out + 16);
        /* the reuse pipeline's PT_1 (rcnext): the vertex after x_k in words 24..27 (pads in the
         * reference layout, PT_4 never reads them) -- the hybrid shift keeps it fixed (RES_RC_NEXT) */
        if (rcnext && k + 1u < length) encode_compact(ps->cs[k + 1u], out + 24);
    }
}

static void init_pixel(const ctx *c, const uint32_t *gbuffer, uint32_t x, uint32_t y, uint32_t *res, int rcnext) {
    const uint32_t W = c->U[U_W];
    compact x1 = decode_compact(gbuffer + 4u * (y * W + x));
    if (!x1.valid) { /* reservoir unobservable: PT_4 returns before LoadReservoir (:1404-1408) */
        memset(res, 0, 4u * PTO_RESERVOIR_WORDS);
        return;
    }
    uint32_t seed = init_seed(c, x, y);
    v3 f = V3(1.0f, 1.0f, 1.0f);
    float p = 1.0f;
    path_state ps;
    memset(&ps, 0, sizeof ps);
    surface X[4];
    memset(X, 0, sizeof X);
    ps.cs[1] = x1;
    X[0].pos = get_x0(c, x, y);
    X[1] = get_surface(c, x1);
    ps.pos[0] = X[0].pos;
    ps.pos[1] = X[1].pos;
    ps.rough[1] = X[1].mat.roughness;
    /* PathReservoir */
    uint32_t C = 0;
    float w_sum = 0.0f, p_hat_sel = 0.0f;
    int sel_i = -1, sel_env = 0;
    light_sample sel_XL;
    memset(&sel_XL, 0, sizeof sel_XL);

    for (int i = 1; i < 4; ++i) {
        const surface *S = &X[i];
        v3 V = vnormalize(vsub(X[i - 1].pos, S->pos));
        /* Submit NEE path, PT_1:1407-1422 */
        ps.nee_seed[i] = seed;
        light_sample XL = sample_nee(c, &seed, S, V);
        v3 L = direction_to_light(S, &XL);
        v3 contrib = vmul(f, l_emit(c, &XL, S));
        contrib = vmul(contrib, bsdf(S, V, L));
        contrib = vscale(contrib, fabsf(vdot(S->nrm, L)));
        contrib = vscale(contrib, visibility(c, S->pos, XL.pos));
        float p_hat = luminance(contrib);
        float ris = p_hat / (p * XL.pdf);
        C += 1u; /* UpdateReservoir, PT_1:1298-1320 */
        w_sum += ris;
        if (pto_random(&seed) < ris / w_sum) { sel_i = i; sel_env = 0; sel_XL = XL; p_hat_sel = p_hat; }
        if (i == 3) break;
        /* Sample BSDF, PT_1:1427-1433 */
        ps.bsdf_seed[i] = seed;
        uint32_t lobe;
        L = sample_bsdf(&seed, S, V, &lobe);
        ps.lobe[i] = lobe;
        /* path throughput + Russian roulette, PT_1:1436-1442 */
        v3 b = vscale(bsdf(S, V, L), fabsf(vdot(S->nrm, L)));
        f = vmul(f, b);
        p *= pdf_bsdf(S, V, L);
        float p_survive = luminance(f) / p;
        if (pto_random(&seed) < p_survive) p *= p_survive;
        else break;
        ray r = {S->pos, L};
        hit h = trace_ray(c, r);
        if (!h.valid) { /* Submit env path, PT_1:1447-1461 */
            light_sample env = create_env_light(S, V, L);
            float ph = luminance(vscale(f, ENV_C));
            float ris_e = ph / p;
            C += 1u;
            w_sum += ris_e;
            if (pto_random(&seed) < ris_e / w_sum) { sel_i = i; sel_env = 1; sel_XL = env; p_hat_sel = ph; }
            break;
        }
        ps.cs[i + 1] = h.s;
        X[i + 1] = get_surface(c, h.s);
        ps.pos[i + 1] = X[i + 1].pos;
        ps.rough[i + 1] = X[i + 1].mat.roughness;
    }
    /* StoreReservoir, PT_1:1475-1483 */
    if (sel_i < 0) memset(res, 0, 4u * PTO_RESERVOIR_WORDS); /* zero Path(): length 0, k 0 */
    else compress_path(&ps, sel_i, sel_env, &sel_XL, res, rcnext);
    res[28] = u32_of(w_sum / p_hat_sel);
    res[29] = C;
}

static void init_rows(const pto_inputs *in, const uint32_t *gbuffer, int x0, int y0, int x1, int y1,
                      uint32_t *reservoir, pto_counters *cnt, int rcnext) {
    ctx c;
    ctx_init(&c, in, EPS_INIT, cnt);
    const uint32_t W = c.U[U_W];
    for (int y = y0; y < y1; ++y)
        for (int x = x0; x < x1; ++x)
            init_pixel(&c, gbuffer, (uint32_t)x, (uint32_t)y,
                       reservoir + PTO_RESERVOIR_WORDS * ((uint32_t)y * W + (uint32_t)x), rcnext);
}
void pto_init(const pto_inputs *in, const uint32_t *gbuffer, int x0, int y0, int x1, int y1, uint32_t *reservoir,
              pto_counters *cnt) {
    init_rows(in, gbuffer, x0, y0, x1, y1, reservoir, cnt, 0);
}

/* ================================================================== PT_4 final shading */
static void write_color(const ctx *c, float *px, v3 col) { /* WriteColor, PT_4:599-606 */
    float t = 1.0f / (float)(c->U[U_FRAME] + 1u);
    px[0] = mixf(px[0], col.x, t);
    px[1] = mixf(px[1], col.y, t);
    px[2] = mixf(px[2], col.z, t);
    px[3] = 1.0f;
}

static void final_pixel(const ctx *c, const uint32_t *gbuffer, const uint32_t *res, uint32_t x, uint32_t y,
                        float *px) {
    const uint32_t W = c->U[U_W];
    compact x1 = decode_compact(gbuffer + 4u * (y * W + x));
    if (!x1.valid) { px[0] = px[1] = px[2] = ENV_C; px[3] = 1.0f; return; }
    const uint32_t C = res[29], length = res[23];
    if (C == 0u || length < 2u) { write_color(c, px, V3(0.0f, 0.0f, 0.0f)); return; }
    light_sample XL;
    XL.dir = V3(f32_of(res[4]), f32_of(res[5]), f32_of(res[6]));
    XL.type = res[7];
    XL.pos = V3(f32_of(res[8]), f32_of(res[9]), f32_of(res[10]));
    XL.id = (int32_t)res[11];
    XL.Le = V3(f32_of(res[12]), f32_of(res[13]), f32_of(res[14]));
    XL.pdf = f32_of(res[15]);
    /* RegeneratePath, PT_4:1357-1384 */
    surface S[8];
    memset(S, 0, sizeof S);
    S[0].pos = get_x0(c, x, y);
    S[1] = get_surface(c, x1);
    for (uint32_t i = 1; i + 1u < length; ++i) {
        v3 V = vnormalize(vsub(S[i - 1].pos, S[i].pos));
        uint32_t seed = res[i - 1u];
        uint32_t lobe;
        v3 dir = sample_bsdf(&seed, &S[i], V, &lobe);
        ray r = {S[i].pos, dir};
        hit h = trace_ray(c, r);
        S[i + 1] = get_surface(c, h.s); /* a miss decodes the zero CompactSurface, as the WGSL does */
    }
    /* PathContribution, PT_4:1306-1336 */
    v3 f = V3(1.0f, 1.0f, 1.0f);
    for (uint32_t i = 1; i + 1u < length; ++i) {
        v3 V = vnormalize(vsub(S[i - 1].pos, S[i].pos));
        v3 L = vnormalize(vsub(S[i + 1].pos, S[i].pos));
        f = vmul(f, vscale(bsdf(&S[i], L, V), fabsf(vdot(S[i].nrm, L))));
    }
    {
        const surface *P = &S[length - 2u], *Xc = &S[length - 1u];
        v3 V = vnormalize(vsub(P->pos, Xc->pos));
        v3 L = direction_to_light(Xc, &XL);
        f = vmul(f, vscale(bsdf(Xc, L, V), fabsf(vdot(Xc->nrm, L))));
        f = vmul(f, vscale(l_emit(c, &XL, Xc), visibility(c, Xc->pos, XL.pos)));
    }
    write_color(c, px, vscale(f, f32_of(res[28])));
}

/* reuse: PT_4 of the reuse pipeline -- a reservoir a reuse pass wrote carries its sample's
 * PathContribution at this pixel (words 26, 27, 30; flag word 31, write_reused): f * UCW, the
 * contribution of the shifted path it holds (a hybrid-shifted sample is NOT its seeds' replay);
 * any other reservoir is PT_4's replay (final_pixel). */
static void final_rows(const pto_inputs *in, const uint32_t *gbuffer, const uint32_t *reservoir, int x0, int y0,
                       int x1, int y1, float *accum, pto_counters *cnt, int reuse) {
    ctx c;
    ctx_init(&c, in, EPS_FINAL, cnt);
    const uint32_t W = c.U[U_W];
    for (int y = y0; y < y1; ++y)
        for (int x = x0; x < x1; ++x) {
            uint32_t p = (uint32_t)y * W + (uint32_t)x;
            const uint32_t *res = reservoir + PTO_RESERVOIR_WORDS * p;
            float *px = accum + 4u * p;
            if (reuse && decode_compact(gbuffer + 4u * p).valid && res[29] != 0u && res[23] >= 2u && res[31] == 1u)
                write_color(&c, px, vscale(V3(f32_of(res[26]), f32_of(res[27]), f32_of(res[30])), f32_of(res[28])));
            else
                final_pixel(&c, gbuffer, res, (uint32_t)x, (uint32_t)y, px);
        }
}
void pto_final(const pto_inputs *in, const uint32_t *gbuffer, const uint32_t *reservoir, int x0, int y0, int x1,
               int y1, float *accum, pto_counters *cnt) {
    final_rows(in, gbuffer, reservoir, x0, y0, x1, y1, accum, cnt, 0);
}

/* ================================================================== reuse passes
 * Temporal and spatial reuse are NOT in the reference code: only specified in
 * docs/theory/ReSTIR_Pipeline.md:259-462 (pass 2 temporal, pass 3 spatial: generalized
 * balance heuristic with confidences, m_i = c_i p_i / sum_j c_j p_j, w_i = m_i p_hat W_i)
 * and docs/theory/memo.md:166-231 (shifts with a Jacobian).  The build-defined rules
 *  are restated here so that the HIP kernels can be checked bit for bit:
 *
 *  - sample = the reservoir's (rSeed, XL, length); PT_4 consumes exactly that, replaying
 *    the BSDF draws from rSeed at ITS OWN pixel (PT_4:1357-1384).  The shift between pixels
 *    is therefore random replay of rSeed from the target pixel's primary hit, with the
 *    light endpoint XL kept (a reconnection on the light).
 *  - target p_hat_d(x) = Luminance(PathContribution) of the sample replayed in domain d
 *    (pixel d's camera point and G-buffer hit), PT_4's formulas: the integrand PT_4 weights.
 *  - Jacobian of the shift x -> y: q(x) / q(y), q = prod_i pdf_bsdf(replayed vertex i) / g,
 *    g = |n_light . l| / r^2 for a rect light (solid angle of the fixed light point), else 1.
 *    q also divides by beta, PT_1's roulette factor on the path (rr_step): PT_1's
 *    contribution weights integrate beta * f, so a sample moved between pixels is
 *    re-weighted by beta_target / beta_source and reuse keeps PT_1 + PT_4's expectation.
 *  - confidences (word 29 of a reused reservoir) depend on geometry and history only,
 *    never on sample values (a sample-dependent MIS weight biases the estimate): a PT_1
 *    reservoir counts 1; neighbours count iff inside the image with a G-buffer hit.
 *  - temporal: same pixel of the previous frame's spatial output (static camera: same
 *    domain, identity shift), history confidence capped at `cap`.
 *  - spatial: M neighbours in a (2R+1)^2 square, pairwise MIS with confidences.
 *  - every reservoir written by a reuse pass stores p_hat (word 24) and q (word 25) of its
 *    sample in its own domain; RNG streams are salted per pass.
 *  - ... and the sample's PathContribution f there (words 26, 27, 30 = f.xyz, word 31 = 1),
 *    when known: eval_sample's f IS PT_4's PathContribution of that reservoir at that pixel
 *    (same replay, same products), so PT_4 of a reused reservoir equals f * UCW; the GPU
 *    final pass uses that instead of replaying (PT_4 below still replays: the check). */
#define SALT_TEMPORAL 0x54454D50u
#define SALT_SPATIAL 0x53504154u

typedef struct eval_out { int valid; float phat, q; v3 f; } eval_out;

static inline uint32_t reuse_seed(const ctx *c, uint32_t x, uint32_t y, uint32_t salt) {
    return pto_pcg(init_seed(c, x, y) ^ salt);
}
static inline int wrs_update(float *w_sum, float w, uint32_t *seed) { /* UpdateReservoir, PT_1:1298-1320 */
    *w_sum += w;
    return pto_random(seed) < w / *w_sum;
}

/* PT_1's throughput recursion and Russian roulette (PT_1:1427-1442) along a replayed
 * vertex: the roulette multiplies p by p_survive even when p_survive > 1, so PT_1's
 * weights carry beta = prod min(1, p_survive) / p_survive; the shift carries it along. */
static void rr_step(const surface *X, v3 V, v3 L, float pdf, v3 *f, float *p, float *beta, int *ok) {
    *f = vmul(*f, vscale(bsdf(X, V, L), fabsf(vdot(X->nrm, L))));
    *p *= pdf;
    const float ps = luminance(*f) / *p;
    if (!(ps > 0.0f)) *ok = 0; /* PT_1 ends such a path: no sample of this shape here */
    *p *= ps;
    if (ps > 1.0f) *beta /= ps;
}

/* ---- the hybrid (reconnection) shift, docs/theory/memo.md:174-229 ----
 * PT_1's CompressPath stores k = SafeReconnectionIndex(path) (PT_1:1262-1353): the first vertex
 * x_k (k >= 2) whose edge from x_{k-1} is long (>= RECONNECTION_DISTANCE) and rough at both ends
 * (>= RECONNECTION_ROUGHNESS; a Lambert lobe counts as rough), else k = length when the last
 * vertex may reconnect to the light sample, else 0.  RcVertex = x_k's compact surface.
 *  - k in [2, length-1] (a surface reconnection): the shifted path into domain y is
 *      y0 -> y1 -> (random replay of the seeds) -> y_{k-1} -> x_k -> x_{k+1} -> .. -> XL:
 *    the prefix up to y_{k-1} replays the sample's seeds from y's primary hit, x_k and the
 *    suffix after it are kept (x_{k+1}: RES_RC_NEXT, the light sample XL).  Valid iff the prefix
 *    replays (every traced ray hits), the shifted path has the SAME reconnection index (its
 *    edges before k are not safe, (y_{k-1}, x_k) is -- the lobes: the replayed ones, then the
 *    stored Lobe_{k-1}, Lobe_k), and nothing lies between y_{k-1} and x_k (the closest hit along
 *    the connection, if any, at >= 0.999 of its length).
 *  - k = length (light) or 0 (unshiftable): random replay of every vertex with the light
 *    endpoint kept (the build's shift of round 1).
 * Measure and Jacobian.  The reuse passes integrate in PT_1's measure (solid angle per sampled
 * direction, the light sample's own at the end), J(x -> y) = q(x) / q(y):
 *    random replay:     q = prod_{replayed i} pdf_i / (g beta)            (g: rect light geometry)
 *    hybrid, vertex k:  q = (prod_{i <= k-2} pdf_i * |x_k - x_{k-1}|^2 / |n_k . w|) / beta
 * -- the replayed directions keep their primary samples (dw_y / dw_x = pdf_x / pdf_y), the
 * reconnection keeps x_k in area (dw = dA |n_k . w| / d^2), the suffix is unchanged.  This is the
 * memo's J = J_y / J_x written in PT_1's measure instead of primary-sample space (there the
 * pdfs of picking x_k and x_{k+1} enter; here the pdfs of the directions the shift changes are
 * not part of the sample's measure).  beta is PT_1's Russian-roulette factor along the path
 * (rr_step), recomputed with the shifted path's own directions.
 * Every shift keeps the sample's reconnection index: the shifted path's own SafeReconnectionIndex
 * must be k (else the shift is invalid), so a path of a domain is reached only under the label
 * PT_1 would give it there and the MIS weights of the techniques that reach it sum to one.  (The
 * lobes: the replayed ones, the stored Lobe_{k-1} / Lobe_k, an env escape's lobe Lobe_{k-1} when
 * k = length, else taken as GGX -- material roughness -- exact whenever the Lambert promotion of
 * IsSafeToReconnect decides nothing, as in the benchmark scenes: opaque roughness >= 0.5, glass 0.)
 * Evaluating the canonical sample AT HOME (its own pixel, the reference-layout PT_1 output)
 * replays it (PT_4's RegeneratePath: same vertices), with q in its sample's form above.
 * Reuse layout: a reservoir a reuse pass wrote (RES_REUSE_LAYOUT in word 20) holds x_{k+1} in
 * words 0..3 -- seeds a hybrid shift at k = 2 never replays -- because words 24..31 carry
 * p_hat, q and f there; PT_1's output holds it in 24..27. */
#define RES_REUSE_LAYOUT 0x100u
static inline int safe_edge(const surface *A, uint32_t la, const surface *B, uint32_t lb) { /* IsSafeToReconnect */
    const float ra = la == LOBE_LAMBERT ? 1.0f : A->mat.roughness;
    const float rb = lb == LOBE_LAMBERT ? 1.0f : B->mat.roughness;
    const int rough = fmin_(ra, rb) >= RECONNECTION_ROUGHNESS;
    const int far = vlength(vsub(A->pos, B->pos)) >= RECONNECTION_DISTANCE;
    return far && rough;
}
/* SafeReconnectionIndex (PT_1:1281-1296) of a shifted path S[0..length-1] with lobes[1..]
 * (compress_path's conventions: the NEE vertex's lobe 0 = Lambert) and light sample XL */
static uint32_t path_label(const surface *S, const uint32_t *lobes, uint32_t length, const light_sample *XL) {
    for (uint32_t kk = 2u; kk < length; ++kk)
        if (safe_edge(&S[kk - 1u], lobes[kk - 1u], &S[kk], lobes[kk])) return kk;
    const int rough = S[length - 1u].mat.roughness >= RECONNECTION_ROUGHNESS;
    const int dirl = XL->type == LIGHT_DIRECTION || XL->type == LIGHT_ENV;
    const int far = dirl || vlength(vsub(S[length - 1u].pos, XL->pos)) >= RECONNECTION_DISTANCE;
    return (far && rough) ? length : 0u;
}
static inline const uint32_t *res_rc_next(const uint32_t *r) { /* RES_RC_NEXT: x_{k+1}'s compact */
    return (r[20] & RES_REUSE_LAYOUT) ? r : r + 24;
}

/* The reservoir sample `res` in the domain of pixel (x, y) with G-buffer hit x1 (home: the
 * pixel's own PT_1 sample, replayed): PathContribution of PT_4:1306-1336 over the shifted path
 * plus the shift's measure q. */
static eval_out eval_sample(const ctx *c, uint32_t x, uint32_t y, compact x1, const uint32_t *res, int home) {
    eval_out o = {0, 0.0f, 0.0f, {0.0f, 0.0f, 0.0f}};
    const uint32_t length = res[23];
    if (!x1.valid || res[29] == 0u || length < 2u) return o;
    light_sample XL;
    XL.dir = V3(f32_of(res[4]), f32_of(res[5]), f32_of(res[6]));
    XL.type = res[7];
    XL.pos = V3(f32_of(res[8]), f32_of(res[9]), f32_of(res[10]));
    XL.id = (int32_t)res[11];
    XL.Le = V3(f32_of(res[12]), f32_of(res[13]), f32_of(res[14]));
    XL.pdf = f32_of(res[15]);
    const uint32_t k = res[20] & 0xFFu;
    const int hyb = k >= 2u && k < length;   /* reconnection at the surface vertex x_k */
    const int shift = hyb && !home;          /* replay only the prefix up to y_{k-1} */
    surface S[8];
    memset(S, 0, sizeof S);
    uint32_t lobes[8] = {0};
    S[0].pos = get_x0(c, x, y);
    S[1] = get_surface(c, x1);
    float prod = 1.0f, beta = 1.0f, rr_p = 1.0f;
    v3 rr_f = V3(1.0f, 1.0f, 1.0f);
    int rr_ok = 1;
    const uint32_t reach = shift ? k - 1u : length - 1u; /* the replay reaches S[reach] */
    for (uint32_t i = 1; i < reach; ++i) {
        v3 V = vnormalize(vsub(S[i - 1].pos, S[i].pos));
        uint32_t seed = res[i - 1u], lobe;
        v3 dir = sample_bsdf(&seed, &S[i], V, &lobe);
        lobes[i] = lobe;
        const float pdf = pdf_bsdf(&S[i], V, dir);
        if (!hyb || i + 2u <= k) prod *= pdf; /* (hybrid: the replayed prefix only) */
        rr_step(&S[i], V, dir, pdf, &rr_f, &rr_p, &beta, &rr_ok);
        ray r = {S[i].pos, dir};
        hit h = trace_ray(c, r);
        if (!h.valid) return o; /* the replayed path escapes: no such path in this domain */
        S[i + 1] = get_surface(c, h.s);
    }
    if (shift) {
        S[k] = get_surface(c, decode_compact(res + 16));
        lobes[k - 1u] = res[21];
        lobes[k] = res[22];
        if (path_label(S, lobes, k + 1u, &XL) != k) return o; /* the same reconnection index */
        const v3 dv = vsub(S[k].pos, S[k - 1u].pos);
        const float dist = vlength(dv);
        const v3 dir = vdivs(dv, dist);
        ray r = {S[k - 1u].pos, dir};
        hit h = trace_ray(c, r);
        if (h.valid && h.t < dist * 0.999f) return o; /* occluded: nothing between y_{k-1} and x_k */
        const v3 V = vnormalize(vsub(S[k - 2u].pos, S[k - 1u].pos));
        rr_step(&S[k - 1u], V, dir, pdf_bsdf(&S[k - 1u], V, dir), &rr_f, &rr_p, &beta, &rr_ok);
        if (k + 1u < length) { /* the kept vertex after x_k */
            S[k + 1u] = get_surface(c, decode_compact(res_rc_next(res)));
            const v3 V2 = vnormalize(vsub(S[k - 1u].pos, S[k].pos));
            const v3 L2 = vnormalize(vsub(S[k + 1u].pos, S[k].pos));
            rr_step(&S[k], V2, L2, pdf_bsdf(&S[k], V2, L2), &rr_f, &rr_p, &beta, &rr_ok);
        }
    } else if (!home) { /* random replay keeps the label too (k = length or 0) */
        if (XL.type == LIGHT_ENV) lobes[length - 1u] = k == length ? res[21] : LOBE_GGX;
        if (path_label(S, lobes, length, &XL) != k) return o;
    }
    v3 f = V3(1.0f, 1.0f, 1.0f);
    for (uint32_t i = 1; i + 1u < length; ++i) {
        v3 V = vnormalize(vsub(S[i - 1].pos, S[i].pos));
        v3 L = vnormalize(vsub(S[i + 1].pos, S[i].pos));
        f = vmul(f, vscale(bsdf(&S[i], L, V), fabsf(vdot(S[i].nrm, L))));
    }
    const surface *P = &S[length - 2u], *Xc = &S[length - 1u];
    v3 V = vnormalize(vsub(P->pos, Xc->pos));
    v3 L = direction_to_light(Xc, &XL);
    if (XL.type == LIGHT_ENV) /* the escape direction passed PT_1's roulette too */
        rr_step(Xc, V, L, pdf_bsdf(Xc, V, L), &rr_f, &rr_p, &beta, &rr_ok);
    f = vmul(f, vscale(bsdf(Xc, L, V), fabsf(vdot(Xc->nrm, L))));
    float g = 1.0f;
    if (XL.type == LIGHT_RECT) {
        v3 r = vsub(XL.pos, Xc->pos);
        v3 Ld = vnormalize(r);
        g = fabsf(vdot(get_light(c, (uint32_t)XL.id).dir, Ld)) / vdot(r, r);
    }
    f = vmul(f, vscale(l_emit(c, &XL, Xc), visibility(c, Xc->pos, XL.pos)));
    float q;
    if (hyb) { /* the reconnection edge's area -> solid angle factor at x_k */
        const v3 dv = vsub(S[k].pos, S[k - 1u].pos);
        const float d2 = vdot(dv, dv);
        const float ck = fabsf(vdot(S[k].nrm, vdivs(dv, sqrtf(d2))));
        q = (prod * (d2 / ck)) / beta;
    } else {
        q = prod / (g * beta);
    }
    o.valid = rr_ok && q > 0.0f && q <= 3.402823466e38f;
    o.phat = o.valid ? luminance(f) : 0.0f;
    o.q = o.valid ? q : 0.0f;
    if (o.valid) o.f = f;
    return o;
}

/* the contribution stored with a reused sample: f (known = its eval was valid) */
typedef struct sel_f { int known; v3 f; } sel_f;
static sel_f stored_f(const uint32_t *r) { /* words 26, 27, 30, 31 of a reused reservoir */
    sel_f o = {r[31] == 1u, V3(f32_of(r[26]), f32_of(r[27]), f32_of(r[30]))};
    return o;
}
static sel_f eval_f(eval_out e) { sel_f o = {e.valid, e.f}; return o; }

static void write_reused(uint32_t *out, const uint32_t *src, float p_sel, float q_sel, sel_f f_sel, float w_sum,
                         uint32_t C) {
    uint32_t tmp[24];
    memcpy(tmp, src, sizeof tmp); /* src may alias out (temporal works in place) */
    if (f_sel.known && !(tmp[20] & RES_REUSE_LAYOUT)) { /* a PT_1 sample: into the reuse layout */
        const uint32_t k = tmp[20] & 0xFFu;
        if (k >= 2u && k + 1u < tmp[23]) memcpy(tmp, src + 24, 4u * 4u); /* x_{k+1} over unused seeds */
        tmp[20] |= RES_REUSE_LAYOUT;
    }
    memset(out, 0, 4u * PTO_RESERVOIR_WORDS);
    memcpy(out, tmp, sizeof tmp);
    out[24] = u32_of(p_sel);
    out[25] = u32_of(q_sel);
    out[28] = u32_of(p_sel > 0.0f ? w_sum / p_sel : 0.0f);
    out[29] = C;
    if (f_sel.known) {
        out[26] = u32_of(f_sel.f.x);
        out[27] = u32_of(f_sel.f.y);
        out[30] = u32_of(f_sel.f.z);
        out[31] = 1u;
    }
}

/* Temporal reuse (ReSTIR_Pipeline.md:259-340) of pixel (x, y): canonical = this frame's
 * PT_1 reservoir, history = the previous frame's spatial output at the same pixel. */
static void temporal_pixel(const ctx *c, const uint32_t *gbuffer, uint32_t *cur, const uint32_t *hist,
                           const pto_reuse_params *prm, uint32_t x, uint32_t y) {
    const uint32_t W = c->U[U_W];
    compact x1 = decode_compact(gbuffer + 4u * (y * W + x));
    if (!x1.valid) return; /* PT_1 wrote the zero reservoir; PT_4 never reads it */
    uint32_t seed = reuse_seed(c, x, y, SALT_TEMPORAL);
    eval_out ec = eval_sample(c, x, y, x1, cur, 1);
    const int canon_ok = ec.valid && ec.phat > 0.0f;
    /* confidences depend on geometry and history only, never on the samples: a PT_1
     * reservoir counts 1, the history min(C_hist, cap) */
    const uint32_t Cp = prm->hist_valid ? (hist[29] < prm->temporal_cap ? hist[29] : prm->temporal_cap) : 0u;
    const float cp = (float)Cp, tot = 1.0f + cp;
    const float pp = f32_of(hist[24]), qp = f32_of(hist[25]);
    const int hist_ok = Cp != 0u && hist[23] >= 2u && pp > 0.0f;
    const float wc = canon_ok ? (1.0f / tot) * ec.phat * f32_of(cur[28]) : 0.0f;
    const float wp = hist_ok ? (cp / tot) * pp * f32_of(hist[28]) : 0.0f;
    float w_sum = 0.0f;
    const uint32_t *src = cur;
    float p_sel = ec.phat, q_sel = ec.q;
    sel_f f_sel = eval_f(ec);
    if (wrs_update(&w_sum, wc, &seed)) { src = cur; p_sel = ec.phat; q_sel = ec.q; f_sel = eval_f(ec); }
    if (wrs_update(&w_sum, wp, &seed)) { src = hist; p_sel = pp; q_sel = qp; f_sel = stored_f(hist); }
    write_reused(cur, src, p_sel, q_sel, f_sel, w_sum, 1u + Cp);
}

/* ---- temporal reuse under camera motion (build-defined; ReSTIR_Pipeline.md:259-340) ----
 * The spec's history is ReservoirBuffer_Prev[CurrentPixel - MotionVector]: the previous
 * frame's spatial output at the pixel p' the current primary hit projected to in the previous
 * frame, whose sample lives in the PREVIOUS frame's domain (its camera point x0' and primary
 * hit x1' at p').  Rules (restated bit for bit by wtmotion_* in ptx_reuse.hip):
 *  - VP' = the f32 rounding of the double-precision inverse of the previous VP^-1
 *    (pto_mat4_inverse: cofactors along the first column, one fixed operation order);
 *  - p' = floor(((VP' (P, 1)).xy / w + 1) * 0.5 * (W, H)), P = the current primary hit;
 *    none when w <= 0 or p' is outside the image (a disocclusion past the border), and none
 *    when p' lies more than `radius` rows from the pixel (motion_rows): a row band's motion
 *    halo holds exactly those rows, so any split of the frame gives the same history;
 *  - the history is used iff x1' exists, n(x1') . n(x1) >= 0.9 and the depths along the
 *    previous view agree within 5 %: | |x1' - x0'| - |P - x0'| | <= 0.05 |P - x0'| (geometry
 *    only: the confidence never depends on a sample);
 *  - MIS: the generalized balance heuristic with confidences (the spec's m_i) = the spatial
 *    pass's pairwise rule with M = 1: the history sample shifted here (random replay, its
 *    Jacobian q_h / q_c), the canonical sample shifted into the previous domain for its own
 *    weight; c_c = 1, c_h = min(C_hist, cap); canonical draw first, then the history. */
typedef struct pto_motion {
    const uint32_t *prev_uniform;  /* the previous frame's 33 words (its VP^-1, camera position) */
    const uint32_t *gbuffer_prev;  /* the previous frame's G-buffer (W*H*4)                      */
} pto_motion;

/* 4x4 inverse (column-major f32 in, f32 out) in double precision by cofactors (zeros when
 * singular) -- the host side of the reprojection; ptx_api.cpp uses the same expression order. */
void pto_mat4_inverse(const float *mf, float *out) {
    double m[16], inv[16];
    for (int i = 0; i < 16; ++i) m[i] = (double)mf[i];
    inv[0] = m[5] * m[10] * m[15] - m[5] * m[11] * m[14] - m[9] * m[6] * m[15] + m[9] * m[7] * m[14] + m[13] * m[6] * m[11] - m[13] * m[7] * m[10];
    inv[4] = -m[4] * m[10] * m[15] + m[4] * m[11] * m[14] + m[8] * m[6] * m[15] - m[8] * m[7] * m[14] - m[12] * m[6] * m[11] + m[12] * m[7] * m[10];
    inv[8] = m[4] * m[9] * m[15] - m[4] * m[11] * m[13] - m[8] * m[5] * m[15] + m[8] * m[7] * m[13] + m[12] * m[5] * m[11] - m[12] * m[7] * m[9];
    inv[12] = -m[4] * m[9] * m[14] + m[4] * m[10] * m[13] + m[8] * m[5] * m[14] - m[8] * m[6] * m[13] - m[12] * m[5] * m[10] + m[12] * m[6] * m[9];
    inv[1] = -m[1] * m[10] * m[15] + m[1] * m[11] * m[14] + m[9] * m[2] * m[15] - m[9] * m[3] * m[14] - m[13] * m[2] * m[11] + m[13] * m[3] * m[10];
    inv[5] = m[0] * m[10] * m[15] - m[0] * m[11] * m[14] - m[8] * m[2] * m[15] + m[8] * m[3] * m[14] + m[12] * m[2] * m[11] - m[12] * m[3] * m[10];
    inv[9] = -m[0] * m[9] * m[15] + m[0] * m[11] * m[13] + m[8] * m[1] * m[15] - m[8] * m[3] * m[13] - m[12] * m[1] * m[11] + m[12] * m[3] * m[9];
    inv[13] = m[0] * m[9] * m[14] - m[0] * m[10] * m[13] - m[8] * m[1] * m[14] + m[8] * m[2] * m[13] + m[12] * m[1] * m[10] - m[12] * m[2] * m[9];
    inv[2] = m[1] * m[6] * m[15] - m[1] * m[7] * m[14] - m[5] * m[2] * m[15] + m[5] * m[3] * m[14] + m[13] * m[2] * m[7] - m[13] * m[3] * m[6];
    inv[6] = -m[0] * m[6] * m[15] + m[0] * m[7] * m[14] + m[4] * m[2] * m[15] - m[4] * m[3] * m[14] - m[12] * m[2] * m[7] + m[12] * m[3] * m[6];
    inv[10] = m[0] * m[5] * m[15] - m[0] * m[7] * m[13] - m[4] * m[1] * m[15] + m[4] * m[3] * m[13] + m[12] * m[1] * m[7] - m[12] * m[3] * m[5];
    inv[14] = -m[0] * m[5] * m[14] + m[0] * m[6] * m[13] + m[4] * m[1] * m[14] - m[4] * m[2] * m[13] - m[12] * m[1] * m[6] + m[12] * m[2] * m[5];
    inv[3] = -m[1] * m[6] * m[11] + m[1] * m[7] * m[10] + m[5] * m[2] * m[11] - m[5] * m[3] * m[10] - m[9] * m[2] * m[7] + m[9] * m[3] * m[6];
    inv[7] = m[0] * m[6] * m[11] - m[0] * m[7] * m[10] - m[4] * m[2] * m[11] + m[4] * m[3] * m[10] + m[8] * m[2] * m[7] - m[8] * m[3] * m[6];
    inv[11] = -m[0] * m[5] * m[11] + m[0] * m[7] * m[9] + m[4] * m[1] * m[11] - m[4] * m[3] * m[9] - m[8] * m[1] * m[7] + m[8] * m[3] * m[5];
    inv[15] = m[0] * m[5] * m[10] - m[0] * m[6] * m[9] - m[4] * m[1] * m[10] + m[4] * m[2] * m[9] + m[8] * m[1] * m[6] - m[8] * m[2] * m[5];
    const double det = m[0] * inv[0] + m[1] * inv[4] + m[2] * inv[8] + m[3] * inv[12];
    for (int i = 0; i < 16; ++i) out[i] = det != 0.0 ? (float)(inv[i] / det) : 0.0f;
}

/* p' of world point P through the previous frame's VP (column-major f32): 0 if none */
static int reproject(const float *vp, v3 P, uint32_t W, uint32_t H, uint32_t *px, uint32_t *py) {
    const float cx = ((vp[0] * P.x + vp[4] * P.y) + vp[8] * P.z) + vp[12];
    const float cy = ((vp[1] * P.x + vp[5] * P.y) + vp[9] * P.z) + vp[13];
    const float cw = ((vp[3] * P.x + vp[7] * P.y) + vp[11] * P.z) + vp[15];
    if (!(cw > 0.0f)) return 0;
    const float fx = ((cx / cw + 1.0f) * 0.5f) * (float)W, fy = ((cy / cw + 1.0f) * 0.5f) * (float)H;
    if (!(fx >= 0.0f && fx < (float)W && fy >= 0.0f && fy < (float)H)) return 0;
    *px = (uint32_t)fx;
    *py = (uint32_t)fy;
    return 1;
}
/* p' row within `radius` rows of the pixel's row y (the build's motion rule above) */
static inline int motion_rows(uint32_t py, uint32_t y, uint32_t radius) {
    return (py > y ? py - y : y - py) <= radius;
}
/* the disocclusion test of the history at p' (x1' = Sp with camera point x0p) for the
 * current primary hit P with normal Nc */
static int motion_valid(const surface *Sp, v3 x0p, v3 P, v3 Nc) {
    if (!(vdot(Sp->nrm, Nc) >= 0.9f)) return 0;
    const float dp = vlength(vsub(Sp->pos, x0p)), dc = vlength(vsub(P, x0p));
    return fabsf(dp - dc) <= 0.05f * dc;
}

/* The history of pixel (x, y) under camera motion (DI and GI): its primary hit S1 reprojected to p'
 * = (px, py) in the previous frame, with that frame's hit x1p there passing the disocclusion test;
 * 0 if none (the rules above) */
static int motion_lookup(const ctx *c, const ctx *cprev, const float *vp_prev, const surface *S1, uint32_t y,
                         const uint32_t *gbuffer_prev, uint32_t radius, uint32_t *px, uint32_t *py, compact *x1p) {
    const uint32_t W = c->U[U_W], H = c->U[U_H];
    if (!reproject(vp_prev, S1->pos, W, H, px, py) || !motion_rows(*py, y, radius)) return 0;
    *x1p = decode_compact(gbuffer_prev + 4u * (*py * W + *px));
    if (!x1p->valid) return 0;
    const surface Sp = get_surface(c, *x1p);
    return motion_valid(&Sp, get_x0(cprev, *px, *py), S1->pos, S1->nrm);
}

static void temporal_motion_pixel(const ctx *c, const ctx *cprev, const float *vp_prev, const uint32_t *gbuffer,
                                  uint32_t *cur, const uint32_t *hist_all, const uint32_t *gbuffer_prev,
                                  const pto_reuse_params *prm, uint32_t x, uint32_t y) {
    const uint32_t W = c->U[U_W];
    compact x1 = decode_compact(gbuffer + 4u * (y * W + x));
    if (!x1.valid) return; /* PT_1 wrote the zero reservoir; PT_4 never reads it */
    uint32_t seed = reuse_seed(c, x, y, SALT_TEMPORAL);
    eval_out ec = eval_sample(c, x, y, x1, cur, 1);
    const int canon_ok = ec.valid && ec.phat > 0.0f;
    const float cc = 1.0f, pc = ec.phat, qc = ec.q, Wc = f32_of(cur[28]);
    /* the history pixel p' and its domain */
    uint32_t Cp = 0u, px = 0u, py = 0u;
    compact x1p = {0u, 0u, 0u, 0u, 0.0f, 0.0f};
    const uint32_t *h = NULL;
    if (prm->hist_valid) {
        const surface S1 = get_surface(c, x1);
        if (motion_lookup(c, cprev, vp_prev, &S1, y, gbuffer_prev, prm->radius, &px, &py, &x1p)) {
            h = hist_all + PTO_RESERVOIR_WORDS * (py * W + px);
            Cp = h[29] < prm->temporal_cap ? h[29] : prm->temporal_cap;
        }
    }
    const float cp = (float)Cp;
    /* forward: the history sample in this pixel's domain */
    float wh = 0.0f, pf = 0.0f, qf = 0.0f;
    sel_f ff = {0, {0.0f, 0.0f, 0.0f}};
    if (Cp != 0u && h[23] >= 2u && f32_of(h[24]) > 0.0f) {
        const float ph = f32_of(h[24]), qh = f32_of(h[25]), Wh = f32_of(h[28]);
        eval_out F = eval_sample(c, x, y, x1, h, 0);
        if (F.valid) {
            const float J = qh / F.q;
            const float pb = ph / J;
            const float den = cc * F.phat + cp * pb;
            const float m = den > 0.0f ? (cp * pb) / den : 0.0f;
            wh = m * F.phat * Wh * J;
            pf = F.phat;
            qf = F.q;
            ff = eval_f(F);
        }
    }
    /* backward: this pixel's sample in the previous domain (its weight) */
    float Q = 1.0f;
    if (canon_ok && Cp != 0u) {
        eval_out B = eval_sample(cprev, px, py, x1p, cur, 0);
        if (B.valid) {
            const float pbc = B.phat * qc / B.q;
            const float den = cc * pc + cp * pbc;
            Q = den > 0.0f ? (cc * pc) / den : 1.0f;
        }
    }
    const float wc = canon_ok ? Q * pc * Wc : 0.0f;
    float w_sum = 0.0f, p_sel = ec.phat, q_sel = ec.q;
    const uint32_t *src = cur;
    sel_f f_sel = eval_f(ec);
    if (wrs_update(&w_sum, wc, &seed)) { src = cur; p_sel = ec.phat; q_sel = ec.q; f_sel = eval_f(ec); }
    if (wrs_update(&w_sum, wh, &seed)) { src = h; p_sel = pf; q_sel = qf; f_sel = ff; }
    write_reused(cur, src, p_sel, q_sel, f_sel, w_sum, 1u + Cp);
}

void pto_temporal_motion(const pto_inputs *in, const pto_motion *mot, const uint32_t *gbuffer, uint32_t *res_cur,
                         const uint32_t *res_hist, const pto_reuse_params *prm, int x0, int y0, int x1, int y1,
                         pto_counters *cnt) {
    ctx c, cprev;
    ctx_init(&c, in, EPS_FINAL, cnt);
    pto_inputs pin = *in;
    pin.uniform = mot->prev_uniform;
    ctx_init(&cprev, &pin, EPS_FINAL, cnt);
    float vp_prev[16];
    pto_mat4_inverse((const float *)(mot->prev_uniform + U_VPINV), vp_prev);
    const uint32_t W = c.U[U_W];
    for (int y = y0; y < y1; ++y)
        for (int x = x0; x < x1; ++x) {
            const uint32_t p = (uint32_t)y * W + (uint32_t)x;
            temporal_motion_pixel(&c, &cprev, vp_prev, gbuffer, res_cur + PTO_RESERVOIR_WORDS * p, res_hist,
                                  mot->gbuffer_prev, prm, (uint32_t)x, (uint32_t)y);
        }
}

/* Spatial neighbour k of (x, y): two draws, offsets in [-R, R]^2. Returns 1 if inside the
 * image and not the pixel itself. */
static int spatial_neighbor(uint32_t *seed, uint32_t R, uint32_t x, uint32_t y, uint32_t W, uint32_t H,
                            uint32_t *nx, uint32_t *ny) {
    const float side = (float)(2u * R + 1u);
    uint32_t ix = (uint32_t)(pto_random(seed) * side), iy = (uint32_t)(pto_random(seed) * side);
    if (ix > 2u * R) ix = 2u * R; /* Random() can return exactly 1.0 */
    if (iy > 2u * R) iy = 2u * R;
    const int64_t X = (int64_t)x + (int64_t)ix - (int64_t)R, Y = (int64_t)y + (int64_t)iy - (int64_t)R;
    if (X < 0 || Y < 0 || X >= (int64_t)W || Y >= (int64_t)H || (ix == R && iy == R)) return 0;
    *nx = (uint32_t)X;
    *ny = (uint32_t)Y;
    return 1;
}

/* Spatial reuse (ReSTIR_Pipeline.md:342-462) with pairwise MIS: for neighbour n and shift
 * y = T(x_n), m_n(y) = c_n p_n->c(y) / (c_c p_c(y) + M c_n p_n->c(y)); the canonical sample
 * gets m_c = (1/M) sum_n c_c p_c / (c_c p_c + M c_n p_n->c(x_c)). */
static void spatial_pixel(const ctx *c, const uint32_t *gbuffer, const uint32_t *cur, uint32_t *out,
                          const pto_reuse_params *prm, uint32_t x, uint32_t y) {
    const uint32_t W = c->U[U_W], H = c->U[U_H];
    const uint32_t p = y * W + x;
    compact x1 = decode_compact(gbuffer + 4u * p);
    uint32_t *o = out + PTO_RESERVOIR_WORDS * p;
    if (!x1.valid) { memset(o, 0, 4u * PTO_RESERVOIR_WORDS); return; }
    const uint32_t *rc = cur + PTO_RESERVOIR_WORDS * p;
    uint32_t seed = reuse_seed(c, x, y, SALT_SPATIAL);
    const uint32_t M = prm->neighbors;
    uint32_t nb[16];
    int present[16];
    for (uint32_t k = 0; k < M; ++k) {
        uint32_t nx = 0, ny = 0;
        present[k] = spatial_neighbor(&seed, prm->radius, x, y, W, H, &nx, &ny);
        nb[k] = ny * W + nx;
        if (present[k]) present[k] = decode_compact(gbuffer + 4u * nb[k]).valid; /* geometry only */
    }
    const float Mf = (float)M, cc = (float)rc[29];
    const float pc = f32_of(rc[24]), qc = f32_of(rc[25]), Wc = f32_of(rc[28]);
    const int canon_ok = rc[29] != 0u && rc[23] >= 2u && pc > 0.0f;
    float wn[16], pf[16], qf[16], sumQ = 0.0f;
    sel_f ff[16];
    uint32_t Csum = rc[29];
    for (uint32_t k = 0; k < M; ++k) {
        wn[k] = 0.0f; pf[k] = 0.0f; qf[k] = 0.0f;
        ff[k].known = 0; ff[k].f = V3(0.0f, 0.0f, 0.0f);
        float Q = 1.0f;
        if (present[k]) {
            const uint32_t *rn = cur + PTO_RESERVOIR_WORDS * nb[k];
            const uint32_t nx = nb[k] % W, ny = nb[k] / W;
            const float cn = (float)rn[29], pn = f32_of(rn[24]), qn = f32_of(rn[25]), Wn = f32_of(rn[28]);
            Csum += rn[29];
            if (rn[23] >= 2u && pn > 0.0f) { /* forward: the neighbour's sample in this pixel's domain */
                eval_out F = eval_sample(c, x, y, x1, rn, 0);
                if (F.valid) {
                    const float J = qn / F.q;
                    const float pb = pn / J;
                    const float den = cc * F.phat + Mf * cn * pb;
                    const float m = den > 0.0f ? (cn * pb) / den : 0.0f;
                    wn[k] = m * F.phat * Wn * J;
                    pf[k] = F.phat;
                    qf[k] = F.q;
                    ff[k] = eval_f(F);
                }
            }
            if (canon_ok) { /* backward: this pixel's sample in the neighbour's domain */
                eval_out B = eval_sample(c, nx, ny, decode_compact(gbuffer + 4u * nb[k]), rc, 0);
                if (B.valid) {
                    const float pbc = B.phat * qc / B.q;
                    const float den = cc * pc + Mf * cn * pbc;
                    Q = den > 0.0f ? (cc * pc) / den : 1.0f;
                }
            }
        }
        sumQ += Q;
    }
    const float wc = canon_ok ? (sumQ / Mf) * pc * Wc : 0.0f;
    float w_sum = 0.0f, p_sel = pc, q_sel = qc;
    const uint32_t *src = rc;
    sel_f f_sel = stored_f(rc);
    if (wrs_update(&w_sum, wc, &seed)) { src = rc; p_sel = pc; q_sel = qc; f_sel = stored_f(rc); }
    for (uint32_t k = 0; k < M; ++k)
        if (wrs_update(&w_sum, wn[k], &seed)) {
            src = cur + PTO_RESERVOIR_WORDS * nb[k];
            p_sel = pf[k];
            q_sel = qf[k];
            f_sel = ff[k];
        }
    write_reused(o, src, p_sel, q_sel, f_sel, w_sum, Csum);
}

/* Test helper: eval_sample of reservoir `res` in the domain of pixel (x, y). out = {valid, p_hat, q}. */
void pto_eval_sample(const pto_inputs *in, const uint32_t *gbuffer, uint32_t x, uint32_t y, const uint32_t *res,
                     float out[3]) {
    ctx c;
    ctx_init(&c, in, EPS_FINAL, NULL);
    eval_out o = eval_sample(&c, x, y, decode_compact(gbuffer + 4u * (y * c.U[U_W] + x)), res, 0);
    out[0] = (float)o.valid;
    out[1] = o.phat;
    out[2] = o.q;
}

void pto_temporal(const pto_inputs *in, const uint32_t *gbuffer, uint32_t *res_cur, const uint32_t *res_hist,
                  const pto_reuse_params *prm, int x0, int y0, int x1, int y1, pto_counters *cnt) {
    ctx c;
    ctx_init(&c, in, EPS_FINAL, cnt);
    const uint32_t W = c.U[U_W];
    for (int y = y0; y < y1; ++y)
        for (int x = x0; x < x1; ++x) {
            const uint32_t p = (uint32_t)y * W + (uint32_t)x;
            temporal_pixel(&c, gbuffer, res_cur + PTO_RESERVOIR_WORDS * p, res_hist + PTO_RESERVOIR_WORDS * p, prm,
                           (uint32_t)x, (uint32_t)y);
        }
}

void pto_spatial(const pto_inputs *in, const uint32_t *gbuffer, const uint32_t *res_cur, uint32_t *res_out,
                 const pto_reuse_params *prm, int x0, int y0, int x1, int y1, pto_counters *cnt) {
    ctx c;
    ctx_init(&c, in, EPS_FINAL, cnt);
    for (int y = y0; y < y1; ++y)
        for (int x = x0; x < x1; ++x) spatial_pixel(&c, gbuffer, res_cur, res_out, prm, (uint32_t)x, (uint32_t)y);
}

/* ================================================================== TEST_MCPT */
/* GetLightColor, SH/TEST_MCPT.wgsl:1261-1309 */
static v3 light_color(const ctx *c, uint32_t *seed, const surface *X, v3 V, uint32_t id) {
    light_sample XL;
    memset(&XL, 0, sizeof XL);
    light ls = get_light(c, id);
    XL.type = ls.type;
    XL.Le = vscale(ls.color, ls.intensity);
    switch (ls.type) {
    case LIGHT_DIRECTION:
        XL.pos = vsub(X->pos, vscale(ls.dir, INF_F));
        XL.dir = ls.dir;
        XL.pdf = 1.0f;
        break;
    case LIGHT_POINT:
        XL.pos = ls.pos;
        XL.dir = vnormalize(vsub(X->pos, ls.pos));
        XL.pdf = 1.0f;
        break;
    case LIGHT_RECT: {
        float ru = pto_random(seed) * 2.0f - 1.0f;
        float rv = pto_random(seed) * 2.0f - 1.0f;
        v3 off = vadd(vscale(ls.U, ru), vscale(ls.V, rv));
        XL.pos = vadd(ls.pos, off);
        XL.dir = vnormalize(vsub(X->pos, XL.pos));
        v3 r = vsub(XL.pos, X->pos);
        v3 L = vnormalize(r);
        XL.pdf = vdot(r, r) / fmax_(ls.area * fabsf(vdot(ls.dir, L)), EPS_F);
        break;
    }
    default: break;
    }
    v3 L = direction_to_light(X, &XL);
    v3 out = vmul(l_emit(c, &XL, X), bsdf(X, V, L));
    out = vscale(out, fabsf(vdot(X->nrm, L)));
    out = vscale(out, visibility(c, X->pos, XL.pos));
    return vdivs(out, XL.pdf);
}

static void mcpt_pixel(const ctx *c, uint32_t x, uint32_t y, float *px) { /* TEST_MCPT.wgsl:1315-1372 */
    uint32_t seed = init_seed(c, x, y);
    ray r = camera_ray(c, x, y);
    v3 color = V3(0.0f, 0.0f, 0.0f), f = V3(1.0f, 1.0f, 1.0f);
    float p = 1.0f;
    const uint32_t nl = c->U[U_LIGHT_COUNT];
    for (int bounce = 0; bounce < 3; ++bounce) {
        hit h = trace_ray(c, r);
        if (!h.valid) {
            color = vadd(color, vscale(vdivs(f, p), ENV_C));
            break;
        }
        surface X = get_surface(c, h.s);
        v3 V = vnormalize(vsub(r.o, X.pos));
        for (uint32_t id = 0; id < nl; ++id)
            color = vadd(color, vmul(vdivs(f, p), light_color(c, &seed, &X, V, id)));
        uint32_t lobe;
        v3 L = sample_bsdf(&seed, &X, V, &lobe);
        f = vmul(f, vscale(bsdf(&X, V, L), fabsf(vdot(X.nrm, L))));
        p *= pdf_bsdf(&X, V, L);
        r.o = X.pos;
        r.d = L;
        float ps = luminance(f) / p;
        if (pto_random(&seed) < ps) p *= ps;
        else break;
    }
    write_color(c, px, color);
}

void pto_mcpt(const pto_inputs *in, int x0, int y0, int x1, int y1, float *accum, pto_counters *cnt) {
    ctx c;
    ctx_init(&c, in, EPS_MCPT, cnt);
    const uint32_t W = c.U[U_W];
    for (int y = y0; y < y1; ++y)
        for (int x = x0; x < x1; ++x)
            mcpt_pixel(&c, (uint32_t)x, (uint32_t)y, accum + 4u * ((uint32_t)y * W + (uint32_t)x));
}

/* ================================================================== ray queries */
void pto_trace(const pto_inputs *in, const float *rays, float *hits, size_t n, int eps_mode, pto_counters *cnt) {
    ctx c;
    ctx_init(&c, in, eps_mode == 0 ? EPS_GBUFFER : EPS_INIT, cnt);
    for (size_t i = 0; i < n; ++i) {
        const float *r = rays + 8 * i;
        ray q = {V3(r[0], r[1], r[2]), V3(r[3], r[4], r[5])};
        hit h = trace_ray(&c, q);
        float *o = hits + 8 * i;
        uint32_t enc = ((uint32_t)h.valid << 31) | (h.s.inst << 16) | h.s.mat;
        v3 pos = V3(0.0f, 0.0f, 0.0f);
        if (h.valid) pos = get_surface(&c, h.s).pos;
        o[0] = h.t; o[1] = f32_of(enc); o[2] = f32_of(h.s.prim); o[3] = h.s.bu;
        o[4] = h.s.bv; o[5] = pos.x; o[6] = pos.y; o[7] = pos.z;
    }
}

/* ================================================================== KAT helpers */
static surface kat_surface(const float *n, const float *mat) {
    surface s;
    memset(&s, 0, sizeof s);
    s.nrm = V3(n[0], n[1], n[2]);
    s.mat.albedo = V3(mat[0], mat[1], mat[2]);
    s.mat.metalness = mat[3];
    s.mat.roughness = mat[4];
    s.mat.transmission = mat[5];
    s.mat.ior = mat[6];
    return s;
}
void pto_bsdf(const float n[3], const float mat[7], const float v[3], const float l[3], float out[3]) {
    surface s = kat_surface(n, mat);
    v3 r = bsdf(&s, V3(v[0], v[1], v[2]), V3(l[0], l[1], l[2]));
    out[0] = r.x; out[1] = r.y; out[2] = r.z;
}
float pto_pdf_bsdf(const float n[3], const float mat[7], const float v[3], const float l[3]) {
    surface s = kat_surface(n, mat);
    return pdf_bsdf(&s, V3(v[0], v[1], v[2]), V3(l[0], l[1], l[2]));
}
void pto_sample_bsdf(const float n[3], const float mat[7], const float v[3], uint32_t *seed, float out_dir[3],
                     uint32_t *out_lobe) {
    surface s = kat_surface(n, mat);
    v3 d = sample_bsdf(seed, &s, V3(v[0], v[1], v[2]), out_lobe);
    out_dir[0] = d.x; out_dir[1] = d.y; out_dir[2] = d.z;
}
float pto_ray_triangle(const float o[3], const float d[3], const float p0[3], const float p1[3], const float p2[3],
                       float det_eps) {
    ray r = {V3(o[0], o[1], o[2]), V3(d[0], d[1], d[2])};
    return ray_triangle(r, V3(p0[0], p0[1], p0[2]), V3(p1[0], p1[1], p1[2]), V3(p2[0], p2[1], p2[2]), det_eps);
}

/* ================================================================== threaded driver */
typedef struct job {
    int pass, tid, nthreads, x0, y0, x1, y1;
    const pto_inputs *in;
    uint32_t *gbuffer, *reservoir, *res_hist;
    float *accum;
    const pto_reuse_params *prm;
    pto_counters cnt;
    const pto_motion *mot;
} job;

static void *worker(void *arg) {
    job *j = (job *)arg;
    for (int y = j->y0 + j->tid; y < j->y1; y += j->nthreads) {
        switch (j->pass) {
        case 0: pto_gbuffer(j->in, j->x0, y, j->x1, y + 1, j->gbuffer, &j->cnt); break;
        case 1: pto_init(j->in, j->gbuffer, j->x0, y, j->x1, y + 1, j->reservoir, &j->cnt); break;
        case 11: init_rows(j->in, j->gbuffer, j->x0, y, j->x1, y + 1, j->reservoir, &j->cnt, 1); break;
        case 12: final_rows(j->in, j->gbuffer, j->reservoir, j->x0, y, j->x1, y + 1, j->accum, &j->cnt, 1); break;
        case 2: pto_final(j->in, j->gbuffer, j->reservoir, j->x0, y, j->x1, y + 1, j->accum, &j->cnt); break;
        case 3: pto_mcpt(j->in, j->x0, y, j->x1, y + 1, j->accum, &j->cnt); break;
        case 5: pto_temporal(j->in, j->gbuffer, j->reservoir, j->res_hist, j->prm, j->x0, y, j->x1, y + 1, &j->cnt); break;
        case 6: pto_spatial(j->in, j->gbuffer, j->reservoir, j->res_hist, j->prm, j->x0, y, j->x1, y + 1, &j->cnt); break;
        case 7:
            pto_temporal_motion(j->in, j->mot, j->gbuffer, j->reservoir, j->res_hist, j->prm, j->x0, y, j->x1, y + 1,
                                &j->cnt);
            break;
        default: break;
        }
    }
    return NULL;
}

static int run_pass_m(int pass, int nthreads, const pto_inputs *in, int x0, int y0, int x1, int y1,
                      uint32_t *gbuffer, uint32_t *reservoir, uint32_t *res_hist, const pto_reuse_params *prm,
                      float *accum, pto_counters *cnt, const pto_motion *mot);
static int run_pass(int pass, int nthreads, const pto_inputs *in, int x0, int y0, int x1, int y1,
                    uint32_t *gbuffer, uint32_t *reservoir, uint32_t *res_hist, const pto_reuse_params *prm,
                    float *accum, pto_counters *cnt) {
    return run_pass_m(pass, nthreads, in, x0, y0, x1, y1, gbuffer, reservoir, res_hist, prm, accum, cnt, NULL);
}
static int run_pass_m(int pass, int nthreads, const pto_inputs *in, int x0, int y0, int x1, int y1,
                      uint32_t *gbuffer, uint32_t *reservoir, uint32_t *res_hist, const pto_reuse_params *prm,
                      float *accum, pto_counters *cnt, const pto_motion *mot) {
    if (nthreads < 1) nthreads = 1;
    job *jobs = (job *)calloc((size_t)nthreads, sizeof(job));
    pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
    if (!jobs || !th) { free(jobs); free(th); return -1; }
    for (int t = 0; t < nthreads; ++t) {
        job j = {pass, t, nthreads, x0, y0, x1, y1, in, gbuffer, reservoir, res_hist, accum, prm, {0, 0, 0, 0, 0}, mot};
        jobs[t] = j;
        if (nthreads > 1) pthread_create(&th[t], NULL, worker, &jobs[t]);
    }
    if (nthreads == 1) worker(&jobs[0]);
    for (int t = 0; t < nthreads; ++t) {
        if (nthreads > 1) pthread_join(th[t], NULL);
        if (cnt) {
            cnt->rays += jobs[t].cnt.rays;
            cnt->instance_xforms += jobs[t].cnt.instance_xforms;
            cnt->aabb_tests += jobs[t].cnt.aabb_tests;
            cnt->tri_tests += jobs[t].cnt.tri_tests;
            cnt->hits += jobs[t].cnt.hits;
        }
    }
    free(jobs);
    free(th);
    return 0;
}

int pto_run(int pass, int nthreads, const pto_inputs *in, int x0, int y0, int x1, int y1, uint32_t *gbuffer,
            uint32_t *reservoir, float *accum, pto_counters *cnt) {
    if (pass == 4) {
        int rc = run_pass(0, nthreads, in, x0, y0, x1, y1, gbuffer, reservoir, NULL, NULL, accum, cnt);
        if (!rc) rc = run_pass(1, nthreads, in, x0, y0, x1, y1, gbuffer, reservoir, NULL, NULL, accum, cnt);
        if (!rc) rc = run_pass(2, nthreads, in, x0, y0, x1, y1, gbuffer, reservoir, NULL, NULL, accum, cnt);
        return rc;
    }
    if ((pass < 0 || pass > 3) && pass != 11 && pass != 12) return -2;
    return run_pass(pass, nthreads, in, x0, y0, x1, y1, gbuffer, reservoir, NULL, NULL, accum, cnt);
}

int pto_run_reuse(int pass, int nthreads, const pto_inputs *in, int x0, int y0, int x1, int y1,
                  const uint32_t *gbuffer, uint32_t *res_cur, uint32_t *res_hist, const pto_reuse_params *prm,
                  pto_counters *cnt) {
    if ((pass != 5 && pass != 6) || !prm || prm->neighbors > 16u) return -2;
    return run_pass(pass, nthreads, in, x0, y0, x1, y1, (uint32_t *)gbuffer, res_cur, res_hist, prm, NULL, cnt);
}
/* pass 7: temporal reuse under camera motion (temporal_motion_pixel) */
int pto_run_temporal_motion(int nthreads, const pto_inputs *in, int x0, int y0, int x1, int y1,
                            const uint32_t *gbuffer, uint32_t *res_cur, const uint32_t *res_hist,
                            const uint32_t *prev_uniform, const uint32_t *gbuffer_prev, const pto_reuse_params *prm,
                            pto_counters *cnt) {
    if (!prm || !prev_uniform || !gbuffer_prev) return -2;
    pto_motion mot = {prev_uniform, gbuffer_prev};
    return run_pass_m(7, nthreads, in, x0, y0, x1, y1, (uint32_t *)gbuffer, res_cur, (uint32_t *)res_hist, prm, NULL,
                      cnt, &mot);
}
#include "pt_oracle_gi.c"
