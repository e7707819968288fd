// ptx_device.h -- device-side scene layout, f32 math and BVH traversal for gfx950.
//
// Semantics follow the reference WGSL (SH/ = apps/frontend/src/graphics-core/shaders/),
// with every implementation-defined WGSL detail fixed as in DESIGN.md §Numerics and
// compiled with -ffp-contract=off so that ray setup, slab tests, Moller-Trumbore and
// barycentrics are bit-identical to the CPU oracle.
//
// MI355X layout (built once per scene by ptx_api.cpp from the reference arrays):
//   * tris:  per triangle 3 x float4 = {v0.xyz, e1.x} {e1.yz, e2.xy} {e2.z, -, -, -}
//            (local space, leaf order; e1 = v1 - v0, e2 = v2 - v0 exactly as
//            GetRayTriangleHitDistance computes them, SH/PT_1_InitPass.wgsl:522-523)
//   * nodes: one 64-byte record per interior BVH node holding BOTH children's boxes and
//            refs, so a node visit is 4 x 16-byte loads instead of the reference's
//            3 x 32-byte node fetches (GetBlasNode x3, SH/PT_1_InitPass.wgsl:633-642);
//            the same binary tree, visited in the same order.
//   * subs:  per (mesh, sub-mesh) root box + root ref.
//   * insts: per instance M, M^-1, mesh, sub range, triangle base.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ptx {

// ------------------------------------------------------------------ constants
// SH/PT_1_InitPass.wgsl:193-221
constexpr uint32_t STRIDE_INSTANCE = 33u;
constexpr uint32_t STRIDE_LIGHT = 18u;
constexpr uint32_t STRIDE_DESCRIPTOR = 6u;
constexpr uint32_t STRIDE_MATERIAL = 15u;
constexpr uint32_t STRIDE_VERTEX = 8u;
constexpr float RECONNECTION_DISTANCE = 0.1f;
constexpr float RECONNECTION_ROUGHNESS = 0.5f;
constexpr float INF_F = 1e11f;
constexpr float EPS_F = 1e-4f;
constexpr float PI_F = 3.141592f;
constexpr float ENV_C = 0.5f;
constexpr uint32_t LIGHT_DIRECTION = 0u, LIGHT_POINT = 1u, LIGHT_RECT = 2u, LIGHT_ENV = 3u;
constexpr uint32_t LOBE_LAMBERT = 0u, LOBE_GGX = 1u, LOBE_LIGHT = 3u;

enum : uint32_t {
    U_W = 0, U_H = 1, U_VPINV = 4, U_CAMPOS = 20, U_FRAME = 23, U_OFF_DESC = 24, U_OFF_MAT = 25,
    U_OFF_LIGHT = 26, U_OFF_CDF = 27, U_OFF_INDEX = 28, U_OFF_SUBROOT = 29, U_OFF_BLAS = 30,
    U_INST_COUNT = 31, U_LIGHT_COUNT = 32
};

// child / stack reference encoding: interior node index, or LEAF_BIT | count<<24 | first tri
constexpr uint32_t LEAF_BIT = 0x80000000u;
constexpr uint32_t LEAF_FIRST_MASK = 0x00FFFFFFu;

// Both children's boxes by axis: {lmin.a, rmin.a, lmax.a, rmax.a} for a = x, y, z, then the
// refs -- each axis's slab terms of the two children are one packed-FP32 pair (box_pair).
struct alignas(16) NodePair {   // 64 B
    float x[4], y[4], z[4];
    uint32_t lref, rref, pad0, pad1;
};
struct alignas(16) SubRoot {    // 32 B: the root box by axis, {min, max} pairs (box_root)
    float x[2], y[2], z[2];
    uint32_t ref;
    uint32_t pad;  // the sub-mesh's transmission (f32 bits, Scene::mats word 5): subs_transmission
};
struct alignas(16) Inst {       // 176 B
    float m[16];
    float minv[16];
    uint32_t mesh, sub_base, nsub, tri_base;  // mesh: | kInstIdentity when M and M^-1 are exactly I
    // Conservative world-space box of the instance's sub-mesh roots (inst_may_hit): the local
    // root boxes' union mapped back through (M^-1)^-1 in double precision, rounded outward; a ray
    // is tested against it padded by wpad + wscale * max|o| (wpad < 0: never culled)
    float wlo[3], wpad;
    float whi[3], wscale;
};
constexpr uint32_t kInstIdentity = 0x80000000u;

// Everything a kernel reads, passed by value (lives in the kernarg segment).
struct Scene {
    uint32_t U[33];       // uniform block (33 words), by value: race-free per-frame update
    const uint32_t *S;    // SceneBuffer
    const uint32_t *G;    // GeometryBuffer
    const float4 *tris;   // 3 float4 per triangle
    const NodePair *nodes;
    const SubRoot *subs;
    const Inst *insts;
    const float4 *mats;   // 2 float4 per sub-mesh (SubRoot numbering): GetMaterial, pre-applied
    const float4 *tverts; // 5 float4 per triangle (triangle-table order): its 3 vertices' position + normal
    uint32_t n_inst, n_subs;
    uint32_t width, height, row_begin, row_end;
    unsigned long long *counters;  // nullptr unless PTX_FLAG_COUNT_WORK
    // PTX_FLAG_ROW_CENSUS (counting builds): the work counters go to per-region blocks of
    // kCensusWords instead -- block r < census_tile_rows(): G-buffer rays of band tile row r
    // (8 pixel rows); block census_tile_rows() + s: every query of trace-queue slot s
    // (segments of contiguous tiles in census mode, so the host maps them to tile rows)
    unsigned long long *census;
#ifdef PTX_WG_TIMES
    unsigned long long *wgt;  // diagnostic build only: per-wave {start, end, kernel | block, hw id} records
#endif
};

// Diagnostic build (make wgt -> libptx_wgt.so, tools/wave_timeline.py): every instrumented
// kernel's waves record their start / end on the 100 MHz real-time clock, so the tool can
// draw the chip's wave occupancy over a frame and each launch's tail.  No-op otherwise.
enum : uint32_t { KID_TRACE = 1, KID_GBUF, KID_INIT_START, KID_INIT_STEP, KID_FINAL_START, KID_FINAL_STEP,
                  KID_TEMP_START, KID_TEMP_COMBINE, KID_SPAT_START, KID_JOB_STEP, KID_SPAT_COMBINE };
#ifdef PTX_WG_TIMES
struct WaveTimer {
    unsigned long long *buf;
    unsigned long long t0;
    uint32_t kid;
    __device__ WaveTimer(unsigned long long *b, uint32_t k) : buf(b), t0(__builtin_amdgcn_s_memrealtime()), kid(k) {}
    __device__ ~WaveTimer() {
        if (!buf || __lane_id() != 0u) return;
        const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
        const unsigned long long i = atomicAdd(buf, 1ull);
        if (i >= (1ull << 20)) return;
        unsigned long long *r = buf + 4u + 4u * i;
        r[0] = t0;
        r[1] = t1;
        r[2] = ((unsigned long long)kid << 32) | blockIdx.x;
        r[3] = ((unsigned long long)(threadIdx.x >> 6) << 32) | (unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 4);
    }
};
#define PTX_WAVE_TIMER(sc, k) WaveTimer wave_timer_((sc).wgt, (k))
// one dynamic trace batch {start, end, KID_BATCH << 32 | batch, round << 32 | hw id} (lane 0)
constexpr uint32_t KID_BATCH = 12;
// + {dbg[0] | dbg[1] << 32, dbg[2] | dbg[3] << 32, KID_BATCH_DBG << 32 | dbg[4], dbg[5]} (trace_core_flat)
constexpr uint32_t KID_BATCH_DBG = 15;
__device__ __forceinline__ void batch_record(unsigned long long *buf, unsigned long long t0, uint32_t bi, uint32_t round,
                                             const uint32_t *dbg) {
    if (!buf || __lane_id() != 0u) return;
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    const unsigned long long i = atomicAdd(buf, 2ull);
    if (i + 1u >= (1ull << 20)) return;
    unsigned long long *r = buf + 4u + 4u * i;
    r[0] = t0;
    r[1] = t1;
    r[2] = ((unsigned long long)KID_BATCH << 32) | bi;
    r[3] = ((unsigned long long)round << 32) | (unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 4);
    r[4] = (unsigned long long)dbg[0] | ((unsigned long long)dbg[1] << 32);
    r[5] = (unsigned long long)dbg[2] | ((unsigned long long)dbg[3] << 32);
    r[6] = ((unsigned long long)KID_BATCH_DBG << 32) | dbg[4];
    r[7] = dbg[5];
}
// straggler queries (tools/stragglers.py): a trace call with >= kStragglerAabb slab tests leaves
// two records {o.xy, o.z d.x, KID_STRAGGLER << 32 | slab tests, triangle tests | t_max << 32} and
// {d.yz, t | inst << 32, KID_STRAGGLER2 << 32 | prim, sub-mesh}
constexpr uint32_t KID_STRAGGLER = 13, KID_STRAGGLER2 = 14, kStragglerAabb = 256;
__device__ __forceinline__ unsigned long long pk2(float a, float b) {
    return (unsigned long long)__float_as_uint(a) | ((unsigned long long)__float_as_uint(b) << 32);
}
#else
#define PTX_WAVE_TIMER(sc, k) ((void)0)
#endif

// ------------------------------------------------------------------ f32 vector algebra
// Operation order is fixed (left-to-right sums, no contraction): DESIGN.md §Numerics.
struct f3 { float x, y, z; };
__device__ __forceinline__ f3 mk(float x, float y, float z) { return f3{x, y, z}; }
__device__ __forceinline__ f3 operator+(f3 a, f3 b) { return f3{a.x + b.x, a.y + b.y, a.z + b.z}; }
__device__ __forceinline__ f3 operator-(f3 a, f3 b) { return f3{a.x - b.x, a.y - b.y, a.z - b.z}; }
__device__ __forceinline__ f3 operator*(f3 a, f3 b) { return f3{a.x * b.x, a.y * b.y, a.z * b.z}; }
__device__ __forceinline__ f3 operator*(f3 a, float s) { return f3{a.x * s, a.y * s, a.z * s}; }
// f3 / s = three correctly rounded divisions by one s (normalize is v / length(v)).  (Sharing one
// refined reciprocal over the three, same bits, left the logic kernels within +-3 % and the
// headline -0.6 %: they are not bound by the divisions' issue -- round 4)
__device__ __forceinline__ f3 operator/(f3 a, float s) { return f3{a.x / s, a.y / s, a.z / s}; }
__device__ __forceinline__ f3 operator-(f3 a) { return f3{-a.x, -a.y, -a.z}; }
__device__ __forceinline__ float dot(f3 a, f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ f3 cross(f3 a, f3 b) {
    return f3{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
__device__ __forceinline__ float length(f3 a) { return __builtin_sqrtf(dot(a, a)); }
__device__ __forceinline__ f3 normalize(f3 a) { return a / length(a); }
__device__ __forceinline__ float length3(f3 a) { return length(a); }
__device__ __forceinline__ float mixf(float a, float b, float t) { return a * (1.0f - t) + b * t; }
__device__ __forceinline__ f3 mix3(f3 a, f3 b, float t) { return f3{mixf(a.x, b.x, t), mixf(a.y, b.y, t), mixf(a.z, b.z, t)}; }
__device__ __forceinline__ float saturate(float a) { return fminf(fmaxf(a, 0.0f), 1.0f); }
__device__ __forceinline__ float luminance(f3 c) { return c.x * 0.2126f + c.y * 0.7152f + c.z * 0.0722f; }
__device__ __forceinline__ float asf(uint32_t u) { return __uint_as_float(u); }
__device__ __forceinline__ uint32_t asu(float f) { return __float_as_uint(f); }

// The perspective divide of TransformVec3WithMat4x4.  For affine matrices and finite
// points w is exactly 1.0 and x / 1.0f == x bit for bit (IEEE), so the ~10-instruction
// correctly rounded division is skipped; any other w (projective VP^-1, NaN/inf inputs)
// takes the division, so results are identical to dividing unconditionally.
__device__ __forceinline__ f3 wdivide(float x, float y, float z, float w) {
    if (w == 1.0f) return f3{x, y, z};
    return f3{x / w, y / w, z / w};
}
// column-major mat4 * (p,1) then /w (TransformVec3WithMat4x4, SH/PT_1_InitPass.wgsl:480-484)
__device__ __forceinline__ f3 xform_point(const float *m, f3 p);
__device__ __forceinline__ f3 xform_point_t(const float *m, f3 p);
// The same products for an instance whose matrices are exactly the identity (bitwise 1 / +0):
// ((1 x + 0 y) + 0 z) + 0 * 1 is x + 0 for finite x, y, z (a -0 becomes +0 -- the last term is
// +0 -- and w is exactly 1), so the 28-operation transform reduces to three additions with
// the same bits.  Non-finite points take the full product (0 * inf is NaN there).
__device__ __forceinline__ bool finite3(f3 p) {
    return __builtin_isfinite(p.x) && __builtin_isfinite(p.y) && __builtin_isfinite(p.z);
}
__device__ __forceinline__ f3 inst_point(const Inst &I, const float *m, f3 p) {
    if ((I.mesh & kInstIdentity) && finite3(p)) return f3{p.x + 0.0f, p.y + 0.0f, p.z + 0.0f};
    return xform_point(m, p);
}
__device__ __forceinline__ f3 inst_point_t(const Inst &I, const float *m, f3 p) {
    if ((I.mesh & kInstIdentity) && finite3(p)) return f3{p.x + 0.0f, p.y + 0.0f, p.z + 0.0f};
    return xform_point_t(m, p);
}
__device__ __forceinline__ f3 xform_point(const float *m, f3 p) {
    float x = ((m[0] * p.x + m[4] * p.y) + m[8] * p.z) + m[12] * 1.0f;
    float y = ((m[1] * p.x + m[5] * p.y) + m[9] * p.z) + m[13] * 1.0f;
    float z = ((m[2] * p.x + m[6] * p.y) + m[10] * p.z) + m[14] * 1.0f;
    float w = ((m[3] * p.x + m[7] * p.y) + m[11] * p.z) + m[15] * 1.0f;
    return wdivide(x, y, z, w);
}
// transpose(m) * (p,1) then /w (normal transform, SH/PT_1_InitPass.wgsl:395)
__device__ __forceinline__ f3 xform_point_t(const float *m, f3 p) {
    float x = ((m[0] * p.x + m[1] * p.y) + m[2] * p.z) + m[3] * 1.0f;
    float y = ((m[4] * p.x + m[5] * p.y) + m[6] * p.z) + m[7] * 1.0f;
    float z = ((m[8] * p.x + m[9] * p.y) + m[10] * p.z) + m[11] * 1.0f;
    float w = ((m[12] * p.x + m[13] * p.y) + m[14] * p.z) + m[15] * 1.0f;
    return wdivide(x, y, z, w);
}

// ------------------------------------------------------------------ RNG, SH/PT_1_InitPass.wgsl:810-826
__device__ __forceinline__ uint32_t pcg(uint32_t seed) {
    uint32_t state = seed * 747796405u + 2891336453u;
    uint32_t word = ((state >> ((state >> 28u) + 4u)) ^ state) * 277803737u;
    return (word >> 22u) ^ word;
}
__device__ __forceinline__ float rnd(uint32_t &seed) {
    uint32_t h = pcg(seed);
    seed += 1u;
    return (float)h / 4294967295.0f;
}

// ------------------------------------------------------------------ counters
enum { CNT_RAYS = 0, CNT_INST = 1, CNT_AABB = 2, CNT_TRI = 3, CNT_HITS = 4 };
// SIMD-utilisation profile of trace_core (COUNT == 2 builds, diagnostics only): per region
// {wave-level executions, active lanes summed over them} at counters[8 + 2*region]
enum { PROF_ROOT = 0, PROF_NODE = 1, PROF_LEAF = 2, PROF_TRI = 3, PROF_INST = 4, PROF_REGIONS = 5 };
constexpr int kCounterWords = 32;
constexpr int kCensusWords = 8;  // one census block: CNT_* counters (5 used)
struct Prof {
    uint32_t wave[PROF_REGIONS], lane[PROF_REGIONS];
    __device__ __forceinline__ void hit(int r) {
        lane[r] += 1u;
        if (__lane_id() == (uint32_t)__builtin_ctzll(__ballot(1))) wave[r] += 1u;
    }
};

// A lane mask of a boolean: the ballot builtin on the i1 itself.  (HIP's __ballot takes an
// int, so a bool predicate went through a VGPR -- v_cndmask + v_cmp -- before the mask; in the
// traversal's per-iteration loop tests that is two VALU instructions each.)
__device__ __forceinline__ unsigned long long wballot(bool b) { return __builtin_amdgcn_ballot_w64(b); }

// ------------------------------------------------------------------ ray / hit
struct Ray { f3 o, d; };
struct Compact { uint32_t valid, inst, mat, prim; float bu, bv; };
struct Hit { bool valid; float t; Compact s; f3 pos; };

struct PassEps { float det_eps, bary_eps; };

// GetRayAABBIntersectionRange + DoRangesOverlap(RayValidRange, .) (SH/PT_1_InitPass.wgsl:475-514)
// with InvDirection hoisted (it is the same 1/dir for every test of the ray): per axis
// t1 = (min - o) * inv, t2 = (max - o) * inv; tmin = max of the per-axis mins, tmax = min of
// the maxes; an empty range becomes (1, 0); overlap with the closed [vx, vy].
// The slab test for a node's two children at once.  The slab terms (b - o) * inv of both
// children go through packed FP32 (v_pk_add_f32 / v_pk_mul_f32: two IEEE f32 operations per
// lane, rounded exactly as the scalar ones -- no contraction under -ffp-contract=off), the
// min/max reduction per child stays scalar.  Same results as two scalar slab tests.
typedef float v2f __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void box_pair(f3 o, f3 inv, float4 qx, float4 qy, float4 qz, float vx, float vy, bool &hl,
                                         bool &hr, float &tl, float &tr) {
    const v2f ox = {o.x, o.x}, oy = {o.y, o.y}, oz = {o.z, o.z};
    const v2f ix = {inv.x, inv.x}, iy = {inv.y, inv.y}, iz = {inv.z, inv.z};
    const v2f t1x = (v2f{qx.x, qx.y} - ox) * ix, t2x = (v2f{qx.z, qx.w} - ox) * ix;
    const v2f t1y = (v2f{qy.x, qy.y} - oy) * iy, t2y = (v2f{qy.z, qy.w} - oy) * iy;
    const v2f t1z = (v2f{qz.x, qz.y} - oz) * iz, t2z = (v2f{qz.z, qz.w} - oz) * iz;
    const float lmin = fmaxf(fminf(t1x.x, t2x.x), fmaxf(fminf(t1y.x, t2y.x), fminf(t1z.x, t2z.x)));
    const float lmax = fminf(fmaxf(t1x.x, t2x.x), fminf(fmaxf(t1y.x, t2y.x), fmaxf(t1z.x, t2z.x)));
    const float rmin = fmaxf(fminf(t1x.y, t2x.y), fmaxf(fminf(t1y.y, t2y.y), fminf(t1z.y, t2z.y)));
    const float rmax = fminf(fmaxf(t1x.y, t2x.y), fminf(fmaxf(t1y.y, t2y.y), fmaxf(t1z.y, t2z.y)));
    // The reference maps an empty range (min > max) to (1, 0) before the overlap test with
    // [vx, vy]; with vx = 1e-4 > 0 the mapped range never overlaps, so the test is the
    // non-empty check plus the overlap -- same result (NaN terms fail both forms).  tl / tr
    // only order two children that BOTH hit (both non-empty, so never remapped).
    tl = lmin;
    tr = rmin;
    hl = (lmin <= lmax) && (vx <= lmax) && (lmin <= vy);
    hr = (rmin <= rmax) && (vx <= rmax) && (rmin <= vy);
}

// The slab test of a sub-mesh root, each axis's {min, max} slab terms as one packed pair
__device__ __forceinline__ bool box_root(f3 o, f3 inv, const SubRoot &R, float vx, float vy) {
    const v2f t_x = (v2f{R.x[0], R.x[1]} - v2f{o.x, o.x}) * v2f{inv.x, inv.x};
    const v2f t_y = (v2f{R.y[0], R.y[1]} - v2f{o.y, o.y}) * v2f{inv.y, inv.y};
    const v2f t_z = (v2f{R.z[0], R.z[1]} - v2f{o.z, o.z}) * v2f{inv.z, inv.z};
    const float tmin = fmaxf(fminf(t_x.x, t_x.y), fmaxf(fminf(t_y.x, t_y.y), fminf(t_z.x, t_z.y)));
    const float tmax = fminf(fmaxf(t_x.x, t_x.y), fminf(fmaxf(t_y.x, t_y.y), fmaxf(t_z.x, t_z.y)));
    return (tmin <= tmax) && (vx <= tmax) && (tmin <= vy);  // (empty -> (1, 0) never overlaps: box_pair)
}

// The root pre-filter of one chunk of nc <= 32 sub-mesh roots: bit k is set when root k
// passes at the bound vy.  (Two roots per iteration, both LDS reads in flight before either
// test, measured +-0: DESIGN 4.1e.)
template <bool PROF>
__device__ __forceinline__ uint32_t root_mask(const SubRoot *rs, uint32_t nc, f3 lo, f3 inv, float vx, float vy,
                                              Prof &pf) {
    uint32_t mask = 0u;
#pragma unroll 1
    for (uint32_t k = 0; k < nc; ++k) {
        if (PROF) pf.hit(PROF_ROOT);
        if (box_root(lo, inv, rs[k], vx, vy)) mask |= 1u << k;
    }
    return mask;
}

// GetRayTriangleHitDistance (SH/PT_1_InitPass.wgsl:516-547) on the precomputed edges.
__device__ __forceinline__ float ray_tri(f3 o, f3 d, float4 a, float4 b, float4 c, float det_eps) {
    f3 p0 = mk(a.x, a.y, a.z);
    f3 e1 = mk(a.w, b.x, b.y);
    f3 e2 = mk(b.z, b.w, c.x);
    f3 pvec = cross(d, e2);
    float det = dot(e1, pvec);
    if (fabsf(det) < det_eps) return 1e11f;
    float inv_det = 1.0f / det;
    f3 tvec = o - p0;
    float u = dot(tvec, pvec) * inv_det;
    if (u < 0.0f || u > 1.0f) return 1e11f;
    f3 qvec = cross(tvec, e1);
    float v = dot(d, qvec) * inv_det;
    if (v < 0.0f || (u + v) > 1.0f) return 1e11f;
    float t = dot(e2, qvec) * inv_det;
    if (t <= 1e-4f) return 1e11f;
    return t;
}

// Reference-layout accessors (cold paths: hit reconstruction and shading).
__device__ __forceinline__ const uint32_t *desc_ptr(const Scene &sc, uint32_t mesh) {
    return sc.S + sc.U[U_OFF_DESC] + STRIDE_DESCRIPTOR * mesh;
}
__device__ __forceinline__ void tri_vertex_ids(const Scene &sc, const uint32_t *desc, uint32_t prim, uint32_t id[3]) {
    const uint32_t *p = sc.G + sc.U[U_OFF_INDEX] + desc[1] + 3u * prim;
    id[0] = p[0]; id[1] = p[1]; id[2] = p[2];
}
__device__ __forceinline__ f3 vtx_pos(const Scene &sc, const uint32_t *desc, uint32_t vid) {
    const uint32_t *p = sc.G + desc[0] + STRIDE_VERTEX * vid;
    return mk(asf(p[0]), asf(p[1]), asf(p[2]));
}
__device__ __forceinline__ f3 vtx_nrm(const Scene &sc, const uint32_t *desc, uint32_t vid) {
    const uint32_t *p = sc.G + desc[0] + STRIDE_VERTEX * vid;
    return mk(asf(p[3]), asf(p[4]), asf(p[5]));
}

// The three vertices (object-space position + normal, the GeometryBuffer's f32 values) of
// triangle `tri` = Inst::tri_base + prim: one 80-byte record instead of the descriptor ->
// index -> vertex chain (GetTriangleWorldSpace, SH/PT_1_InitPass.wgsl:390-407).
struct TriVerts { f3 p[3], n[3]; };
__device__ __forceinline__ TriVerts tri_verts(const Scene &sc, uint32_t tri) {
    const float4 *q = sc.tverts + 5u * (size_t)tri;
    const float4 a = q[0], b = q[1], c = q[2], d = q[3], e = q[4];
    TriVerts t;
    t.p[0] = mk(a.x, a.y, a.z); t.n[0] = mk(a.w, b.x, b.y);
    t.p[1] = mk(b.z, b.w, c.x); t.n[1] = mk(c.y, c.z, c.w);
    t.p[2] = mk(d.x, d.y, d.z); t.n[2] = mk(d.w, e.x, e.y);
    return t;
}

// GetBaryCentricWeights (SH/PT_1_InitPass.wgsl:549-575): returns (w,u) = bary.xy
__device__ __forceinline__ void barycentric(f3 P, f3 A, f3 B, f3 C, float eps, float &bx, float &by) {
    f3 v0 = B - A, v1 = C - A, v2 = P - A;
    float d00 = dot(v0, v0), d01 = dot(v0, v1), d11 = dot(v1, v1);
    float d20 = dot(v2, v0), d21 = dot(v2, v1);
    float denom = d00 * d11 - d01 * d01;
    if (fabsf(denom) < eps) { bx = 1.0f; by = 0.0f; return; }
    float inv = 1.0f / denom;
    float u = (d11 * d20 - d01 * d21) * inv;
    float v = (d00 * d21 - d01 * d20) * inv;
    bx = 1.0f - u - v;
    by = u;
}

// Barycentrics and world position of a closest hit whose inst/prim/t are set.
// (`insts`: the instance table, or the trace kernel's LDS copy of it)
__device__ __forceinline__ void complete_hit(const Scene &sc, const Ray &ray, PassEps eps, Hit &best,
                                             const Inst *insts = nullptr) {
    best.s.valid = 1u;
    const Inst &I = (insts ? insts : sc.insts)[best.s.inst];
    const TriVerts tv = tri_verts(sc, I.tri_base + best.s.prim);
    f3 A = xform_point(I.m, tv.p[0]);
    f3 B = xform_point(I.m, tv.p[1]);
    f3 C = xform_point(I.m, tv.p[2]);
    f3 P = ray.o + ray.d * best.t;
    barycentric(P, A, B, C, eps.bary_eps, best.s.bu, best.s.bv);
    const float U = best.s.bu, V = best.s.bv, W = 1.0f - U - V;
    best.pos = (A * U + B * V) + C * W;
}
// Instance cull (not in the reference, which transforms every ray into every instance and tests
// every sub-mesh root, SH/PT_1_InitPass.wgsl:613-624): may this ray (world origin o, reciprocal
// direction winv) reach a root of instance I within [0, vy]?  The test is conservative: a ray
// whose local-space root test passes (the point lo + t ld, lo = M^-1 o, ld = M^-1 (o + d) - lo,
// lies in a root box for some t in [vx, vy]) runs within the f32 rounding of the transform -- a
// relative 1e-7 of the coordinates -- of the world box the host maps the local union box to,
// and the box is padded by 1e-5 of the coordinates' magnitude (>= 40x that rounding) plus
// 2^-12 * max|o| for the ray origin's own rounding, so such a ray always passes here.  A NaN bound
// (an idle lane) never passes, as no root test would.  The counting build checks the claim on
// every query it traces (CNT_CULL_MISS: a culled lane whose root pre-filter passed) without
// culling; the other builds skip an instance when no lane of the wave may reach it.
constexpr int CNT_CULL_MISS = 5;
// every build: pixels of a moved camera's temporal pass whose reprojection fell past the rows of
// the previous frame the band holds (its motion halo; ReuseArgs::prev_row_lo / hi) -- such a
// pixel gets no history, where the whole image would have had it (0 keeps bands bit-identical)
constexpr int CNT_MOTION_CLIP = 6;
__device__ __forceinline__ bool inst_may_hit(const Inst &I, f3 o, f3 winv, float omax, float vy) {
    if (!(I.wpad >= 0.0f)) return true;
    const float p = I.wpad + I.wscale * omax;
    const float t0x = ((I.wlo[0] - p) - o.x) * winv.x, t1x = ((I.whi[0] + p) - o.x) * winv.x;
    const float t0y = ((I.wlo[1] - p) - o.y) * winv.y, t1y = ((I.whi[1] + p) - o.y) * winv.y;
    const float t0z = ((I.wlo[2] - p) - o.z) * winv.z, t1z = ((I.whi[2] + p) - o.z) * winv.z;
    const float tmin = fmaxf(fmaxf(fminf(t0x, t1x), fminf(t0y, t1y)), fminf(t0z, t1z));
    const float tmax = fminf(fminf(fmaxf(t0x, t1x), fmaxf(t0y, t1y)), fmaxf(t0z, t1z));
    return tmin <= tmax && tmax >= 0.0f && tmin <= vy + fabsf(vy) * 0x1p-10f + 1e-3f;
}
#ifndef PTX_INST_CULL
#define PTX_INST_CULL 1
#endif
#ifndef PTX_EARLY_LEAF_K  // trace_core_flat's early leaf phase (0 = off)
#define PTX_EARLY_LEAF_K 16
#endif
#ifndef PTX_EARLY_LEAF_L
#define PTX_EARLY_LEAF_L 4
#endif
#ifndef PTX_EARLY_LEAF_TAB  // the same in trace_core_tab (scenes of < 3 instances, G-buffer, PT_4)
#define PTX_EARLY_LEAF_TAB 1
#endif
#ifndef PTX_EARLY_LEAF_TAB_K
#define PTX_EARLY_LEAF_TAB_K PTX_EARLY_LEAF_K
#endif
#ifndef PTX_EARLY_LEAF_TAB_L
#define PTX_EARLY_LEAF_TAB_L PTX_EARLY_LEAF_L
#endif
#ifndef PTX_EARLY_REFILL_K  // trace_core_flat's early exit from the refill loop (0 = off; K = 4 / 8 / 16 measured -0.5 to -1 %)
#define PTX_EARLY_REFILL_K 0
#endif

// TraceRay (SH/PT_1_InitPass.wgsl:605-715; PT_01:509-621): closest hit over every
// instance and sub-mesh root, ordered-stack BLAS traversal, ties replace (`if (best < t)
// continue`).  `stack` is this thread's column of the workgroup's LDS stack
// (entry k at stack[k * stride]).  Also returns the hit position exactly as
// GetSurface(hit).Position computes it (same world-space vertices and barycentrics).
// `subs` / `insts` are the scene's sub-root and instance tables, or LDS copies of them.
// ROOTQ: sub-mesh roots of an instance go through one per-lane root queue (incoherent
// secondary rays); otherwise one root at a time for the whole wave (coherent primary rays,
// whose lanes mostly enter the same roots).  Same per-lane order and results either way.
// ANY (occlusion queries): stop at the first accepted hit, position not reconstructed.
// Until that hit the visit order -- and the bound t_max -- are the closest-hit walk's, so
// "some hit with t <= t_max" comes out exactly when the closest hit has t <= t_max.
// COOP (`coop` = this wave's LDS scratch, used when the whole wave entered): the leaves the
// lanes hold after a node phase are tested by the whole wave -- their triangles are dealt
// out 64 at a time, each lane testing one (lane, triangle) pair with the owning lane's ray
// and bound.  A leaf's sequential loop (`if (best < t) continue`: ties replace) ends with the
// minimum accepted t and the LAST triangle reaching it, which is exactly a min over the key
// (t bits, ~triangle index) -- t > 0, so its bits order like the floats -- taken with an LDS atomic per
// owner.  Every lane's own walk (pops, pushes, bound, counts) is unchanged; a NaN t (which
// the sequential loop accepts and then poisons the bound with) sends the phase through the
// sequential loop instead.  Cross-lane data moves only through shuffles and LDS atomics
// (atomic loads / stores for the keys: plain accesses would let the compiler assume no
// other lane writes them).
struct CoopLds { unsigned long long *key; uint32_t *mark; };  // 64 entries of each per wave
// Inclusive prefix sum over the 64 lanes of the wave (every lane active) in six DPP adds: a
// Hillis-Steele scan inside each row of 16 lanes (row_shr 1, 2, 4, 8; lanes shifted in from
// outside the row add 0), then row 15's sum broadcast into rows 1 and 3 and row 31's into
// rows 2 and 3 (row_bcast).  No LDS round trips (__shfl_up is a ds_bpermute each step).
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
    uint32_t t = v;
    t += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)t, 0x111, 0xf, 0xf, false);  // row_shr:1
    t += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)t, 0x112, 0xf, 0xf, false);  // row_shr:2
    t += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)t, 0x114, 0xf, 0xf, false);  // row_shr:4
    t += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)t, 0x118, 0xf, 0xf, false);  // row_shr:8
    t += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)t, 0x142, 0xa, 0xf, false);  // row_bcast:15
    t += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)t, 0x143, 0xc, 0xf, false);  // row_bcast:31
    return t;
}
// Inclusive prefix maximum over the wave, the same six DPP steps (lanes shifted in add 0).
__device__ __forceinline__ uint32_t wave_incl_max(uint32_t v) {
    uint32_t t = v;
    t = max(t, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)t, 0x111, 0xf, 0xf, false));
    t = max(t, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)t, 0x112, 0xf, 0xf, false));
    t = max(t, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)t, 0x114, 0xf, 0xf, false));
    t = max(t, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)t, 0x118, 0xf, 0xf, false));
    t = max(t, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)t, 0x142, 0xa, 0xf, false));
    t = max(t, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)t, 0x143, 0xc, 0xf, false));
    return t;
}
__device__ __forceinline__ uint32_t wave_excl_sum(uint32_t v, uint32_t &total) {
    const uint32_t incl = wave_incl_scan(v);
    total = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
    return incl - v;
}
// A deal over the wave: lane l holds work items [excl, excl + cnt) of `total` (excl =
// wave_excl_sum(cnt)), dealt out 64 at a time.  The owner of item c0 + lane = the last lane
// with cnt != 0 whose excl <= c0 + lane: each such lane whose range starts inside the chunk
// marks its start position (lane + 1; starts are distinct and ascend with the lane), position
// 0 also takes the last owner that started before the chunk, and a prefix maximum over the
// positions carries every mark forward.  Called by every lane; -1 past the last item.
__device__ __forceinline__ int deal_owner(CoopLds coop, uint32_t lane, uint32_t cnt, uint32_t excl, uint32_t c0) {
    __hip_atomic_store(&coop.mark[lane], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    if (cnt != 0u && excl >= c0 && excl - c0 < 64u)
        __hip_atomic_store(&coop.mark[excl - c0], lane + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    uint32_t m = __hip_atomic_load(&coop.mark[lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    const unsigned long long before = wballot(cnt != 0u && excl < c0);
    if (lane == 0u && before != 0ull) m = max(m, 64u - (uint32_t)__builtin_clzll(before));
    return (int)wave_incl_max(m) - 1;
}
// UNI: `subs` is the workgroup's LDS copy of the root table (like `stack`): pops and root takes
// share one code path (fewer exec-mask branches per node-loop iteration; same per-lane sequence).
template <bool COUNT, bool PROF = false, bool ROOTQ = true, bool ANY = false, bool COOP = false, bool UNI = false>
__device__ __forceinline__ Hit trace_core_tab(const Scene &sc, const SubRoot *subs, const Inst *insts, Ray ray,
                                              PassEps eps, uint32_t *stack, uint32_t stride, float t_max = 1e10f,
                                              CoopLds coop = CoopLds{nullptr}, bool want_pos = true) {
    Prof pf{};
    Hit best;
    best.valid = false;
    best.t = 0.0f;
    best.s = Compact{0u, 0u, 0u, 0u, 0.0f, 0.0f};
    best.pos = mk(0.0f, 0.0f, 0.0f);
    const float vx = 1e-4f;
    float vy = t_max;  // 1e10 in the reference; a smaller bound only prunes hits beyond it
    uint32_t n_aabb = 0, n_tri = 0;
    bool stop = false;
    const bool wave_coop = COOP && __ballot(1) == ~0ull;  // wave-uniform
    // instance cull inputs (inst_may_hit): a ray with a non-finite component is never culled
    const bool rfin = finite3(ray.o) && finite3(ray.d);
    const f3 winv = mk(__builtin_amdgcn_rcpf(ray.d.x), __builtin_amdgcn_rcpf(ray.d.y), __builtin_amdgcn_rcpf(ray.d.z));
    const float omax = fmaxf(fmaxf(fabsf(ray.o.x), fabsf(ray.o.y)), fabsf(ray.o.z));
    // (with COOP an occluded lane keeps iterating, without work, so the wave stays whole)
    for (uint32_t ii = 0; ii < sc.n_inst && (COOP || !stop); ++ii) {
        const Inst &I = insts[ii];
        const bool may = !PTX_INST_CULL || !rfin || inst_may_hit(I, ray.o, winv, omax, vy);
        if (PTX_INST_CULL && !COUNT && wballot(may) == 0ull) continue;  // (wave-uniform)
        if (PROF) pf.hit(PROF_INST);
        // TransformRayWithMat4x4(InRay, M^-1, false), SH/PT_1_InitPass.wgsl:486-496
        // (the identity shortcut of inst_point is not used here: at the trace kernel's 128-VGPR
        // budget its extra live values spill, +3.4 % on trace_queue)
        f3 lo = xform_point(I.minv, ray.o);
        f3 le = xform_point(I.minv, ray.o + ray.d);
        f3 ld = le - lo;
        f3 inv = mk(1.0f / ld.x, 1.0f / ld.y, 1.0f / ld.z);
        const uint32_t nsub = I.nsub;
        const SubRoot *roots = subs + I.sub_base;
        const float4 *tris = sc.tris + 3u * I.tri_base;
        n_aabb += nsub;  // the reference tests every sub-mesh root once
        for (uint32_t s0 = 0; s0 < nsub && (COOP || !stop); s0 += 32u) {
            const uint32_t nc = nsub - s0 < 32u ? nsub - s0 : 32u;
            // Coherent pre-filter: every root against the best t at this point.  The
            // reference tests root s against the best t after roots < s (never larger), so
            // this keeps every root it enters; the exact test is repeated when the root is
            // taken below, with the then-current best -- the reference's own test.
#pragma unroll 1
            for (uint32_t kk = 0; kk < (ROOTQ ? 1u : nc) && (COOP || !stop); ++kk) {
            uint32_t mask = 0u;
            if (stop) {
                // occluded (ANY): nothing more to test
            } else if (ROOTQ) {
                mask = root_mask<PROF>(roots + s0, nc, lo, inv, vx, vy, pf);
                if (COUNT && PTX_INST_CULL && !may && mask != 0u && t_max == t_max)
                    atomicAdd(&sc.counters[CNT_CULL_MISS], 1ull);
            } else {
                if (PROF) pf.hit(PROF_ROOT);
                if (box_root(lo, inv, roots[s0 + kk], vx, vy)) mask = 1u << kk;
            }
            // while-while traversal over all of this lane's roots: lanes descend interior
            // nodes (taking their next root, in index order, when the stack runs dry) until
            // each has a leaf or nothing left, then the wave tests leaves together.  Per lane
            // the root tests, pops, tests and pushes happen in exactly the reference's order
            // (SH/PT_1_InitPass.wgsl:605-715), so hits, ties and work counts are unchanged.
            int sp = -1;
            uint32_t grp = 0u, leaf = 0u;
            // the pre-filter's bound: while no hit has shrunk vy since, its result for a root
            // IS the reference's test of that root (same function, same arguments)
            const float vy_pf = vy;
            for (;;) {
                // One wave-uniform loop; per iteration a lane with an empty stack takes its next
                // root and a lane with a stack pops -- and a root that passes its test IS the
                // lane's next node (its push + pop folded), tested in the same iteration.  Per
                // lane the root tests, pops, tests and pushes are the reference's sequence.
                for (;;) {
                    const bool want = leaf == 0u && (sp >= 0 || mask != 0u);
                    const unsigned long long wm = wballot(want);
                    if (wm == 0ull) break;
                    // early leaf phase (as trace_core_flat; only where the cooperative phase runs)
                    if constexpr (PTX_EARLY_LEAF_K > 0 && PTX_EARLY_LEAF_TAB && COOP) {
                        if (wave_coop && __builtin_popcountll(wm) <= PTX_EARLY_LEAF_TAB_K &&
                            __builtin_popcountll(wballot(leaf != 0u)) >= PTX_EARLY_LEAF_TAB_L)
                            break;
                    }
                    if (PROF && want) pf.hit(PROF_NODE);
                    uint32_t ref = 0u;
                    bool node = false;
                    if (UNI) {
                        // One path for a pop and a root take (`subs` and the stack both in LDS):
                        // the next reference is read from the stack top, or -- with an empty stack
                        // -- from the next queued root's record, through one selected LDS address.
                        // A root is re-tested only when a hit has moved the bound since the
                        // pre-filter (else the pre-filter's result is the reference's test).
                        // (predicated: lanes without work read a valid slot and keep their state)
                        const bool from_root = sp < 0;
                        const uint32_t k = (from_root && mask != 0u) ? (uint32_t)__builtin_ctz(mask) : 0u;
                        const uint32_t *src = from_root ? &roots[s0 + k].ref : &stack[(uint32_t)(from_root ? 0 : sp) * stride];
                        ref = *src;
                        const bool tk_root = want && from_root;
                        bool take = want;
                        if (tk_root && !(ROOTQ && vy == vy_pf)) take = box_root(lo, inv, roots[s0 + k], vx, vy);
                        mask = tk_root ? (mask & (mask - 1u)) : mask;
                        sp = (want && !from_root) ? sp - 1 : sp;
                        grp = (tk_root && take) ? s0 + k : grp;
                        const bool is_leaf = (ref & LEAF_BIT) != 0u;
                        leaf = (take && is_leaf) ? ref : leaf;
                        node = take && !is_leaf;
                    } else if (leaf == 0u && sp < 0 && mask != 0u) {
                        const uint32_t k = (uint32_t)__builtin_ctz(mask);
                        mask &= mask - 1u;
                        const SubRoot &R = roots[s0 + k];
                        if ((ROOTQ && vy == vy_pf) || box_root(lo, inv, R, vx, vy)) {
                            grp = s0 + k;
                            if (R.ref & LEAF_BIT) leaf = R.ref;  // a one-leaf root
                            else { ref = R.ref; node = true; }
                        }
                    } else if (leaf == 0u && sp >= 0) {
                        ref = stack[(uint32_t)sp * stride];
                        --sp;
                        if (ref & LEAF_BIT) leaf = ref;
                        else node = true;
                    }
                    if (!node) continue;
                    const float4 *np = reinterpret_cast<const float4 *>(sc.nodes + ref);
                    float4 q0 = np[0], q1 = np[1], q2 = np[2], q3 = np[3];
                    uint32_t lref = __float_as_uint(q3.x), rref = __float_as_uint(q3.y);
                    float tl, tr;
                    bool hl, hr;
                    box_pair(lo, inv, q0, q1, q2, vx, vy, hl, hr, tl, tr);
                    n_aabb += 2;
                    // branch-free pushes: both entries are written, the stack pointer moves by
                    // the number of hits (entries above the top are never read; the slots are
                    // the two-hit case's, within the max_depth + 2 entries per lane)
                    const bool both = hl && hr;
                    const uint32_t near = tl < tr ? lref : rref, far = tl < tr ? rref : lref;
                    stack[(uint32_t)(sp + 1) * stride] = both ? far : (hl ? lref : rref);
                    stack[(uint32_t)(sp + 2) * stride] = near;
                    sp += both ? 2 : ((hl || hr) ? 1 : 0);
                }
                // (the whole wave must be here: after a NaN fallback lanes leave one by one)
                if (wave_coop && __ballot(1) == ~0ull) {  // a wave-uniform leaf phase
                    if (wballot(leaf != 0u) == 0ull) break;
                    if (PROF) pf.hit(PROF_LEAF);
                    const uint32_t lane = __lane_id();
                    const uint32_t cnt = leaf ? (leaf >> 24) & 0x7Fu : 0u, lfirst = leaf & LEAF_FIRST_MASK;
                    uint32_t total;
                    const uint32_t excl = wave_excl_sum(cnt, total);
                    __hip_atomic_store(&coop.key[lane], ~0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
                    __atomic_signal_fence(__ATOMIC_SEQ_CST);  // (compiler order; one wave's LDS ops run in order)
                    bool nan_seen = false;
                    for (uint32_t c0 = 0; c0 < total; c0 += 64u) {
                        const uint32_t u = c0 + lane;
                        // owner of triangle u = the last lane with a nonempty leaf whose
                        // exclusive count is <= u: each such lane whose leaf starts inside this
                        // chunk marks its start position (lane + 1; starts are distinct and
                        // ascend with the lane), position 0 also takes the last owner that
                        // started before the chunk, and a prefix maximum over the positions
                        // carries every mark forward
                        __hip_atomic_store(&coop.mark[lane], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
                        __atomic_signal_fence(__ATOMIC_SEQ_CST);
                        if (cnt != 0u && excl >= c0 && excl - c0 < 64u)
                            __hip_atomic_store(&coop.mark[excl - c0], lane + 1u, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_WAVEFRONT);
                        __atomic_signal_fence(__ATOMIC_SEQ_CST);
                        uint32_t m = __hip_atomic_load(&coop.mark[lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
                        const unsigned long long before = wballot(cnt != 0u && excl < c0);
                        if (lane == 0u && before != 0ull) m = max(m, 64u - (uint32_t)__builtin_clzll(before));
                        const int owner = (int)wave_incl_max(m) - 1;
                        // triangle u of the deal is the owner's leaf triangle lfirst + (u - excl)
                        const uint32_t tri = u + __shfl(lfirst - excl, owner);
                        const f3 olo = mk(__shfl(lo.x, owner), __shfl(lo.y, owner), __shfl(lo.z, owner));
                        const f3 old = mk(__shfl(ld.x, owner), __shfl(ld.y, owner), __shfl(ld.z, owner));
                        const float ovy = __shfl(vy, owner);
                        if (u < total) {
                            if (PROF) pf.hit(PROF_TRI);
                            const float4 *tp = tris + 3u * tri;
                            const float t = ray_tri(olo, old, tp[0], tp[1], tp[2], eps.det_eps);
                            if (t != t) nan_seen = true;
                            else if (!(ovy < t))
                                atomicMin(&coop.key[owner], ((unsigned long long)__float_as_uint(t) << 32) |
                                                                (unsigned long long)(0xffffffffu - tri));
                        }
                    }
                    __atomic_signal_fence(__ATOMIC_SEQ_CST);
                    if (wballot(nan_seen) == 0ull) {
                        if (leaf) {
                            const unsigned long long key =
                                __hip_atomic_load(&coop.key[lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
                            n_tri += cnt;
                            if (key != ~0ull) {
                                vy = __uint_as_float((uint32_t)(key >> 32));
                                best.valid = true;
                                best.s.inst = ii;
                                best.s.mat = grp;
                                best.s.prim = 0xffffffffu - (uint32_t)key;
                                if (ANY) {  // occluded: no more work for this lane
                                    stop = true;
                                    sp = -1;
                                    mask = 0u;
                                }
                            }
                            leaf = 0u;
                        }
                        continue;
                    }
                }
                if (leaf == 0u) {  // roots and stack exhausted -- or still descending after an
                    if (sp >= 0 || mask != 0u) continue;  // early leaf phase that saw a NaN t
                    break;
                }
                if (PROF && !wave_coop) pf.hit(PROF_LEAF);
                const uint32_t first = leaf & LEAF_FIRST_MASK;
                const uint32_t count = (leaf >> 24) & 0x7Fu;
                leaf = 0u;
                const float4 *tp = tris + 3u * first;
                for (uint32_t k = 0; k < count; ++k) {
                    if (PROF) pf.hit(PROF_TRI);
                    float4 a = tp[3u * k + 0u], b = tp[3u * k + 1u], c = tp[3u * k + 2u];
                    float t = ray_tri(lo, ld, a, b, c, eps.det_eps);
                    ++n_tri;
                    if (vy < t) continue;
                    vy = t;
                    best.valid = true;
                    best.s.inst = ii;
                    best.s.mat = grp;
                    best.s.prim = first + k;
                    if (ANY) break;
                }
                if (ANY && best.valid) {  // occluded: drop the rest of the walk
                    stop = true;
                    break;
                }
            }
            }  // roots (ROOTQ: one queue per chunk of 32; else one root at a time)
        }
    }
    const bool counted = t_max == t_max;  // a NaN bound: an idle lane keeping its wave whole
    if (PROF && counted) {
        for (int r = 0; r < PROF_REGIONS; ++r) {
            if (pf.wave[r]) atomicAdd(&sc.counters[8 + 2 * r], (unsigned long long)pf.wave[r]);
            if (pf.lane[r]) atomicAdd(&sc.counters[9 + 2 * r], (unsigned long long)pf.lane[r]);
        }
    }
    if (COUNT && counted) {
        atomicAdd(&sc.counters[CNT_RAYS], 1ull);
        atomicAdd(&sc.counters[CNT_INST], (unsigned long long)sc.n_inst);
        atomicAdd(&sc.counters[CNT_AABB], (unsigned long long)n_aabb);
        atomicAdd(&sc.counters[CNT_TRI], (unsigned long long)n_tri);
        if (best.valid) atomicAdd(&sc.counters[CNT_HITS], 1ull);
    }
    if (best.valid) {
        best.t = vy;
        if (!ANY && want_pos) complete_hit(sc, ray, eps, best, insts);
    }
    return best;
}
// The same walk with the instance loop flattened into the lanes (trace_queue's form: whole-wave
// calls, root and instance tables in LDS).  Each lane keeps its own place in the instance list:
// a lane whose roots and stack of one instance are exhausted moves on to the next instance its
// ray may reach (inst_may_hit) at the next refill -- after the current leaf phase -- instead of
// idling until every lane of the wave has finished that instance; lanes in different instances
// share the node loop and the cooperative leaf phases (the owner's triangle base travels with
// its ray).  Per lane the order of instances, roots, pops, node tests, pushes and triangle
// tests is the reference's (SH/PT_1_InitPass.wgsl:605-715), so hits, ties and work counts are
// unchanged; a leaf phase in which a lane computed a NaN t runs its leaves sequentially.
template <bool COUNT, bool PROF = false, bool ANY = false>
__device__ __forceinline__ Hit trace_core_flat(const Scene &sc, const SubRoot *subs, const Inst *insts, Ray ray,
                                               PassEps eps, uint32_t *stack, uint32_t stride, float t_max,
                                               CoopLds coop, bool want_pos, uint32_t *dbg = nullptr) {
    // dbg (diagnostic build, tools/trace_tail.py): wave-level {refill iterations, node-loop
    // iterations, leaf phases, triangle-deal chunks, calls, max slab tests of a lane}
#ifndef PTX_WG_TIMES
    (void)dbg;
#endif
    Prof pf{};
    Hit best;
    best.valid = false;
    best.t = 0.0f;
    best.s = Compact{0u, 0u, 0u, 0u, 0.0f, 0.0f};
    best.pos = mk(0.0f, 0.0f, 0.0f);
    const float vx = 1e-4f;
    float vy = t_max;
    uint32_t n_aabb = 0, n_tri = 0;
    const bool counted = t_max == t_max;  // a NaN bound: an idle lane keeping its wave whole
    const bool rfin = finite3(ray.o) && finite3(ray.d);
    const float omax = fmaxf(fmaxf(fabsf(ray.o.x), fabsf(ray.o.y)), fabsf(ray.o.z));
    uint32_t next = 0u;                       // the next instance to consider
    uint32_t cur = 0u, s0 = 0u, nsub = 0u;    // the instance walked, its root chunk, its root count
    uint32_t sub_base = 0u, tri_base = 0u;
    bool done = !counted;                     // (no box passes a NaN bound: nothing to walk)
    f3 lo = mk(0.0f, 0.0f, 0.0f), ld = lo, inv = lo;
    uint32_t mask = 0u, grp = 0u, leaf = 0u;
    int sp = -1;
    float vy_pf = vy;
    for (;;) {
        // refill: a lane with no leaf, no stack and no queued root takes its instance's next
        // chunk of 32 roots or its next instance (transform + root pre-filter)
        for (uint32_t refills = 0u;; ++refills) {
            const bool need = !done && leaf == 0u && sp < 0 && mask == 0u;
            const unsigned long long nm = wballot(need);
            if (nm == 0ull) break;
            // early exit (PTX_EARLY_REFILL_K > 0): after one refill, when at most K lanes still
            // look for a root that passes, the lanes that have one walk it now and those K go on
            // at the next refill.  Per lane nothing moves; only the interleaving across lanes.
            if constexpr (PTX_EARLY_REFILL_K > 0) {
                if (refills > 0u && __builtin_popcountll(nm) <= PTX_EARLY_REFILL_K &&
                    wballot(leaf != 0u || sp >= 0 || mask != 0u) != 0ull)
                    break;
            }
#ifdef PTX_WG_TIMES
            if (dbg) dbg[0]++;
#endif
            if (need) {
                bool may = true;
                if (s0 + 32u < nsub) {
                    s0 += 32u;
                } else {
                    const f3 winv = mk(__builtin_amdgcn_rcpf(ray.d.x), __builtin_amdgcn_rcpf(ray.d.y),
                                       __builtin_amdgcn_rcpf(ray.d.z));
                    // (COUNT: every instance is walked; the cull is only checked below)
                    while (next < sc.n_inst) {
                        may = !PTX_INST_CULL || !rfin || inst_may_hit(insts[next], ray.o, winv, omax, vy);
                        if (may || COUNT) break;
                        ++next;
                    }
                    if (next >= sc.n_inst) {
                        done = true;
                    } else {
                        cur = next++;
                        const Inst &I = insts[cur];
                        if (PROF) pf.hit(PROF_INST);
                        // TransformRayWithMat4x4(InRay, M^-1, false), SH/PT_1_InitPass.wgsl:486-496
                        lo = xform_point(I.minv, ray.o);
                        const f3 le = xform_point(I.minv, ray.o + ray.d);
                        ld = le - lo;
                        inv = mk(1.0f / ld.x, 1.0f / ld.y, 1.0f / ld.z);
                        sub_base = I.sub_base;
                        nsub = I.nsub;
                        tri_base = I.tri_base;
                        s0 = 0u;
                        n_aabb += nsub;  // the reference tests every sub-mesh root once
                    }
                }
                if (!done && nsub != 0u) {
                    // pre-filter: every root of the chunk against the best t at this point (the
                    // reference tests root s with the best t after roots < s, never larger; the
                    // exact test is repeated when a root is taken, below)
                    const uint32_t nc = nsub - s0 < 32u ? nsub - s0 : 32u;
                    mask |= root_mask<PROF>(subs + (sub_base + s0), nc, lo, inv, vx, vy, pf);
                    vy_pf = vy;
                    if (COUNT && PTX_INST_CULL && !may && mask != 0u) atomicAdd(&sc.counters[CNT_CULL_MISS], 1ull);
                }
            }
        }
        // node loop: pops and root takes through one LDS read (as trace_core_tab UNI)
        for (;;) {
            const bool want = leaf == 0u && (sp >= 0 || mask != 0u);
            const unsigned long long wm = wballot(want);
            if (wm == 0ull) break;
            // early leaf phase (PTX_EARLY_LEAF_K > 0): once at most K lanes still descend and
            // at least L hold a leaf, the holders test their leaves now and the descending lanes
            // go on after it, joined by the holders' next pops.  Per lane nothing moves (its leaf
            // is tested before its next pop either way); only the interleaving across lanes.
            if constexpr (PTX_EARLY_LEAF_K > 0) {
                if (__builtin_popcountll(wm) <= PTX_EARLY_LEAF_K &&
                    __builtin_popcountll(wballot(leaf != 0u)) >= PTX_EARLY_LEAF_L)
                    break;
            }
#ifdef PTX_WG_TIMES
            if (dbg) dbg[1]++;
#endif
            if (PROF && want) pf.hit(PROF_NODE);
            const bool from_root = sp < 0;
            const uint32_t k = (from_root && mask != 0u) ? (uint32_t)__builtin_ctz(mask) : 0u;
            const SubRoot *R = subs + (sub_base + s0 + k);
            const uint32_t *src = from_root ? &R->ref : &stack[(uint32_t)(from_root ? 0 : sp) * stride];
            const uint32_t ref = *src;
            const bool tk_root = want && from_root;
            bool take = want;
            if (tk_root && !(vy == vy_pf)) take = box_root(lo, inv, *R, vx, vy);
            mask = tk_root ? (mask & (mask - 1u)) : mask;
            sp = (want && !from_root) ? sp - 1 : sp;
            grp = (tk_root && take) ? s0 + k : grp;
            const bool is_leaf = (ref & LEAF_BIT) != 0u;
            leaf = (take && is_leaf) ? ref : leaf;
            if (!(take && !is_leaf)) continue;
            const float4 *np = reinterpret_cast<const float4 *>(sc.nodes + ref);
            float4 q0 = np[0], q1 = np[1], q2 = np[2], q3 = np[3];
            uint32_t lref = __float_as_uint(q3.x), rref = __float_as_uint(q3.y);
            float tl, tr;
            bool hl, hr;
            box_pair(lo, inv, q0, q1, q2, vx, vy, hl, hr, tl, tr);
            n_aabb += 2;
            const bool both = hl && hr;
            const uint32_t near = tl < tr ? lref : rref, far = tl < tr ? rref : lref;
            stack[(uint32_t)(sp + 1) * stride] = both ? far : (hl ? lref : rref);
            stack[(uint32_t)(sp + 2) * stride] = near;
            sp += both ? 2 : ((hl || hr) ? 1 : 0);
        }
        const unsigned long long holders = wballot(leaf != 0u);
        if (holders == 0ull) {
            if (wballot(!done) == 0ull) break;  // every lane has walked every instance
            continue;
        }
        // cooperative leaf phase (trace_core_tab COOP), the owner's triangle base included
        if (PROF) pf.hit(PROF_LEAF);
        const uint32_t lane = __lane_id();
        const uint32_t cnt = leaf ? (leaf >> 24) & 0x7Fu : 0u, lfirst = leaf & LEAF_FIRST_MASK;
        uint32_t total;
        const uint32_t excl = wave_excl_sum(cnt, total);
#ifdef PTX_WG_TIMES
        if (dbg) {
            dbg[2]++;
            dbg[3] += (total + 63u) / 64u;
        }
#endif
        __hip_atomic_store(&coop.key[lane], ~0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        __atomic_signal_fence(__ATOMIC_SEQ_CST);
        bool nan_seen = false;
        for (uint32_t c0 = 0; c0 < total; c0 += 64u) {
            const uint32_t u = c0 + lane;
            const int owner = deal_owner(coop, lane, cnt, excl, c0);
            // triangle u of the deal: the owner's leaf triangle lfirst + (u - excl), in its instance
            const uint32_t tri = u + __shfl(lfirst - excl, owner);
            const uint32_t tb = __shfl(tri_base, owner);
            const f3 olo = mk(__shfl(lo.x, owner), __shfl(lo.y, owner), __shfl(lo.z, owner));
            const f3 old = mk(__shfl(ld.x, owner), __shfl(ld.y, owner), __shfl(ld.z, owner));
            const float ovy = __shfl(vy, owner);
            if (u < total) {
                if (PROF) pf.hit(PROF_TRI);
                const float4 *tp = sc.tris + 3u * (tb + tri);
                const float t = ray_tri(olo, old, tp[0], tp[1], tp[2], eps.det_eps);
                if (t != t) nan_seen = true;
                else if (!(ovy < t))
                    atomicMin(&coop.key[owner],
                              ((unsigned long long)__float_as_uint(t) << 32) | (unsigned long long)(0xffffffffu - tri));
            }
        }
        __atomic_signal_fence(__ATOMIC_SEQ_CST);
        if (wballot(nan_seen) == 0ull) {
            if (leaf) {
                const unsigned long long key = __hip_atomic_load(&coop.key[lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
                n_tri += cnt;
                if (key != ~0ull) {
                    vy = __uint_as_float((uint32_t)(key >> 32));
                    best.valid = true;
                    best.s.inst = cur;
                    best.s.mat = grp;
                    best.s.prim = 0xffffffffu - (uint32_t)key;
                }
            }
        } else if (leaf) {  // a NaN t somewhere in the wave: this phase's leaves one by one
            const uint32_t first = leaf & LEAF_FIRST_MASK, count = (leaf >> 24) & 0x7Fu;
            const float4 *tp = sc.tris + 3u * (tri_base + first);
            for (uint32_t k = 0; k < count; ++k) {
                if (PROF) pf.hit(PROF_TRI);
                const float t = ray_tri(lo, ld, tp[3u * k + 0u], tp[3u * k + 1u], tp[3u * k + 2u], eps.det_eps);
                ++n_tri;
                if (vy < t) continue;
                vy = t;
                best.valid = true;
                best.s.inst = cur;
                best.s.mat = grp;
                best.s.prim = first + k;
                if (ANY) break;
            }
        }
        leaf = 0u;
        if (ANY && best.valid && !done) {  // occluded: no more work for this lane
            done = true;
            sp = -1;
            mask = 0u;
        }
    }
    if (PROF && counted) {
        for (int r = 0; r < PROF_REGIONS; ++r) {
            if (pf.wave[r]) atomicAdd(&sc.counters[8 + 2 * r], (unsigned long long)pf.wave[r]);
            if (pf.lane[r]) atomicAdd(&sc.counters[9 + 2 * r], (unsigned long long)pf.lane[r]);
        }
    }
#ifdef PTX_WG_TIMES
    if (dbg) {
        dbg[4]++;
        uint32_t m = counted ? n_aabb : 0u;
        for (int o = 32; o >= 1; o >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, o));
        dbg[5] = max(dbg[5], m);
    }
    if (sc.wgt && counted && n_aabb >= kStragglerAabb) {
        const unsigned long long i = atomicAdd(sc.wgt, 2ull);
        if (i + 1u < (1ull << 20)) {
            unsigned long long *r = sc.wgt + 4u + 4u * i;
            r[0] = pk2(ray.o.x, ray.o.y);
            r[1] = pk2(ray.o.z, ray.d.x);
            r[2] = ((unsigned long long)KID_STRAGGLER << 32) | n_aabb;
            r[3] = (unsigned long long)n_tri | ((unsigned long long)__float_as_uint(t_max) << 32);
            r[4] = pk2(ray.d.y, ray.d.z);
            r[5] = (unsigned long long)__float_as_uint(best.valid ? vy : -1.0f) | ((unsigned long long)best.s.inst << 32);
            r[6] = ((unsigned long long)KID_STRAGGLER2 << 32) | best.s.prim;
            r[7] = best.s.mat;
        }
    }
#endif
    if ((COUNT || PROF) && counted) {  // (PROF alone: the culled walk's executed tests)
        atomicAdd(&sc.counters[CNT_RAYS], 1ull);
        atomicAdd(&sc.counters[CNT_INST], (unsigned long long)sc.n_inst);
        atomicAdd(&sc.counters[CNT_AABB], (unsigned long long)n_aabb);
        atomicAdd(&sc.counters[CNT_TRI], (unsigned long long)n_tri);
        if (best.valid) atomicAdd(&sc.counters[CNT_HITS], 1ull);
    }
    if (best.valid) {
        best.t = vy;
        if (!ANY && want_pos) complete_hit(sc, ray, eps, best, insts);
    }
    return best;
}

// Sub-root and instance tables staged in LDS when they fit: every ray tests every root of
// every instance, ~16 table reads per query otherwise paid as scalar-load round trips.  The
// tables sit at the start of the kernel's dynamic LDS, sized to the scene (32 B per sub-mesh
// root, 144 B per instance) up to kLdsTableMax: ~700 sub-meshes, or 100 furnished instances
// of a few sub-meshes each.  Larger scenes read the global tables.
constexpr uint32_t kLdsTableMax = 24576u;
__host__ __device__ __forceinline__ uint32_t tables_lds_bytes(const Scene &sc) {
    return ((sc.n_subs * (uint32_t)sizeof(SubRoot) + 15u) & ~15u) + sc.n_inst * (uint32_t)sizeof(Inst);
}
__host__ __device__ __forceinline__ bool tables_fit_lds(const Scene &sc) { return tables_lds_bytes(sc) <= kLdsTableMax; }
struct LdsTables { const SubRoot *subs; const Inst *insts; };
// Copies the tables to `lds` (16-byte aligned dynamic LDS); called by every thread of the
// workgroup (ends with a barrier).  Returns the LDS tables.
__device__ __forceinline__ LdsTables stage_tables(const Scene &sc, uint32_t *lds) {
    SubRoot *l_subs = reinterpret_cast<SubRoot *>(lds);
    Inst *l_insts = reinterpret_cast<Inst *>(lds + ((sc.n_subs * (uint32_t)sizeof(SubRoot) + 15u) & ~15u) / 4u);
    const uint32_t *gs = reinterpret_cast<const uint32_t *>(sc.subs);
    uint32_t *ls = reinterpret_cast<uint32_t *>(l_subs);
    for (uint32_t i = threadIdx.x; i < sc.n_subs * (uint32_t)(sizeof(SubRoot) / 4u); i += blockDim.x) ls[i] = gs[i];
    const uint32_t *gi = reinterpret_cast<const uint32_t *>(sc.insts);
    uint32_t *li = reinterpret_cast<uint32_t *>(l_insts);
    for (uint32_t i = threadIdx.x; i < sc.n_inst * (uint32_t)(sizeof(Inst) / 4u); i += blockDim.x) li[i] = gi[i];
    __syncthreads();
    return LdsTables{l_subs, l_insts};
}

template <bool COUNT, bool PROF = false>
__device__ __forceinline__ Hit trace_core(const Scene &sc, Ray ray, PassEps eps, uint32_t *stack, uint32_t stride,
                                          float t_max = 1e10f) {
    return trace_core_tab<COUNT, PROF>(sc, sc.subs, sc.insts, ray, eps, stack, stride, t_max);
}
template <bool COUNT>
__device__ __attribute__((noinline)) Hit trace_ray(const Scene &sc, Ray ray, PassEps eps, uint32_t *stack,
                                                  uint32_t stride) {
    return trace_core<COUNT>(sc, ray, eps, stack, stride);
}

}  // namespace ptx
