// ptx_persist.hip -- persistent-lane versions of the secondary passes (the fast path).
//
// Same per-pixel semantics as ptx_kernels.hip (SH/PT_1_InitPass.wgsl:1361-1486,
// SH/PT_4_FinalShadingPass.wgsl:1392-1428, SH/TEST_MCPT.wgsl:1315-1372), restructured
// for CDNA4:
//   * each pass is a per-pixel state machine with ONE inlined TraceRay site, so the
//     64 lanes of a wave always traverse together (NEE shadow segments, BSDF rays and
//     Visibility restarts of different pixels share the same trace call) and no call
//     ABI spills to scratch;
//   * lanes are persistent: when a lane's pixel finishes it pulls the next pixel from a
//     global counter (one wave-aggregated atomic per refill), so short paths do not idle
//     the wave while long ones finish (path regeneration);
//   * pixels are handed out in 8x8 tile order, so a freshly filled wave traces a
//     coherent tile.
// Results are per-pixel functions of (pixel, uniform, scene) only, hence identical to
// the straightforward kernels whatever lane or wave processes a pixel.
#include "ptx_launch.h"
#include "ptx_shading.h"

namespace ptx {

constexpr uint32_t PBLOCK = kBlock;
extern __shared__ uint32_t lds_pstack[];

struct PixelQueue {
    uint32_t tiles_x, n;  // n = padded pixel count (whole 8x8 tiles of the band)
};
__device__ __forceinline__ PixelQueue make_queue(const Scene &sc) {
    PixelQueue q;
    q.tiles_x = (sc.width + 7u) / 8u;
    q.n = q.tiles_x * ((sc.row_end - sc.row_begin + 7u) / 8u) * 64u;
    return q;
}
__device__ __forceinline__ bool pixel_at(const Scene &sc, const PixelQueue &q, uint32_t p, uint32_t &x, uint32_t &y) {
    const uint32_t t = p >> 6, l = p & 63u;
    x = (t % q.tiles_x) * 8u + (l & 7u);
    y = sc.row_begin + (t / q.tiles_x) * 8u + (l >> 3);
    return x < sc.width && y < sc.row_end;
}
// Wave-aggregated dequeue: lanes with `need` get consecutive indices from *counter.
__device__ __forceinline__ uint32_t dequeue(unsigned int *counter, bool need) {
    const unsigned long long mask = __ballot(need);
    if (mask == 0ull) return 0xffffffffu;
    const uint32_t lane = __lane_id();
    const uint32_t leader = (uint32_t)__ffsll((long long)mask) - 1u;
    uint32_t base = 0u;
    if (lane == leader) base = atomicAdd(counter, (unsigned int)__popcll(mask));
    base = __shfl(base, (int)leader);
    const uint32_t rank = (uint32_t)__popcll(mask & ((1ull << lane) - 1ull));
    return need ? base + rank : 0xffffffffu;
}

__device__ __forceinline__ f3 get_x0p(const Scene &sc, uint32_t x, uint32_t y) {  // Get_X0, PT_1:732-738
    const float *vpinv = reinterpret_cast<const float *>(sc.U + U_VPINV);
    float u = ((float)x + 0.5f) / (float)sc.U[U_W];
    float v = ((float)y + 0.5f) / (float)sc.U[U_H];
    return xform_point(vpinv, mk(2.0f * u - 1.0f, 2.0f * v - 1.0f, 0.0f));
}
__device__ __forceinline__ Ray camera_rayp(const Scene &sc, uint32_t x, uint32_t y) {  // PT_01:496-507
    const float *vpinv = reinterpret_cast<const float *>(sc.U + U_VPINV);
    float u = ((float)x + 0.5f) / (float)sc.U[U_W];
    float v = ((float)y + 0.5f) / (float)sc.U[U_H];
    f3 start = xform_point(vpinv, mk(2.0f * u - 1.0f, 2.0f * v - 1.0f, 0.0f));
    f3 end = xform_point(vpinv, mk(2.0f * u - 1.0f, 2.0f * v - 1.0f, 0.0f + 1.0f));
    return Ray{start, normalize(end - start)};
}
__device__ __forceinline__ Compact decode_g(uint4 g) {
    return Compact{(g.x & 0x80000000u) ? 1u : 0u, (g.x & 0x7fff0000u) >> 16, g.x & 0xffffu, g.y, asf(g.z), asf(g.w)};
}
__device__ __forceinline__ uint4 encode_g(const Compact &s) {
    return make_uint4((s.valid << 31) | (s.inst << 16) | s.mat, s.prim, asu(s.bu), asu(s.bv));
}
__device__ __forceinline__ void write_colorp(const Scene &sc, float4 *accum, size_t i, f3 c) {
    float t = 1.0f / (float)(sc.U[U_FRAME] + 1u);  // WriteColor, PT_4:599-606
    float4 a = accum[i];
    accum[i] = make_float4(mixf(a.x, c.x, t), mixf(a.y, c.y, t), mixf(a.z, c.z, t), 1.0f);
}
// Visibility state (SH/PT_1_InitPass.wgsl:774-802) shared by every pass.
struct Vis {
    f3 org, dir;
    float T, remain;
    uint32_t iter;
};
__device__ __forceinline__ void vis_begin(Vis &v, f3 start, f3 end) {
    v.T = 1.0f;
    float dist = length(end - start);
    v.dir = (end - start) / dist;
    v.org = start;
    v.remain = dist;
    v.iter = 0u;
}
// Consume one closest hit: returns true when the Visibility result is known (in *out).
__device__ __forceinline__ bool vis_step(const Scene &sc, Vis &v, const Hit &h, float &out) {
    if (!h.valid || h.t > v.remain) { out = v.T; return true; }
    float tr = get_transmission(sc, h.s.inst, h.s.mat);
    if (tr == 0.0f) { out = 0.0f; return true; }
    v.T *= tr;
    v.remain -= h.t;
    v.org = h.pos;
    v.iter += 1u;
    if (v.iter == 5u) { out = 0.0f; return true; }
    return false;
}

// =========================================================================== PT_1 (init)
// The path tree has at most 4 vertices (Surface[0..3]), so the per-vertex chain is kept
// in named fields and CompressPath is unrolled on constant indices: a runtime-indexed
// array here would push the whole lane state into scratch.  Fields of a kind are kept
// non-adjacent on purpose (adjacent same-type fields + a runtime select get folded into
// one indexed load, which blocks SROA).
struct InitState {
    uint32_t pix, seed, i, phase;  // vertex index 1..3; phase: 0 = NEE visibility, 1 = BSDF ray
    f3 f; float p;
    f3 prev; Surface X; f3 V; f3 L;   // L = BSDF direction while phase == 1
    LightSample XL; f3 contrib;       // current NEE candidate
    Vis vis;
    uint32_t C; float w_sum, p_hat_sel; bool selected;
    // path-tree chain for CompressPath (SH/PT_1_InitPass.wgsl:1262-1353)
    f3 p1; uint32_t lobe1; float r1; uint4 cs2;  // Surface[1] pos / roughness, Lobe[1], CSurface[2]
    f3 p2; uint32_t bseed1; float r2;            // rSeed[2] = seed before SampleBSDF at vertex 1
    uint32_t nee_seed; f3 p3; uint32_t lobe2;     // rSeed[i+1] before SampleNEE at the current i
    float r3; uint4 cs3; uint32_t bseed2;         // rSeed[3] = seed before SampleBSDF at vertex 2
};

// CompressPath of the snapshot the chosen candidate (vertex i, NEE or env) stands for,
// written straight into this pixel's reservoir slot (words 0..27).  Snapshot rules:
// Lobe[k] is set for k < i (and k == i for env), rSeed[k+1] holds the seed before
// SampleBSDF at k for k < i and, at k == i, the seed before SampleNEE (NEE) or before
// SampleBSDF (env); every later entry is still zero (Path() is zero-initialised).
__device__ __forceinline__ void write_compressed(const InitState &s, bool is_env, const LightSample &XL, uint4 *out) {
    const uint32_t i = s.i;
    const uint32_t length = i + 1u;
    const uint32_t L1 = (i > 1u || is_env) ? s.lobe1 : 0u;
    const uint32_t L2 = (i > 2u || (is_env && i == 2u)) ? s.lobe2 : 0u;  // Lobe[3] is never set
    const uint32_t s2 = (i >= 2u || is_env) ? s.bseed1 : s.nee_seed;
    const uint32_t s3 = (i >= 3u || (i == 2u && is_env)) ? s.bseed2 : (i == 2u ? s.nee_seed : 0u);
    const uint32_t s4 = (i == 3u) ? s.nee_seed : 0u;
    uint32_t k = 0u;
    if (length > 2u) {  // SafeReconnectionIndex (PT_1:1283-1296), pair (1,2)
        float ra = L1 == LOBE_LAMBERT ? 1.0f : s.r1;
        float rb = L2 == LOBE_LAMBERT ? 1.0f : s.r2;
        if (length3(s.p1 - s.p2) >= RECONNECTION_DISTANCE && fminf(ra, rb) >= RECONNECTION_ROUGHNESS) k = 2u;
    }
    if (k == 0u && length > 3u) {  // pair (2,3); Lobe[3] = 0 = LOBE_LAMBERT
        float ra = L2 == LOBE_LAMBERT ? 1.0f : s.r2;
        if (length3(s.p2 - s.p3) >= RECONNECTION_DISTANCE && fminf(ra, 1.0f) >= RECONNECTION_ROUGHNESS) k = 3u;
    }
    if (k == 0u) {  // IsSafeToReconnect_Light on Surface[length-1] = the current vertex
        bool rough = s.X.mat.rough >= RECONNECTION_ROUGHNESS;
        bool dirl = XL.type == LIGHT_DIRECTION || XL.type == LIGHT_ENV;
        if ((dirl || length3(s.X.pos - XL.pos) >= RECONNECTION_DISTANCE) && rough) k = length;
    }
    uint4 rc = make_uint4(0u, 0u, 0u, 0u);
    uint32_t lk = 0u, lk1 = 0u;
    if (k == length) {
        lk = LOBE_LIGHT;
        lk1 = (k == 2u) ? L1 : (k == 3u) ? L2 : 0u;
    } else if (k == 2u) {
        lk = L2; lk1 = L1; rc = s.cs2;
    } else if (k == 3u) {
        lk = 0u; lk1 = L2; rc = s.cs3;
    }
    out[0] = make_uint4(s2, s3, s4, 0u);
    out[1] = make_uint4(asu(XL.dir.x), asu(XL.dir.y), asu(XL.dir.z), XL.type);
    out[2] = make_uint4(asu(XL.pos.x), asu(XL.pos.y), asu(XL.pos.z), (uint32_t)XL.id);
    out[3] = make_uint4(asu(XL.Le.x), asu(XL.Le.y), asu(XL.Le.z), asu(XL.pdf));
    out[4] = rc;
    out[5] = make_uint4(k, lk1, lk, length);
    out[6] = make_uint4(0u, 0u, 0u, 0u);
}

// Start vertex i: NEE sample and its first Visibility ray (PT_1:1403-1414).
__device__ __forceinline__ void init_begin_vertex(const Scene &sc, InitState &s, Ray &ray) {
    s.V = normalize(s.prev - s.X.pos);
    s.nee_seed = s.seed;
    s.XL = sample_nee(sc, s.seed, s.X, s.V);
    f3 L = direction_to_light(s.X, s.XL);
    f3 c = s.f * l_emit<false>(s.XL, s.X);
    c = c * bsdf(s.X, s.V, L);
    s.contrib = c * fabsf(dot(s.X.nrm, L));
    vis_begin(s.vis, s.X.pos, s.XL.pos);
    s.phase = 0u;
    ray = Ray{s.vis.org, s.vis.dir};
}

__device__ __forceinline__ void init_finish(const Scene &sc, InitState &s, uint4 *reservoir) {
    uint4 *out = reservoir + 8u * (size_t)s.pix;
    if (!s.selected) {  // zero Path(): length 0, k 0 (no candidate ever accepted)
        for (int q = 0; q < 7; ++q) out[q] = make_uint4(0u, 0u, 0u, 0u);
    }
    out[7] = make_uint4(asu(s.w_sum / s.p_hat_sel), s.C, 0u, 0u);
}

// Returns true if the lane has a ray to trace next; false when the pixel is complete.
__device__ __forceinline__ bool init_after_nee(const Scene &sc, InitState &s, float vis, uint4 *reservoir, Ray &ray) {
    f3 contrib = s.contrib * vis;
    float p_hat = luminance(contrib);
    float ris = p_hat / (s.p * s.XL.pdf);
    s.C += 1u;  // UpdateReservoir, PT_1:1298-1320
    s.w_sum += ris;
    if (rnd(s.seed) < ris / s.w_sum) {
        s.selected = true;
        s.p_hat_sel = p_hat;
        write_compressed(s, false, s.XL, reservoir + 8u * (size_t)s.pix);
    }
    if (s.i == 3u) { init_finish(sc, s, reservoir); return false; }
    // Sample BSDF (PT_1:1427-1433), throughput + Russian roulette (:1436-1442)
    if (s.i == 1u) s.bseed1 = s.seed;
    else s.bseed2 = s.seed;
    uint32_t lobe;
    s.L = sample_bsdf(s.seed, s.X, s.V, lobe);
    if (s.i == 1u) s.lobe1 = lobe;
    else s.lobe2 = lobe;
    s.f = s.f * (bsdf(s.X, s.V, s.L) * fabsf(dot(s.X.nrm, s.L)));
    s.p *= pdf_bsdf(s.X, s.V, s.L);
    float ps = luminance(s.f) / s.p;
    if (rnd(s.seed) < ps) s.p *= ps;
    else { init_finish(sc, s, reservoir); return false; }
    s.phase = 1u;
    ray = Ray{s.X.pos, s.L};
    return true;
}

template <bool COUNT>
__global__ __launch_bounds__(PBLOCK) void init_persistent(Scene sc, const uint4 *gbuf, uint4 *reservoir,
                                                          unsigned int *queue_ctr) {
    uint32_t *stack = lds_pstack + threadIdx.x;
    const PixelQueue q = make_queue(sc);
    const PassEps eps{1e-4f, 1e-8f};
    InitState s;
    Ray ray;
    bool has_ray = false, exhausted = false;
    for (;;) {
        // ---- refill: lanes without work take pixels until they have a ray (or the queue ends)
        for (;;) {
            const bool want = !has_ray && !exhausted;
            if (!__ballot(want)) break;
            const uint32_t p = dequeue(queue_ctr, want);
            if (!want) continue;
            if (p >= q.n) { exhausted = true; continue; }
            uint32_t x, y;
            if (!pixel_at(sc, q, p, x, y)) continue;
            s.pix = (y - sc.row_begin) * sc.width + x;
            const Compact x1 = decode_g(gbuf[s.pix]);
            if (!x1.valid) {  // reservoir unobservable: PT_4 returns before LoadReservoir (:1404-1408)
                uint4 *out = reservoir + 8u * (size_t)s.pix;
                for (int k = 0; k < 8; ++k) out[k] = make_uint4(0u, 0u, 0u, 0u);
                continue;
            }
            s.seed = pcg(x * 1973u + y * 9277u + sc.U[U_FRAME] * 26699u);
            s.f = mk(1.0f, 1.0f, 1.0f);
            s.p = 1.0f;
            s.C = 0u; s.w_sum = 0.0f; s.p_hat_sel = 0.0f; s.selected = false;
            s.lobe1 = 0u; s.lobe2 = 0u; s.bseed1 = 0u; s.bseed2 = 0u;
            s.cs2 = make_uint4(0u, 0u, 0u, 0u); s.cs3 = s.cs2;
            s.prev = get_x0p(sc, x, y);
            s.X = get_surface(sc, x1);
            s.p1 = s.X.pos; s.r1 = s.X.mat.rough;
            s.p2 = s.p1; s.r2 = 0.0f; s.p3 = s.p1; s.r3 = 0.0f;
            s.i = 1u;
            init_begin_vertex(sc, s, ray);
            has_ray = true;
        }
        if (!__ballot(has_ray)) break;
        Hit h;
        if (has_ray) h = trace_core<COUNT>(sc, ray, eps, stack, PBLOCK);
        if (!has_ray) continue;
        if (s.phase == 0u) {  // NEE visibility segment
            float v;
            if (!vis_step(sc, s.vis, h, v)) { ray = Ray{s.vis.org, s.vis.dir}; continue; }
            has_ray = init_after_nee(sc, s, v, reservoir, ray);
        } else if (!h.valid) {  // BSDF ray escaped: env candidate (PT_1:1447-1461)
            LightSample env;
            env.pos = s.X.pos + s.L * INF_F;
            env.type = LIGHT_ENV;
            env.dir = -s.L;
            env.id = -1;
            env.Le = mk(ENV_C, ENV_C, ENV_C);
            env.pdf = pdf_bsdf(s.X, s.V, s.L);
            float ph = luminance(s.f * ENV_C);
            float ris = ph / s.p;
            s.C += 1u;
            s.w_sum += ris;
            if (rnd(s.seed) < ris / s.w_sum) {
                s.selected = true;
                s.p_hat_sel = ph;
                write_compressed(s, true, env, reservoir + 8u * (size_t)s.pix);
            }
            init_finish(sc, s, reservoir);
            has_ray = false;
        } else {  // BSDF ray hit: next vertex (PT_1:1464-1468)
            s.prev = s.X.pos;
            s.X = surface_at(sc, h.s, h.pos);
            s.i += 1u;
            if (s.i == 2u) { s.p2 = s.X.pos; s.r2 = s.X.mat.rough; s.cs2 = encode_g(h.s); }
            else { s.p3 = s.X.pos; s.r3 = s.X.mat.rough; s.cs3 = encode_g(h.s); }
            init_begin_vertex(sc, s, ray);
        }
    }
}

// =========================================================================== PT_4 (final)
struct FinalState {
    uint32_t pix, i, length, phase;  // phase 0 = regenerating BSDF rays, 1 = light visibility
    uint32_t seeds0, seeds1, seeds2;  // rSeed[0..2] (rSeed[3] is never replayed for length <= 4)
    float ucw;
    LightSample XL;
    f3 f, prev, V, Le;
    Surface cur;
    Vis vis;
};

__device__ __forceinline__ void final_last_segment(FinalState &s, Ray &ray) {
    // PathContribution's last vertex (PT_4:1323-1333); Visibility follows
    s.V = normalize(s.prev - s.cur.pos);
    f3 L = direction_to_light(s.cur, s.XL);
    s.f = s.f * (bsdf(s.cur, L, s.V) * fabsf(dot(s.cur.nrm, L)));
    s.Le = l_emit<true>(s.XL, s.cur);
    vis_begin(s.vis, s.cur.pos, s.XL.pos);
    s.phase = 1u;
    ray = Ray{s.vis.org, s.vis.dir};
}
__device__ __forceinline__ void final_regen_ray(FinalState &s, Ray &ray) {
    // RegeneratePath step i (PT_4:1367-1381)
    s.V = normalize(s.prev - s.cur.pos);
    uint32_t seed = s.seeds0;  // rSeed[i-1]: consumed in order, then shifted down
    s.seeds0 = s.seeds1;
    s.seeds1 = s.seeds2;
    uint32_t lobe;
    f3 dir = sample_bsdf(seed, s.cur, s.V, lobe);
    s.phase = 0u;
    ray = Ray{s.cur.pos, dir};
}

template <bool COUNT>
__global__ __launch_bounds__(PBLOCK) void final_persistent(Scene sc, const uint4 *gbuf, const uint4 *reservoir,
                                                           float4 *accum, unsigned int *queue_ctr) {
    uint32_t *stack = lds_pstack + threadIdx.x;
    const PixelQueue q = make_queue(sc);
    const PassEps eps{1e-4f, 1e-8f};
    FinalState s;
    Ray ray;
    bool has_ray = false, exhausted = false;
    for (;;) {
        for (;;) {
            const bool want = !has_ray && !exhausted;
            if (!__ballot(want)) break;
            const uint32_t p = dequeue(queue_ctr, want);
            if (!want) continue;
            if (p >= q.n) { exhausted = true; continue; }
            uint32_t x, y;
            if (!pixel_at(sc, q, p, x, y)) continue;
            s.pix = (y - sc.row_begin) * sc.width + x;
            const Compact x1 = decode_g(gbuf[s.pix]);
            if (!x1.valid) { accum[s.pix] = make_float4(ENV_C, ENV_C, ENV_C, 1.0f); continue; }
            const uint4 *res = reservoir + 8u * (size_t)s.pix;
            const uint4 r0 = res[0], r1 = res[1], r2 = res[2], r3 = res[3], r5 = res[5], r7 = res[7];
            s.length = r5.w;
            if (r7.y == 0u || s.length < 2u) { write_colorp(sc, accum, s.pix, mk(0.0f, 0.0f, 0.0f)); continue; }
            s.seeds0 = r0.x; s.seeds1 = r0.y; s.seeds2 = r0.z;
            s.ucw = asf(r7.x);
            s.XL.dir = mk(asf(r1.x), asf(r1.y), asf(r1.z));
            s.XL.type = r1.w;
            s.XL.pos = mk(asf(r2.x), asf(r2.y), asf(r2.z));
            s.XL.id = (int32_t)r2.w;
            s.XL.Le = mk(asf(r3.x), asf(r3.y), asf(r3.z));
            s.XL.pdf = asf(r3.w);
            s.prev = get_x0p(sc, x, y);
            s.cur = get_surface(sc, x1);
            s.f = mk(1.0f, 1.0f, 1.0f);
            s.i = 1u;
            if (s.i + 1u < s.length) final_regen_ray(s, ray);
            else final_last_segment(s, ray);
            has_ray = true;
        }
        if (!__ballot(has_ray)) break;
        Hit h;
        if (has_ray) h = trace_core<COUNT>(sc, ray, eps, stack, PBLOCK);
        if (!has_ray) continue;
        if (s.phase == 0u) {
            // a miss decodes the zero CompactSurface, exactly as the WGSL does
            Surface next = h.valid ? surface_at(sc, h.s, h.pos) : get_surface(sc, h.s);
            f3 L = normalize(next.pos - s.cur.pos);
            s.f = s.f * (bsdf(s.cur, L, s.V) * fabsf(dot(s.cur.nrm, L)));
            s.prev = s.cur.pos;
            s.cur = next;
            s.i += 1u;
            if (s.i + 1u < s.length) final_regen_ray(s, ray);
            else final_last_segment(s, ray);
        } else {
            float v;
            if (!vis_step(sc, s.vis, h, v)) { ray = Ray{s.vis.org, s.vis.dir}; continue; }
            s.f = s.f * (s.Le * v);
            write_colorp(sc, accum, s.pix, s.f * s.ucw);
            has_ray = false;
        }
    }
}

// =========================================================================== TEST_MCPT
struct McptState {
    uint32_t pix, seed, bounce, light, phase;  // phase 0 = path ray, 1 = light visibility
    Ray path;
    f3 color, f;
    float p;
    Surface X;
    f3 V, c;
    float lpdf;
    Vis vis;
};

// GetLightColor up to its Visibility (SH/TEST_MCPT.wgsl:1261-1308)
__device__ __forceinline__ void mcpt_begin_light(const Scene &sc, McptState &s, Ray &ray) {
    Light ls = get_light(sc, s.light);
    LightSample XL;
    XL.type = ls.type;
    XL.Le = ls.color * ls.intensity;
    XL.pos = mk(0.0f, 0.0f, 0.0f);
    XL.dir = mk(0.0f, 0.0f, 0.0f);
    XL.pdf = 0.0f;
    if (ls.type == LIGHT_DIRECTION) {
        XL.pos = s.X.pos - ls.dir * INF_F; XL.dir = ls.dir; XL.pdf = 1.0f;
    } else if (ls.type == LIGHT_POINT) {
        XL.pos = ls.pos; XL.dir = normalize(s.X.pos - ls.pos); XL.pdf = 1.0f;
    } else if (ls.type == LIGHT_RECT) {
        float ru = rnd(s.seed) * 2.0f - 1.0f;
        float rv = rnd(s.seed) * 2.0f - 1.0f;
        XL.pos = ls.pos + (ls.U * ru + ls.V * rv);
        XL.dir = normalize(s.X.pos - XL.pos);
        f3 rr = XL.pos - s.X.pos;
        f3 Ld = normalize(rr);
        XL.pdf = dot(rr, rr) / fmaxf(ls.area * fabsf(dot(ls.dir, Ld)), EPS_F);
    }
    f3 L = direction_to_light(s.X, XL);
    f3 c = l_emit<false>(XL, s.X) * bsdf(s.X, s.V, L);
    s.c = c * fabsf(dot(s.X.nrm, L));
    s.lpdf = XL.pdf;
    vis_begin(s.vis, s.X.pos, XL.pos);
    s.phase = 1u;
    ray = Ray{s.vis.org, s.vis.dir};
}

// After all lights of a bounce: BSDF sample, throughput, Russian roulette (TEST_MCPT:1356-1366).
__device__ __forceinline__ bool mcpt_bsdf_step(const Scene &sc, McptState &s, float4 *accum, Ray &ray) {
    uint32_t lobe;
    f3 L = sample_bsdf(s.seed, s.X, s.V, lobe);
    s.f = s.f * (bsdf(s.X, s.V, L) * fabsf(dot(s.X.nrm, L)));
    s.p *= pdf_bsdf(s.X, s.V, L);
    s.path = Ray{s.X.pos, L};
    float ps = luminance(s.f) / s.p;
    if (rnd(s.seed) < ps) s.p *= ps;
    else { write_colorp(sc, accum, s.pix, s.color); return false; }
    s.bounce += 1u;
    if (s.bounce == 3u) { write_colorp(sc, accum, s.pix, s.color); return false; }
    s.phase = 0u;
    ray = s.path;
    return true;
}

template <bool COUNT>
__global__ __launch_bounds__(PBLOCK) void mcpt_persistent(Scene sc, float4 *accum, unsigned int *queue_ctr) {
    uint32_t *stack = lds_pstack + threadIdx.x;
    const PixelQueue q = make_queue(sc);
    const PassEps eps{1e-4f, 1e-8f};
    const uint32_t nl = sc.U[U_LIGHT_COUNT];
    McptState s;
    Ray ray;
    bool has_ray = false, exhausted = false;
    for (;;) {
        for (;;) {
            const bool want = !has_ray && !exhausted;
            if (!__ballot(want)) break;
            const uint32_t p = dequeue(queue_ctr, want);
            if (!want) continue;
            if (p >= q.n) { exhausted = true; continue; }
            uint32_t x, y;
            if (!pixel_at(sc, q, p, x, y)) continue;
            s.pix = (y - sc.row_begin) * sc.width + x;
            s.seed = pcg(x * 1973u + y * 9277u + sc.U[U_FRAME] * 26699u);
            s.path = camera_rayp(sc, x, y);
            s.color = mk(0.0f, 0.0f, 0.0f);
            s.f = mk(1.0f, 1.0f, 1.0f);
            s.p = 1.0f;
            s.bounce = 0u;
            s.phase = 0u;
            ray = s.path;
            has_ray = true;
        }
        if (!__ballot(has_ray)) break;
        Hit h;
        if (has_ray) h = trace_core<COUNT>(sc, ray, eps, stack, PBLOCK);
        if (!has_ray) continue;
        if (s.phase == 0u) {
            if (!h.valid) {
                s.color = s.color + (s.f / s.p) * ENV_C;
                write_colorp(sc, accum, s.pix, s.color);
                has_ray = false;
                continue;
            }
            s.X = surface_at(sc, h.s, h.pos);
            s.V = normalize(s.path.o - s.X.pos);
            s.light = 0u;
            if (nl > 0u) mcpt_begin_light(sc, s, ray);
            else has_ray = mcpt_bsdf_step(sc, s, accum, ray);
        } else {
            float v;
            if (!vis_step(sc, s.vis, h, v)) { ray = Ray{s.vis.org, s.vis.dir}; continue; }
            s.color = s.color + (s.f / s.p) * ((s.c * v) / s.lpdf);
            s.light += 1u;
            if (s.light < nl) mcpt_begin_light(sc, s, ray);
            else has_ray = mcpt_bsdf_step(sc, s, accum, ray);
        }
    }
}

// =========================================================================== tile + LDS ray exchange
// One workgroup owns a 16x16 pixel tile for the whole pass; lane states stay in
// registers.  Every iteration all 256 lanes post their pending ray to LDS with a bin key
// (light id for shadow / Visibility rays, direction octant for BSDF and camera rays), a
// counting sort orders the rays by key, and lane j traces the j-th sorted ray.  The rays
// of a tile are therefore compacted into the fewest waves and grouped so that a wave
// traverses rays aimed at the same light or octant (coherent node fetches), while the
// state machine stays per pixel.  Results remain per-pixel functions: only who traces a
// ray changes, never what is traced.
constexpr uint32_t XBINS = 64;           // bin keys: [0,56) lights (id % 56), [56,64) octants
constexpr uint32_t XLIGHT_BINS = 56;

struct alignas(16) XchgLds {
    float4 ray0[PBLOCK];   // o.xyz, d.x
    float4 ray1[PBLOCK];   // d.y, d.z
    float4 hit0[PBLOCK];   // t, enc(valid|inst|mat), prim, bu
    float4 hit1[PBLOCK];   // bv, pos.xyz
    uint32_t cnt[XBINS];
    uint32_t base[XBINS];
    uint16_t perm[PBLOCK];
    uint32_t nrays, pad[3];
};
constexpr size_t kXchgBytes = (sizeof(XchgLds) + 15u) & ~size_t(15);

__device__ __forceinline__ uint32_t octant_key(f3 d) {
    return XLIGHT_BINS + (d.x < 0.0f ? 1u : 0u) + (d.y < 0.0f ? 2u : 0u) + (d.z < 0.0f ? 4u : 0u);
}
__device__ __forceinline__ uint32_t light_key(int32_t id, f3 d) {
    return id >= 0 ? (uint32_t)id % XLIGHT_BINS : octant_key(d);
}

template <bool COUNT>
__device__ __forceinline__ void xchg_trace(const Scene &sc, XchgLds &X, uint32_t *stack, PassEps eps, bool has_ray,
                                           const Ray &ray, uint32_t key, Hit &out) {
    const uint32_t tid = threadIdx.x;
    if (tid < XBINS) X.cnt[tid] = 0u;
    __syncthreads();
    uint32_t rank = 0u;
    if (has_ray) {
        rank = atomicAdd(&X.cnt[key], 1u);
        X.ray0[tid] = make_float4(ray.o.x, ray.o.y, ray.o.z, ray.d.x);
        X.ray1[tid] = make_float4(ray.d.y, ray.d.z, 0.0f, 0.0f);
    }
    __syncthreads();
    if (tid < 64u) {  // wave 0: exclusive scan of the 64 bin counts
        uint32_t v = X.cnt[tid], incl = v;
        for (uint32_t o = 1u; o < 64u; o <<= 1) {
            uint32_t t = __shfl_up(incl, o);
            if (tid >= o) incl += t;
        }
        X.base[tid] = incl - v;
        if (tid == 63u) X.nrays = incl;
    }
    __syncthreads();
    if (has_ray) X.perm[X.base[key] + rank] = (uint16_t)tid;
    __syncthreads();
    if (tid < X.nrays) {
        const uint32_t src = X.perm[tid];
        const float4 a = X.ray0[src], b = X.ray1[src];
        Hit h = trace_core<COUNT>(sc, Ray{mk(a.x, a.y, a.z), mk(a.w, b.x, b.y)}, eps, stack, PBLOCK);
        const uint32_t enc = ((h.valid ? 1u : 0u) << 31) | (h.s.inst << 16) | h.s.mat;
        X.hit0[src] = make_float4(h.t, asf(enc), asf(h.s.prim), h.s.bu);
        X.hit1[src] = make_float4(h.s.bv, h.pos.x, h.pos.y, h.pos.z);
    }
    __syncthreads();
    if (has_ray) {
        const float4 a = X.hit0[tid], b = X.hit1[tid];
        const uint32_t enc = asu(a.y);
        out.valid = (enc >> 31) != 0u;
        out.t = a.x;
        out.s = Compact{enc >> 31, (enc >> 16) & 0x7fffu, enc & 0xffffu, asu(a.z), a.w, b.x};
        out.pos = mk(b.y, b.z, b.w);
    }
}

__device__ __forceinline__ bool tile_pixel(const Scene &sc, uint32_t &x, uint32_t &y) {
    const uint32_t tiles_x = (sc.width + 15u) / 16u;
    const uint32_t t = threadIdx.x, w = t >> 6, lane = t & 63u;
    x = (blockIdx.x % tiles_x) * 16u + (w & 1u) * 8u + (lane & 7u);
    y = sc.row_begin + (blockIdx.x / tiles_x) * 16u + (w >> 1) * 8u + (lane >> 3);
    return x < sc.width && y < sc.row_end;
}

template <bool COUNT>
__global__ __launch_bounds__(PBLOCK) void init_tiled(Scene sc, const uint4 *gbuf, uint4 *reservoir) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
    XchgLds &X = *reinterpret_cast<XchgLds *>(lds_raw);
    uint32_t *stack = reinterpret_cast<uint32_t *>(lds_raw + kXchgBytes) + threadIdx.x;
    const PassEps eps{1e-4f, 1e-8f};
    InitState s;
    Ray ray;
    bool has_ray = false;
    uint32_t x, y;
    if (tile_pixel(sc, x, y)) {
        s.pix = (y - sc.row_begin) * sc.width + x;
        const Compact x1 = decode_g(gbuf[s.pix]);
        if (!x1.valid) {  // reservoir unobservable: PT_4 returns before LoadReservoir (:1404-1408)
            uint4 *out = reservoir + 8u * (size_t)s.pix;
            for (int k = 0; k < 8; ++k) out[k] = make_uint4(0u, 0u, 0u, 0u);
        } else {
            s.seed = pcg(x * 1973u + y * 9277u + sc.U[U_FRAME] * 26699u);
            s.f = mk(1.0f, 1.0f, 1.0f);
            s.p = 1.0f;
            s.C = 0u; s.w_sum = 0.0f; s.p_hat_sel = 0.0f; s.selected = false;
            s.lobe1 = 0u; s.lobe2 = 0u; s.bseed1 = 0u; s.bseed2 = 0u;
            s.cs2 = make_uint4(0u, 0u, 0u, 0u); s.cs3 = s.cs2;
            s.prev = get_x0p(sc, x, y);
            s.X = get_surface(sc, x1);
            s.p1 = s.X.pos; s.r1 = s.X.mat.rough;
            s.p2 = s.p1; s.r2 = 0.0f; s.p3 = s.p1; s.r3 = 0.0f;
            s.i = 1u;
            init_begin_vertex(sc, s, ray);
            has_ray = true;
        }
    }
    while (__syncthreads_or(has_ray)) {
        const uint32_t key = has_ray ? (s.phase == 0u ? light_key(s.XL.id, ray.d) : octant_key(ray.d)) : 0u;
        Hit h;
        xchg_trace<COUNT>(sc, X, stack, eps, has_ray, ray, key, h);
        if (!has_ray) continue;
        if (s.phase == 0u) {  // NEE visibility segment
            float v;
            if (!vis_step(sc, s.vis, h, v)) { ray = Ray{s.vis.org, s.vis.dir}; continue; }
            has_ray = init_after_nee(sc, s, v, reservoir, ray);
        } else if (!h.valid) {  // BSDF ray escaped: env candidate (PT_1:1447-1461)
            LightSample env;
            env.pos = s.X.pos + s.L * INF_F;
            env.type = LIGHT_ENV;
            env.dir = -s.L;
            env.id = -1;
            env.Le = mk(ENV_C, ENV_C, ENV_C);
            env.pdf = pdf_bsdf(s.X, s.V, s.L);
            float ph = luminance(s.f * ENV_C);
            float ris = ph / s.p;
            s.C += 1u;
            s.w_sum += ris;
            if (rnd(s.seed) < ris / s.w_sum) {
                s.selected = true;
                s.p_hat_sel = ph;
                write_compressed(s, true, env, reservoir + 8u * (size_t)s.pix);
            }
            init_finish(sc, s, reservoir);
            has_ray = false;
        } else {  // BSDF ray hit: next vertex (PT_1:1464-1468)
            s.prev = s.X.pos;
            s.X = surface_at(sc, h.s, h.pos);
            s.i += 1u;
            if (s.i == 2u) { s.p2 = s.X.pos; s.r2 = s.X.mat.rough; s.cs2 = encode_g(h.s); }
            else { s.p3 = s.X.pos; s.r3 = s.X.mat.rough; s.cs3 = encode_g(h.s); }
            init_begin_vertex(sc, s, ray);
        }
    }
}

template <bool COUNT>
__global__ __launch_bounds__(PBLOCK) void final_tiled(Scene sc, const uint4 *gbuf, const uint4 *reservoir,
                                                      float4 *accum) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
    XchgLds &X = *reinterpret_cast<XchgLds *>(lds_raw);
    uint32_t *stack = reinterpret_cast<uint32_t *>(lds_raw + kXchgBytes) + threadIdx.x;
    const PassEps eps{1e-4f, 1e-8f};
    FinalState s;
    Ray ray;
    bool has_ray = false;
    uint32_t x, y;
    if (tile_pixel(sc, x, y)) {
        s.pix = (y - sc.row_begin) * sc.width + x;
        const Compact x1 = decode_g(gbuf[s.pix]);
        const uint4 *res = reservoir + 8u * (size_t)s.pix;
        if (!x1.valid) {
            accum[s.pix] = make_float4(ENV_C, ENV_C, ENV_C, 1.0f);
        } else {
            const uint4 r0 = res[0], r1 = res[1], r2 = res[2], r3 = res[3], r5 = res[5], r7 = res[7];
            s.length = r5.w;
            if (r7.y == 0u || s.length < 2u) {
                write_colorp(sc, accum, s.pix, mk(0.0f, 0.0f, 0.0f));
            } else {
                s.seeds0 = r0.x; s.seeds1 = r0.y; s.seeds2 = r0.z;
                s.ucw = asf(r7.x);
                s.XL.dir = mk(asf(r1.x), asf(r1.y), asf(r1.z));
                s.XL.type = r1.w;
                s.XL.pos = mk(asf(r2.x), asf(r2.y), asf(r2.z));
                s.XL.id = (int32_t)r2.w;
                s.XL.Le = mk(asf(r3.x), asf(r3.y), asf(r3.z));
                s.XL.pdf = asf(r3.w);
                s.prev = get_x0p(sc, x, y);
                s.cur = get_surface(sc, x1);
                s.f = mk(1.0f, 1.0f, 1.0f);
                s.i = 1u;
                if (s.i + 1u < s.length) final_regen_ray(s, ray);
                else final_last_segment(s, ray);
                has_ray = true;
            }
        }
    }
    while (__syncthreads_or(has_ray)) {
        const uint32_t key = has_ray ? (s.phase == 0u ? octant_key(ray.d) : light_key(s.XL.id, ray.d)) : 0u;
        Hit h;
        xchg_trace<COUNT>(sc, X, stack, eps, has_ray, ray, key, h);
        if (!has_ray) continue;
        if (s.phase == 0u) {
            Surface next = h.valid ? surface_at(sc, h.s, h.pos) : get_surface(sc, h.s);
            f3 L = normalize(next.pos - s.cur.pos);
            s.f = s.f * (bsdf(s.cur, L, s.V) * fabsf(dot(s.cur.nrm, L)));
            s.prev = s.cur.pos;
            s.cur = next;
            s.i += 1u;
            if (s.i + 1u < s.length) final_regen_ray(s, ray);
            else final_last_segment(s, ray);
        } else {
            float v;
            if (!vis_step(sc, s.vis, h, v)) { ray = Ray{s.vis.org, s.vis.dir}; continue; }
            s.f = s.f * (s.Le * v);
            write_colorp(sc, accum, s.pix, s.f * s.ucw);
            has_ray = false;
        }
    }
}

template <bool COUNT>
__global__ __launch_bounds__(PBLOCK) void mcpt_tiled(Scene sc, float4 *accum) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
    XchgLds &X = *reinterpret_cast<XchgLds *>(lds_raw);
    uint32_t *stack = reinterpret_cast<uint32_t *>(lds_raw + kXchgBytes) + threadIdx.x;
    const PassEps eps{1e-4f, 1e-8f};
    const uint32_t nl = sc.U[U_LIGHT_COUNT];
    McptState s;
    Ray ray;
    bool has_ray = false;
    uint32_t x, y;
    if (tile_pixel(sc, x, y)) {
        s.pix = (y - sc.row_begin) * sc.width + x;
        s.seed = pcg(x * 1973u + y * 9277u + sc.U[U_FRAME] * 26699u);
        s.path = camera_rayp(sc, x, y);
        s.color = mk(0.0f, 0.0f, 0.0f);
        s.f = mk(1.0f, 1.0f, 1.0f);
        s.p = 1.0f;
        s.bounce = 0u;
        s.phase = 0u;
        ray = s.path;
        has_ray = true;
    }
    while (__syncthreads_or(has_ray)) {
        const uint32_t key = has_ray ? (s.phase == 0u ? octant_key(ray.d) : s.light % XLIGHT_BINS) : 0u;
        Hit h;
        xchg_trace<COUNT>(sc, X, stack, eps, has_ray, ray, key, h);
        if (!has_ray) continue;
        if (s.phase == 0u) {
            if (!h.valid) {
                s.color = s.color + (s.f / s.p) * ENV_C;
                write_colorp(sc, accum, s.pix, s.color);
                has_ray = false;
                continue;
            }
            s.X = surface_at(sc, h.s, h.pos);
            s.V = normalize(s.path.o - s.X.pos);
            s.light = 0u;
            if (nl > 0u) mcpt_begin_light(sc, s, ray);
            else has_ray = mcpt_bsdf_step(sc, s, accum, ray);
        } else {
            float v;
            if (!vis_step(sc, s.vis, h, v)) { ray = Ray{s.vis.org, s.vis.dir}; continue; }
            s.color = s.color + (s.f / s.p) * ((s.c * v) / s.lpdf);
            s.light += 1u;
            if (s.light < nl) mcpt_begin_light(sc, s, ray);
            else has_ray = mcpt_bsdf_step(sc, s, accum, ray);
        }
    }
}

static dim3 tiled_grid(const Scene &sc) {
    return dim3(((sc.width + 15u) / 16u) * ((sc.row_end - sc.row_begin + 15u) / 16u));
}
static size_t tiled_lds(uint32_t depth) { return kXchgBytes + stack_lds_bytes(depth); }

hipError_t launch_init_tiled(const Scene &sc, const uint4 *gbuf, uint4 *reservoir, uint32_t depth, hipStream_t s) {
    if (sc.counters) hipLaunchKernelGGL(init_tiled<true>, tiled_grid(sc), dim3(PBLOCK), tiled_lds(depth), s, sc, gbuf, reservoir);
    else hipLaunchKernelGGL(init_tiled<false>, tiled_grid(sc), dim3(PBLOCK), tiled_lds(depth), s, sc, gbuf, reservoir);
    return hipGetLastError();
}
hipError_t launch_final_tiled(const Scene &sc, const uint4 *gbuf, const uint4 *reservoir, float4 *accum,
                              uint32_t depth, hipStream_t s) {
    if (sc.counters)
        hipLaunchKernelGGL(final_tiled<true>, tiled_grid(sc), dim3(PBLOCK), tiled_lds(depth), s, sc, gbuf, reservoir, accum);
    else
        hipLaunchKernelGGL(final_tiled<false>, tiled_grid(sc), dim3(PBLOCK), tiled_lds(depth), s, sc, gbuf, reservoir, accum);
    return hipGetLastError();
}
hipError_t launch_mcpt_tiled(const Scene &sc, float4 *accum, uint32_t depth, hipStream_t s) {
    if (sc.counters) hipLaunchKernelGGL(mcpt_tiled<true>, tiled_grid(sc), dim3(PBLOCK), tiled_lds(depth), s, sc, accum);
    else hipLaunchKernelGGL(mcpt_tiled<false>, tiled_grid(sc), dim3(PBLOCK), tiled_lds(depth), s, sc, accum);
    return hipGetLastError();
}

// =========================================================================== launches
static uint32_t persistent_grid(const Scene &sc) {
    const uint32_t wgs_needed = ((sc.width + 7u) / 8u) * ((sc.row_end - sc.row_begin + 7u) / 8u) * 64u / PBLOCK + 1u;
    const uint32_t cap = 256u * 8u;  // 256 CUs x 8 resident 256-thread workgroups at most
    return wgs_needed < cap ? wgs_needed : cap;
}
hipError_t launch_init_persistent(const Scene &sc, const uint4 *gbuf, uint4 *reservoir, unsigned int *ctr,
                                  uint32_t depth, hipStream_t s) {
    if (sc.counters)
        hipLaunchKernelGGL(init_persistent<true>, dim3(persistent_grid(sc)), dim3(PBLOCK), stack_lds_bytes(depth), s,
                           sc, gbuf, reservoir, ctr);
    else
        hipLaunchKernelGGL(init_persistent<false>, dim3(persistent_grid(sc)), dim3(PBLOCK), stack_lds_bytes(depth), s,
                           sc, gbuf, reservoir, ctr);
    return hipGetLastError();
}
hipError_t launch_final_persistent(const Scene &sc, const uint4 *gbuf, const uint4 *reservoir, float4 *accum,
                                   unsigned int *ctr, uint32_t depth, hipStream_t s) {
    if (sc.counters)
        hipLaunchKernelGGL(final_persistent<true>, dim3(persistent_grid(sc)), dim3(PBLOCK), stack_lds_bytes(depth), s,
                           sc, gbuf, reservoir, accum, ctr);
    else
        hipLaunchKernelGGL(final_persistent<false>, dim3(persistent_grid(sc)), dim3(PBLOCK), stack_lds_bytes(depth), s,
                           sc, gbuf, reservoir, accum, ctr);
    return hipGetLastError();
}
hipError_t launch_mcpt_persistent(const Scene &sc, float4 *accum, unsigned int *ctr, uint32_t depth, hipStream_t s) {
    if (sc.counters)
        hipLaunchKernelGGL(mcpt_persistent<true>, dim3(persistent_grid(sc)), dim3(PBLOCK), stack_lds_bytes(depth), s,
                           sc, accum, ctr);
    else
        hipLaunchKernelGGL(mcpt_persistent<false>, dim3(persistent_grid(sc)), dim3(PBLOCK), stack_lds_bytes(depth), s,
                           sc, accum, ctr);
    return hipGetLastError();
}

}  // namespace ptx
