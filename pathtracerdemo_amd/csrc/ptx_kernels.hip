// ptx_kernels.hip -- the per-pixel passes of the reference renderer as gfx950 kernels.
//
//   gbuffer_kernel <- SH/PT_01_GBufferPass.wgsl:627-659
//   init_kernel    <- SH/PT_1_InitPass.wgsl:1361-1486
//   final_kernel   <- SH/PT_4_FinalShadingPass.wgsl:1392-1428 (+ Result->Scene copy folded in)
//   mcpt_kernel    <- SH/TEST_MCPT.wgsl:1315-1372
//
// Launch shape: 256-thread workgroups covering a 16x16 pixel tile, each wave64 an 8x8
// sub-tile (ray coherence inside a wave).  Every thread owns one column of an LDS
// traversal stack sized from the scene's deepest BLAS (dynamic LDS).
#include "ptx_launch.h"
#include "ptx_shading.h"

namespace ptx {

constexpr int TILE = kTile;
constexpr int BLOCK = kBlock;

__device__ __forceinline__ bool pixel_of(const Scene &sc, uint32_t &x, uint32_t &y) {
    const uint32_t t = threadIdx.x;
    const uint32_t w = t >> 6, lane = t & 63u;
    x = blockIdx.x * TILE + (w & 1u) * 8u + (lane & 7u);
    y = sc.row_begin + blockIdx.y * TILE + (w >> 1) * 8u + (lane >> 3);
    return x < sc.width && y < sc.row_end;
}
__device__ __forceinline__ size_t band_index(const Scene &sc, uint32_t x, uint32_t y) {
    return (size_t)(y - sc.row_begin) * sc.width + x;
}

extern __shared__ __attribute__((aligned(16))) uint32_t lds_stack[];

// GenerateRayFromThreadID (SH/PT_01_GBufferPass.wgsl:496-507)
__device__ __forceinline__ Ray camera_ray(const Scene &sc, uint32_t x, uint32_t y) {
    const float *vpinv = reinterpret_cast<const float *>(sc.U + U_VPINV);
    float u = ((float)x + 0.5f) / (float)sc.U[U_W];
    float v = ((float)y + 0.5f) / (float)sc.U[U_H];
    f3 start = xform_point(vpinv, mk(2.0f * u - 1.0f, 2.0f * v - 1.0f, 0.0f));
    f3 end = xform_point(vpinv, mk(2.0f * u - 1.0f, 2.0f * v - 1.0f, 0.0f + 1.0f));
    return Ray{start, normalize(end - start)};
}
// Get_X0 (SH/PT_1_InitPass.wgsl:732-738)
__device__ __forceinline__ f3 get_x0(const Scene &sc, uint32_t x, uint32_t y) {
    const float *vpinv = reinterpret_cast<const float *>(sc.U + U_VPINV);
    float u = ((float)x + 0.5f) / (float)sc.U[U_W];
    float v = ((float)y + 0.5f) / (float)sc.U[U_H];
    return xform_point(vpinv, mk(2.0f * u - 1.0f, 2.0f * v - 1.0f, 0.0f));
}
__device__ __forceinline__ uint32_t init_seed(const Scene &sc, uint32_t x, uint32_t y) {
    return pcg(x * 1973u + y * 9277u + sc.U[U_FRAME] * 26699u);  // SH/PT_1_InitPass.wgsl:823-826
}
__device__ __forceinline__ uint4 encode(const Compact &s) {
    return make_uint4((s.valid << 31) | (s.inst << 16) | s.mat, s.prim, asu(s.bu), asu(s.bv));
}
__device__ __forceinline__ Compact decode(uint4 g) {
    Compact s;
    s.valid = (g.x & 0x80000000u) ? 1u : 0u;
    s.inst = (g.x & 0x7fff0000u) >> 16;
    s.mat = g.x & 0xffffu;
    s.prim = g.y;
    s.bu = asf(g.z);
    s.bv = asf(g.w);
    return s;
}
// WriteColor (SH/PT_4_FinalShadingPass.wgsl:599-606); the Scene texture is updated in
// place (each texel reads only itself), which replaces copyTextureToTexture(Result->Scene).
__device__ __forceinline__ void write_color(const Scene &sc, float4 *accum, size_t i, f3 c) {
    float t = 1.0f / (float)(sc.U[U_FRAME] + 1u);
    float4 a = accum[i];
    accum[i] = make_float4(mixf(a.x, c.x, t), mixf(a.y, c.y, t), mixf(a.z, c.z, t), 1.0f);
}

// =========================================================================== PT_01
template <bool COUNT, bool LDS_TABLES = false>
__global__ __launch_bounds__(BLOCK) void gbuffer_kernel(Scene sc, uint4 *gbuf) {
    // dynamic LDS: [scene tables (LDS_TABLES)] [stacks]
    const LdsTables T = LDS_TABLES ? stage_tables(sc, lds_stack) : LdsTables{sc.subs, sc.insts};
    uint32_t x, y;
    if (!pixel_of(sc, x, y)) return;
    if (COUNT && sc.census) sc.counters = sc.census + (size_t)kCensusWords * ((y - sc.row_begin) / 8u);  // row census
    uint32_t *stack = lds_stack + (LDS_TABLES ? tables_lds_bytes(sc) / 4u : 0u) + threadIdx.x;
    Hit h = trace_core_tab<COUNT, false, false>(sc, T.subs, T.insts, camera_ray(sc, x, y), PassEps{1e-8f, 1e-6f},
                                                stack, BLOCK);
    Compact s = h.s;
    s.valid = h.valid ? 1u : 0u;
    gbuf[band_index(sc, x, y)] = encode(s);
}

// =========================================================================== PT_1
struct Chain {                 // what CompressPath needs of the path tree
    f3 pos[4];
    float rough[4];
    uint32_t lobe[4], nee_seed[4], bsdf_seed[4];
    Compact cs[4];
};

__device__ void store_reservoir(uint4 *out, const Chain &ch, int sel_i, bool sel_env, const LightSample &XL,
                                float ucw, uint32_t C) {
    uint32_t w[32];
#pragma unroll
    for (int k = 0; k < 32; ++k) w[k] = 0u;
    if (sel_i > 0) {
        // CompressPath + SafeReconnectionIndex (SH/PT_1_InitPass.wgsl:1262-1353) on the
        // snapshot Path the chosen candidate stands for.
        uint32_t lobe[4] = {0u, 0u, 0u, 0u}, seed[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
        for (int k = 1; k < sel_i; ++k) { lobe[k] = ch.lobe[k]; seed[k + 1] = ch.bsdf_seed[k]; }
        if (sel_env) { lobe[sel_i] = ch.lobe[sel_i]; seed[sel_i + 1] = ch.bsdf_seed[sel_i]; }
        else seed[sel_i + 1] = ch.nee_seed[sel_i];
        const uint32_t length = (uint32_t)sel_i + 1u;
        uint32_t k = 0u;
        for (uint32_t kk = 2u; kk < length; ++kk) {
            float ra = lobe[kk - 1] == LOBE_LAMBERT ? 1.0f : ch.rough[kk - 1];
            float rb = lobe[kk] == LOBE_LAMBERT ? 1.0f : ch.rough[kk];
            bool rough = fminf(ra, rb) >= RECONNECTION_ROUGHNESS;
            bool far = length3(ch.pos[kk - 1] - ch.pos[kk]) >= RECONNECTION_DISTANCE;
            if (far && rough) { k = kk; break; }
        }
        if (k == 0u) {
            bool rough = ch.rough[length - 1] >= RECONNECTION_ROUGHNESS;
            bool dirl = XL.type == LIGHT_DIRECTION || XL.type == LIGHT_ENV;
            bool far = dirl || length3(ch.pos[length - 1] - XL.pos) >= RECONNECTION_DISTANCE;
            if (far && rough) k = length;
        }
        w[0] = seed[2]; w[1] = seed[3]; w[2] = seed[4]; w[3] = seed[5];
        w[4] = asu(XL.dir.x); w[5] = asu(XL.dir.y); w[6] = asu(XL.dir.z); w[7] = XL.type;
        w[8] = asu(XL.pos.x); w[9] = asu(XL.pos.y); w[10] = asu(XL.pos.z); w[11] = (uint32_t)XL.id;
        w[12] = asu(XL.Le.x); w[13] = asu(XL.Le.y); w[14] = asu(XL.Le.z); w[15] = asu(XL.pdf);
        w[20] = k;
        w[23] = length;
        if (k != 0u) {
            bool is_light = (k == length);
            w[22] = is_light ? LOBE_LIGHT : lobe[k];
            w[21] = lobe[k - 1];
            if (!is_light) {
                uint4 rc = encode(ch.cs[k]);
                w[16] = rc.x; w[17] = rc.y; w[18] = rc.z; w[19] = rc.w;
            }
        }
    }
    w[28] = asu(ucw);
    w[29] = C;
#pragma unroll
    for (int q = 0; q < 8; ++q) out[q] = make_uint4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
}

template <bool COUNT>
__global__ __launch_bounds__(BLOCK) void init_kernel(Scene sc, const uint4 *gbuf, uint4 *reservoir) {
    uint32_t x, y;
    if (!pixel_of(sc, x, y)) return;
    uint32_t *stack = lds_stack + threadIdx.x;
    const size_t pi = band_index(sc, x, y);
    uint4 *out = reservoir + 8u * pi;
    Compact x1 = decode(gbuf[pi]);
    if (!x1.valid) {  // reservoir unobservable: PT_4 returns before LoadReservoir (:1404-1408)
#pragma unroll
        for (int q = 0; q < 8; ++q) out[q] = make_uint4(0u, 0u, 0u, 0u);
        return;
    }
    const PassEps eps{1e-4f, 1e-8f};
    uint32_t seed = init_seed(sc, x, y);
    f3 f = mk(1.0f, 1.0f, 1.0f);
    float p = 1.0f;
    Chain ch;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        ch.rough[k] = 0.0f; ch.lobe[k] = 0u; ch.nee_seed[k] = 0u; ch.bsdf_seed[k] = 0u;
        ch.pos[k] = mk(0.0f, 0.0f, 0.0f); ch.cs[k] = Compact{0u, 0u, 0u, 0u, 0.0f, 0.0f};
    }
    ch.cs[1] = x1;
    f3 prev = get_x0(sc, x, y);
    Surface X = get_surface(sc, x1);
    ch.pos[0] = prev;
    ch.pos[1] = X.pos;
    ch.rough[1] = X.mat.rough;
    uint32_t C = 0u;
    float w_sum = 0.0f, p_hat_sel = 0.0f;
    int sel_i = -1;
    bool sel_env = false;
    LightSample sel_XL{};

    for (int i = 1; i < 4; ++i) {
        f3 V = normalize(prev - X.pos);
        // Submit NEE path (SH/PT_1_InitPass.wgsl:1407-1422)
        ch.nee_seed[i] = seed;
        LightSample XL = sample_nee(sc, seed, X, V);
        f3 L = direction_to_light(X, XL);
        f3 contrib = f * l_emit<false>(XL, X);
        contrib = contrib * bsdf(X, V, L);
        contrib = contrib * fabsf(dot(X.nrm, L));
        contrib = contrib * visibility<COUNT>(sc, X.pos, XL.pos, eps, stack, BLOCK);
        float p_hat = luminance(contrib);
        float ris = p_hat / (p * XL.pdf);
        C += 1u;  // UpdateReservoir (SH/PT_1_InitPass.wgsl:1298-1320)
        w_sum += ris;
        if (rnd(seed) < ris / w_sum) { sel_i = i; sel_env = false; sel_XL = XL; p_hat_sel = p_hat; }
        if (i == 3) break;
        // Sample BSDF (SH/PT_1_InitPass.wgsl:1427-1433)
        ch.bsdf_seed[i] = seed;
        uint32_t lobe;
        L = sample_bsdf(seed, X, V, lobe);
        ch.lobe[i] = lobe;
        // throughput and Russian roulette (SH/PT_1_InitPass.wgsl:1436-1442)
        f = f * (bsdf(X, V, L) * fabsf(dot(X.nrm, L)));
        p *= pdf_bsdf(X, V, L);
        float p_survive = luminance(f) / p;
        if (rnd(seed) < p_survive) p *= p_survive;
        else break;
        Hit h = trace_ray<COUNT>(sc, Ray{X.pos, L}, eps, stack, BLOCK);
        if (!h.valid) {  // Submit env path (SH/PT_1_InitPass.wgsl:1447-1461)
            LightSample env;
            env.pos = X.pos + L * INF_F;
            env.type = LIGHT_ENV;
            env.dir = -L;
            env.id = -1;
            env.Le = mk(ENV_C, ENV_C, ENV_C);
            env.pdf = pdf_bsdf(X, V, L);
            float ph = luminance(f * ENV_C);
            float ris_e = ph / p;
            C += 1u;
            w_sum += ris_e;
            if (rnd(seed) < ris_e / w_sum) { sel_i = i; sel_env = true; sel_XL = env; p_hat_sel = ph; }
            break;
        }
        ch.cs[i + 1] = h.s;
        prev = X.pos;
        X = get_surface(sc, h.s);
        ch.pos[i + 1] = X.pos;
        ch.rough[i + 1] = X.mat.rough;
    }
    store_reservoir(out, ch, sel_i, sel_env, sel_XL, w_sum / p_hat_sel, C);
}

// =========================================================================== PT_4
template <bool COUNT>
__global__ __launch_bounds__(BLOCK) void final_kernel(Scene sc, const uint4 *gbuf, const uint4 *reservoir,
                                                      float4 *accum) {
    uint32_t x, y;
    if (!pixel_of(sc, x, y)) return;
    uint32_t *stack = lds_stack + threadIdx.x;
    const size_t pi = band_index(sc, x, y);
    Compact x1 = decode(gbuf[pi]);
    if (!x1.valid) { accum[pi] = make_float4(ENV_C, ENV_C, ENV_C, 1.0f); return; }
    const uint4 *res = reservoir + 8u * pi;
    uint4 r0 = res[0], r1 = res[1], r2 = res[2], r3 = res[3], r5 = res[5], r7 = res[7];
    const uint32_t length = r5.w, C = r7.y;
    if (C == 0u || length < 2u) { write_color(sc, accum, pi, mk(0.0f, 0.0f, 0.0f)); return; }
    const PassEps eps{1e-4f, 1e-8f};
    LightSample XL;
    XL.dir = mk(asf(r1.x), asf(r1.y), asf(r1.z));
    XL.type = r1.w;
    XL.pos = mk(asf(r2.x), asf(r2.y), asf(r2.z));
    XL.id = (int32_t)r2.w;
    XL.Le = mk(asf(r3.x), asf(r3.y), asf(r3.z));
    XL.pdf = asf(r3.w);
    const uint32_t seeds[4] = {r0.x, r0.y, r0.z, r0.w};
    // RegeneratePath + PathContribution (SH/PT_4_FinalShadingPass.wgsl:1306-1384), fused:
    // the product over intermediate vertices is accumulated as vertices are regenerated.
    f3 prev = get_x0(sc, x, y);
    Surface cur = get_surface(sc, x1);
    f3 f = mk(1.0f, 1.0f, 1.0f);
    for (uint32_t i = 1; i + 1u < length; ++i) {
        f3 V = normalize(prev - cur.pos);
        uint32_t seed = seeds[i - 1u];
        uint32_t lobe;
        f3 dir = sample_bsdf(seed, cur, V, lobe);
        Hit h = trace_ray<COUNT>(sc, Ray{cur.pos, dir}, eps, stack, BLOCK);
        Surface next = get_surface(sc, h.s);  // a miss decodes the zero CompactSurface (WGSL behaviour)
        f3 L = normalize(next.pos - cur.pos);
        f = f * (bsdf(cur, L, V) * fabsf(dot(cur.nrm, L)));
        prev = cur.pos;
        cur = next;
    }
    f3 V = normalize(prev - cur.pos);
    f3 L = direction_to_light(cur, XL);
    f = f * (bsdf(cur, L, V) * fabsf(dot(cur.nrm, L)));
    f = f * (l_emit<true>(XL, cur) * visibility<COUNT>(sc, cur.pos, XL.pos, eps, stack, BLOCK));
    write_color(sc, accum, pi, f * asf(r7.x));
}

// =========================================================================== TEST_MCPT
template <bool COUNT>
__global__ __launch_bounds__(BLOCK) void mcpt_kernel(Scene sc, float4 *accum) {
    uint32_t x, y;
    if (!pixel_of(sc, x, y)) return;
    uint32_t *stack = lds_stack + threadIdx.x;
    const size_t pi = band_index(sc, x, y);
    const PassEps eps{1e-4f, 1e-8f};
    uint32_t seed = init_seed(sc, x, y);
    Ray r = camera_ray(sc, x, y);
    f3 color = mk(0.0f, 0.0f, 0.0f), f = mk(1.0f, 1.0f, 1.0f);
    float p = 1.0f;
    const uint32_t nl = sc.U[U_LIGHT_COUNT];
    for (int bounce = 0; bounce < 3; ++bounce) {
        Hit h = trace_ray<COUNT>(sc, r, eps, stack, BLOCK);
        if (!h.valid) { color = color + (f / p) * ENV_C; break; }
        Surface X = get_surface(sc, h.s);
        f3 V = normalize(r.o - X.pos);
        for (uint32_t id = 0; id < nl; ++id) {  // GetLightColor (SH/TEST_MCPT.wgsl:1261-1309)
            Light ls = get_light(sc, id);
            LightSample XL;
            XL.type = ls.type;
            XL.Le = ls.color * ls.intensity;
            XL.pos = mk(0.0f, 0.0f, 0.0f);
            XL.dir = mk(0.0f, 0.0f, 0.0f);
            XL.pdf = 0.0f;
            if (ls.type == LIGHT_DIRECTION) {
                XL.pos = X.pos - ls.dir * INF_F; XL.dir = ls.dir; XL.pdf = 1.0f;
            } else if (ls.type == LIGHT_POINT) {
                XL.pos = ls.pos; XL.dir = normalize(X.pos - ls.pos); XL.pdf = 1.0f;
            } else if (ls.type == LIGHT_RECT) {
                float ru = rnd(seed) * 2.0f - 1.0f;
                float rv = rnd(seed) * 2.0f - 1.0f;
                XL.pos = ls.pos + (ls.U * ru + ls.V * rv);
                XL.dir = normalize(X.pos - XL.pos);
                f3 rr = XL.pos - X.pos;
                f3 Ld = normalize(rr);
                XL.pdf = dot(rr, rr) / fmaxf(ls.area * fabsf(dot(ls.dir, Ld)), EPS_F);
            }
            f3 L = direction_to_light(X, XL);
            f3 c = l_emit<false>(XL, X) * bsdf(X, V, L);
            c = c * fabsf(dot(X.nrm, L));
            c = c * visibility<COUNT>(sc, X.pos, XL.pos, eps, stack, BLOCK);
            color = color + (f / p) * (c / XL.pdf);
        }
        uint32_t lobe;
        f3 L = sample_bsdf(seed, X, V, lobe);
        f = f * (bsdf(X, V, L) * fabsf(dot(X.nrm, L)));
        p *= pdf_bsdf(X, V, L);
        r = Ray{X.pos, L};
        float ps = luminance(f) / p;
        if (rnd(seed) < ps) p *= ps;
        else break;
    }
    write_color(sc, accum, pi, color);
}

// =========================================================================== launches
static dim3 grid_of(const Scene &sc) {
    return dim3((sc.width + TILE - 1) / TILE, (sc.row_end - sc.row_begin + TILE - 1) / TILE, 1);
}
hipError_t launch_gbuffer(const Scene &sc, uint4 *gbuf, uint32_t depth, hipStream_t s) {
    const bool tables_fit = tables_fit_lds(sc);
    if (sc.counters)
        hipLaunchKernelGGL(gbuffer_kernel<true>, grid_of(sc), dim3(BLOCK), stack_lds_bytes(depth), s, sc, gbuf);
    else if (tables_fit)
        hipLaunchKernelGGL((gbuffer_kernel<false, true>), grid_of(sc), dim3(BLOCK),
                           tables_lds_bytes(sc) + stack_lds_bytes(depth), s, sc, gbuf);
    else
        hipLaunchKernelGGL(gbuffer_kernel<false>, grid_of(sc), dim3(BLOCK), stack_lds_bytes(depth), s, sc, gbuf);
    return hipGetLastError();
}
hipError_t launch_init(const Scene &sc, const uint4 *gbuf, uint4 *reservoir, uint32_t depth, hipStream_t s) {
    if (sc.counters) hipLaunchKernelGGL(init_kernel<true>, grid_of(sc), dim3(BLOCK), stack_lds_bytes(depth), s, sc, gbuf, reservoir);
    else hipLaunchKernelGGL(init_kernel<false>, grid_of(sc), dim3(BLOCK), stack_lds_bytes(depth), s, sc, gbuf, reservoir);
    return hipGetLastError();
}
hipError_t launch_final(const Scene &sc, const uint4 *gbuf, const uint4 *reservoir, float4 *accum, uint32_t depth,
                        hipStream_t s) {
    if (sc.counters) hipLaunchKernelGGL(final_kernel<true>, grid_of(sc), dim3(BLOCK), stack_lds_bytes(depth), s, sc, gbuf, reservoir, accum);
    else hipLaunchKernelGGL(final_kernel<false>, grid_of(sc), dim3(BLOCK), stack_lds_bytes(depth), s, sc, gbuf, reservoir,
                       accum);
    return hipGetLastError();
}
hipError_t launch_mcpt(const Scene &sc, float4 *accum, uint32_t depth, hipStream_t s) {
    if (sc.counters) hipLaunchKernelGGL(mcpt_kernel<true>, grid_of(sc), dim3(BLOCK), stack_lds_bytes(depth), s, sc, accum);
    else hipLaunchKernelGGL(mcpt_kernel<false>, grid_of(sc), dim3(BLOCK), stack_lds_bytes(depth), s, sc, accum);
    return hipGetLastError();
}

// =========================================================================== ray queries
// One thread per ray; the traversal is trace_core (same code as every pass).
template <bool COUNT>
__global__ __launch_bounds__(BLOCK) void trace_rays_kernel(Scene sc, const float4 *rays, float4 *hits, uint32_t n,
                                                           PassEps eps) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    uint32_t *stack = lds_stack + threadIdx.x;
    const float4 a = rays[2u * i], b = rays[2u * i + 1u];
    Hit h = trace_core<COUNT>(sc, Ray{mk(a.x, a.y, a.z), mk(a.w, b.x, b.y)}, eps, stack, BLOCK);
    const uint32_t enc = ((h.valid ? 1u : 0u) << 31) | (h.s.inst << 16) | h.s.mat;
    hits[2u * i] = make_float4(h.t, asf(enc), asf(h.s.prim), h.s.bu);
    hits[2u * i + 1u] = make_float4(h.s.bv, h.pos.x, h.pos.y, h.pos.z);
}
hipError_t launch_trace_rays(const Scene &sc, const float4 *rays, float4 *hits, uint32_t n, int eps_mode,
                             uint32_t depth, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const PassEps eps = eps_mode == 0 ? PassEps{1e-8f, 1e-6f} : PassEps{1e-4f, 1e-8f};
    const dim3 grid((n + BLOCK - 1) / BLOCK);
    if (sc.counters)
        hipLaunchKernelGGL(trace_rays_kernel<true>, grid, dim3(BLOCK), stack_lds_bytes(depth), s, sc, rays, hits, n, eps);
    else
        hipLaunchKernelGGL(trace_rays_kernel<false>, grid, dim3(BLOCK), stack_lds_bytes(depth), s, sc, rays, hits, n, eps);
    return hipGetLastError();
}

// ---------------------------------------------------------------- present (the reference's render pass)
// Renderer_TEST.Render's render pass (GC/Renderer_TEST.ts:233-255) draws a fullscreen quad
// (SH/VertexShader.wgsl: PixelUV = (NDC + 1) / 2) whose fragment shader loads texel
// (floor(PixelUV.x * 600), floor(PixelUV.y * 450)) of the Scene texture -- a fixed 600 x 450
// window whatever the canvas size (SH/FragmentShader.wgsl:7-10) -- and writes rgb with alpha 1
// to the canvas (its preferred format, unorm8).  Canvas pixel (px, py), py = 0 the top row, is
// the fragment at NDC y = 1 - (2 py + 1) / ch, so PixelUV = ((2 px + 1) / 2cw, 1 - (2 py + 1) / 2ch):
// the texel is floor((2 px + 1) * 600 / 2cw), floor((2 ch - 2 py - 1) * 450 / 2ch) in exact
// integer arithmetic (the rasterizer's own rounding of PixelUV is implementation-defined, and
// matters only where the product is an exact integer).  A texel outside the texture reads as
// 0 (WGSL leaves out-of-bounds textureLoad implementation-defined).  unorm8: clamp to [0, 1],
// x * 255 rounded to nearest even (NaN -> 0).  bgra: the byte order of a bgra8unorm canvas.
__device__ __forceinline__ uint32_t unorm8(float x) {
    const float c = fminf(fmaxf(x, 0.0f), 1.0f);  // (NaN -> 0: maxNum)
    return (uint32_t)__builtin_rintf(c * 255.0f);
}
__global__ __launch_bounds__(BLOCK) void present_kernel(const float4 *tex, uint32_t W, uint32_t H, uint32_t cw,
                                                        uint32_t ch, uint32_t bgra, uint32_t *out) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= cw * ch) return;
    const uint32_t px = i % cw, py = i / cw;
    const uint64_t tx = ((uint64_t)(2u * px + 1u) * 600u) / (2ull * cw);
    const uint64_t ty = ((uint64_t)(2u * ch - 2u * py - 1u) * 450u) / (2ull * ch);
    float4 c = make_float4(0.0f, 0.0f, 0.0f, 1.0f);
    if (tx < W && ty < H) c = tex[ty * W + tx];
    const uint32_t r = unorm8(c.x), g = unorm8(c.y), b = unorm8(c.z);
    out[i] = bgra ? (b | (g << 8) | (r << 16) | (255u << 24)) : (r | (g << 8) | (b << 16) | (255u << 24));
}
hipError_t launch_present(const float4 *tex, uint32_t W, uint32_t H, uint32_t cw, uint32_t ch, bool bgra,
                          uint32_t *out, hipStream_t s) {
    const uint32_t n = cw * ch;
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(present_kernel, dim3((n + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, s, tex, W, H, cw, ch,
                       bgra ? 1u : 0u, out);
    return hipGetLastError();
}

}  // namespace ptx
