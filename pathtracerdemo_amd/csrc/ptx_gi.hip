// ptx_gi.hip -- ReSTIR GI (BASELINE configs[4]: 1-bounce indirect reservoirs) in wavefront form.
//
// Build-defined (no reference code; the rules are oracle/pt_oracle_gi.c's):
// the reconnection shift of docs/theory/memo.md:166-231 at x2 on top of the reference's
// GetSurface / SampleNEE / L_emit / Visibility / BSDF (SH/PT_1_InitPass.wgsl:285-1260).
// Every reservoir, direct-light texel and pixel these kernels write is bit-identical to
// the oracle's.
//
//   init      wgi_start (NEE shadow ray + candidate ray per pixel) -> trace ->
//             wgi_step<1> (direct light; x2: NEE shadow ray from x2) -> trace -> wgi_step<2>
//   temporal  wgi_temporal: per pixel, no rays (identity shift, stored contributions)
//   spatial   wgis_start (2 shift jobs per neighbour, ONE occlusion ray each, the job's
//             contribution and q riding in the ray's result slot) -> trace -> wgis_combine
//   final     wgi_final: direct + f * W, accumulated
// Same segment queues and trace_queue as the other passes; the shift's binary visibility
// is the Q_OCC query kind (closest hit, any surface occludes).
#include "ptx_wave_common.h"

namespace ptx {

constexpr uint32_t SALT_GI = 0x47494E49u, SALT_GI_TEMPORAL = 0x47495450u, SALT_GI_SPATIAL = 0x47495350u;
constexpr float GI_VIS_SHORTEN = 0.999f, FLT_MAX_F = 3.402823466e38f;
constexpr uint32_t GI_NO_RAY = 0xffffffffu;

// init pixel state (SoA float4 slots of w.state)
enum : uint32_t { GS_B1, GS_X1, GS_L1, GS_X2, GS_L2, GS_COUNT };
static_assert(GS_COUNT <= kWaveStateSlots, "GI init state exceeds the wavefront state slots");

__device__ __forceinline__ float gi_q(f3 y, const Surface &X2) {
    const f3 r = X2.pos - y;
    return dot(r, r) / fabsf(dot(X2.nrm, normalize(r)));
}
__device__ __forceinline__ f3 gi_lo(const Surface &X2, f3 V2, f3 L2, f3 lt) {
    return (bsdf(X2, V2, L2) * lt) * fabsf(dot(X2.nrm, L2));
}
__device__ __forceinline__ bool gi_q_ok(float q) { return q > 0.0f && q <= FLT_MAX_F; }
// two-sided cosine candidate direction with its exact pdf (oracle gi_sample_dir)
__device__ __forceinline__ f3 gi_sample_dir(uint32_t &seed, const Surface &X, f3 V, float &pdf) {
    const float T = X.mat.trans;
    f3 N = dot(V, X.nrm) >= 0.0f ? X.nrm : -X.nrm;
    if (rnd(seed) < T) N = -N;
    const f3 L = tbn_mul(tbn(N), sample_cosine(seed));
    const bool same = dot(L, X.nrm) * dot(V, X.nrm) > 0.0f;
    pdf = ((same ? 1.0f - T : T) * fabsf(dot(X.nrm, L))) / PI_F;
    return L;
}
__device__ __forceinline__ f3 ld3(const uint4 &v) { return mk(asf(v.x), asf(v.y), asf(v.z)); }

// the candidate reservoir (oracle gi_init_pixel's tail): one-candidate RIS, C = 1
__device__ __forceinline__ void gi_store_candidate(uint4 *out, uint4 x2, f3 dir, f3 lt, f3 f, float q, float pdf1) {
    const float p_hat = luminance(f);
    const float w_sum = pdf1 > 0.0f ? p_hat / pdf1 : 0.0f;
    const bool ok = p_hat > 0.0f && gi_q_ok(q) && w_sum > 0.0f && w_sum <= FLT_MAX_F;
    out[0] = x2;
    out[1] = make_uint4(asu(dir.x), asu(dir.y), asu(dir.z), asu(ok ? w_sum / p_hat : 0.0f));
    out[2] = make_uint4(asu(lt.x), asu(lt.y), asu(lt.z), 1u);
    out[3] = make_uint4(asu(f.x), asu(f.y), asu(f.z), asu(q));
}

// ---------------------------------------------------------------- init
__global__ __launch_bounds__(WB) __attribute__((amdgpu_waves_per_eu(LOGIC_WAVES, 8)))
void wgi_start(Scene sc, WaveBufs w, GiArgs A) {
    __shared__ uint32_t lds[2];
    const Seg g = seg_begin(w, 0u, lds);
    const uint32_t npix = w.npix, np = padded_pixels(sc);
    for (uint32_t k = 0; k < w.seg_px; k += WB) {
        const uint32_t q = seg_pixel(w, g.j, k);
        uint32_t x, y, pix = 0u;
        bool active = false;
        f3 xl_pos{}, u{}, L1{}, b1{};
        Surface X1;
        float pdf1 = 0.0f;
        uint32_t seed = 0u;
        if (q < np && tile_xy(sc, q, x, y)) {
            pix = (y - sc.row_begin) * sc.width + x;
            const Compact x1 = gdecode(A.gbuf[pix]);
            if (!x1.valid) {
                uint4 *out = A.cur + 4u * (size_t)pix;
                for (int t = 0; t < 4; ++t) out[t] = make_uint4(0u, 0u, 0u, 0u);
                A.direct[pix] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            } else {
                active = true;
                seed = pcg(pcg(x * 1973u + y * 9277u + sc.U[U_FRAME] * 26699u) ^ SALT_GI);
                X1 = get_surface(sc, x1);
                const f3 V1 = normalize(x0_of(sc, x, y) - X1.pos);
                const LightSample XL = sample_nee(sc, seed, X1, V1);
                const f3 L = direction_to_light(X1, XL);
                u = (l_emit<false>(XL, X1) * bsdf(X1, V1, L)) * fabsf(dot(X1.nrm, L));
                u = XL.pdf > 0.0f ? u / XL.pdf : mk(0.0f, 0.0f, 0.0f);
                xl_pos = XL.pos;
                L1 = gi_sample_dir(seed, X1, V1, pdf1);
                b1 = bsdf(X1, V1, L1) * fabsf(dot(X1.nrm, L1));
            }
        }
        // two rays per active pixel: [base] the direct light's Visibility, [base+1] the candidate
        const uint32_t base = g.rbase + wave_alloc(g.l_ray, active ? 2u : 0u);
        if (active) {
            const float dist = length(xl_pos - X1.pos);
            put_ray(g.rays, base, X1.pos, (xl_pos - X1.pos) / dist, dist, Q_VIS);
            g.res_out[2u * base] = make_float4(0.0f, u.x, u.y, u.z);
            put_ray(g.rays, base + 1u, X1.pos, L1, -1.0f, Q_CLOSEST);
            float4 *st = w.state;
            st[GS_B1 * npix + pix] = make_float4(b1.x, b1.y, b1.z, pdf1);
            st[GS_X1 * npix + pix] = make_float4(X1.pos.x, X1.pos.y, X1.pos.z, asf(seed));
            st[GS_L1 * npix + pix] = make_float4(asf(base), L1.x, L1.y, L1.z);
        }
        seg_keep(g, active, pix);
    }
    seg_end(w, g);
}

// ROUND 1: direct light + the candidate's hit (NEE from x2 or the environment);
// ROUND 2: x2's light Visibility -> the candidate reservoir.
template <int ROUND>
__global__ __launch_bounds__(WB) __attribute__((amdgpu_waves_per_eu(LOGIC_WAVES, 8)))
void wgi_step(Scene sc, WaveBufs w, GiArgs A) {
    __shared__ uint32_t lds[2];
    const Seg g = seg_begin(w, (uint32_t)ROUND, lds);
    const uint32_t npix = w.npix, n = g.n_in;
    float4 *st = w.state;
    for (uint32_t b0 = 0; b0 < n; b0 += WB) {
        const uint32_t qi = b0 + threadIdx.x;
        bool emit = false;
        uint32_t pix = 0u;
        f3 o{}, xl_pos{}, lt{};
        if (qi < n) {
            pix = g.act_in[qi];
            const float4 sb = st[GS_B1 * npix + pix], sx = st[GS_X1 * npix + pix];
            const f3 b1 = mk(sb.x, sb.y, sb.z), x1pos = mk(sx.x, sx.y, sx.z);
            uint4 *out = A.cur + 4u * (size_t)pix;
            if (ROUND == 1) {
                const float4 sl = st[GS_L1 * npix + pix];
                const uint32_t base = asu(sl.x);
                const float4 a = g.res_in[2u * base];
                const f3 d = mk(a.y, a.z, a.w) * a.x;
                A.direct[pix] = make_float4(d.x, d.y, d.z, 0.0f);
                const Hit h = get_hit(g.res_in, base + 1u);
                if (!h.valid) {  // escapes: the environment in direction L1
                    const f3 L1 = mk(sl.y, sl.z, sl.w);
                    gi_store_candidate(out, make_uint4(0u, 0u, 0u, 0u), L1, mk(0.0f, 0.0f, 0.0f), b1 * ENV_C, 1.0f,
                                       sb.w);
                } else {
                    uint32_t seed = asu(sx.w);
                    const Surface X2 = surface_at(sc, h.s, h.pos);
                    const f3 V2 = normalize(x1pos - X2.pos);
                    const LightSample XL2 = sample_nee(sc, seed, X2, V2);
                    const f3 L2 = direction_to_light(X2, XL2);
                    lt = l_emit<false>(XL2, X2);
                    lt = XL2.pdf > 0.0f ? lt / XL2.pdf : mk(0.0f, 0.0f, 0.0f);
                    o = X2.pos;
                    xl_pos = XL2.pos;
                    uint4 c = gencode(h.s);
                    c.x |= 0x80000000u;
                    st[GS_X2 * npix + pix] = make_float4(asf(c.x), asf(c.y), asf(c.z), asf(c.w));
                    st[GS_L2 * npix + pix] = make_float4(L2.x, L2.y, L2.z, 0.0f);
                    emit = true;
                }
            } else {
                const float4 s2 = st[GS_X2 * npix + pix], sl2 = st[GS_L2 * npix + pix];
                const uint4 c = make_uint4(asu(s2.x), asu(s2.y), asu(s2.z), asu(s2.w));
                const float4 a = g.res_in[2u * asu(sl2.w)];
                const f3 ltv = mk(a.y, a.z, a.w) * a.x;
                const f3 L2 = mk(sl2.x, sl2.y, sl2.z);
                const Surface X2 = get_surface(sc, gdecode(c));
                const f3 V2 = normalize(x1pos - X2.pos);
                const f3 f = b1 * gi_lo(X2, V2, L2, ltv);
                gi_store_candidate(out, c, L2, ltv, f, gi_q(x1pos, X2), sb.w);
            }
        }
        const uint32_t idx = g.rbase + wave_alloc(g.l_ray, emit ? 1u : 0u);
        if (emit) {
            const float dist = length(xl_pos - o);
            put_ray(g.rays, idx, o, (xl_pos - o) / dist, dist, Q_VIS);
            g.res_out[2u * idx] = make_float4(0.0f, lt.x, lt.y, lt.z);
            st[GS_L2 * npix + pix].w = asf(idx);
        }
        seg_keep(g, emit, pix);
    }
    seg_end(w, g);
}

// ---------------------------------------------------------------- temporal
__device__ __forceinline__ uint32_t gi_seed(const Scene &sc, uint32_t x, uint32_t y, uint32_t salt) {
    return pcg(pcg(x * 1973u + y * 9277u + sc.U[U_FRAME] * 26699u) ^ salt);
}
// reservoir `src`'s sample (words 0..10) with contribution f, q, W = w_sum / p_hat(f), C
__device__ __forceinline__ void gi_write(uint4 *out, const uint4 *src, f3 f, float q, float w_sum, uint32_t C) {
    const uint4 s0 = src[0], s1 = src[1], s2 = src[2];  // src may be out itself
    const float p = luminance(f);
    out[0] = s0;
    out[1] = make_uint4(s1.x, s1.y, s1.z, asu(p > 0.0f ? w_sum / p : 0.0f));
    out[2] = make_uint4(s2.x, s2.y, s2.z, C);
    out[3] = make_uint4(asu(f.x), asu(f.y), asu(f.z), asu(q));
}

__global__ __launch_bounds__(WB) void wgi_temporal(Scene sc, WaveBufs w, GiArgs A) {
    const uint32_t j = w.seg_base + blockIdx.x, np = padded_pixels(sc);
    for (uint32_t k = 0; k < w.seg_px; k += WB) {
        const uint32_t q = seg_pixel(w, j, k);
        uint32_t x, y;
        if (q >= np || !tile_xy(sc, q, x, y)) continue;
        const uint32_t pix = (y - sc.row_begin) * sc.width + x;
        if (!gdecode(A.gbuf[pix]).valid) continue;
        uint4 *cur = A.cur + 4u * (size_t)pix;
        const uint4 *hist = A.hist + 4u * (size_t)pix;
        uint32_t seed = gi_seed(sc, x, y, SALT_GI_TEMPORAL);
        const uint4 c1 = cur[1], c2 = cur[2], c3 = cur[3], h1 = hist[1], h2 = hist[2], h3 = hist[3];
        const float pc = luminance(ld3(c3)), ph = luminance(ld3(h3));
        const bool canon_ok = c2.w != 0u && pc > 0.0f;
        const uint32_t Cp = A.hist_valid ? min(h2.w, A.cap) : 0u;
        const float cp = (float)Cp, tot = 1.0f + cp;
        const bool hist_ok = Cp != 0u && ph > 0.0f;
        const float wc = canon_ok ? (1.0f / tot) * pc * asf(c1.w) : 0.0f;
        const float wp = hist_ok ? (cp / tot) * ph * asf(h1.w) : 0.0f;
        float w_sum = 0.0f;
        bool from_hist = false;
        w_sum += wc;
        if (rnd(seed) < wc / w_sum) from_hist = false;
        w_sum += wp;
        if (rnd(seed) < wp / w_sum) from_hist = true;
        const uint4 s3 = from_hist ? h3 : c3;
        gi_write(cur, from_hist ? hist : cur, ld3(s3), asf(s3.w), w_sum, 1u + Cp);
    }
}

// ---------------------------------------------------------------- spatial
__device__ __forceinline__ bool gi_neighbor(uint32_t &seed, uint32_t R, uint32_t x, uint32_t y, uint32_t W, uint32_t H,
                                            uint32_t &nx, uint32_t &ny) {  // oracle spatial_neighbor
    const float side = (float)(2u * R + 1u);
    uint32_t ix = (uint32_t)(rnd(seed) * side);
    uint32_t iy = (uint32_t)(rnd(seed) * side);
    ix = min(ix, 2u * R);
    iy = min(iy, 2u * R);
    const int X = (int)x + (int)ix - (int)R, Y = (int)y + (int)iy - (int)R;
    if (X < 0 || Y < 0 || X >= (int)W || Y >= (int)H || (ix == R && iy == R)) return false;
    nx = (uint32_t)X;
    ny = (uint32_t)Y;
    return true;
}
__device__ __forceinline__ int32_t gi_band_index(const Scene &sc, uint32_t x, uint32_t y) {
    return ((int32_t)y - (int32_t)sc.row_begin) * (int32_t)sc.width + (int32_t)x;
}

// The shift of GI reservoir s into domain (x, y) with hit y1, up to its occlusion query
// (oracle gi_shift): false when no such path exists (q invalid).  Split in the two halves
// a pixel's jobs share: the domain (camera point + hit surface: every forward job of a
// pixel) and the sample (x2 surface: every backward job of a pixel).
struct GiDomain { Surface Y; f3 Vy; };
struct GiSample { bool env; f3 dir, lt; Surface X2; };
__device__ __forceinline__ GiDomain gi_domain(const Scene &sc, uint32_t x, uint32_t y, const Compact &y1) {
    GiDomain d;
    d.Y = get_surface(sc, y1);
    d.Vy = normalize(x0_of(sc, x, y) - d.Y.pos);
    return d;
}
__device__ __forceinline__ GiSample gi_sample(const Scene &sc, const uint4 *s) {
    const uint4 s0 = s[0];
    GiSample m;
    m.env = !(s0.x & 0x80000000u);
    m.dir = ld3(s[1]);
    m.lt = ld3(s[2]);
    if (!m.env) m.X2 = get_surface(sc, gdecode(s0));
    return m;
}
__device__ __forceinline__ bool gi_shift_begin(const GiDomain &d, const GiSample &m, f3 &f, float &q, f3 &o,
                                               f3 &dir, float &remain) {
    if (m.env) {
        dir = m.dir;
        f = (bsdf(d.Y, d.Vy, dir) * fabsf(dot(d.Y.nrm, dir))) * ENV_C;
        q = 1.0f;
        remain = FLT_MAX_F;
    } else {
        const f3 r = m.X2.pos - d.Y.pos;
        const float dist = length(r);
        dir = r / dist;
        const f3 V2 = normalize(d.Y.pos - m.X2.pos);
        f = (bsdf(d.Y, d.Vy, dir) * fabsf(dot(d.Y.nrm, dir))) * gi_lo(m.X2, V2, m.dir, m.lt);
        q = gi_q(d.Y.pos, m.X2);
        remain = dist * GI_VIS_SHORTEN;
    }
    o = d.Y.pos;
    return gi_q_ok(q);
}

// the spatial pass's job (pixel, slot): slot 2m forward from neighbour m, 2m + 1 backward
__device__ __forceinline__ uint32_t gi_jid(const GiArgs &A, uint32_t pix, uint32_t slot) {
    return pix * A.jpx + slot * A.jslot;
}

// The jobs of one pixel of one kind (workgroup-uniform): forward jobs (slot 2m: neighbour
// m's sample -> this pixel) share this pixel's domain, backward jobs (2m+1: this pixel's
// sample -> neighbour m) its sample; each job's contribution and q ride in its ray's
// result slot.  Called by every lane of the wave (wave_alloc).
template <bool BACKWARD>
__device__ __forceinline__ void gis_pixel_jobs(const Scene &sc, const Seg &g, const GiArgs &A, bool valid, uint32_t x,
                                               uint32_t y, uint32_t pix, const Compact &x1) {
    uint32_t seed = valid ? gi_seed(sc, x, y, SALT_GI_SPATIAL) : 0u;
    bool own_ok = false;
    GiDomain D{};
    GiSample S{};
    if (valid && !BACKWARD) D = gi_domain(sc, x, y, x1);
    if (valid && BACKWARD) {
        const uint4 *rc = A.cur + 4u * (size_t)pix;
        own_ok = rc[2].w != 0u && luminance(ld3(rc[3])) > 0.0f;
        if (own_ok) S = gi_sample(sc, rc);
    }
    for (uint32_t m = 0; m < A.neighbors; ++m) {  // uniform
        const uint32_t jid = gi_jid(A, pix, 2u * m + (BACKWARD ? 1u : 0u));
        bool ray = false;
        f3 f{}, o{}, dir{};
        float qv = 0.0f, remain = 0.0f;
        if (valid) {
            uint32_t nx = 0u, ny = 0u;
            bool present = gi_neighbor(seed, A.radius, x, y, sc.width, sc.height, nx, ny);
            const int32_t nidx = present ? gi_band_index(sc, nx, ny) : 0;
            Compact xn{};
            if (present) {
                xn = gdecode(A.gbuf[nidx]);
                present = xn.valid != 0u;
            }
            if (BACKWARD) {
                if (present && own_ok) ray = gi_shift_begin(gi_domain(sc, nx, ny, xn), S, f, qv, o, dir, remain);
            } else if (present) {  // (the neighbour's confidence is >= 1: it has a G-buffer hit)
                const uint4 *rn = A.cur + 4 * (ptrdiff_t)nidx;
                if (luminance(ld3(rn[3])) > 0.0f) ray = gi_shift_begin(D, gi_sample(sc, rn), f, qv, o, dir, remain);
            }
        }
        const uint32_t idx = g.rbase + wave_alloc(g.l_ray, ray ? 1u : 0u);
        if (ray) {
            put_ray(g.rays, idx, o, dir, remain, Q_OCC);
            g.res_out[2u * idx] = make_float4(0.0f, f.x, f.y, f.z);
            g.res_out[2u * idx + 1u] = make_float4(qv, 0.0f, 0.0f, 0.0f);
        }
        if (valid) A.jray[jid] = ray ? idx : GI_NO_RAY;
    }
}

#ifndef GIS_START_WAVES
#define GIS_START_WAVES 3  // 3: 168 VGPRs, 12 B/lane spilled; 4: 128 VGPRs, 148 B spilled
#endif
__global__ __launch_bounds__(WB) __attribute__((amdgpu_waves_per_eu(GIS_START_WAVES, 8)))
void wgis_start(Scene sc, WaveBufs w, GiArgs A) {
    __shared__ uint32_t lds[2];
    const Seg g = seg_begin(w, 0u, lds);
    const uint32_t np = padded_pixels(sc);
    for (uint32_t base = 0; base < w.seg_px * 2u; base += WB) {  // workgroup-uniform: kind, then pixels
        const uint32_t q = seg_pixel(w, g.j, base % w.seg_px);
        uint32_t x = 0u, y = 0u, pix = 0u;
        Compact x1{};
        if (q < np && tile_xy(sc, q, x, y)) {
            pix = (y - sc.row_begin) * sc.width + x;
            x1 = gdecode(A.gbuf[pix]);
        }
        if (base >= w.seg_px) gis_pixel_jobs<true>(sc, g, A, x1.valid != 0u, x, y, pix, x1);
        else gis_pixel_jobs<false>(sc, g, A, x1.valid != 0u, x, y, pix, x1);
    }
    seg_end(w, g);
}

// a job's result: valid, contribution (visibility applied), q
__device__ __forceinline__ bool gi_job(const GiArgs &A, const float4 *res, uint32_t jid, f3 &f, float &q) {
    const uint32_t idx = A.jray[jid];
    if (idx == GI_NO_RAY) return false;
    const float4 a = res[2u * idx], b = res[2u * idx + 1u];
    f = mk(a.y, a.z, a.w) * a.x;
    q = b.x;
    return true;
}

// Pairwise-MIS resampling (oracle gi_spatial_pixel); res = trace round 0's results.
// MT = the neighbour count when it is a compile-time constant (the default 3): every
// neighbour's G-buffer word, reservoir and job ray index are loaded in one round trip and
// the job results in a second, instead of ~3 dependent loads per neighbour and pass;
// MT = 0: any count, per neighbour (the same arithmetic in the same order either way).
template <uint32_t MT>
__device__ __forceinline__ void gis_combine_pixel(const Scene &sc, const GiArgs &A, const float4 *res, uint32_t x,
                                                  uint32_t y, uint32_t pix) {
    uint4 *out = A.hist + 4u * (size_t)pix;
    const uint32_t M = MT ? MT : A.neighbors;
    if constexpr (MT > 0) {
        const uint4 *rc = A.cur + 4u * (size_t)pix;
        const uint4 c1 = rc[1], c2 = rc[2], c3 = rc[3];
        const float Mf = (float)M, cc = (float)c2.w;
        const f3 fcv = ld3(c3);
        const float pc = luminance(fcv), qc = asf(c3.w), Wc = asf(c1.w);
        const bool canon_ok = c2.w != 0u && pc > 0.0f;
        const uint32_t seed0 = gi_seed(sc, x, y, SALT_GI_SPATIAL);
        uint32_t seed = seed0, Csum = c2.w;
        int32_t nid[MT];
        bool pres[MT];
#pragma unroll
        for (uint32_t m = 0; m < MT; ++m) {
            uint32_t nx = 0u, ny = 0u;
            pres[m] = gi_neighbor(seed, A.radius, x, y, sc.width, sc.height, nx, ny);
            nid[m] = pres[m] ? gi_band_index(sc, nx, ny) : (int32_t)pix;
        }
        uint32_t gv[MT], jf[MT], jb[MT];
        uint4 n1[MT], n2[MT], n3[MT];
#pragma unroll
        for (uint32_t m = 0; m < MT; ++m) {
            const uint4 *rn = A.cur + 4 * (ptrdiff_t)nid[m];
            gv[m] = A.gbuf[nid[m]].x;
            n1[m] = rn[1]; n2[m] = rn[2]; n3[m] = rn[3];
            jf[m] = A.jray[gi_jid(A, pix, 2u * m)];
            jb[m] = A.jray[gi_jid(A, pix, 2u * m + 1u)];
        }
        bool valid[MT], hf[MT], hb[MT];
        float pn[MT];
        float4 fa[MT], fb[MT], ba[MT], bb[MT];
#pragma unroll
        for (uint32_t m = 0; m < MT; ++m) {  // (a job index is read only where gi_job would read it)
            valid[m] = pres[m] && (gv[m] >> 31) != 0u;
            pn[m] = luminance(ld3(n3[m]));
            hb[m] = valid[m] && canon_ok && jb[m] != GI_NO_RAY;
            hf[m] = valid[m] && pn[m] > 0.0f && jf[m] != GI_NO_RAY;
            ba[m] = bb[m] = fa[m] = fb[m] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            if (hb[m]) { ba[m] = res[2u * jb[m]]; bb[m] = res[2u * jb[m] + 1u]; }
            if (hf[m]) { fa[m] = res[2u * jf[m]]; fb[m] = res[2u * jf[m] + 1u]; }
        }
        float sumQ = 0.0f;
#pragma unroll
        for (uint32_t m = 0; m < MT; ++m) {  // confidences + the canonical MIS weight
            float Q = 1.0f;
            if (valid[m]) {
                const uint32_t Cn = n2[m].w;
                Csum += Cn;
                if (hb[m]) {
                    const f3 B = mk(ba[m].y, ba[m].z, ba[m].w) * ba[m].x;
                    const float qB = bb[m].x;
                    const float pbc = luminance(B) * qc / qB;
                    const float den = cc * pc + Mf * (float)Cn * pbc;
                    Q = den > 0.0f ? (cc * pc) / den : 1.0f;
                }
            }
            sumQ += Q;
        }
        const float wc = canon_ok ? (sumQ / Mf) * pc * Wc : 0.0f;
        float w_sum = 0.0f;
        const uint4 *src = rc;
        f3 fsel = fcv;
        float qsel = qc;
        w_sum += wc;
        if (rnd(seed) < wc / w_sum) { src = rc; fsel = fcv; qsel = qc; }
#pragma unroll
        for (uint32_t m = 0; m < MT; ++m) {
            float wn = 0.0f;
            f3 F = mk(0.0f, 0.0f, 0.0f);
            float qF = 0.0f;
            if (pres[m] && hf[m]) {
                F = mk(fa[m].y, fa[m].z, fa[m].w) * fa[m].x;
                qF = fb[m].x;
                const float pF = luminance(F);
                const float J = asf(n3[m].w) / qF;
                const float pb = pn[m] / J;
                const float den = cc * pF + Mf * (float)n2[m].w * pb;
                const float mw = den > 0.0f ? ((float)n2[m].w * pb) / den : 0.0f;
                wn = mw * pF * asf(n1[m].w) * J;
            }
            w_sum += wn;
            if (rnd(seed) < wn / w_sum) { src = A.cur + 4 * (ptrdiff_t)(pres[m] ? nid[m] : 0); fsel = F; qsel = qF; }
        }
        gi_write(out, src, fsel, qsel, w_sum, Csum);
    } else {
    const uint4 *rc = A.cur + 4u * (size_t)pix;
    const uint4 c1 = rc[1], c2 = rc[2], c3 = rc[3];
    const float Mf = (float)M, cc = (float)c2.w;
    const f3 fcv = ld3(c3);
    const float pc = luminance(fcv), qc = asf(c3.w), Wc = asf(c1.w);
    const bool canon_ok = c2.w != 0u && pc > 0.0f;
    const uint32_t seed0 = gi_seed(sc, x, y, SALT_GI_SPATIAL);
    uint32_t seed = seed0, Csum = c2.w;
    float sumQ = 0.0f;
    for (uint32_t m = 0; m < M; ++m) {  // confidences + the canonical MIS weight
        uint32_t nx = 0u, ny = 0u;
        float Q = 1.0f;
        if (gi_neighbor(seed, A.radius, x, y, sc.width, sc.height, nx, ny)) {
            const int32_t nidx = gi_band_index(sc, nx, ny);
            if (gdecode(A.gbuf[nidx]).valid) {
                const uint32_t Cn = A.cur[4 * (ptrdiff_t)nidx + 2].w;
                Csum += Cn;
                f3 B;
                float qB;
                if (canon_ok && gi_job(A, res, gi_jid(A, pix, 2u * m + 1u), B, qB)) {
                    const float pbc = luminance(B) * qc / qB;
                    const float den = cc * pc + Mf * (float)Cn * pbc;
                    Q = den > 0.0f ? (cc * pc) / den : 1.0f;
                }
            }
        }
        sumQ += Q;
    }
    const float wc = canon_ok ? (sumQ / Mf) * pc * Wc : 0.0f;
    float w_sum = 0.0f;
    const uint4 *src = rc;
    f3 fsel = fcv;
    float qsel = qc;
    w_sum += wc;
    if (rnd(seed) < wc / w_sum) { src = rc; fsel = fcv; qsel = qc; }
    uint32_t nseed = seed0;
    for (uint32_t m = 0; m < M; ++m) {
        uint32_t nx = 0u, ny = 0u;
        float wn = 0.0f;
        f3 F = mk(0.0f, 0.0f, 0.0f);
        float qF = 0.0f;
        int32_t nidx = 0;
        if (gi_neighbor(nseed, A.radius, x, y, sc.width, sc.height, nx, ny)) {
            nidx = gi_band_index(sc, nx, ny);
            const uint4 *rn = A.cur + 4 * (ptrdiff_t)nidx;
            const uint4 n1 = rn[1], n2 = rn[2], n3 = rn[3];
            const float pn = luminance(ld3(n3));
            if (gdecode(A.gbuf[nidx]).valid && pn > 0.0f && gi_job(A, res, gi_jid(A, pix, 2u * m), F, qF)) {
                const float pF = luminance(F);
                const float J = asf(n3.w) / qF;
                const float pb = pn / J;
                const float den = cc * pF + Mf * (float)n2.w * pb;
                const float mw = den > 0.0f ? ((float)n2.w * pb) / den : 0.0f;
                wn = mw * pF * asf(n1.w) * J;
            } else {
                F = mk(0.0f, 0.0f, 0.0f);
                qF = 0.0f;
            }
        }
        w_sum += wn;
        if (rnd(seed) < wn / w_sum) { src = A.cur + 4 * (ptrdiff_t)nidx; fsel = F; qsel = qF; }
    }
        gi_write(out, src, fsel, qsel, w_sum, Csum);
    }
}
__global__ __launch_bounds__(WB) void wgis_combine(Scene sc, WaveBufs w, GiArgs A) {
    const uint32_t j = w.seg_base + blockIdx.x, np = padded_pixels(sc);
    const float4 *res = w.res[0];
    for (uint32_t k = 0; k < w.seg_px; k += WB) {
        const uint32_t q = seg_pixel(w, j, k);
        uint32_t x, y;
        if (q >= np || !tile_xy(sc, q, x, y)) continue;
        const uint32_t pix = (y - sc.row_begin) * sc.width + x;
        if (!gdecode(A.gbuf[pix]).valid) {
            uint4 *out = A.hist + 4u * (size_t)pix;
            for (int t = 0; t < 4; ++t) out[t] = make_uint4(0u, 0u, 0u, 0u);
            continue;
        }
        if (A.neighbors == 3u) gis_combine_pixel<3>(sc, A, res, x, y, pix);
        else gis_combine_pixel<0>(sc, A, res, x, y, pix);
    }
}

// ---------------------------------------------------------------- temporal, moved camera
// The history of pixel p lives at the reprojection p' of its primary hit in the previous
// frame, in that frame's domain (oracle gi_temporal_motion_pixel; the DI pass's lookup,
// ptx_reuse.hip motion_hist, with the previous frame's G-buffer in place of its surface
// records): the spatial pass's pairwise rule with M = 1 over two occlusion jobs -- slot 0 the
// history sample shifted here, slot 1 this pixel's sample shifted to p' (its MIS weight).
__device__ __forceinline__ f3 gi_x0_prev(const GiArgs &A, const Scene &sc, uint32_t x, uint32_t y) {
    float u = ((float)x + 0.5f) / (float)sc.U[U_W];  // (x0_of with the previous frame's VP^-1)
    float v = ((float)y + 0.5f) / (float)sc.U[U_H];
    return xform_point(A.vpinv_prev, mk(2.0f * u - 1.0f, 2.0f * v - 1.0f, 0.0f));
}
struct GiMotion { bool ok; int32_t pp; uint32_t px, py, C; Compact x1p; };
__device__ __forceinline__ GiMotion gi_motion(const Scene &sc, const GiArgs &A, const Surface &X1, uint32_t y) {
    GiMotion m{false, 0, 0u, 0u, 0u, Compact{}};
    if (!A.hist_valid) return m;
    const float *vp = A.vp_prev;
    const f3 P = X1.pos;
    const float cx = ((vp[0] * P.x + vp[4] * P.y) + vp[8] * P.z) + vp[12];
    const float cy = ((vp[1] * P.x + vp[5] * P.y) + vp[9] * P.z) + vp[13];
    const float cw = ((vp[3] * P.x + vp[7] * P.y) + vp[11] * P.z) + vp[15];
    if (!(cw > 0.0f)) return m;
    const float W = (float)sc.width, H = (float)sc.height;
    const float fx = ((cx / cw + 1.0f) * 0.5f) * W, fy = ((cy / cw + 1.0f) * 0.5f) * H;
    if (!(fx >= 0.0f && fx < W && fy >= 0.0f && fy < H)) return m;
    m.px = (uint32_t)fx;
    m.py = (uint32_t)fy;
    const int32_t ry = (int32_t)m.py - (int32_t)sc.row_begin;
    if (abs((int32_t)m.py - (int32_t)y) > (int32_t)A.radius || ry < A.prev_row_lo || ry >= A.prev_row_hi) {
        if (A.clip) atomicAdd(A.clip, 1ull);
        return m;
    }
    m.pp = ry * (int32_t)sc.width + (int32_t)m.px;
    m.x1p = gdecode(A.pgbuf[m.pp]);
    if (!m.x1p.valid) return m;
    const Surface Sp = get_surface(sc, m.x1p);
    if (!(dot(Sp.nrm, X1.nrm) >= 0.9f)) return m;
    const f3 x0p = gi_x0_prev(A, sc, m.px, m.py);
    const float dp = length(Sp.pos - x0p), dc = length(P - x0p);
    if (!(fabsf(dp - dc) <= 0.05f * dc)) return m;
    m.C = min(A.hist[4 * (ptrdiff_t)m.pp + 2].w, A.cap);
    m.ok = m.C != 0u;
    return m;
}

__global__ __launch_bounds__(WB) __attribute__((amdgpu_waves_per_eu(GIS_START_WAVES, 8)))
void wgim_start(Scene sc, WaveBufs w, GiArgs A) {
    __shared__ uint32_t lds[2];
    const Seg g = seg_begin(w, 0u, lds);
    const uint32_t np = padded_pixels(sc);
    for (uint32_t k = 0; k < w.seg_px; k += WB) {  // workgroup-uniform (wave_alloc below)
        const uint32_t q = seg_pixel(w, g.j, k);
        uint32_t x = 0u, y = 0u, pix = 0u;
        Compact x1{};
        if (q < np && tile_xy(sc, q, x, y)) {
            pix = (y - sc.row_begin) * sc.width + x;
            x1 = gdecode(A.gbuf[pix]);
        }
        const bool valid = x1.valid != 0u;
        GiMotion mh{false, 0, 0u, 0u, 0u, Compact{}};
        GiDomain D{};
        if (valid) {
            D.Y = get_surface(sc, x1);
            mh = gi_motion(sc, A, D.Y, y);
        }
        for (uint32_t slot = 0; slot < 2u; ++slot) {
            bool ray = false;
            f3 f{}, o{}, dir{};
            float qv = 0.0f, remain = 0.0f;
            if (mh.ok && slot == 0u) {  // the history's sample in this pixel's domain
                const uint4 *hs = A.hist + 4 * (ptrdiff_t)mh.pp;
                if (luminance(ld3(hs[3])) > 0.0f) {
                    D.Vy = normalize(x0_of(sc, x, y) - D.Y.pos);
                    ray = gi_shift_begin(D, gi_sample(sc, hs), f, qv, o, dir, remain);
                }
            } else if (mh.ok) {  // this pixel's sample in the previous frame's domain at p'
                const uint4 *rc = A.cur + 4u * (size_t)pix;
                if (rc[2].w != 0u && luminance(ld3(rc[3])) > 0.0f) {
                    GiDomain Dp;
                    Dp.Y = get_surface(sc, mh.x1p);
                    Dp.Vy = normalize(gi_x0_prev(A, sc, mh.px, mh.py) - Dp.Y.pos);
                    ray = gi_shift_begin(Dp, gi_sample(sc, rc), f, qv, o, dir, remain);
                }
            }
            const uint32_t idx = g.rbase + wave_alloc(g.l_ray, ray ? 1u : 0u);
            if (ray) {
                put_ray(g.rays, idx, o, dir, remain, Q_OCC);
                g.res_out[2u * idx] = make_float4(0.0f, f.x, f.y, f.z);
                g.res_out[2u * idx + 1u] = make_float4(qv, 0.0f, 0.0f, 0.0f);
            }
            if (valid) A.jray[gi_jid(A, pix, slot)] = ray ? idx : GI_NO_RAY;
        }
        if (valid) {
            A.jray[gi_jid(A, pix, 2u)] = (uint32_t)mh.pp;
            A.jray[gi_jid(A, pix, 3u)] = mh.ok ? mh.C : 0u;
        }
    }
    seg_end(w, g);
}

__global__ __launch_bounds__(WB) void wgim_combine(Scene sc, WaveBufs w, GiArgs A) {
    const uint32_t j = w.seg_base + blockIdx.x, np = padded_pixels(sc);
    const float4 *res = w.res[0];
    for (uint32_t k = 0; k < w.seg_px; k += WB) {
        const uint32_t q = seg_pixel(w, j, k);
        uint32_t x, y;
        if (q >= np || !tile_xy(sc, q, x, y)) continue;
        const uint32_t pix = (y - sc.row_begin) * sc.width + x;
        if (!gdecode(A.gbuf[pix]).valid) continue;
        uint4 *cur = A.cur + 4u * (size_t)pix;
        uint32_t seed = gi_seed(sc, x, y, SALT_GI_TEMPORAL);
        const uint4 c1 = cur[1], c2 = cur[2], c3 = cur[3];
        const f3 fc = ld3(c3);
        const float pc = luminance(fc), qc = asf(c3.w), Wc = asf(c1.w);
        const bool canon_ok = c2.w != 0u && pc > 0.0f;
        const int32_t pp = (int32_t)A.jray[gi_jid(A, pix, 2u)];
        const uint32_t Cp = A.jray[gi_jid(A, pix, 3u)];
        const float cp = (float)Cp;
        const uint4 *hs = A.hist + 4 * (ptrdiff_t)(Cp ? pp : 0);
        float wh = 0.0f, qf = 0.0f;
        f3 ff = mk(0.0f, 0.0f, 0.0f);
        f3 F;
        float qF;
        if (Cp != 0u && gi_job(A, res, gi_jid(A, pix, 0u), F, qF)) {
            const uint4 h1 = hs[1], h3 = hs[3];
            const float ph = luminance(ld3(h3)), qh = asf(h3.w), Wh = asf(h1.w);
            const float pF = luminance(F);
            const float J = qh / qF;
            const float pb = ph / J;
            const float den = 1.0f * pF + cp * pb;
            const float m = den > 0.0f ? (cp * pb) / den : 0.0f;
            wh = m * pF * Wh * J;
            ff = F;
            qf = qF;
        }
        float Q = 1.0f;
        f3 B;
        float qB;
        if (canon_ok && Cp != 0u && gi_job(A, res, gi_jid(A, pix, 1u), B, qB)) {
            const float pbc = luminance(B) * qc / qB;
            const float den = 1.0f * pc + cp * pbc;
            Q = den > 0.0f ? (1.0f * pc) / den : 1.0f;
        }
        const float wc = canon_ok ? Q * pc * Wc : 0.0f;
        float w_sum = 0.0f;
        bool from_hist = false;
        w_sum += wc;
        if (rnd(seed) < wc / w_sum) from_hist = false;
        w_sum += wh;
        if (rnd(seed) < wh / w_sum) from_hist = true;
        gi_write(cur, from_hist ? hs : cur, from_hist ? ff : fc, from_hist ? qf : qc, w_sum, 1u + Cp);
    }
}

// ---------------------------------------------------------------- final
__global__ __launch_bounds__(WB) void wgi_final(Scene sc, WaveBufs w, GiArgs A) {
    const uint32_t j = w.seg_base + blockIdx.x, np = padded_pixels(sc);
    for (uint32_t k = 0; k < w.seg_px; k += WB) {
        const uint32_t q = seg_pixel(w, j, k);
        uint32_t x, y;
        if (q >= np || !tile_xy(sc, q, x, y)) continue;
        const uint32_t pix = (y - sc.row_begin) * sc.width + x;
        if (!gdecode(A.gbuf[pix]).valid) {
            A.accum[pix] = make_float4(ENV_C, ENV_C, ENV_C, 1.0f);
            continue;
        }
        const uint4 *r = A.hist + 4u * (size_t)pix;
        const float4 d = A.direct[pix];
        const f3 col = mk(d.x, d.y, d.z) + ld3(r[3]) * asf(r[1].w);
        mix_color(sc, A.accum, pix, col);
    }
}

// ---------------------------------------------------------------- host side
hipError_t wave_gi_round(const Scene &sc, const WaveBufs &w, int pass, int round, const GiArgs &A, hipStream_t s) {
    const dim3 grid(w.seg_count), blk(WB);
    switch (pass) {
    case 0:  // init: rounds 0, 1, 2
        if (round == 0) hipLaunchKernelGGL(wgi_start, grid, blk, 0, s, sc, w, A);
        else if (round == 1) hipLaunchKernelGGL(wgi_step<1>, grid, blk, 0, s, sc, w, A);
        else hipLaunchKernelGGL(wgi_step<2>, grid, blk, 0, s, sc, w, A);
        break;
    case 1: hipLaunchKernelGGL(wgi_temporal, grid, blk, 0, s, sc, w, A); break;
    case 2:  // spatial: rounds 0, 1
        if (round == 0) hipLaunchKernelGGL(wgis_start, grid, blk, 0, s, sc, w, A);
        else hipLaunchKernelGGL(wgis_combine, grid, blk, 0, s, sc, w, A);
        break;
    case 4:  // temporal under camera motion: rounds 0, 1
        if (round == 0) hipLaunchKernelGGL(wgim_start, grid, blk, 0, s, sc, w, A);
        else hipLaunchKernelGGL(wgim_combine, grid, blk, 0, s, sc, w, A);
        break;
    default: hipLaunchKernelGGL(wgi_final, grid, blk, 0, s, sc, w, A); break;
    }
    return hipGetLastError();
}

}  // namespace ptx
