// ptx_shading.h -- materials, lights, BSDF evaluation / sampling / pdfs on gfx950.
// Restates SH/PT_1_InitPass.wgsl:285-314,717-1260 (PT_4 and TEST_MCPT variants flagged).
#pragma once

#include "ptx_device.h"

namespace ptx {

struct Material { f3 albedo; float metal, rough, trans, ior; };
struct Surface { f3 pos, nrm; Material mat; };

// GetMaterial (SH/PT_1_InitPass.wgsl:285-314): transmissive -> yellow albedo, roughness >= 0.01.
// Applied once per sub-mesh on the host (ptx_api.cpp build_layout) into Scene::mats, indexed
// by the flat sub-mesh number Inst::sub_base + sub: one load instead of inst -> desc -> material.
__device__ __forceinline__ uint32_t mat_index(const Scene &sc, uint32_t inst, uint32_t sub) {
    return sc.insts[inst].sub_base + sub;
}
__device__ __forceinline__ Material material_at(const Scene &sc, uint32_t flat) {
    const float4 a = sc.mats[2u * flat], b = sc.mats[2u * flat + 1u];
    Material m;
    m.albedo = mk(a.x, a.y, a.z);
    m.metal = a.w;
    m.rough = b.x;
    m.trans = b.y;
    m.ior = b.z;
    return m;
}
__device__ __forceinline__ float get_transmission(const Scene &sc, uint32_t inst, uint32_t mid) {
    return sc.mats[2u * mat_index(sc, inst, mid) + 1u].y;
}
// The same value from the root and instance tables (the trace kernels' LDS copies): each root
// record carries its sub-mesh's transmission (SubRoot::pad, ptx_api.cpp build_layout), so a
// Visibility restart test costs two LDS reads instead of two dependent global loads.
__device__ __forceinline__ float subs_transmission(const SubRoot *subs, const Inst *insts, uint32_t inst, uint32_t mid) {
    return asf(subs[insts[inst].sub_base + mid].pad);
}

// GetSurface (SH/PT_1_InitPass.wgsl:438-467) with GetTriangleWorldSpace (:390-407)
__device__ __forceinline__ Surface get_surface(const Scene &sc, Compact x) {
    const Inst &I = sc.insts[x.inst];
    Surface s;
    s.mat = material_at(sc, I.sub_base + x.mat);
    const TriVerts tv = tri_verts(sc, I.tri_base + x.prim);
    f3 p0 = inst_point(I, I.m, tv.p[0]);
    f3 n0 = inst_point_t(I, I.minv, tv.n[0]);
    f3 p1 = inst_point(I, I.m, tv.p[1]);
    f3 n1 = inst_point_t(I, I.minv, tv.n[1]);
    f3 p2 = inst_point(I, I.m, tv.p[2]);
    f3 n2 = inst_point_t(I, I.minv, tv.n[2]);
    float U = x.bu, V = x.bv, W = 1.0f - U - V;
    s.nrm = normalize((n0 * U + n1 * V) + n2 * W);
    s.pos = (p0 * U + p1 * V) + p2 * W;
    return s;
}
// GetSurface at a hit whose position trace_core already produced: normal + material only
// (the position is bit-identical: same world-space vertices and barycentrics).
__device__ __forceinline__ Surface surface_at(const Scene &sc, const Compact &x, f3 pos) {
    const Inst &I = sc.insts[x.inst];
    Surface s;
    s.mat = material_at(sc, I.sub_base + x.mat);
    const TriVerts tv = tri_verts(sc, I.tri_base + x.prim);
    f3 n0 = inst_point_t(I, I.minv, tv.n[0]);
    f3 n1 = inst_point_t(I, I.minv, tv.n[1]);
    f3 n2 = inst_point_t(I, I.minv, tv.n[2]);
    float U = x.bu, V = x.bv, W = 1.0f - U - V;
    s.nrm = normalize((n0 * U + n1 * V) + n2 * W);
    s.pos = pos;
    return s;
}
// Position-only GetSurface for Visibility restarts (the normal is unused there).
__device__ __forceinline__ f3 get_surface_pos(const Scene &sc, Compact x) {
    const Inst &I = sc.insts[x.inst];
    const TriVerts tv = tri_verts(sc, I.tri_base + x.prim);
    f3 p0 = inst_point(I, I.m, tv.p[0]);
    f3 p1 = inst_point(I, I.m, tv.p[1]);
    f3 p2 = inst_point(I, I.m, tv.p[2]);
    float U = x.bu, V = x.bv, W = 1.0f - U - V;
    return (p0 * U + p1 * V) + p2 * W;
}

// ------------------------------------------------------------------ lights
struct Light { f3 pos, dir, color, U, V; uint32_t type; float intensity, area; };
struct LightSample { f3 dir; uint32_t type; f3 pos; int32_t id; f3 Le; float pdf; };

__device__ __forceinline__ Light get_light(const Scene &sc, uint32_t id) {
    const uint32_t *p = sc.S + sc.U[U_OFF_LIGHT] + STRIDE_LIGHT * id;
    Light l;
    l.pos = mk(asf(p[0]), asf(p[1]), asf(p[2]));
    l.dir = mk(asf(p[3]), asf(p[4]), asf(p[5]));
    l.color = mk(asf(p[6]), asf(p[7]), asf(p[8]));
    l.U = mk(asf(p[9]), asf(p[10]), asf(p[11]));
    l.V = mk(asf(p[12]), asf(p[13]), asf(p[14]));
    l.type = p[15];
    l.intensity = asf(p[16]);
    l.area = asf(p[17]);
    return l;
}
__device__ __forceinline__ float light_cdf(const Scene &sc, uint32_t i) { return asf(sc.S[sc.U[U_OFF_CDF] + i]); }

// ------------------------------------------------------------------ BSDF (SH/PT_1_InitPass.wgsl:834-929)
__device__ __forceinline__ float ggx_d(float NdotH, float R) {
    float a = R * R, a2 = a * a;
    float X = NdotH * NdotH * (a2 - 1.0f) + 1.0f;
    float denom = PI_F * X * X;
    return a2 / fmaxf(denom, EPS_F);
}
__device__ __forceinline__ float geom_shadow(float NdotV, float NdotL, float R) {
    float r = R + 1.0f;
    float K = r * r / 8.0f;
    return 1.0f / ((NdotV * (1.0f - K) + K) * (NdotL * (1.0f - K) + K));
}
// Fixed f32 pow(x, 5) / sin / cos shared with the oracle (oracle/pt_oracle.c pow5_,
// sincos_): WGSL leaves them implementation-defined, and one definition on both sides
// keeps the whole path bit-exact (libm and ocml differ in the last ulp).  ~2 ulp of true.
__device__ __forceinline__ float pow5(float x) {
    float x2 = x * x;
    return (x2 * x2) * x;
}
// x >= 0 only (BSDF sampling angles): Cody-Waite reduction by pi/4, minimax polynomials.
__device__ __forceinline__ void fsincos(float x, float &s, float &c) {
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
    const bool swap = (j & 2) != 0;           // octants 2, 6: sin <- cos poly, cos <- sin poly
    const float sv = swap ? pc : ps, cv = swap ? ps : pc;
    s = (j == 4 || j == 6) ? -sv : sv;        // sin negative in octants 4, 6
    c = (j == 2 || j == 4) ? -cv : cv;        // cos negative in octants 2, 4
}
__device__ __forceinline__ f3 fresnel(float d, f3 F0) {
    float p = pow5(1.0f - saturate(d));
    return mk(F0.x + (1.0f - F0.x) * p, F0.y + (1.0f - F0.y) * p, F0.z + (1.0f - F0.z) * p);
}
__device__ __forceinline__ f3 brdf(const Surface &X, f3 V, f3 L) {
    f3 N = X.nrm;
    f3 H = normalize(L + V);
    float NdotV = fmaxf(dot(N, V), 0.0f), NdotL = fmaxf(dot(N, L), 0.0f);
    float NdotH = fmaxf(dot(N, H), 0.0f), VdotH = fmaxf(dot(V, H), 0.0f);
    f3 base = X.mat.albedo;
    float metal = X.mat.metal, R = X.mat.rough;
    f3 F0 = mix3(mk(0.04f, 0.04f, 0.04f), base, metal);
    float D = ggx_d(NdotH, R);
    float G0 = geom_shadow(NdotV, NdotL, R);
    f3 F = fresnel(VdotH, F0);
    f3 kD = mk(1.0f - F.x, 1.0f - F.y, 1.0f - F.z) * (1.0f - metal);
    f3 diffuse = (kD / PI_F) * base;
    f3 spec = ((F * D) * G0) * 0.25f;
    return diffuse + spec;
}
__device__ __forceinline__ f3 btdf(const Surface &X, f3 V, f3 L) {
    float R = X.mat.rough;
    bool same = dot(V, X.nrm) > 0.0f;
    float n_in = same ? X.mat.ior : 1.0f;
    float n_out = same ? 1.0f : X.mat.ior;
    f3 hv = L * n_in + V * n_out;
    float H_norm = length(hv);
    f3 N = same ? X.nrm : -X.nrm;
    f3 H = normalize(hv);
    float NdotL = fabsf(dot(N, L)), NdotV = fabsf(dot(N, V)), NdotH = fabsf(dot(N, H));
    float LdotH = fabsf(dot(L, H)), VdotH = fabsf(dot(V, H));
    float G0 = geom_shadow(NdotL, NdotV, R);
    float D = ggx_d(NdotH, R);
    float nr = (n_out - n_in) / (n_out + n_in);
    f3 F = fresnel(LdotH, mk(nr * nr, nr * nr, nr * nr));
    f3 num = mk(1.0f - F.x, 1.0f - F.y, 1.0f - F.z) * (n_out * n_out);
    num = ((((num * LdotH) * VdotH) * G0) * D) * X.mat.albedo;
    return num / fmaxf(H_norm * H_norm, EPS_F);
}
__device__ __forceinline__ f3 bsdf(const Surface &X, f3 V, f3 L) {
    float T = X.mat.trans;
    if (dot(L, X.nrm) * dot(V, X.nrm) > 0.0f) return brdf(X, V, L) * (1.0f - T);
    return btdf(X, V, L) * T;
}

// ------------------------------------------------------------------ sampling (SH/PT_1_InitPass.wgsl:577-589,937-1106)
struct Tbn { f3 T, B, N; };
__device__ __forceinline__ Tbn tbn(f3 N) {
    bool same = fabsf(dot(N, mk(0.0f, 1.0f, 0.0f))) > 0.9999f;
    f3 cv = same ? mk(1.0f, 0.0f, 0.0f) : mk(0.0f, 1.0f, 0.0f);
    Tbn m;
    m.T = normalize(cross(cv, N));
    m.B = cross(N, m.T);
    m.N = N;
    return m;
}
__device__ __forceinline__ f3 tbn_mul(const Tbn &m, f3 v) { return (m.T * v.x + m.B * v.y) + m.N * v.z; }
__device__ __forceinline__ f3 reflect3(f3 I, f3 N) { return I - N * (2.0f * dot(N, I)); }
__device__ __forceinline__ f3 refract3(f3 I, f3 N, float eta) {
    float d = dot(N, I);
    float k = 1.0f - eta * eta * (1.0f - d * d);
    if (k < 0.0f) return mk(0.0f, 0.0f, 0.0f);
    return I * eta - N * (eta * d + __builtin_sqrtf(k));
}
__device__ __forceinline__ f3 sample_cosine(uint32_t &seed) {
    float r1 = rnd(seed), r2 = rnd(seed);
    float R = __builtin_sqrtf(r1);
    float phi = 2.0f * PI_F * r2, sp, cp;
    fsincos(phi, sp, cp);
    return mk(R * cp, R * sp, __builtin_sqrtf(1.0f - r1));
}
__device__ __forceinline__ f3 sample_ggx(uint32_t &seed, float R) {
    float r1 = rnd(seed), r2 = rnd(seed);
    float a = R * R;
    float phi = 2.0f * PI_F * r1;
    float ct = __builtin_sqrtf((1.0f - r2) / (1.0f + (a * a - 1.0f) * r2));
    float st = __builtin_sqrtf(1.0f - ct * ct), sp, cp;
    fsincos(phi, sp, cp);
    return normalize(mk(st * cp, st * sp, ct));
}
__device__ __forceinline__ f3 sample_bsdf(uint32_t &seed, const Surface &X, f3 V, uint32_t &lobe) {
    bool transparent = rnd(seed) < X.mat.trans;
    if (transparent) {  // SampleBTDF, SH/PT_1_InitPass.wgsl:1063-1098
        bool same = dot(V, X.nrm) > 0.0f;
        float n_in = same ? 1.0f : X.mat.ior;
        float n_out = same ? X.mat.ior : 1.0f;
        f3 N = same ? X.nrm : -X.nrm;
        float ratio = n_in / n_out;
        float r = (1.0f - ratio) / (1.0f + ratio);
        float R2 = ratio * ratio;
        float cos_t = fabsf(dot(V, N));
        float p_refl = fresnel(cos_t, mk(r * r, r * r, r * r)).x;
        if (cos_t * cos_t < (R2 - 1.0f) / R2) p_refl = 1.0f;
        bool refl = rnd(seed) < p_refl;
        Tbn m = tbn(N);
        f3 H = tbn_mul(m, sample_ggx(seed, X.mat.rough));
        f3 Lr = refract3(-V, H, ratio);
        f3 Ll = reflect3(-V, H);
        lobe = LOBE_GGX;
        return normalize(refl ? Ll : Lr);
    }
    // SampleBRDF, SH/PT_1_InitPass.wgsl:1027-1061
    float metal = X.mat.metal;
    f3 F0 = mix3(mk(0.04f, 0.04f, 0.04f), X.mat.albedo, metal);
    float p_spec = mixf(luminance(F0), 1.0f, metal);
    Tbn m = tbn(X.nrm);
    bool spec = rnd(seed) < p_spec;
    f3 L;
    if (spec) {
        f3 H = tbn_mul(m, sample_ggx(seed, X.mat.rough));
        L = reflect3(-V, H);
    } else {
        L = tbn_mul(m, sample_cosine(seed));
    }
    lobe = spec ? LOBE_GGX : LOBE_LAMBERT;
    return L;
}

// ------------------------------------------------------------------ pdfs (SH/PT_1_InitPass.wgsl:1114-1218)
__device__ __forceinline__ float pdf_brdf(const Surface &X, f3 V, f3 L) {
    float metal = X.mat.metal, R = X.mat.rough;
    f3 F0 = mix3(mk(0.04f, 0.04f, 0.04f), X.mat.albedo, metal);
    float p_spec = mixf(luminance(F0), 1.0f, metal);
    f3 N = X.nrm;
    f3 H = normalize(L + V);
    float LdotN = fmaxf(dot(L, N), 0.0f);
    float NdotH = fmaxf(dot(N, H), 0.0f);
    float VdotH = fmaxf(dot(V, H), 0.0f);
    float pdf_s = ggx_d(NdotH, R) / fmaxf(4.0f * VdotH, EPS_F);
    float pdf_d = LdotN / PI_F;
    return mixf(pdf_d, pdf_s, p_spec);
}
__device__ __forceinline__ float pdf_btdf(const Surface &X, f3 V, f3 L) {
    float R = X.mat.rough;
    bool same = dot(V, X.nrm) > 0.0f;
    float n_in = same ? 1.0f : X.mat.ior;
    float n_out = same ? X.mat.ior : 1.0f;
    float ratio = n_in / n_out;
    f3 N = same ? X.nrm : -X.nrm;
    float r0 = (1.0f - ratio) / (1.0f + ratio);
    float R0 = r0 * r0;
    float cos_t = fabsf(dot(V, N));
    float p_refl = fresnel(cos_t, mk(R0, R0, R0)).x;
    float sin2 = 1.0f - cos_t * cos_t;
    float R2 = ratio * ratio;
    if (sin2 * R2 > 1.0f) p_refl = 1.0f;
    float p_trans = 1.0f - p_refl;
    float pdf_r = 0.0f;
    if (p_refl > 0.0f) {
        f3 Hr = normalize(V + L);
        float NdotHr = fmaxf(0.0f, dot(N, Hr));
        float VdotHr = fmaxf(0.0f, dot(V, Hr));
        if (VdotHr > 0.0f) pdf_r = ggx_d(NdotHr, R) / (4.0f * VdotHr);
    }
    float pdf_t = 0.0f;
    if (p_trans > 0.0f) {
        f3 Ht = normalize(V * n_out + L * n_in);
        float NdotHt = fmaxf(0.0f, dot(N, Ht));
        float VdotHt = fmaxf(0.0f, dot(V, Ht));
        float LdotHt = fmaxf(0.0f, dot(L, Ht));
        float denom = n_in * LdotHt + n_out * VdotHt;
        if (denom > 0.0f) {
            float J = (n_out * n_out * VdotHt) / (denom * denom);
            pdf_t = ggx_d(NdotHt, R) * fabsf(J);
        }
    }
    return p_refl * pdf_r + p_trans * pdf_t;
}
__device__ __forceinline__ float pdf_bsdf(const Surface &X, f3 V, f3 L) {
    if (dot(L, X.nrm) * dot(V, X.nrm) > 0.0f) return pdf_brdf(X, V, L);
    return pdf_btdf(X, V, L);
}

// bsdf(X, V, L) and pdf_bsdf(X, V, L) together (a sampled direction's throughput factor and its
// pdf, PT_1:1427-1434): each value computed exactly as the two functions compute it, the
// reflection branch's half vector, D, F0 and N.L shared instead of evaluated twice.
__device__ __forceinline__ f3 bsdf_pdf(const Surface &X, f3 V, f3 L, float &pdf) {
    const f3 N = X.nrm;
    if (dot(L, N) * dot(V, N) > 0.0f) {
        const f3 H = normalize(L + V);
        const float NdotV = fmaxf(dot(N, V), 0.0f), NdotL = fmaxf(dot(N, L), 0.0f);
        const float LdotN = fmaxf(dot(L, N), 0.0f);
        const float NdotH = fmaxf(dot(N, H), 0.0f), VdotH = fmaxf(dot(V, H), 0.0f);
        const f3 base = X.mat.albedo;
        const float metal = X.mat.metal, R = X.mat.rough;
        const f3 F0 = mix3(mk(0.04f, 0.04f, 0.04f), base, metal);
        const float D = ggx_d(NdotH, R);
        const float G0 = geom_shadow(NdotV, NdotL, R);
        const f3 F = fresnel(VdotH, F0);
        const f3 kD = mk(1.0f - F.x, 1.0f - F.y, 1.0f - F.z) * (1.0f - metal);
        const f3 diffuse = (kD / PI_F) * base;
        const f3 spec = ((F * D) * G0) * 0.25f;
        const float p_spec = mixf(luminance(F0), 1.0f, metal);
        pdf = mixf(LdotN / PI_F, D / fmaxf(4.0f * VdotH, EPS_F), p_spec);
        return (diffuse + spec) * (1.0f - X.mat.trans);
    }
    pdf = pdf_btdf(X, V, L);
    return btdf(X, V, L) * X.mat.trans;
}

// DirectionToLight, SH/PT_1_InitPass.wgsl:746-772
__device__ __forceinline__ f3 direction_to_light(const Surface &X, const LightSample &XL) {
    switch (XL.type) {
    case LIGHT_DIRECTION: return -XL.dir;
    case LIGHT_POINT:
    case LIGHT_RECT: return normalize(XL.pos - X.pos);
    case LIGHT_ENV: return -XL.dir;
    default: return mk(0.0f, 0.0f, 0.0f);
    }
}

// SampleNEE + PDF_LIGHT (SH/PT_1_InitPass.wgsl:970-1025,1220-1245)
__device__ __forceinline__ LightSample sample_nee(const Scene &sc, uint32_t &seed, const Surface &X, f3 V) {
    LightSample s;
    float P = rnd(seed);
    uint32_t L = 0, R = sc.U[U_LIGHT_COUNT] - 1u, M = (L + R) >> 1;
    while (L < R) {
        if (P < light_cdf(sc, M)) R = M;
        else L = M + 1u;
        M = (L + R) >> 1;
    }
    s.id = (int32_t)M;
    Light ls = get_light(sc, M);
    s.type = ls.type;
    s.Le = ls.color * ls.intensity;
    s.pos = mk(0.0f, 0.0f, 0.0f);
    s.dir = mk(0.0f, 0.0f, 0.0f);
    if (ls.type == LIGHT_DIRECTION) {
        s.pos = X.pos - ls.dir * INF_F;
        s.dir = ls.dir;
    } else if (ls.type == LIGHT_POINT) {
        s.pos = ls.pos;
        s.dir = normalize(X.pos - ls.pos);
    } else if (ls.type == LIGHT_RECT) {
        float ru = rnd(seed) * 2.0f - 1.0f;
        float rv = rnd(seed) * 2.0f - 1.0f;
        s.pos = ls.pos + (ls.U * ru + ls.V * rv);
        s.dir = normalize(X.pos - s.pos);
    }
    // PDF_LIGHT (never the env branch here: NEE samples are scene lights)
    float before = (M == 0u) ? 0.0f : light_cdf(sc, M - 1u);
    float choose = light_cdf(sc, M) - before;
    float pdf_point = 1.0f;
    if (s.type == LIGHT_RECT) {
        f3 r = s.pos - X.pos;
        f3 Ld = normalize(r);
        pdf_point = dot(r, r) / fmaxf(ls.area * fabsf(dot(ls.dir, Ld)), EPS_F);
    }
    s.pdf = choose * pdf_point;
    return s;
}

// L_emit: SH/PT_1_InitPass.wgsl:1253-1260 (guarded), SH/PT_4_FinalShadingPass.wgsl:1261-1268 (unguarded)
template <bool FINAL>
__device__ __forceinline__ f3 l_emit(const LightSample &XL, const Surface &X) {
    f3 r = XL.pos - X.pos;
    float rr = dot(r, r);
    float att = (XL.type == LIGHT_POINT) ? 1.0f / (FINAL ? rr : fmaxf(rr, EPS_F)) : 1.0f;
    return XL.Le * att;
}

// Visibility (SH/PT_1_InitPass.wgsl:774-802): up to 5 traces through transmissive hits.
template <bool COUNT>
__device__ __noinline__ float visibility(const Scene &sc, f3 start, f3 end, PassEps eps, uint32_t *stack,
                                         uint32_t stride) {
    float T = 1.0f;
    float dist = length(end - start);
    f3 dir = (end - start) / dist;
    Ray r{start, dir};
    float remain = dist;
    for (int it = 0; it < 5; ++it) {
        Hit h = trace_ray<COUNT>(sc, r, eps, stack, stride);
        if (!h.valid || h.t > remain) return T;
        float tr = get_transmission(sc, h.s.inst, h.s.mat);
        if (tr == 0.0f) return 0.0f;
        T *= tr;
        remain -= h.t;
        r.o = get_surface_pos(sc, h.s);
    }
    return 0.0f;
}

}  // namespace ptx
