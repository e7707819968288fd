// ptx_wave_common.h -- wave-level queue helpers shared by the wavefront kernels
// (ptx_wave.hip: PT_01/PT_1/PT_4/TEST_MCPT; ptx_reuse.hip: temporal/spatial reuse).
#pragma once
#include "ptx_launch.h"
#include "ptx_shading.h"

namespace ptx {

constexpr uint32_t WB = kBlock;
#ifndef LOGIC_WAVES
#define LOGIC_WAVES 4  // start/step kernels: <=128 VGPRs, 4 waves/SIMD, no spill (5 spills)
#endif
// query kinds of the ray queues: closest hit; Visibility (through transmissive hits, result
// in res.x, payload kept); occlusion (any hit inside `remain` occludes: binary, payload kept)
enum : uint32_t { Q_CLOSEST = 0u, Q_VIS = 1u, Q_OCC = 2u };

// ---------------------------------------------------------------- wave helpers
// Exclusive prefix sum of `v` over the wave and the wave total.
__device__ __forceinline__ uint32_t wave_scan(uint32_t v, uint32_t &total) { return wave_excl_sum(v, total); }
// Reserve `n` consecutive slots of this workgroup's segment (one LDS atomic per wave).
// Must be reached by every lane of the wave.
__device__ __forceinline__ uint32_t wave_alloc(uint32_t *lds_ctr, uint32_t n) {
    uint32_t total;
    const uint32_t excl = wave_scan(n, total);
    uint32_t base = 0u;
    if (__lane_id() == 0u && total) base = atomicAdd(lds_ctr, total);
    base = (uint32_t)__builtin_amdgcn_readfirstlane((int)base);  // (lane 0 is active: every lane is)
    return base + excl;
}

// This workgroup's view of one logic round: its segments of the queues and LDS counters.
struct Seg {
    uint32_t j, round;         // virtual segment (pixel layout), round
    uint32_t pj;               // its physical queue slot
    uint32_t rbase;            // first ray slot of the segment
    float4 *rays, *res_out;    // rays emitted this round + their result/payload slots
    const float4 *res_in;      // results of the previous trace round
    uint32_t out_sel;          // res_out's index in WaveBufs::res
    uint32_t *act_out;         // active list written this round (segment-local)
    const uint32_t *act_in;    // active list of the previous round
    uint32_t n_in;             // its length
    uint32_t *l_ray, *l_act;   // LDS counters
};
// The result buffer of trace round `round`.
__device__ __forceinline__ uint32_t res_sel(const WaveBufs &w, uint32_t round) {
    return w.nres == 3u ? round % 3u : round & 1u;
}
__device__ __forceinline__ float4 *res_buf(const WaveBufs &w, uint32_t round) { return w.res[res_sel(w, round)]; }
__device__ __forceinline__ Seg seg_begin(const WaveBufs &w, uint32_t round, uint32_t *lds) {
    Seg g;
    g.j = w.seg_base + blockIdx.x;
    g.pj = w.seg_phys + g.j;
    g.round = round;
    g.rbase = g.pj * w.ray_stride;
    g.rays = w.rays;
    g.res_out = res_buf(w, round);
    g.res_in = round ? res_buf(w, round - 1u) : w.res[1];  // (round 0 reads no results)
    g.out_sel = res_sel(w, round);
    g.act_out = w.act[round & 1u] + (size_t)g.pj * w.act_stride;
    g.act_in = w.act[(round + 1u) & 1u] + (size_t)g.pj * w.act_stride;
    g.n_in = round ? w.cnt[(2u * (round - 1u)) * w.cnt_stride + g.pj] : 0u;
    g.l_ray = lds;
    g.l_act = lds + 1;
    if (threadIdx.x == 0) { lds[0] = 0u; lds[1] = 0u; }
    // the batch counter of the trace round this launch feeds (the trace kernel runs after
    // this launch on the same stream)
    if (w.dyn && blockIdx.x == 0 && threadIdx.x < kDynHeads) w.dyn[round * kDynRoundWords + threadIdx.x * kDynStride] = 0u;
    __syncthreads();
    return g;
}
__device__ __forceinline__ void seg_end(const WaveBufs &w, const Seg &g) {
    __syncthreads();
    if (threadIdx.x == 0) {
        w.cnt[(2u * g.round) * w.cnt_stride + g.pj] = *g.l_act;
        w.cnt[(2u * g.round + 1u) * w.cnt_stride + g.pj] = *g.l_ray;
    }
}
// Padded pixel handled by this thread at offset k of segment j.  A segment is seg_px/64
// 8x8 tiles spread over the whole band (tile j + t * nseg, cluster 1): each wave still
// shades one coherent tile, while every segment -- and so every trace workgroup -- sees a
// sample of the whole image, which keeps the per-segment trace cost even.  Measured at
// 1080p: spreading beats clustering adjacent tiles (cluster 4: -5 %, 16: -33 %), and
// 512-pixel segments beat 1024 (+1-3 %), 256 (-9 %) and 2048 (-11 %); since the split active
// lists and the cooperative traversal, 768 beats 512 (+1 to +4 % per pipeline).
// Band tile of virtual tile v of the launch's tile set (WaveBufs::tile0..ntile1); past the
// set's end a tile index whose pixels fail every `q < padded_pixels` test.
__device__ __forceinline__ uint32_t set_tile(const WaveBufs &w, uint32_t v) {
    return v < w.ntile0 ? w.tile0 + v : v - w.ntile0 < w.ntile1 ? w.tile1 + (v - w.ntile0) : 0x3ffffffu;
}
__device__ __forceinline__ uint32_t seg_pixel(const WaveBufs &w, uint32_t j, uint32_t k) {
    const uint32_t s = (k + threadIdx.x) >> 6;  // tile slot within the segment (seg_px / 64)
    const uint32_t cl = w.cluster;              // runs of `cl` adjacent tiles
    const uint32_t t = set_tile(w, ((s / cl) * w.nseg + j) * cl + s % cl);
    return t * 64u + (threadIdx.x & 63u);
}
// append the active pixel to this round's list (all lanes)
__device__ __forceinline__ void seg_keep(const Seg &g, bool keep, uint32_t pix) {
    const uint32_t slot = wave_alloc(g.l_act, keep ? 1u : 0u);
    if (keep) g.act_out[slot] = pix;
}

// Active lists split by what the next logic round does with the entry: "heavy" entries (a
// new path vertex: surface, BSDF, next rays) from the front of the segment's list, "light"
// ones (only a Visibility result or a path's end to book) from the back, so the next
// round's waves run one kind, not both.  The count word is heavy | light << 16 (a segment
// holds at most seg_px * 32 entries).  Results never depend on list order.  Readers:
// split_count, split_at.
struct JobLists { uint32_t *l_light; uint32_t stride; };
__device__ __forceinline__ JobLists job_lists(const WaveBufs &w, uint32_t *lds) {
    if (threadIdx.x == 0) lds[2] = 0u;  // (seg_begin's barrier publishes it)
    return JobLists{lds + 2, w.act_stride};
}
__device__ __forceinline__ void job_keep(const Seg &g, const JobLists &L, bool keep, bool light, uint32_t jid) {
    const uint32_t sh = wave_alloc(g.l_act, keep && !light ? 1u : 0u);
    const uint32_t sl = wave_alloc(L.l_light, keep && light ? 1u : 0u);
    if (keep) g.act_out[light ? L.stride - 1u - sl : sh] = jid;
}
__device__ __forceinline__ void job_seg_end(const WaveBufs &w, const Seg &g, const JobLists &L) {
    __syncthreads();
    if (threadIdx.x == 0) {
        w.cnt[(2u * g.round) * w.cnt_stride + g.pj] = *g.l_act | (*L.l_light << 16);
        w.cnt[(2u * g.round + 1u) * w.cnt_stride + g.pj] = *g.l_ray;
    }
}

__device__ __forceinline__ uint32_t split_count(const Seg &g, uint32_t &nh) {
    nh = g.n_in & 0xffffu;
    return nh + (g.n_in >> 16);
}
__device__ __forceinline__ uint32_t split_at(const Seg &g, const JobLists &L, uint32_t q, uint32_t nh) {
    return g.act_in[q < nh ? q : L.stride - 1u - (q - nh)];
}

__device__ __forceinline__ void put_ray(float4 *rays, uint32_t idx, f3 o, f3 d, float remain, uint32_t kind) {
    rays[2u * idx] = make_float4(o.x, o.y, o.z, remain);
    rays[2u * idx + 1u] = make_float4(d.x, d.y, d.z, asf(kind));
}
__device__ __forceinline__ Hit get_hit(const float4 *res, uint32_t idx) {
    const float4 a = res[2u * idx], b = res[2u * idx + 1u];
    const uint32_t enc = asu(a.y);
    Hit h;
    h.valid = (enc >> 31) != 0u;
    h.t = a.x;
    h.s = Compact{enc >> 31, (enc >> 16) & 0x7fffu, enc & 0xffffu, asu(a.z), a.w, b.x};
    h.pos = mk(b.y, b.z, b.w);
    return h;
}
__device__ __forceinline__ f3 x0_of(const Scene &sc, uint32_t x, uint32_t y) {  // Get_X0, PT_1:732-738
    const float *vpinv = reinterpret_cast<const float *>(sc.U + U_VPINV);
    float u = ((float)x + 0.5f) / (float)sc.U[U_W];
    float v = ((float)y + 0.5f) / (float)sc.U[U_H];
    return xform_point(vpinv, mk(2.0f * u - 1.0f, 2.0f * v - 1.0f, 0.0f));
}
__device__ __forceinline__ Compact gdecode(uint4 g) {
    return Compact{(g.x & 0x80000000u) ? 1u : 0u, (g.x & 0x7fff0000u) >> 16, g.x & 0xffffu, g.y, asf(g.z), asf(g.w)};
}
__device__ __forceinline__ uint4 gencode(const Compact &s) {
    return make_uint4((s.valid << 31) | (s.inst << 16) | s.mat, s.prim, asu(s.bu), asu(s.bv));
}
__device__ __forceinline__ void mix_color(const Scene &sc, float4 *accum, uint32_t i, f3 c) {
    float t = 1.0f / (float)(sc.U[U_FRAME] + 1u);  // WriteColor, PT_4:599-606
    float4 a = accum[i];
    accum[i] = make_float4(mixf(a.x, c.x, t), mixf(a.y, c.y, t), mixf(a.z, c.z, t), 1.0f);
}
// pixel -> (x, y) for the start kernels: 8x8 tiles so a wave's first rays are coherent
__device__ __forceinline__ bool tile_xy(const Scene &sc, uint32_t p, uint32_t &x, uint32_t &y) {
    const uint32_t tiles_x = (sc.width + 7u) / 8u, t = p >> 6, l = p & 63u;
    x = (t % tiles_x) * 8u + (l & 7u);
    y = sc.row_begin + (t / tiles_x) * 8u + (l >> 3);
    return x < sc.width && y < sc.row_end;
}
__device__ __forceinline__ uint32_t padded_pixels(const Scene &sc) {
    return ((sc.width + 7u) / 8u) * ((sc.row_end - sc.row_begin + 7u) / 8u) * 64u;
}

// Primary-hit surface records (DI reuse pipeline, WaveBufs::surf / ReuseArgs::surf): per band
// (+ halo) pixel, GetSurface of its G-buffer hit -- {pos, flat material index}, {normal, 0} --
// written once per frame by PT_1's start kernel (which computes it anyway) or wsurface, and
// gathered by the temporal / spatial shift jobs instead of recomputing it (an 80-byte vertex
// record, the instance transform and a normalize) for every job of every domain.  Same bits
// as get_surface: the record is its output.  kNoSurface: the G-buffer has no hit there.
constexpr uint32_t kNoSurface = 0xFFFFFFFFu;
__device__ __forceinline__ void surf_store(uint4 *surf, ptrdiff_t i, const Surface &X, uint32_t matref) {
    surf[2 * i] = make_uint4(asu(X.pos.x), asu(X.pos.y), asu(X.pos.z), matref);
    surf[2 * i + 1] = make_uint4(asu(X.nrm.x), asu(X.nrm.y), asu(X.nrm.z), 0u);
}
__device__ __forceinline__ void surf_store_none(uint4 *surf, ptrdiff_t i) {
    surf[2 * i] = make_uint4(0u, 0u, 0u, kNoSurface);
}
// the record of band pixel i; false (X untouched) when the pixel has no G-buffer hit
__device__ __forceinline__ bool surf_load(const Scene &sc, const uint4 *surf, ptrdiff_t i, Surface &X,
                                          uint32_t &matref) {
    const uint4 a = surf[2 * i];
    if (a.w == kNoSurface) return false;
    const uint4 b = surf[2 * i + 1];
    X.pos = mk(asf(a.x), asf(a.y), asf(a.z));
    X.nrm = mk(asf(b.x), asf(b.y), asf(b.z));
    X.mat = material_at(sc, a.w);
    matref = a.w;
    return true;
}
// GetSurface of a G-buffer texel into the record (wsurface, halo rows of wnbr_summary)
__device__ __forceinline__ void surf_from_gbuf(const Scene &sc, uint4 *surf, ptrdiff_t i, uint4 g) {
    const Compact x1 = gdecode(g);
    if (!x1.valid) surf_store_none(surf, i);
    else surf_store(surf, i, get_surface(sc, x1), mat_index(sc, x1.inst, x1.mat));
}

__device__ __forceinline__ LightSample load_xl(const uint4 *res) {
    const uint4 r1 = res[1], r2 = res[2], r3 = res[3];
    LightSample XL;
    XL.dir = mk(asf(r1.x), asf(r1.y), asf(r1.z));
    XL.type = r1.w;
    XL.pos = mk(asf(r2.x), asf(r2.y), asf(r2.z));
    XL.id = (int32_t)r2.w;
    XL.Le = mk(asf(r3.x), asf(r3.y), asf(r3.z));
    XL.pdf = asf(r3.w);
    return XL;
}
}  // namespace ptx
