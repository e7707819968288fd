// ptx_wave.hip -- wavefront form of the secondary passes (the default fast path).
//
// Observation that makes this work: in the reference, a Visibility() result never feeds
// back into the RNG stream or into path construction.  UpdateReservoir always draws
// exactly one Random() (SH/PT_1_InitPass.wgsl:1298-1320); f, p and Russian roulette do
// not depend on visibility; in TEST_MCPT the light terms only add to the colour
// (SH/TEST_MCPT.wgsl:1351-1366).  So at every path vertex the shadow ray(s) AND the next
// BSDF ray are known before any of them is traced: each vertex costs ONE trace round,
// and the reservoir update / colour accumulation that needs the visibility is resolved
// in the next logic step, in the reference's order.  The random draws happen at the same
// points of the stream as in the WGSL, so results are identical per pixel.
//
// Queues are segmented by workgroup: workgroup j of every logic kernel owns pixel segment
// j (seg_px padded pixels, 8x8 tiles) for the whole pass, keeps that segment's active
// list, and appends its rays to ray segment j through LDS counters; trace workgroup j
// traces ray segment j.  No global atomics anywhere (a single device-wide queue counter
// serialises at ~4 ns per wave-level append, which cost more than the shading itself).
//
// Kernels (256-thread workgroups, one per segment):
//   trace_queue  -- lean closest-hit / Visibility queries over a ray segment (≈70
//                   VGPRs); the Visibility loop (<=5 traces through transmissive hits,
//                   SH/PT_1_InitPass.wgsl:774-802) runs inside it, pruned at the light.
//   *_start      -- per pixel: first vertex, emits the first round of rays.
//   *_step       -- per active pixel: consumes its results, advances to the next vertex,
//                   emits the next round.  Pixel state lives in HBM (SoA float4 slots).
// Rounds: init <= 3 traces (vertices 1..3), final <= 3 (two regenerated BSDF rays + the
// light visibility), MCPT <= 4 (primary + 3 bounces with all lights' shadow rays).
#include "ptx_wave_common.h"

#include <algorithm>
#include <cstdlib>

namespace ptx {

// ---------------------------------------------------------------- trace queue
// Workgroup j traces ray segment j of `round`.  A Visibility query is traced with its
// hit range capped at the remaining distance to the light: Visibility only looks at the
// closest hit when its t <= remain, and the cap leaves the visit order -- hence which of
// several equal-t triangles wins -- unchanged for every hit inside the cap.
// OCC: every query of the launch is Q_OCC (the GI shift's binary visibility): an any-hit
// walk (trace_core_tab ANY), exact for "is there a hit with t <= remain".
#ifndef TRACE_OCC_WAVES
#define TRACE_OCC_WAVES 5  // occupancy of the occlusion-query instance (GI spatial rounds)
#endif
#ifndef TRACE_COOP
#define TRACE_COOP true
#endif
// One wave's batch of up to 64 queries (lane i of `rays` / `res`; `active` = lane has one).
// Every lane of the wave calls the traversal every time -- lanes without a query (past the
// segment's end, or whose Visibility walk is over) with a NaN bound, which no box overlaps --
// so the whole wave takes part in the cooperative leaf phases.
#ifndef PTX_NODE_UNI
#define PTX_NODE_UNI 1  // one pop / root-take path in the node loop when the tables sit in LDS
#endif
#ifndef PTX_FLAT_INST
#define PTX_FLAT_INST 1  // the instance loop flattened into the lanes (trace_core_flat) for scenes
#endif                   // of >= kFlatMinInstances instances (host side, wave_trace)
// Measured same box (1080p): furnished C3 (13 instances) +9.7 %, GI on C3 (3) +3.2 %, reuse on
// C3 +0.6 %, TEST_MCPT on C1 (2 instances) -3.2 % (round 3, batch walk).  With the streamed lanes
// (trace_stream, flat walk only) C1 gains too -- TEST_MCPT 1448 -> 1512, ReSTIR 1388 -> 1417
// Msamples/s (round 5) -- so every scene takes the flat walk.
constexpr uint32_t kFlatMinInstances = 1u;
#ifndef PTX_LDS_TRANS
#define PTX_LDS_TRANS 1  // the restart test's transmission from the LDS root table (A/B: 0 = Scene::mats)
#endif
// The queries of one wave: lane state {ray, kind, transmittance T, remaining distance, segment}
// for query slot gi (its result at res[2 gi]).  Visibility (SH/PT_1_InitPass.wgsl:774-802) walks
// through transmissive hits: one trace site, looped, so the traversal code is emitted once.
// (A form that parked a wave's few restarting lanes in a per-wave pool and walked them later as
// one batch measured -7.5 % on the headline, 442 vs 477 Msamples/s: round 4)
template <bool COUNT, bool PROF, bool OCC, bool LDS_TABLES, bool FLAT>
__device__ __forceinline__ void trace_lanes(const Scene &sc, const SubRoot *subs, const Inst *insts, PassEps eps,
                                            uint32_t *stack, CoopLds coop, Ray r, uint32_t kind, float T, float remain,
                                            uint32_t seg, bool active, float4 *res, uint32_t gi, uint32_t *dbg) {
    const bool vis = kind != Q_CLOSEST;
    for (;;) {
        const float t_max = !active ? __builtin_nanf("") : vis ? fminf(remain, 1e10f) : 1e10f;
        // a Visibility hit's position is only needed to restart through a transmissive surface:
        // it is reconstructed below for those lanes only
        Hit h = (LDS_TABLES && FLAT)
                    ? trace_core_flat<COUNT, PROF, OCC>(sc, subs, insts, r, eps, stack, WB, t_max, coop, !vis, dbg)
                    : trace_core_tab<COUNT, PROF, true, OCC, TRACE_COOP, LDS_TABLES && PTX_NODE_UNI>(
                          sc, subs, insts, r, eps, stack, WB, t_max, coop, !vis);
        if (active && !vis) {
            const uint32_t enc = ((h.valid ? 1u : 0u) << 31) | (h.s.inst << 16) | h.s.mat;
            res[2u * gi] = make_float4(h.t, asf(enc), asf(h.s.prim), h.s.bu);
            res[2u * gi + 1u] = make_float4(h.s.bv, h.pos.x, h.pos.y, h.pos.z);
            active = false;
        } else if (active) {
            float out = -1.0f;
            if (!h.valid || h.t > remain) out = T;
            else {
                const float tr = kind == Q_OCC              ? 0.0f
                                 : PTX_LDS_TRANS ? subs_transmission(subs, insts, h.s.inst, h.s.mat)
                                                 : get_transmission(sc, h.s.inst, h.s.mat);
                if (tr == 0.0f) out = 0.0f;
                else {
                    T *= tr;
                    remain -= h.t;
                    complete_hit(sc, r, eps, h, insts);
                    r.o = h.pos;
                    if (seg == 4u) out = 0.0f;  // Visibility gives up after 5 segments
                    ++seg;
                }
            }
            if (out >= 0.0f) {  // only res.x is written: .yzw and res[2i+1] carry the payload
                res[2u * gi].x = out;
                active = false;
            }
        }
        if (wballot(active) == 0ull) break;
    }
}
// Lane i of the wave traces query i of a batch (`rays` / `res` = the segment's, slot
// gbase + i of the launch's buffers rays_all / res_all).
template <bool COUNT, bool PROF, bool OCC, bool LDS_TABLES = false, bool FLAT = false>
__device__ __forceinline__ void trace_batch(const Scene &sc, const SubRoot *subs, const Inst *insts, PassEps eps,
                                            uint32_t *stack, CoopLds coop, float4 *res_all, const float4 *rays_all,
                                            uint32_t gbase, uint32_t i, bool active, uint32_t *dbg = nullptr) {
    const uint32_t gi = gbase + i;
    float4 a = make_float4(0.0f, 0.0f, 0.0f, 0.0f), b = make_float4(0.0f, 0.0f, 1.0f, 0.0f);
    if (active) {
        a = rays_all[2u * gi];
        b = rays_all[2u * gi + 1u];
    }
    trace_lanes<COUNT, PROF, OCC, LDS_TABLES, FLAT>(sc, subs, insts, eps, stack, coop, Ray{mk(a.x, a.y, a.z), mk(b.x, b.y, b.z)},
                                                    asu(b.w), 1.0f, a.w, 0u, active, res_all, gi, dbg);
}
}  // namespace ptx
#include "ptx_stream.h"
namespace ptx {

// Dynamic batches (WaveBufs::dyn): the launch's rays -- every slot of the launch's segment
// range -- are one list of 64-query batches (a slot's batch k = its queries 64k .. 64k+63,
// consecutive entries of one tile, coherent), and every wave takes the next batch from a
// per-(part, round) counter until the list is exhausted.  A launch then ends when the
// last batch ends, not when the heaviest segment does: with a fixed slot per workgroup
// the spatial pass's largest trace launch ran its median workgroup 1.14 ms and its slowest
// 1.90 ms (tools/wave_timeline.py).  Each query's result goes to its own slot, so the
// assignment of batches to waves changes nothing in the output.  The workgroup's first
// (seg_count + 1) dynamic-LDS words hold the exclusive prefix of the slots' batch counts.
__device__ __forceinline__ uint32_t dyn_prefix_words(const WaveBufs &w) { return (w.seg_count + 4u) & ~3u; }
__device__ __forceinline__ void dyn_prefix(const WaveBufs &w, uint32_t round, uint32_t *pref) {
    __shared__ uint32_t l_wsum[WB / 64];
    const uint32_t n = w.seg_count, per = (n + WB - 1u) / WB, t0 = threadIdx.x * per;
    const uint32_t *cnt = w.cnt + (2u * round + 1u) * w.cnt_stride + w.seg_phys + w.seg_base;
    uint32_t loc = 0u;
    for (uint32_t k = 0; k < per && t0 + k < n; ++k) loc += (cnt[t0 + k] + 63u) >> 6;
    uint32_t total;
    uint32_t ex = wave_scan(loc, total);
    if (__lane_id() == 63u) l_wsum[threadIdx.x >> 6] = ex + loc;
    __syncthreads();
    for (uint32_t q = 0; q < (threadIdx.x >> 6); ++q) ex += l_wsum[q];
    for (uint32_t k = 0; k < per && t0 + k < n; ++k) {
        pref[t0 + k] = ex;
        ex += (cnt[t0 + k] + 63u) >> 6;
    }
    if (threadIdx.x == WB - 1u) pref[n] = ex;
    __syncthreads();
}

// The dynamic trace batches (WaveBufs::dyn) and split segments (WaveBufs::trace_split) are A/B
// modes of the measurement build since late round 5 (every production frame traces static slots,
// one workgroup per segment: use_dyn_batches): the shipped kernel is compiled without those
// branches (their batch walks spilled 28 B per lane into the streamed static path).
#ifndef PTX_TRACE_AB_PATHS
#ifdef PTX_AB_BUILD
#define PTX_TRACE_AB_PATHS 1
#else
#define PTX_TRACE_AB_PATHS 0
#endif
#endif
constexpr bool kAbBuild = PTX_TRACE_AB_PATHS != 0;
template <bool COUNT, int WAVES, bool PROF = false, bool LDS_TABLES = true, bool OCC = false, bool FLAT = false>
__global__ __launch_bounds__(WB) __attribute__((amdgpu_waves_per_eu(WAVES, 8)))
void trace_queue(Scene sc, WaveBufs w, uint32_t round, PassEps eps) {
    PTX_WAVE_TIMER(sc, KID_TRACE | (w.seg_base ? 0x80u : 0u));
    // dynamic LDS: [scene tables (LDS_TABLES)] [batch prefix (dynamic batches)] [stacks]
    extern __shared__ __attribute__((aligned(16))) uint32_t wstack[];
    const bool dyn = kAbBuild && !COUNT && w.dyn != nullptr;
    const uint32_t tw = LDS_TABLES ? tables_lds_bytes(sc) / 4u : 0u;
    uint32_t *pref = wstack + tw;
    uint32_t *stack = wstack + tw + (dyn ? dyn_prefix_words(w) : 0u) + threadIdx.x;
    __shared__ unsigned long long c_key[WB];
    __shared__ uint32_t c_mark[WB];
    const CoopLds coop{c_key + (threadIdx.x & ~63u), c_mark + (threadIdx.x & ~63u)};
    if (dyn) {
        dyn_prefix(w, round, pref);
        const uint32_t total = pref[w.seg_count];
        if (blockIdx.x * (WB / 64u) >= total) return;  // (workgroup-uniform) more waves than batches
        const LdsTables T = LDS_TABLES ? stage_tables(sc, wstack) : LdsTables{sc.subs, sc.insts};
        const SubRoot *subs = T.subs;
        const Inst *insts = T.insts;
        // the batch list in kDynHeads contiguous chunks, chunk x dequeued through head x by the
        // waves of XCD x (workgroups are dealt to the XCDs round-robin: block b on XCD b % 8);
        // a wave whose chunk is drained moves on to the next one
        uint32_t *heads = w.dyn + round * kDynRoundWords;
        const uint32_t lane = __lane_id();
        float4 *res_all = res_buf(w, round);
        if constexpr (PTX_TRACE_STREAM && LDS_TABLES && FLAT && !COUNT) {  // lane refill (trace_stream)
            trace_stream<PROF, OCC, true>(sc, subs, insts, eps, stack, coop, w, round, pref, heads, res_all);
            return;
        }
        uint32_t x = blockIdx.x % kDynHeads, visited = 0u;
        uint32_t c0 = (uint32_t)((uint64_t)total * x / kDynHeads), c1 = (uint32_t)((uint64_t)total * (x + 1u) / kDynHeads);
        // each dequeue takes G consecutive batches (WaveBufs::trace_split in this mode): one
        // atomic per G * 64 queries, traced back to back by the same wave
        const uint32_t G = w.trace_split;
        uint32_t bnext = 0u;
        if (lane == 0u) bnext = atomicAdd(heads + x * kDynStride, 1u);
        // one trace_batch per dequeued batch, every Visibility restart in place
        uint32_t bi = c0 + G * (uint32_t)__builtin_amdgcn_readfirstlane((int)bnext);
        for (;;) {  // wave-uniform
            if (bi >= c1) {  // this chunk is drained: the next head
                if (++visited == kDynHeads) break;
                x = (x + 1u) % kDynHeads;
                c0 = (uint32_t)((uint64_t)total * x / kDynHeads);
                c1 = (uint32_t)((uint64_t)total * (x + 1u) / kDynHeads);
                if (lane == 0u) bnext = atomicAdd(heads + x * kDynStride, 1u);
                bi = c0 + G * (uint32_t)__builtin_amdgcn_readfirstlane((int)bnext);
                continue;
            }
            if (lane == 0u) bnext = atomicAdd(heads + x * kDynStride, 1u);  // the next dequeue, fetched ahead
            const uint32_t bend = min(bi + G, c1);
            uint32_t lo = 0u;
            for (; bi < bend; ++bi) {
                uint32_t hi = w.seg_count;  // last slot with pref <= bi (batches ascend: search from lo)
                while (hi - lo > 1u) {
                    const uint32_t mid = (lo + hi) >> 1;
                    if (pref[mid] <= bi) lo = mid;
                    else hi = mid;
                }
                const uint32_t j = w.seg_phys + w.seg_base + lo;
                const uint32_t n = w.cnt[(2u * round + 1u) * w.cnt_stride + j];
                const uint32_t i = (bi - pref[lo]) * 64u + lane;
#ifdef PTX_WG_TIMES
                const unsigned long long tb0 = __builtin_amdgcn_s_memrealtime();
                uint32_t dbg[6] = {0u, 0u, 0u, 0u, 0u, 0u};
#else
                uint32_t *dbg = nullptr;
#endif
                trace_batch<COUNT, PROF, OCC, LDS_TABLES, FLAT>(sc, subs, insts, eps, stack, coop,
                                                                 res_all + 2u * (size_t)j * w.ray_stride,
                                                                 w.rays + 2u * (size_t)j * w.ray_stride, 0u, i, i < n, dbg);
#ifdef PTX_WG_TIMES
                batch_record(sc.wgt, tb0, bi, round, dbg);
#endif
            }
            bi = c0 + G * (uint32_t)__builtin_amdgcn_readfirstlane((int)bnext);
        }
        return;
    }
    // Static: workgroup -> (segment, share): the trace_split workgroups of a segment take its
    // 256-ray batches round-robin; results go to the rays' own slots, so the split is exact.
    // A segment's shares are consecutive blocks, so they spread over XCDs (blocks b and b+8
    // share one: MI355X_MICROARCH.md, workgroup dispatch) -- measured faster than keeping
    // them on one XCD.  For K | 8 the share index rotates with b / 8, else share 0 (the
    // heaviest) would always land on the same XCDs.
    const uint32_t K = w.trace_split, b = blockIdx.x;
    const uint32_t share = (b % K + ((8u % K) == 0u ? (b >> 3) : 0u)) % K, local = b / K;
    const uint32_t j = w.seg_phys + w.seg_base + local;  // physical queue slot
    const uint32_t n = w.cnt[(2u * round + 1u) * w.cnt_stride + j];
    if (share * WB >= n) return;  // (workgroup-uniform) nothing for this share
    __shared__ uint32_t l_next;   // (trace_stream's batch counter)
    if (threadIdx.x == 0u) l_next = 0u;  // (ordered by stage_tables' barrier)
    const LdsTables T = LDS_TABLES ? stage_tables(sc, wstack) : LdsTables{sc.subs, sc.insts};
    const SubRoot *subs = T.subs;
    const Inst *insts = T.insts;
    if constexpr (PTX_TRACE_STREAM && LDS_TABLES && FLAT && !COUNT) {  // lane refill over the segment
        if (!kAbBuild || K == 1u) {
            trace_stream<PROF, OCC, false>(sc, subs, insts, eps, stack, coop, w, round, nullptr, nullptr,
                                           res_buf(w, round), &l_next, j, n);
            return;
        }
    }
    if (COUNT && sc.census)  // row census: this slot's queries count into its own block
        sc.counters = sc.census + (size_t)kCensusWords * ((sc.row_end - sc.row_begin + 7u) / 8u + j);
    for (uint32_t i0 = share * WB; i0 < n; i0 += K * WB) {  // workgroup-uniform
        const uint32_t i = i0 + threadIdx.x;
        trace_batch<COUNT, PROF, OCC, LDS_TABLES, FLAT>(sc, subs, insts, eps, stack, coop, res_buf(w, round), w.rays,
                                                         j * w.ray_stride, i, i < n);
    }
}

// Lane-refill form of the same queries.  The whole traversal -- instance loop, sub-root
// loop, BLAS stack walk, leaf triangle loop and the Visibility continuation -- is one
// flat per-lane state machine: every iteration a lane does ONE unit of work (a node-pair
// test, a triangle test, or a root/instance step), and a lane whose ray is done takes
// the segment's next ray at once instead of idling until the wave's slowest ray ends.
// Per ray the visit order (and so the hit, ties included, and the work counters) is the
// reference's exactly: only the interleaving across lanes changes.
// Workgroup j handles segment j: `cnt` given -> cnt[j] rays at j * stride (queue layout
// {o, remain}, {d, kind}); `cnt` null -> rays [j * stride, min((j+1) * stride, n_total))
// in the public ptx_trace layout {o.xyz, d.x}, {d.yz, -, -} (closest hit only).
template <bool COUNT>
__global__ __launch_bounds__(WB) void trace_queue_sm(Scene sc, const float4 *rays_all, float4 *res_all,
                                                     const uint32_t *cnt, uint32_t stride, uint32_t n_total,
                                                     PassEps eps) {
    extern __shared__ __attribute__((aligned(16))) uint32_t wstack[];
    uint32_t *stack = wstack + threadIdx.x;
    const uint32_t j = blockIdx.x;
    const bool pub = cnt == nullptr;
    const uint32_t n = pub ? min(stride, n_total - j * stride) : cnt[j];
    const float4 *rays = rays_all + 2u * (size_t)j * stride;
    float4 *res = res_all + 2u * (size_t)j * stride;
    const float vx = 1e-4f;
    const uint32_t n_inst = sc.n_inst;

    uint32_t next = threadIdx.x, cur = 0u;
    bool have = false;
    Ray r{};                       // world ray of the current trace
    bool vis = false;              // Visibility / occlusion query (else closest hit)
    bool occ = false;              // occlusion query: every hit inside `remain` blocks
    float T = 1.0f, remain = 0.0f; // Visibility product / remaining distance
    uint32_t vit = 0u;             // Visibility segment (0..4)
    uint32_t ii = 0u, s = 0u, nsub = 0u, grp = 0u, sub_base = 0u, tri_base = 0u;
    f3 lo{}, ld{}, inv{};          // ray in the current instance's space
    int sp = -1;
    uint32_t tcount = 0u, tprim = 0u, tidx = 0u;  // leaf cursor
    float vy = 1e10f;
    bool bvalid = false;
    uint32_t binst = 0u, bmat = 0u, bprim = 0u;
    uint32_t n_aabb = 0u, n_tri = 0u;

    for (;;) {
        if (!have && next < n) {  // fetch the next ray of the segment
            cur = next;
            next += WB;
            const float4 a = rays[2u * cur], b = rays[2u * cur + 1u];
            r = pub ? Ray{mk(a.x, a.y, a.z), mk(a.w, b.x, b.y)} : Ray{mk(a.x, a.y, a.z), mk(b.x, b.y, b.z)};
            vis = !pub && asu(b.w) != Q_CLOSEST;
            occ = !pub && asu(b.w) == Q_OCC;
            T = 1.0f;
            remain = a.w;
            vit = 0u;
            have = true;
            ii = 0xffffffffu; s = 0u; nsub = 0u; sp = -1; tcount = 0u;
            vy = vis ? fminf(remain, 1e10f) : 1e10f;
            bvalid = false; n_aabb = 0u; n_tri = 0u;
        }
        if (__ballot(have) == 0ull) break;
        if (!have) continue;

        bool do_node = false;
        uint32_t node = 0u;
        if (tcount == 0u) {
            if (sp >= 0) {
                const uint32_t ref = stack[(uint32_t)sp * WB];
                --sp;
                if (ref & LEAF_BIT) {
                    tcount = (ref >> 24) & 0x7Fu;
                    tprim = ref & LEAF_FIRST_MASK;
                    tidx = 3u * (tri_base + tprim);
                } else {
                    do_node = true;
                    node = ref;
                }
            } else if (s < nsub) {  // next sub-mesh root of this instance
                const SubRoot &R = sc.subs[sub_base + s];
                grp = s;
                ++s;
                ++n_aabb;
                if (box_root(lo, inv, R, vx, vy)) {
                    sp = 0;
                    stack[0] = R.ref;
                }
            } else if (ii + 1u < n_inst) {  // next instance (ii starts at ~0u: wraps to 0)
                ii = ii + 1u;
                const Inst &I = sc.insts[ii];
                lo = xform_point(I.minv, r.o);
                const f3 le = xform_point(I.minv, r.o + r.d);
                ld = le - lo;
                inv = mk(1.0f / ld.x, 1.0f / ld.y, 1.0f / ld.z);
                nsub = I.nsub;
                sub_base = I.sub_base;
                tri_base = I.tri_base;
                s = 0u;
            } else {  // this trace is complete
                if (COUNT) {
                    atomicAdd(&sc.counters[CNT_RAYS], 1ull);
                    atomicAdd(&sc.counters[CNT_INST], (unsigned long long)n_inst);
                    atomicAdd(&sc.counters[CNT_AABB], (unsigned long long)n_aabb);
                    atomicAdd(&sc.counters[CNT_TRI], (unsigned long long)n_tri);
                    if (bvalid) atomicAdd(&sc.counters[CNT_HITS], 1ull);
                }
                Hit h;
                h.valid = bvalid;
                h.t = bvalid ? vy : 0.0f;
                h.s = Compact{0u, bvalid ? binst : 0u, bvalid ? bmat : 0u, bvalid ? bprim : 0u, 0.0f, 0.0f};
                h.pos = mk(0.0f, 0.0f, 0.0f);
                if (!vis) {
                    if (bvalid) complete_hit(sc, r, eps, h);
                    const uint32_t enc = ((h.valid ? 1u : 0u) << 31) | (h.s.inst << 16) | h.s.mat;
                    res[2u * cur] = make_float4(h.t, asf(enc), asf(h.s.prim), h.s.bu);
                    res[2u * cur + 1u] = make_float4(h.s.bv, h.pos.x, h.pos.y, h.pos.z);
                    have = false;
                } else {  // Visibility step (SH/PT_1_InitPass.wgsl:774-802)
                    float out = -1.0f;
                    if (!h.valid || h.t > remain) out = T;
                    else {
                        const float tr = occ ? 0.0f : get_transmission(sc, h.s.inst, h.s.mat);
                        if (tr == 0.0f) out = 0.0f;
                        else {
                            T *= tr;
                            remain -= h.t;
                            if (vit == 4u) out = 0.0f;  // gives up after 5 segments
                            else {
                                complete_hit(sc, r, eps, h);
                                r.o = h.pos;
                                ++vit;
                                ii = 0xffffffffu; s = 0u; nsub = 0u; sp = -1; tcount = 0u;
                                vy = fminf(remain, 1e10f);
                                bvalid = false; n_aabb = 0u; n_tri = 0u;
                            }
                        }
                    }
                    if (out >= 0.0f) {  // only res.x: .yzw and res[2i+1] carry the payload
                        res[2u * cur].x = out;
                        have = false;
                    }
                }
                continue;
            }
        }
        if (tcount > 0u) {  // one triangle of the current leaf
            const float4 a = sc.tris[tidx], b = sc.tris[tidx + 1u], c = sc.tris[tidx + 2u];
            const float t = ray_tri(lo, ld, a, b, c, eps.det_eps);
            ++n_tri;
            if (!(vy < t)) {
                vy = t;
                bvalid = true;
                binst = ii;
                bmat = grp;
                bprim = tprim;
            }
            tidx += 3u;
            ++tprim;
            --tcount;
        } else if (do_node) {  // one interior node: both children, nearer on top
            const float4 *np = reinterpret_cast<const float4 *>(sc.nodes + node);
            const float4 q0 = np[0], q1 = np[1], q2 = np[2], q3 = np[3];
            const uint32_t lref = __float_as_uint(q3.x), rref = __float_as_uint(q3.y);
            float tl, tr;
            bool hl, hr;
            box_pair(lo, inv, q0, q1, q2, vx, vy, hl, hr, tl, tr);
            n_aabb += 2u;
            if (hl && hr) {
                stack[(uint32_t)(sp + 1) * WB] = tl < tr ? rref : lref;
                stack[(uint32_t)(sp + 2) * WB] = tl < tr ? lref : rref;
                sp += 2;
            } else if (hl || hr) {
                stack[(uint32_t)(sp + 1) * WB] = hl ? lref : rref;
                sp += 1;
            }
        }
    }
}

// =========================================================================== PT_01 (G-buffer)
// PT_01 over the pixels of segments [seg_base, seg_base + seg_count): 4 workgroups per
// segment, one 8x8 tile per wave, so a frame can run G-buffer -> init -> final per segment
// group with no dependency between groups.  Same ray, epsilons and traversal as
// gbuffer_kernel (SH/PT_01_GBufferPass.wgsl:496-507,643-656).
template <bool ROOTQ>
__global__ __launch_bounds__(WB) void wgbuffer(Scene sc, WaveBufs w, uint4 *gbuf) {
    PTX_WAVE_TIMER(sc, KID_GBUF);
    extern __shared__ __attribute__((aligned(16))) uint32_t wstack[];  // [scene tables] [stacks]
    uint32_t *stack = wstack + tables_lds_bytes(sc) / 4u + threadIdx.x;
    const LdsTables T = stage_tables(sc, wstack);
    // The group's pixels are the tiles t = m * nseg + r, r in [seg_base, seg_base + seg_count)
    // (seg_pixel's layout, cluster 1); walking them in raster order gives each workgroup 4
    // adjacent tiles (a 32x8 strip) -- primary rays of one CU then share BVH nodes in L1.
    const uint32_t L = blockIdx.x * 4u + threadIdx.x / 64u, run = w.cluster * w.seg_count;
    const uint32_t t = set_tile(w, (L / run) * w.cluster * w.nseg + w.cluster * w.seg_base + L % run);
    const uint32_t q = t * 64u + (threadIdx.x & 63u);
    uint32_t x, y;
    if (q >= padded_pixels(sc) || !tile_xy(sc, q, x, y)) return;
    const float *vpinv = reinterpret_cast<const float *>(sc.U + U_VPINV);
    const float u = ((float)x + 0.5f) / (float)sc.U[U_W];
    const float v = ((float)y + 0.5f) / (float)sc.U[U_H];
    const f3 st = xform_point(vpinv, mk(2.0f * u - 1.0f, 2.0f * v - 1.0f, 0.0f));
    const f3 en = xform_point(vpinv, mk(2.0f * u - 1.0f, 2.0f * v - 1.0f, 0.0f + 1.0f));
    const Hit h = trace_core_tab<false, false, ROOTQ>(sc, T.subs, T.insts, Ray{st, normalize(en - st)},
                                                      PassEps{1e-8f, 1e-6f}, stack, WB);
    Compact c = h.s;
    c.valid = h.valid ? 1u : 0u;
    gbuf[(y - sc.row_begin) * sc.width + x] = gencode(c);
}

// =========================================================================== PT_1 (init)
// Pixel state, SoA float4 slots (slot k of pixel p at state[k * npix + p]).
enum : uint32_t { IS_HDR, IS_FP, IS_RES, IS_X, IS_XL, IS_L, IS_BSEED, IS_CS2, IS_CS3, IS_TSEL, IS_COUNT };
static_assert(IS_CS2 == kStateCs2 && IS_CS3 == kStateCs3 && IS_TSEL == kStateTsel && IS_COUNT <= kWaveStateSlots,
              "PT_1 state slots read by the temporal pass (ptx_reuse.hip)");
// flags (IS_HDR.y >> 8): bit0 selected, bit1 has BSDF ray, bit2 far12, bit3 far23,
// bit4 rough1 >= 0.5, bit5 rough2 >= 0.5, bits 8-9 Lobe[1], bits 10-11 Lobe[2]
enum : uint32_t { F_SEL = 1u, F_BSDF = 2u, F_FAR12 = 4u, F_FAR23 = 8u, F_R1 = 16u, F_R2 = 32u };

struct WInit {
    uint32_t seed, i, flags, C, vis_idx, bsdf_idx;
    f3 f; float p;
    float w_sum, p_hat_sel, pdf_env;
    f3 xpos; float xrough;
    f3 xlpos; uint32_t nee_seed;
    f3 L;
    uint32_t bseed1, bseed2;
};
__device__ __forceinline__ uint32_t lobe_of(uint32_t flags, uint32_t k) { return (flags >> (8u + 2u * (k - 1u))) & 3u; }

// CompressPath for the candidate (vertex i, NEE or env) -- same rules as ptx_persist.hip.
// rcnext (the reuse pipeline): x_{k+1}'s compact in pad words 24..27 when the hybrid shift keeps
// a vertex after x_k (k = 2, length 4: x3), as the oracle's compress_path.
__device__ __forceinline__ void wcompress(const Scene &sc, const WInit &s, const float4 *state, uint32_t npix,
                                          uint32_t pix, bool is_env, const LightSample &XL, uint4 *out,
                                          bool rcnext) {
    const uint32_t i = s.i, length = i + 1u;
    const uint32_t L1 = (i > 1u || is_env) ? lobe_of(s.flags, 1u) : 0u;
    const uint32_t L2 = (i > 2u || (is_env && i == 2u)) ? lobe_of(s.flags, 2u) : 0u;
    const uint32_t s2 = (i >= 2u || is_env) ? s.bseed1 : s.nee_seed;
    const uint32_t s3 = (i >= 3u || (i == 2u && is_env)) ? s.bseed2 : (i == 2u ? s.nee_seed : 0u);
    const uint32_t s4 = (i == 3u) ? s.nee_seed : 0u;
    uint32_t k = 0u;
    if (length > 2u) {
        bool ok = (L1 == LOBE_LAMBERT || (s.flags & F_R1)) && (L2 == LOBE_LAMBERT || (s.flags & F_R2));
        if ((s.flags & F_FAR12) && ok) k = 2u;
    }
    if (k == 0u && length > 3u) {
        bool ok = (L2 == LOBE_LAMBERT || (s.flags & F_R2));
        if ((s.flags & F_FAR23) && ok) k = 3u;
    }
    if (k == 0u) {
        bool rough = s.xrough >= RECONNECTION_ROUGHNESS;
        bool dirl = XL.type == LIGHT_DIRECTION || XL.type == LIGHT_ENV;
        if ((dirl || length3(s.xpos - XL.pos) >= RECONNECTION_DISTANCE) && rough) k = length;
    }
    uint4 rc = make_uint4(0u, 0u, 0u, 0u);
    uint32_t lk = 0u, lk1 = 0u;
    if (k == length) {
        lk = LOBE_LIGHT;
        lk1 = (k == 2u) ? L1 : (k == 3u) ? L2 : 0u;
    } else if (k == 2u) {
        lk = L2; lk1 = L1;
        const float4 c = state[IS_CS2 * npix + pix];
        rc = make_uint4(asu(c.x), asu(c.y), asu(c.z), asu(c.w));
    } else if (k == 3u) {
        lk1 = L2;
        const float4 c = state[IS_CS3 * npix + pix];
        rc = make_uint4(asu(c.x), asu(c.y), asu(c.z), asu(c.w));
    }
    out[0] = make_uint4(s2, s3, s4, 0u);
    out[1] = make_uint4(asu(XL.dir.x), asu(XL.dir.y), asu(XL.dir.z), XL.type);
    out[2] = make_uint4(asu(XL.pos.x), asu(XL.pos.y), asu(XL.pos.z), (uint32_t)XL.id);
    out[3] = make_uint4(asu(XL.Le.x), asu(XL.Le.y), asu(XL.Le.z), asu(XL.pdf));
    out[4] = rc;
    out[5] = make_uint4(k, lk1, lk, length);
    uint4 nx = make_uint4(0u, 0u, 0u, 0u);
    if (rcnext && k == 2u && length == 4u) {
        const float4 c = state[IS_CS3 * npix + pix];
        nx = make_uint4(asu(c.x), asu(c.y), asu(c.z), asu(c.w));
    }
    out[6] = nx;
}

// Vertex i of the path tree up to (not including) its traces (PT_1:1403-1442): NEE sample,
// its contribution before Visibility, the UpdateReservoir draw, BSDF sample, throughput,
// Russian roulette.  Emits the shadow ray (payload in its result slot) and the BSDF ray.
// Called by every lane of the wave (queue slots are reserved per wave); `emit` selects
// the lanes that actually have a vertex.
__device__ __forceinline__ void winit_vertex(const Scene &sc, const Seg &g, bool emit, WInit &s, const Surface &X,
                                             f3 prev) {
    float4 *rays = g.rays, *res = g.res_out;
    const uint32_t vbase = g.rbase + wave_alloc(g.l_ray, emit ? 1u : 0u);
    bool bsdf_ray = false;
    if (emit) {
        const f3 V = normalize(prev - X.pos);
        s.nee_seed = s.seed;
        const LightSample XL = sample_nee(sc, s.seed, X, V);
        const f3 Ln = direction_to_light(X, XL);
        f3 contrib = s.f * l_emit<false>(XL, X);
        contrib = contrib * bsdf(X, V, Ln);
        contrib = contrib * fabsf(dot(X.nrm, Ln));
        const float denom = s.p * XL.pdf;
        const float u_update = rnd(s.seed);
        s.xlpos = XL.pos;
        s.xpos = X.pos;
        s.xrough = X.mat.rough;
        s.vis_idx = vbase;
        const float dist = length(XL.pos - X.pos);
        put_ray(rays, vbase, X.pos, (XL.pos - X.pos) / dist, dist, Q_VIS);
        res[2u * vbase] = make_float4(0.0f, contrib.x, contrib.y, contrib.z);
        res[2u * vbase + 1u] = make_float4(denom, u_update, XL.pdf, asf((uint32_t)XL.id));
        if (s.i < 3u) {
            if (s.i == 1u) s.bseed1 = s.seed;
            else s.bseed2 = s.seed;
            uint32_t lobe;
            const f3 Lb = sample_bsdf(s.seed, X, V, lobe);
            s.flags |= lobe << (8u + 2u * (s.i - 1u));
            float pdfv;
            const f3 bv = bsdf_pdf(X, V, Lb, pdfv);
            s.f = s.f * (bv * fabsf(dot(X.nrm, Lb)));
            s.p *= pdfv;
            const float ps = luminance(s.f) / s.p;
            if (rnd(s.seed) < ps) {
                s.p *= ps;
                s.pdf_env = pdfv;
                s.L = Lb;
                bsdf_ray = true;
            }
        }
        s.flags = bsdf_ray ? (s.flags | F_BSDF) : (s.flags & ~F_BSDF);
    }
    const uint32_t bbase = g.rbase + wave_alloc(g.l_ray, bsdf_ray ? 1u : 0u);
    if (bsdf_ray) {
        s.bsdf_idx = bbase;
        put_ray(rays, bbase, s.xpos, s.L, -1.0f, Q_CLOSEST);
    }
}

__device__ __forceinline__ void winit_store(float4 *state, uint32_t npix, uint32_t pix, const WInit &s) {
    state[IS_HDR * npix + pix] = make_float4(asf(s.seed), asf(s.i | (s.flags << 8)), asf(s.C), asf(s.vis_idx));
    state[IS_FP * npix + pix] = make_float4(s.f.x, s.f.y, s.f.z, s.p);
    state[IS_RES * npix + pix] = make_float4(s.w_sum, s.p_hat_sel, s.pdf_env, asf(s.bsdf_idx));
    state[IS_X * npix + pix] = make_float4(s.xpos.x, s.xpos.y, s.xpos.z, s.xrough);
    state[IS_XL * npix + pix] = make_float4(s.xlpos.x, s.xlpos.y, s.xlpos.z, asf(s.nee_seed));
    state[IS_L * npix + pix] = make_float4(s.L.x, s.L.y, s.L.z, 0.0f);
    state[IS_BSEED * npix + pix] = make_float4(asf(s.bseed1), asf(s.bseed2), 0.0f, 0.0f);
}
__device__ __forceinline__ void winit_load(const float4 *state, uint32_t npix, uint32_t pix, WInit &s) {
    const float4 h = state[IS_HDR * npix + pix], fp = state[IS_FP * npix + pix], r = state[IS_RES * npix + pix];
    const float4 x = state[IS_X * npix + pix], xl = state[IS_XL * npix + pix], l = state[IS_L * npix + pix];
    const float4 b = state[IS_BSEED * npix + pix];
    s.seed = asu(h.x); s.i = asu(h.y) & 0xffu; s.flags = asu(h.y) >> 8; s.C = asu(h.z); s.vis_idx = asu(h.w);
    s.f = mk(fp.x, fp.y, fp.z); s.p = fp.w;
    s.w_sum = r.x; s.p_hat_sel = r.y; s.pdf_env = r.z; s.bsdf_idx = asu(r.w);
    s.xpos = mk(x.x, x.y, x.z); s.xrough = x.w;
    s.xlpos = mk(xl.x, xl.y, xl.z); s.nee_seed = asu(xl.w);
    s.L = mk(l.x, l.y, l.z);
    s.bseed1 = asu(b.x); s.bseed2 = asu(b.y);
}
__device__ __forceinline__ void winit_finish(const WInit &s, uint4 *reservoir, uint32_t pix) {
    uint4 *out = reservoir + 8u * (size_t)pix;
    if (!(s.flags & F_SEL))  // zero Path(): length 0, k 0 (no candidate ever accepted)
        for (int q = 0; q < 7; ++q) out[q] = make_uint4(0u, 0u, 0u, 0u);
    out[7] = make_uint4(asu(s.w_sum / s.p_hat_sel), s.C, 0u, 0u);
}

__global__ __launch_bounds__(WB) __attribute__((amdgpu_waves_per_eu(LOGIC_WAVES, 8))) void winit_start(Scene sc, WaveBufs w, const uint4 *gbuf, uint4 *reservoir) {
    PTX_WAVE_TIMER(sc, KID_INIT_START | (w.seg_base ? 0x80u : 0u));
    __shared__ uint32_t lds[3];
    const JobLists JL = job_lists(w, lds);
    const Seg g = seg_begin(w, 0u, lds);
    float4 *state = w.state;
    const uint32_t npix = w.npix, np = padded_pixels(sc);
    for (uint32_t k = 0; k < w.seg_px; k += WB) {  // workgroup-uniform loop
        const uint32_t q = seg_pixel(w, g.j, k);
        uint32_t x, y, pix = 0u;
        bool active = false;
        WInit s;
        Surface X;
        f3 prev;
        if (q < np && tile_xy(sc, q, x, y)) {
            pix = (y - sc.row_begin) * sc.width + x;
            const Compact x1 = gdecode(gbuf[pix]);
            if (!x1.valid) {  // reservoir unobservable: PT_4 returns before LoadReservoir (:1404-1408)
                uint4 *out = reservoir + 8u * (size_t)pix;
                for (int q8 = 0; q8 < 8; ++q8) out[q8] = make_uint4(0u, 0u, 0u, 0u);
                if (w.surf) surf_store_none(w.surf, pix);
            } else {
                active = true;
                s.seed = pcg(x * 1973u + y * 9277u + sc.U[U_FRAME] * 26699u);
                s.i = 1u; s.flags = 0u; s.C = 0u;
                s.f = mk(1.0f, 1.0f, 1.0f); s.p = 1.0f;
                s.w_sum = 0.0f; s.p_hat_sel = 0.0f; s.pdf_env = 0.0f;
                s.L = mk(0.0f, 0.0f, 0.0f); s.bseed1 = 0u; s.bseed2 = 0u; s.bsdf_idx = 0u;
                prev = x0_of(sc, x, y);
                X = get_surface(sc, x1);
                if (w.surf) surf_store(w.surf, pix, X, mat_index(sc, x1.inst, x1.mat));  // for the reuse passes
                if (X.mat.rough >= RECONNECTION_ROUGHNESS) s.flags |= F_R1;
            }
        }
        // ray emission is executed by the whole wave (wave_alloc), active or not
        winit_vertex(sc, g, active, s, X, prev);
        if (active) winit_store(state, npix, pix, s);
        // light next round: no BSDF ray out, only the NEE candidate to book and the path to end
        job_keep(g, JL, active, active && !(s.flags & F_BSDF), pix);
    }
    job_seg_end(w, g, JL);
}

__global__ __launch_bounds__(WB) __attribute__((amdgpu_waves_per_eu(LOGIC_WAVES, 8))) void winit_step(Scene sc, WaveBufs w, uint32_t round, uint4 *reservoir) {
    PTX_WAVE_TIMER(sc, KID_INIT_STEP | (w.seg_base ? 0x80u : 0u));
    __shared__ uint32_t lds[3];
    const JobLists JL = job_lists(w, lds);
    const Seg g = seg_begin(w, round, lds);
    float4 *state = w.state;
    const float4 *res_in = g.res_in;
    const uint32_t npix = w.npix;
    uint32_t nh;
    const uint32_t n = split_count(g, nh);
    for (uint32_t base = 0; base < n; base += WB) {
        const uint32_t q = base + threadIdx.x;
        bool emit = false;
        uint32_t pix = 0u;
        WInit s;
        Surface X;
        f3 prev;
        if (q < n) {
            pix = split_at(g, JL, q, nh);
            winit_load(state, npix, pix, s);
            // 1. resolve the NEE candidate of vertex i with its Visibility (PT_1:1413-1421)
            const float4 a = res_in[2u * s.vis_idx], b = res_in[2u * s.vis_idx + 1u];
            const f3 contrib = mk(a.y, a.z, a.w) * a.x;
            const float p_hat = luminance(contrib);
            const float ris = p_hat / b.x;
            s.C += 1u;
            s.w_sum += ris;
            if (b.y < ris / s.w_sum) {
                s.flags |= F_SEL;
                s.p_hat_sel = p_hat;
                // the selected NEE candidate's Visibility (the temporal pass's canonical
                // evaluation reuses it instead of re-tracing the light segment)
                state[IS_TSEL * npix + pix] = make_float4(a.x, 0.0f, 0.0f, 0.0f);
                LightSample XL;
                const Light ls = get_light(sc, asu(b.w));
                XL.id = (int32_t)asu(b.w);
                XL.type = ls.type;
                XL.Le = ls.color * ls.intensity;
                XL.pos = s.xlpos;
                XL.pdf = b.z;
                XL.dir = ls.type == LIGHT_DIRECTION ? ls.dir
                         : ls.type == LIGHT_POINT  ? normalize(s.xpos - ls.pos)
                         : ls.type == LIGHT_RECT   ? normalize(s.xpos - s.xlpos)
                                                   : mk(0.0f, 0.0f, 0.0f);
                wcompress(sc, s, state, npix, pix, false, XL, reservoir + 8u * (size_t)pix, w.surf != nullptr);
            }
            if (!(s.flags & F_BSDF)) {
                winit_finish(s, reservoir, pix);  // i == 3 or Russian roulette ended the path
            } else {
                const Hit h = get_hit(res_in, s.bsdf_idx);
                if (!h.valid) {  // 2a. BSDF ray escaped: env candidate (PT_1:1447-1461)
                    const float u = rnd(s.seed);
                    const float ph = luminance(s.f * ENV_C);
                    const float ris_e = ph / s.p;
                    s.C += 1u;
                    s.w_sum += ris_e;
                    if (u < ris_e / s.w_sum) {
                        s.flags |= F_SEL;
                        s.p_hat_sel = ph;
                        state[IS_TSEL * npix + pix] = make_float4(-1.0f, 0.0f, 0.0f, 0.0f);  // env: traced later
                        LightSample env;
                        env.pos = s.xpos + s.L * INF_F;
                        env.type = LIGHT_ENV;
                        env.dir = -s.L;
                        env.id = -1;
                        env.Le = mk(ENV_C, ENV_C, ENV_C);
                        env.pdf = s.pdf_env;
                        wcompress(sc, s, state, npix, pix, true, env, reservoir + 8u * (size_t)pix, w.surf != nullptr);
                    }
                    winit_finish(s, reservoir, pix);
                } else {  // 2b. next vertex (PT_1:1464-1468)
                    X = surface_at(sc, h.s, h.pos);
                    prev = s.xpos;
                    s.i += 1u;
                    if (s.i == 2u) {
                        if (length3(prev - X.pos) >= RECONNECTION_DISTANCE) s.flags |= F_FAR12;
                        if (X.mat.rough >= RECONNECTION_ROUGHNESS) s.flags |= F_R2;
                        const uint4 e = gencode(h.s);
                        state[IS_CS2 * npix + pix] = make_float4(asf(e.x), asf(e.y), asf(e.z), asf(e.w));
                    } else {
                        if (length3(prev - X.pos) >= RECONNECTION_DISTANCE) s.flags |= F_FAR23;
                        const uint4 e = gencode(h.s);
                        state[IS_CS3 * npix + pix] = make_float4(asf(e.x), asf(e.y), asf(e.z), asf(e.w));
                    }
                    emit = true;
                }
            }
        }
        winit_vertex(sc, g, emit, s, X, prev);
        if (emit) winit_store(state, npix, pix, s);
        job_keep(g, JL, emit, emit && !(s.flags & F_BSDF), pix);
    }
    job_seg_end(w, g, JL);
}

// =========================================================================== PT_4 (final)
enum : uint32_t { FS_HDR, FS_F, FS_CUR, FS_NRM, FS_PREV, FS_COUNT };
// HDR: {i | length<<8 | phase<<16, seed1 (rSeed[1]), ray idx, -}; F: {f.xyz, UCW};
// CUR: {cur.pos, inst|mat}; NRM: {cur.nrm, -}; PREV: {prev.pos, -}

struct WFinal {
    uint32_t i, length, phase, seed1, idx;
    f3 f; float ucw;
    Surface cur;
    f3 prev;
};
// Either the next RegeneratePath BSDF ray or the light segment's Visibility ray.
// Called by every lane of the wave; `emit` selects the lanes with a ray.
__device__ __forceinline__ void wfinal_emit(const Scene &sc, const Seg &g, bool emit, WFinal &s, const uint4 *resv) {
    float4 *rays = g.rays, *res = g.res_out;
    const uint32_t idx = g.rbase + wave_alloc(g.l_ray, emit ? 1u : 0u);
    if (!emit) return;
    const f3 V = normalize(s.prev - s.cur.pos);
    s.idx = idx;
    if (s.i + 1u < s.length) {  // RegeneratePath step i (PT_4:1367-1381), seed rSeed[i-1]
        uint32_t seed = s.i == 1u ? resv[0].x : s.seed1;
        uint32_t lobe;
        const f3 dir = sample_bsdf(seed, s.cur, V, lobe);
        s.phase = 0u;
        put_ray(rays, idx, s.cur.pos, dir, -1.0f, Q_CLOSEST);
    } else {  // PathContribution's light segment (PT_4:1323-1333)
        const LightSample XL = load_xl(resv);
        const f3 L = direction_to_light(s.cur, XL);
        s.f = s.f * (bsdf(s.cur, L, V) * fabsf(dot(s.cur.nrm, L)));
        const f3 Le = l_emit<true>(XL, s.cur);
        s.phase = 1u;
        const float dist = length(XL.pos - s.cur.pos);
        put_ray(rays, idx, s.cur.pos, (XL.pos - s.cur.pos) / dist, dist, Q_VIS);
        res[2u * idx] = make_float4(0.0f, Le.x, Le.y, Le.z);
    }
}
__device__ __forceinline__ void wfinal_store(float4 *state, uint32_t npix, uint32_t pix, const WFinal &s,
                                             uint32_t matref) {
    state[FS_HDR * npix + pix] = make_float4(asf(s.i | (s.length << 8) | (s.phase << 16)), asf(s.seed1),
                                             asf(s.idx), 0.0f);
    state[FS_F * npix + pix] = make_float4(s.f.x, s.f.y, s.f.z, s.ucw);
    if (s.phase != 0u) return;  // waiting for the light segment: nothing else is read
    state[FS_CUR * npix + pix] = make_float4(s.cur.pos.x, s.cur.pos.y, s.cur.pos.z, asf(matref));
    state[FS_NRM * npix + pix] = make_float4(s.cur.nrm.x, s.cur.nrm.y, s.cur.nrm.z, 0.0f);
    state[FS_PREV * npix + pix] = make_float4(s.prev.x, s.prev.y, s.prev.z, 0.0f);
}

__global__ __launch_bounds__(WB) __attribute__((amdgpu_waves_per_eu(LOGIC_WAVES, 8))) void wfinal_start(Scene sc, WaveBufs w, const uint4 *gbuf, const uint4 *reservoir,
                                                   float4 *accum) {
    PTX_WAVE_TIMER(sc, KID_FINAL_START | (w.seg_base ? 0x80u : 0u));
    __shared__ uint32_t lds[3];
    const JobLists JL = job_lists(w, lds);
    const Seg g = seg_begin(w, 0u, lds);
    float4 *state = w.state;
    const uint32_t npix = w.npix, np = padded_pixels(sc);
    for (uint32_t k = 0; k < w.seg_px; k += WB) {
        const uint32_t q = seg_pixel(w, g.j, k);
        uint32_t x, y, pix = 0u, matref = 0u;
        bool active = false;
        WFinal s;
        if (q < np && tile_xy(sc, q, x, y)) {
            pix = (y - sc.row_begin) * sc.width + x;
            const Compact x1 = gdecode(gbuf[pix]);
            const uint4 *rv = reservoir + 8u * (size_t)pix;
            if (!x1.valid) {
                accum[pix] = make_float4(ENV_C, ENV_C, ENV_C, 1.0f);
            } else {
                const uint4 r0 = rv[0], r5 = rv[5], r7 = rv[7];
                s.length = r5.w;
                if (r7.y == 0u || s.length < 2u) {
                    mix_color(sc, accum, pix, mk(0.0f, 0.0f, 0.0f));
                } else if (r7.w == 1u) {
                    // a reused reservoir carrying its sample's PathContribution at this pixel
                    // (words 26, 27, 30; ptx_reuse.hip write_reused): PT_4's f without the replay
                    const uint4 r6 = rv[6];
                    mix_color(sc, accum, pix, mk(asf(r6.z), asf(r6.w), asf(r7.z)) * asf(r7.x));
                } else {
                    active = true;
                    s.seed1 = r0.y;
                    s.ucw = asf(r7.x);
                    s.prev = x0_of(sc, x, y);
                    s.cur = get_surface(sc, x1);
                    matref = mat_index(sc, x1.inst, x1.mat);
                    s.f = mk(1.0f, 1.0f, 1.0f);
                    s.i = 1u;
                }
            }
        }
        wfinal_emit(sc, g, active, s, reservoir + 8u * (size_t)pix);
        if (active) wfinal_store(state, npix, pix, s, matref);
        job_keep(g, JL, active, active && s.phase != 0u, pix);  // light: a Visibility result
    }
    job_seg_end(w, g, JL);
}

__global__ __launch_bounds__(WB) __attribute__((amdgpu_waves_per_eu(LOGIC_WAVES, 8))) void wfinal_step(Scene sc, WaveBufs w, uint32_t round, const uint4 *reservoir,
                                                  float4 *accum) {
    PTX_WAVE_TIMER(sc, KID_FINAL_STEP | (w.seg_base ? 0x80u : 0u));
    __shared__ uint32_t lds[3];
    const JobLists JL = job_lists(w, lds);
    const Seg g = seg_begin(w, round, lds);
    float4 *state = w.state;
    const float4 *res_in = g.res_in;
    const uint32_t npix = w.npix;
    uint32_t nh;
    const uint32_t n = split_count(g, nh);
    for (uint32_t base = 0; base < n; base += WB) {
        const uint32_t q = base + threadIdx.x;
        bool emit = false;
        uint32_t pix = 0u, matref = 0u;
        WFinal s;
        if (q < n) {
            pix = split_at(g, JL, q, nh);
            const float4 hd = state[FS_HDR * npix + pix], fv = state[FS_F * npix + pix];
            const uint32_t hw = asu(hd.x);
            s.i = hw & 0xffu; s.length = (hw >> 8) & 0xffu; s.phase = hw >> 16;
            s.seed1 = asu(hd.y); s.idx = asu(hd.z);
            s.f = mk(fv.x, fv.y, fv.z); s.ucw = fv.w;
            if (s.phase == 0u) {  // (the light-segment phase needs only HDR and F)
                const float4 cu = state[FS_CUR * npix + pix], nr = state[FS_NRM * npix + pix];
                const float4 pv = state[FS_PREV * npix + pix];
                s.prev = mk(pv.x, pv.y, pv.z);
                matref = asu(cu.w);
                s.cur.pos = mk(cu.x, cu.y, cu.z);
                s.cur.nrm = mk(nr.x, nr.y, nr.z);
                s.cur.mat = material_at(sc, matref);
            }
            if (s.phase == 0u) {  // regenerated vertex i+1 (PT_4:1378-1380) and f over vertex i
                const Hit h = get_hit(res_in, s.idx);
                const Surface next = h.valid ? surface_at(sc, h.s, h.pos) : get_surface(sc, h.s);
                const f3 V = normalize(s.prev - s.cur.pos);
                const f3 L = normalize(next.pos - s.cur.pos);
                s.f = s.f * (bsdf(s.cur, L, V) * fabsf(dot(s.cur.nrm, L)));
                s.prev = s.cur.pos;
                s.cur = next;
                matref = mat_index(sc, h.s.inst, h.s.mat);
                s.i += 1u;
                emit = true;
            } else {  // light segment's Visibility arrived (PT_4:1332)
                const float4 a = res_in[2u * s.idx];
                s.f = s.f * (mk(a.y, a.z, a.w) * a.x);
                mix_color(sc, accum, pix, s.f * s.ucw);
            }
        }
        wfinal_emit(sc, g, emit, s, reservoir + 8u * (size_t)pix);
        if (emit) wfinal_store(state, npix, pix, s, matref);
        job_keep(g, JL, emit, emit && s.phase != 0u, pix);
    }
    job_seg_end(w, g, JL);
}

// PT_4 of the reuse pipeline as ONE launch.  Its pixels almost all carry their sample's stored
// contribution (the spatial combine's), so wfinal_start shades them and the three {trace, step}
// rounds after it replay next to nothing -- six dependent launches of ~10 us dispatch gap each on
// the frame's critical path.  Here the replays run inline: each wave's live pixels emit their
// ray into their own queue slot, the whole wave walks it (trace_batch, every lane, the
// traversal kernel's code), and the step consumes it -- the same rays, results and arithmetic as
// wfinal_emit / trace_queue / wfinal_step, so the frame is bit-identical.
template <bool FLAT>
__global__ __launch_bounds__(WB) __attribute__((amdgpu_waves_per_eu(2, 8)))
void wfinal_one(Scene sc, WaveBufs w, const uint4 *gbuf, const uint4 *reservoir, float4 *accum, PassEps eps) {
    PTX_WAVE_TIMER(sc, KID_FINAL_START | (w.seg_base ? 0x80u : 0u));
    extern __shared__ __attribute__((aligned(16))) uint32_t wstack[];
    __shared__ unsigned long long c_key[WB];
    __shared__ uint32_t c_mark[WB];
    const LdsTables T = stage_tables(sc, wstack);
    uint32_t *stack = wstack + tables_lds_bytes(sc) / 4u + threadIdx.x;
    const CoopLds coop{c_key + (threadIdx.x & ~63u), c_mark + (threadIdx.x & ~63u)};
    const uint32_t j = w.seg_base + blockIdx.x, pj = w.seg_phys + j, np = padded_pixels(sc);
    // this thread's queue slot (the segment's first WB ray / result slots)
    float4 *rays = w.rays + 2u * (size_t)pj * w.ray_stride, *res = w.res[0] + 2u * (size_t)pj * w.ray_stride;
    const uint32_t slot = threadIdx.x;
    for (uint32_t k = 0; k < w.seg_px; k += WB) {  // (workgroup-uniform)
        const uint32_t q = seg_pixel(w, j, k);
        uint32_t x, y, pix = 0u;
        bool active = false;
        WFinal s;
        if (q < np && tile_xy(sc, q, x, y)) {  // wfinal_start's cases
            pix = (y - sc.row_begin) * sc.width + x;
            const Compact x1 = gdecode(gbuf[pix]);
            const uint4 *rv = reservoir + 8u * (size_t)pix;
            if (!x1.valid) {
                accum[pix] = make_float4(ENV_C, ENV_C, ENV_C, 1.0f);
            } else {
                const uint4 r0 = rv[0], r5 = rv[5], r7 = rv[7];
                s.length = r5.w;
                if (r7.y == 0u || s.length < 2u) {
                    mix_color(sc, accum, pix, mk(0.0f, 0.0f, 0.0f));
                } else if (r7.w == 1u) {
                    const uint4 r6 = rv[6];
                    mix_color(sc, accum, pix, mk(asf(r6.z), asf(r6.w), asf(r7.z)) * asf(r7.x));
                } else {
                    active = true;
                    s.seed1 = r0.y;
                    s.ucw = asf(r7.x);
                    s.prev = x0_of(sc, x, y);
                    s.cur = get_surface(sc, x1);
                    s.f = mk(1.0f, 1.0f, 1.0f);
                    s.i = 1u;
                }
            }
        }
        const uint4 *resv = reservoir + 8u * (size_t)pix;
        // (wave-uniform) one replayed vertex per iteration, as many as the queued form's trace
        // rounds: a path needing more is dropped there, so it is here
        for (uint32_t it = 0u; it < (uint32_t)kWaveRoundsFinal; ++it) {
            if (wballot(active) == 0ull) break;
            if (active) {  // wfinal_emit, into this thread's slot
                const f3 V = normalize(s.prev - s.cur.pos);
                if (s.i + 1u < s.length) {
                    uint32_t seed = s.i == 1u ? resv[0].x : s.seed1;
                    uint32_t lobe;
                    const f3 dir = sample_bsdf(seed, s.cur, V, lobe);
                    s.phase = 0u;
                    put_ray(rays, slot, s.cur.pos, dir, -1.0f, Q_CLOSEST);
                } else {
                    const LightSample XL = load_xl(resv);
                    const f3 L = direction_to_light(s.cur, XL);
                    s.f = s.f * (bsdf(s.cur, L, V) * fabsf(dot(s.cur.nrm, L)));
                    const f3 Le = l_emit<true>(XL, s.cur);
                    s.phase = 1u;
                    const float dist = length(XL.pos - s.cur.pos);
                    put_ray(rays, slot, s.cur.pos, (XL.pos - s.cur.pos) / dist, dist, Q_VIS);
                    res[2u * slot] = make_float4(0.0f, Le.x, Le.y, Le.z);
                }
            }
            // the traversal kernel's walk, every lane of the wave (idle ones with a NaN bound)
            trace_batch<false, false, false, true, FLAT>(sc, T.subs, T.insts, eps, stack, coop, res, rays, 0u, slot, active);
            if (active) {  // wfinal_step
                if (s.phase == 0u) {
                    const Hit h = get_hit(res, slot);
                    const Surface next = h.valid ? surface_at(sc, h.s, h.pos) : get_surface(sc, h.s);
                    const f3 V = normalize(s.prev - s.cur.pos);
                    const f3 L = normalize(next.pos - s.cur.pos);
                    s.f = s.f * (bsdf(s.cur, L, V) * fabsf(dot(s.cur.nrm, L)));
                    s.prev = s.cur.pos;
                    s.cur = next;
                    s.i += 1u;
                } else {
                    const float4 a = res[2u * slot];
                    s.f = s.f * (mk(a.y, a.z, a.w) * a.x);
                    mix_color(sc, accum, pix, s.f * s.ucw);
                    active = false;
                }
            }
        }
    }
}

// =========================================================================== TEST_MCPT
enum : uint32_t { MS_HDR, MS_COL, MS_FP, MS_ORG, MS_COUNT };
// HDR: {seed, bounce | flags<<8, light-ray base idx, path ray idx}; COL: {color, -};
// FP: {f, p}; ORG: {path ray origin (for V), -}.  flags: 1 = path ray pending
struct WMcpt {
    uint32_t seed, bounce, flags, lbase, pidx;
    f3 color, f;
    float p;
    f3 org;
};
__device__ __forceinline__ void wmcpt_store(float4 *state, uint32_t npix, uint32_t pix, const WMcpt &s) {
    state[MS_HDR * npix + pix] = make_float4(asf(s.seed), asf(s.bounce | (s.flags << 8)), asf(s.lbase), asf(s.pidx));
    state[MS_COL * npix + pix] = make_float4(s.color.x, s.color.y, s.color.z, 0.0f);
    state[MS_FP * npix + pix] = make_float4(s.f.x, s.f.y, s.f.z, s.p);
    state[MS_ORG * npix + pix] = make_float4(s.org.x, s.org.y, s.org.z, 0.0f);
}
// GetLightColor of light `id` up to its Visibility (TEST_MCPT:1261-1308); the shadow ray
// goes to queue slot `idx`, the light term {c, pdf, f/p} into that slot's result record.
__device__ __forceinline__ void mcpt_light_ray(const Scene &sc, uint32_t &seed, const Surface &X, f3 V, f3 fp,
                                               uint32_t id, uint32_t idx, float4 *rays, float4 *res) {
    const Light ls = get_light(sc, id);
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
        const float ru = rnd(seed) * 2.0f - 1.0f;
        const float rv = rnd(seed) * 2.0f - 1.0f;
        XL.pos = ls.pos + (ls.U * ru + ls.V * rv);
        XL.dir = normalize(X.pos - XL.pos);
        const f3 rr = XL.pos - X.pos;
        const f3 Ld = normalize(rr);
        XL.pdf = dot(rr, rr) / fmaxf(ls.area * fabsf(dot(ls.dir, Ld)), EPS_F);
    }
    const f3 L = direction_to_light(X, XL);
    f3 c = l_emit<false>(XL, X) * bsdf(X, V, L);
    c = c * fabsf(dot(X.nrm, L));
    const float dist = length(XL.pos - X.pos);
    put_ray(rays, idx, X.pos, (XL.pos - X.pos) / dist, dist, Q_VIS);
    res[2u * idx] = make_float4(0.0f, c.x, c.y, c.z);
    res[2u * idx + 1u] = make_float4(XL.pdf, fp.x, fp.y, fp.z);
}

// At a path vertex: every light's GetLightColor up to its Visibility (TEST_MCPT:1261-1308),
// then the BSDF sample + Russian roulette (:1356-1366).  Light terms ride in their shadow
// rays' result slots: {T, c.xyz | pdf, (f/p).xyz}.  Called by every lane of the wave;
// `emit` selects the lanes with a vertex.
__device__ __forceinline__ void wmcpt_vertex(const Scene &sc, const Seg &g, bool emit, WMcpt &s, const Surface &X) {
    float4 *rays = g.rays, *res = g.res_out;
    const uint32_t nl = sc.U[U_LIGHT_COUNT];
    const uint32_t lbase = g.rbase + wave_alloc(g.l_ray, emit ? nl : 0u);
    bool path_ray = false;
    f3 Lb = mk(0.0f, 0.0f, 0.0f);
    if (emit) {
        const f3 V = normalize(s.org - X.pos);
        const f3 fp = s.f / s.p;
        for (uint32_t id = 0; id < nl; ++id) mcpt_light_ray(sc, s.seed, X, V, fp, id, lbase + id, rays, res);
        s.lbase = lbase;
        uint32_t lobe;
        Lb = sample_bsdf(s.seed, X, V, lobe);
        float pdfv;
        const f3 bv = bsdf_pdf(X, V, Lb, pdfv);
        s.f = s.f * (bv * fabsf(dot(X.nrm, Lb)));
        s.p *= pdfv;
        s.org = X.pos;
        const float ps = luminance(s.f) / s.p;
        if (rnd(s.seed) < ps) {
            s.p *= ps;
            s.bounce += 1u;
            path_ray = s.bounce < 3u;
        }
        s.flags = path_ray ? 1u : 0u;
    }
    const uint32_t pidx = g.rbase + wave_alloc(g.l_ray, path_ray ? 1u : 0u);
    if (path_ray) {
        s.pidx = pidx;
        put_ray(rays, pidx, s.org, Lb, -1.0f, Q_CLOSEST);
    }
}

// a finished path's colour: WriteColor into the accumulation, or (a pipelined frame, `color`
// set) kept per pixel for wmix_frame, which mixes it in after the previous frame's
__device__ __forceinline__ void mcpt_out(const Scene &sc, float4 *accum, float4 *color, uint32_t pix, f3 c) {
    if (color) color[pix] = make_float4(c.x, c.y, c.z, 1.0f);
    else mix_color(sc, accum, pix, c);
}
__global__ __launch_bounds__(WB) void wmcpt_start(Scene sc, WaveBufs w) {
    __shared__ uint32_t lds[2];
    const Seg g = seg_begin(w, 0u, lds);
    float4 *state = w.state, *rays = g.rays;
    const uint32_t npix = w.npix, np = padded_pixels(sc);
    for (uint32_t k = 0; k < w.seg_px; k += WB) {
        const uint32_t q = seg_pixel(w, g.j, k);
        uint32_t x, y, pix = 0u;
        const bool active = q < np && tile_xy(sc, q, x, y);
        WMcpt s;
        const uint32_t idx = g.rbase + wave_alloc(g.l_ray, active ? 1u : 0u);
        if (active) {
            pix = (y - sc.row_begin) * sc.width + x;
            s.seed = pcg(x * 1973u + y * 9277u + sc.U[U_FRAME] * 26699u);
            const float *vpinv = reinterpret_cast<const float *>(sc.U + U_VPINV);  // PT_01:496-507
            const float u = ((float)x + 0.5f) / (float)sc.U[U_W];
            const float v = ((float)y + 0.5f) / (float)sc.U[U_H];
            const f3 st = xform_point(vpinv, mk(2.0f * u - 1.0f, 2.0f * v - 1.0f, 0.0f));
            const f3 en = xform_point(vpinv, mk(2.0f * u - 1.0f, 2.0f * v - 1.0f, 0.0f + 1.0f));
            s.org = st;
            s.bounce = 0u; s.flags = 1u; s.lbase = 0u; s.pidx = idx;
            s.color = mk(0.0f, 0.0f, 0.0f); s.f = mk(1.0f, 1.0f, 1.0f); s.p = 1.0f;
            put_ray(rays, idx, st, normalize(en - st), -1.0f, Q_CLOSEST);
            wmcpt_store(state, npix, pix, s);
        }
        seg_keep(g, active, pix);
    }
    seg_end(w, g);
}

template <int FIRST>
__global__ __launch_bounds__(WB) __attribute__((amdgpu_waves_per_eu(LOGIC_WAVES, 8))) void wmcpt_step(Scene sc, WaveBufs w, uint32_t round, float4 *accum, float4 *color) {
    __shared__ uint32_t lds[3];
    const JobLists JL = job_lists(w, lds);
    const Seg g = seg_begin(w, round, lds);
    float4 *state = w.state;
    const float4 *res_in = g.res_in;
    const uint32_t npix = w.npix;
    uint32_t nh;  // (wmcpt_start's plain count reads as all-heavy)
    const uint32_t n = split_count(g, nh);
    const uint32_t nl = sc.U[U_LIGHT_COUNT];
    for (uint32_t base = 0; base < n; base += WB) {
        const uint32_t q = base + threadIdx.x;
        bool emit = false;
        uint32_t pix = 0u;
        WMcpt s;
        Surface X;
        if (q < n) {
            pix = split_at(g, JL, q, nh);
            const float4 hd = state[MS_HDR * npix + pix], co = state[MS_COL * npix + pix];
            const float4 fp = state[MS_FP * npix + pix], og = state[MS_ORG * npix + pix];
            s.seed = asu(hd.x); s.bounce = asu(hd.y) & 0xffu; s.flags = asu(hd.y) >> 8;
            s.lbase = asu(hd.z); s.pidx = asu(hd.w);
            s.color = mk(co.x, co.y, co.z); s.f = mk(fp.x, fp.y, fp.z); s.p = fp.w;
            s.org = mk(og.x, og.y, og.z);
            // 1. light terms of the previous vertex, in light order (TEST_MCPT:1351-1354)
            if (!FIRST) {
                for (uint32_t id = 0; id < nl; ++id) {
                    const float4 a = res_in[2u * (s.lbase + id)], b = res_in[2u * (s.lbase + id) + 1u];
                    const f3 term = (mk(a.y, a.z, a.w) * a.x) / b.x;
                    s.color = s.color + mk(b.y, b.z, b.w) * term;
                }
            }
            if (!(s.flags & 1u)) {
                mcpt_out(sc, accum, color, pix, s.color);  // RR ended the path or 3 bounces done
            } else {
                const Hit h = get_hit(res_in, s.pidx);
                if (!h.valid) {  // escaped: environment (TEST_MCPT:1340-1344)
                    s.color = s.color + (s.f / s.p) * ENV_C;
                    mcpt_out(sc, accum, color, pix, s.color);
                } else {
                    X = surface_at(sc, h.s, h.pos);
                    emit = true;
                }
            }
        }
        wmcpt_vertex(sc, g, emit, s, X);
        if (emit) wmcpt_store(state, npix, pix, s);
        // light next round: the shadow rays' terms to add and the path to end (no BSDF ray)
        job_keep(g, JL, emit, emit && !(s.flags & 1u), pix);
    }
    job_seg_end(w, g, JL);
}

// =========================================================================== host side
// trace_queue's grid: trace_split workgroups per segment
static inline bool trace_dyn(const WaveBufs &w) { return kAbBuild && w.dyn != nullptr && w.seg_count <= kDynMaxSlots; }
static inline uint32_t trace_grid(const WaveBufs &w) {
    // (PTX_AB=DYN_GROUPS=n: A/B -- the cap dates from the 4-wave trace; at 5 waves per SIMD the chip
    // holds 1280 trace workgroups)
    static const uint32_t groups = (uint32_t)ab_knob("DYN_GROUPS", (int)kDynMaxGroups);
    return trace_dyn(w) ? std::min(w.seg_count, groups) : w.seg_count * w.trace_split;
}

hipError_t wave_trace(const Scene &sc, const WaveBufs &w_in, int round, int eps_mode, uint32_t depth, hipStream_t s,
                      bool occ_only) {
    const PassEps eps = eps_mode == 0 ? PassEps{1e-8f, 1e-6f} : PassEps{1e-4f, 1e-8f};
    WaveBufs w = w_in;
    // counting builds keep the per-slot census (the SIMD-utilisation build profiles the production
    // walk, streamed lanes included, when it applies)
    static const bool prof = ab_knob("TRACE_PROF", 0) != 0;
    const bool prof_stream = PTX_TRACE_STREAM && prof && !occ_only && tables_fit_lds(sc) && PTX_FLAT_INST &&
                             sc.n_inst >= (uint32_t)ab_knob("FLAT_MIN_INST", (int)kFlatMinInstances);
    if ((sc.counters && !prof_stream) || !trace_dyn(w)) w.dyn = nullptr;
    if (w.dyn) {  // batches per dequeue (A/B: PTX_AB=TRACE_DYN_G=g)
        static const uint32_t g = (uint32_t)ab_knob("TRACE_DYN_G", 0);
        w.trace_split = g >= 1u && g <= 16u ? g : 1u;
    }
    // dynamic LDS: scene tables (the LDS-table variants) + batch prefix (dynamic batches) + stacks
    const size_t lds = (tables_fit_lds(sc) ? tables_lds_bytes(sc) : 0u) +
                       (w.dyn ? 4u * (size_t)((w.seg_count + 4u) & ~3u) : 0u) + stack_lds_bytes(depth);
    static const uint32_t flat_min = (uint32_t)ab_knob("FLAT_MIN_INST", (int)kFlatMinInstances);  // A/B
    const bool flat = PTX_FLAT_INST && sc.n_inst >= flat_min;
    if (occ_only && tables_fit_lds(sc)) {  // occlusion rounds (GI spatial)
        if (sc.counters)
            hipLaunchKernelGGL((trace_queue<true, 6, false, true, true>), dim3(trace_grid(w)), dim3(WB), lds, s, sc, w,
                               (uint32_t)round, eps);
        else if (flat)
            hipLaunchKernelGGL((trace_queue<false, TRACE_OCC_WAVES, false, true, true, true>), dim3(trace_grid(w)), dim3(WB), lds,
                               s, sc, w, (uint32_t)round, eps);
        else
            hipLaunchKernelGGL((trace_queue<false, TRACE_OCC_WAVES, false, true, true>), dim3(trace_grid(w)), dim3(WB), lds, s, sc, w,
                               (uint32_t)round, eps);
        return hipGetLastError();
    }
    // (PTX_AB=TRACE_REFILL: the lane-refill kernel of ptx_trace on the queues -- A/B builds)
    static const bool refill = ab_knob("TRACE_REFILL", 0) != 0;
    if (refill) {
        const uint32_t pb = w.seg_phys + w.seg_base;
        const uint32_t *cnt = w.cnt + (2u * round + 1u) * w.cnt_stride + pb;
        float4 *res = w.res[w.nres == 3u ? round % 3 : round & 1] + 2u * (size_t)pb * w.ray_stride;
        if (sc.counters)
            hipLaunchKernelGGL(trace_queue_sm<true>, dim3(w.seg_count), dim3(WB), lds, s, sc,
                               w.rays + 2u * (size_t)pb * w.ray_stride, res, cnt,
                               w.ray_stride, 0u, eps);
        else
            hipLaunchKernelGGL(trace_queue_sm<false>, dim3(w.seg_count), dim3(WB), lds, s, sc,
                               w.rays + 2u * (size_t)pb * w.ray_stride, res, cnt,
                               w.ray_stride, 0u, eps);
    } else if (sc.counters && ab_knob("TRACE_PROF", 0)) {  // SIMD-utilisation diagnostics
        if (flat && tables_fit_lds(sc))  // (the production walk: flattened instances, LDS tables, and
            // COUNT off so that the instance cull applies as in production -- the PROF regions
            // still count into sc.counters; the work counters stay zero)
            hipLaunchKernelGGL((trace_queue<false, 6, true, true, false, true>), dim3(trace_grid(w)), dim3(WB), lds, s, sc, w,
                               (uint32_t)round, eps);
        else
            hipLaunchKernelGGL((trace_queue<true, 6, true, false>), dim3(trace_grid(w)), dim3(WB), lds, s, sc, w,
                               (uint32_t)round, eps);
    }
    else if (sc.counters)
        hipLaunchKernelGGL((trace_queue<true, 6, false, false>), dim3(trace_grid(w)), dim3(WB), lds, s, sc, w, (uint32_t)round, eps);
    else {
        // Occupancy target per pipeline (WaveBufs::trace_waves), LDS-staged tables; A/B
        // switches PTX_AB=TRACE_OCC=n / TRACE_NOLDS.  Measured at 1080p with 768-pixel segments:
        // 4 waves/SIMD (no spill) is fastest for the per-instance walk (with the flat node loop:
        // reuse 369-373 vs 339-340, ReSTIR 1301 vs 1235, TEST_MCPT 1359 vs 1261 at 5); 5 for
        // bands above 4 Mpx; 6+ spills in the node loop.  The flattened walk (>= 3 instances)
        // runs at 5 (96 VGPRs; its 40 B/lane of spills sit at the batch boundaries, none in the
        // walk): reuse 462.6 vs 446.6, GI 769.6 vs 757.7, furnished C3 301.6 vs 282.2 (same box,
        // round 3) -- the launch alone is ~3 % slower, the pipelined frame faster: 96-VGPR
        // waves leave the other frame's logic waves room on the SIMD.
        static const int env_occ = ab_knob("TRACE_OCC", 0);
        const int occ = env_occ ? env_occ : (w.trace_waves == 4u && !flat) ? 4 : 5;
        static const bool no_lds = ab_knob("TRACE_NOLDS", 0) != 0;
        const bool tables_fit = tables_fit_lds(sc) && !no_lds;
        auto k = !tables_fit ? trace_queue<false, 5, false, false>
#ifdef PTX_AB_BUILD
                 : occ >= 8  ? trace_queue<false, 8>
                 : occ == 7  ? (flat ? trace_queue<false, 7, false, true, false, true> : trace_queue<false, 7>)
                 : occ == 6  ? (flat ? trace_queue<false, 6, false, true, false, true> : trace_queue<false, 6>)
#endif
                 : occ == 5  ? (flat ? trace_queue<false, 5, false, true, false, true> : trace_queue<false, 5>)
                             : (flat ? trace_queue<false, 4, false, true, false, true> : trace_queue<false, 4>);
        hipLaunchKernelGGL(k, dim3(trace_grid(w)), dim3(WB), lds, s, sc, w, (uint32_t)round, eps);
    }
    return hipGetLastError();
}

// ptx_trace / ptx_trace_device queries (public ray layout) through the same kernel.
hipError_t launch_trace_rays_sm(const Scene &sc, const float4 *rays, float4 *hits, uint32_t n, int eps_mode,
                                uint32_t depth, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const PassEps eps = eps_mode == 0 ? PassEps{1e-8f, 1e-6f} : PassEps{1e-4f, 1e-8f};
    const uint32_t per_wg = 4u * WB;
    const dim3 grid((n + per_wg - 1u) / per_wg);
    if (sc.counters)
        hipLaunchKernelGGL(trace_queue_sm<true>, grid, dim3(WB), stack_lds_bytes(depth), s, sc, rays, hits, nullptr,
                           per_wg, n, eps);
    else
        hipLaunchKernelGGL(trace_queue_sm<false>, grid, dim3(WB), stack_lds_bytes(depth), s, sc, rays, hits, nullptr,
                           per_wg, n, eps);
    return hipGetLastError();
}

hipError_t wave_gbuffer(const Scene &sc, const WaveBufs &w, uint4 *gbuf, uint32_t depth, hipStream_t s) {
    if (!tables_fit_lds(sc)) return hipErrorInvalidValue;  // caller falls back to gbuffer_kernel
    static const bool rootq = ab_knob("GBUF_ROOTQ", 0) != 0;  // A/B
    if (rootq)
        hipLaunchKernelGGL(wgbuffer<true>, dim3(w.seg_px / WB * w.seg_count), dim3(WB),
                           tables_lds_bytes(sc) + stack_lds_bytes(depth), s, sc,
                           w, gbuf);
    else
        hipLaunchKernelGGL(wgbuffer<false>, dim3(w.seg_px / WB * w.seg_count), dim3(WB),
                           tables_lds_bytes(sc) + stack_lds_bytes(depth), s,
                           sc, w, gbuf);
    return hipGetLastError();
}

// Logic round r consumes the results of trace round r-1 and emits the rays of trace round r.
hipError_t wave_init_round(const Scene &sc, const WaveBufs &w, int round, const uint4 *gbuf, uint4 *reservoir,
                           hipStream_t s) {
    if (round == 0)
        hipLaunchKernelGGL(winit_start, dim3(w.seg_count), dim3(WB), 0, s, sc, w, gbuf, reservoir);
    else
        hipLaunchKernelGGL(winit_step, dim3(w.seg_count), dim3(WB), 0, s, sc, w, (uint32_t)round, reservoir);
    return hipGetLastError();
}

hipError_t wave_final_round(const Scene &sc, const WaveBufs &w, int round, const uint4 *gbuf, const uint4 *reservoir,
                            float4 *accum, hipStream_t s) {
    if (round == 0)
        hipLaunchKernelGGL(wfinal_start, dim3(w.seg_count), dim3(WB), 0, s, sc, w, gbuf, reservoir, accum);
    else
        hipLaunchKernelGGL(wfinal_step, dim3(w.seg_count), dim3(WB), 0, s, sc, w, (uint32_t)round, reservoir, accum);
    return hipGetLastError();
}

hipError_t wave_final_one(const Scene &sc, const WaveBufs &w, const uint4 *gbuf, const uint4 *reservoir, float4 *accum,
                          uint32_t depth, hipStream_t s) {
    const PassEps eps{1e-4f, 1e-8f};  // (wave_trace's eps_mode 1, every wavefront pass)
    const size_t lds = tables_lds_bytes(sc) + stack_lds_bytes(depth);
    static const uint32_t flat_min = (uint32_t)ab_knob("FLAT_MIN_INST", (int)kFlatMinInstances);
    if (PTX_FLAT_INST && sc.n_inst >= flat_min)
        hipLaunchKernelGGL(wfinal_one<true>, dim3(w.seg_count), dim3(WB), lds, s, sc, w, gbuf, reservoir, accum, eps);
    else
        hipLaunchKernelGGL(wfinal_one<false>, dim3(w.seg_count), dim3(WB), lds, s, sc, w, gbuf, reservoir, accum, eps);
    return hipGetLastError();
}

hipError_t wave_mcpt_round(const Scene &sc, const WaveBufs &w, int round, float4 *accum, float4 *color,
                           hipStream_t s) {
    if (round == 0)
        hipLaunchKernelGGL(wmcpt_start, dim3(w.seg_count), dim3(WB), 0, s, sc, w);
    else if (round == 1)
        hipLaunchKernelGGL(wmcpt_step<1>, dim3(w.seg_count), dim3(WB), 0, s, sc, w, (uint32_t)round, accum, color);
    else
        hipLaunchKernelGGL(wmcpt_step<0>, dim3(w.seg_count), dim3(WB), 0, s, sc, w, (uint32_t)round, accum, color);
    return hipGetLastError();
}

// A pipelined TEST_MCPT frame's WriteColor, after the previous frame's: each band pixel's path
// colour (wmcpt_step wrote it to `color`) mixed into the accumulation, the same mix_color
__global__ __launch_bounds__(WB) void wmix_frame(Scene sc, const float4 *color, float4 *accum, uint32_t npx) {
    const uint32_t i = blockIdx.x * WB + threadIdx.x;
    if (i >= npx) return;
    const float4 c = color[i];
    mix_color(sc, accum, i, mk(c.x, c.y, c.z));
}
hipError_t wave_mix_frame(const Scene &sc, const float4 *color, float4 *accum, hipStream_t s) {
    const uint32_t npx = (sc.row_end - sc.row_begin) * sc.width;
    if (npx == 0u) return hipSuccess;
    hipLaunchKernelGGL(wmix_frame, dim3((npx + WB - 1u) / WB), dim3(WB), 0, s, sc, color, accum, npx);
    return hipGetLastError();
}

}  // namespace ptx
