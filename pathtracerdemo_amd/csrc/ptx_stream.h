// ptx_stream.h -- the streamed-lanes trace walk (trace_stream) of the trace kernel (ptx_wave.hip:
// trace_queue), in a header of its own so that another kernel can walk a segment's queries the same
// way (round 6 built a fused spatial-rounds kernel on it: bit-exact, but 7 % slower -- DESIGN §9).
#pragma once
#include "ptx_wave_common.h"

#ifndef PTX_LDS_TRANS
#define PTX_LDS_TRANS 1  // the restart test's transmission from the LDS root table (A/B: 0 = Scene::mats)
#endif

namespace ptx {

// ---------------------------------------------------------------- streamed lanes
// The production walk (flattened instances, LDS tables, dynamic batches) with LANE REFILL: a
// lane whose query is over takes the next query of the wave's batch stream at once, instead of
// idling until the wave's slowest query of a fixed 64-query batch ends.  The walk is
// trace_core_flat's -- refill (instance + root pre-filter), node loop, cooperative leaf phase,
// the same early leaf phase -- and trace_lanes' Visibility continuation through transmissive
// hits; what a lane does for one query is exactly what it did there (same instance / root /
// pop / push / triangle order, same bound at every test), so every result is bit-identical.
// Only the interleaving across lanes changes: a straggler's node loop now runs beside other
// lanes' new queries.  Lanes whose query is over are finalised (result written, or the
// Visibility walk continued from the transmissive hit) and given new queries once at least
// kStreamRefill of them wait, or when no lane is still walking (the result write and the ray
// load then serve many lanes at once).  The stream (DYN): the launch's 64-query batches
// (WaveBufs::dyn chunk heads, as trace_queue), taken by the wave as its lanes need them; or
// (static slots) the workgroup's segment `sj` (`sn` queries), its 64-query batches taken by the
// workgroup's waves through an LDS counter.
#ifndef PTX_STREAM_REFILL
#define PTX_STREAM_REFILL 32
#endif
#ifndef PTX_TRACE_STREAM
#define PTX_TRACE_STREAM 1
#endif
template <bool PROF, bool OCC, bool DYN>
__device__ __forceinline__ void trace_stream(const Scene &sc, const SubRoot *subs, const Inst *insts, PassEps eps,
                                             uint32_t *stack, CoopLds coop, const WaveBufs &w, uint32_t round,
                                             const uint32_t *pref, uint32_t *heads, float4 *res_all,
                                             uint32_t *l_next = nullptr, uint32_t sj = 0u, uint32_t sn = 0u) {
    constexpr uint32_t stride = WB;
    const uint32_t lane = __lane_id();
    // ---- the batch stream (wave-uniform)
    const uint32_t total = DYN ? pref[w.seg_count] : 0u;
    uint32_t x = blockIdx.x % kDynHeads, visited = 0u;
    uint32_t c0 = (uint32_t)((uint64_t)total * x / kDynHeads), c1 = (uint32_t)((uint64_t)total * (x + 1u) / kDynHeads);
    uint32_t bnext = 0u;
    if (DYN && lane == 0u) bnext = atomicAdd(heads + x * kDynStride, 1u);
    bool src_done = false;
    uint32_t qbase = 0u, qleft = 0u;  // the current batch's untaken queries: ray slots qbase ..
    // ---- this lane's query
    bool has = false;
    uint32_t gi = 0u, kind = 0u, seg = 0u;
    float T = 1.0f, remain = 0.0f;
    Ray ray{mk(0.0f, 0.0f, 0.0f), mk(0.0f, 0.0f, 1.0f)};
    // ---- its walk (trace_core_flat's state)
    Prof pf{};
    const float vx = 1e-4f;
    float vy = 0.0f, vy_pf = 0.0f, omax = 0.0f;
    bool rfin = true, bvalid = false, done = true;
    uint32_t binst = 0u, bmat = 0u, bprim = 0u;
    uint32_t next = 0u, cur = 0u, s0 = 0u, nsub = 0u, sub_base = 0u, tri_base = 0u;
    f3 lo = mk(0.0f, 0.0f, 0.0f), ld = lo, inv = lo;
    uint32_t mask = 0u, grp = 0u, leaf = 0u;
    int sp = -1;
    uint32_t n_aabb = 0u, n_tri = 0u;
    auto begin_walk = [&]() {  // a query (or a Visibility continuation) from ray.o along ray.d
        vy = kind != Q_CLOSEST ? fminf(remain, 1e10f) : 1e10f;
        vy_pf = vy;
        rfin = finite3(ray.o) && finite3(ray.d);
        omax = fmaxf(fmaxf(fabsf(ray.o.x), fabsf(ray.o.y)), fabsf(ray.o.z));
        bvalid = false;
        binst = bmat = bprim = 0u;
        next = cur = s0 = nsub = sub_base = tri_base = 0u;
        mask = grp = leaf = 0u;
        sp = -1;
        done = false;
        n_aabb = n_tri = 0u;
    };
    for (;;) {  // wave-uniform
        // ---- finalise + take new queries, once enough lanes wait or none walks
        const unsigned long long walking = wballot(has && !done);
        const uint32_t waiting = (uint32_t)__popcll(wballot(!(has && !done)));
        if (walking == 0ull || (waiting >= PTX_STREAM_REFILL && !src_done)) {
            if (has && done) {
                if (PROF) {
                    atomicAdd(&sc.counters[CNT_RAYS], 1ull);
                    atomicAdd(&sc.counters[CNT_INST], (unsigned long long)sc.n_inst);
                    atomicAdd(&sc.counters[CNT_AABB], (unsigned long long)n_aabb);
                    atomicAdd(&sc.counters[CNT_TRI], (unsigned long long)n_tri);
                    if (bvalid) atomicAdd(&sc.counters[CNT_HITS], 1ull);
                }
                Hit h;
                h.valid = bvalid;
                h.t = bvalid ? vy : 0.0f;
                h.s = Compact{0u, binst, bmat, bprim, 0.0f, 0.0f};
                h.pos = mk(0.0f, 0.0f, 0.0f);
                if (kind == Q_CLOSEST) {
                    if (bvalid) complete_hit(sc, ray, eps, h, insts);
                    const uint32_t enc = ((h.valid ? 1u : 0u) << 31) | (h.s.inst << 16) | h.s.mat;
                    res_all[2u * gi] = make_float4(h.t, asf(enc), asf(h.s.prim), h.s.bu);
                    res_all[2u * gi + 1u] = make_float4(h.s.bv, h.pos.x, h.pos.y, h.pos.z);
                    has = false;
                } else {
                    float out = -1.0f;
                    if (!h.valid || h.t > remain) out = T;
                    else {
                        const float tr = kind == Q_OCC    ? 0.0f
                                         : PTX_LDS_TRANS ? subs_transmission(subs, insts, h.s.inst, h.s.mat)
                                                         : get_transmission(sc, h.s.inst, h.s.mat);
                        if (tr == 0.0f) out = 0.0f;
                        else {
                            T *= tr;
                            remain -= h.t;
                            complete_hit(sc, ray, eps, h, insts);
                            ray.o = h.pos;
                            if (seg == 4u) out = 0.0f;  // Visibility gives up after 5 segments
                            ++seg;
                        }
                    }
                    if (out >= 0.0f) {  // only res.x is written: .yzw and res[2i+1] carry the payload
                        res_all[2u * gi].x = out;
                        has = false;
                    } else {
                        begin_walk();  // the next segment of the same Visibility query
                    }
                }
            }
            // new queries for the free lanes, in lane order from the stream
            unsigned long long want = wballot(!has);
            while (want != 0ull && !src_done) {  // wave-uniform
                if (!DYN && qleft == 0u) {  // the workgroup's next batch of its segment
                    uint32_t b = 0u;
                    if (lane == 0u) b = __hip_atomic_fetch_add(l_next, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    b = (uint32_t)__builtin_amdgcn_readfirstlane((int)b);
                    if (b * 64u >= sn) {
                        src_done = true;
                        break;
                    }
                    qbase = sj * w.ray_stride + b * 64u;
                    qleft = min(64u, sn - b * 64u);
                }
                if (DYN && qleft == 0u) {
                    for (;;) {  // the next batch of this wave's chunk, or of the next chunk
                        const uint32_t bi = c0 + (uint32_t)__builtin_amdgcn_readfirstlane((int)bnext);
                        if (bi < c1) {
                            if (lane == 0u) bnext = atomicAdd(heads + x * kDynStride, 1u);  // fetched ahead
                            uint32_t lo_i = 0u, hi_i = w.seg_count;  // last slot with pref <= bi
                            while (hi_i - lo_i > 1u) {
                                const uint32_t mid = (lo_i + hi_i) >> 1;
                                if (pref[mid] <= bi) lo_i = mid;
                                else hi_i = mid;
                            }
                            const uint32_t j = w.seg_phys + w.seg_base + lo_i;
                            const uint32_t n = w.cnt[(2u * round + 1u) * w.cnt_stride + j];
                            const uint32_t i0 = (bi - pref[lo_i]) * 64u;
                            qbase = j * w.ray_stride + i0;
                            qleft = min(64u, n - i0);
                            break;
                        }
                        if (++visited == kDynHeads) {
                            src_done = true;
                            break;
                        }
                        x = (x + 1u) % kDynHeads;
                        c0 = (uint32_t)((uint64_t)total * x / kDynHeads);
                        c1 = (uint32_t)((uint64_t)total * (x + 1u) / kDynHeads);
                        if (lane == 0u) bnext = atomicAdd(heads + x * kDynStride, 1u);
                    }
                    if (src_done) break;
                }
                const uint32_t m = (uint32_t)__popcll(want), take = min(m, qleft);
                const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(want >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)want, 0u));
                if (!has && rank < take) {
                    gi = qbase + rank;
                    const float4 a = w.rays[2u * gi], b = w.rays[2u * gi + 1u];
                    ray = Ray{mk(a.x, a.y, a.z), mk(b.x, b.y, b.z)};
                    remain = a.w;
                    kind = asu(b.w);
                    T = 1.0f;
                    seg = 0u;
                    has = true;
                    begin_walk();
                }
                qbase += take;
                qleft -= take;
                want = wballot(!has);
            }
            if (wballot(has) == 0ull) break;  // the stream is drained and every query written
        }
        // ---- refill: a walking lane with no leaf, no stack and no queued root takes its
        // instance's next chunk of 32 roots or its next instance (trace_core_flat)
        for (;;) {
            const bool need = has && !done && leaf == 0u && sp < 0 && mask == 0u;
            if (wballot(need) == 0ull) break;
            if (need) {
                if (s0 + 32u < nsub) {
                    s0 += 32u;
                } else {
                    const f3 winv = mk(__builtin_amdgcn_rcpf(ray.d.x), __builtin_amdgcn_rcpf(ray.d.y),
                                       __builtin_amdgcn_rcpf(ray.d.z));
                    while (next < sc.n_inst) {
                        if (!PTX_INST_CULL || !rfin || inst_may_hit(insts[next], ray.o, winv, omax, vy)) break;
                        ++next;
                    }
                    if (next >= sc.n_inst) {
                        done = true;
                    } else {
                        cur = next++;
                        const Inst &I = insts[cur];
                        if (PROF) pf.hit(PROF_INST);
                        lo = xform_point(I.minv, ray.o);
                        const f3 le = xform_point(I.minv, ray.o + ray.d);
                        ld = le - lo;
                        inv = mk(1.0f / ld.x, 1.0f / ld.y, 1.0f / ld.z);
                        sub_base = I.sub_base;
                        nsub = I.nsub;
                        tri_base = I.tri_base;
                        s0 = 0u;
                        n_aabb += nsub;
                    }
                }
                if (!done && nsub != 0u) {
                    const uint32_t nc = nsub - s0 < 32u ? nsub - s0 : 32u;
                    mask |= root_mask<PROF>(subs + (sub_base + s0), nc, lo, inv, vx, vy, pf);
                    vy_pf = vy;
                }
            }
        }
        // ---- node loop (trace_core_flat's, with its early leaf phase)
        for (;;) {
            const bool want = has && leaf == 0u && (sp >= 0 || mask != 0u);
            const unsigned long long wm = wballot(want);
            if (wm == 0ull) break;
            if constexpr (PTX_EARLY_LEAF_K > 0) {
                if (__builtin_popcountll(wm) <= PTX_EARLY_LEAF_K &&
                    __builtin_popcountll(wballot(leaf != 0u)) >= PTX_EARLY_LEAF_L)
                    break;
            }
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
        if (wballot(leaf != 0u) == 0ull) continue;
        // ---- cooperative leaf phase (trace_core_flat's)
        if (PROF) pf.hit(PROF_LEAF);
        const uint32_t cnt = leaf ? (leaf >> 24) & 0x7Fu : 0u, lfirst = leaf & LEAF_FIRST_MASK;
        uint32_t tot;
        const uint32_t excl = wave_excl_sum(cnt, tot);
        __hip_atomic_store(&coop.key[lane], ~0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        __atomic_signal_fence(__ATOMIC_SEQ_CST);
        bool nan_seen = false;
        for (uint32_t d0 = 0; d0 < tot; d0 += 64u) {
            const uint32_t u = d0 + lane;
            const int owner = deal_owner(coop, lane, cnt, excl, d0);
            const uint32_t tri = u + __shfl(lfirst - excl, owner);
            const uint32_t tb = __shfl(tri_base, owner);
            const f3 olo = mk(__shfl(lo.x, owner), __shfl(lo.y, owner), __shfl(lo.z, owner));
            const f3 old = mk(__shfl(ld.x, owner), __shfl(ld.y, owner), __shfl(ld.z, owner));
            const float ovy = __shfl(vy, owner);
            if (u < tot) {
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
                    bvalid = true;
                    binst = cur;
                    bmat = grp;
                    bprim = 0xffffffffu - (uint32_t)key;
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
                bvalid = true;
                binst = cur;
                bmat = grp;
                bprim = first + k;
                if (OCC) break;
            }
        }
        leaf = 0u;
        if (OCC && bvalid && !done) {  // occluded: no more work for this query
            done = true;
            sp = -1;
            mask = 0u;
        }
    }
    if (PROF) {
        for (int r = 0; r < PROF_REGIONS; ++r) {
            if (pf.wave[r]) atomicAdd(&sc.counters[8 + 2 * r], (unsigned long long)pf.wave[r]);
            if (pf.lane[r]) atomicAdd(&sc.counters[9 + 2 * r], (unsigned long long)pf.lane[r]);
        }
    }
}

}  // namespace ptx
