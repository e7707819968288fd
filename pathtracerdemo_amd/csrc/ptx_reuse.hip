// ptx_reuse.hip -- temporal and spatial reuse passes in wavefront form.
//
// Not in the reference code: specified only in docs/theory/ReSTIR_Pipeline.md:259-462
// (pass 2 temporal, pass 3 spatial; confidence-weighted generalized balance heuristic) and
// docs/theory/memo.md:166-231 (shift + Jacobian).  The build-defined rules are those of
// oracle/pt_oracle.c (eval_sample, temporal_pixel, spatial_pixel), and
// every reservoir these kernels write is bit-identical to the oracle's.
//
// Both passes are made of "shift jobs": evaluate a reservoir sample (rSeed, XL, length) in
// the domain of some pixel (its camera point and G-buffer hit) -- PT_4's RegeneratePath +
// PathContribution (SH/PT_4_FinalShadingPass.wgsl:1306-1384) plus the shift's pdf product
// and PT_1's roulette factor -- giving (p_hat, q).  A job is <= 3 traces (two regenerated
// BSDF rays, then the light's Visibility), so a pass is: start (create jobs, emit round 0),
// {trace, step} x 3, combine (per pixel: MIS weights, resampling, reservoir out).
//   temporal: 1 job per pixel (its PT_1 sample in its own domain)
//   spatial:  2 per neighbour (neighbour sample -> this pixel, this sample -> neighbour)
// Jobs live in the segment of their pixel; job id = pixel * jobs_per_pixel + slot.
#include "ptx_wave_common.h"

namespace ptx {

constexpr uint32_t SALT_TEMPORAL = 0x54454D50u, SALT_SPATIAL = 0x53504154u;

// Job state, SoA float4 slots (slot k of job j at jstate[k * njobs + j]):
// HDR {hw, rSeed[1], ray idx, sample ref}; F {f, prod | q};
// CUR {pos, inst << 16 | mat}; NRM {nrm, beta}; PREV {prev pos, rr_p}; RRF {rr_f, -}.
// A FRESH job (its first regenerated ray just emitted from the domain's primary hit: i == 1,
// phase 0 -- most jobs of a start kernel) stores 48 B instead of 96: HDR {.. | 1 << 24, domain
// pixel, ray idx, ref}, F {rr_f, prod}, RRF {beta, rr_p, -, -}.  Everything else is a copy of
// data the next step can gather with the same bits: f = (1, 1, 1), the current vertex = the
// domain's surface record, the previous one = its camera point (x0_of), rSeed[1] = word 1 of
// the sample's reservoir.
// hw = i | length << 8 | phase << 16 (2 bits) | lab << 18 (3) | rok << 21 | shift << 22 |
// fresh << 24 | k << 25 (3).  phase: 0 a regenerated BSDF ray out, 1 the light segment's
// Visibility out, 2 the hybrid shift's connection ray out.  shift / k / lab / rok: the hybrid
// shift and the label check (oracle eval_sample), below.
enum : uint32_t { JS_HDR, JS_F, JS_CUR, JS_NRM, JS_PREV, JS_RRF, JS_COUNT };
constexpr uint32_t kJobFresh = 1u << 24;
constexpr uint32_t kResReuseLayout = 0x100u;  // word 20 of a reservoir a reuse pass wrote (oracle RES_REUSE_LAYOUT)
#ifndef PTX_JOB_FRESH
#define PTX_JOB_FRESH 1  // (A/B: 0 stores every job in the full 96-byte layout)
#endif

struct Job {
    uint32_t i, length, phase, seed1, idx, matref;
    uint32_t k, lab;  // the sample's reconnection index; shift: the shifted path's first safe edge so far
    bool shift, rok;  // a shift into another domain (else the sample at home); the current vertex's rough bit
    int32_t ref;  // reservoir index of the sample (band-relative; halo rows are < 0 or >= npix)
    int32_t dom;  // band index of the domain pixel (its camera point and primary hit)
    f3 f;
    float prod;   // pdf product of the regenerated directions; q once the light ray is out
    Surface cur;
    f3 prev;
    float beta, rr_p;
    f3 rr_f;
};

// the spatial pass's job of pixel `pix`, slot `slot` (2m: forward shift from neighbour m, 2m+1: backward)
__device__ __forceinline__ uint32_t job_id(const ReuseArgs &A, uint32_t pix, uint32_t slot) {
    return pix * A.jpx + slot * A.jslot;
}
__device__ __forceinline__ const uint4 *res_at(const uint4 *base, int32_t idx) { return base + 8 * (ptrdiff_t)idx; }
// A job's sample reservoir: a band index into cur (the pass's reservoirs, halo rows < 0 or
// >= npix), or kHistRef + index into hist -- the motion temporal pass's reprojected history
// sample, which lives in the previous frame's spatial output.
// (hist indices may be negative too -- a band's motion halo rows above it: every index of either
// buffer lies within 2^28 of 0, so refs at or above 2^29 are history refs)
constexpr int32_t kHistRef = 1 << 30;
__device__ __forceinline__ const uint4 *res_of(const ReuseArgs &A, int32_t ref) {
    return ref >= (kHistRef >> 1) ? A.hist + 8 * (ptrdiff_t)(ref - kHistRef) : A.cur + 8 * (ptrdiff_t)ref;
}
// a job whose domain is not a pixel of this frame (the previous frame's, motion temporal pass):
// stored in the full layout, as the fresh one re-derives the domain from this frame's records
constexpr int32_t kDomPrev = INT32_MIN;

__device__ __forceinline__ uint32_t job_hw(const Job &s) {
    return s.i | (s.length << 8) | (s.phase << 16) | (s.lab << 18) | (s.rok ? 1u << 21 : 0u) |
           (s.shift ? 1u << 22 : 0u) | (s.k << 25);
}
__device__ __forceinline__ void job_unhw(Job &s, uint32_t hw) {
    s.i = hw & 0xffu; s.length = (hw >> 8) & 0xffu; s.phase = (hw >> 16) & 3u;
    s.lab = (hw >> 18) & 7u; s.rok = (hw >> 21) & 1u; s.shift = (hw >> 22) & 1u; s.k = (hw >> 25) & 7u;
}
// A job waiting for its light segment's Visibility (phase 1) only needs HDR and F.
__device__ __forceinline__ void job_store(const ReuseArgs &A, uint32_t jid, const Job &s) {
    const size_t n = A.njobs;
    float4 *st = A.jstate;
    if (PTX_JOB_FRESH && s.i == 1u && s.phase == 0u && s.dom != kDomPrev) {  // fresh: 48 B (see above)
        st[JS_HDR * n + jid] = make_float4(asf(job_hw(s) | kJobFresh), asf((uint32_t)s.dom), asf(s.idx),
                                           asf((uint32_t)s.ref));
        st[JS_F * n + jid] = make_float4(s.rr_f.x, s.rr_f.y, s.rr_f.z, s.prod);
        st[JS_RRF * n + jid] = make_float4(s.beta, s.rr_p, 0.0f, 0.0f);
        return;
    }
    st[JS_HDR * n + jid] = make_float4(asf(job_hw(s)), asf(s.seed1), asf(s.idx), asf((uint32_t)s.ref));
    st[JS_F * n + jid] = make_float4(s.f.x, s.f.y, s.f.z, s.prod);
    if (s.phase == 1u) return;
    st[JS_CUR * n + jid] = make_float4(s.cur.pos.x, s.cur.pos.y, s.cur.pos.z, asf(s.matref));
    st[JS_NRM * n + jid] = make_float4(s.cur.nrm.x, s.cur.nrm.y, s.cur.nrm.z, s.beta);
    st[JS_PREV * n + jid] = make_float4(s.prev.x, s.prev.y, s.prev.z, s.rr_p);
    st[JS_RRF * n + jid] = make_float4(s.rr_f.x, s.rr_f.y, s.rr_f.z, 0.0f);
}
// (every field is assigned once, after the layouts' branches: stores of different fields sunk into
// one store with a selected address kept the job in scratch memory -- 32 B/lane in wjob_step)
__device__ __forceinline__ void job_load(const Scene &sc, const ReuseArgs &A, uint32_t jid, Job &s) {
    const size_t n = A.njobs;
    const float4 *st = A.jstate;
    const float4 hd = st[JS_HDR * n + jid], fv = st[JS_F * n + jid];
    const uint32_t hw = asu(hd.x);
    job_unhw(s, hw);
    s.idx = asu(hd.z); s.ref = (int32_t)asu(hd.w);
    s.prod = fv.w;
    const bool fresh = (hw & kJobFresh) != 0u;
    uint32_t seed1 = asu(hd.y), matref = 0u;
    int32_t dom = s.dom;
    f3 f = mk(fv.x, fv.y, fv.z), rr_f = mk(0.0f, 0.0f, 0.0f), prev = rr_f;
    float beta = 0.0f, rr_p = 0.0f;
    Surface cur{};
    if (fresh) {  // the fresh layout: gather what it leaves out (same bits)
        const float4 rf = st[JS_RRF * n + jid];
        dom = (int32_t)asu(hd.y);
        seed1 = res_of(A, s.ref)[0].y;
        f = mk(1.0f, 1.0f, 1.0f);
        rr_f = mk(fv.x, fv.y, fv.z);
        beta = rf.x; rr_p = rf.y;
        (void)surf_load(sc, A.surf, dom, cur, matref);  // (a job exists only where it is valid)
        const int32_t W = (int32_t)sc.width, q = dom >= 0 ? dom / W : -((-dom + W - 1) / W);
        prev = x0_of(sc, (uint32_t)(dom - q * W), (uint32_t)((int32_t)sc.row_begin + q));
    } else if (s.phase != 1u) {  // (a job waiting for its Visibility needs HDR and F only)
        const float4 cu = st[JS_CUR * n + jid], nr = st[JS_NRM * n + jid];
        const float4 pv = st[JS_PREV * n + jid], rf = st[JS_RRF * n + jid];
        matref = asu(cu.w);
        cur.pos = mk(cu.x, cu.y, cu.z);
        cur.nrm = mk(nr.x, nr.y, nr.z);
        cur.mat = material_at(sc, matref);
        beta = nr.w;
        prev = mk(pv.x, pv.y, pv.z); rr_p = pv.w;
        rr_f = mk(rf.x, rf.y, rf.z);
    }
    s.seed1 = seed1; s.matref = matref; s.dom = dom;
    s.f = f; s.rr_f = rr_f; s.prev = prev;
    s.beta = beta; s.rr_p = rr_p;
    s.cur = cur;
}

// PT_1's throughput recursion + Russian roulette at one replayed vertex (oracle rr_step).
// (fv = bsdf(X, V, L), pdf = pdf_bsdf(X, V, L): bsdf_pdf)
__device__ __forceinline__ bool rr_step(Job &s, const Surface &X, f3 L, f3 fv, float pdf) {
    s.rr_f = s.rr_f * (fv * fabsf(dot(X.nrm, L)));
    s.rr_p *= pdf;
    const float ps = luminance(s.rr_f) / s.rr_p;
    const bool ok = ps > 0.0f;
    s.rr_p *= ps;
    if (ps > 1.0f) s.beta /= ps;
    return ok;
}

// A fresh job: sample `ref` (length >= 2, reconnection index k) in the domain of camera point x0
// and primary-hit surface X1 (flat material index matref); shift: a shift into that domain (the
// hybrid shift at k, else random replay, either keeping the sample's label), else the sample at
// home (its own PT_1 path, replayed).
__device__ __forceinline__ void job_init(Job &s, f3 x0, const Surface &X1, uint32_t matref, int32_t ref,
                                         uint32_t length, uint32_t seed1, int32_t dom, uint32_t k, bool shift) {
    s.i = 1u; s.length = length; s.phase = 0u; s.seed1 = seed1; s.idx = 0u; s.ref = ref; s.dom = dom;
    s.k = min(k, 7u); s.lab = 0u; s.shift = shift; s.rok = false;
    s.f = mk(1.0f, 1.0f, 1.0f); s.prod = 1.0f;
    s.prev = x0;
    s.cur = X1;
    s.matref = matref;
    s.beta = 1.0f; s.rr_p = 1.0f; s.rr_f = mk(1.0f, 1.0f, 1.0f);
}
// Job at domain pixel (x, y) (band index dom, its surface record), sample `ref`: false if
// eval_sample's preconditions fail (no job; its result is invalid).
__device__ __forceinline__ bool job_begin(const Scene &sc, const ReuseArgs &A, Job &s, uint32_t x, uint32_t y,
                                          int32_t dom, int32_t ref) {
    const uint4 *rv = res_at(A.cur, ref);
    const uint4 r5 = rv[5];
    const uint32_t C = rv[7].y, length = r5.w;
    Surface X1;
    uint32_t matref;
    if (C == 0u || length < 2u || !surf_load(sc, A.surf, dom, X1, matref)) return false;
    job_init(s, x0_of(sc, x, y), X1, matref, ref, length, rv[0].y, dom, r5.x & 0xffu, false);
    return true;
}
// The hybrid shift (oracle eval_sample): a sample whose reconnection index k lies in [2, length-1]
// reconnects its shifted prefix y_{k-1} to its stored x_k; `hyb` also selects that sample's
// measure q = (prod_{i <= k-2} pdf_i * d^2 / |n_k . w|) / beta.
__device__ __forceinline__ bool job_hyb(const Job &s) { return s.k >= 2u && s.k < s.length; }
// IsSafeToReconnect (PT_1:1262-1271) of the edge (a, b), each end's rough bit under its lobe given
// (min(ra, rb) >= R of the oracle's safe_edge: the roughnesses are finite)
__device__ __forceinline__ bool rough_under(const Surface &X, uint32_t lobe) {
    return (lobe == LOBE_LAMBERT ? 1.0f : X.mat.rough) >= RECONNECTION_ROUGHNESS;
}
__device__ __forceinline__ bool safe_edge(bool ra, bool rb, f3 a, f3 b) {
    return length(a - b) >= RECONNECTION_DISTANCE && ra && rb;
}
// the area -> solid angle factor of the reconnection edge prev -> Xk (oracle: d2 / ck)
__device__ __forceinline__ float rc_geo(f3 prev, const Surface &Xk) {
    const f3 dv = Xk.pos - prev;
    const float d2 = dot(dv, dv);
    const float ck = fabsf(dot(Xk.nrm, dv / __builtin_sqrtf(d2)));
    return d2 / ck;
}
// x_{k+1} of a sample: reservoir words 0..3 in the reuse layout, PT_1's pad words 24..27 otherwise
__device__ __forceinline__ uint4 rc_next(const uint4 *rv, uint32_t w20) {
    return (w20 & kResReuseLayout) ? rv[0] : rv[6];
}

// The job's next ray: a regenerated BSDF direction (PT_4:1367-1381), the hybrid shift's
// connection y_{k-1} -> x_k (a closest-hit query: nothing may lie between), or the light
// segment's Visibility (PT_4:1323-1333).  A shift job tracks the shifted path's
// SafeReconnectionIndex on the way (the first safe edge, `lab`; each vertex's rough bit under its
// lobe, `rok`, once that lobe is known) and is invalid unless it equals the sample's k (oracle
// path_label).  Called by every lane of the wave; `emit` selects the lanes with a live job.
// Returns whether the job continues (else its result is out).
// seed0: word 0 of the sample's reservoir (its first replayed draw's seed), read when s.i == 1.
__device__ __forceinline__ bool job_emit(const Scene &sc, const Seg &g, const ReuseArgs &A, bool emit, Job &s,
                                         uint32_t jid, uint32_t seed0) {
    bool ray = false, vis = false, go = false;
    f3 o = mk(0.0f, 0.0f, 0.0f), d = o, Le = o;
    float remain = -1.0f;
    if (emit) {
        const uint4 *rv = res_of(A, s.ref);
        const f3 V = normalize(s.prev - s.cur.pos);
        const bool hyb = job_hyb(s);
        bool ok = true;
        if (s.i + 1u < s.length) {
            // the direction out of the current vertex: to the stored x_k from y_{k-1} (conn, the
            // connection ray follows), to the kept x_{k+1} from x_k (fixd, no ray: the next step
            // takes the vertex), or a regenerated BSDF sample
            const bool conn = s.shift && hyb && s.i + 1u == s.k;
            const bool fixd = s.shift && hyb && s.i == s.k;  // (then k + 1 < length)
            f3 dir;
            uint32_t lobe = LOBE_LAMBERT;
            if (conn || fixd) {
                const uint4 r5 = rv[5];
                const Surface Xt = get_surface(sc, gdecode(conn ? rv[4] : rc_next(rv, r5.x)));
                if (conn) {  // the shifted path's label: edges (k-2, k-1) and (k-1, k)
                    const bool rk1 = rough_under(s.cur, r5.y), rk = rough_under(Xt, r5.z);
                    if (s.i >= 2u && s.lab == 0u && safe_edge(s.rok, rk1, s.prev, s.cur.pos)) s.lab = s.i;
                    if (s.lab == 0u && safe_edge(rk1, rk, s.cur.pos, Xt.pos)) s.lab = s.k;
                    ok = s.lab == s.k;
                }
                const f3 dv = Xt.pos - s.cur.pos;
                dir = dv / length(dv);
            } else {
                uint32_t seed = s.i == 1u ? seed0 : s.seed1;
                dir = sample_bsdf(seed, s.cur, V, lobe);
            }
            float pdf;
            const f3 fv = bsdf_pdf(s.cur, V, dir, pdf);
            if (!conn && !fixd && (!hyb || s.i + 2u <= s.k)) s.prod *= pdf;  // (hybrid: the replayed prefix only)
            ok = rr_step(s, s.cur, dir, fv, pdf) && ok;
            if (s.shift && !conn && !fixd) {
                const bool rl = rough_under(s.cur, lobe);
                if (s.i >= 2u && s.lab == 0u && safe_edge(s.rok, rl, s.prev, s.cur.pos)) s.lab = s.i;
                s.rok = rl;
            }
            s.phase = conn ? 2u : (fixd ? 3u : 0u);
            o = s.cur.pos; d = dir;
            ray = ok && !fixd;
            go = ok;
        } else {
            const LightSample XL = load_xl(rv);
            if (s.shift && !hyb) {  // random replay: the label of the whole path (the last vertex's lobe:
                                   // NEE Lambert, an env escape's stored Lobe_{k-1} when k = length)
                const uint32_t ll = XL.type == LIGHT_ENV ? (s.k == s.length ? rv[5].y : LOBE_GGX) : LOBE_LAMBERT;
                const bool rl = rough_under(s.cur, ll);
                if (s.i >= 2u && s.lab == 0u && safe_edge(s.rok, rl, s.prev, s.cur.pos)) s.lab = s.i;
                if (s.lab == 0u) {
                    const bool rough = s.cur.mat.rough >= RECONNECTION_ROUGHNESS;
                    const bool dirl = XL.type == LIGHT_DIRECTION || XL.type == LIGHT_ENV;
                    if ((dirl || length(s.cur.pos - XL.pos) >= RECONNECTION_DISTANCE) && rough) s.lab = s.length;
                }
                ok = s.lab == s.k;
            }
            const f3 L = direction_to_light(s.cur, XL);
            if (XL.type == LIGHT_ENV) {
                float pdf;
                const f3 fv = bsdf_pdf(s.cur, V, L, pdf);
                ok = rr_step(s, s.cur, L, fv, pdf) && ok;
            }
            s.f = s.f * (bsdf(s.cur, L, V) * fabsf(dot(s.cur.nrm, L)));
            float gl = 1.0f;
            if (XL.type == LIGHT_RECT) {
                const f3 r = XL.pos - s.cur.pos;
                const f3 Ld = normalize(r);
                gl = fabsf(dot(get_light(sc, (uint32_t)XL.id).dir, Ld)) / dot(r, r);
            }
            s.prod = hyb ? s.prod / s.beta : s.prod / (gl * s.beta);  // q
            Le = l_emit<true>(XL, s.cur);
            s.phase = 1u;
            const float dist = length(XL.pos - s.cur.pos);
            o = s.cur.pos; d = (XL.pos - s.cur.pos) / dist; remain = dist;
            vis = true;
            ray = go = ok;
        }
        if (!go) A.jres[jid] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);  // PT_1 would have ended such a path
    }
    const uint32_t idx = g.rbase + wave_alloc(g.l_ray, ray ? 1u : 0u);
    if (ray) {
        s.idx = idx;
        put_ray(g.rays, idx, o, d, remain, vis ? Q_VIS : Q_CLOSEST);
        if (vis) g.res_out[2u * idx] = make_float4(0.0f, Le.x, Le.y, Le.z);
    }
    return go;
}

// After job_emit: store a live job's state and queue it for the next step -- except a job whose
// light ray just went out in a pass that folds light segments into its combine
// (ReuseArgs::fold_last): its jres slot names the ray and its result buffer instead, and no
// step sees it again (its F slot, stored here, is what the combine multiplies).
__device__ __forceinline__ void job_finish(const Seg &g, const JobLists &JL, const ReuseArgs &A, bool live,
                                           const Job &s, uint32_t jid) {
    if (live) job_store(A, jid, s);
    const bool fold = live && A.fold_last && s.phase == 1u;
    if (fold) A.jres[jid] = make_float4(asf(s.idx), asf(g.out_sel), 0.0f, asf(kJobPending));
    job_keep(g, JL, live && !fold, live && s.phase == 1u, jid);
}

#ifndef JOB_STEP_WAVES
// 4 waves per SIMD since the hybrid shift (round 5): its connection / kept-vertex arrivals spill
// 160 B/lane at 96 VGPRs -- reuse 467.4 vs 460.1 at 5 (2 reps, tools/cl/r5_hyb4.sh).  Before it, 5
// (96 VGPRs, 80 B/lane spilled) beside the 5-wave flattened trace: 464.6 vs 461.8 at 4
// (tools/cl/js5_ab.sh); every start / step kernel at 5 (LOGIC_WAVES): reuse +1.0 %, but ReSTIR
// -3.2 %, TEST_MCPT -10 % (tools/cl/lw5_ab.sh)
#define JOB_STEP_WAVES 4
#endif
// One job step of this workgroup's segment (wjob_step, and the fused spatial rounds below);
// `lds` = 3 words of LDS.  Returns the segment's ray count for the next trace round.
__device__ __forceinline__ uint32_t job_step_segment(const Scene &sc, const WaveBufs &w, uint32_t round,
                                                     const ReuseArgs &A, uint32_t *lds) {
    const JobLists JL = job_lists(w, lds);
    const Seg g = seg_begin(w, round, lds);
    uint32_t nh;
    const uint32_t n = split_count(g, nh);
    for (uint32_t base = 0; base < n; base += WB) {
        const uint32_t q = base + threadIdx.x;
        bool emit = false;
        uint32_t jid = 0u;
        Job s;
        if (q < n) {
            jid = split_at(g, JL, q, nh);
            job_load(sc, A, jid, s);
            if (s.phase != 1u) {  // the next vertex: a regenerated BSDF ray's hit (PT_4:1378-1380), or the
                                  // hybrid shift's x_k once its connection is clear / its kept x_{k+1}
                bool ok = true;
                Surface next;
                uint32_t nref = 0u;
                if (s.phase == 0u) {
                    const Hit h = get_hit(g.res_in, s.idx);
                    ok = h.valid;  // (else the replayed path escapes here)
                    if (ok) {
                        next = surface_at(sc, h.s, h.pos);
                        nref = mat_index(sc, h.s.inst, h.s.mat);
                    }
                } else {
                    const uint4 *rv = res_of(A, s.ref);
                    const Compact cc = gdecode(s.phase == 2u ? rv[4] : rc_next(rv, rv[5].x));
                    next = get_surface(sc, cc);
                    nref = mat_index(sc, cc.inst, cc.mat);
                    if (s.phase == 2u) {  // nothing between y_{k-1} and x_k
                        const Hit h = get_hit(g.res_in, s.idx);
                        ok = !(h.valid && h.t < length(next.pos - s.cur.pos) * 0.999f);
                    }
                }
                if (!ok) {
                    A.jres[jid] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
                } else {
                    const f3 V = normalize(s.prev - s.cur.pos);
                    const f3 L = normalize(next.pos - s.cur.pos);
                    s.f = s.f * (bsdf(s.cur, L, V) * fabsf(dot(s.cur.nrm, L)));
                    if (s.phase == 2u || (!s.shift && job_hyb(s) && s.i + 1u == s.k))  // arriving at x_k
                        s.prod = s.prod * rc_geo(s.cur.pos, next);
                    s.prev = s.cur.pos;
                    s.cur = next;
                    s.matref = nref;
                    s.i += 1u;
                    emit = true;
                }
            } else {  // the light segment's Visibility arrived
                const float4 a = g.res_in[2u * s.idx];
                s.f = s.f * (mk(a.y, a.z, a.w) * a.x);
                const float qv = s.prod;
                const bool valid = qv > 0.0f && qv <= 3.402823466e38f;
                // the job's PathContribution f (PT_4's, of this sample at this pixel) and q
                A.jres[jid] = valid ? make_float4(s.f.x, s.f.y, s.f.z, qv) : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            }
        }
        const bool live = job_emit(sc, g, A, emit, s, jid, 0u);  // (s.i >= 2 here)
        job_finish(g, JL, A, live, s, jid);
    }
    job_seg_end(w, g, JL);
    return *g.l_ray;  // (stable after job_seg_end's barrier)
}
__global__ __launch_bounds__(WB) __attribute__((amdgpu_waves_per_eu(JOB_STEP_WAVES, 8)))
void wjob_step(Scene sc, WaveBufs w, uint32_t round, ReuseArgs A) {
    PTX_WAVE_TIMER(sc, KID_JOB_STEP | (w.seg_base ? 0x80u : 0u));
    __shared__ uint32_t lds[3];
    (void)job_step_segment(sc, w, round, A, lds);
}

__device__ __forceinline__ uint32_t reuse_seed(const Scene &sc, uint32_t x, uint32_t y, uint32_t salt) {
    return pcg(pcg(x * 1973u + y * 9277u + sc.U[U_FRAME] * 26699u) ^ salt);
}
__device__ __forceinline__ bool wrs_update(float &w_sum, float wt, uint32_t &seed) {  // PT_1:1298-1320
    w_sum += wt;
    return rnd(seed) < wt / w_sum;
}
// The selected sample's PathContribution at this pixel, when known (oracle sel_f): a job's
// valid result, or what an earlier reuse pass stored (words 26, 27, 30 + flag word 31).
struct SelF { bool known; f3 f; };
__device__ __forceinline__ SelF job_f(float4 r) { return SelF{r.w > 0.0f, mk(r.x, r.y, r.z)}; }
// A job result as the combine reads it: a job folded into the combine (ReuseArgs::fold_last)
// is finished here with wjob_step's phase-1 arithmetic -- its light segment's Visibility
// result (res) and the F slot of its state.
__device__ __forceinline__ float4 job_result(const ReuseArgs &A, const WaveBufs &w, float4 r, uint32_t jid) {
    // (a slot the combine loads but never uses may hold anything: a stale or uninitialised
    // word pair is kept inside the buffers, its value is discarded by the caller)
    if (asu(r.w) != kJobPending || asu(r.x) >= A.ray_cap || asu(r.y) >= w.nres) return r;
    const float4 a = w.res[asu(r.y)][2u * asu(r.x)], fv = A.jstate[JS_F * (size_t)A.njobs + jid];
    const f3 f = mk(fv.x, fv.y, fv.z) * (mk(a.y, a.z, a.w) * a.x);
    const float qv = fv.w;
    const bool valid = qv > 0.0f && qv <= 3.402823466e38f;
    return valid ? make_float4(f.x, f.y, f.z, qv) : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
}
__device__ __forceinline__ float4 job_at(const ReuseArgs &A, const WaveBufs &w, uint32_t pix, uint32_t slot) {
    const uint32_t jid = job_id(A, pix, slot);
    return job_result(A, w, A.jres[jid], jid);
}
__device__ __forceinline__ SelF stored_f(const uint4 *r) {
    const uint4 r6 = r[6], r7 = r[7];
    return SelF{r7.w == 1u, mk(asf(r6.z), asf(r6.w), asf(r7.z))};
}
__device__ __forceinline__ void write_reused(uint4 *out, const uint4 *src, float p_sel, float q_sel, SelF fs,
                                             float w_sum, uint32_t C) {
    // all loads before the stores: src may be out itself (temporal)
    uint4 a0 = src[0], a5 = src[5];
    const uint4 a1 = src[1], a2 = src[2], a3 = src[3], a4 = src[4];
    if (fs.known && !(a5.x & kResReuseLayout)) {  // a PT_1 sample: into the reuse layout (oracle write_reused)
        const uint32_t k = a5.x & 0xffu;
        if (k >= 2u && k + 1u < a5.w) a0 = src[6];  // x_{k+1} over seeds the hybrid shift never replays
        a5.x |= kResReuseLayout;
    }
    out[0] = a0; out[1] = a1; out[2] = a2; out[3] = a3; out[4] = a4; out[5] = a5;
    out[6] = make_uint4(asu(p_sel), asu(q_sel), fs.known ? asu(fs.f.x) : 0u, fs.known ? asu(fs.f.y) : 0u);
    out[7] = make_uint4(asu(p_sel > 0.0f ? w_sum / p_sel : 0.0f), C, fs.known ? asu(fs.f.z) : 0u, fs.known ? 1u : 0u);
}

// The spatial pass's 16-byte neighbour summary of a reservoir (see wnbr_summary below).
constexpr uint32_t kNbrEscape = 0xFFFFFFFFu;
// word w: valid << 31 | length << 27 | k << 23 | C (r5 = words 20..23: {k | layout, -, -, length});
// a length or k past 15 or a C past 2^23 - 2 takes the escape
__device__ __forceinline__ uint4 nbr_pack(bool valid, uint4 r5, uint4 r6, uint4 r7) {
    uint32_t w = 0u;
    const uint32_t k = r5.x & 0xffu;
    if (valid)
        w = (r5.w > 0xfu || k > 0xfu || r7.y > 0x7ffffeu) ? kNbrEscape : (1u << 31) | (r5.w << 27) | (k << 23) | r7.y;
    return make_uint4(r6.x, r6.y, r7.x, w);
}

// ---------------------------------------------------------------- temporal
// The canonical sample is PT_1's own path: replaying its BSDF draws from its pixel's hit
// gives back PT_1's vertices, whose hits PT_1 left in its wave state (vertex 2 / 3 compacts),
// and its light segment's Visibility is the one PT_1 traced for the selected NEE candidate.
// So the job runs without tracing -- the same operations as job_emit + wjob_step, with the
// trace results read instead of recomputed (identical bits: same rays, deterministic
// traversal).  Returns true when the job still needs its light ray (an env candidate).
__device__ __forceinline__ bool temporal_from_init(const Scene &sc, const WaveBufs &w, const ReuseArgs &A, Job &s,
                                                   uint32_t pix, uint32_t jid) {
    const uint4 *rv = res_at(A.cur, s.ref);
    const bool hyb = job_hyb(s);
    while (s.i + 1u < s.length) {
        f3 V = normalize(s.prev - s.cur.pos);
        uint32_t seed = s.i == 1u ? rv[0].x : s.seed1, lobe;
        const f3 dir = sample_bsdf(seed, s.cur, V, lobe);
        float pdf;
        const f3 fv = bsdf_pdf(s.cur, V, dir, pdf);
        if (!hyb || s.i + 2u <= s.k) s.prod *= pdf;
        if (!rr_step(s, s.cur, dir, fv, pdf)) {
            A.jres[jid] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            return false;
        }
        const float4 c = w.state[(s.i == 1u ? kStateCs2 : kStateCs3) * w.npix + pix];
        const Surface next = get_surface(sc, gdecode(make_uint4(asu(c.x), asu(c.y), asu(c.z), asu(c.w))));
        V = normalize(s.prev - s.cur.pos);
        const f3 L = normalize(next.pos - s.cur.pos);
        s.f = s.f * (bsdf(s.cur, L, V) * fabsf(dot(s.cur.nrm, L)));
        if (hyb && s.i + 1u == s.k) s.prod = s.prod * rc_geo(s.cur.pos, next);
        s.prev = s.cur.pos;
        s.cur = next;
        s.i += 1u;
    }
    const float T = w.state[kStateTsel * w.npix + pix].x;
    if (T < 0.0f) return true;  // env candidate: its Visibility was never traced
    const LightSample XL = load_xl(rv);
    const f3 V = normalize(s.prev - s.cur.pos);
    const f3 L = direction_to_light(s.cur, XL);
    s.f = s.f * (bsdf(s.cur, L, V) * fabsf(dot(s.cur.nrm, L)));
    float gl = 1.0f;
    if (XL.type == LIGHT_RECT) {
        const f3 r = XL.pos - s.cur.pos;
        const f3 Ld = normalize(r);
        gl = fabsf(dot(get_light(sc, (uint32_t)XL.id).dir, Ld)) / dot(r, r);
    }
    s.prod = hyb ? s.prod / s.beta : s.prod / (gl * s.beta);
    const f3 Le = l_emit<true>(XL, s.cur);
    s.f = s.f * (Le * T);
    const float qv = s.prod;
    const bool valid = qv > 0.0f && qv <= 3.402823466e38f;
    A.jres[jid] = valid ? make_float4(s.f.x, s.f.y, s.f.z, qv) : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    return false;
}

// (the inlined replay needs more registers than the 4-wave budget: 160 B/lane spilled there)
__global__ __launch_bounds__(WB) __attribute__((amdgpu_waves_per_eu(2, 8)))
void wtemporal_start(Scene sc, WaveBufs w, ReuseArgs A) {
    PTX_WAVE_TIMER(sc, KID_TEMP_START | (w.seg_base ? 0x80u : 0u));
    __shared__ uint32_t lds[3];
    const JobLists JL = job_lists(w, lds);
    const Seg g = seg_begin(w, 0u, lds);
    const uint32_t np = padded_pixels(sc);
    for (uint32_t k = 0; k < w.seg_px; k += WB) {
        const uint32_t q = seg_pixel(w, g.j, k);
        uint32_t x, y, pix = 0u;
        bool active = false;
        Job s;
        if (q < np && tile_xy(sc, q, x, y)) {
            pix = (y - sc.row_begin) * sc.width + x;
            active = job_begin(sc, A, s, x, y, (int32_t)pix, (int32_t)pix);
            if (active && A.use_init) active = temporal_from_init(sc, w, A, s, pix, pix);
        }
        const bool live = job_emit(sc, g, A, active, s, pix, active ? A.cur[8u * (size_t)pix].x : 0u);
        job_finish(g, JL, A, live, s, pix);
    }
    job_seg_end(w, g, JL);
}

// Temporal resampling of the pixel's PT_1 reservoir with the previous frame's output at
// the same pixel (oracle temporal_pixel): static camera, identity shift.
__global__ __launch_bounds__(WB) void wtemporal_combine(Scene sc, WaveBufs w, ReuseArgs A) {
    PTX_WAVE_TIMER(sc, KID_TEMP_COMBINE | (w.seg_base ? 0x80u : 0u));
    const uint32_t j = w.seg_base + blockIdx.x, np = padded_pixels(sc);
    for (uint32_t k = 0; k < w.seg_px; k += WB) {
        const uint32_t q = seg_pixel(w, j, k);
        uint32_t x, y;
        if (q >= np || !tile_xy(sc, q, x, y)) continue;
        const uint32_t pix = (y - sc.row_begin) * sc.width + x;
        if (!gdecode(A.gbuf[pix]).valid) {  // PT_1 wrote the zero reservoir
            A.nbr_out[pix] = make_uint4(0u, 0u, 0u, 0u);
            continue;
        }
        uint4 *rv = A.cur + 8u * (size_t)pix;
        const uint4 *hv = A.hist + 8u * (size_t)pix;
        uint32_t seed = reuse_seed(sc, x, y, SALT_TEMPORAL);
        const uint4 r5 = rv[5], r7 = rv[7];
        const float4 er = (r7.y != 0u && r5.w >= 2u) ? job_result(A, w, A.jres[pix], pix) : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        const float2 ec = make_float2(er.w > 0.0f ? luminance(mk(er.x, er.y, er.z)) : 0.0f, er.w);
        const bool canon_ok = ec.y > 0.0f && ec.x > 0.0f;
        const uint4 h5 = hv[5], h6 = hv[6], h7 = hv[7];
        const uint32_t Cp = A.hist_valid ? min(h7.y, A.cap) : 0u;
        const float cp = (float)Cp, tot = 1.0f + cp;
        const float pp = asf(h6.x), qp = asf(h6.y);
        const bool hist_ok = Cp != 0u && h5.w >= 2u && pp > 0.0f;
        const float wc = canon_ok ? (1.0f / tot) * ec.x * asf(r7.x) : 0.0f;
        const float wp = hist_ok ? (cp / tot) * pp * asf(h7.x) : 0.0f;
        float w_sum = 0.0f, p_sel = ec.x, q_sel = ec.y;
        bool from_hist = false;
        if (wrs_update(w_sum, wc, seed)) { from_hist = false; p_sel = ec.x; q_sel = ec.y; }
        if (wrs_update(w_sum, wp, seed)) { from_hist = true; p_sel = pp; q_sel = qp; }
        write_reused(rv, from_hist ? hv : rv, p_sel, q_sel, from_hist ? stored_f(hv) : job_f(er), w_sum, 1u + Cp);
        // the spatial pass's summary of the output (words 23, 24, 25, 28, 29 as written above)
        const float W = p_sel > 0.0f ? w_sum / p_sel : 0.0f;
        A.nbr_out[pix] = nbr_pack(true, make_uint4(from_hist ? h5.x : r5.x, 0u, 0u, from_hist ? h5.w : r5.w),
                                  make_uint4(asu(p_sel), asu(q_sel), 0u, 0u), make_uint4(asu(W), 1u + Cp, 0u, 0u));
    }
}

// ---------------------------------------------------------------- temporal, moved camera
// The history of pixel p lives at its reprojection p' in the previous frame, in that frame's
// domain (oracle temporal_motion_pixel, the rules and their constants are stated there): three
// shift jobs per pixel -- slot 0 the canonical PT_1 sample at home (from PT_1's state, as the
// still-camera pass), slot 1 the history sample at p' replayed here, slot 2 the canonical sample
// replayed from the previous frame's camera point and primary hit at p' -- then a combine with
// the generalized balance heuristic (the spatial pass's pairwise rule with M = 1).
__device__ __forceinline__ f3 x0_prev(const ReuseArgs &A, const Scene &sc, uint32_t x, uint32_t y) {
    float u = ((float)x + 0.5f) / (float)sc.U[U_W];  // (x0_of with the previous frame's VP^-1)
    float v = ((float)y + 0.5f) / (float)sc.U[U_H];
    return xform_point(A.vpinv_prev, mk(2.0f * u - 1.0f, 2.0f * v - 1.0f, 0.0f));
}
struct MotionHist { bool ok; int32_t pp; uint32_t px, py, C; };
// p' of pixel (x, y)'s primary hit X1 and the disocclusion test (oracle reproject / motion_valid):
// C = min(C_hist, cap) when the history at p' is usable, else 0.  A reprojection more than
// `radius` rows from y gets none, in every handle (oracle motion_rows): a band's motion halo
// holds exactly those rows, so a split frame matches one handle under any motion.
// (count: this call counts such a clipped reprojection in A.clip)
__device__ __forceinline__ MotionHist motion_hist(const Scene &sc, const ReuseArgs &A, const Surface &X1, uint32_t y,
                                                  bool count = false) {
    MotionHist m{false, 0, 0u, 0u, 0u};
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
    // p' in the band's addressing: the previous frame's rows this handle holds are its band and
    // the motion halo received from the neighbours (the whole image: every row)
    const int32_t ry = (int32_t)m.py - (int32_t)sc.row_begin;
    if (abs((int32_t)m.py - (int32_t)y) > (int32_t)A.radius || ry < A.prev_row_lo || ry >= A.prev_row_hi) {
        if (count && A.clip) atomicAdd(A.clip, 1ull);
        return m;
    }
    m.pp = ry * (int32_t)sc.width + (int32_t)m.px;
    const uint4 a = A.psurf[2 * (ptrdiff_t)m.pp];
    if (a.w == kNoSurface) return m;
    const uint4 b = A.psurf[2 * (ptrdiff_t)m.pp + 1];
    const f3 pp = mk(asf(a.x), asf(a.y), asf(a.z)), pn = mk(asf(b.x), asf(b.y), asf(b.z));
    if (!(dot(pn, X1.nrm) >= 0.9f)) return m;
    const f3 x0p = x0_prev(A, sc, m.px, m.py);
    const float dp = length(pp - x0p), dc = length(P - x0p);
    if (!(fabsf(dp - dc) <= 0.05f * dc)) return m;
    m.C = min(A.hist[8 * (ptrdiff_t)m.pp + 7].y, A.cap);
    m.ok = m.C != 0u;
    return m;
}

#ifndef MOTION_START_WAVES
#define MOTION_START_WAVES 3
#endif
__global__ __launch_bounds__(WB) __attribute__((amdgpu_waves_per_eu(MOTION_START_WAVES, 8)))
void wtmotion_start(Scene sc, WaveBufs w, ReuseArgs A) {
    PTX_WAVE_TIMER(sc, KID_TEMP_START | (w.seg_base ? 0x80u : 0u));
    __shared__ uint32_t lds[3];
    const JobLists JL = job_lists(w, lds);
    const Seg g = seg_begin(w, 0u, lds);
    const uint32_t np = padded_pixels(sc);
    for (uint32_t k = 0; k < w.seg_px; k += WB) {
        const uint32_t q = seg_pixel(w, g.j, k);
        uint32_t x = 0u, y = 0u, pix = 0u;
        bool valid = false;
        Surface X1{};
        uint32_t mref = 0u;
        if (q < np && tile_xy(sc, q, x, y)) {
            pix = (y - sc.row_begin) * sc.width + x;
            valid = surf_load(sc, A.surf, pix, X1, mref);
        }
        const uint4 *rv = A.cur + 8u * (size_t)pix;
        const uint4 r5c = valid ? rv[5] : make_uint4(0u, 0u, 0u, 0u);
        const uint32_t cC = valid ? rv[7].y : 0u, clen = r5c.w, ck = r5c.x & 0xffu;
        const bool canon = valid && cC != 0u && clen >= 2u;
        const MotionHist mh = valid ? motion_hist(sc, A, X1, y, true) : MotionHist{false, 0, 0u, 0u, 0u};
        // the pixel's jobs through ONE job_emit site (three inlined copies needed 256 VGPRs)
#pragma unroll 1
        for (uint32_t slot = 0; slot < kMotionJobs; ++slot) {  // (uniform)
            const uint32_t jid = job_id(A, pix, slot);
            Job s;
            bool act = false;
            uint32_t s0 = 0u;
            if (slot == 0u) {  // the canonical sample at home (PT_1's state when it still describes it)
                act = canon && job_begin(sc, A, s, x, y, (int32_t)pix, (int32_t)pix);
                if (act && A.use_init) act = temporal_from_init(sc, w, A, s, pix, jid);
                if (act) s0 = rv[0].x;
            } else if (slot == 1u) {  // the history sample at p' in this pixel's domain
                if (mh.ok) {
                    const uint4 *hv = A.hist + 8 * (ptrdiff_t)mh.pp;
                    const uint4 h0 = hv[0], h5 = hv[5], h6 = hv[6];
                    act = h5.w >= 2u && asf(h6.x) > 0.0f;
                    if (act) {
                        job_init(s, x0_of(sc, x, y), X1, mref, kHistRef + mh.pp, h5.w, h0.y, (int32_t)pix, h5.x & 0xffu,
                                 true);
                        s0 = h0.x;
                    }
                }
            } else if (mh.ok && canon) {  // the canonical sample in the previous frame's domain at p'
                // (used only when the canonical evaluation is valid; created whenever it may be)
                Surface Xp;
                uint32_t pref;
                act = surf_load(sc, A.psurf, mh.pp, Xp, pref);
                if (act) {
                    job_init(s, x0_prev(A, sc, mh.px, mh.py), Xp, pref, (int32_t)pix, clen, rv[0].y, kDomPrev, ck, true);
                    s0 = rv[0].x;
                }
            }
            const bool live = job_emit(sc, g, A, act, s, jid, s0);
            job_finish(g, JL, A, live, s, jid);
        }
    }
    job_seg_end(w, g, JL);
}

__global__ __launch_bounds__(WB) void wtmotion_combine(Scene sc, WaveBufs w, ReuseArgs A) {
    PTX_WAVE_TIMER(sc, KID_TEMP_COMBINE | (w.seg_base ? 0x80u : 0u));
    const uint32_t j = w.seg_base + blockIdx.x, np = padded_pixels(sc);
    for (uint32_t k = 0; k < w.seg_px; k += WB) {
        const uint32_t q = seg_pixel(w, j, k);
        uint32_t x, y;
        if (q >= np || !tile_xy(sc, q, x, y)) continue;
        const uint32_t pix = (y - sc.row_begin) * sc.width + x;
        Surface X1;
        uint32_t mref;
        if (!surf_load(sc, A.surf, pix, X1, mref)) {  // PT_1 wrote the zero reservoir
            A.nbr_out[pix] = make_uint4(0u, 0u, 0u, 0u);
            continue;
        }
        uint4 *rv = A.cur + 8u * (size_t)pix;
        uint32_t seed = reuse_seed(sc, x, y, SALT_TEMPORAL);
        const uint4 r5 = rv[5], r7 = rv[7];
        const float4 er = (r7.y != 0u && r5.w >= 2u) ? job_at(A, w, pix, 0u) : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        const float ecp = er.w > 0.0f ? luminance(mk(er.x, er.y, er.z)) : 0.0f, ecq = er.w;
        const bool canon_ok = ecq > 0.0f && ecp > 0.0f;
        const float cc = 1.0f, pc = ecp, qc = ecq, Wc = asf(r7.x);
        const MotionHist mh = motion_hist(sc, A, X1, y);
        const uint32_t Cp = mh.ok ? mh.C : 0u;
        const float cp = (float)Cp;
        const uint4 *hv = A.hist + 8 * (ptrdiff_t)mh.pp;
        // forward: the history sample shifted here
        float wh = 0.0f, pf = 0.0f, qf = 0.0f;
        SelF ff{false, mk(0.0f, 0.0f, 0.0f)};
        uint32_t hlen = 0u, hk = 0u;
        if (Cp != 0u) {
            const uint4 h5 = hv[5], h6 = hv[6], h7 = hv[7];
            hlen = h5.w;
            hk = h5.x;
            const float ph = asf(h6.x), qh = asf(h6.y), Wh = asf(h7.x);
            if (h5.w >= 2u && ph > 0.0f) {
                const float4 Fr = job_at(A, w, pix, 1u);
                if (Fr.w > 0.0f) {
                    const float Fp = luminance(mk(Fr.x, Fr.y, Fr.z)), Fq = Fr.w;
                    const float J = qh / Fq;
                    const float pb = ph / J;
                    const float den = cc * Fp + cp * pb;
                    const float m = den > 0.0f ? (cp * pb) / den : 0.0f;
                    wh = m * Fp * Wh * J;
                    pf = Fp;
                    qf = Fq;
                    ff = job_f(Fr);
                }
            }
        }
        // backward: the canonical sample's weight from its shift into the previous domain
        float Q = 1.0f;
        if (canon_ok && Cp != 0u) {
            const float4 B = job_at(A, w, pix, 2u);
            if (B.w > 0.0f) {
                const float pbc = luminance(mk(B.x, B.y, B.z)) * qc / B.w;
                const float den = cc * pc + cp * pbc;
                Q = den > 0.0f ? (cc * pc) / den : 1.0f;
            }
        }
        const float wc = canon_ok ? Q * pc * Wc : 0.0f;
        float w_sum = 0.0f, p_sel = ecp, q_sel = ecq;
        bool from_hist = false;
        if (wrs_update(w_sum, wc, seed)) { from_hist = false; p_sel = ecp; q_sel = ecq; }
        if (wrs_update(w_sum, wh, seed)) { from_hist = true; p_sel = pf; q_sel = qf; }
        write_reused(rv, from_hist ? hv : rv, p_sel, q_sel, from_hist ? ff : job_f(er), w_sum, 1u + Cp);
        const float Wo = p_sel > 0.0f ? w_sum / p_sel : 0.0f;
        A.nbr_out[pix] = nbr_pack(true, make_uint4(from_hist ? hk : r5.x, 0u, 0u, from_hist ? hlen : r5.w),
                                  make_uint4(asu(p_sel), asu(q_sel), 0u, 0u), make_uint4(asu(Wo), 1u + Cp, 0u, 0u));
    }
}

// ---------------------------------------------------------------- spatial
// Spatial neighbour of (x, y): two draws, offsets in [-R, R]^2 (oracle spatial_neighbor).
__device__ __forceinline__ bool spatial_neighbor(uint32_t &seed, uint32_t R, uint32_t x, uint32_t y, uint32_t W,
                                                 uint32_t H, uint32_t &nx, uint32_t &ny) {
    const float side = (float)(2u * R + 1u);
    uint32_t ix = (uint32_t)(rnd(seed) * side);
    uint32_t iy = (uint32_t)(rnd(seed) * side);
    ix = min(ix, 2u * R);  // Random() can return exactly 1.0
    iy = min(iy, 2u * R);
    const int X = (int)x + (int)ix - (int)R, Y = (int)y + (int)iy - (int)R;
    if (X < 0 || Y < 0 || X >= (int)W || Y >= (int)H || (ix == R && iy == R)) return false;
    nx = (uint32_t)X;
    ny = (uint32_t)Y;
    return true;
}
__device__ __forceinline__ int32_t band_index(const Scene &sc, uint32_t x, uint32_t y) {
    return ((int32_t)y - (int32_t)sc.row_begin) * (int32_t)sc.width + (int32_t)x;
}

// Neighbour summary (one uint4 per band + halo pixel, written by wnbr_summary before the
// spatial jobs start): {p_hat (word 24), q (25), W (28), G-buffer valid << 31 | length << 24 |
// C}, or w = kNbrEscape when length or C does not fit (then read the reservoir itself).  A
// neighbour costs one 16-byte gather instead of a G-buffer line and a reservoir line.
struct Nbr { bool valid; uint32_t length, C; float p, q, W; uint32_t k; };
__device__ __forceinline__ Nbr nbr_unpack(uint4 v) {
    return Nbr{(v.w >> 31) != 0u, (v.w >> 27) & 0xfu, v.w & 0x7fffffu, asf(v.x), asf(v.y), asf(v.z), (v.w >> 23) & 0xfu};
}
__device__ __forceinline__ Nbr nbr_at(const ReuseArgs &A, int32_t idx) {
    const uint4 v = A.nbr[idx];
    if (v.w != kNbrEscape)
        return nbr_unpack(v);
    const uint4 *rv = res_at(A.cur, idx);
    const uint4 r5 = rv[5], r6 = rv[6], r7 = rv[7];
    return Nbr{gdecode(A.gbuf[idx]).valid != 0u, r5.w, r7.y, asf(r6.x), asf(r6.y), asf(r7.x), r5.x & 0xffu};
}
__global__ __launch_bounds__(WB) void wnbr_summary(Scene sc, const uint4 *gbuf, const uint4 *res, uint4 *nbr,
                                                   uint4 *surf, size_t npx) {
    const size_t i = (size_t)blockIdx.x * WB + threadIdx.x;
    if (i >= npx) return;
    const uint4 *rv = res + 8u * i;
    const uint4 g = gbuf[i];
    nbr[i] = nbr_pack((g.x >> 31) != 0u, rv[5], rv[6], rv[7]);
    if (surf) surf_from_gbuf(sc, surf, (ptrdiff_t)i, g);
}
hipError_t wave_reuse_summary(const Scene &sc, const uint4 *gbuf, const uint4 *res, uint4 *nbr, uint4 *surf,
                              size_t npx, hipStream_t s) {
    if (npx == 0) return hipSuccess;
    hipLaunchKernelGGL(wnbr_summary, dim3((unsigned)((npx + WB - 1) / WB)), dim3(WB), 0, s, sc, gbuf, res, nbr, surf,
                       npx);
    return hipGetLastError();
}

// The surface records of the launch's segments (WaveBufs::surf) from the G-buffer.
__global__ __launch_bounds__(WB) void wsurface(Scene sc, WaveBufs w, const uint4 *gbuf) {
    const uint32_t j = w.seg_base + blockIdx.x, np = padded_pixels(sc);
    for (uint32_t k = 0; k < w.seg_px; k += WB) {
        const uint32_t q = seg_pixel(w, j, k);
        uint32_t x, y;
        if (q >= np || !tile_xy(sc, q, x, y)) continue;
        const uint32_t pix = (y - sc.row_begin) * sc.width + x;
        surf_from_gbuf(sc, w.surf, (ptrdiff_t)pix, gbuf[pix]);
    }
}
hipError_t wave_surface(const Scene &sc, const WaveBufs &w, const uint4 *gbuf, hipStream_t s) {
    if (!w.surf || !w.seg_count) return hipSuccess;
    hipLaunchKernelGGL(wsurface, dim3(w.seg_count), dim3(WB), 0, s, sc, w, gbuf);
    return hipGetLastError();
}

// One thread per (pixel, kind): the forward shifts (slots 2m: neighbour m's sample in this
// pixel's domain) share the pixel's camera point and hit surface, the backward ones (2m+1:
// this pixel's sample in neighbour m's domain) its reservoir; the neighbour offsets come
// from one pass over the pixel's salted stream.  A workgroup walks its segment kind by kind
// and neighbour by neighbour, so a wave emits one 8x8 tile's jobs of one slot at a time.
constexpr uint32_t kMaxPrefetch = 3u;  // neighbours whose data wspatial_start gathers up front
#ifndef SPATIAL_START_WAVES
#define SPATIAL_START_WAVES 3  // the shared surface + one job: 128 VGPRs spill 108 B/lane
#endif
__global__ __launch_bounds__(WB) __attribute__((amdgpu_waves_per_eu(SPATIAL_START_WAVES, 8)))
void wspatial_start(Scene sc, WaveBufs w, ReuseArgs A) {
    PTX_WAVE_TIMER(sc, KID_SPAT_START | (w.seg_base ? 0x80u : 0u));
    __shared__ uint32_t lds[3];
    const JobLists JL = job_lists(w, lds);
    const Seg g = seg_begin(w, 0u, lds);
    const uint32_t np = padded_pixels(sc), M = A.neighbors;
    for (uint32_t base = 0; base < w.seg_px * 2u; base += WB) {  // workgroup-uniform
        const bool backward = base >= w.seg_px;
        const uint32_t q = seg_pixel(w, g.j, base % w.seg_px);
        uint32_t x = 0u, y = 0u, pix = 0u, seed = 0u, mref = 0u;
        bool valid = false, canon = false;
        Surface X1{};
        f3 x0{};
        uint4 c0 = make_uint4(0u, 0u, 0u, 0u);
        uint32_t clen = 0u, ck = 0u;
        if (q < np && tile_xy(sc, q, x, y)) {
            pix = (y - sc.row_begin) * sc.width + x;
            seed = reuse_seed(sc, x, y, SALT_SPATIAL);
            if (!backward) {
                valid = surf_load(sc, A.surf, pix, X1, mref);
                if (valid) x0 = x0_of(sc, x, y);
            } else {
                valid = A.surf[2u * (size_t)pix].w != kNoSurface;
                const uint4 *rc = A.cur + 8u * (size_t)pix;  // this pixel's sample, shifted to each neighbour
                const uint4 r5 = rc[5];
                canon = valid && rc[7].y != 0u && r5.w >= 2u && asf(rc[6].x) > 0.0f;
                if (canon) { c0 = rc[0]; clen = r5.w; ck = r5.x & 0xffu; }
            }
        }
        // every neighbour's offset first, then its summary + seeds (forward) or surface record
        // (backward) for all of them in one round trip, then the jobs one by one
        uint32_t nxy[kMaxPrefetch];
        int32_t nidx[kMaxPrefetch];
        uint4 pa[kMaxPrefetch], pb[kMaxPrefetch];
        const uint32_t MP = M < kMaxPrefetch ? M : kMaxPrefetch;
#pragma unroll
        for (uint32_t m = 0; m < kMaxPrefetch; ++m) {
            uint32_t nx = 0u, ny = 0u;
            const bool present = m < MP && valid && spatial_neighbor(seed, A.radius, x, y, sc.width, sc.height, nx, ny);
            nxy[m] = present ? (nx | (ny << 16)) : 0xffffffffu;
            nidx[m] = present ? band_index(sc, nx, ny) : 0;
        }
#pragma unroll
        for (uint32_t m = 0; m < kMaxPrefetch; ++m) {
            pa[m] = make_uint4(0u, 0u, 0u, kNoSurface);
            pb[m] = make_uint4(0u, 0u, 0u, 0u);
            if (nxy[m] != 0xffffffffu) {
                if (!backward) { pa[m] = A.nbr[nidx[m]]; pb[m] = A.cur[8 * (ptrdiff_t)nidx[m]]; }
                else if (canon) { pa[m] = A.surf[2 * (ptrdiff_t)nidx[m]]; pb[m] = A.surf[2 * (ptrdiff_t)nidx[m] + 1]; }
            }
        }
        for (uint32_t m = 0; m < M; ++m) {  // uniform
            const uint32_t jid = job_id(A, pix, 2u * m + (backward ? 1u : 0u));
            bool act = false;
            uint32_t s0 = 0u;
            Job s;
            if (valid) {
                uint32_t nx = 0u, ny = 0u, pxy = 0xffffffffu;
                int32_t ni = 0;
                uint4 a = make_uint4(0u, 0u, 0u, kNoSurface), b = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
                for (uint32_t k = 0; k < kMaxPrefetch; ++k)
                    if (k == m) { pxy = nxy[k]; ni = nidx[k]; a = pa[k]; b = pb[k]; }
                if (m >= kMaxPrefetch) {  // (more neighbours than prefetched: this one's draws now)
                    uint32_t sm = reuse_seed(sc, x, y, SALT_SPATIAL) + 2u * m;  // draws 2m, 2m + 1
                    if (spatial_neighbor(sm, A.radius, x, y, sc.width, sc.height, nx, ny)) {
                        pxy = nx | (ny << 16);
                        ni = band_index(sc, nx, ny);
                        if (!backward) { a = A.nbr[ni]; b = A.cur[8 * (ptrdiff_t)ni]; }
                        else if (canon) { a = A.surf[2 * (ptrdiff_t)ni]; b = A.surf[2 * (ptrdiff_t)ni + 1]; }
                    }
                }
                const bool present = pxy != 0xffffffffu;
                nx = pxy & 0xffffu; ny = pxy >> 16;
                bool want = false;
                if (present && !backward) {  // the neighbour's sample in this pixel's domain
                    const Nbr nb = a.w != kNbrEscape ? nbr_unpack(a) : nbr_at(A, ni);
                    want = nb.valid && nb.length >= 2u && nb.p > 0.0f;
                    act = want && nb.C != 0u;
                    if (act) { job_init(s, x0, X1, mref, ni, nb.length, b.y, (int32_t)pix, nb.k, true); s0 = b.x; }
                } else if (present && canon) {  // this pixel's sample in the neighbour's domain
                    want = act = a.w != kNoSurface;
                    if (act) {
                        Surface Xn;
                        Xn.pos = mk(asf(a.x), asf(a.y), asf(a.z));
                        Xn.nrm = mk(asf(b.x), asf(b.y), asf(b.z));
                        Xn.mat = material_at(sc, a.w);
                        job_init(s, x0_of(sc, nx, ny), Xn, a.w, (int32_t)pix, clen, c0.y, ni, ck, true);
                        s0 = c0.x;
                    }
                }
                if (want && !act) A.jres[jid] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            }
            const bool live = job_emit(sc, g, A, act, s, jid, s0);
            job_finish(g, JL, A, live, s, jid);
        }
    }
    job_seg_end(w, g, JL);
}

// Pairwise-MIS resampling of the pixel's temporal reservoir and its neighbours' shifted
// samples (oracle spatial_pixel); writes the reservoir PT_4 reads.  Pass 1 sums the
// neighbours' confidences and the canonical sample's MIS weight, pass 2 resamples (canonical
// first; the selection draws follow the offset draws).
struct CombineCanon { float cc, pc, qc, Wc; bool ok; };
__device__ __forceinline__ float canon_q(const CombineCanon &c, float Mf, uint32_t Cn, float4 B) {
    float Q = 1.0f;
    if (c.ok && B.w > 0.0f) {
        const float pbc = luminance(mk(B.x, B.y, B.z)) * c.qc / B.w;
        const float den = c.cc * c.pc + Mf * (float)Cn * pbc;
        Q = den > 0.0f ? (c.cc * c.pc) / den : 1.0f;
    }
    return Q;
}
// the neighbour's sample shifted here: resampling weight, p_hat, q, f (zeros if unusable)
__device__ __forceinline__ float neighbour_weight(const CombineCanon &c, float Mf, const Nbr &nb, float4 Fr, float &pf,
                                                  float &qf, SelF &fj) {
    float wn = 0.0f;
    pf = 0.0f; qf = 0.0f; fj = SelF{false, mk(0.0f, 0.0f, 0.0f)};
    const float pn = nb.p;
    if (nb.valid && nb.length >= 2u && pn > 0.0f && Fr.w > 0.0f) {
        const float2 F = make_float2(luminance(mk(Fr.x, Fr.y, Fr.z)), Fr.w);
        const float cn = (float)nb.C, qn = nb.q, Wn = nb.W;
        const float J = qn / F.y;
        const float pb = pn / J;
        const float den = c.cc * F.x + Mf * cn * pb;
        const float mw = den > 0.0f ? (cn * pb) / den : 0.0f;
        wn = mw * F.x * Wn * J;
        pf = F.x;
        qf = F.y;
        fj = job_f(Fr);
    }
    return wn;
}

// MT = the launch's neighbour count when it is a compile-time constant: every neighbour's
// summary and job results are gathered up front (one memory round trip instead of 2 MT
// dependent ones); MT = 0: any count, gathered per neighbour.
template <uint32_t MT>
__device__ __forceinline__ void combine_pixel(const Scene &sc, const ReuseArgs &A, const WaveBufs &w, uint32_t x,
                                              uint32_t y, uint32_t pix) {
    uint4 *out = A.hist + 8u * (size_t)pix;
    const uint4 *rc = A.cur + 8u * (size_t)pix;
    const uint32_t M = MT ? MT : A.neighbors;
    const uint4 c5 = rc[5], c6 = rc[6], c7 = rc[7];
    const float Mf = (float)M;
    const CombineCanon c{(float)c7.y, asf(c6.x), asf(c6.y), asf(c7.x), c7.y != 0u && c5.w >= 2u && asf(c6.x) > 0.0f};
    const uint32_t seed0 = reuse_seed(sc, x, y, SALT_SPATIAL);
    uint32_t seed = seed0, Csum = c7.y;
    float sumQ = 0.0f, w_sum = 0.0f, p_sel = c.pc, q_sel = c.qc;
    int32_t src = (int32_t)pix;
    SelF f_sel = stored_f(rc);
    if constexpr (MT > 0) {
        int32_t nid[MT];
        bool pres[MT];
#pragma unroll
        for (uint32_t m = 0; m < MT; ++m) {
            uint32_t nx = 0u, ny = 0u;
            pres[m] = spatial_neighbor(seed, A.radius, x, y, sc.width, sc.height, nx, ny);
            nid[m] = pres[m] ? band_index(sc, nx, ny) : (int32_t)pix;
        }
        uint4 nv[MT];
        float4 Fr[MT], B[MT];
#pragma unroll
        for (uint32_t m = 0; m < MT; ++m) {  // (job results of absent neighbours are never used)
            nv[m] = A.nbr[nid[m]];
            Fr[m] = job_at(A, w, pix, 2u * m);
            B[m] = job_at(A, w, pix, 2u * m + 1u);
        }
        Nbr nb[MT];
#pragma unroll
        for (uint32_t m = 0; m < MT; ++m) {
            nb[m] = nv[m].w != kNbrEscape ? nbr_unpack(nv[m]) : nbr_at(A, nid[m]);
            if (!pres[m]) nb[m].valid = false;
        }
#pragma unroll
        for (uint32_t m = 0; m < MT; ++m) {
            float Q = 1.0f;
            if (nb[m].valid) {
                Csum += nb[m].C;
                Q = canon_q(c, Mf, nb[m].C, B[m]);
            }
            sumQ += Q;
        }
        const float wc = c.ok ? (sumQ / Mf) * c.pc * c.Wc : 0.0f;
        if (wrs_update(w_sum, wc, seed)) { src = (int32_t)pix; p_sel = c.pc; q_sel = c.qc; f_sel = stored_f(rc); }
#pragma unroll
        for (uint32_t m = 0; m < MT; ++m) {
            float pf, qf;
            SelF fj;
            const float wn = neighbour_weight(c, Mf, nb[m], Fr[m], pf, qf, fj);
            if (wrs_update(w_sum, wn, seed)) { src = pres[m] ? nid[m] : 0; p_sel = pf; q_sel = qf; f_sel = fj; }
        }
    } else {
        for (uint32_t m = 0; m < M; ++m) {
            uint32_t nx = 0u, ny = 0u;
            float Q = 1.0f;
            if (spatial_neighbor(seed, A.radius, x, y, sc.width, sc.height, nx, ny)) {
                const Nbr nb = nbr_at(A, band_index(sc, nx, ny));
                if (nb.valid) {
                    Csum += nb.C;
                    Q = canon_q(c, Mf, nb.C, job_at(A, w, pix, 2u * m + 1u));
                }
            }
            sumQ += Q;
        }
        const float wc = c.ok ? (sumQ / Mf) * c.pc * c.Wc : 0.0f;
        uint32_t nseed = seed0;
        if (wrs_update(w_sum, wc, seed)) { src = (int32_t)pix; p_sel = c.pc; q_sel = c.qc; f_sel = stored_f(rc); }
        for (uint32_t m = 0; m < M; ++m) {
            uint32_t nx = 0u, ny = 0u;
            float wn = 0.0f, pf = 0.0f, qf = 0.0f;
            SelF fj{false, mk(0.0f, 0.0f, 0.0f)};
            int32_t nidx = 0;
            if (spatial_neighbor(nseed, A.radius, x, y, sc.width, sc.height, nx, ny)) {
                nidx = band_index(sc, nx, ny);
                wn = neighbour_weight(c, Mf, nbr_at(A, nidx), job_at(A, w, pix, 2u * m), pf,
                                      qf, fj);
            }
            if (wrs_update(w_sum, wn, seed)) { src = nidx; p_sel = pf; q_sel = qf; f_sel = fj; }
        }
    }
    write_reused(out, res_at(A.cur, src), p_sel, q_sel, f_sel, w_sum, Csum);
}

// The same combine for M = 3 with four lanes per pixel: lane 0 holds the canonical sample,
// lane 1 + m neighbour m (its offset draws, summary and two job results gathered by that
// lane).  The neighbourhood sums (confidences, the canonical MIS weight sum_n Q_n) and the
// resampling weights' running sum are gathered with __shfl inside the pixel's four lanes and
// added in the sequential order of combine_pixel (((0 + Q_0) + Q_1) + Q_2, w_c first), so the
// floats are the same; each lane then evaluates its own UpdateReservoir draw (draw k of the
// selection stream is seed + 2M + k), the last accepted lane is the selection (ballot), and
// the 128-byte output reservoir is written 32 bytes per lane.  Bit-identical to combine_pixel.
constexpr uint32_t kShflLanes = 4u;  // lanes per pixel (M + 1 with M = 3)
__global__ __launch_bounds__(WB) void wspatial_combine_shfl(Scene sc, WaveBufs w, ReuseArgs A) {
    PTX_WAVE_TIMER(sc, KID_SPAT_COMBINE | (w.seg_base ? 0x80u : 0u));
    constexpr uint32_t M = 3u;
    const uint32_t j = w.seg_base + blockIdx.x, np = padded_pixels(sc);
    const uint32_t lane = __lane_id(), r = lane & 3u, base = lane & ~3u;
    for (uint32_t k = 0; k < w.seg_px; k += WB / kShflLanes) {  // workgroup-uniform
        // pixel k + threadIdx.x / 4 of the segment (seg_pixel's tile layout)
        const uint32_t off = k + (threadIdx.x >> 2), sl = off >> 6;
        const uint32_t q = set_tile(w, ((sl / w.cluster) * w.nseg + j) * w.cluster + sl % w.cluster) * 64u + (off & 63u);
        uint32_t x = 0u, y = 0u;
        const bool inside = q < np && tile_xy(sc, q, x, y);
        const uint32_t pix = inside ? (y - sc.row_begin) * sc.width + x : 0u;
        const bool hit = inside && gdecode(A.gbuf[pix]).valid;
        uint4 c5 = make_uint4(0u, 0u, 0u, 0u), c6 = c5, c7 = c5;
        if (hit) { const uint4 *rc = A.cur + 8u * (size_t)pix; c5 = rc[5]; c6 = rc[6]; c7 = rc[7]; }
        const CombineCanon c{(float)c7.y, asf(c6.x), asf(c6.y), asf(c7.x), c7.y != 0u && c5.w >= 2u && asf(c6.x) > 0.0f};
        const float Mf = (float)M;
        const uint32_t seed0 = hit ? reuse_seed(sc, x, y, SALT_SPATIAL) : 0u;
        // lane 1 + m: neighbour m
        bool pres = false;
        int32_t nid = (int32_t)pix;
        Nbr nb{false, 0u, 0u, 0.0f, 0.0f, 0.0f};
        float4 Fr = make_float4(0.0f, 0.0f, 0.0f, 0.0f), B = Fr;
        if (hit && r > 0u) {
            const uint32_t m = r - 1u;
            uint32_t seed = seed0 + 2u * m, nx = 0u, ny = 0u;
            pres = spatial_neighbor(seed, A.radius, x, y, sc.width, sc.height, nx, ny);
            if (pres) nid = band_index(sc, nx, ny);
            const uint4 nv = A.nbr[nid];
            Fr = job_at(A, w, pix, 2u * m);
            B = job_at(A, w, pix, 2u * m + 1u);
            nb = nv.w != kNbrEscape ? nbr_unpack(nv) : nbr_at(A, nid);
            if (!pres) nb.valid = false;
        }
        const float Q = nb.valid ? canon_q(c, Mf, nb.C, B) : 1.0f;
        const uint32_t Cn = nb.valid ? nb.C : 0u;
        // neighbourhood sums in combine_pixel's order
        const float Q0 = __shfl(Q, base + 1u), Q1 = __shfl(Q, base + 2u), Q2 = __shfl(Q, base + 3u);
        const uint32_t Csum = c7.y + __shfl(Cn, base + 1u) + __shfl(Cn, base + 2u) + __shfl(Cn, base + 3u);
        float sumQ = 0.0f;
        sumQ += Q0;
        sumQ += Q1;
        sumQ += Q2;
        const float wc = c.ok ? (sumQ / Mf) * c.pc * c.Wc : 0.0f;
        float pf = 0.0f, qf = 0.0f;
        SelF fj{false, mk(0.0f, 0.0f, 0.0f)};
        const float wn = r > 0u ? neighbour_weight(c, Mf, nb, Fr, pf, qf, fj) : wc;
        // running sum of the resampling weights (canonical first), this lane's draw
        const float w0 = __shfl(wn, base), w1 = __shfl(wn, base + 1u), w2 = __shfl(wn, base + 2u),
                    w3 = __shfl(wn, base + 3u);
        float w_sum = 0.0f, w_upto = 0.0f;
        w_sum += w0; if (r == 0u) w_upto = w_sum;
        w_sum += w1; if (r == 1u) w_upto = w_sum;
        w_sum += w2; if (r == 2u) w_upto = w_sum;
        w_sum += w3; if (r == 3u) w_upto = w_sum;
        uint32_t dseed = seed0 + 2u * M + r;
        const bool accept = hit && rnd(dseed) < wn / w_upto;
        const uint32_t grp = (uint32_t)(__ballot(accept) >> base) & 0xfu;
        const uint32_t sel = grp ? 31u - (uint32_t)__builtin_clz(grp) : 0u;  // the last accepted lane
        // the selected lane's sample: source reservoir, p_hat, q and stored contribution
        const int32_t src_l = r == 0u ? (int32_t)pix : (pres ? nid : 0);
        const int32_t src = __shfl(src_l, base + sel);
        const float p_sel = sel ? __shfl(pf, base + sel) : c.pc, q_sel = sel ? __shfl(qf, base + sel) : c.qc;
        const float fx = __shfl(fj.f.x, base + sel), fy = __shfl(fj.f.y, base + sel), fz = __shfl(fj.f.z, base + sel);
        const bool fk = __shfl(fj.known ? 1 : 0, base + sel) != 0;
        if (!inside) continue;
        uint4 *out = A.hist + 8u * (size_t)pix;
        if (!hit) {
            out[2u * r] = make_uint4(0u, 0u, 0u, 0u);
            out[2u * r + 1u] = make_uint4(0u, 0u, 0u, 0u);
            continue;
        }
        if (r < 3u) {  // words 8r .. 8r + 7 of the selected sample
            const uint4 *sv = res_at(A.cur, src);
            const uint4 a0 = sv[2u * r], a1 = sv[2u * r + 1u];
            out[2u * r] = a0;
            out[2u * r + 1u] = a1;
        } else {
            const SelF fs = sel ? SelF{fk, mk(fx, fy, fz)} : stored_f(A.cur + 8u * (size_t)pix);
            out[6] = make_uint4(asu(p_sel), asu(q_sel), fs.known ? asu(fs.f.x) : 0u, fs.known ? asu(fs.f.y) : 0u);
            out[7] = make_uint4(asu(p_sel > 0.0f ? w_sum / p_sel : 0.0f), Csum, fs.known ? asu(fs.f.z) : 0u,
                                fs.known ? 1u : 0u);
        }
    }
}

__global__ __launch_bounds__(WB) void wspatial_combine(Scene sc, WaveBufs w, ReuseArgs A) {
    PTX_WAVE_TIMER(sc, KID_SPAT_COMBINE | (w.seg_base ? 0x80u : 0u));
    const uint32_t j = w.seg_base + blockIdx.x, np = padded_pixels(sc);
    for (uint32_t k = 0; k < w.seg_px; k += WB) {
        const uint32_t q = seg_pixel(w, j, k);
        uint32_t x, y;
        if (q >= np || !tile_xy(sc, q, x, y)) continue;
        const uint32_t pix = (y - sc.row_begin) * sc.width + x;
        if (!gdecode(A.gbuf[pix]).valid) {
            uint4 *out = A.hist + 8u * (size_t)pix;
            for (int t = 0; t < 8; ++t) out[t] = make_uint4(0u, 0u, 0u, 0u);
            continue;
        }
        if (A.neighbors == 3u) combine_pixel<3>(sc, A, w, x, y, pix);
        else combine_pixel<0>(sc, A, w, x, y, pix);
    }
}

// ---------------------------------------------------------------- host side
// Logic round 0 creates the jobs, rounds 1..kWaveRoundsReuse step them, the last round
// combines (so round r > 0 consumes trace round r-1).
// temporal from PT_1's state: only env candidates trace (one light ray each)
int reuse_rounds(int pass_temporal, const ReuseArgs &A) {
    return pass_temporal && A.use_init && !A.motion ? 1 : kWaveRoundsReuse;
}

hipError_t wave_reuse_round(const Scene &sc, const WaveBufs &w, int pass_temporal, int round, const ReuseArgs &A,
                            hipStream_t s) {
    const dim3 grid(w.seg_count), blk(WB);
    if (round == 0) {
        if (pass_temporal && A.motion) hipLaunchKernelGGL(wtmotion_start, grid, blk, 0, s, sc, w, A);
        else if (pass_temporal) hipLaunchKernelGGL(wtemporal_start, grid, blk, 0, s, sc, w, A);
        else hipLaunchKernelGGL(wspatial_start, grid, blk, 0, s, sc, w, A);
    } else if (round <= reuse_rounds(pass_temporal, A)) {
        hipLaunchKernelGGL(wjob_step, grid, blk, 0, s, sc, w, (uint32_t)round, A);
    } else {
        if (pass_temporal && A.motion) hipLaunchKernelGGL(wtmotion_combine, grid, blk, 0, s, sc, w, A);
        else if (pass_temporal) hipLaunchKernelGGL(wtemporal_combine, grid, blk, 0, s, sc, w, A);
        else if (A.neighbors == 3u && !ab_knob("COMBINE_SCALAR", 0))  // (A/B switch)
            hipLaunchKernelGGL(wspatial_combine_shfl, dim3(w.seg_count), blk, 0, s, sc, w, A);
        else hipLaunchKernelGGL(wspatial_combine, grid, blk, 0, s, sc, w, A);
    }
    return hipGetLastError();
}

}  // namespace ptx
