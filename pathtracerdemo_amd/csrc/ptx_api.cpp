// ptx_api.cpp -- C-ABI boundary (include/ptx.h) of the MI355X path tracer.
//
// Mirrors the WebGPU host of the reference (apps/frontend/src/graphics-core/
// Renderer_TEST.ts; GC/ below): buffers of CreateGPUResources (:445-460), the uniform
// block of Update (:165-206), the three dispatches of Render (:208-261).  On top of the
// reference arrays it derives the MI355X traversal layout described in ptx_device.h.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <new>
#include <string>
#include <unordered_map>
#include <vector>

#include "ptx_internal.h"

namespace ptx {


// The keys of PTX_AB, and those this build does not honour: the shipped library reads only
// kShippedKnobs (every other switch is compiled to its default, ab_knob in ptx_launch.h), so a
// PTX_AB meant for the measurement build would silently measure the product.  Warned once on
// stderr and listed by ptx_build_info (bench.py puts that in its line).
[[maybe_unused]] static const char *const kShippedKnobs[] = {"COMM_TIMEOUT_S", "DEBUG_FILL", "HALO_PROXY_US"};
#if defined(PTX_WG_TIMES)
static const char *const kBuildKind = "wgt";
#elif defined(PTX_AB_BUILD)
static const char *const kBuildKind = "ab";
#else
static const char *const kBuildKind = "product";
#endif
static std::vector<std::string> ignored_knobs() {
    std::vector<std::string> out;
#ifndef PTX_AB_BUILD
    const char *ab = getenv("PTX_AB");
    for (const char *p = ab ? ab : ""; *p;) {
        const char *end = std::strchr(p, ',');
        if (!end) end = p + std::strlen(p);
        const char *eq = static_cast<const char *>(std::memchr(p, '=', (size_t)(end - p)));
        const std::string key(p, eq ? eq : end);
        bool known = key.empty();
        for (const char *k : kShippedKnobs) known = known || key == k;
        if (!known) out.push_back(key);
        p = *end ? end + 1 : end;
    }
#endif
    return out;
}
static void warn_ignored_knobs() {
    static const bool once = [] {
        for (const std::string &k : ignored_knobs())
            std::fprintf(stderr, "libptx (%s build): PTX_AB key %s is not honoured here -- A/B switches need the "
                                 "measurement build (make -C pathtracerdemo_amd/csrc ab; PTX_LIB_PATH=.../libptx_ab.so)\n",
                         kBuildKind, k.c_str());
        return true;
    }();
    (void)once;
}

int env_knob(const char *key, int dflt) {
    static const std::string ab = getenv("PTX_AB") ? getenv("PTX_AB") : "";
    warn_ignored_knobs();
    const size_t n = std::strlen(key);
    for (size_t pos = 0; pos < ab.size();) {
        size_t end = ab.find(',', pos);
        if (end == std::string::npos) end = ab.size();
        if (end - pos >= n && ab.compare(pos, n, key) == 0 && (end - pos == n || ab[pos + n] == '='))
            return end - pos == n ? 1 : std::atoi(ab.c_str() + pos + n + 1);
        pos = end + 1;
    }
    return dflt;
}

int fail(ptx_handle *h, int code, const char *fmt, ...) {
    if (h) {
        char buf[512];
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(buf, sizeof buf, fmt, ap);
        va_end(ap);
        h->err = buf;
    }
    return code;
}
void free_buf(DevBuf &b) {
    if (b.p) (void)hipFree(b.p);
    b.p = nullptr;
    b.bytes = 0;
}
// Every copy and fill between the host and a handle's buffers runs on the handle's current
// stream and is waited for there.  The handle's streams are non-blocking, so nothing on the
// null stream is ordered before their kernels: a null-stream fill still in flight when a frame
// started once overwrote what the frame wrote (a reuse mismatch seen when another handle kept
// the null stream busy), and a pageable host-to-device hipMemcpy may return before its DMA has
// landed.  On the handle's stream the transfer is ordered after everything enqueued before it,
// and the sync orders it before everything enqueued after.
static hipError_t memset_sync(ptx_handle *h, void *p, int value, size_t bytes) {
    hipError_t e = hipMemsetAsync(p, value, bytes, h->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
    return e;
}
static hipError_t copy_sync(ptx_handle *h, void *dst, const void *src, size_t bytes, hipMemcpyKind kind) {
    hipError_t e = hipMemcpyAsync(dst, src, bytes, kind, h->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
    return e;
}
// Device -> caller memory after everything enqueued on h->stream, through the handle's pinned
// staging buffer in chunks of up to 8 MB: the caller's memory may be any host memory, and
// pageable device-to-host async copies into a V8 ArrayBuffer (the Node host) came back
// incomplete for multi-MB transfers; a pinned destination is a plain DMA.
int read_to_host(ptx_handle *h, void *dst, const void *src, size_t bytes) {
    constexpr size_t kChunk = (size_t)8 << 20;
    const size_t want = std::min(bytes, kChunk);
    if (want > h->host_stage_bytes) {
        if (h->host_stage) (void)hipHostFree(h->host_stage);
        h->host_stage = nullptr;
        h->host_stage_bytes = 0;
        HIP_CHECK(h, hipHostMalloc(&h->host_stage, want, hipHostMallocDefault));
        h->host_stage_bytes = want;
    }
    for (size_t off = 0; off < bytes; off += kChunk) {
        const size_t n = std::min(kChunk, bytes - off);
        HIP_CHECK(h, hipMemcpyAsync(h->host_stage, (const char *)src + off, n, hipMemcpyDeviceToHost, h->stream));
        HIP_CHECK(h, hipStreamSynchronize(h->stream));
        std::memcpy((char *)dst + off, h->host_stage, n);
    }
    return PTX_OK;
}

int alloc_buf(ptx_handle *h, DevBuf &b, size_t bytes) {
    if (b.bytes == bytes && b.p) return PTX_OK;
    free_buf(b);
    if (bytes == 0) return PTX_OK;
    hipError_t e = hipMalloc(&b.p, bytes);
    if (e != hipSuccess) return fail(h, PTX_E_NOMEM, "hipMalloc(%zu): %s", bytes, hipGetErrorString(e));
    b.bytes = bytes;
    // diagnostics: PTX_AB=DEBUG_FILL=<byte> fills every new buffer with that byte (an
    // uninitialised read then shows up as a parity failure)
    static const int fill = env_knob("DEBUG_FILL", -1);
    if (fill >= 0) HIP_CHECK(h, memset_sync(h, b.p, fill & 0xff, bytes));
    return PTX_OK;
}
static int upload(ptx_handle *h, DevBuf &b, const void *src, size_t bytes) {
    int rc = alloc_buf(h, b, std::max<size_t>(bytes, 16));
    if (rc) return rc;
    if (bytes) HIP_CHECK(h, copy_sync(h, b.p, src, bytes, hipMemcpyHostToDevice));
    return PTX_OK;
}

// first band row of the halo-extended G-buffer / reservoir allocations
uint4 *gbuf_band(ptx_handle *h) { return (uint4 *)h->d_gbuf.p + (size_t)h->halo_top * h->cfg.width; }
uint4 *res_band(ptx_handle *h) { return (uint4 *)h->d_res.p + h->res_u4 * (size_t)h->halo_top * h->cfg.width; }
// the history (spatial output) carries the same halo rows: a band's motion halo, received from
// the neighbours before a moved camera's temporal pass (ptx_comm.cpp)
uint4 *hist_band(ptx_handle *h) { return (uint4 *)h->d_hist.p + h->res_u4 * (size_t)h->halo_top * h->cfg.width; }
// pipelines with the build-defined temporal / spatial passes (DI reuse, GI)
bool has_reuse(const ptx_handle *h) {
    return h->cfg.pipeline == PTX_PIPELINE_RESTIR_REUSE || h->cfg.pipeline == PTX_PIPELINE_RESTIR_GI;
}
// ReSTIR without reuse pipelines its frames too: frame N + 1's G-buffer + PT_1 beside frame N's
// PT_4 (C1 1080p, one sequence per context at 768-pixel segments: 1536-1543 Msamples/s against
// 1406-1414 one frame at a time; PTX_AB=PIPE_RESTIR=0: A/B).  Its timed-alone region keeps static
// slots, as its pipelined frames do (use_dyn_batches).
static bool restir_pipe() {
    static const bool on = ab_knob("PIPE_RESTIR", 1) != 0;
    return on;
}
// The DI reuse pipeline's whole-image frames on static trace slots with 2 front sequences per
// context, as ReSTIR's and TEST_MCPT's, instead of dynamic batches with one (PTX_AB=REUSE_STATIC=0:
// A/B); its segments stay seg_pixels' reuse rule (1024 px at 1080p)
static bool reuse_static() {
    static const bool on = ab_knob("REUSE_STATIC", 1) != 0;
    return on;
}
// TEST_MCPT likewise: frame N + 1's paths beside frame N's, each frame's colours mixed into the
// accumulation after the previous frame's (C1 1080p at 1792-pixel segments, 2 sequences per
// context: 1744-1758 Msamples/s against 1509-1515 one frame at a time; PTX_AB=PIPE_MCPT=0: A/B)
static bool mcpt_pipe() {
    static const bool on = ab_knob("PIPE_MCPT", 1) != 0;
    return on;
}

static inline float as_f32(uint32_t u) {
    float f;
    std::memcpy(&f, &u, 4);
    return f;
}

// The instance cull's world box (Inst::wlo / whi / wpad / wscale, inst_may_hit in ptx_device.h):
// the union of the instance's sub-mesh root boxes in local space, mapped to world space through
// the inverse of M^-1 (the matrix the kernels transform rays with; M itself may differ from that
// inverse by rounding) in double precision, its 8 corners' bounds rounded outward to f32.  The
// pad covers the f32 rounding of the kernels' ray transform with >= 40x margin: 1e-5 of the
// local box's and M^-1's translation magnitudes mapped through |A^-1| (A = M^-1's linear part),
// and per ray 1e-5 * cond(A) * max|o| (wscale).  Never culled (wpad = -1): a projective or
// singular M^-1, non-finite values, an instance without sub-meshes.
static void inst_world_box(Inst &I, const SubRoot *roots, uint32_t nsub) {
    I.wpad = -1.0f;
    I.wscale = 0.0f;
    for (int k = 0; k < 3; ++k) I.wlo[k] = I.whi[k] = 0.0f;
    const float *m = I.minv;  // column-major: local = A * world + t
    if (nsub == 0 || m[3] != 0.0f || m[7] != 0.0f || m[11] != 0.0f || m[15] != 1.0f) return;
    double A[3][3], t[3];
    for (int r = 0; r < 3; ++r) {
        for (int c = 0; c < 3; ++c) A[r][c] = m[4 * c + r];
        t[r] = m[12 + r];
    }
    const double det = A[0][0] * (A[1][1] * A[2][2] - A[1][2] * A[2][1]) - A[0][1] * (A[1][0] * A[2][2] - A[1][2] * A[2][0]) +
                       A[0][2] * (A[1][0] * A[2][1] - A[1][1] * A[2][0]);
    if (!std::isfinite(det) || std::fabs(det) < 1e-30) return;
    double B[3][3];  // A^-1
    B[0][0] = (A[1][1] * A[2][2] - A[1][2] * A[2][1]) / det;
    B[0][1] = (A[0][2] * A[2][1] - A[0][1] * A[2][2]) / det;
    B[0][2] = (A[0][1] * A[1][2] - A[0][2] * A[1][1]) / det;
    B[1][0] = (A[1][2] * A[2][0] - A[1][0] * A[2][2]) / det;
    B[1][1] = (A[0][0] * A[2][2] - A[0][2] * A[2][0]) / det;
    B[1][2] = (A[0][2] * A[1][0] - A[0][0] * A[1][2]) / det;
    B[2][0] = (A[1][0] * A[2][1] - A[1][1] * A[2][0]) / det;
    B[2][1] = (A[0][1] * A[2][0] - A[0][0] * A[2][1]) / det;
    B[2][2] = (A[0][0] * A[1][1] - A[0][1] * A[1][0]) / det;
    double lo[3], hi[3];
    for (int k = 0; k < 3; ++k) { lo[k] = HUGE_VAL; hi[k] = -HUGE_VAL; }
    for (uint32_t s = 0; s < nsub; ++s) {
        const float *ax[3] = {roots[s].x, roots[s].y, roots[s].z};
        for (int k = 0; k < 3; ++k) { lo[k] = std::min(lo[k], (double)ax[k][0]); hi[k] = std::max(hi[k], (double)ax[k][1]); }
    }
    double lmax = 0.0, tmax = 0.0, na = 0.0, nb = 0.0;  // magnitudes, |A|inf, |A^-1|inf
    for (int k = 0; k < 3; ++k) {
        if (!std::isfinite(lo[k]) || !std::isfinite(hi[k]) || lo[k] > hi[k]) return;
        lmax = std::max({lmax, std::fabs(lo[k]), std::fabs(hi[k])});
        tmax = std::max(tmax, std::fabs(t[k]));
        na = std::max(na, std::fabs(A[k][0]) + std::fabs(A[k][1]) + std::fabs(A[k][2]));
        nb = std::max(nb, std::fabs(B[k][0]) + std::fabs(B[k][1]) + std::fabs(B[k][2]));
    }
    double wlo[3] = {HUGE_VAL, HUGE_VAL, HUGE_VAL}, whi[3] = {-HUGE_VAL, -HUGE_VAL, -HUGE_VAL}, wmax = 0.0;
    for (int c = 0; c < 8; ++c) {
        const double p[3] = {(c & 1) ? hi[0] : lo[0], (c & 2) ? hi[1] : lo[1], (c & 4) ? hi[2] : lo[2]};
        for (int r = 0; r < 3; ++r) {
            const double w = B[r][0] * (p[0] - t[0]) + B[r][1] * (p[1] - t[1]) + B[r][2] * (p[2] - t[2]);
            wlo[r] = std::min(wlo[r], w);
            whi[r] = std::max(whi[r], w);
            wmax = std::max(wmax, std::fabs(w));
        }
    }
    const double pad = 1e-5 * (1.0 + wmax) + 1e-5 * nb * (lmax + tmax);
    const double scale = 1e-5 * std::max(1.0, na * nb);
    if (!std::isfinite(pad) || !std::isfinite(scale) || !std::isfinite(wmax)) return;
    for (int k = 0; k < 3; ++k) {
        I.wlo[k] = std::nextafter((float)wlo[k], -HUGE_VALF);
        I.whi[k] = std::nextafter((float)whi[k], HUGE_VALF);
    }
    I.wpad = std::nextafter((float)pad, HUGE_VALF);
    I.wscale = std::nextafter((float)scale, HUGE_VALF);
}

// ---------------------------------------------------------------- layout derivation
// Walks the reference's per-sub-mesh BLAS (three-mesh-bvh node format, GC/Structs.ts:73-80;
// read by GetBlasNode, SH/PT_01_GBufferPass.wgsl:310-322) and emits the child-pair node
// records, the edge-form triangle table and the instance table of ptx_device.h.
int build_layout(ptx_handle *h) {
    // frames in flight (either pipelined context) still read the layout being replaced
    if (int rc = quiesce(h)) return rc;
    const uint32_t *U = h->uniform;
    const auto &S = h->scene, &G = h->geometry, &A = h->accel;
    const uint32_t off_desc = U[U_OFF_DESC], off_mat = U[U_OFF_MAT], off_index = U[U_OFF_INDEX];
    const uint32_t off_subroot = U[U_OFF_SUBROOT], off_blas = U[U_OFF_BLAS], n_inst = U[U_INST_COUNT];
    if (off_mat < off_desc || (off_mat - off_desc) % STRIDE_DESCRIPTOR)
        return fail(h, PTX_E_SCENE, "uniform offsets: descriptor block [%u,%u) is not a multiple of 6", off_desc, off_mat);
    const uint32_t n_mesh = (off_mat - off_desc) / STRIDE_DESCRIPTOR;
    if ((size_t)n_inst * STRIDE_INSTANCE > off_desc)
        return fail(h, PTX_E_SCENE, "instance count %u overlaps the descriptor block", n_inst);
    if (off_desc + (size_t)n_mesh * STRIDE_DESCRIPTOR > S.size()) return fail(h, PTX_E_SCENE, "scene buffer too short");

    std::vector<SubRoot> subs;
    std::vector<NodePair> nodes;
    std::vector<float> tris;  // 12 floats per triangle
    std::vector<float> mats;  // 8 floats per sub-mesh, in SubRoot order (Scene::mats)
    std::vector<float> tverts;  // 20 floats per triangle, triangle-table order (Scene::tverts)
    std::vector<uint32_t> mesh_sub_base(n_mesh), mesh_nsub(n_mesh), mesh_tri_base(n_mesh);
    uint32_t max_depth = 0;

    for (uint32_t m = 0; m < n_mesh; ++m) {
        const uint32_t *d = S.data() + off_desc + STRIDE_DESCRIPTOR * m;
        const uint32_t off_vertex = d[0], off_idx = d[1], off_root = d[3], off_b = d[4], nsub = d[5];
        mesh_sub_base[m] = (uint32_t)subs.size();
        mesh_nsub[m] = nsub;
        mesh_tri_base[m] = (uint32_t)(tris.size() / 12);
        // GetMaterial (SH/PT_1_InitPass.wgsl:285-314) per sub-mesh: material d[2] + 15*sub.  A record
        // past the scene buffer reads as zeros (WebGPU's robust buffer access would clamp or zero).
        for (uint32_t s = 0; s < nsub; ++s) {
            const size_t mi = (size_t)off_mat + d[2] + (size_t)STRIDE_MATERIAL * s;
            auto word = [&](uint32_t k) { return mi + k < S.size() ? as_f32(S[mi + k]) : 0.0f; };
            const float trans = word(10);
            const bool yellow = trans > 0.0f;
            const float rec[8] = {yellow ? 1.0f : word(0), yellow ? 1.0f : word(1), yellow ? 0.0f : word(2), word(8),
                                  std::fmax(word(9), 0.01f), trans, word(11), 0.0f};
            mats.insert(mats.end(), rec, rec + 8);
        }
        uint32_t mesh_tris = 0;
        struct Pending { uint32_t base; std::vector<uint32_t> order; };
        std::vector<Pending> per_sub;
        for (uint32_t s = 0; s < nsub; ++s) {
            size_t ri = (size_t)off_subroot + off_root + s;
            if (ri >= G.size()) return fail(h, PTX_E_SCENE, "sub-BLAS root index out of range");
            const uint32_t base = off_blas + off_b + G[ri];
            // DFS over the sub-BVH to number interior nodes
            std::unordered_map<uint32_t, uint32_t> gidx;
            std::vector<std::pair<uint32_t, uint32_t>> st{{0u, 0u}};
            std::vector<uint32_t> interior;
            while (!st.empty()) {
                auto [n, depth] = st.back();
                st.pop_back();
                size_t w = (size_t)base + 8u * n;
                if (w + 8 > A.size()) return fail(h, PTX_E_SCENE, "BLAS node %u out of range", n);
                max_depth = std::max(max_depth, depth);
                if (A[w + 7] & 0xffff0000u) {
                    uint32_t first = A[w + 6], count = A[w + 7] & 0xffffu;
                    mesh_tris = std::max(mesh_tris, first + count);
                    continue;
                }
                gidx[n] = (uint32_t)(nodes.size() + interior.size());
                interior.push_back(n);
                st.push_back({n + 1u, depth + 1});
                st.push_back({A[w + 6] / 8u, depth + 1});
                if (depth > 1000) return fail(h, PTX_E_SCENE, "BLAS too deep / cyclic");
            }
            auto ref_of = [&](uint32_t n, uint32_t &ref) -> int {
                size_t w = (size_t)base + 8u * n;
                if (A[w + 7] & 0xffff0000u) {
                    uint32_t first = A[w + 6], count = A[w + 7] & 0xffffu;
                    if (count >= 128u || first > LEAF_FIRST_MASK)
                        return fail(h, PTX_E_SCENE, "leaf (first %u, count %u) exceeds the packed ref", first, count);
                    ref = LEAF_BIT | (count << 24) | first;
                } else {
                    ref = gidx.at(n);
                }
                return PTX_OK;
            };
            SubRoot r{};
            float *axis[3] = {r.x, r.y, r.z};
            for (int k = 0; k < 3; ++k) { axis[k][0] = as_f32(A[base + k]); axis[k][1] = as_f32(A[base + 3 + k]); }
            if (int rc = ref_of(0u, r.ref)) return rc;
            subs.push_back(r);
            for (uint32_t n : interior) {
                size_t w = (size_t)base + 8u * n;
                uint32_t L = n + 1u, R = A[w + 6] / 8u;
                size_t wl = (size_t)base + 8u * L, wr = (size_t)base + 8u * R;
                NodePair np{};
                float *naxis[3] = {np.x, np.y, np.z};
                for (int k = 0; k < 3; ++k) {
                    naxis[k][0] = as_f32(A[wl + k]); naxis[k][1] = as_f32(A[wr + k]);
                    naxis[k][2] = as_f32(A[wl + 3 + k]); naxis[k][3] = as_f32(A[wr + 3 + k]);
                }
                if (int rc = ref_of(L, np.lref)) return rc;
                if (int rc = ref_of(R, np.rref)) return rc;
                nodes.push_back(np);
            }
        }
        // edge-form triangles in index (leaf) order, local space
        for (uint32_t prim = 0; prim < mesh_tris; ++prim) {
            size_t ii = (size_t)off_index + off_idx + 3u * prim;
            if (ii + 3 > G.size()) return fail(h, PTX_E_SCENE, "index buffer out of range");
            float P[3][3];
            for (int v = 0; v < 3; ++v) {
                size_t vi = (size_t)off_vertex + STRIDE_VERTEX * G[ii + v];
                if (vi + 3 > G.size()) return fail(h, PTX_E_SCENE, "vertex out of range");
                for (int k = 0; k < 3; ++k) P[v][k] = as_f32(G[vi + k]);
            }
            const float e1[3] = {P[1][0] - P[0][0], P[1][1] - P[0][1], P[1][2] - P[0][2]};
            const float e2[3] = {P[2][0] - P[0][0], P[2][1] - P[0][1], P[2][2] - P[0][2]};
            const float rec[12] = {P[0][0], P[0][1], P[0][2], e1[0], e1[1], e1[2], e2[0], e2[1], e2[2], 0, 0, 0};
            tris.insert(tris.end(), rec, rec + 12);
            float N[3][3];
            for (int v = 0; v < 3; ++v) {
                const size_t vi = (size_t)off_vertex + STRIDE_VERTEX * G[ii + v];
                if (vi + 6 > G.size()) return fail(h, PTX_E_SCENE, "vertex normal out of range");
                for (int k = 0; k < 3; ++k) N[v][k] = as_f32(G[vi + 3 + k]);
            }
            const float tv[20] = {P[0][0], P[0][1], P[0][2], N[0][0], N[0][1], N[0][2], P[1][0], P[1][1], P[1][2], N[1][0],
                                  N[1][1], N[1][2], P[2][0], P[2][1], P[2][2], N[2][0], N[2][1], N[2][2], 0.0f, 0.0f};
            tverts.insert(tverts.end(), tv, tv + 20);
        }
    }
    std::vector<Inst> insts(n_inst);
    for (uint32_t i = 0; i < n_inst; ++i) {
        const uint32_t *p = S.data() + STRIDE_INSTANCE * i;
        Inst &I = insts[i];
        std::memcpy(I.m, p, 64);
        std::memcpy(I.minv, p + 16, 64);
        I.mesh = p[32];
        if (I.mesh >= n_mesh) return fail(h, PTX_E_SCENE, "instance %u references mesh %u of %u", i, I.mesh, n_mesh);
        I.sub_base = mesh_sub_base[I.mesh];
        I.nsub = mesh_nsub[I.mesh];
        I.tri_base = mesh_tri_base[I.mesh];
        // exactly the identity (bitwise 1 / +0, M and M^-1): the kernels' transforms of this
        // instance reduce to x + 0 (inst_point, ptx_device.h) with the same bits
        static const float kId[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
        if (!std::memcmp(I.m, kId, sizeof kId) && !std::memcmp(I.minv, kId, sizeof kId)) I.mesh |= kInstIdentity;
        inst_world_box(I, subs.data() + I.sub_base, I.nsub);
    }
    if (tris.empty()) tris.resize(12, 0.0f);
    if (tverts.empty()) tverts.resize(20, 0.0f);
    if (nodes.empty()) nodes.resize(1);
    if (subs.empty()) subs.resize(1);
    if (mats.empty()) mats.resize(8, 0.0f);
    // each root record carries its sub-mesh's transmission (the Visibility restart test reads
    // it from the trace kernel's LDS root table: subs_transmission)
    if (mats.size() != 8u * subs.size()) return fail(h, PTX_E_SCENE, "material / sub-mesh tables disagree");
    for (size_t k = 0; k < subs.size(); ++k) std::memcpy(&subs[k].pad, &mats[8u * k + 5u], 4);
    if (int rc = upload(h, h->d_tris, tris.data(), tris.size() * sizeof(float))) return rc;
    if (int rc = upload(h, h->d_nodes, nodes.data(), nodes.size() * sizeof(NodePair))) return rc;
    if (int rc = upload(h, h->d_subs, subs.data(), subs.size() * sizeof(SubRoot))) return rc;
    h->n_subs = (uint32_t)subs.size();
    if (int rc = upload(h, h->d_insts, insts.data(), std::max<size_t>(1, insts.size()) * sizeof(Inst))) return rc;
    if (int rc = upload(h, h->d_mats, mats.data(), mats.size() * sizeof(float))) return rc;
    if (int rc = upload(h, h->d_tverts, tverts.data(), tverts.size() * sizeof(float))) return rc;
    h->n_tris = (uint32_t)(tris.size() / 12);
    h->n_nodes = (uint32_t)nodes.size();
    h->n_inst = n_inst;
    h->max_depth = max_depth;
    h->stack_depth = max_depth + 2u;
    if ((size_t)h->stack_depth * kBlock * 4u > 160u * 1024u)
        return fail(h, PTX_E_SCENE, "BLAS depth %u needs more LDS than a CU has", max_depth);
    h->layout_valid = true;
    h->surf_valid = h->alt.surf_valid = h->alt2.surf_valid = false;  // the surface records name the old layout's materials
    return PTX_OK;
}

Scene make_scene(ptx_handle *h) {
    Scene sc{};
    std::memcpy(sc.U, h->uniform, sizeof sc.U);
    sc.S = (const uint32_t *)h->d_scene.p;
    sc.G = (const uint32_t *)h->d_geometry.p;
    sc.tris = (const float4 *)h->d_tris.p;
    sc.nodes = (const NodePair *)h->d_nodes.p;
    sc.subs = (const SubRoot *)h->d_subs.p;
    sc.insts = (const Inst *)h->d_insts.p;
    sc.mats = (const float4 *)h->d_mats.p;
    sc.tverts = (const float4 *)h->d_tverts.p;
    sc.n_inst = h->n_inst;
    sc.n_subs = h->n_subs;
    sc.width = h->cfg.width;
    sc.height = h->cfg.height;
    sc.row_begin = h->cfg.row_begin;
    sc.row_end = h->cfg.row_end;
    sc.counters = (h->cfg.flags & PTX_FLAG_COUNT_WORK) ? (unsigned long long *)h->d_counters.p : nullptr;
    sc.census = (h->cfg.flags & PTX_FLAG_ROW_CENSUS) ? (unsigned long long *)h->d_census.p : nullptr;
#ifdef PTX_WG_TIMES
    sc.wgt = (unsigned long long *)h->d_wgt.p;
#endif
    return sc;
}

void resolve_event(TimedLaunch &t, ptx_handle *h) {
    if (!t.pending) return;
    float ms = 0.0f;
    if (hipEventSynchronize(t.stop) == hipSuccess && hipEventElapsedTime(&ms, t.start, t.stop) == hipSuccess) {
        h->ms_total[t.pass] += ms;
        h->launches[t.pass] += 1;
    }
    t.pending = false;
}

// Padded pixels per wavefront segment.  Measured round 3 (same box, 1080p, flattened instance
// loop + fresh shift jobs): the reuse pipeline +1.5 % at 1024 (768: 378.1, 1024: 383.7, 1536:
// 372.0, 2048: 369.3 Msamples/s; 4K ±0); GI -2.5 %, TEST_MCPT -4.4 %, ReSTIR -1.7 % at 1024, so
// they keep kWaveSegPixels.  PTX_AB=SEG_PX=n: A/B.
// The reuse pipeline's segment grows with the band: ~1500-3000 segments per frame (the largest
// power of two from 512 to 4096 with >= 1500 segments), measured late in round 3 with the 5-wave
// trace (tools/cl/seg_sweep2.sh, seg_sweep3.sh): 1 Mpx bands (configs[3] over 8 GPUs, each band
// alone) 512 px: summed band time 19.6 vs 21.3 ms at 1024; 1080p 1024 px (466.4 vs 443.7 at 512,
// 456.7 at 1536); ~4 Mpx bands (2 GPUs) 2048: 8.15 vs 8.35 ms; the 3840x2160 frame on one GPU
// 4096: 519.1 / 524.6 vs 505.1 / 504.9 at 1024 (2048: 513.4 / 518.5).
static uint32_t seg_pixels(const ptx_handle *h) {
    static const uint32_t env_px = (uint32_t)ab_knob("SEG_PX", 0);
    if (env_px >= 256u && env_px <= 8192u && env_px % 256u == 0u) return env_px;
    const size_t npx = (size_t)h->band_h * h->cfg.width;
    if ((h->cfg.pipeline == PTX_PIPELINE_RESTIR && restir_pipe()) || (h->cfg.pipeline == PTX_PIPELINE_MCPT && mcpt_pipe()) ||
        h->cfg.pipeline == PTX_PIPELINE_RESTIR_GI) {
        // ReSTIR, TEST_MCPT and GI: ~1150 segments (1792 px at 1080p), 768 below 1 Mpx; the
        // pipelined frames and the same segments timed alone.  C1 1080p, static trace slots (one
        // workgroup per segment), 2 sequences per context -- ReSTIR: 1536 / 1792 / 2048 / 2560 px
        // 1695 / 1717 / 1703 / 1697 Msamples/s, the trace launches 0.538 / 0.563 / 0.550 / 0.531
        // of the roofline (tools/cl/r5_piperestir5.sh); TEST_MCPT: 1024 / 1792 px 1715-1722 /
        // 1744-1758, 0.88 / 0.92 (r5_pipemcpt2.sh).  GI C3 1080p: 768 / 1280 / 1536 / 1792 / 2048 px
        // 1033-1043 / 1052-1060 / 1061-1076 / 1078-1083 / 1059-1061 (r5_segall.sh, r5_giseg.sh)
        const size_t p = (npx / 1152u + 128u) / 256u * 256u;
        return (uint32_t)std::min<size_t>(4096u, std::max<size_t>(kWaveSegPixels, p));
    }
    if (h->cfg.pipeline != PTX_PIPELINE_RESTIR_REUSE) return kWaveSegPixels;
    // DI reuse (whole image and bands): 512 px at 1 Mpx .. 4096 at 8.3 Mpx.  Its whole-image frames
    // on static slots measured 1024 / 1280 / 1536 / 1792 px at 1080p: still 516.7 / 499-502 /
    // 511-512 / 515 Msamples/s (trace frac 0.627 / 0.60 / 0.62 / 0.663), moving camera 355.5-355.7
    // / 340-342 / 343-344 / 342-343 (tools/cl/r5_cam4.sh): 1024 keeps both frames fastest
    uint32_t p = 512u;
    while (p < 4096u && (size_t)(2u * p) * 1500u <= npx) p *= 2u;
    return p;
}

// shift jobs per pixel the DI reuse passes may hold at once: the spatial pass's 2M, the motion
// temporal pass's kMotionJobs
static size_t reuse_jobs_per_px(const ptx_handle *h) { return std::max<size_t>(2u * h->reuse_neighbors, kMotionJobs); }
// Wavefront buffers, sized for the largest round: PT_1 emits <= 2 rays per pixel, PT_4
// <= 1, TEST_MCPT <= LightCount + 1 (all shadow rays of a vertex + the next path ray).
int wave_buffers(ptx_handle *h, WaveBufs &w) {
    const size_t npix = (size_t)h->band_h * h->cfg.width;
    const uint32_t nl = h->uniform[U_LIGHT_COUNT];
    const size_t jpp = !has_reuse(h) ? 1u : h->cfg.pipeline == PTX_PIPELINE_RESTIR_GI ? 2u * h->reuse_neighbors
                                                                                         : reuse_jobs_per_px(h);
    const size_t per_px = std::max<size_t>(std::max<size_t>(2u, (size_t)nl + 1u), jpp);
    const size_t padded = (size_t)((h->cfg.width + 7u) / 8u) * ((h->band_h + 7u) / 8u) * 64u;
    const uint32_t seg_px = seg_pixels(h);
    const size_t nseg = (padded + seg_px - 1u) / seg_px;
    // queue slots: the whole band, or two tile sets in flight at once (interior + edge rows of
    // a band's spatial pass: ceil(a/s) + ceil(b/s) <= ceil((a+b)/s) + 1)
    const size_t slots = nseg + 1u;
    const size_t cap = per_px * seg_px * slots;
    // (sized by the segment size: re-checked every call, alloc_buf keeps a buffer of the right size)
    const size_t state_b = (size_t)kWaveStateSlots * npix * 16u, act_b = slots * seg_px * jpp * 4u;
    // counts per round and slot, then the dynamic-batch counters of trace_queue: one per
    // (tile set, launch sequence, round) -- kDynCounters words
    const size_t ctr_b = (2u * kWaveMaxRounds * slots + kDynCounters) * 4u;
    const bool resize = (h->d_wstate.p && h->d_wstate.bytes != state_b) || (h->d_wact0.p && h->d_wact0.bytes != act_b) ||
                        (h->d_wact1.p && h->d_wact1.bytes != act_b) || (h->d_wctr.p && h->d_wctr.bytes != ctr_b) ||
                        (h->wave_ray_cap && cap > h->wave_ray_cap);
    // a buffer is only replaced when its size changes; the other frame context (and this one's
    // last frame) may still run on it, so everything in flight finishes first
    if (resize)
        if (int rc = quiesce(h)) return rc;
    if (int rc = alloc_buf(h, h->d_wstate, state_b)) return rc;
    if (int rc = alloc_buf(h, h->d_wact0, act_b)) return rc;
    if (int rc = alloc_buf(h, h->d_wact1, act_b)) return rc;
    const void *ctr_before = h->d_wctr.p;
    if (int rc = alloc_buf(h, h->d_wctr, ctr_b)) return rc;
    // a new counter buffer starts from zero (the dynamic-batch heads count from it)
    if (h->d_wctr.p != ctr_before) HIP_CHECK(h, memset_sync(h, h->d_wctr.p, 0, h->d_wctr.bytes));
    if (cap > h->wave_ray_cap) {
        free_buf(h->d_wrays);
        free_buf(h->d_wres0);
        free_buf(h->d_wres1);
        free_buf(h->d_wres2);
        h->wave_ray_cap = 0;
        if (int rc = alloc_buf(h, h->d_wrays, cap * 32u)) return rc;
        if (int rc = alloc_buf(h, h->d_wres0, cap * 32u)) return rc;
        if (int rc = alloc_buf(h, h->d_wres1, cap * 32u)) return rc;
        // the spatial reuse pass keeps one result buffer per trace round (ReuseArgs::fold_last)
        if (h->cfg.pipeline == PTX_PIPELINE_RESTIR_REUSE)
            if (int rc = alloc_buf(h, h->d_wres2, cap * 32u)) return rc;
        h->wave_ray_cap = cap;
    }
    w.surf = nullptr;
    if (h->cfg.pipeline == PTX_PIPELINE_RESTIR_REUSE) {
        const size_t rows = (size_t)h->halo_top + h->band_h + h->halo_bot;
        if (h->d_surf.bytes != rows * h->cfg.width * 32u) h->surf_valid = false;
        if (int rc = alloc_buf(h, h->d_surf, rows * h->cfg.width * 32u)) return rc;
        w.surf = (uint4 *)h->d_surf.p + 2u * (size_t)h->halo_top * h->cfg.width;
    }
    w.state = (float4 *)h->d_wstate.p;
    w.npix = (uint32_t)npix;
    w.seg_px = seg_px;
    w.nseg = (uint32_t)nseg;
    w.ray_stride = (uint32_t)(per_px * seg_px);
    w.rays = (float4 *)h->d_wrays.p;
    w.res[0] = (float4 *)h->d_wres0.p;
    w.res[1] = (float4 *)h->d_wres1.p;
    w.res[2] = (float4 *)h->d_wres2.p;
    w.nres = 2;
    w.act[0] = (uint32_t *)h->d_wact0.p;
    w.act[1] = (uint32_t *)h->d_wact1.p;
    // one stride for every pass: passes of different kinds run concurrently on the two
    // streams (e.g. one half's spatial pass beside the other half's PT_4)
    w.act_stride = (uint32_t)(seg_px * jpp);
    w.cnt = (uint32_t *)h->d_wctr.p;
    // measured (with the flat node loop): 4 waves per SIMD (no spill) for every
    // pipeline at 1080p (GI 720 vs 714 Msamples/s at 5), 5 for bands of more than 4 Mpx (a
    // 3840x2160 frame on one GPU: 414.6 vs 413.9 Msamples/s, trace roofline 0.611 vs 0.597)
    w.trace_waves = npix > ((size_t)4u << 20) ? 5u : 4u;
    static const uint32_t env_split = (uint32_t)ab_knob("TRACE_SPLIT", 0);
    w.trace_split = env_split >= 1u && env_split <= 16u ? env_split : 1u;
    w.seg_base = 0;
    w.seg_count = w.nseg;
    static const uint32_t cl = (uint32_t)ab_knob("SEG_CLUSTER", 1);  // A/B
    w.cluster = (cl == 2u || cl == 4u || cl == 8u || cl == 16u) ? cl : 1u;
    // row census: a segment is seg_px / 64 tiles adjacent in raster order, so its queue
    // slot's work belongs to one tile row (two where a tile row's width is not a multiple)
    if (h->cfg.flags & PTX_FLAG_ROW_CENSUS) w.cluster = seg_px / 64u;
    w.tile0 = 0;
    w.ntile0 = (uint32_t)(padded / 64u);
    w.tile1 = w.ntile1 = 0;
    w.seg_phys = 0;
    w.cnt_stride = (uint32_t)slots;
    w.dyn = nullptr;  // set per launch sequence (launch_wave_parts)
    h->wave_slots = (uint32_t)slots;
    return PTX_OK;
}

// One secondary pass as a fixed sequence of wavefront rounds (no host sync inside).
// Event pair around one launch, accounted to stats slot `slot` (resolved lazily).
static TimedLaunch *event_begin(ptx_handle *h, int slot, hipStream_t st) {
    if (!(h->cfg.flags & PTX_FLAG_TIME_LAUNCHES)) return nullptr;  // events cost ~5% of a frame
    TimedLaunch &t = h->ring[h->ring_pos];
    h->ring_pos = (h->ring_pos + 1) % kEventRing;
    resolve_event(t, h);
    if (hipEventRecord(t.start, st) != hipSuccess) return nullptr;
    t.pass = slot;
    return &t;
}
static void event_end(TimedLaunch *t, hipStream_t st) {
    if (t && hipEventRecord(t->stop, st) == hipSuccess) t->pending = true;
}

static size_t px_with_halo(const ptx_handle *h) {
    return (size_t)(h->halo_top + h->band_h + h->halo_bot) * h->cfg.width;
}
// GI job words per pixel: the spatial pass's 2 per neighbour, the motion pass's kGiMotionSlots
static uint32_t gi_job_slots(const ptx_handle *h) { return std::max(2u * h->reuse_neighbors, kGiMotionSlots); }
int reuse_buffers(ptx_handle *h) {
    const size_t njobs = (size_t)h->band_h * h->cfg.width *
                         (h->cfg.pipeline == PTX_PIPELINE_RESTIR_GI ? gi_job_slots(h) : reuse_jobs_per_px(h));
    if (h->cfg.pipeline == PTX_PIPELINE_RESTIR_GI) return alloc_buf(h, h->d_jres, njobs * 4u);  // ray index per job
    if (int rc = alloc_buf(h, h->d_jstate, njobs * 6u * 16u)) return rc;
    if (int rc = alloc_buf(h, h->d_nbr, px_with_halo(h) * 16u)) return rc;
    // per frame context: the temporal pass's jobs (one per pixel; the motion pass's kMotionJobs)
    const size_t npix = (size_t)h->band_h * h->cfg.width;
    if (int rc = alloc_buf(h, h->d_tjstate, npix * kMotionJobs * 6u * 16u)) return rc;
    if (int rc = alloc_buf(h, h->d_tjres, npix * kMotionJobs * 16u)) return rc;
    return alloc_buf(h, h->d_jres, njobs * 16u);
}
static ReuseArgs reuse_args(ptx_handle *h, int pass) {
    ReuseArgs A{};
    A.gbuf = gbuf_band(h);
    A.cur = res_band(h);
    A.hist = hist_band(h);
    const bool temporal = pass == PTX_PASS_TEMPORAL;
    A.jstate = (float4 *)(temporal ? h->d_tjstate.p : h->d_jstate.p);
    A.jres = (float4 *)(temporal ? h->d_tjres.p : h->d_jres.p);
    A.jpp = temporal ? 1u : 2u * h->reuse_neighbors;
    A.njobs = h->band_h * h->cfg.width * A.jpp;
    static const bool planes = ab_knob("JOB_PLANES", 1) != 0;  // A/B: 0 = pixel-major job ids
    A.jpx = planes ? 1u : A.jpp;
    A.jslot = planes ? h->band_h * h->cfg.width : 1u;
    A.radius = h->reuse_radius;
    A.neighbors = h->reuse_neighbors;
    A.cap = h->temporal_cap;
    // (a moved camera's history is only usable through the motion pass: motion_args)
    A.hist_valid = h->hist_valid && !h->hist_moved ? 1u : 0u;
    A.use_init = (pass == PTX_PASS_TEMPORAL && h->init_state_valid) ? 1u : 0u;
    A.nbr_out = (uint4 *)h->d_nbr.p + (size_t)h->halo_top * h->cfg.width;
    A.nbr = A.nbr_out;
    A.surf = h->d_surf.p ? (const uint4 *)h->d_surf.p + 2u * (size_t)h->halo_top * h->cfg.width : nullptr;
    static const bool fold_off = ab_knob("FOLD_LAST_STEP", 1) == 0;  // A/B
    A.fold_last = ((pass == PTX_PASS_SPATIAL || pass == PTX_PASS_TEMPORAL) && !fold_off) ? 1u : 0u;
    A.ray_cap = (uint32_t)std::min<size_t>(h->wave_ray_cap, 0xffffffffu);
    return A;
}

// The motion temporal pass (wtmotion_*): the frame context's temporal job buffers (three job
// planes), the history reprojected through the previous frame's camera.
void mat4_inverse(const float *mf, float *out);
static ReuseArgs motion_args(ptx_handle *h) {
    ReuseArgs A = reuse_args(h, PTX_PASS_SPATIAL);
    A.jstate = (float4 *)h->d_tjstate.p;
    A.jres = (float4 *)h->d_tjres.p;
    A.jpp = kMotionJobs;
    A.njobs = h->band_h * h->cfg.width * A.jpp;
    static const bool planes = ab_knob("JOB_PLANES", 1) != 0;
    A.jpx = planes ? 1u : A.jpp;
    A.jslot = planes ? h->band_h * h->cfg.width : 1u;
    A.hist_valid = h->hist_valid ? 1u : 0u;
    A.use_init = h->init_state_valid ? 1u : 0u;
    // light segments finished by the combine, as in the still passes (PTX_AB=FOLD_LAST_STEP=0: off)
    static const bool fold_on = ab_knob("FOLD_LAST_STEP", 1) != 0;
    A.fold_last = fold_on ? 1u : 0u;
    A.motion = 1u;
    std::memcpy(A.vpinv_prev, h->hist_camera, sizeof A.vpinv_prev);  // (words 4..19 of that frame)
    mat4_inverse(A.vpinv_prev, A.vp_prev);
    const size_t W = h->cfg.width;
    A.psurf = (const uint4 *)h->d_psurf.p + 2u * (size_t)h->halo_top * W;
    // the previous frame's rows held here: the band and its halo rows (the neighbours' surface
    // records from that frame's exchange, their spatial output from this frame's motion halo)
    A.prev_row_lo = -(int32_t)h->halo_top;
    A.prev_row_hi = (int32_t)(h->band_h + h->halo_bot);
    A.clip = (unsigned long long *)h->d_counters.p + CNT_MOTION_CLIP;
    return A;
}

static GiArgs gi_args(ptx_handle *h, bool motion) {
    GiArgs A{};
    A.gbuf = gbuf_band(h);
    A.cur = res_band(h);
    A.hist = hist_band(h);
    A.direct = (float4 *)h->d_direct.p;
    A.accum = (float4 *)h->d_accum.p;
    A.jray = (uint32_t *)h->d_jres.p;
    A.jpp = 2u * h->reuse_neighbors;
    // slot planes (as the DI pass's shift jobs, reuse_args): a wave's 64 jobs of one slot write
    // 256 contiguous bytes instead of 4-byte pieces 4 * jpp bytes apart; PTX_AB=GI_JOB_PLANES=0: A/B
    static const bool planes = ab_knob("GI_JOB_PLANES", 1) != 0;
    A.jpx = planes ? 1u : A.jpp;
    A.jslot = planes ? h->band_h * h->cfg.width : 1u;
    if (!planes && motion) A.jpx = gi_job_slots(h);
    A.radius = h->reuse_radius;
    A.neighbors = h->reuse_neighbors;
    A.cap = h->temporal_cap;
    // (a moved camera's history is only usable through the motion pass)
    A.hist_valid = h->hist_valid && (motion || !h->hist_moved) ? 1u : 0u;
    if (motion) {  // the previous frame's camera and G-buffer (motion_prepare), as motion_args
        std::memcpy(A.vpinv_prev, h->hist_camera, sizeof A.vpinv_prev);
        mat4_inverse(A.vpinv_prev, A.vp_prev);
        A.pgbuf = (const uint4 *)h->d_psurf.p + (size_t)h->halo_top * h->cfg.width;
        A.prev_row_lo = -(int32_t)h->halo_top;
        A.prev_row_hi = (int32_t)(h->band_h + h->halo_bot);
        A.clip = (unsigned long long *)h->d_counters.p + CNT_MOTION_CLIP;
    }
    return A;
}

// One pass over the segments [w.seg_base, w.seg_base + w.seg_count) on stream `st`.
static hipError_t launch_wave_seq(ptx_handle *h, const Scene &sc, const WaveBufs &w, int pass, hipStream_t st) {
    const uint4 *gb = gbuf_band(h);
    uint4 *res = res_band(h);
    float4 *acc = (float4 *)h->d_accum.p;
    hipError_t e = hipSuccess;  // every round rewrites all of its segment counts: no memset
    if (h->cfg.pipeline == PTX_PIPELINE_RESTIR_GI) {
        // GI passes: init = 3 logic rounds around 2 traces, spatial = start, trace, combine,
        // temporal / final = one per-pixel launch
        const bool motion = is_motion_pass(pass);
        const GiArgs A = gi_args(h, motion);
        const int gp = motion ? 4 : pass == PTX_PASS_INIT ? 0 : pass == PTX_PASS_TEMPORAL ? 1 : pass == PTX_PASS_SPATIAL ? 2 : 3;
        const int rounds = gp == 0 ? kWaveRoundsGiInit : gp == 2 || gp == 4 ? kWaveRoundsGiSpatial : 0;
        for (int r = 0; e == hipSuccess && r <= rounds; ++r) {
            if (r > 0) {
                TimedLaunch *t = event_begin(h, PTX_STAT_WAVE_TRACE, st);
                e = wave_trace(sc, w, r - 1, 1, h->stack_depth, st, gp >= 2);  // spatial / motion: occlusion only
                event_end(t, st);
                if (e != hipSuccess) break;
            }
            TimedLaunch *t = event_begin(h, PTX_STAT_WAVE_LOGIC, st);
            e = wave_gi_round(sc, w, gp, r, A, st);
            event_end(t, st);
        }
        return e;
    }
    if (pass == PTX_PASS_TEMPORAL || pass == PTX_PASS_SPATIAL || pass == kPassTemporalJobs ||
        pass == kPassTemporalCombine || is_motion_pass(pass)) {
        const bool temporal = pass != PTX_PASS_SPATIAL;
        ReuseArgs A = is_motion_pass(pass) ? motion_args(h)
                                           : reuse_args(h, temporal ? PTX_PASS_TEMPORAL : PTX_PASS_SPATIAL);
        WaveBufs wj = w;
        if (A.fold_last && wj.res[2]) wj.nres = 3;  // light segments finished by the combine
        else A.fold_last = 0u;
        const int nr = reuse_rounds(temporal, A);
        // (the temporal pass in parts: its jobs = rounds 0..nr, its combine = round nr + 1)
        const int r_first = pass == kPassTemporalCombine ? nr + 1 : 0;
        const int r_last = pass == kPassTemporalJobs ? nr : nr + 1;
        for (int r = r_first; e == hipSuccess && r <= r_last; ++r) {
            if (r > 0 && r <= nr) {
                TimedLaunch *t = event_begin(h, PTX_STAT_WAVE_TRACE, st);
                e = wave_trace(sc, wj, r - 1, 1, h->stack_depth, st);
                event_end(t, st);
            }
            if (e != hipSuccess) break;
            if (r == nr && A.fold_last) continue;  // (the combine finishes these jobs)
            TimedLaunch *t = event_begin(h, PTX_STAT_WAVE_LOGIC, st);
            e = wave_reuse_round(sc, wj, temporal, r, A, st);
            event_end(t, st);
        }
        return e;
    }
    // the reuse pipeline's PT_4 reads the spatial output
    const uint4 *fres = h->cfg.pipeline == PTX_PIPELINE_RESTIR_REUSE ? (const uint4 *)hist_band(h) : res;
    // the reuse pipeline's PT_4: one launch, replays inline (PTX_AB=FINAL_ONE=0: the queued rounds)
    static const bool final_one = ab_knob("FINAL_ONE", 1) != 0;
    if (pass == PTX_PASS_FINAL && final_one && h->cfg.pipeline == PTX_PIPELINE_RESTIR_REUSE && tables_fit_lds(sc)) {
        TimedLaunch *t = event_begin(h, PTX_STAT_WAVE_LOGIC, st);
        e = wave_final_one(sc, w, gb, fres, (float4 *)h->d_accum.p, h->stack_depth, st);
        event_end(t, st);
        h->launches[PTX_STAT_FINAL_FUSED] += 1;  // (bench.py: PT_4's queries are not trace_queue's)
        h->init_state_valid = false;  // (its queue slots are rewritten, as by the queued form)
        return e;
    }
    // PT_1 fills the wave state the temporal pass may read; PT_4 / MCPT reuse those slots
    h->init_state_valid = pass == PTX_PASS_INIT && h->cfg.pipeline == PTX_PIPELINE_RESTIR_REUSE;
    const int rounds = pass == PTX_PASS_INIT ? kWaveRoundsInit : pass == PTX_PASS_FINAL ? kWaveRoundsFinal
                                                                                        : kWaveRoundsMcpt;
    for (int r = 0; e == hipSuccess && r <= rounds; ++r) {
        if (r > 0) {
            TimedLaunch *t = event_begin(h, PTX_STAT_WAVE_TRACE, st);
            e = wave_trace(sc, w, r - 1, 1, h->stack_depth, st);
            event_end(t, st);
        }
        if (e != hipSuccess) break;
        TimedLaunch *t = event_begin(h, PTX_STAT_WAVE_LOGIC, st);
        e = pass == PTX_PASS_INIT    ? wave_init_round(sc, w, r, gb, res, st)
            : pass == PTX_PASS_FINAL ? wave_final_round(sc, w, r, gb, fres, acc, st)
                                     : wave_mcpt_round(sc, w, r, acc, h->mcpt_color, st);
        event_end(t, st);
    }
    return e;
}

// Passes over the segments split into K independent launch sequences on K streams
// (fork/join through events on the handle's stream), so one part's latency-bound traces
// overlap another's ALU-bound shading and trace tails.  Each part runs `passes` in order
// over its own segments (a frame: G-buffer -> init -> final per part, nothing shared).
// PTX_AB=WAVE_STREAMS=1..4 overrides K (A/B: 3 measured best since the cooperative traversal,
// +2.5 % over 2 on reuse / ReSTIR; 4 oversubscribes the 4 hardware queues).
hipError_t spatial_summaries(ptx_handle *h, hipStream_t st) {
    if (h->cfg.pipeline != PTX_PIPELINE_RESTIR_REUSE) return hipSuccess;  // GI gathers the buffers
    const size_t W = h->cfg.width, top = h->halo_top * W, band = (size_t)h->band_h * W;
    const uint4 *gb = (const uint4 *)h->d_gbuf.p, *rs = (const uint4 *)h->d_res.p;
    uint4 *nb = (uint4 *)h->d_nbr.p, *sf = (uint4 *)h->d_surf.p;  // (halo rows: surface records too)
    const Scene sc = make_scene(h);
    TimedLaunch *t = event_begin(h, PTX_STAT_WAVE_LOGIC, st);
    hipError_t e;
    if (!h->nbr_valid) {
        e = wave_reuse_summary(sc, gb, rs, nb, sf, px_with_halo(h), st);
    } else {
        e = top ? wave_reuse_summary(sc, gb, rs, nb, sf, top, st) : hipSuccess;
        const size_t b0 = top + band;
        if (e == hipSuccess && px_with_halo(h) > b0)
            e = wave_reuse_summary(sc, gb + b0, rs + 8u * b0, nb + b0, sf ? sf + 2u * b0 : nullptr, px_with_halo(h) - b0,
                                   st);
    }
    event_end(t, st);
    return e;
}

static bool whole_band_sequences(const ptx_handle *h);
// Dynamic trace batches (trace_queue's launch-wide batch stream) for the whole-band launch
// sequences of a whole-image handle; a band handle (halo rows or a communicator) keeps one slot per
// workgroup -- measured at the streamed walk on configs[3]'s 8 re-cut bands, each alone with the
// exchange proxy: static 2.34-2.50 ms against dynamic 2.45-2.56 (the headline: dynamic 515 against
// static 506-510 Msamples/s; tools/cl/r5_bands2.sh).  PTX_AB=TRACE_DYN=0 / 1 forces it off / on.
static bool use_dyn_batches(const ptx_handle *h) {
    static const int dyn_env = ab_knob("TRACE_DYN", -1);
    const bool band = h->comm || h->halo_top || h->halo_bot;
    // (every pipeline keeps static slots in its pipelined frames since late round 5: C1 1080p
    // ReSTIR 1536-1543 Msamples/s against 1431-1443 with dynamic batches, 1406-1414 one frame at a
    // time (tools/cl/r5_piperestir2.sh); TEST_MCPT 1663-1668 against 1598-1609, 1509-1515
    // (r5_pipemcpt.sh); GI C3 at 1792-pixel segments 1104-1107 against 1082 (r5_pipemcpt3.sh);
    // the reuse headline through REUSE_STATIC (reuse_static))
    return dyn_env == 1 ||
           (dyn_env != 0 && whole_band_sequences(h) && !band && h->cfg.pipeline == PTX_PIPELINE_RESTIR_REUSE &&
            !reuse_static());
}
// A band's spatial pass + PT_4 with the halo in flight (PTX_FLAG_HALO_OVERLAP): only the start
// kernel runs per tile set -- the interior rows' shift jobs (their neighbourhood lies inside the
// band) while the halo is in flight, the edge rows' once it has landed (`halo`) -- and every
// trace round is ONE launch over both sets' queue slots (the edge set's slots follow the
// interior's: band_sets), so the overlap costs no extra trace launch tails; steps and combines
// run per set.  One launch sequence.  The same jobs, rays and results as the whole-band pass.
static hipError_t spatial_overlap_seq(ptx_handle *h, const Scene &sc, const WaveBufs &interior, const WaveBufs &edge,
                                      hipEvent_t halo) {
    hipError_t e = hipSuccess;
    // launch sequences as the plain pass runs its back half (two when pipelined): sequence q
    // takes share q of each tile set, and its two shares get ADJACENT physical queue slots --
    // interior share q at slots [a_q + E_q, b_q + E_q), edge share q right after (E_q = the edge
    // slots of the sequences before) -- so each sequence's trace rounds are one launch over one
    // contiguous slot range
    static const int env_bk = ab_knob("PIPE_BACK_STREAMS", 2);
    int k = env_bk > 0 && h->alt_stream && pipelined(h) ? env_bk : 1;
    if (h->cfg.flags & PTX_FLAG_SINGLE_STREAM) k = 1;
    k = std::max(1, std::min<int>({k, ptx_handle::kMaxSplit, (int)interior.nseg, (int)edge.nseg}));
    const bool use_dyn = use_dyn_batches(h);
    const size_t dyn0 = 2u * kWaveMaxRounds * (size_t)interior.cnt_stride;
    ReuseArgs A = reuse_args(h, PTX_PASS_SPATIAL);
    const bool fold = A.fold_last && interior.res[2];
    if (!fold) A.fold_last = 0u;
    const int nr = reuse_rounds(0, A);
    if (k > 1) {
        if (!h->ev_fork && (e = hipEventCreateWithFlags(&h->ev_fork, hipEventDisableTiming)) != hipSuccess) return e;
        for (int q = 1; q < k; ++q) {
            if (!h->sub[q] && (e = hipStreamCreateWithFlags(&h->sub[q], hipStreamNonBlocking)) != hipSuccess) return e;
            if (!h->ev_join[q] && (e = hipEventCreateWithFlags(&h->ev_join[q], hipEventDisableTiming)) != hipSuccess)
                return e;
        }
        if ((e = hipEventRecord(h->ev_fork, h->stream)) != hipSuccess) return e;
        for (int q = 1; q < k; ++q)
            if ((e = hipStreamWaitEvent(h->sub[q], h->ev_fork, 0)) != hipSuccess) return e;
    }
    const bool surf_stale = interior.surf && !h->surf_valid;
    uint32_t E = 0u;  // edge slots of the sequences before
    for (int q = 0; q < k && e == hipSuccess; ++q) {
        hipStream_t st = q ? h->sub[q] : h->stream;
        WaveBufs wi = interior, we = edge;
        wi.seg_base = (uint32_t)((uint64_t)interior.nseg * q / k);
        wi.seg_count = (uint32_t)((uint64_t)interior.nseg * (q + 1) / k) - wi.seg_base;
        we.seg_base = (uint32_t)((uint64_t)edge.nseg * q / k);
        we.seg_count = (uint32_t)((uint64_t)edge.nseg * (q + 1) / k) - we.seg_base;
        wi.seg_phys = interior.seg_phys + E;
        we.seg_phys = interior.seg_phys + E + wi.seg_base + wi.seg_count - we.seg_base;
        E += we.seg_count;
        wi.dyn = use_dyn ? (uint32_t *)h->d_wctr.p + dyn0 + (size_t)q * kWaveMaxRounds * kDynRoundWords : nullptr;
        we.dyn = use_dyn ? (uint32_t *)h->d_wctr.p + dyn0 +
                               (size_t)(ptx_handle::kMaxSplit + q) * kWaveMaxRounds * kDynRoundWords
                         : nullptr;
        if (fold) wi.nres = we.nres = 3;
        WaveBufs wt = wi;  // this sequence's trace launches: both shares' slots
        wt.seg_count = wi.seg_count + we.seg_count;
        if (surf_stale) {  // (primary-hit surface records older than the G-buffer)
            if ((e = wave_surface(sc, wi, gbuf_band(h), st)) != hipSuccess) return e;
            if ((e = wave_surface(sc, we, gbuf_band(h), st)) != hipSuccess) return e;
        }
        for (int r = 0; e == hipSuccess && r <= nr + 1; ++r) {
            if (r > 0 && r <= nr) {
                TimedLaunch *t = event_begin(h, PTX_STAT_WAVE_TRACE, st);
                e = wave_trace(sc, wt, r - 1, 1, h->stack_depth, st);
                event_end(t, st);
                if (e != hipSuccess) break;
            }
            if (r == nr && A.fold_last) continue;  // (the combine finishes these jobs)
            TimedLaunch *t = event_begin(h, PTX_STAT_WAVE_LOGIC, st);
            e = wave_reuse_round(sc, wi, 0, r, A, st);
            if (e == hipSuccess && r == 0 && halo) e = hipStreamWaitEvent(st, halo, 0);
            if (e == hipSuccess) e = wave_reuse_round(sc, we, 0, r, A, st);
            event_end(t, st);
        }
        for (const WaveBufs *ws : {&wi, &we})
            if (e == hipSuccess) e = launch_wave_seq(h, sc, *ws, PTX_PASS_FINAL, st);
    }
    if (surf_stale && e == hipSuccess) h->surf_valid = true;
    for (int q = 1; q < k && e == hipSuccess; ++q) {
        if ((e = hipEventRecord(h->ev_join[q], h->sub[q])) != hipSuccess) return e;
        if ((e = hipStreamWaitEvent(h->stream, h->ev_join[q], 0)) != hipSuccess) return e;
    }
    return e;
}

hipError_t launch_wave_parts(ptx_handle *h, const Scene &sc, const WaveBufs &w, const int *passes, int npasses,
                             bool summaries, const WaveBufs *then, hipEvent_t then_wait) {
    // (PTX_AB=OVERLAP_START=0: the overlapped band pass as two whole sequences, one per tile set)
    static const bool overlap_start = ab_knob("OVERLAP_START", 1) != 0;
    if (then && overlap_start && npasses == 2 && passes[0] == PTX_PASS_SPATIAL && passes[1] == PTX_PASS_FINAL &&
        h->cfg.pipeline == PTX_PIPELINE_RESTIR_REUSE && !summaries)
        return spatial_overlap_seq(h, sc, w, *then, then_wait);
    static const int env_k = ab_knob("WAVE_STREAMS", 0);
    // pipelined frames: each of the two contexts in flight runs its passes as ONE launch
    // sequence (whole-band launches, dynamic trace batches); measured at 1080p C3 reuse: 1
    // stream per context 338 Msamples/s, 2 streams 308, unpipelined 3 streams 320
    // (PTX_AB=PIPE_STREAMS=k: A/B)
    // (ReSTIR without reuse, TEST_MCPT and the reuse pipeline's whole-image frames: 2 per context
    // -- C1 1080p ReSTIR at 1792-pixel segments 1717 against 1620 with one, three 1294
    // (tools/cl/r5_piperestir4.sh, r5_piperestir5.sh); TEST_MCPT 1744-1758 against 1706-1714
    // (r5_pipemcpt2.sh); reuse still 509-514 against 509-513, moving 334 against 329 (r5_gicam2.sh))
    static const int env_pk = ab_knob("PIPE_STREAMS", 0);
    // (a band handle keeps one: a configs[3] band alone with the exchange proxy 2.38 ms against 2.88
    // with two -- tools/cl/r5_bandps.sh)
    const bool band_h = h->comm || h->halo_top || h->halo_bot || (h->cfg.flags & PTX_FLAG_HALO_SKIP);
    // (GI keeps one too: its moving camera 779-784 Msamples/s against 753-759 with two, still
    // 1104-1107 against 1111-1113 -- tools/cl/r5_gicam2.sh, r5_pipemcpt3.sh)
    const int pipe_k = env_pk > 0 ? env_pk
                       : band_h || h->cfg.pipeline == PTX_PIPELINE_RESTIR_GI ||
                                 (h->cfg.pipeline == PTX_PIPELINE_RESTIR_REUSE && !reuse_static())
                           ? 1
                           : 2;
    int k = h->alt_stream && pipelined(h) ? pipe_k : env_k > 0 ? env_k : 3;
    // a pipelined frame's spatial pass + PT_4 (the serial back half every frame waits for) as
    // two launch sequences: one half's trace rounds overlap the other's logic kernels.  Same
    // box, 1080p C3 reuse: 1 sequence 387.2, 2: 396.1, 3: 369.7 Msamples/s (3 contexts' streams
    // oversubscribe the 4 hardware queues).  PTX_AB=PIPE_BACK_STREAMS=k: A/B.
    static const int env_bk = ab_knob("PIPE_BACK_STREAMS", 2);
    if (env_bk > 0 && h->alt_stream && pipelined(h))
        for (int i = 0; i < npasses; ++i)
            if (passes[i] == PTX_PASS_SPATIAL) k = env_bk;
    if (h->cfg.flags & PTX_FLAG_SINGLE_STREAM) k = 1;
    k = std::max(1, std::min<int>(k, ptx_handle::kMaxSplit));
    if ((uint32_t)k > std::max(w.nseg, then ? then->nseg : 0u)) k = (int)std::max(w.nseg, then ? then->nseg : 0u);
    hipError_t e = hipSuccess;
    // the spatial pass gathers neighbours (halo rows included) through their summaries: the
    // temporal pass wrote the band's; halo rows (just received) or a band whose buffers were
    // written since get them here
    for (int i = 0; i < npasses; ++i) {
        if (passes[i] == PTX_PASS_SPATIAL) {
            if (summaries && (e = spatial_summaries(h, h->stream)) != hipSuccess) return e;
        } else if (passes[i] != PTX_PASS_FINAL && passes[i] != PTX_PASS_TEMPORAL && passes[i] != kPassTemporalJobs &&
                   passes[i] != kPassTemporalCombine && !is_motion_pass(passes[i])) {
            h->nbr_valid = false;  // G-buffer / PT_1 / MCPT rewrite what the summaries describe
        }
    }
    // primary-hit surface records (DI reuse): PT_1 writes the band's; a reuse pass that finds
    // them stale (G-buffer or scene changed since) computes them first, per launch sequence
    bool need_surf[8] = {false};
    bool surf_ok = h->surf_valid;
    for (int i = 0; i < npasses && i < 8; ++i) {
        if (passes[i] == PTX_PASS_GBUFFER) surf_ok = false;
        else if (passes[i] == PTX_PASS_INIT && w.surf) surf_ok = true;
        else if ((passes[i] == PTX_PASS_TEMPORAL || passes[i] == kPassTemporalJobs || passes[i] == PTX_PASS_SPATIAL ||
                  is_motion_pass(passes[i])) &&
                 w.surf) {
            need_surf[i] = !surf_ok;
            surf_ok = true;
        }
    }
    h->surf_valid = surf_ok && w.surf;
    if (k == 0) return hipSuccess;  // empty tile set
    if (k > 1) {
        if (!h->ev_fork && (e = hipEventCreateWithFlags(&h->ev_fork, hipEventDisableTiming)) != hipSuccess) return e;
        for (int q = 1; q < k; ++q) {
            if (!h->sub[q] && (e = hipStreamCreateWithFlags(&h->sub[q], hipStreamNonBlocking)) != hipSuccess)
                return e;
            if (!h->ev_join[q] &&
                (e = hipEventCreateWithFlags(&h->ev_join[q], hipEventDisableTiming)) != hipSuccess)
                return e;
        }
        if ((e = hipEventRecord(h->ev_fork, h->stream)) != hipSuccess) return e;
        for (int q = 1; q < k; ++q)
            if ((e = hipStreamWaitEvent(h->sub[q], h->ev_fork, 0)) != hipSuccess) return e;
    }
    for (int q = 0; q < k; ++q) {
        hipStream_t st = q ? h->sub[q] : h->stream;
        for (int set = 0; set < (then ? 2 : 1); ++set) {
            const WaveBufs &ws = set ? *then : w;
            if (set && then_wait && (e = hipStreamWaitEvent(st, then_wait, 0)) != hipSuccess) return e;
            WaveBufs part = ws;
            // dynamic trace batches: with the pipelined frames' whole-band launch sequences
            // (+5.6 % there); with three concurrent sequences per frame the other sequences
            // already fill a launch's tail and the per-workgroup prefix costs more than it
            // saves (1080p, static vs dynamic: ReSTIR 1240 vs 1081, GI 675 vs 625, TEST_MCPT
            // 1264 vs 1229 Msamples/s).  PTX_AB=TRACE_DYN=0 / 1 forces it off / on.
            const bool use_dyn = use_dyn_batches(h);
            part.dyn = !use_dyn ? nullptr
                               : (uint32_t *)h->d_wctr.p + 2u * kWaveMaxRounds * ws.cnt_stride +
                                     (uint32_t)((set * ptx_handle::kMaxSplit + q) * kWaveMaxRounds) * kDynRoundWords;
            part.seg_base = (uint32_t)((uint64_t)ws.nseg * q / k);
            part.seg_count = (uint32_t)((uint64_t)ws.nseg * (q + 1) / k) - part.seg_base;
            if (!part.seg_count) continue;
            for (int i = 0; i < npasses; ++i) {
                if (passes[i] == PTX_PASS_GBUFFER) {
                    TimedLaunch *t = event_begin(h, PTX_PASS_GBUFFER, st);
                    e = wave_gbuffer(sc, part, gbuf_band(h), h->stack_depth, st);
                    h->init_state_valid = false;  // PT_1's state described the previous G-buffer
                    event_end(t, st);
                } else {
                    if (i < 8 && need_surf[i]) {
                        TimedLaunch *t = event_begin(h, PTX_STAT_WAVE_LOGIC, st);
                        e = wave_surface(sc, part, gbuf_band(h), st);
                        event_end(t, st);
                        if (e != hipSuccess) return e;
                    }
                    e = launch_wave_seq(h, sc, part, passes[i], st);
                }
                if (e != hipSuccess) return e;
            }
        }
    }
    for (int q = 1; q < k; ++q) {
        if ((e = hipEventRecord(h->ev_join[q], h->sub[q])) != hipSuccess) return e;
        if ((e = hipStreamWaitEvent(h->stream, h->ev_join[q], 0)) != hipSuccess) return e;
    }
    // the temporal pass rewrote the reservoirs PT_1's state describes, and summarised them
    for (int i = 0; i < npasses; ++i)
        if (passes[i] == PTX_PASS_TEMPORAL || passes[i] == kPassTemporalCombine || passes[i] == kPassTemporalMotion) {
            h->init_state_valid = false;
            h->nbr_valid = h->cfg.pipeline == PTX_PIPELINE_RESTIR_REUSE;
        }
    return hipSuccess;
}
static hipError_t launch_wave_pass(ptx_handle *h, const Scene &sc, const WaveBufs &w, int pass) {
    return launch_wave_parts(h, sc, w, &pass, 1);
}

// The spatial pass just wrote d_hist for the current camera: the next frame's temporal
// pass may use it (ptx_set_frame drops it when the camera moves).
void mark_history(ptx_handle *h) {
    std::memcpy(h->hist_camera, h->uniform + 4, sizeof h->hist_camera);
    h->hist_valid = true;
    h->hist_moved = false;
}

// 4x4 inverse of a column-major f32 matrix in double by cofactors, rounded to f32 (zeros when
// singular): the previous frame's VP for the motion pass's reprojection.  The same expressions
// in the same order as the oracle's pto_mat4_inverse (both built without FMA contraction), so
// the kernels and the oracle reproject through the same f32 matrix.
void mat4_inverse(const float *mf, float *out) {
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

// Before a moved-camera frame's passes: the previous frame's surface records -> d_psurf, on the
// stream of that frame (`st`, ordered after its PT_1; a pipelined frame's next G-buffer on that
// stream comes after the copy).  DI reuse handles (a band's halo rows included: that frame's
// summaries wrote them from the exchanged G-buffer rows); GI handles copy the G-buffer itself
// (halo rows included: that frame's exchange).
int motion_prepare(ptx_handle *h, hipStream_t st) {
    if (h->cfg.pipeline == PTX_PIPELINE_RESTIR_GI) {
        if (int rc = alloc_buf(h, h->d_psurf, h->d_gbuf.bytes)) return rc;
        HIP_CHECK(h, hipMemcpyAsync(h->d_psurf.p, h->d_gbuf.p, h->d_gbuf.bytes, hipMemcpyDeviceToDevice, st));
        return PTX_OK;
    }
    if (!h->d_surf.p) {  // (no surface records yet: nothing to reproject)
        h->hist_valid = false;
        h->hist_moved = false;
        return PTX_OK;
    }
    if (int rc = alloc_buf(h, h->d_psurf, h->d_surf.bytes)) return rc;
    HIP_CHECK(h, hipMemcpyAsync(h->d_psurf.p, h->d_surf.p, h->d_surf.bytes, hipMemcpyDeviceToDevice, st));
    return PTX_OK;
}

// ---------------------------------------------------------------- frame pipelining
// Frames whose passes run as whole-band launch sequences: pipelined frames, or the same
// handle timed launch by launch (PTX_FLAG_TIME_LAUNCHES + SINGLE_STREAM, bench.py's roofline
// region), so both run the same trace kernel mode
static bool whole_band_sequences(const ptx_handle *h) {
    const uint32_t fl = h->cfg.flags;
    const bool timed_alone = (fl & PTX_FLAG_TIME_LAUNCHES) && (fl & PTX_FLAG_SINGLE_STREAM);
    return (h->alt_stream && pipelined(h)) ||
           (timed_alone && (h->cfg.pipeline == PTX_PIPELINE_RESTIR_REUSE || h->cfg.pipeline == PTX_PIPELINE_RESTIR_GI) &&
            !h->comm && !h->halo_top && !h->halo_bot &&
            (size_t)h->band_h * h->cfg.width <= ((size_t)4u << 20));
}
bool pipelined(const ptx_handle *h) {
    static const bool off = ab_knob("PIPELINE_FRAMES", 1) == 0;  // A/B
    // band handles (a rank's band of a split frame: communicator, halo rows or HALO_SKIP) pipeline
    // their band frames the same way (ptx_comm.cpp band_prepare); PTX_AB=PIPELINE_BANDS=0: A/B
    static const bool bands_off = ab_knob("PIPELINE_BANDS", 1) == 0;
    const uint32_t fl = h->cfg.flags;
    const bool band = h->comm || h->halo_top || h->halo_bot;
    // up to 16 Mpx per frame.  (Round 2 capped it at 4 Mpx -- configs[3]'s 3840x2160 frame on one
    // GPU then measured 384 Msamples/s unpipelined, 355 pipelined; with the temporal jobs ahead of
    // the previous-frame wait and the light segments folded into the combines, same box: 465.7
    // unpipelined, 474.9 pipelined.)  PTX_AB=PIPE_MAX_KPX=<n>: A/B
    static const size_t max_px = (size_t)ab_knob("PIPE_MAX_KPX", 16384) << 10;
    const size_t px = (size_t)h->band_h * h->cfg.width;
    // (ReSTIR GI: whole-image handles; its band frames stay one frame at a time)
    const bool pipe_kind = h->cfg.pipeline == PTX_PIPELINE_RESTIR_REUSE ||
                           (h->cfg.pipeline == PTX_PIPELINE_RESTIR_GI && !band) ||
                           (h->cfg.pipeline == PTX_PIPELINE_RESTIR && !band && restir_pipe()) ||
                           (h->cfg.pipeline == PTX_PIPELINE_MCPT && !band && mcpt_pipe());
    return !off && !(band && bands_off) && pipe_kind &&
           px <= max_px &&
           !(fl & (PTX_FLAG_SIMPLE_KERNELS | PTX_FLAG_COUNT_WORK |
                   PTX_FLAG_TIME_LAUNCHES | PTX_FLAG_SINGLE_STREAM | PTX_FLAG_ROW_CENSUS)) &&
           h->stream == (h->ctx_idx == 0 ? h->own_stream : h->ctx_idx == 1 ? h->alt_stream : h->alt2_stream);
}
int pipe_depth() {
    static const int d = ab_knob("PIPE_DEPTH", 2) == 3 ? 3 : 2;
    return d;
}
int quiesce(ptx_handle *h) {
    for (hipStream_t q : {h->stream, h->alt.stream, h->alt2.stream})
        if (q) HIP_CHECK(h, hipStreamSynchronize(q));
    for (int k = 1; k < ptx_handle::kMaxSplit; ++k) {
        if (h->sub[k]) HIP_CHECK(h, hipStreamSynchronize(h->sub[k]));
        if (h->alt.sub[k]) HIP_CHECK(h, hipStreamSynchronize(h->alt.sub[k]));
        if (h->alt2.sub[k]) HIP_CHECK(h, hipStreamSynchronize(h->alt2.sub[k]));
    }
    return PTX_OK;
}
static void swap_two(ptx_handle *h);
// The next context (round robin over pipe_depth() contexts): the members become the next
// context's, `alt` (and `alt2`) the ones after it.
void swap_frame_ctx(ptx_handle *h) {
    swap_two(h);
    if (pipe_depth() == 3) std::swap(h->alt, h->alt2);
    h->ctx_idx = (h->ctx_idx + 1) % pipe_depth();
    h->alt_active = h->ctx_idx != 0;
}
static void swap_two(ptx_handle *h) {
    ptx_handle::FrameCtx &a = h->alt;
    std::swap(h->d_gbuf, a.gbuf);
    std::swap(h->d_res, a.res);
    std::swap(h->d_nbr, a.nbr);
    std::swap(h->d_surf, a.surf);
    std::swap(h->d_wstate, a.wstate);
    std::swap(h->d_wrays, a.wrays);
    std::swap(h->d_wres0, a.wres0);
    std::swap(h->d_wres1, a.wres1);
    std::swap(h->d_wres2, a.wres2);
    std::swap(h->d_tjstate, a.tjstate);
    std::swap(h->d_tjres, a.tjres);
    std::swap(h->d_direct, a.direct);  // (GI: the direct light PT_1's init writes and the shade reads)
    std::swap(h->d_wact0, a.wact0);
    std::swap(h->d_wact1, a.wact1);
    std::swap(h->d_wctr, a.wctr);
    std::swap(h->wave_ray_cap, a.wave_ray_cap);
    std::swap(h->wave_slots, a.wave_slots);
    std::swap(h->stream, a.stream);
    for (int k = 0; k < ptx_handle::kMaxSplit; ++k) {
        std::swap(h->sub[k], a.sub[k]);
        std::swap(h->ev_join[k], a.ev_join[k]);
    }
    std::swap(h->ev_fork, a.ev_fork);
    std::swap(h->init_state_valid, a.init_state_valid);
    std::swap(h->nbr_valid, a.nbr_valid);
    std::swap(h->surf_valid, a.surf_valid);
}
// the second context's G-buffer, reservoirs and stream (its queues, wave state and summaries
// are allocated by wave_buffers / reuse_buffers on its first frame)
int ensure_alt(ptx_handle *h) {
    if (!h->alt_stream) {  // (called with the first context in the members: alt is the second)
        HIP_CHECK(h, hipStreamCreateWithFlags(&h->alt_stream, hipStreamNonBlocking));
        h->alt.stream = h->alt_stream;
    }
    if (pipe_depth() == 3 && !h->alt2_stream) {
        HIP_CHECK(h, hipStreamCreateWithFlags(&h->alt2_stream, hipStreamNonBlocking));
        h->alt2.stream = h->alt2_stream;
    }
    if (!h->ev_prev) HIP_CHECK(h, hipEventCreateWithFlags(&h->ev_prev, hipEventDisableTiming));
    // every context's G-buffer and reservoirs (the other buffers come with its first frame)
    DevBuf *gs[3] = {&h->d_gbuf, &h->alt.gbuf, &h->alt2.gbuf}, *rs[3] = {&h->d_res, &h->alt.res, &h->alt2.res};
    size_t gbytes = 0, rbytes = 0;
    for (int c = 0; c < 3; ++c) {
        gbytes = std::max(gbytes, gs[c]->bytes);
        rbytes = std::max(rbytes, rs[c]->bytes);
    }
    for (int c = 0; c < pipe_depth(); ++c) {
        if (!gs[c]->p) {
            if (int rc = alloc_buf(h, *gs[c], gbytes)) return rc;
            HIP_CHECK(h, memset_sync(h, gs[c]->p, 0, gs[c]->bytes));
        }
        if (!rs[c]->p) {
            if (int rc = alloc_buf(h, *rs[c], rbytes)) return rc;
            HIP_CHECK(h, memset_sync(h, rs[c]->p, 0, rs[c]->bytes));
        }
    }
    if (h->cfg.pipeline == PTX_PIPELINE_RESTIR_GI) {  // GI: each context's direct light too
        DevBuf *ds[3] = {&h->d_direct, &h->alt.direct, &h->alt2.direct};
        for (int c = 0; c < pipe_depth(); ++c)
            if (!ds[c]->p) {
                if (int rc = alloc_buf(h, *ds[c], h->d_direct.bytes)) return rc;
                HIP_CHECK(h, memset_sync(h, ds[c]->p, 0, ds[c]->bytes));
            }
    }
    return PTX_OK;
}
// Back to the first context (its stream is own_stream) before the stream is replaced.
int leave_alt(ptx_handle *h) {
    if (!h->alt_active) return PTX_OK;
    if (int rc = quiesce(h)) return rc;
    while (h->ctx_idx != 0) swap_frame_ctx(h);
    return PTX_OK;
}

// A whole ReSTIR frame in wavefront form (G-buffer -> init -> final per segment group), timed
// as one unit in stats slot PTX_STAT_FRAME.  Returns 1 if this path does not apply.
static int timed_wave_frame(ptx_handle *h) {
    const uint32_t fl = h->cfg.flags;
    if (fl & (PTX_FLAG_SIMPLE_KERNELS | PTX_FLAG_COUNT_WORK))
        return 1;
    if (!h->scene_loaded || !h->frame_set) return fail(h, PTX_E_INVALID, "scene and frame must be set before rendering");
    if (!h->layout_valid) {
        if (int rc = build_layout(h)) return rc;
    }
    Scene sc = make_scene(h);
    if (!tables_fit_lds(sc)) return 1;
    const bool pipe = pipelined(h);
    // a moved camera (DI reuse or GI): the history is reprojected, from the previous frame's
    // surface records (GI: G-buffer), copied first on the previous frame's stream (the current
    // one here); the whole motion pass runs after the wait for that frame.  (A split form --
    // the canonical sample's jobs before the wait -- measured 313 vs 315 Msamples/s on the
    // moving-camera bench: round 4)
    bool moved = h->hist_valid && h->hist_moved && has_reuse(h);
    if (moved) {
        if (int rc = motion_prepare(h, h->stream)) return rc;
        moved = h->hist_moved;
    }
    if (pipe) {
        // frame N goes to the other context; ev_prev marks everything enqueued before it
        // (frame N-1 and any host operation since) on the current context's stream
        if (int rc = ensure_alt(h)) return rc;
        HIP_CHECK(h, hipEventRecord(h->ev_prev, h->stream));
        swap_frame_ctx(h);
    }
    WaveBufs w{};
    if (int rc = wave_buffers(h, w)) return rc;
    TimedLaunch &t = h->ring[h->ring_pos];
    h->ring_pos = (h->ring_pos + 1) % kEventRing;
    resolve_event(t, h);
    HIP_CHECK(h, hipEventRecord(t.start, h->stream));
    hipError_t e;
    if (pipe && h->cfg.pipeline == PTX_PIPELINE_MCPT) {
        // TEST_MCPT: this frame's paths overlap the previous frame's; their colours are kept per
        // pixel (this context's d_direct) and mixed in after the previous frame's mix (ev_prev)
        if (int rc = alloc_buf(h, h->d_direct, (size_t)h->band_h * h->cfg.width * 16u)) return rc;
        static const int mcpt[1] = {PTX_PASS_MCPT};
        h->mcpt_color = (float4 *)h->d_direct.p;
        e = launch_wave_parts(h, sc, w, mcpt, 1);
        h->mcpt_color = nullptr;
        if (e == hipSuccess) e = hipStreamWaitEvent(h->stream, h->ev_prev, 0);
        if (e == hipSuccess) {
            TimedLaunch *tl = event_begin(h, PTX_STAT_WAVE_LOGIC, h->stream);
            e = wave_mix_frame(sc, (const float4 *)h->d_direct.p, (float4 *)h->d_accum.p, h->stream);
            event_end(tl, h->stream);
        }
    } else if (pipe && !has_reuse(h)) {
        // ReSTIR: G-buffer + PT_1 of this frame overlap the previous frame's PT_4, whose
        // accumulation this frame's PT_4 follows (ev_prev)
        static const int front[2] = {PTX_PASS_GBUFFER, PTX_PASS_INIT}, back[1] = {PTX_PASS_FINAL};
        e = launch_wave_parts(h, sc, w, front, 2);
        if (e == hipSuccess) e = hipStreamWaitEvent(h->stream, h->ev_prev, 0);
        if (e == hipSuccess) e = launch_wave_parts(h, sc, w, back, 1);
    } else if (pipe) {
        // G-buffer + PT_1 of this frame overlap the previous frame's spatial pass + PT_4; the
        // temporal pass reads that frame's spatial output (d_hist) and shares its job buffers
        if (int rc = reuse_buffers(h)) return rc;
        // (the temporal pass's shift jobs read only this frame's PT_1 output: they run before the
        // wait, its combine after; PTX_AB=TEMPORAL_SPLIT=0: the whole pass after the wait)
        // (a moved camera: the whole motion temporal pass after the wait -- its history jobs read
        // the previous frame's spatial output)
        // (GI: its temporal pass is one per-pixel launch without rays -- never split)
        static const bool split_on = ab_knob("TEMPORAL_SPLIT", 1) != 0;
        const bool split = split_on && h->cfg.pipeline == PTX_PIPELINE_RESTIR_REUSE;
        static const int front[2] = {PTX_PASS_GBUFFER, PTX_PASS_INIT};
        static const int jobs[1] = {kPassTemporalJobs};
        static const int temporal[1] = {PTX_PASS_TEMPORAL}, temporal_b[1] = {kPassTemporalCombine};
        static const int temporal_m[1] = {kPassTemporalMotion};
        static const int back[2] = {PTX_PASS_SPATIAL, PTX_PASS_FINAL};
        e = launch_wave_parts(h, sc, w, front, 2);
        if (e == hipSuccess && split && !moved) e = launch_wave_parts(h, sc, w, jobs, 1);
        if (e == hipSuccess) e = hipStreamWaitEvent(h->stream, h->ev_prev, 0);
        if (e == hipSuccess)
            e = launch_wave_parts(h, sc, w, moved ? temporal_m : split ? temporal_b : temporal, 1);
        if (e == hipSuccess) e = launch_wave_parts(h, sc, w, back, 2);
        if (e == hipSuccess) mark_history(h);
    } else if (has_reuse(h)) {
        // per-pixel passes up to the temporal output, then (after every segment is done:
        // the spatial pass reads neighbours) spatial + PT_4
        if (int rc = reuse_buffers(h)) return rc;
        static const int front[3] = {PTX_PASS_GBUFFER, PTX_PASS_INIT, PTX_PASS_TEMPORAL};
        static const int front_m[3] = {PTX_PASS_GBUFFER, PTX_PASS_INIT, kPassTemporalMotion};
        static const int back[2] = {PTX_PASS_SPATIAL, PTX_PASS_FINAL};
        e = launch_wave_parts(h, sc, w, moved ? front_m : front, 3);
        if (e == hipSuccess) e = launch_wave_parts(h, sc, w, back, 2);
        if (e == hipSuccess) mark_history(h);
    } else {
        static const int passes[3] = {PTX_PASS_GBUFFER, PTX_PASS_INIT, PTX_PASS_FINAL};
        e = launch_wave_parts(h, sc, w, passes, 3);
    }
    if (e != hipSuccess) return fail(h, PTX_E_HIP, "wavefront frame launch: %s", hipGetErrorString(e));
    HIP_CHECK(h, hipEventRecord(t.stop, h->stream));
    t.pass = PTX_STAT_FRAME;
    t.pending = true;
    return PTX_OK;
}

static int timed_launch(ptx_handle *h, int pass) {
    if (!h->scene_loaded || !h->frame_set) return fail(h, PTX_E_INVALID, "scene and frame must be set before rendering");
    if (pass != PTX_PASS_TEMPORAL && pass != PTX_PASS_SPATIAL && pass != PTX_PASS_FINAL) h->nbr_valid = false;
    if (!h->layout_valid) {
        if (int rc = build_layout(h)) return rc;
    }
    TimedLaunch &t = h->ring[h->ring_pos];
    h->ring_pos = (h->ring_pos + 1) % kEventRing;
    resolve_event(t, h);
    Scene sc = make_scene(h);
    // kernel variant: wavefront (default) or one thread per pixel (PTX_FLAG_SIMPLE_KERNELS: the
    // independent per-pixel form the parity tests check the wavefront queues against)
    const uint32_t fl = h->cfg.flags;
    const int variant = (fl & PTX_FLAG_SIMPLE_KERNELS) ? 2 : 3;
    WaveBufs w{};
    const bool reuse_pass = pass == PTX_PASS_TEMPORAL || pass == PTX_PASS_SPATIAL;
    if (reuse_pass && (variant != 3 || !has_reuse(h)))
        return fail(h, PTX_E_INVALID, "pass %d needs the reuse or GI pipeline (wavefront kernels)", pass);
    if (h->cfg.pipeline == PTX_PIPELINE_RESTIR_GI && pass == PTX_PASS_MCPT)
        return fail(h, PTX_E_INVALID, "the GI pipeline has no MCPT pass");
    if (variant == 3 && pass != PTX_PASS_GBUFFER) {
        if (int rc = wave_buffers(h, w)) return rc;
        if (reuse_pass)
            if (int rc = reuse_buffers(h)) return rc;
    }
    HIP_CHECK(h, hipEventRecord(t.start, h->stream));
    hipError_t e = hipSuccess;
    const uint4 *gb = gbuf_band(h);
    uint4 *res = res_band(h);
    float4 *acc = (float4 *)h->d_accum.p;
    const uint32_t d = h->stack_depth;
    if (variant == 3 && ((pass >= PTX_PASS_INIT && pass <= PTX_PASS_MCPT) || reuse_pass)) {
        e = launch_wave_pass(h, sc, w, pass);
        if (e != hipSuccess) return fail(h, PTX_E_HIP, "wavefront launch (pass %d): %s", pass, hipGetErrorString(e));
        if (pass == PTX_PASS_SPATIAL) mark_history(h);
        HIP_CHECK(h, hipEventRecord(t.stop, h->stream));
        t.pass = pass;
        t.pending = true;
        return PTX_OK;
    }
    switch (pass) {
    case PTX_PASS_GBUFFER:
        e = launch_gbuffer(sc, gbuf_band(h), d, h->stream);
        h->init_state_valid = false;
        h->nbr_valid = false;
        h->surf_valid = false;
        break;
    case PTX_PASS_INIT:
        e = launch_init(sc, gb, res, d, h->stream);
        break;
    case PTX_PASS_FINAL:
        e = launch_final(sc, gb, res, acc, d, h->stream);
        break;
    case PTX_PASS_MCPT:
        e = launch_mcpt(sc, acc, d, h->stream);
        break;
    default: return fail(h, PTX_E_INVALID, "unknown pass %d", pass);
    }
    if (e != hipSuccess) return fail(h, PTX_E_HIP, "kernel launch (pass %d): %s", pass, hipGetErrorString(e));
    HIP_CHECK(h, hipEventRecord(t.stop, h->stream));
    t.pass = pass;
    t.pending = true;
    return PTX_OK;
}

// The band part of a public buffer (the G-buffer / reservoir allocations carry halo rows).
static bool buffer_view(ptx_handle *h, int which, DevBuf &v) {
    const size_t px = (size_t)h->band_h * h->cfg.width;
    switch (which) {
    case PTX_BUF_GBUFFER: v.p = gbuf_band(h); v.bytes = px * 16u; return true;
    case PTX_BUF_RESERVOIR: v.p = res_band(h); v.bytes = px * 16u * h->res_u4; return true;
    case PTX_BUF_DIRECT: v = h->d_direct; return v.p != nullptr && h->cfg.pipeline == PTX_PIPELINE_RESTIR_GI;
    case PTX_BUF_ACCUM: v = h->d_accum; return true;
    case PTX_BUF_COUNTERS: v = h->d_counters; return true;
    case PTX_BUF_RESERVOIR_HIST: v.p = h->d_hist.p ? hist_band(h) : nullptr; v.bytes = px * 16u * h->res_u4; return v.p != nullptr;
    default: return false;
    }
}

}  // namespace ptx

// ================================================================ exported C ABI
extern "C" {

int ptx_abi_version(void) { return PTX_ABI_VERSION; }

int ptx_build_info(char *out, size_t bytes) {
    auto esc = [](const std::string &v) {
        std::string o;
        for (char c : v) {
            if (c == '"' || c == '\\') o += '\\';
            if ((unsigned char)c >= 0x20) o += c;
        }
        return o;
    };
    const char *ab = getenv("PTX_AB");
    std::string ign;
    for (const std::string &k : ignored_knobs()) ign += (ign.empty() ? "\"" : ",\"") + esc(k) + "\"";
    char buf[1024];
    const int n = std::snprintf(buf, sizeof buf,
                                "{\"abi\": %d, \"build\": \"%s\", \"arch\": \"gfx950\", \"ptx_ab\": \"%s\", "
                                "\"ptx_ab_ignored\": [%s], \"rccl\": \"%s\"}",
                                PTX_ABI_VERSION, kBuildKind, esc(ab ? ab : "").c_str(), ign.c_str(),
                                esc(comm_library()).c_str());
    if (out && bytes) {
        std::memcpy(out, buf, std::min<size_t>((size_t)std::max(n, 0), bytes - 1));
        out[std::min<size_t>((size_t)std::max(n, 0), bytes - 1)] = 0;
    }
    return n;
}

int ptx_create(const ptx_config *cfg, ptx_handle **out) {
    warn_ignored_knobs();  // (once per process: PTX_AB keys this build ignores)
    if (!cfg || !out) return PTX_E_INVALID;
    *out = nullptr;
    if (cfg->width == 0 || cfg->height == 0 || cfg->pipeline > PTX_PIPELINE_RESTIR_GI) return PTX_E_INVALID;
    if (cfg->flags & PTX_FLAGS_RETIRED) return PTX_E_INVALID;  // the removed A/B kernel variants
    if ((cfg->pipeline == PTX_PIPELINE_RESTIR_REUSE || cfg->pipeline == PTX_PIPELINE_RESTIR_GI) &&
        (cfg->flags & (PTX_FLAG_SIMPLE_KERNELS)))
        return PTX_E_INVALID;  // the reuse passes exist in wavefront form only
    if (cfg->reuse_neighbors > 16u) return PTX_E_INVALID;
    if ((cfg->flags & PTX_FLAG_ROW_CENSUS) &&
        (cfg->flags & (PTX_FLAG_SIMPLE_KERNELS)))
        return PTX_E_INVALID;  // the census maps wavefront queue slots to tile rows
    ptx_handle *h = new (std::nothrow) ptx_handle();
    if (!h) return PTX_E_NOMEM;
    h->cfg = *cfg;
    if (h->cfg.flags & PTX_FLAG_ROW_CENSUS) h->cfg.flags |= PTX_FLAG_COUNT_WORK;
    if (h->cfg.row_begin == 0 && h->cfg.row_end == 0) h->cfg.row_end = h->cfg.height;
    if (h->cfg.row_begin >= h->cfg.row_end || h->cfg.row_end > h->cfg.height) {
        delete h;
        return PTX_E_INVALID;
    }
    h->band_h = h->cfg.row_end - h->cfg.row_begin;
    if (h->cfg.pipeline == PTX_PIPELINE_RESTIR_GI) h->res_u4 = kGiResU4;
    if (has_reuse(h)) {
        h->reuse_radius = h->cfg.reuse_radius ? h->cfg.reuse_radius : 30u;
        h->reuse_neighbors = h->cfg.reuse_neighbors ? h->cfg.reuse_neighbors : 3u;
        h->temporal_cap = h->cfg.temporal_cap ? h->cfg.temporal_cap : 20u;
        h->halo_top = std::min(h->reuse_radius, h->cfg.row_begin);
        h->halo_bot = std::min(h->reuse_radius, h->cfg.height - h->cfg.row_end);
        if ((h->halo_top || h->halo_bot) && h->band_h < h->reuse_radius) {  // halos come from adjacent bands only
            delete h;
            return PTX_E_INVALID;
        }
    }
    int rc = PTX_OK;
    hipError_t e;
    if (cfg->device >= 0) {
        if ((e = hipSetDevice(cfg->device)) != hipSuccess) rc = PTX_E_HIP;
    }
    if (!rc && (e = hipGetDevice(&h->device)) != hipSuccess) rc = PTX_E_HIP;
    if (!rc && (e = hipStreamCreateWithFlags(&h->own_stream, hipStreamNonBlocking)) != hipSuccess) rc = PTX_E_HIP;
    for (int i = 0; !rc && i < kEventRing; ++i) {
        if (hipEventCreate(&h->ring[i].start) != hipSuccess || hipEventCreate(&h->ring[i].stop) != hipSuccess)
            rc = PTX_E_HIP;
    }
    h->stream = h->own_stream;
    const size_t px = (size_t)h->band_h * h->cfg.width;
    const size_t px_halo = (size_t)(h->halo_top + h->band_h + h->halo_bot) * h->cfg.width;
    if (!rc) rc = alloc_buf(h, h->d_gbuf, px_halo * 16u);
    if (!rc) rc = alloc_buf(h, h->d_res, px_halo * 16u * h->res_u4);
    if (!rc && has_reuse(h)) {
        rc = alloc_buf(h, h->d_hist, px_halo * 16u * h->res_u4);
        if (!rc && memset_sync(h, h->d_hist.p, 0, h->d_hist.bytes) != hipSuccess) rc = PTX_E_HIP;
    }
    if (!rc && h->cfg.pipeline == PTX_PIPELINE_RESTIR_GI) {
        rc = alloc_buf(h, h->d_direct, px * 16u);
        if (!rc && memset_sync(h, h->d_direct.p, 0, h->d_direct.bytes) != hipSuccess) rc = PTX_E_HIP;
    }
    if (!rc) rc = alloc_buf(h, h->d_accum, px * 16u);
    if (!rc) rc = alloc_buf(h, h->d_counters, kCounterWords * 8u);
    if (!rc) rc = alloc_buf(h, h->d_queue, 64u);
    if (!rc && (h->cfg.flags & PTX_FLAG_ROW_CENSUS)) {
        // G-buffer tile rows + queue slots (segments hold >= 256 padded pixels: <= padded/256 + 2)
        const size_t tile_rows = (h->band_h + 7u) / 8u, tiles = tile_rows * ((h->cfg.width + 7u) / 8u);
        h->census_blocks = (uint32_t)(tile_rows + tiles * 64u / 256u + 2u);
        rc = alloc_buf(h, h->d_census, (size_t)h->census_blocks * kCensusWords * 8u);
        if (!rc && memset_sync(h, h->d_census.p, 0, h->d_census.bytes) != hipSuccess) rc = PTX_E_HIP;
    }
#ifdef PTX_WG_TIMES
    if (!rc && ab_knob("WGT", 0)) {  // 4 header words + 2^20 records of 4 words
        rc = alloc_buf(h, h->d_wgt, (4u + 4u * (1u << 20)) * 8u);
        if (!rc && memset_sync(h, h->d_wgt.p, 0, 32u) != hipSuccess) rc = PTX_E_HIP;
    }
#endif
    if (!rc && memset_sync(h, h->d_accum.p, 0, h->d_accum.bytes) != hipSuccess) rc = PTX_E_HIP;
    if (!rc && memset_sync(h, h->d_counters.p, 0, h->d_counters.bytes) != hipSuccess) rc = PTX_E_HIP;
    if (!rc && memset_sync(h, h->d_gbuf.p, 0, h->d_gbuf.bytes) != hipSuccess) rc = PTX_E_HIP;
    if (!rc && memset_sync(h, h->d_res.p, 0, h->d_res.bytes) != hipSuccess) rc = PTX_E_HIP;
    if (rc) {
        ptx_destroy(h);
        return rc;
    }
    *out = h;
    return PTX_OK;
}

int ptx_upload_scene(ptx_handle *h, const uint32_t *scene, size_t n_scene, const uint32_t *geometry,
                     size_t n_geometry, const uint32_t *accel, size_t n_accel) {
    if (!h) return PTX_E_INVALID;
    HIP_CHECK(h, hipSetDevice(h->device));  // handles of one process may sit on several GPUs
    if (!scene || !geometry || (!accel && n_accel)) return fail(h, PTX_E_INVALID, "null scene array");
    if (int rc = quiesce(h)) return rc;  // frames in flight still read the old scene and layout
    h->scene.assign(scene, scene + n_scene);
    h->geometry.assign(geometry, geometry + n_geometry);
    h->accel.assign(accel ? accel : scene, accel ? accel + n_accel : scene);
    if (int rc = upload(h, h->d_scene, scene, n_scene * 4u)) return rc;
    if (int rc = upload(h, h->d_geometry, geometry, n_geometry * 4u)) return rc;
    h->layout_valid = false;
    h->scene_loaded = true;
    h->hist_valid = false;
    h->init_state_valid = false;
    h->nbr_valid = false;
    h->surf_valid = h->alt.surf_valid = h->alt2.surf_valid = false;
    if (h->frame_set) return build_layout(h);
    return PTX_OK;
}

int ptx_set_frame(ptx_handle *h, const uint32_t uniform[PTX_UNIFORM_WORDS]) {
    if (!h || !uniform) return PTX_E_INVALID;
    HIP_CHECK(h, hipSetDevice(h->device));  // handles of one process may sit on several GPUs
    if (uniform[0] != h->cfg.width || uniform[1] != h->cfg.height)
        return fail(h, PTX_E_INVALID, "uniform resolution %ux%u != handle %ux%u", uniform[0], uniform[1],
                    h->cfg.width, h->cfg.height);
    uint32_t key[8];
    for (int k = 0; k < 8; ++k) key[k] = uniform[24 + k];
    if (std::memcmp(key, h->layout_key, sizeof key) != 0) {
        std::memcpy(h->layout_key, key, sizeof key);
        h->layout_valid = false;
    }
    std::memcpy(h->uniform, uniform, sizeof h->uniform);
    h->frame_set = true;
    // temporal history: a reuse or GI handle reprojects it when the camera moved (the motion
    // temporal pass; a band through ptx_render with a communicator or ptx_render_bands, which
    // bring the neighbours' rows of it); pass by pass it is reusable only for the camera that
    // produced it (reuse_args / gi_args)
    h->hist_moved = std::memcmp(h->hist_camera, uniform + 4, sizeof h->hist_camera) != 0;
    if (h->hist_moved && !has_reuse(h)) h->hist_valid = false;
    if (h->scene_loaded && !h->layout_valid) return build_layout(h);
    return PTX_OK;
}

int ptx_run_pass(ptx_handle *h, int pass) {
    if (!h) return PTX_E_INVALID;
    HIP_CHECK(h, hipSetDevice(h->device));  // handles of one process may sit on several GPUs
    return timed_launch(h, pass);
}

int ptx_run_passes(ptx_handle *h, const int *passes, int n) {
    if (!h || (!passes && n)) return PTX_E_INVALID;
    if (n < 0 || n > 8) return fail(h, PTX_E_INVALID, "ptx_run_passes: %d passes", n);
    HIP_CHECK(h, hipSetDevice(h->device));
    for (int i = 0; i < n; ++i) {
        const int p = passes[i];
        const bool ok = p == PTX_PASS_GBUFFER || p == PTX_PASS_INIT || p == PTX_PASS_FINAL || p == PTX_PASS_MCPT ||
                        p == PTX_PASS_TEMPORAL || (p == PTX_PASS_SPATIAL && i == 0);
        if (!ok) return fail(h, PTX_E_INVALID, "ptx_run_passes: pass %d at position %d", p, i);
        if ((p == PTX_PASS_TEMPORAL || p == PTX_PASS_SPATIAL) && !has_reuse(h))
            return fail(h, PTX_E_INVALID, "pass %d needs the reuse or GI pipeline", p);
        if (p == PTX_PASS_MCPT && h->cfg.pipeline == PTX_PIPELINE_RESTIR_GI)
            return fail(h, PTX_E_INVALID, "the GI pipeline has no MCPT pass");
    }
    const uint32_t fl = h->cfg.flags;
    if (fl & (PTX_FLAG_SIMPLE_KERNELS | PTX_FLAG_COUNT_WORK)) {
        for (int i = 0; i < n; ++i)
            if (int rc = timed_launch(h, passes[i])) return rc;
        return PTX_OK;
    }
    if (!h->scene_loaded || !h->frame_set) return fail(h, PTX_E_INVALID, "scene and frame must be set before rendering");
    if (!h->layout_valid) {
        if (int rc = build_layout(h)) return rc;
    }
    Scene sc = make_scene(h);
    bool gb = false, reuse = false;
    for (int i = 0; i < n; ++i) {
        gb |= passes[i] == PTX_PASS_GBUFFER;
        reuse |= passes[i] == PTX_PASS_TEMPORAL || passes[i] == PTX_PASS_SPATIAL;
    }
    if (gb && !tables_fit_lds(sc)) {  // the segment-mapped G-buffer needs LDS tables
        for (int i = 0; i < n; ++i)
            if (int rc = timed_launch(h, passes[i])) return rc;
        return PTX_OK;
    }
    WaveBufs w{};
    if (int rc = wave_buffers(h, w)) return rc;
    if (reuse)
        if (int rc = reuse_buffers(h)) return rc;
    TimedLaunch &t = h->ring[h->ring_pos];
    h->ring_pos = (h->ring_pos + 1) % kEventRing;
    resolve_event(t, h);
    HIP_CHECK(h, hipEventRecord(t.start, h->stream));
    const hipError_t e = launch_wave_parts(h, sc, w, passes, n);
    if (e != hipSuccess) return fail(h, PTX_E_HIP, "ptx_run_passes: %s", hipGetErrorString(e));
    HIP_CHECK(h, hipEventRecord(t.stop, h->stream));
    t.pass = PTX_STAT_PASS_GROUP;
    t.pending = true;
    for (int i = 0; i < n; ++i)
        if (passes[i] == PTX_PASS_SPATIAL) mark_history(h);
    return PTX_OK;
}

int ptx_halo_rows(ptx_handle *h, uint32_t *rows_top, uint32_t *rows_bottom, size_t *bytes_per_row) {
    if (!h) return PTX_E_INVALID;
    if (rows_top) *rows_top = h->halo_top;
    if (rows_bottom) *rows_bottom = h->halo_bot;
    if (bytes_per_row) *bytes_per_row = (size_t)h->cfg.width * (16u + 16u * h->res_u4);
    return PTX_OK;
}

// Rows [r0, r0 + rows) of the halo-extended G-buffer / reservoir (row 0 = first halo row)
// <-> one contiguous message (G-buffer rows, then reservoir rows).
static int halo_copy(ptx_handle *h, uint32_t r0, uint32_t rows, void *msg, bool to_msg) {
    if (!rows) return PTX_OK;
    const size_t W = h->cfg.width, rpx = 16u * h->res_u4, gb = rows * W * 16u, rb = rows * W * rpx;
    char *g = (char *)h->d_gbuf.p + (size_t)r0 * W * 16u, *r = (char *)h->d_res.p + (size_t)r0 * W * rpx;
    char *m = (char *)msg;
    // hipMemcpyDefault: the message may be device memory (RCCL) or host memory (gloo)
    if (to_msg) {
        HIP_CHECK(h, hipMemcpyAsync(m, g, gb, hipMemcpyDefault, h->stream));
        HIP_CHECK(h, hipMemcpyAsync(m + gb, r, rb, hipMemcpyDefault, h->stream));
    } else {
        HIP_CHECK(h, hipMemcpyAsync(g, m, gb, hipMemcpyDefault, h->stream));
        HIP_CHECK(h, hipMemcpyAsync(r, m + gb, rb, hipMemcpyDefault, h->stream));
    }
    return PTX_OK;
}

int ptx_halo_pack(ptx_handle *h, void *dev_top, void *dev_bottom) {
    if (!h) return PTX_E_INVALID;
    if ((h->halo_top && !dev_top) || (h->halo_bot && !dev_bottom)) return fail(h, PTX_E_INVALID, "ptx_halo_pack: null buffer");
    // the band's first halo_top rows go up (the band above keeps them as its bottom halo)
    if (int rc = halo_copy(h, h->halo_top, h->halo_top, dev_top, true)) return rc;
    return halo_copy(h, h->halo_top + h->band_h - h->halo_bot, h->halo_bot, dev_bottom, true);
}

int ptx_halo_unpack(ptx_handle *h, const void *dev_top, const void *dev_bottom) {
    if (!h) return PTX_E_INVALID;
    if ((h->halo_top && !dev_top) || (h->halo_bot && !dev_bottom)) return fail(h, PTX_E_INVALID, "ptx_halo_unpack: null buffer");
    if (int rc = halo_copy(h, 0u, h->halo_top, (void *)dev_top, false)) return rc;
    return halo_copy(h, h->halo_top + h->band_h, h->halo_bot, (void *)dev_bottom, false);
}

int ptx_render(ptx_handle *h, float *rgba_out) {
    if (!h) return PTX_E_INVALID;
    HIP_CHECK(h, hipSetDevice(h->device));  // handles of one process may sit on several GPUs
    if (h->cfg.pipeline == PTX_PIPELINE_RESTIR) {
        int rc = timed_wave_frame(h);
        if (rc < 0) return rc;
        if (rc == 1)  // other variants / counting builds: pass by pass
            for (int p : {PTX_PASS_GBUFFER, PTX_PASS_INIT, PTX_PASS_FINAL})
                if ((rc = timed_launch(h, p))) return rc;
    } else if (has_reuse(h) && h->comm) {  // a band of a multi-GPU frame: halo over RCCL
        if (int rc = render_band_nccl(h)) return rc;
        if (rgba_out)
            if (int rc = read_to_host(h, rgba_out, h->d_accum.p, h->d_accum.bytes)) return rc;
        return PTX_OK;
    } else if (has_reuse(h) && (h->halo_top || h->halo_bot) && (h->cfg.flags & PTX_FLAG_HALO_SKIP)) {
        if (int rc = render_band_solo(h)) return rc;  // (counts its frame)
        if (rgba_out)
            if (int rc = read_to_host(h, rgba_out, h->d_accum.p, h->d_accum.bytes)) return rc;
        return PTX_OK;
    } else if (has_reuse(h)) {
        if (h->halo_top || h->halo_bot)
            return fail(h, PTX_E_INVALID, "a band of the reuse pipeline renders with a communicator "
                                          "(ptx_comm_init), through ptx_render_bands, or ptx_run_passes + ptx_halo_*");
        int rc = timed_wave_frame(h);
        if (rc < 0) return rc;
        if (rc == 1)  // counting builds: pass by pass
            for (int p : {PTX_PASS_GBUFFER, PTX_PASS_INIT, PTX_PASS_TEMPORAL, PTX_PASS_SPATIAL, PTX_PASS_FINAL})
                if ((rc = timed_launch(h, p))) return rc;
    } else if (pipelined(h)) {  // TEST_MCPT frames two in flight
        int rc = timed_wave_frame(h);
        if (rc < 0) return rc;
        if (rc == 1 && (rc = timed_launch(h, PTX_PASS_MCPT))) return rc;
    } else {
        if (int rc = timed_launch(h, PTX_PASS_MCPT)) return rc;
    }
    h->frames++;
    if (rgba_out)
        if (int rc = read_to_host(h, rgba_out, h->d_accum.p, h->d_accum.bytes)) return rc;
    return PTX_OK;
}

int ptx_reset_accumulation(ptx_handle *h) {
    if (!h) return PTX_E_INVALID;
    HIP_CHECK(h, hipMemsetAsync(h->d_accum.p, 0, h->d_accum.bytes, h->stream));
    h->hist_valid = false;
    return PTX_OK;
}

int ptx_synchronize(ptx_handle *h) {
    if (!h) return PTX_E_INVALID;
    HIP_CHECK(h, hipStreamSynchronize(h->stream));
    return PTX_OK;
}

int ptx_get_stats(ptx_handle *h, ptx_stats *out) {
    if (!h || !out) return PTX_E_INVALID;
    for (auto &t : h->ring) resolve_event(t, h);
    std::memset(out, 0, sizeof *out);
    out->frames = h->frames;
    for (int p = 0; p < kPasses; ++p) {
        out->kernel_ms_total[p] = h->ms_total[p];
        out->kernel_launches[p] = h->launches[p];
    }
    out->triangles = h->n_tris;
    out->bvh_nodes = h->n_nodes;
    out->instances = h->n_inst;
    out->max_bvh_depth = h->max_depth;
    out->device_bytes = h->d_scene.bytes + h->d_geometry.bytes + h->d_tris.bytes + h->d_nodes.bytes +
                        h->d_subs.bytes + h->d_insts.bytes + h->d_mats.bytes + h->d_tverts.bytes + h->d_gbuf.bytes + h->d_res.bytes + h->d_accum.bytes +
                        h->d_hist.bytes + h->d_jstate.bytes + h->d_jres.bytes + h->d_tjstate.bytes + h->d_tjres.bytes + h->d_nbr.bytes + h->d_surf.bytes + h->d_psurf.bytes + h->d_direct.bytes;
    return PTX_OK;
}

int ptx_reset_stats(ptx_handle *h) {
    if (!h) return PTX_E_INVALID;
    for (auto &t : h->ring) t.pending = false;
    HIP_CHECK(h, hipStreamSynchronize(h->stream));
    for (int p = 0; p < kPasses; ++p) { h->ms_total[p] = 0.0; h->launches[p] = 0; }
    h->frames = 0;
    HIP_CHECK(h, memset_sync(h, h->d_counters.p, 0, h->d_counters.bytes));
    if (h->d_census.p) HIP_CHECK(h, memset_sync(h, h->d_census.p, 0, h->d_census.bytes));
    return PTX_OK;
}

#ifdef PTX_WG_TIMES
// Diagnostic build only: copies up to max_records per-wave records {start, end (100 MHz
// ticks), kernel id << 32 | block, wave-in-block << 32 | HW_ID} recorded since the last call
// and restarts the log.  Returns the record count (>= 0) or a PTX_E_* status.
int ptx_diag_wave_times(ptx_handle *h, uint64_t *out, size_t max_records) {
    if (!h || !h->d_wgt.p) return PTX_E_INVALID;
    HIP_CHECK(h, hipDeviceSynchronize());
    uint64_t n = 0;
    HIP_CHECK(h, copy_sync(h, &n, h->d_wgt.p, 8, hipMemcpyDeviceToHost));
    n = std::min<uint64_t>(std::min<uint64_t>(n, 1u << 20), max_records);
    if (n && out) HIP_CHECK(h, copy_sync(h, out, (uint64_t *)h->d_wgt.p + 4, n * 32u, hipMemcpyDeviceToHost));
    HIP_CHECK(h, memset_sync(h, h->d_wgt.p, 0, 8));
    return (int)n;
}
#endif

int ptx_row_census(ptx_handle *h, uint64_t *out, size_t n_tile_rows) {
    if (!h || !out) return PTX_E_INVALID;
    if (!(h->cfg.flags & PTX_FLAG_ROW_CENSUS)) return fail(h, PTX_E_INVALID, "handle has no PTX_FLAG_ROW_CENSUS");
    const uint32_t tile_rows = (h->band_h + 7u) / 8u, tiles_x = (h->cfg.width + 7u) / 8u;
    if (n_tile_rows != tile_rows) return fail(h, PTX_E_INVALID, "census: %zu tile rows, band has %u", n_tile_rows, tile_rows);
    std::vector<unsigned long long> c((size_t)h->census_blocks * kCensusWords);
    HIP_CHECK(h, copy_sync(h, c.data(), h->d_census.p, c.size() * 8u, hipMemcpyDeviceToHost));
    std::memset(out, 0, (size_t)tile_rows * 5u * sizeof(uint64_t));
    for (uint32_t r = 0; r < tile_rows; ++r)
        for (int k = 0; k < 5; ++k) out[5u * r + k] += c[(size_t)kCensusWords * r + k];
    // queue slot s traced the rays of segment s: tiles [s*m, s*m + m) in raster order
    // (m = seg_px / 64); a slot spanning two tile rows is split by its tiles in each
    const uint32_t m = seg_pixels(h) / 64u, ntiles = tile_rows * tiles_x;
    for (uint32_t s = 0; tile_rows + s < h->census_blocks && (size_t)s * m < ntiles; ++s) {
        const unsigned long long *b = c.data() + (size_t)kCensusWords * (tile_rows + s);
        const uint32_t t0 = s * m, t1 = std::min(ntiles, t0 + m), r0 = t0 / tiles_x, r1 = (t1 - 1u) / tiles_x;
        for (int k = 0; k < 5; ++k) {
            uint64_t left = b[k];
            for (uint32_t r = r0; r <= r1; ++r) {
                const uint32_t a = std::max(t0, r * tiles_x), z = std::min(t1, (r + 1u) * tiles_x);
                const uint64_t part = r == r1 ? left : b[k] * (z - a) / (t1 - t0);
                out[5u * r + k] += part;
                left -= part;
            }
        }
    }
    return PTX_OK;
}

int ptx_read_buffer(ptx_handle *h, int which, void *host_dst, size_t bytes) {
    if (!h || !host_dst) return PTX_E_INVALID;
    DevBuf b;
    if (!buffer_view(h, which, b) || bytes > b.bytes)
        return fail(h, PTX_E_INVALID, "read of %zu bytes from buffer %d", bytes, which);
    if (int rc = read_to_host(h, host_dst, b.p, bytes)) return rc;
    return PTX_OK;
}

int ptx_write_buffer(ptx_handle *h, int which, const void *host_src, size_t bytes) {
    if (!h || !host_src) return PTX_E_INVALID;
    DevBuf b;
    if (!buffer_view(h, which, b) || bytes > b.bytes)
        return fail(h, PTX_E_INVALID, "write of %zu bytes to buffer %d", bytes, which);
    HIP_CHECK(h, copy_sync(h, b.p, host_src, bytes, hipMemcpyHostToDevice));
    h->init_state_valid = false;  // the wave state no longer matches the buffers
    h->nbr_valid = false;
    h->surf_valid = false;  // (a G-buffer write: the surface records describe the old one)
    return PTX_OK;
}

int ptx_device_pointer(ptx_handle *h, int which, void **dev_ptr, size_t *bytes) {
    if (!h || !dev_ptr) return PTX_E_INVALID;
    DevBuf b;
    if (!buffer_view(h, which, b)) return fail(h, PTX_E_INVALID, "unknown buffer %d", which);
    *dev_ptr = b.p;
    if (bytes) *bytes = b.bytes;
    return PTX_OK;
}

int ptx_present(ptx_handle *h, uint32_t canvas_w, uint32_t canvas_h, int bgra, uint8_t *out) {
    if (!h || !out) return PTX_E_INVALID;
    if (canvas_w == 0 || canvas_h == 0 || (uint64_t)canvas_w * canvas_h > (1ull << 28))
        return fail(h, PTX_E_INVALID, "ptx_present: canvas %ux%u", canvas_w, canvas_h);
    if (h->cfg.row_begin != 0 || h->band_h != h->cfg.height)
        return fail(h, PTX_E_INVALID, "ptx_present: a band handle (rows %u..%u) holds part of the texture: present the "
                                      "gathered frame on the host", h->cfg.row_begin, h->cfg.row_end);
    if (!h->d_accum.p) return fail(h, PTX_E_INVALID, "ptx_present: nothing rendered");
    HIP_CHECK(h, hipSetDevice(h->device));
    const size_t bytes = (size_t)canvas_w * canvas_h * 4u;
    if (int rc = alloc_buf(h, h->d_canvas, bytes)) return rc;
    const hipError_t e = launch_present((const float4 *)h->d_accum.p, h->cfg.width, h->cfg.height, canvas_w, canvas_h,
                                        bgra != 0, (uint32_t *)h->d_canvas.p, h->stream);
    if (e != hipSuccess) return fail(h, PTX_E_HIP, "ptx_present: %s", hipGetErrorString(e));
    return read_to_host(h, out, h->d_canvas.p, bytes);
}

int ptx_present_async(ptx_handle *h, uint32_t canvas_w, uint32_t canvas_h, int bgra) {
    if (!h) return PTX_E_INVALID;
    if (h->present_pending) return fail(h, PTX_E_INVALID, "ptx_present_async: a present is in flight (poll it first)");
    if (canvas_w == 0 || canvas_h == 0 || (uint64_t)canvas_w * canvas_h > (1ull << 28))
        return fail(h, PTX_E_INVALID, "ptx_present_async: canvas %ux%u", canvas_w, canvas_h);
    if (h->cfg.row_begin != 0 || h->band_h != h->cfg.height)
        return fail(h, PTX_E_INVALID, "ptx_present_async: a band handle holds part of the texture");
    if (!h->d_accum.p) return fail(h, PTX_E_INVALID, "ptx_present_async: nothing rendered");
    HIP_CHECK(h, hipSetDevice(h->device));
    const size_t bytes = (size_t)canvas_w * canvas_h * 4u;
    if (int rc = alloc_buf(h, h->d_canvas_async, bytes)) return rc;
    if (bytes > h->present_host_bytes) {
        if (h->present_host) (void)hipHostFree(h->present_host);
        h->present_host = nullptr;
        h->present_host_bytes = 0;
        HIP_CHECK(h, hipHostMalloc(&h->present_host, bytes, hipHostMallocDefault));
        h->present_host_bytes = bytes;
    }
    if (!h->ev_present) HIP_CHECK(h, hipEventCreateWithFlags(&h->ev_present, hipEventDisableTiming));
    // on the current frame's stream, after it: a pipelined handle's next frame records ev_prev
    // on this stream before it enqueues anything, and its accumulation waits for ev_prev
    const hipError_t e = launch_present((const float4 *)h->d_accum.p, h->cfg.width, h->cfg.height, canvas_w, canvas_h,
                                        bgra != 0, (uint32_t *)h->d_canvas_async.p, h->stream);
    if (e != hipSuccess) return fail(h, PTX_E_HIP, "ptx_present_async: %s", hipGetErrorString(e));
    HIP_CHECK(h, hipMemcpyAsync(h->present_host, h->d_canvas_async.p, bytes, hipMemcpyDeviceToHost, h->stream));
    HIP_CHECK(h, hipEventRecord(h->ev_present, h->stream));
    h->present_bytes = bytes;
    h->present_pending = true;
    return PTX_OK;
}

int ptx_present_poll(ptx_handle *h, uint8_t *out, size_t bytes) {
    if (!h || !out) return PTX_E_INVALID;
    if (!h->present_pending) return fail(h, PTX_E_INVALID, "ptx_present_poll: no present in flight");
    if (bytes < h->present_bytes)
        return fail(h, PTX_E_INVALID, "ptx_present_poll: %zu bytes; the canvas needs %zu", bytes, h->present_bytes);
    const hipError_t e = hipEventQuery(h->ev_present);
    if (e == hipErrorNotReady) return PTX_E_PENDING;
    if (e != hipSuccess) {
        h->present_pending = false;
        return fail(h, PTX_E_HIP, "ptx_present_poll: %s", hipGetErrorString(e));
    }
    std::memcpy(out, h->present_host, h->present_bytes);
    h->present_pending = false;
    return PTX_OK;
}

int ptx_trace_device(ptx_handle *h, const void *rays_dev, void *hits_dev, size_t n, int eps_mode) {
    if (!h || (n && (!rays_dev || !hits_dev)) || n > 0xffffffffu || (eps_mode != 0 && eps_mode != 1))
        return fail(h, PTX_E_INVALID, "ptx_trace: bad arguments");
    if (!h->scene_loaded || !h->frame_set) return fail(h, PTX_E_INVALID, "scene and frame must be set before tracing");
    if (!h->layout_valid) {
        if (int rc = build_layout(h)) return rc;
    }
    TimedLaunch &t = h->ring[h->ring_pos];
    h->ring_pos = (h->ring_pos + 1) % kEventRing;
    resolve_event(t, h);
    Scene sc = make_scene(h);
    HIP_CHECK(h, hipEventRecord(t.start, h->stream));
    // one thread per ray with the SIMPLE_KERNELS flag; otherwise the lane-refill kernel the
    // wavefront passes trace with
    const bool simple = (h->cfg.flags & PTX_FLAG_SIMPLE_KERNELS) != 0;
    hipError_t e = (simple ? launch_trace_rays : launch_trace_rays_sm)(
        sc, (const float4 *)rays_dev, (float4 *)hits_dev, (uint32_t)n, eps_mode, h->stack_depth, h->stream);
    if (e != hipSuccess) return fail(h, PTX_E_HIP, "trace launch: %s", hipGetErrorString(e));
    HIP_CHECK(h, hipEventRecord(t.stop, h->stream));
    t.pass = PTX_PASS_TRACE;
    t.pending = true;
    return PTX_OK;
}

int ptx_trace(ptx_handle *h, const float *rays, float *hits, size_t n, int eps_mode) {
    if (!h || (n && (!rays || !hits))) return fail(h, PTX_E_INVALID, "ptx_trace: null arrays");
    if (n == 0) return PTX_OK;
    if (int rc = alloc_buf(h, h->d_qrays, std::max(h->d_qrays.bytes, n * 32u))) return rc;
    if (int rc = alloc_buf(h, h->d_qhits, std::max(h->d_qhits.bytes, n * 32u))) return rc;
    HIP_CHECK(h, hipMemcpyAsync(h->d_qrays.p, rays, n * 32u, hipMemcpyHostToDevice, h->stream));
    if (int rc = ptx_trace_device(h, h->d_qrays.p, h->d_qhits.p, n, eps_mode)) return rc;
    return read_to_host(h, hits, h->d_qhits.p, n * 32u);
}

int ptx_set_stream(ptx_handle *h, void *hip_stream) {
    if (!h) return PTX_E_INVALID;
    if (int rc = leave_alt(h)) return rc;
    h->stream = hip_stream ? (hipStream_t)hip_stream : h->own_stream;
    return PTX_OK;
}

int ptx_destroy(ptx_handle *h) {
    if (!h) return PTX_E_INVALID;
    (void)hipSetDevice(h->device);
    // everything enqueued (a band frame's sends / receives on the exchange stream included)
    // finishes before the communicator and the exchange stream go
    (void)quiesce(h);
    if (h->xstream) (void)hipStreamSynchronize(h->xstream);
    comm_destroy(h);
    while (h->ctx_idx != 0) swap_frame_ctx(h);
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    for (hipStream_t q : h->sub)
        if (q) (void)hipStreamSynchronize(q);
    if (h->own_stream) (void)hipStreamSynchronize(h->own_stream);
    for (auto &t : h->ring) {
        if (t.start) (void)hipEventDestroy(t.start);
        if (t.stop) (void)hipEventDestroy(t.stop);
    }
    if (h->host_stage) (void)hipHostFree(h->host_stage);
    if (h->ev_present) {
        (void)hipEventSynchronize(h->ev_present);
        (void)hipEventDestroy(h->ev_present);
    }
    if (h->present_host) (void)hipHostFree(h->present_host);
    for (DevBuf *b : {&h->d_canvas, &h->d_canvas_async, &h->d_scene, &h->d_geometry, &h->d_tris, &h->d_nodes, &h->d_subs, &h->d_insts, &h->d_mats, &h->d_tverts, &h->d_gbuf,
                      &h->d_res, &h->d_accum, &h->d_counters, &h->d_queue, &h->d_qrays, &h->d_qhits,
                      &h->d_wstate, &h->d_wrays, &h->d_wres0, &h->d_wres1, &h->d_wres2, &h->d_wact0, &h->d_wact1, &h->d_wctr,
                      &h->d_hist, &h->d_jstate, &h->d_jres, &h->d_tjstate, &h->d_tjres, &h->d_nbr, &h->d_surf, &h->d_psurf, &h->d_direct, &h->d_census})
        free_buf(*b);
    for (ptx_handle::FrameCtx *ap : {&h->alt, &h->alt2}) {
        ptx_handle::FrameCtx &a = *ap;
        for (DevBuf *b : {&a.gbuf, &a.res, &a.nbr, &a.surf, &a.wstate, &a.wrays, &a.wres0, &a.wres1, &a.wres2, &a.wact0, &a.wact1,
                          &a.wctr, &a.tjstate, &a.tjres, &a.direct})
            free_buf(*b);
        if (a.ev_fork) (void)hipEventDestroy(a.ev_fork);
        for (int q = 0; q < ptx_handle::kMaxSplit; ++q) {
            if (a.ev_join[q]) (void)hipEventDestroy(a.ev_join[q]);
            if (a.sub[q]) (void)hipStreamDestroy(a.sub[q]);
        }
    }
    if (h->alt_stream) (void)hipStreamDestroy(h->alt_stream);
    if (h->alt2_stream) (void)hipStreamDestroy(h->alt2_stream);
    if (h->ev_prev) (void)hipEventDestroy(h->ev_prev);
    if (h->ev_fork) (void)hipEventDestroy(h->ev_fork);
    for (int q = 0; q < ptx_handle::kMaxSplit; ++q) {
        if (h->ev_join[q]) (void)hipEventDestroy(h->ev_join[q]);
        if (h->sub[q]) (void)hipStreamDestroy(h->sub[q]);
    }
    if (h->own_stream) (void)hipStreamDestroy(h->own_stream);
    delete h;
    return PTX_OK;
}

const char *ptx_last_error(const ptx_handle *h) { return h ? h->err.c_str() : "null handle"; }

}  // extern "C"
