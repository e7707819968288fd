// ptx_comm.cpp -- multi-GPU frames of the reuse pipelines: the RCCL
// communicator a band handle owns, the spatial-reuse halo exchange, and frames split over
// several band handles of one process.
//
// The reference has no exchange: every WGSL pass reads only its own pixel
// (GC/Renderer_TEST.ts:208-261).  The build-defined spatial pass
// (docs/theory/ReSTIR_Pipeline.md:354-462) reads neighbours up to reuse_radius rows away, so
// a row band needs the G-buffer + reservoir rows of the bands above and below between its
// temporal and spatial passes.  Here that exchange is device to device on the handle's
// streams, no host synchronisation anywhere in a frame:
//   * across processes (one rank per GPU): grouped ncclSend / ncclRecv straight from the
//     band's first / last rows into the neighbour's halo rows (no pack / unpack copies);
//   * inside one process (ptx_render_bands, e.g. one Node host driving every GPU, or several
//     bands on one GPU): the same through the handles' communicators, or hipMemcpyPeerAsync
//     when the handles have none.
// PTX_FLAG_HALO_OVERLAP splits the spatial pass into the rows whose neighbourhood lies inside
// the band (run while the halo is in flight) and the edge rows (run when it has landed).
//
// RCCL is loaded with dlopen at ptx_comm_init: in a process that already holds one (torch's
// bundled librccl.so.1) the loader hands back that copy, and libptx.so stays loadable where
// no RCCL is installed.  PTX_RCCL_LIB names another library with the same entry points (the
// tests' in-process loopback communicator, tests/loopback/, runs several band handles of one
// GPU through this exact code).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "ptx_internal.h"

namespace ptx {
namespace {

struct Rccl {
    ncclResult_t (*get_unique_id)(ncclUniqueId *) = nullptr;
    ncclResult_t (*init_rank)(ncclComm_t *, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*init_all)(ncclComm_t *, int, const int *) = nullptr;
    ncclResult_t (*send)(const void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*recv)(void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*group_start)() = nullptr;
    ncclResult_t (*group_end)() = nullptr;
    ncclResult_t (*destroy)(ncclComm_t) = nullptr;
    ncclResult_t (*async_error)(ncclComm_t, ncclResult_t *) = nullptr;
    const char *(*error_string)(ncclResult_t) = nullptr;
    // optional (non-blocking communicator init with a deadline; absent -> blocking init)
    ncclResult_t (*init_rank_config)(ncclComm_t *, int, ncclUniqueId, int, ncclConfig_t *) = nullptr;
    ncclResult_t (*abort)(ncclComm_t) = nullptr;
    ncclResult_t (*finalize)(ncclComm_t) = nullptr;
    bool ok = false;
    std::string why;
};

// the library rccl() opened (ptx_build_info reports it: a PTX_RCCL_LIB stand-in is never silent)
std::string g_comm_library;

const Rccl &rccl() {
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        const char *path = std::getenv("PTX_RCCL_LIB");
        void *lib = nullptr;
        if (path && *path) {
            // a test hook (tests/loopback/): said on stderr, and in ptx_build_info's "rccl"
            std::fprintf(stderr, "libptx: PTX_RCCL_LIB=%s replaces RCCL as the communicator library\n", path);
            lib = dlopen(path, RTLD_NOW | RTLD_LOCAL);
        } else {
            path = "librccl.so.1";
            lib = dlopen(path, RTLD_NOW | RTLD_GLOBAL);
            if (!lib) lib = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        }
        if (!lib) {
            const char *e = dlerror();
            r.why = std::string("dlopen ") + path + ": " + (e ? e : "not found");
            g_comm_library = std::string("(not loaded: ") + r.why + ")";
            return;
        }
        g_comm_library = path;
        bool all = true;
        auto sym = [&](auto &fn, const char *name) {
            fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(lib, name));
            if (!fn) {
                all = false;
                r.why = std::string("librccl.so.1 lacks ") + name;
            }
        };
        sym(r.get_unique_id, "ncclGetUniqueId");
        sym(r.init_rank, "ncclCommInitRank");
        sym(r.init_all, "ncclCommInitAll");
        sym(r.send, "ncclSend");
        sym(r.recv, "ncclRecv");
        sym(r.group_start, "ncclGroupStart");
        sym(r.group_end, "ncclGroupEnd");
        sym(r.destroy, "ncclCommDestroy");
        sym(r.async_error, "ncclCommGetAsyncError");
        sym(r.error_string, "ncclGetErrorString");
        r.ok = all;
        r.init_rank_config = reinterpret_cast<decltype(r.init_rank_config)>(dlsym(lib, "ncclCommInitRankConfig"));
        r.abort = reinterpret_cast<decltype(r.abort)>(dlsym(lib, "ncclCommAbort"));
        r.finalize = reinterpret_cast<decltype(r.finalize)>(dlsym(lib, "ncclCommFinalize"));
    });
    return r;
}

#define NCCL_CHECK(h, expr)                                                                                  \
    do {                                                                                                     \
        ncclResult_t r_ = (expr);                                                                            \
        if (r_ != ncclSuccess) {                                                                             \
            (h)->comm_broken = (h)->comm != nullptr;                                                         \
            return fail((h), PTX_E_HIP, "%s: %s (%s:%d)", #expr, rccl().error_string(r_), __FILE__, __LINE__); \
        }                                                                                                    \
    } while (0)

// Non-blocking communicators (ptx_comm_init): the init and every group end return at once and
// complete in the background; their state is polled here until it leaves ncclInProgress or the
// deadline passes.  A rank whose peers never join (one died before its ncclCommInitRank, or
// failed inside it) thus gets an error status after `seconds` instead of hanging for ever, and
// the communicator is aborted (PTX_AB=COMM_TIMEOUT_S=n overrides the 120 s default).
int comm_timeout_s() {
    static const int t = env_knob("COMM_TIMEOUT_S", 120);
    return t > 0 ? t : 120;
}
ncclResult_t comm_wait(ncclComm_t c, int seconds) {
    const auto end = std::chrono::steady_clock::now() + std::chrono::seconds(seconds);
    for (uint32_t spin = 0;; ++spin) {
        ncclResult_t st = ncclSuccess;
        const ncclResult_t r = rccl().async_error(c, &st);
        if (r != ncclSuccess) return r;
        if (st != ncclInProgress) return st;
        if (std::chrono::steady_clock::now() >= end) return ncclInProgress;  // (the deadline)
        if (spin >= 64u) std::this_thread::sleep_for(std::chrono::microseconds(200));
    }
}
// ncclGroupEnd on a band handle's communicator: complete (enqueued on the streams) on return.
int group_end_wait(ptx_handle *h) {
    ncclResult_t r = rccl().group_end();
    if (r == ncclInProgress) r = comm_wait((ncclComm_t)h->comm, comm_timeout_s());
    if (r != ncclSuccess) h->comm_broken = true;
    if (r == ncclInProgress)
        return fail(h, PTX_E_HIP, "RCCL group (rank %d of %d) not enqueued within %d s", h->rank, h->world,
                    comm_timeout_s());
    if (r != ncclSuccess) return fail(h, PTX_E_HIP, "ncclGroupEnd: %s", rccl().error_string(r));
    return PTX_OK;
}

// Byte ranges of the halo-extended G-buffer and reservoir allocations: rows [r0, r0 + rows)
// (row 0 = the first top-halo row).
struct Rows {
    char *g, *r;
    size_t gb, rb;
};
Rows rows_of(ptx_handle *h, uint32_t r0, uint32_t rows) {
    const size_t W = h->cfg.width, rpx = 16u * h->res_u4;
    return Rows{(char *)h->d_gbuf.p + (size_t)r0 * W * 16u, (char *)h->d_res.p + (size_t)r0 * W * rpx,
                rows * W * 16u, rows * W * rpx};
}
// what this band sends up (its first halo_top rows) / down (its last halo_bot rows), and the
// halo rows it receives into
Rows send_up(ptx_handle *h) { return rows_of(h, h->halo_top, h->halo_top); }
Rows send_down(ptx_handle *h) { return rows_of(h, h->halo_top + h->band_h - h->halo_bot, h->halo_bot); }
Rows recv_top(ptx_handle *h) { return rows_of(h, 0u, h->halo_top); }
Rows recv_bottom(ptx_handle *h) { return rows_of(h, h->halo_top + h->band_h, h->halo_bot); }
// The motion halo: the same rows of the history (the previous frame's spatial output), which a
// moved camera's temporal pass reprojects into (ReuseArgs::prev_row_lo / hi).
struct HistRows {
    char *p;
    size_t bytes;
};
HistRows hist_rows_of(ptx_handle *h, uint32_t r0, uint32_t rows) {
    const size_t W = h->cfg.width, rpx = 16u * h->res_u4;
    return HistRows{(char *)h->d_hist.p + (size_t)r0 * W * rpx, rows * W * rpx};
}
HistRows hist_send_up(ptx_handle *h) { return hist_rows_of(h, h->halo_top, h->halo_top); }
HistRows hist_send_down(ptx_handle *h) { return hist_rows_of(h, h->halo_top + h->band_h - h->halo_bot, h->halo_bot); }
HistRows hist_recv_top(ptx_handle *h) { return hist_rows_of(h, 0u, h->halo_top); }
HistRows hist_recv_bottom(ptx_handle *h) { return hist_rows_of(h, h->halo_top + h->band_h, h->halo_bot); }

bool overlap(const ptx_handle *h) { return (h->cfg.flags & PTX_FLAG_HALO_OVERLAP) != 0; }

// The band's tile sets: interior rows (neighbourhood inside the band) and edge rows.
struct BandSets {
    WaveBufs interior, edge;
    bool split = false;
};
WaveBufs tile_set(const WaveBufs &w, uint32_t t0, uint32_t n0, uint32_t t1, uint32_t n1, uint32_t phys) {
    WaveBufs s = w;
    s.tile0 = t0;
    s.ntile0 = n0;
    s.tile1 = t1;
    s.ntile1 = n1;
    s.nseg = (uint32_t)(((size_t)(n0 + n1) * 64u + w.seg_px - 1u) / w.seg_px);
    s.seg_base = 0;
    s.seg_count = s.nseg;
    s.seg_phys = phys;
    return s;
}
BandSets band_sets(const ptx_handle *h, const WaveBufs &w) {
    BandSets b;
    const uint32_t tx = (h->cfg.width + 7u) / 8u, T = (h->band_h + 7u) / 8u, R = h->reuse_radius;
    // a pixel of band row y reads rows y - R .. y + R: the top edge is rows [0, R) (tile rows
    // [0, ceil(R/8))), the bottom edge rows [band_h - R, band_h)
    const uint32_t e_top = h->halo_top ? std::min(T, (R + 7u) / 8u) : 0u;
    const uint32_t e_bot = h->halo_bot ? T - std::min(T, (h->band_h - std::min(h->band_h, R)) / 8u) : 0u;
    if (e_top + e_bot >= T || !(e_top || e_bot)) return b;
    b.split = true;
    b.interior = tile_set(w, e_top * tx, (T - e_top - e_bot) * tx, 0u, 0u, 0u);
    b.edge = tile_set(w, 0u, e_top * tx, (T - e_bot) * tx, e_bot * tx, b.interior.nseg);
    return b;
}

// Layout, queue and reuse buffers of a band frame.  Band frames are pipelined like whole-image
// frames (pipelined(): two contexts in flight): the frame goes to the other context, and `pipe`
// tells band_front to run its G-buffer + PT_1 beside the previous frame's exchange, spatial
// pass and PT_4 (the previous context's stream), its temporal pass after them.  Per context: the
// G-buffer and reservoirs with their halo rows (what this band sends and receives), summaries,
// surface records, queues; shared: history, shift jobs, accumulation.  The previous frame's
// sends read the other context's rows, and a context's next frame starts on its stream after
// its back passes, which wait for that frame's exchange (ev_halo): nothing is overwritten in
// flight.  A moved camera (DI reuse or GI, history valid: `moved`) reprojects the history: the previous
// frame's surface records (GI: G-buffer) are copied first (motion_prepare, before the context swap), and the
// neighbours' rows of its spatial output arrive as the motion halo before the temporal pass.
// ev_prev marks everything enqueued before this frame on the previous frame's stream (pipelined
// or not: a neighbour's motion-halo copy waits for it).
//
// Whether the motion halo is exchanged (`xchg`, motion_exchange) is decided from state every rank
// shares -- the frames rendered and the uniform sequence -- never from this rank's history state:
// a rank that dropped its history (a reset, a scene upload) still sends and receives its rows and
// renders the frame without history (`moved` false), so no rank waits on a send its neighbour
// never posts.
bool motion_exchange(const ptx_handle *h) {
    return has_reuse(h) && h->band_frames > 0 &&
           std::memcmp(h->band_camera, h->uniform + 4, sizeof h->band_camera) != 0;
}
int band_prepare(ptx_handle *h, Scene &sc, WaveBufs &w, bool &pipe, bool &moved) {
    if (!has_reuse(h)) return fail(h, PTX_E_INVALID, "band frames need the reuse or GI pipeline");
    if (h->cfg.flags & (PTX_FLAG_SIMPLE_KERNELS | PTX_FLAG_COUNT_WORK))
        return fail(h, PTX_E_INVALID, "band frames run the wavefront kernels (no counting / A-B variants)");
    if (!h->scene_loaded || !h->frame_set) return fail(h, PTX_E_INVALID, "scene and frame must be set before rendering");
    if (!h->layout_valid)
        if (int rc = build_layout(h)) return rc;
    sc = make_scene(h);
    if (!tables_fit_lds(sc)) return fail(h, PTX_E_SCENE, "band frames need the LDS root / instance tables");
    moved = motion_exchange(h) && h->hist_valid && h->hist_moved;
    if (moved) {
        if (int rc = motion_prepare(h, h->stream)) return rc;
        moved = h->hist_moved;
    }
    pipe = pipelined(h);
    if (pipe)
        if (int rc = ensure_alt(h)) return rc;
    if (!h->ev_prev) HIP_CHECK(h, hipEventCreateWithFlags(&h->ev_prev, hipEventDisableTiming));
    HIP_CHECK(h, hipEventRecord(h->ev_prev, h->stream));
    if (pipe) swap_frame_ctx(h);
    if (int rc = wave_buffers(h, w)) return rc;
    if (int rc = reuse_buffers(h)) return rc;
    hipError_t e = hipSuccess;
    if (!h->ev_front && (e = hipEventCreateWithFlags(&h->ev_front, hipEventDisableTiming)) != hipSuccess)
        return fail(h, PTX_E_HIP, "event: %s", hipGetErrorString(e));
    if (!h->ev_halo && (e = hipEventCreateWithFlags(&h->ev_halo, hipEventDisableTiming)) != hipSuccess)
        return fail(h, PTX_E_HIP, "event: %s", hipGetErrorString(e));
    if (!h->xstream && (e = hipStreamCreateWithFlags(&h->xstream, hipStreamNonBlocking)) != hipSuccess)
        return fail(h, PTX_E_HIP, "stream: %s", hipGetErrorString(e));
    return PTX_OK;
}

// G-buffer -> PT_1 -> temporal over the whole band, then ev_front on h->stream, in two calls:
// band_front (everything before the wait for the previous frame: G-buffer, PT_1 and, pipelined,
// the still camera's temporal jobs; unpipelined and still, the whole temporal pass) and
// band_temporal (after it: the temporal combine, or a moved camera's whole motion pass, once the
// motion halo has landed -- the caller exchanges it in between).
int band_front(ptx_handle *h, const Scene &sc, const WaveBufs &w, TimedLaunch *&frame_t, bool pipe, bool moved) {
    frame_t = &h->ring[h->ring_pos];
    h->ring_pos = (h->ring_pos + 1) % kEventRing;
    resolve_event(*frame_t, h);
    HIP_CHECK(h, hipEventRecord(frame_t->start, h->stream));
    static const int front[3] = {PTX_PASS_GBUFFER, PTX_PASS_INIT, PTX_PASS_TEMPORAL};
    static const int front_split[3] = {PTX_PASS_GBUFFER, PTX_PASS_INIT, kPassTemporalJobs};
    // (the temporal jobs before the wait, the temporal combine after: timed_wave_frame)
    const hipError_t e = launch_wave_parts(h, sc, w, pipe ? front_split : front, moved ? 2 : 3);
    if (e != hipSuccess) return fail(h, PTX_E_HIP, "band front passes: %s", hipGetErrorString(e));
    if (pipe) HIP_CHECK(h, hipStreamWaitEvent(h->stream, h->ev_prev, 0));
    return PTX_OK;
}
int band_temporal(ptx_handle *h, const Scene &sc, const WaveBufs &w, bool pipe, bool moved) {
    static const int combine[1] = {kPassTemporalCombine}, motion[1] = {kPassTemporalMotion};
    if (moved || pipe) {
        const hipError_t e = launch_wave_parts(h, sc, w, moved ? motion : combine, 1);
        if (e != hipSuccess) return fail(h, PTX_E_HIP, "band temporal pass: %s", hipGetErrorString(e));
    }
    HIP_CHECK(h, hipEventRecord(h->ev_front, h->stream));
    return PTX_OK;
}

// The stream the halo of this band is received on: the exchange stream when the spatial pass
// overlaps it (forked from ev_front), else the band's own stream.
int exchange_stream(ptx_handle *h, hipStream_t &xs) {
    xs = h->stream;
    if (overlap(h)) {
        xs = h->xstream;
        HIP_CHECK(h, hipStreamWaitEvent(xs, h->ev_front, 0));
    }
    return PTX_OK;
}

// Enqueue this band's sends / receives on its communicator (inside a group).
int nccl_halo(ptx_handle *h, hipStream_t xs) {
    const Rccl &R = rccl();
    ncclComm_t c = (ncclComm_t)h->comm;
    if (h->halo_top) {
        const Rows s = send_up(h), r = recv_top(h);
        NCCL_CHECK(h, R.send(s.g, s.gb, ncclUint8, h->rank - 1, c, xs));
        NCCL_CHECK(h, R.send(s.r, s.rb, ncclUint8, h->rank - 1, c, xs));
        NCCL_CHECK(h, R.recv(r.g, r.gb, ncclUint8, h->rank - 1, c, xs));
        NCCL_CHECK(h, R.recv(r.r, r.rb, ncclUint8, h->rank - 1, c, xs));
    }
    if (h->halo_bot) {
        const Rows s = send_down(h), r = recv_bottom(h);
        NCCL_CHECK(h, R.send(s.g, s.gb, ncclUint8, h->rank + 1, c, xs));
        NCCL_CHECK(h, R.send(s.r, s.rb, ncclUint8, h->rank + 1, c, xs));
        NCCL_CHECK(h, R.recv(r.g, r.gb, ncclUint8, h->rank + 1, c, xs));
        NCCL_CHECK(h, R.recv(r.r, r.rb, ncclUint8, h->rank + 1, c, xs));
    }
    return PTX_OK;
}

// A moved camera's motion halo over the communicator, on h->stream after the wait for the previous
// frame (its spatial output is complete there, and this frame's spatial pass comes after):
// this band's first / last rows of the history to the neighbours, theirs into its halo rows.
// Every rank of a frame moves or none (the same camera): the groups stay matched.
int nccl_motion_halo(ptx_handle *h) {
    const Rccl &R = rccl();
    ncclComm_t c = (ncclComm_t)h->comm;
    if (h->halo_top) {
        const HistRows s = hist_send_up(h), r = hist_recv_top(h);
        NCCL_CHECK(h, R.send(s.p, s.bytes, ncclUint8, h->rank - 1, c, h->stream));
        NCCL_CHECK(h, R.recv(r.p, r.bytes, ncclUint8, h->rank - 1, c, h->stream));
        h->halo_bytes_sent += s.bytes;
    }
    if (h->halo_bot) {
        const HistRows s = hist_send_down(h), r = hist_recv_bottom(h);
        NCCL_CHECK(h, R.send(s.p, s.bytes, ncclUint8, h->rank + 1, c, h->stream));
        NCCL_CHECK(h, R.recv(r.p, r.bytes, ncclUint8, h->rank + 1, c, h->stream));
        h->halo_bytes_sent += s.bytes;
    }
    return PTX_OK;
}

// After the halo landed on xs: the halo rows' neighbour summaries, then ev_halo.
int halo_landed(ptx_handle *h, hipStream_t xs) {
    if (overlap(h)) {
        const hipError_t e = spatial_summaries(h, xs);
        if (e != hipSuccess) return fail(h, PTX_E_HIP, "halo summaries: %s", hipGetErrorString(e));
    }
    HIP_CHECK(h, hipEventRecord(h->ev_halo, xs));
    return PTX_OK;
}

// Spatial + PT_4.  Without overlap: the whole band after the halo (h->stream carries it).
// With overlap: each of the K streams runs its share of the interior rows, waits for the
// halo, then its share of the edge rows (disjoint queue slots, so no join in between).
int band_back(ptx_handle *h, const Scene &sc, const WaveBufs &w, TimedLaunch *frame_t) {
    static const int back[2] = {PTX_PASS_SPATIAL, PTX_PASS_FINAL};
    hipError_t e = hipSuccess;
    const BandSets b = overlap(h) ? band_sets(h, w) : BandSets{};
    if (!b.split) {
        if (overlap(h)) HIP_CHECK(h, hipStreamWaitEvent(h->stream, h->ev_halo, 0));
        // (with overlap the summaries already ran on the exchange stream)
        e = launch_wave_parts(h, sc, w, back, 2, !overlap(h));
    } else {
        e = launch_wave_parts(h, sc, b.interior, back, 2, false, &b.edge, h->ev_halo);
    }
    if (e != hipSuccess) return fail(h, PTX_E_HIP, "band spatial / final passes: %s", hipGetErrorString(e));
    mark_history(h);
    std::memcpy(h->band_camera, h->uniform + 4, sizeof h->band_camera);
    h->band_frames++;
    HIP_CHECK(h, hipEventRecord(frame_t->stop, h->stream));
    frame_t->pass = PTX_STAT_FRAME;
    frame_t->pending = true;
    h->frames++;
    return PTX_OK;
}

// An error a previous frame's sends / receives raised asynchronously (a peer that died, a
// broken link): checked once per frame, so a failed exchange surfaces as a status instead of
// a hang or a silently stale halo (failure handling).
int comm_health(ptx_handle *h) {
    ncclResult_t st = ncclSuccess;
    NCCL_CHECK(h, rccl().async_error((ncclComm_t)h->comm, &st));
    if (st != ncclSuccess && st != ncclInProgress) {
        h->comm_broken = true;
        return fail(h, PTX_E_HIP, "RCCL communicator (rank %d of %d) reports: %s", h->rank, h->world,
                    rccl().error_string(st));
    }
    return PTX_OK;
}

// Once, at ptx_comm_init: every rank swaps its band geometry {width, height, row_begin, row_end,
// halo_top, halo_bot} with the ranks above and below, and refuses a neighbour whose rows do
// not continue its own or whose halo would not match what this band sends -- such a mismatch
// would otherwise hang in ncclGroupEnd or carry rows from past the band.
int check_neighbours(ptx_handle *h) {
    if (h->world < 2) return PTX_OK;
    const Rccl &R = rccl();
    ncclComm_t c = (ncclComm_t)h->comm;
    uint32_t mine[6] = {h->cfg.width, h->cfg.height, h->cfg.row_begin, h->cfg.row_end, h->halo_top, h->halo_bot};
    uint32_t got[2][6] = {};
    uint32_t *d = nullptr;
    HIP_CHECK(h, hipMalloc(&d, 18 * sizeof(uint32_t)));
    auto done = [&](int rc) { (void)hipFree(d); return rc; };
    hipError_t e = hipMemcpyAsync(d, mine, sizeof mine, hipMemcpyHostToDevice, h->stream);
    if (e != hipSuccess) return done(fail(h, PTX_E_HIP, "neighbour check: %s", hipGetErrorString(e)));
    ncclResult_t r = R.group_start();
    if (r == ncclSuccess && h->rank > 0) {
        r = R.send(d, 6, ncclUint32, h->rank - 1, c, h->stream);
        if (r == ncclSuccess) r = R.recv(d + 6, 6, ncclUint32, h->rank - 1, c, h->stream);
    }
    if (r == ncclSuccess && h->rank + 1 < h->world) {
        r = R.send(d, 6, ncclUint32, h->rank + 1, c, h->stream);
        if (r == ncclSuccess) r = R.recv(d + 12, 6, ncclUint32, h->rank + 1, c, h->stream);
    }
    if (r != ncclSuccess) {
        (void)R.group_end();
        h->comm_broken = true;
        return done(fail(h, PTX_E_HIP, "neighbour check: %s", R.error_string(r)));
    }
    if (int rc = group_end_wait(h)) return done(rc);
    e = hipMemcpyAsync(got, d + 6, sizeof got, hipMemcpyDeviceToHost, h->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
    if (e != hipSuccess) {
        h->comm_broken = true;
        return done(fail(h, PTX_E_HIP, "neighbour check: %s", hipGetErrorString(e)));
    }
    const uint32_t *up = got[0], *dn = got[1];
    if (h->rank > 0 && (up[0] != mine[0] || up[1] != mine[1] || up[3] != mine[2] || up[5] != mine[4]))
        return done(fail(h, PTX_E_INVALID,
                         "ptx_comm_init: rank %d has rows [%u,%u) with a %u-row halo below in a %ux%u frame; this band "
                         "(rank %d) starts at row %u with a %u-row halo above in a %ux%u frame",
                         h->rank - 1, up[2], up[3], up[5], up[0], up[1], h->rank, mine[2], mine[4], mine[0], mine[1]));
    if (h->rank + 1 < h->world && (dn[0] != mine[0] || dn[1] != mine[1] || dn[2] != mine[3] || dn[4] != mine[5]))
        return done(fail(h, PTX_E_INVALID,
                         "ptx_comm_init: rank %d has rows [%u,%u) with a %u-row halo above in a %ux%u frame; this band "
                         "(rank %d) ends at row %u with a %u-row halo below in a %ux%u frame",
                         h->rank + 1, dn[2], dn[3], dn[4], dn[0], dn[1], h->rank, mine[3], mine[5], mine[0], mine[1]));
    return done(PTX_OK);
}

}  // namespace

// ptx_render of a band handle that owns a communicator: one whole frame, exchange included.
int render_band_nccl(ptx_handle *h) {
    if (int rc = comm_health(h)) return rc;
    Scene sc{};
    WaveBufs w{};
    bool pipe = false, moved = false;
    const bool xchg = motion_exchange(h);  // (before band_prepare: the same on every rank)
    if (int rc = band_prepare(h, sc, w, pipe, moved)) return rc;
    TimedLaunch *ft = nullptr;
    if (int rc = band_front(h, sc, w, ft, pipe, moved)) return rc;
    if (xchg) {
        NCCL_CHECK(h, rccl().group_start());
        const int rc = nccl_motion_halo(h);
        if (rc) {
            (void)rccl().group_end();
            return rc;
        }
        if (int r2 = group_end_wait(h)) return r2;
    }
    if (int rc = band_temporal(h, sc, w, pipe, moved)) return rc;
    hipStream_t xs;
    if (int rc = exchange_stream(h, xs)) return rc;
    NCCL_CHECK(h, rccl().group_start());
    const int rc = nccl_halo(h, xs);
    if (rc) {
        (void)rccl().group_end();
        return rc;
    }
    if (int r2 = group_end_wait(h)) return r2;
    if (h->halo_top) h->halo_bytes_sent += send_up(h).gb + send_up(h).rb;
    if (h->halo_bot) h->halo_bytes_sent += send_down(h).gb + send_down(h).rb;
    if (int r2 = halo_landed(h, xs)) return r2;
    return band_back(h, sc, w, ft);
}

// The exchange's proxy on one GPU (PTX_AB=HALO_PROXY_US=n, with PTX_FLAG_HALO_SKIP: timing
// only; the shipped library honours it): the band's edge rows copied into its own halo rows on the exchange stream (the same
// bytes an exchange moves, device to device), then a one-workgroup wait of n microseconds
// standing for the xGMI transfer (2 x 16.6 MB per direction at 153 GB/s: ~110 us), so the
// band's frame time shows where the exchange sits on its critical chain.
__global__ void halo_proxy_wait(uint32_t us) {
    const unsigned long long end = __builtin_amdgcn_s_memrealtime() + 100ull * us;  // (100 MHz)
    for (uint32_t i = 0; i < (1u << 24); ++i) {  // (bounded: every wave leaves)
        if (__builtin_amdgcn_s_memrealtime() >= end) break;
        __builtin_amdgcn_s_sleep(2);
    }
}
static int halo_proxy(ptx_handle *h, hipStream_t xs, uint32_t us) {
    if (h->halo_top) {
        const Rows s = send_up(h), r = recv_top(h);
        HIP_CHECK(h, hipMemcpyAsync(r.g, s.g, s.gb, hipMemcpyDeviceToDevice, xs));
        HIP_CHECK(h, hipMemcpyAsync(r.r, s.r, s.rb, hipMemcpyDeviceToDevice, xs));
    }
    if (h->halo_bot) {
        const Rows s = send_down(h), r = recv_bottom(h);
        HIP_CHECK(h, hipMemcpyAsync(r.g, s.g, s.gb, hipMemcpyDeviceToDevice, xs));
        HIP_CHECK(h, hipMemcpyAsync(r.r, s.r, s.rb, hipMemcpyDeviceToDevice, xs));
    }
    hipLaunchKernelGGL(halo_proxy_wait, dim3(1), dim3(64), 0, xs, us);
    HIP_CHECK(h, hipGetLastError());
    return PTX_OK;
}

// PTX_FLAG_HALO_SKIP: the same band frame without the exchange (the halo rows keep what they
// hold) -- a rank's band timed alone on one GPU (bench.py's band calibration, tools/band_alone.py).
int render_band_solo(ptx_handle *h) {
    Scene sc{};
    WaveBufs w{};
    bool pipe = false, moved = false;
    if (int rc = band_prepare(h, sc, w, pipe, moved)) return rc;
    TimedLaunch *ft = nullptr;
    if (int rc = band_front(h, sc, w, ft, pipe, moved)) return rc;
    if (int rc = band_temporal(h, sc, w, pipe, moved)) return rc;  // (a motion halo keeps what it holds)
    hipStream_t xs;
    if (int rc = exchange_stream(h, xs)) return rc;
    // (honoured by the shipped library: it only acts on a HALO_SKIP handle, a band timed alone)
    static const int proxy_us = env_knob("HALO_PROXY_US", 0);
    if (proxy_us > 0 && proxy_us <= 100000)
        if (int rc = halo_proxy(h, xs, (uint32_t)proxy_us)) return rc;
    if (int rc = halo_landed(h, xs)) return rc;
    return band_back(h, sc, w, ft);
}

}  // namespace ptx

extern "C" {

int ptx_comm_unique_id(void *id_out, size_t bytes) {
    if (!id_out || bytes != PTX_COMM_ID_BYTES) return PTX_E_INVALID;
    const Rccl &R = rccl();
    if (!R.ok) return PTX_E_HIP;
    ncclUniqueId id;
    if (R.get_unique_id(&id) != ncclSuccess) return PTX_E_HIP;
    std::memcpy(id_out, &id, sizeof id);
    return PTX_OK;
}

int ptx_comm_init(ptx_handle *h, const void *unique_id, size_t bytes, int rank, int world) {
    if (!h) return PTX_E_INVALID;
    if (!unique_id || bytes != PTX_COMM_ID_BYTES || world < 1 || rank < 0 || rank >= world)
        return fail(h, PTX_E_INVALID, "ptx_comm_init: bad id / rank %d / world %d", rank, world);
    if (h->comm) return fail(h, PTX_E_INVALID, "ptx_comm_init: the handle already owns a communicator");
    if ((h->halo_top && rank == 0) || (h->halo_bot && rank == world - 1))
        return fail(h, PTX_E_INVALID, "ptx_comm_init: band rows [%u,%u) need neighbours rank %d of %d cannot have",
                    h->cfg.row_begin, h->cfg.row_end, rank, world);
    if ((h->halo_top || h->halo_bot) && h->band_h < std::max(h->halo_top, h->halo_bot))
        return fail(h, PTX_E_INVALID, "ptx_comm_init: band of %u rows cannot feed a %u / %u-row halo", h->band_h,
                    h->halo_top, h->halo_bot);
    const Rccl &R = rccl();
    if (!R.ok) return fail(h, PTX_E_HIP, "RCCL unavailable: %s", R.why.c_str());
    HIP_CHECK(h, hipSetDevice(h->device));
    if (int rc = leave_alt(h)) return rc;  // band frames run on the first context's stream
    ncclUniqueId id;
    std::memcpy(&id, unique_id, sizeof id);
    ncclComm_t c = nullptr;
    if (R.init_rank_config && R.abort) {
        // non-blocking init, polled against a deadline: every rank exits with an error status
        // instead of hanging when a peer never joins (comm_wait)
        ncclConfig_t config = NCCL_CONFIG_INITIALIZER;
        config.blocking = 0;
        ncclResult_t r = R.init_rank_config(&c, world, id, rank, &config);
        if (r == ncclSuccess || r == ncclInProgress) r = comm_wait(c, comm_timeout_s());
        if (r != ncclSuccess) {
            if (c) (void)R.abort(c);
            if (r == ncclInProgress)
                return fail(h, PTX_E_HIP,
                            "ptx_comm_init: rank %d of %d: the communicator was not complete after %d s (a peer "
                            "rank never joined or failed); aborted",
                            rank, world, comm_timeout_s());
            return fail(h, PTX_E_HIP, "ptx_comm_init: ncclCommInitRankConfig (rank %d of %d): %s", rank, world,
                        R.error_string(r));
        }
    } else {
        NCCL_CHECK(h, R.init_rank(&c, world, id, rank));
    }
    h->comm = c;
    h->rank = rank;
    h->world = world;
    h->comm_broken = false;
    // every rank calls this collectively: the motion-halo decision's shared state (motion_exchange)
    // restarts in lockstep, whatever frames a rank rendered before
    h->band_frames = 0;
    std::memset(h->band_camera, 0, sizeof h->band_camera);
    if (int rc = check_neighbours(h)) {
        h->comm_broken = true;  // (the peers' view of this exchange is unknown: abort, never flush)
        comm_destroy(h);
        return rc;
    }
    return PTX_OK;
}

int ptx_comm_info(ptx_handle *h, int *rank, int *world, uint64_t *halo_bytes_sent) {
    if (!h) return PTX_E_INVALID;
    if (rank) *rank = h->comm ? h->rank : 0;
    if (world) *world = h->comm ? h->world : 1;
    if (halo_bytes_sent) *halo_bytes_sent = h->halo_bytes_sent;
    return PTX_OK;
}

int ptx_comm_init_all(ptx_handle *const *hs, int n) {
    if (!hs || n < 1 || n > 64) return PTX_E_INVALID;
    std::vector<int> devs(n);
    for (int i = 0; i < n; ++i) {
        if (!hs[i]) return PTX_E_INVALID;
        if (hs[i]->comm) return fail(hs[i], PTX_E_INVALID, "ptx_comm_init_all: the handle already owns a communicator");
        devs[i] = hs[i]->device;
        for (int k = 0; k < i; ++k)
            if (devs[k] == devs[i])
                return fail(hs[i], PTX_E_INVALID, "ptx_comm_init_all: two handles on device %d (RCCL needs one rank per GPU)",
                            devs[i]);
    }
    const Rccl &R = rccl();
    if (!R.ok) return fail(hs[0], PTX_E_HIP, "RCCL unavailable: %s", R.why.c_str());
    for (int i = 0; i < n; ++i) {
        HIP_CHECK(hs[i], hipSetDevice(hs[i]->device));
        if (int rc = leave_alt(hs[i])) return rc;
    }
    std::vector<ncclComm_t> comms(n);
    NCCL_CHECK(hs[0], R.init_all(comms.data(), n, devs.data()));
    for (int i = 0; i < n; ++i) {
        hs[i]->comm = comms[i];
        hs[i]->rank = i;
        hs[i]->world = n;
        hs[i]->band_frames = 0;
        std::memset(hs[i]->band_camera, 0, sizeof hs[i]->band_camera);
    }
    return PTX_OK;
}

int ptx_render_bands(ptx_handle *const *hs, int n, float *rgba_out) {
    if (!hs || n < 1 || n > 64) return PTX_E_INVALID;
    for (int i = 0; i < n; ++i)
        if (!hs[i]) return PTX_E_INVALID;
    ptx_handle *h0 = hs[0];
    const bool nccl = h0->comm != nullptr;
    for (int i = 0; i < n; ++i) {
        ptx_handle *h = hs[i];
        if (h->cfg.width != h0->cfg.width || h->cfg.height != h0->cfg.height || h->cfg.pipeline != h0->cfg.pipeline)
            return fail(h, PTX_E_INVALID, "ptx_render_bands: band %d differs in size or pipeline", i);
        if ((h->comm != nullptr) != nccl)
            return fail(h, PTX_E_INVALID, "ptx_render_bands: either every band owns a communicator or none");
        if (nccl && (h->rank != i || h->world != n))
            return fail(h, PTX_E_INVALID, "ptx_render_bands: band %d is rank %d of %d", i, h->rank, h->world);
        if (i && hs[i - 1]->cfg.row_end != h->cfg.row_begin)
            return fail(h, PTX_E_INVALID, "ptx_render_bands: band %d does not start where band %d ends", i, i - 1);
        if ((i == 0 && h->halo_top) || (i == n - 1 && h->halo_bot))
            return fail(h, PTX_E_INVALID, "ptx_render_bands: the bands do not cover the halo rows of the ends");
        if (h->band_h < h->reuse_radius && n > 1)
            return fail(h, PTX_E_INVALID, "ptx_render_bands: band %d has fewer rows than the reuse radius", i);
    }
    // the bands agree on the motion halo before any of them enqueues work (motion_exchange)
    const bool xchg = motion_exchange(h0);
    for (int i = 1; i < n; ++i)
        if (motion_exchange(hs[i]) != xchg)
            return fail(hs[i], PTX_E_INVALID,
                        "ptx_render_bands: band %d %s the motion halo and band 0 %s (different camera or frame count)",
                        i, xchg ? "skips" : "needs", xchg ? "needs it" : "skips it");
    std::vector<Scene> sc(n);
    std::vector<WaveBufs> w(n);
    std::vector<TimedLaunch *> ft(n);
    std::vector<hipStream_t> xs(n);
    std::vector<char> pipe(n), moved(n);
    for (int i = 0; i < n; ++i) {
        HIP_CHECK(hs[i], hipSetDevice(hs[i]->device));
        bool p = false, m = false;
        if (int rc = band_prepare(hs[i], sc[i], w[i], p, m)) return rc;
        pipe[i] = p;
        moved[i] = m;
        if (int rc = band_front(hs[i], sc[i], w[i], ft[i], p, m)) return rc;
    }
    if (xchg) {  // the motion halo: the neighbours' rows of the previous frame's spatial output
        if (nccl) {
            NCCL_CHECK(h0, rccl().group_start());
            int rc = PTX_OK;
            for (int i = 0; i < n && !rc; ++i) rc = nccl_motion_halo(hs[i]);
            NCCL_CHECK(h0, rccl().group_end());
            if (rc) return rc;
        } else {
            // peer copies once the neighbour's previous frame is complete (its ev_prev); the
            // neighbours' spatial passes, which rewrite those rows, wait for ev_mhalo (below)
            for (int i = 0; i < n; ++i) {
                ptx_handle *h = hs[i];
                HIP_CHECK(h, hipSetDevice(h->device));
                if (i > 0 && h->halo_top) {
                    ptx_handle *a = hs[i - 1];
                    const HistRows s = hist_send_down(a), r = hist_recv_top(h);
                    if (s.bytes != r.bytes) return fail(h, PTX_E_INVALID, "motion halo of band %d does not match band %d", i, i - 1);
                    HIP_CHECK(h, hipStreamWaitEvent(h->stream, a->ev_prev, 0));
                    HIP_CHECK(h, hipMemcpyPeerAsync(r.p, h->device, s.p, a->device, r.bytes, h->stream));
                }
                if (i + 1 < n && h->halo_bot) {
                    ptx_handle *b = hs[i + 1];
                    const HistRows s = hist_send_up(b), r = hist_recv_bottom(h);
                    if (s.bytes != r.bytes) return fail(h, PTX_E_INVALID, "motion halo of band %d does not match band %d", i, i + 1);
                    HIP_CHECK(h, hipStreamWaitEvent(h->stream, b->ev_prev, 0));
                    HIP_CHECK(h, hipMemcpyPeerAsync(r.p, h->device, s.p, b->device, r.bytes, h->stream));
                }
                if (!h->ev_mhalo) HIP_CHECK(h, hipEventCreateWithFlags(&h->ev_mhalo, hipEventDisableTiming));
                HIP_CHECK(h, hipEventRecord(h->ev_mhalo, h->stream));
            }
        }
    }
    for (int i = 0; i < n; ++i) {
        HIP_CHECK(hs[i], hipSetDevice(hs[i]->device));
        if (int rc = band_temporal(hs[i], sc[i], w[i], pipe[i], moved[i])) return rc;
    }
    for (int i = 0; i < n; ++i)
        if (int rc = exchange_stream(hs[i], xs[i])) return rc;
    if (nccl) {
        NCCL_CHECK(h0, rccl().group_start());
        int rc = PTX_OK;
        for (int i = 0; i < n && !rc; ++i) rc = nccl_halo(hs[i], xs[i]);
        NCCL_CHECK(h0, rccl().group_end());
        if (rc) return rc;
    } else {
        // peer copies: band i pulls its halo rows from its neighbours' band rows once their
        // front passes are done
        for (int i = 0; i < n; ++i) {
            ptx_handle *h = hs[i];
            HIP_CHECK(hs[i], hipSetDevice(h->device));
            if (i > 0 && h->halo_top) {
                ptx_handle *a = hs[i - 1];
                const Rows s = send_down(a), r = recv_top(h);
                if (a->halo_bot != h->halo_top || s.gb != r.gb || s.rb != r.rb)
                    return fail(h, PTX_E_INVALID, "halo of band %d does not match band %d", i, i - 1);
                HIP_CHECK(h, hipStreamWaitEvent(xs[i], a->ev_front, 0));
                HIP_CHECK(h, hipMemcpyPeerAsync(r.g, h->device, s.g, a->device, r.gb, xs[i]));
                HIP_CHECK(h, hipMemcpyPeerAsync(r.r, h->device, s.r, a->device, r.rb, xs[i]));
            }
            if (i + 1 < n && h->halo_bot) {
                ptx_handle *b = hs[i + 1];
                const Rows s = send_up(b), r = recv_bottom(h);
                if (b->halo_top != h->halo_bot || s.gb != r.gb || s.rb != r.rb)
                    return fail(h, PTX_E_INVALID, "halo of band %d does not match band %d", i, i + 1);
                HIP_CHECK(h, hipStreamWaitEvent(xs[i], b->ev_front, 0));
                HIP_CHECK(h, hipMemcpyPeerAsync(r.g, h->device, s.g, b->device, r.gb, xs[i]));
                HIP_CHECK(h, hipMemcpyPeerAsync(r.r, h->device, s.r, b->device, r.rb, xs[i]));
            }
        }
    }
    for (int i = 0; i < n; ++i) {
        HIP_CHECK(hs[i], hipSetDevice(hs[i]->device));
        if (int rc = halo_landed(hs[i], xs[i])) return rc;
    }
    for (int i = 0; i < n; ++i) {
        HIP_CHECK(hs[i], hipSetDevice(hs[i]->device));
        if (xchg && !nccl) {  // (the neighbours have copied this band's history rows)
            if (i > 0) HIP_CHECK(hs[i], hipStreamWaitEvent(hs[i]->stream, hs[i - 1]->ev_mhalo, 0));
            if (i + 1 < n) HIP_CHECK(hs[i], hipStreamWaitEvent(hs[i]->stream, hs[i + 1]->ev_mhalo, 0));
        }
        if (int rc = band_back(hs[i], sc[i], w[i], ft[i])) return rc;
    }
    if (!nccl) {  // the next frame's front passes must not overwrite rows a neighbour still copies
        for (int i = 0; i < n; ++i) {
            HIP_CHECK(hs[i], hipSetDevice(hs[i]->device));
            if (i > 0) HIP_CHECK(hs[i], hipStreamWaitEvent(hs[i]->stream, hs[i - 1]->ev_halo, 0));
            if (i + 1 < n) HIP_CHECK(hs[i], hipStreamWaitEvent(hs[i]->stream, hs[i + 1]->ev_halo, 0));
        }
    }
    if (rgba_out) {  // the bands' accumulated images, in order (rows row_begin(0) .. row_end(n-1))
        size_t off = 0;
        for (int i = 0; i < n; ++i) {
            ptx_handle *h = hs[i];
            HIP_CHECK(hs[i], hipSetDevice(h->device));
            if (int rc = read_to_host(h, (char *)rgba_out + off, h->d_accum.p, h->d_accum.bytes)) return rc;
            off += h->d_accum.bytes;
        }
    }
    return PTX_OK;
}

}  // extern "C"

namespace ptx {
const char *comm_library() { return g_comm_library.c_str(); }
// A communicator that timed out or reported an error is aborted: ncclCommDestroy would flush
// operations a dead or absent peer never matches.  A healthy non-blocking one is finalized
// against the deadline first (an abort if that does not complete), then destroyed.
void comm_destroy(ptx_handle *h) {
    if (h->comm && rccl().ok) {  // (no communicator: RCCL is never opened)
        const Rccl &R = rccl();
        ncclComm_t c = (ncclComm_t)h->comm;
        bool gone = false;
        if (h->comm_broken && R.abort) {
            (void)R.abort(c);
            gone = true;
        } else if (R.finalize) {
            ncclResult_t r = R.finalize(c);
            if (r == ncclInProgress) r = comm_wait(c, comm_timeout_s());
            if (r != ncclSuccess && R.abort) {
                (void)R.abort(c);
                gone = true;
            }
        }
        if (!gone) (void)R.destroy(c);
    }
    h->comm = nullptr;
    h->comm_broken = false;
    if (h->xstream) {
        (void)hipStreamSynchronize(h->xstream);
        (void)hipStreamDestroy(h->xstream);
    }
    h->xstream = nullptr;
    if (h->ev_front) (void)hipEventDestroy(h->ev_front);
    if (h->ev_halo) (void)hipEventDestroy(h->ev_halo);
    if (h->ev_mhalo) (void)hipEventDestroy(h->ev_mhalo);
    h->ev_front = h->ev_halo = h->ev_mhalo = nullptr;
}
}  // namespace ptx
