// ptx_internal.h -- the handle behind the C ABI (include/ptx.h) and the host helpers shared
// by ptx_api.cpp (single-handle entry points) and ptx_comm.cpp (RCCL communicator, halo
// exchange and multi-band frames).  Not installed; not part of the ABI.
#pragma once
#include <hip/hip_runtime.h>

#include <string>

#include "../../include/ptx.h"
#include "ptx_launch.h"

namespace ptx {
constexpr int kPasses = 16;
constexpr int kEventRing = 256;  // ~15 event pairs per wavefront frame
struct DevBuf {
    void *p = nullptr;
    size_t bytes = 0;
};
struct TimedLaunch {
    hipEvent_t start = nullptr, stop = nullptr;
    int pass = -1;
    bool pending = false;
};
}  // namespace ptx

using namespace ptx;

// Internal pass codes (launch_wave_parts): the temporal pass in two parts -- its shift jobs
// (start, trace rounds; they read only this frame's PT_1 output) and its combine (reads the
// previous frame's spatial output) -- so a pipelined frame runs the jobs before waiting for
// the previous frame.
constexpr int kPassTemporalJobs = 0x100, kPassTemporalCombine = 0x101;
// the temporal pass of a frame whose camera moved since the history's (wtmotion_* / wgim_*),
// run whole after the wait for the previous frame (a split form measured slower: DESIGN §4)
constexpr int kPassTemporalMotion = 0x102;
inline bool is_motion_pass(int p) {
    return p == kPassTemporalMotion;
}

struct ptx_handle {
    ptx_config cfg{};
    int device = 0;
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;
    std::string err;

    // reference arrays (host copies: the derived layout is rebuilt when offsets change)
    std::vector<uint32_t> scene, geometry, accel;
    DevBuf d_scene, d_geometry;
    // derived MI355X layout
    DevBuf d_tris, d_nodes, d_subs, d_insts, d_mats, d_tverts;
    uint32_t n_tris = 0, n_nodes = 0, n_inst = 0, n_subs = 0, max_depth = 0, stack_depth = 0;
    uint32_t layout_key[8] = {0};
    bool layout_valid = false;
    bool scene_loaded = false;
    // frame
    uint32_t uniform[PTX_UNIFORM_WORDS] = {0};
    bool frame_set = false;
    // band buffers; the G-buffer and PT_1 reservoirs carry halo_top / halo_bot extra rows
    // (reuse pipeline on a band: the spatial pass reads neighbours up to reuse_radius away)
    uint32_t band_h = 0, halo_top = 0, halo_bot = 0;
    DevBuf d_gbuf, d_res, d_accum, d_counters, d_queue;
    // reuse pipeline: spatial output / history, shift-job state and results
    DevBuf d_hist, d_jstate, d_jres, d_nbr;
    // the temporal pass's shift jobs, per frame context: its jobs run before the previous
    // frame's spatial pass (which owns d_jstate / d_jres) has finished
    DevBuf d_tjstate, d_tjres;
    // reservoir size in uint4 (8: the reference's 128-byte Reservoir; 4: the GI reservoir)
    // and the GI pipeline's per-pixel direct light
    uint32_t res_u4 = 8;
    DevBuf d_direct;
    // the wave state holds the PT_1 pass of the reservoirs in d_res (enqueued, nothing since
    // rewrote them): the reuse temporal pass may read its path hits instead of re-tracing
    bool init_state_valid = false;
    // d_nbr holds the summaries of the band's reservoirs as the temporal pass left them
    // (set by that pass, dropped by anything else that rewrites G-buffer or reservoirs)
    bool nbr_valid = false;
    // DI reuse pipeline: primary-hit surface records of the band (+ halo rows), 32 B per pixel
    // (WaveBufs::surf); surf_valid: the band rows describe the current G-buffer and scene (PT_1
    // wrote them; a reuse pass runs wsurface first otherwise; halo rows come with the summaries)
    DevBuf d_surf;
    bool surf_valid = false;
    uint32_t reuse_radius = 0, reuse_neighbors = 0, temporal_cap = 0;
    // set while a pipelined TEST_MCPT frame's pass is enqueued: its path colours go to this
    // context's d_direct, mixed into d_accum after the previous frame's (wave_mix_frame)
    float4 *mcpt_color = nullptr;
    bool hist_valid = false;           // d_hist holds the previous frame of this camera/scene
    uint32_t hist_camera[19] = {0};    // uniform words 4..22 of the frame that wrote d_hist
    // the camera moved since d_hist's frame (whole-image DI reuse handles): ptx_render reprojects
    // the history (the motion temporal pass) with d_psurf = that frame's primary-hit surface
    // records, copied on its stream before the next frame's G-buffer may overwrite them
    bool hist_moved = false;
    DevBuf d_psurf;
    DevBuf d_qrays, d_qhits;  // staging for ptx_trace (host arrays)
    // wavefront variant: pixel state, ray queue + ping-pong results / active lists, counters
    DevBuf d_wstate, d_wrays, d_wres0, d_wres1, d_wres2, d_wact0, d_wact1, d_wctr;
    DevBuf d_wpool;  // Visibility restart pools of the dynamic-batch trace launches (WaveBufs::pool)
    size_t wave_ray_cap = 0;
    // second stream: the two halves of the segments run as independent launch sequences so
    // one half's latency-bound traces overlap the other's ALU-bound shading
    static constexpr int kMaxSplit = 4;  // GPU_MAX_HW_QUEUES is 4 on the target boxes
    hipStream_t sub[kMaxSplit] = {nullptr, nullptr, nullptr, nullptr};  // sub[0] unused (= stream)
    hipEvent_t ev_fork = nullptr, ev_join[kMaxSplit] = {nullptr, nullptr, nullptr, nullptr};
    // queue slots wave_buffers allocated (WaveBufs::cnt_stride)
    uint32_t wave_slots = 0;
    // row census (PTX_FLAG_ROW_CENSUS): kCensusWords u64 per G-buffer tile row + queue slot
    DevBuf d_census;
    uint32_t census_blocks = 0;
    // diagnostic build (PTX_WG_TIMES) with PTX_WGT=1 in the environment: per-wave timing records
    DevBuf d_wgt;
    // Frame pipelining (pipelined(): reuse handles on their own streams, whole-image or band): two frames
    // in flight, each with its own G-buffer, reservoirs, neighbour summaries, wave state,
    // queues and streams.  Frame N's G-buffer + PT_1 run beside frame N-1's spatial pass + PT_4;
    // its temporal pass (which reads frame N-1's spatial output, d_hist, and reuses the shared
    // shift-job buffers) waits for ev_prev, recorded on N-1's stream when N was enqueued.
    // ptx_render swaps the members above with `alt` per frame, so everything else always sees
    // the latest frame's buffers; the shared ones (accumulation, history, jobs, scene) never move.
    struct FrameCtx {
        DevBuf gbuf, res, nbr, surf, wstate, wrays, wres0, wres1, wres2, wact0, wact1, wctr, tjstate, tjres, direct;
        size_t wave_ray_cap = 0;
        uint32_t wave_slots = 0;
        hipStream_t stream = nullptr;
        hipStream_t sub[kMaxSplit] = {nullptr, nullptr, nullptr, nullptr};
        hipEvent_t ev_fork = nullptr, ev_join[kMaxSplit] = {nullptr, nullptr, nullptr, nullptr};
        bool init_state_valid = false, nbr_valid = false, surf_valid = false;
    } alt, alt2;  // (alt2: the third context when pipe_depth() == 3; swap_frame_ctx rotates)
    bool alt_active = false;      // the members above hold a context other than the first
    int ctx_idx = 0;              // which context the members above hold (0: own_stream's)
    hipStream_t alt_stream = nullptr, alt2_stream = nullptr;  // the other contexts' streams (owned)
    hipEvent_t ev_prev = nullptr;
    // multi-GPU (ptx_comm.cpp): the RCCL communicator this handle owns (ncclComm_t), its
    // rank and world; the halo exchange stream and its fork / done events
    void *comm = nullptr;
    int rank = 0, world = 1;
    hipStream_t xstream = nullptr;
    hipEvent_t ev_front = nullptr, ev_halo = nullptr;
    // ptx_render_bands without communicators, moved camera: this band has copied its motion halo
    // (the neighbours' previous spatial output) -- their spatial passes overwrite it after this
    hipEvent_t ev_mhalo = nullptr;
    uint64_t halo_bytes_sent = 0;  // halo bytes this handle's communicator has sent (ptx_comm_info)
    // the communicator timed out or reported an error: torn down with ncclCommAbort (a destroy
    // would flush operations a dead peer never matches)
    bool comm_broken = false;
    // the motion-halo decision of band frames, from state every rank shares (the uniform sequence
    // and the frame count, never the per-rank history state): band frames rendered and the camera
    // words (uniform 4..22) of the last one
    uint64_t band_frames = 0;
    uint32_t band_camera[19] = {0};
    // ptx_present's canvas on the device; the pinned staging buffer of read_to_host
    DevBuf d_canvas;
    void *host_stage = nullptr;
    size_t host_stage_bytes = 0;
    // ptx_present_async: its own device canvas and pinned host copy (a blocking ptx_present may
    // run while it is in flight), the event after its copy, and what is in flight
    DevBuf d_canvas_async;
    void *present_host = nullptr;
    size_t present_host_bytes = 0, present_bytes = 0;
    hipEvent_t ev_present = nullptr;
    bool present_pending = false;
    // stats
    TimedLaunch ring[kEventRing];
    int ring_pos = 0;
    double ms_total[kPasses] = {};
    uint64_t launches[kPasses] = {};
    uint64_t frames = 0;
};

namespace ptx {
int fail(ptx_handle *h, int code, const char *fmt, ...);
#define HIP_CHECK(h, expr)                                                                                   \
    do {                                                                                                     \
        hipError_t e_ = (expr);                                                                              \
        if (e_ != hipSuccess) return fail((h), PTX_E_HIP, "%s: %s (%s:%d)", #expr, hipGetErrorString(e_),      \
                                          __FILE__, __LINE__);                                               \
    } while (0)
void free_buf(DevBuf &b);
int alloc_buf(ptx_handle *h, DevBuf &b, size_t bytes);
// device -> caller memory after the work enqueued on h->stream (pinned staging, blocking)
int read_to_host(ptx_handle *h, void *dst, const void *src, size_t bytes);
// first band row of the halo-extended G-buffer / reservoir allocations
uint4 *gbuf_band(ptx_handle *h);
uint4 *res_band(ptx_handle *h);
bool has_reuse(const ptx_handle *h);
int build_layout(ptx_handle *h);
Scene make_scene(ptx_handle *h);
void resolve_event(TimedLaunch &t, ptx_handle *h);
int wave_buffers(ptx_handle *h, WaveBufs &w);
int reuse_buffers(ptx_handle *h);
// Passes over the launch's segments as K independent sequences on K streams, joined on
// h->stream.  summaries: the spatial pass's neighbour-summary prologue (halo rows) runs
// first; an interior tile set (halo not yet received) runs without it.  then: a second tile
// set (disjoint queue slots) each stream runs after its share of the first, once
// `then_wait` has fired -- no join in between.
hipError_t launch_wave_parts(ptx_handle *h, const Scene &sc, const WaveBufs &w, const int *passes, int npasses,
                             bool summaries = true, const WaveBufs *then = nullptr, hipEvent_t then_wait = nullptr);
// the neighbour summaries of the halo rows (or of everything when the band's are stale)
hipError_t spatial_summaries(ptx_handle *h, hipStream_t st);
void mark_history(ptx_handle *h);
int motion_prepare(ptx_handle *h, hipStream_t st);
uint4 *hist_band(ptx_handle *h);
// frame pipelining: whether ptx_render runs this handle's frames two in flight; wait for both
// frames' streams (before anything that replaces shared buffers or the stream)
bool pipelined(const ptx_handle *h);
int quiesce(ptx_handle *h);
// the second frame context's G-buffer, reservoirs and stream; swap the two contexts
int ensure_alt(ptx_handle *h);
// frames in flight when pipelined: 2, or 3 with PTX_AB=PIPE_DEPTH=3 (A/B)
int pipe_depth();
void swap_frame_ctx(ptx_handle *h);
// back to the first frame context (quiesce + swap) before the handle's stream or mode changes
int leave_alt(ptx_handle *h);
// ptx_comm.cpp: a frame of a band handle that owns a communicator; a band frame without the
// exchange (PTX_FLAG_HALO_SKIP, timing only); the communicator's teardown
int render_band_nccl(ptx_handle *h);
int render_band_solo(ptx_handle *h);
void comm_destroy(ptx_handle *h);
// the communicator library ptx_comm.cpp opened ("" before the first ptx_comm_* call), for ptx_build_info
const char *comm_library();
}  // namespace ptx
