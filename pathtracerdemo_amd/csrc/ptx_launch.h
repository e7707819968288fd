// ptx_launch.h -- host-side launch wrappers exported by ptx_kernels.hip to ptx_api.cpp.
#pragma once

#include <hip/hip_runtime.h>

#include "ptx_device.h"

namespace ptx {

constexpr int kTile = 16;
constexpr int kBlock = 256;

// Runtime switches are read from ONE environment variable, PTX_AB, a comma-separated list of
// KEY or KEY=int; a key that is absent gives `dflt`.  env_knob (ptx_api.cpp): the few the
// shipped library honours, each covered by a test -- COMM_TIMEOUT_S (test_gpu_loopback.py),
// DEBUG_FILL (test_gpu_debug_fill.py), HALO_PROXY_US (a band timed alone with PTX_FLAG_HALO_SKIP:
// the exchange's one-GPU stand-in, test_gpu_bands.py).  Any other key in PTX_AB is named on stderr
// and in ptx_build_info.  ab_knob: the A/B and diagnostic switches of the measurement builds
// (make variant NAME=x ALT_DEFS=-DPTX_AB_BUILD, make wgt; selected with PTX_LIB_PATH) -- in the
// shipped library every one is its default, a compile-time constant, and the losing branches
// fold away.  bench.py echoes PTX_AB (and any other PTX_* variable) in its line.
int env_knob(const char *key, int dflt);
#ifdef PTX_AB_BUILD
inline int ab_knob(const char *key, int dflt) { return env_knob(key, dflt); }
#else
constexpr int ab_knob(const char *, int dflt) { return dflt; }
#endif

// dynamic LDS bytes for a traversal stack of `depth` entries per thread
inline size_t stack_lds_bytes(uint32_t depth) { return (size_t)depth * kBlock * sizeof(uint32_t); }

hipError_t launch_gbuffer(const Scene &sc, uint4 *gbuf, uint32_t stack_depth, hipStream_t s);
hipError_t launch_init(const Scene &sc, const uint4 *gbuf, uint4 *reservoir, uint32_t stack_depth, hipStream_t s);
hipError_t launch_final(const Scene &sc, const uint4 *gbuf, const uint4 *reservoir, float4 *accum,
                        uint32_t stack_depth, hipStream_t s);
hipError_t launch_mcpt(const Scene &sc, float4 *accum, uint32_t stack_depth, hipStream_t s);
// the reference's render pass: the Scene texture's fixed 600 x 450 window onto a cw x ch unorm8 canvas
hipError_t launch_present(const float4 *tex, uint32_t W, uint32_t H, uint32_t cw, uint32_t ch, bool bgra,
                          uint32_t *out, hipStream_t s);

// closest-hit queries for a ray array (ptx_kernels.hip)
hipError_t launch_trace_rays(const Scene &sc, const float4 *rays, float4 *hits, uint32_t n, int eps_mode,
                             uint32_t stack_depth, hipStream_t s);

// wavefront variant (ptx_wave.hip): the default.  A pass is a fixed sequence of rounds:
// logic round 0 (start), then {trace r, logic r+1} for r < kWaveRounds[pass].  Every
// launch has one workgroup per segment; queue lengths live on the device
// (cnt[(2r) * nseg + j] pixels of segment j active after logic round r, cnt[(2r+1) *
// nseg + j] rays it emitted), so the host never synchronises inside a pass.
constexpr uint32_t kWaveStateSlots = 10u;  // float4 per pixel (PT_1 needs the most)
// PT_1 state slots the reuse pipeline's temporal pass reads (vertex 2 / 3 hit compacts, the
// selected NEE candidate's Visibility or -1 for an env candidate): ptx_wave.hip IS_*
constexpr uint32_t kStateCs2 = 7u, kStateCs3 = 8u, kStateTsel = 9u;
constexpr uint32_t kWaveSegPixels = 768u;  // padded pixels per segment (12 8x8 tiles); 768 > 512 > 1024 > 256
constexpr int kWaveRoundsInit = 3, kWaveRoundsFinal = 3, kWaveRoundsMcpt = 4;
constexpr int kWaveMaxRounds = 5;
// dynamic trace batches: per (tile set, launch sequence, round) kDynHeads dequeue heads, one
// per XCD, each on its own 128-byte line (kDynStride words): one device-scope head saturates
// at ~88 dequeues/us (MI355X_MICROARCH.md, dequeue), far below a trace launch's demand
constexpr uint32_t kDynHeads = 8u, kDynStride = 32u;
constexpr uint32_t kDynRoundWords = kDynHeads * kDynStride;
constexpr uint32_t kDynCounters = 2u * 4u * kWaveMaxRounds * kDynRoundWords;
struct WaveBufs {
    float4 *state;       // kWaveStateSlots * npix, SoA
    uint32_t npix;       // pixels of the band
    uint32_t seg_px;     // padded pixels per segment
    uint32_t nseg;       // segments of the band
    uint32_t seg_base;   // first segment of this launch sequence (workgroup j -> segment
    uint32_t seg_count;  //   seg_base + j), and how many it covers
    uint32_t cluster;    // segment layout: 16/cluster runs of `cluster` adjacent 8x8 tiles
    uint32_t ray_stride; // ray slots per segment (seg_px * max rays per pixel per round)
    float4 *rays;        // 2 float4 per ray: {o, remain}, {d, kind}
    float4 *res[3];      // 2 float4 per ray, ping-pong by round parity (nres = 2) or one per
    uint32_t nres;       // round (nres = 3: the spatial reuse pass, whose combine reads every
                         // round's light-ray results; res_buf)
    uint32_t *act[2];    // active pixel / job lists (nseg * act_stride), ping-pong
    uint32_t act_stride; // list entries per segment (seg_px; seg_px * jobs per pixel for reuse)
    uint32_t *cnt;       // 2 * kWaveMaxRounds * nseg counts
    uint32_t trace_waves;  // trace_queue occupancy target (waves per SIMD; 4 or 5, per pipeline)
    uint32_t trace_split;  // workgroups per ray segment in trace_queue (batches of 256 rays dealt
                           // round-robin over them): a segment's rays are not one serial chain
    // Tile set of the launch: virtual tile v (what the segments spread over) is band tile
    // v < ntile0 ? tile0 + v : tile1 + (v - ntile0), for v < ntile0 + ntile1 (8x8 tiles in
    // raster order).  Default: the whole band.  A band's spatial pass runs its interior rows
    // and its halo-dependent edge rows as two tile sets (the exchange overlaps the first).
    uint32_t tile0, ntile0, tile1, ntile1;
    // Queue memory: virtual segment j lives in physical slot seg_phys + j (ray / result / list
    // storage, count words at cnt[(2r or 2r+1) * cnt_stride + slot]).  Two tile sets in flight
    // at once use disjoint physical slots.
    uint32_t seg_phys, cnt_stride;
    // Dynamic trace batches (trace_queue): this launch sequence's kWaveMaxRounds groups of
    // kDynHeads dequeue heads (round r at dyn + r * kDynRoundWords; the logic round that emits
    // trace round r zeroes them in seg_begin); nullptr = one slot per trace workgroup.
    uint32_t *dyn;
    // DI reuse pipeline: primary-hit surface records (2 uint4 per pixel, first band row; halo
    // rows at negative / >= npix indices), written by winit_start; nullptr otherwise
    uint4 *surf;
};
// dynamic trace batches: one workgroup per slot, at most kDynMaxGroups (the chip holds ~1024 trace
// workgroups; later ones find the list drained and leave)
constexpr uint32_t kDynMaxGroups = 1024u, kDynMaxSlots = 4096u;
// occ_only: every query of the round is Q_OCC (any-hit kernel instance)
hipError_t wave_trace(const Scene &sc, const WaveBufs &w, int round, int eps_mode, uint32_t stack_depth,
                      hipStream_t s, bool occ_only = false);
hipError_t wave_init_round(const Scene &sc, const WaveBufs &w, int round, const uint4 *gbuf, uint4 *reservoir,
                           hipStream_t s);
// PT_4 of the reuse pipeline in one launch, replays walked inline (scene tables in LDS)
hipError_t wave_final_one(const Scene &sc, const WaveBufs &w, const uint4 *gbuf, const uint4 *reservoir, float4 *accum,
                          uint32_t depth, hipStream_t s);
hipError_t wave_final_round(const Scene &sc, const WaveBufs &w, int round, const uint4 *gbuf, const uint4 *reservoir,
                            float4 *accum, hipStream_t s);
hipError_t wave_gbuffer(const Scene &sc, const WaveBufs &w, uint4 *gbuf, uint32_t stack_depth, hipStream_t s);
hipError_t launch_trace_rays_sm(const Scene &sc, const float4 *rays, float4 *hits, uint32_t n, int eps_mode,
                                uint32_t stack_depth, hipStream_t s);
// color: nullptr mixes every finished path into accum (WriteColor); else the path colours go to
// color (a pipelined frame) and wave_mix_frame mixes them in after the previous frame's
hipError_t wave_mcpt_round(const Scene &sc, const WaveBufs &w, int round, float4 *accum, float4 *color,
                           hipStream_t s);
hipError_t wave_mix_frame(const Scene &sc, const float4 *color, float4 *accum, hipStream_t s);

// reuse passes (ptx_reuse.hip): round 0 start, 1..kWaveRoundsReuse step, then combine
constexpr int kWaveRoundsReuse = 3;
struct ReuseArgs {
    const uint4 *gbuf;  // G-buffer of the band's first row; halo rows at negative / >= npix indices
    uint4 *cur;         // PT_1 reservoirs (temporal output in place), same addressing
    uint4 *hist;        // spatial output = PT_4 input = next frame's history, cur's addressing
                        // (a band's halo rows: the neighbours' previous spatial output, motion pass)
    float4 *jstate;     // shift-job state, 6 float4 slots x njobs (SoA)
    float4 *jres;       // per job: {f (PathContribution, rgb), q} (q = 0: invalid); p_hat = Luminance(f)
    uint32_t njobs, jpp;  // jobs of the pass (npix * jpp), jobs per pixel
    // job id of (pixel, slot) = pix * jpx + slot * jslot: slot planes (jpx 1, jslot npix), so a
    // wave's jobs -- one 8x8 tile, one slot -- read and write whole 128-byte lines of the SoA
    // state (pixel-major, jpx = jpp: 16-byte pieces 16 * jpp bytes apart)
    uint32_t jpx, jslot;
    uint32_t radius, neighbors, cap, hist_valid;
    uint32_t use_init;  // temporal: this frame's PT_1 wave state (path hits, NEE Visibility) is in w.state
    const uint4 *nbr;   // spatial: per-pixel neighbour summary (wave_reuse_summary), cur's addressing
    uint4 *nbr_out;     // the same buffer: the temporal pass writes its output's summaries
    const uint4 *surf;  // primary-hit surface records (WaveBufs::surf), cur's addressing
    // spatial: a job's light segment is finished by the combine -- every light ray a job emits
    // leaves {ray index, result buffer, -, kJobPending} in jres (the pass keeps one result
    // buffer per trace round, WaveBufs::nres = 3), and the combine reads its Visibility result
    // and the job's F slot itself (wjob_step's phase-1 arithmetic); no step launch after the
    // last trace round, and the steps see heavy jobs only
    uint32_t fold_last;
    uint32_t ray_cap;   // ray slots of the wave buffers: a stale jres word (a slot the combine
                        // loads but does not use) never sends the fold's gather out of bounds
    // temporal reuse under camera motion (wtmotion_*, ptx_reuse.hip): the previous frame's
    // VP^-1 (its camera points) and VP (the reprojection), its primary-hit surface records
    // (cur's addressing); motion = 1 selects the pass.  hist / psurf hold the previous frame's
    // band rows [prev_row_lo, prev_row_hi) (band-relative: a band's motion halo, the whole image
    // [0, H)); a pixel reprojected outside them has no history (and counts in *clip)
    uint32_t motion;
    float vpinv_prev[16], vp_prev[16];
    const uint4 *psurf;
    int32_t prev_row_lo, prev_row_hi;
    unsigned long long *clip;  // nullptr: not counted
};
// the motion temporal pass's jobs per pixel: the canonical sample at home, the reprojected
// history sample here, the canonical sample in the previous frame's domain
constexpr uint32_t kMotionJobs = 3u;
constexpr uint32_t kJobPending = 0xFFFFFFFFu;  // jres.w of such a job (a NaN: never a stored q)
// The fold keeps ONE result buffer per trace round (WaveBufs::res[0..2], res_sel = round % 3):
// a fourth round would overwrite the round-0 light results the combine still reads.
static_assert(kWaveRoundsReuse <= 3, "fold_last: one result buffer per reuse trace round");
// rounds of {trace, step} between a reuse pass's start and combine launches
int reuse_rounds(int pass_temporal, const ReuseArgs &A);
hipError_t wave_reuse_round(const Scene &sc, const WaveBufs &w, int pass_temporal, int round, const ReuseArgs &A,
                            hipStream_t s);
// Spatial pass prologue over every band + halo pixel (npx of them, from the first halo row):
// the 16-byte neighbour summary {p_hat, q, W, valid | length | C} the spatial kernels gather
// instead of a G-buffer line and a reservoir line per neighbour.
// With `surf`, the same pixels' primary-hit surface records too (halo rows just received).
hipError_t wave_reuse_summary(const Scene &sc, const uint4 *gbuf, const uint4 *res, uint4 *nbr, uint4 *surf,
                              size_t npx, hipStream_t s);
// The surface records of the launch's segments from the G-buffer (a reuse pass whose band
// records are stale: no PT_1 since the G-buffer or the scene changed)
hipError_t wave_surface(const Scene &sc, const WaveBufs &w, const uint4 *gbuf, hipStream_t s);

// ReSTIR GI (ptx_gi.hip; pipeline PTX_PIPELINE_RESTIR_GI): pass 0 init (logic rounds 0..2,
// traces between), 1 temporal (one launch), 2 spatial (start, trace, combine), 3 final,
// 4 temporal under camera motion (start, trace, combine).
constexpr int kWaveRoundsGiInit = 2, kWaveRoundsGiSpatial = 1;
constexpr uint32_t kGiResU4 = 4u;  // 64-byte GI reservoir (oracle/pt_oracle_gi.c)
struct GiArgs {
    const uint4 *gbuf;  // G-buffer of the band's first row; halo rows at negative / >= npix indices
    uint4 *cur;         // GI reservoirs (init output, temporal output in place), same addressing
    uint4 *hist;        // spatial output = final input = next frame's history (band only)
    float4 *direct;     // per-pixel direct light (band)
    float4 *accum;      // accumulated radiance (band)
    uint32_t *jray;     // spatial: per job its occlusion ray's index, or 0xffffffff (no path)
    uint32_t jpp;       // spatial jobs per pixel (2 * neighbors)
    uint32_t jpx, jslot;  // job (pixel, slot) at jray[pix * jpx + slot * jslot]: slot planes
                          // (jpx 1, jslot = band pixels) or pixel-major (jpx = jpp, jslot 1)
    uint32_t radius, neighbors, cap, hist_valid;
    // temporal reuse under camera motion (pass 4; ReuseArgs' motion fields): the previous frame's
    // VP^-1 and VP, its G-buffer (gbuf's addressing, rows [prev_row_lo, prev_row_hi) held:
    // the band and its halo rows), history rows the same; a reprojection outside them counts in *clip.
    // Jobs: slot 0 the history here, slot 1 this sample at p', slots 2 / 3 p' and its confidence.
    float vpinv_prev[16], vp_prev[16];
    const uint4 *pgbuf;
    int32_t prev_row_lo, prev_row_hi;
    unsigned long long *clip;
};
constexpr uint32_t kGiMotionSlots = 4u;
hipError_t wave_gi_round(const Scene &sc, const WaveBufs &w, int pass, int round, const GiArgs &A, hipStream_t s);

}  // namespace ptx
