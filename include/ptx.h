/*
 * ptx.h -- C-ABI drop-in boundary of the MI355X path tracer (libptx.so).
 *
 * Replaces the WebGPU compute path behind the reference's Renderer class
 * (apps/frontend/src/graphics-core/Renderer_TEST.ts; GC/ below = graphics-core/):
 *
 *   ptx_create           <- new Renderer(adapter, device, canvas)          GC/Renderer_TEST.ts:83-126
 *   ptx_upload_scene     <- Initialize(world) -> CreateGPUResources         GC/Renderer_TEST.ts:141-163,445-460
 *                           (takes exactly SerializeWorldData's three u32 arrays, :267-420)
 *   ptx_set_frame        <- Update(): the 33-word uniform block             GC/Renderer_TEST.ts:165-206
 *   ptx_render           <- Render(): G-buffer -> Init -> Final dispatches  GC/Renderer_TEST.ts:208-261
 *                           (+ copyTextureToTexture Result->Scene, :223-231) or the
 *                           legacy brute-force TEST_MCPT dispatch            GC/Renderer.ts:580-647
 *   ptx_reset_accumulation <- texture re-creation on Initialize             GC/Renderer_TEST.ts:445-476
 *   ptx_destroy          <- DestroyGPUResources                             GC/Renderer_TEST.ts:462-476
 *   ptx_run_pass         <- ComputePass.Dispatch of one pass                GC/ComputePass.ts:66-78
 *   ptx_run_passes       <- a run of ComputePass.Dispatch calls (Render, :208-261)
 *   PTX_PASS_TEMPORAL / PTX_PASS_SPATIAL and ptx_halo_* <- the reuse passes the reference
 *                           only specifies (docs/theory/ReSTIR_Pipeline.md:259-462; no code)
 *   PTX_PIPELINE_RESTIR_GI <- BASELINE configs[4], ReSTIR GI: build-defined on the reference's
 *                           shading functions with memo.md:166-231's reconnection shift
 *
 * Conventions: every function returns 0 (PTX_OK) or a negative PTX_E* code and never
 * throws; ptx_last_error() holds the handle's last message.  Input arrays are borrowed
 * for the duration of the call only.  A handle is single-threaded and owns one HIP
 * stream on one device.  Multi-GPU: one handle per rank, each rendering the row band
 * [row_begin, row_end) of the full image with global pixel coordinates (RNG seeds and
 * camera rays use global (x, y), so output is independent of the band split).
 */
#ifndef PTX_H
#define PTX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PTX_ABI_VERSION 5

#define PTX_OK 0
#define PTX_E_INVALID (-1)  /* bad argument / state                  */
#define PTX_E_HIP (-2)      /* HIP runtime error                     */
#define PTX_E_SCENE (-3)    /* scene arrays inconsistent/unsupported */
#define PTX_E_NOMEM (-4)    /* allocation failure                    */
#define PTX_E_PENDING (-5)  /* ptx_present_poll: the present is still in flight (not an error) */

#define PTX_UNIFORM_WORDS 33
#define PTX_GBUFFER_WORDS 4     /* rgba32 texel: flags|inst|mat, prim, bary.x, bary.y */
#define PTX_RESERVOIR_WORDS 32  /* 128-byte Reservoir, SH/PT_1_InitPass.wgsl:145-185 */

/* pipelines */
#define PTX_PIPELINE_RESTIR 0  /* PT_01 G-buffer -> PT_1 Init -> PT_4 Final (Renderer_TEST) */
#define PTX_PIPELINE_MCPT 1    /* TEST_MCPT brute force (legacy Renderer)                 */
#define PTX_PIPELINE_RESTIR_REUSE 2 /* G-buffer -> Init -> temporal -> spatial -> Final: the
                                       build-defined reuse passes; wavefront
                                       kernels only                                        */
#define PTX_PIPELINE_RESTIR_GI 3    /* G-buffer -> GI init (direct light + 1-bounce indirect
                                       candidate) -> temporal -> spatial -> GI shade, on 64-byte
                                       GI reservoirs; passes keep their
                                       PTX_PASS_* ids (INIT, TEMPORAL, SPATIAL, FINAL)        */

/* passes for ptx_run_pass */
#define PTX_PASS_GBUFFER 0
#define PTX_PASS_INIT 1
#define PTX_PASS_FINAL 2
#define PTX_PASS_MCPT 3
#define PTX_PASS_TRACE 4  /* ptx_trace / ptx_trace_device (stats slot only) */
#define PTX_PASS_TEMPORAL 8  /* reuse: PT_1 reservoir <- previous frame's output (same pixel) */
#define PTX_PASS_SPATIAL 9   /* reuse: pairwise-MIS resampling over neighbours -> Final's input */
/* stats-only slots: every launch of the wavefront pipeline's kernels, by kind */
#define PTX_STAT_WAVE_TRACE 5  /* trace_queue launches (ray-segment traversal)      */
#define PTX_STAT_WAVE_LOGIC 6  /* start/step launches (shading, RIS, queue appends) */
#define PTX_STAT_FRAME 7       /* whole ptx_render frames of the wavefront ReSTIR path, which
                                  overlaps its passes: slots 0..2 then only get the per-part
                                  G-buffer launches, with PTX_FLAG_TIME_LAUNCHES          */
#define PTX_STAT_PASS_GROUP 10 /* ptx_run_passes calls of the wavefront kernels          */
#define PTX_STAT_FINAL_FUSED 11 /* count only (no time): PT_4 passes of the reuse pipeline that
                                   walked their replays inside their one logic launch
                                   (wfinal_one), so none of their queries reached trace_queue */

/* buffers for ptx_read_buffer / ptx_write_buffer / ptx_device_pointer */
#define PTX_BUF_GBUFFER 0    /* band_h * W * 4 u32   */
#define PTX_BUF_RESERVOIR 1  /* band_h * W * 32 u32 (GI pipeline: 16 u32) */
#define PTX_BUF_ACCUM 2      /* band_h * W * 4 f32 (Scene texture: accumulated radiance) */
#define PTX_BUF_COUNTERS 3   /* 32 u64: work counters [0..4] (PTX_FLAG_COUNT builds), diagnostics [8..) */
/* PTX_BUF_COUNTERS word 6, every build: pixels whose history a band could not reproject (past its
 * motion halo of reuse_radius rows; such a pixel has no temporal history); zeroed by ptx_reset_stats */
#define PTX_COUNTER_MOTION_CLIP 6
#define PTX_BUF_RESERVOIR_HIST 4 /* band_h * W * 32 u32: spatial output = Final's input and the
                                    next frame's temporal history (reuse pipeline)           */
#define PTX_BUF_DIRECT 5     /* band_h * W * 4 f32: direct light of the GI init pass (GI pipeline) */

#define PTX_FLAG_COUNT_WORK 1u     /* count rays / AABB / triangle tests on device (slower)   */
#define PTX_FLAG_SIMPLE_KERNELS 2u   /* A/B: one thread per pixel, no ray exchange            */
#define PTX_FLAGS_RETIRED 12u      /* bits 4, 8: the persistent-lane / tiled-exchange A/B variants
                                      (round 1; both lost to the wavefront kernels, removed):
                                      ptx_create rejects them with PTX_E_INVALID               */
#define PTX_FLAG_TIME_LAUNCHES 16u   /* HIP events around every wavefront launch (stats slots
                                        PTX_STAT_WAVE_*); costs ~5% of frame time            */
#define PTX_FLAG_SINGLE_STREAM 32u   /* run the wavefront passes as one launch sequence (no
                                        two-stream overlap): isolated per-kernel timings     */
#define PTX_FLAG_ROW_CENSUS 64u    /* counting build (implies PTX_FLAG_COUNT_WORK) that also keeps the
                                        work per 8-row tile row of the band, for ptx_row_census;
                                        the totals of PTX_BUF_COUNTERS stay zero              */
#define PTX_FLAG_HALO_OVERLAP 128u /* band frames: the spatial pass of the interior rows runs while
                                        the halo is exchanged, the edge rows after it         */
#define PTX_FLAG_HALO_SKIP 256u    /* a band handle WITHOUT a communicator: ptx_render runs the band
                                        frame exactly as a rank does (pipelined, same launches)
                                        but skips the halo exchange -- the halo rows keep what
                                        they hold, so the edge rows are NOT the split frame's.
                                        Timing only (a band timed alone: bench.py calibration) */
/* no variant flag: the wavefront pipeline (compacted ray queues, one trace round per
   path vertex) -- the default */

typedef struct ptx_config {
    uint32_t width, height;       /* full image size (uniform words 0,1 must match) */
    uint32_t row_begin, row_end;  /* band rendered by this handle; 0,0 = all rows    */
    int32_t device;               /* HIP device ordinal; -1 = current device        */
    uint32_t pipeline;            /* PTX_PIPELINE_*                                  */
    uint32_t flags;               /* PTX_FLAG_*                                      */
    /* reuse pipeline (0 = default): spatial neighbours lie in [-radius, radius]^2 (30),
     * `neighbors` per pixel (3, at most 16), history confidence capped at temporal_cap (20).
     * A band handle keeps min(radius, rows available) halo rows above and below its band. */
    uint32_t reuse_radius, reuse_neighbors, temporal_cap;
    uint32_t reserved[2];
} ptx_config;

typedef struct ptx_stats {
    uint64_t frames;              /* ptx_render calls since the last stats reset    */
    double kernel_ms_total[16];   /* summed device time per PTX_PASS_* / PTX_STAT_* slot */
    uint64_t kernel_launches[16]; /* launches per slot                              */
    uint32_t triangles, bvh_nodes, instances, max_bvh_depth;
    uint64_t device_bytes;        /* device memory held by the handle               */
} ptx_stats;

typedef struct ptx_handle ptx_handle;

int ptx_abi_version(void);
int ptx_create(const ptx_config *cfg, ptx_handle **out);
int ptx_upload_scene(ptx_handle *h, const uint32_t *scene, size_t n_scene, const uint32_t *geometry,
                     size_t n_geometry, const uint32_t *accel, size_t n_accel);
int ptx_set_frame(ptx_handle *h, const uint32_t uniform[PTX_UNIFORM_WORDS]);
/* Run the configured pipeline for the current frame; if rgba_out != NULL copy the band's
 * accumulated RGBA f32 image (band_h * W * 4) into it (blocking). Otherwise asynchronous. */
int ptx_render(ptx_handle *h, float *rgba_out);
/* (reuse pipeline: whole-image handles only -- a band needs the halo exchange between its
 *  passes, see ptx_halo_*) */
int ptx_run_pass(ptx_handle *h, int pass);
/* Passes in order as one launch sequence per segment group (overlapped on two streams).
 * Every pass must read only its own pixel's results of the earlier passes, except that
 * PTX_PASS_SPATIAL may come first (it reads neighbours of the previous passes' output). */
int ptx_run_passes(ptx_handle *h, const int *passes, int n);
/* Spatial-reuse halo of a band handle.  Between TEMPORAL and SPATIAL a band needs the
 * G-buffer and reservoir rows of its neighbours: rows_top rows from the band above (its
 * last rows), rows_bottom from the band below.  A message is rows x W x bytes_per_row
 * (G-buffer rows, then reservoir rows).  pack copies THIS band's first rows_top / last
 * rows_bottom rows (what the neighbours need) into device buffers; unpack copies received
 * messages into the halo rows.  Both are async on the handle's stream; the buffers may be
 * device memory (RCCL) or host memory (then synchronize before reading a packed one). */
int ptx_halo_rows(ptx_handle *h, uint32_t *rows_top, uint32_t *rows_bottom, size_t *bytes_per_row);
int ptx_halo_pack(ptx_handle *h, void *dev_top, void *dev_bottom);
int ptx_halo_unpack(ptx_handle *h, const void *dev_top, const void *dev_bottom);
/* ---- multi-GPU: the frame split into row bands, one handle per band.
 * The one exchange is the spatial-reuse halo: between the temporal and spatial passes a band
 * receives the G-buffer + reservoir rows of its neighbours (rows_top from the band above,
 * rows_bottom from the band below; ptx_halo_rows).  The handle owns the RCCL communicator:
 *   ptx_comm_unique_id  <- ncclGetUniqueId on one rank; the caller ships the 128 bytes to the
 *                          others (e.g. a torch.distributed broadcast)
 *   ptx_comm_init       <- ncclCommInitRank for a band handle: rank r is the band above rank
 *                          r + 1; ptx_render then runs the whole frame, halo included
 *                          (grouped ncclSend / ncclRecv from the band's edge rows straight into
 *                          the neighbours' halo rows on the handle's streams, no host wait)
 *   ptx_comm_init_all   <- ncclCommInitAll: every band handle of ONE process (one per GPU)
 *   ptx_render_bands    <- one frame over n band handles of one process, in band order
 *                          (row_end of band i == row_begin of band i + 1): the halo moves over
 *                          their communicators, or by peer copies when they have none (several
 *                          bands may then share a GPU); rgba_out (optional) receives the bands'
 *                          accumulated rows in order (blocking)
 * Seeds and neighbour offsets use global pixel coordinates: any split renders the single
 * handle's frame bit for bit. */
#define PTX_COMM_ID_BYTES 128
int ptx_comm_unique_id(void *id_out, size_t bytes);
int ptx_comm_init(ptx_handle *h, const void *unique_id, size_t bytes, int rank, int world);
int ptx_comm_init_all(ptx_handle *const *handles, int n);
int ptx_render_bands(ptx_handle *const *handles, int n, float *rgba_out);
/* The communicator a band handle owns: its rank and world size (0 / 1 without one) and the
 * halo bytes it has sent so far -- what a benchmark reports to prove N ranks exchanged.
 * ptx_comm_init also swaps the band geometry with the neighbouring ranks once and fails on
 * rows that do not continue or halos that do not match; ptx_render checks the communicator's
 * asynchronous error state (ncclCommGetAsyncError) every frame. */
int ptx_comm_info(ptx_handle *h, int *rank, int *world, uint64_t *halo_bytes_sent);
/* Work census of a PTX_FLAG_ROW_CENSUS handle since the last ptx_reset_stats: per 8-row tile
 * row of the band, 5 u64 {rays, instance transforms, AABB tests, triangle tests, hits} of every
 * query traced for that row's pixels (the §8(d) algorithmic-bytes counters).  Cost-balanced
 * band boundaries come from it (pathtracerdemo_amd/bands.py). */
int ptx_row_census(ptx_handle *h, uint64_t *tile_row_counts, size_t n_tile_rows);
int ptx_reset_accumulation(ptx_handle *h);
int ptx_synchronize(ptx_handle *h);
int ptx_get_stats(ptx_handle *h, ptx_stats *out);
int ptx_reset_stats(ptx_handle *h);
int ptx_read_buffer(ptx_handle *h, int which, void *host_dst, size_t bytes);
int ptx_write_buffer(ptx_handle *h, int which, const void *host_src, size_t bytes);
/* A buffer's device address.  On a handle whose frames are pipelined (whole-image reuse
 * pipeline on its own stream: two frames in flight) the G-buffer and
 * reservoir buffers alternate between two allocations frame by frame: the pointer returned
 * for PTX_BUF_GBUFFER / PTX_BUF_RESERVOIR is valid until the next ptx_render.  Accumulation,
 * history and counters never move. */
int ptx_device_pointer(ptx_handle *h, int which, void **dev_ptr, size_t *bytes);
/* The reference's render pass (Renderer_TEST.Render, GC/Renderer_TEST.ts:233-255: a fullscreen
 * quad, SH/VertexShader.wgsl + SH/FragmentShader.wgsl:7-10) onto a canvas_w x canvas_h canvas:
 * canvas pixel (x, y), y = 0 the top row, shows texel (floor((2x+1)*600 / 2canvas_w),
 * floor((2canvas_h-2y-1)*450 / 2canvas_h)) of the accumulated image -- the shader's fixed
 * 600 x 450 window, flipped to screen order -- as unorm8 rgb (clamp, round to nearest even) with
 * alpha 255; a texel outside the image reads 0.  out: canvas_w * canvas_h * 4 bytes, RGBA
 * (bgra = 0, a 2D canvas's ImageData) or BGRA (bgra = 1, a bgra8unorm WebGPU canvas); blocking.
 * Whole-image handles (a split frame is presented from its gathered rows by the host). */
int ptx_present(ptx_handle *h, uint32_t canvas_w, uint32_t canvas_h, int bgra, uint8_t *out);
/* The same render pass without blocking the caller (the reference's Render() ends by drawing into
 * the canvas, GC/Renderer_TEST.ts:233-258, and WebGPUEngine's loop calls nothing else,
 * GC/service/WebGPUEngine.ts:199-200): ptx_present_async enqueues it for the frame last rendered,
 * with the copy into handle-owned pinned memory, on the handle's stream, and returns at once;
 * ptx_present_poll copies the bytes into `out` (canvas_w * canvas_h * 4) and returns PTX_OK once
 * that copy has landed, PTX_E_PENDING while it is in flight (hipEventQuery: never waits).  One
 * present may be in flight per handle (a second ptx_present_async before its poll returned
 * PTX_OK fails).  A later frame's accumulation waits for it on the GPU, so the bytes are exactly
 * the frame it was enqueued after. */
int ptx_present_async(ptx_handle *h, uint32_t canvas_w, uint32_t canvas_h, int bgra);
int ptx_present_poll(ptx_handle *h, uint8_t *out, size_t bytes);
/* What this libptx.so is, as one JSON object in `out` (NUL-terminated, truncated to `bytes`):
 * {"abi": 5, "build": "product" | "ab" (every PTX_AB switch live: the measurement build) | "wgt"
 *  (per-wave timing), "arch": "gfx950", "ptx_ab": <PTX_AB as read>, "ptx_ab_ignored": [keys this
 *  build does not honour], "rccl": <the communicator library loaded, "" before ptx_comm_*>}.
 * Returns the full length (like snprintf).  A benchmark line carries it, so a run made on the wrong
 * library, or with switches the shipped library ignores, is labelled as such. */
int ptx_build_info(char *out, size_t bytes);
/* Closest-hit queries (TraceRay, SH/PT_1_InitPass.wgsl:605-715) for arbitrary rays.
 * rays: n x {o.x,o.y,o.z,d.x, d.y,d.z,-,-} f32 (32 B); hits: n x {t, flags|inst|mat (u32 bits),
 * prim (u32 bits), bary.x, bary.y, pos.x, pos.y, pos.z} (32 B; flags bit31 = valid).
 * eps_mode 0 = G-buffer epsilons (PT_01), 1 = secondary-pass epsilons (PT_1/PT_4/MCPT).
 * ptx_trace takes host arrays (blocking); ptx_trace_device takes device pointers (async). */
int ptx_trace(ptx_handle *h, const float *rays, float *hits, size_t n, int eps_mode);
int ptx_trace_device(ptx_handle *h, const void *rays_dev, void *hits_dev, size_t n, int eps_mode);
/* Use an external hipStream_t (e.g. torch's current stream); NULL restores the own stream. */
int ptx_set_stream(ptx_handle *h, void *hip_stream);
int ptx_destroy(ptx_handle *h);
const char *ptx_last_error(const ptx_handle *h);

#ifdef __cplusplus
}
#endif
#endif
