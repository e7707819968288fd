/*
 * pt_oracle.h -- CPU restatement of the reference's per-pixel path (TEST INFRASTRUCTURE).
 *
 * This is the parity CHECKER for the HIP path, never the product: only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 *
 * It restates, function for function and in the same f32 operation order, the WGSL of
 * hdm0922/PathTracerDemo (SH/ = apps/frontend/src/graphics-core/shaders/):
 *   pto_gbuffer  <- SH/PT_01_GBufferPass.wgsl:496-659
 *   pto_init     <- SH/PT_1_InitPass.wgsl:1361-1486
 *   pto_final    <- SH/PT_4_FinalShadingPass.wgsl:1392-1428
 *   pto_mcpt     <- SH/TEST_MCPT.wgsl:1315-1372
 *   pto_temporal, pto_spatial <- build-defined reuse passes (no reference code; spec
 *                   docs/theory/ReSTIR_Pipeline.md:259-462, docs/theory/memo.md:166-231)
 * over the reference's own device inputs (uniform block, SceneBuffer, GeometryBuffer,
 * AccelBuffer; Renderer_TEST.ts:165-206,267-420).  Implementation-defined WGSL details
 * are fixed as documented in DESIGN.md §Numerics (left-to-right dot/mat-vec sums, no
 * FMA contraction, normalize(v) = v / length(v), IEEE minNum/maxNum for min/max).
 *
 * Parity pinning: the reference ships no tests, golden images or runnable WGSL
 * runtime.  The restatement is pinned by the known-answer tests in
 * tests/golden (PCG hash values published with the algorithm, analytic BSDF values)
 * and by an independent numpy spot-checker (tests/numpy_ref.py).
 */
#ifndef PT_ORACLE_H
#define PT_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PTO_UNIFORM_WORDS 33
#define PTO_RESERVOIR_WORDS 32

typedef struct pto_inputs {
    const uint32_t *uniform;   /* 33 words, Renderer_TEST.ts:174-202 */
    const uint32_t *scene;     /* SceneBuffer    */
    const uint32_t *geometry;  /* GeometryBuffer */
    const uint32_t *accel;     /* AccelBuffer    */
} pto_inputs;

/* Work counters for the algorithmic-bytes model of SURVEY.md §8(d). */
typedef struct pto_counters {
    uint64_t rays;            /* TraceRay calls                          */
    uint64_t instance_xforms; /* instance ray transforms (48 B each)     */
    uint64_t aabb_tests;      /* slab tests (32 B each)                  */
    uint64_t tri_tests;       /* Moller-Trumbore tests (36 B each)       */
    uint64_t hits;            /* hit reconstructions (48 B each)         */
} pto_counters;

/* One pass over pixels [x0,x1) x [y0,y1). Buffers are full-frame (W*H). */
void pto_gbuffer(const pto_inputs *in, int x0, int y0, int x1, int y1, uint32_t *gbuffer /* W*H*4 */,
                 pto_counters *cnt);
void pto_init(const pto_inputs *in, const uint32_t *gbuffer, int x0, int y0, int x1, int y1,
              uint32_t *reservoir /* W*H*32 */, pto_counters *cnt);
void pto_final(const pto_inputs *in, const uint32_t *gbuffer, const uint32_t *reservoir, int x0, int y0,
               int x1, int y1, float *accum /* W*H*4 in/out */, pto_counters *cnt);
void pto_mcpt(const pto_inputs *in, int x0, int y0, int x1, int y1, float *accum /* W*H*4 in/out */,
              pto_counters *cnt);

/* Multithreaded driver: pass = 0 gbuffer, 1 init, 2 final, 3 mcpt, 4 restir frame (0,1,2);
 * the reuse pipeline's PT_1 (11: x_{k+1} of a hybrid-shiftable sample in pad words 24..27) and
 * PT_4 (12: a reused reservoir's stored contribution f * UCW, a PT_1 reservoir replayed).
 * Rows [y0,y1) are interleaved over nthreads pthreads.  Returns 0 on success. */
int pto_run(int pass, int nthreads, const pto_inputs *in, int x0, int y0, int x1, int y1, uint32_t *gbuffer,
            uint32_t *reservoir, float *accum, pto_counters *cnt);

/* Reuse passes (build-defined; docs/theory/ReSTIR_Pipeline.md:259-462).
 * Reservoirs are full-frame W*H*32 words; words 24/25 of a reused reservoir hold p_hat and
 * the shift pdf product q of its sample in its own pixel's domain. */
typedef struct pto_reuse_params {
    uint32_t radius;        /* spatial neighbours in [-radius, radius]^2             */
    uint32_t neighbors;     /* spatial neighbours per pixel (<= 16)                   */
    uint32_t temporal_cap;  /* history confidence <= temporal_cap                    */
    uint32_t hist_valid;    /* res_hist holds the previous frame (same camera/scene)  */
} pto_reuse_params;
/* temporal: res_cur (PT_1 output) updated in place from res_hist (previous spatial output) */
void pto_temporal(const pto_inputs *in, const uint32_t *gbuffer, uint32_t *res_cur, const uint32_t *res_hist,
                  const pto_reuse_params *prm, int x0, int y0, int x1, int y1, pto_counters *cnt);
/* temporal under camera motion: res_cur (PT_1 output) updated in place from the previous
 * frame's spatial output res_hist at each pixel's reprojection, in the previous frame's domain
 * (prev_uniform: its 33 words; gbuffer_prev: its G-buffer).  pt_oracle.c temporal_motion_pixel. */
int pto_run_temporal_motion(int nthreads, const pto_inputs *in, int x0, int y0, int x1, int y1,
                            const uint32_t *gbuffer, uint32_t *res_cur, const uint32_t *res_hist,
                            const uint32_t *prev_uniform, const uint32_t *gbuffer_prev, const pto_reuse_params *prm,
                            pto_counters *cnt);
void pto_mat4_inverse(const float *m /* 16, column-major */, float *out /* 16 */);
/* spatial: reads res_cur of the pixel and its neighbours, writes res_out (PT_4's input) */
void pto_spatial(const pto_inputs *in, const uint32_t *gbuffer, const uint32_t *res_cur, uint32_t *res_out,
                 const pto_reuse_params *prm, int x0, int y0, int x1, int y1, pto_counters *cnt);
/* the shift of DESIGN.md §Reuse: reservoir sample `res` replayed in pixel (x, y)'s domain;
 * out = {valid (0/1), p_hat, q} */
void pto_eval_sample(const pto_inputs *in, const uint32_t *gbuffer, uint32_t x, uint32_t y, const uint32_t *res,
                     float out[3]);
/* threaded: pass 5 = temporal (res_cur in/out, res_hist in), 6 = spatial (res_cur in, res_hist out) */
int pto_run_reuse(int pass, int nthreads, const pto_inputs *in, int x0, int y0, int x1, int y1,
                  const uint32_t *gbuffer, uint32_t *res_cur, uint32_t *res_hist, const pto_reuse_params *prm,
                  pto_counters *cnt);

/* ReSTIR GI (build-defined; pt_oracle_gi.c): 16-word GI reservoirs
 * (W*H*16), per-pixel direct light (W*H*4 f32).  init writes res_cur + direct; temporal
 * updates res_cur from res_hist; spatial reads res_cur, writes res_hist; final reads
 * res_hist + direct and accumulates into accum. */
#define PTO_GI_WORDS 16
#define PTO_GI_PASS_INIT 7
#define PTO_GI_PASS_TEMPORAL 8
#define PTO_GI_PASS_SPATIAL 9
#define PTO_GI_PASS_FINAL 10
void pto_gi_init(const pto_inputs *in, const uint32_t *gbuffer, int x0, int y0, int x1, int y1, uint32_t *res,
                 float *direct, pto_counters *cnt);
void pto_gi_temporal(const pto_inputs *in, const uint32_t *gbuffer, uint32_t *res_cur, const uint32_t *res_hist,
                     const pto_reuse_params *prm, int x0, int y0, int x1, int y1);
void pto_gi_spatial(const pto_inputs *in, const uint32_t *gbuffer, const uint32_t *res_cur, uint32_t *res_out,
                    const pto_reuse_params *prm, int x0, int y0, int x1, int y1, pto_counters *cnt);
void pto_gi_final(const pto_inputs *in, const uint32_t *gbuffer, const uint32_t *res, const float *direct, int x0,
                  int y0, int x1, int y1, float *accum);
/* the GI reconnection shift of reservoir s into pixel (x, y): out = {valid, f.rgb, q} */
void pto_gi_shift(const pto_inputs *in, const uint32_t *gbuffer, uint32_t x, uint32_t y, const uint32_t *s,
                  float out[5]);
/* the GI candidate direction (two-sided cosine lobe) on an explicit surface; returns its pdf */
float pto_gi_sample_dir(const float n[3], const float mat[7], const float v[3], uint32_t *seed, float out_dir[3]);
/* threaded: pass = PTO_GI_PASS_* */
int pto_run_gi(int pass, int nthreads, const pto_inputs *in, int x0, int y0, int x1, int y1, const uint32_t *gbuffer,
               uint32_t *res_cur, uint32_t *res_hist, float *direct, float *accum, const pto_reuse_params *prm,
               pto_counters *cnt);
/* GI temporal reuse under camera motion (pt_oracle_gi.c gi_temporal_motion_pixel): res_cur in/out,
 * res_hist = the previous frame's spatial output, rendered with prev_uniform over gbuffer_prev */
#define PTO_GI_PASS_TEMPORAL_MOTION 13
int pto_run_gi_temporal_motion(int nthreads, const pto_inputs *in, int x0, int y0, int x1, int y1,
                               const uint32_t *gbuffer, uint32_t *res_cur, const uint32_t *res_hist,
                               const uint32_t *prev_uniform, const uint32_t *gbuffer_prev,
                               const pto_reuse_params *prm, pto_counters *cnt);

/* Closest-hit queries, same record formats as ptx_trace (include/ptx.h):
 * rays n x 8 f32 {o, d.x | d.y, d.z, -, -}; hits n x 8 {t, flags|inst|mat, prim, bu, bv, pos}.
 * eps_mode 0 = PT_01 epsilons, 1 = PT_1/PT_4/MCPT epsilons. */
void pto_trace(const pto_inputs *in, const float *rays, float *hits, size_t n, int eps_mode, pto_counters *cnt);

/* Known-answer helpers (SH/PT_1_InitPass.wgsl:810-826). */
uint32_t pto_pcg(uint32_t seed);
float pto_random(uint32_t *seed);
/* fixed f32 sin/cos (x >= 0) and pow(x, 5) shared with the HIP path (see pt_oracle.c) */
float pto_sin(float x);
float pto_cos(float x);
float pto_pow5(float x);

/* BSDF / PDF known-answer helpers on an explicit surface (SH/PT_1_InitPass.wgsl:834-1245).
 * mat = {albedo r,g,b, metalness, roughness, transmission, ior} AFTER GetMaterial's tweaks. */
void pto_bsdf(const float n[3], const float mat[7], const float v[3], const float l[3], float out[3]);
float pto_pdf_bsdf(const float n[3], const float mat[7], const float v[3], const float l[3]);
void pto_sample_bsdf(const float n[3], const float mat[7], const float v[3], uint32_t *seed, float out_dir[3],
                     uint32_t *out_lobe);
float pto_ray_triangle(const float o[3], const float d[3], const float p0[3], const float p1[3],
                       const float p2[3], float det_eps);

#ifdef __cplusplus
}
#endif
#endif
