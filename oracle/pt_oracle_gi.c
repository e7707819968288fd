/*
 * pt_oracle_gi.c -- ReSTIR GI restatement (TEST INFRASTRUCTURE; #included by pt_oracle.c,
 * so it shares that file's static f32 helpers and the reference functions they restate).
 *
 * Not in the reference code: BASELINE.json configs[4] ("ReSTIR GI, 1-bounce indirect
 * reservoirs") is build-defined on top of the reference's own pieces -- GetSurface,
 * SampleNEE / PDF_LIGHT / L_emit / Visibility, BSDF / SampleBSDF / PDF_BSDF
 * (SH/PT_1_InitPass.wgsl:285-314,438-467,746-1260) and UpdateReservoir (:1298-1320) --
 * with the reconnection shift at x2 that docs/theory/memo.md:166-231 specifies (the
 * reconnection vertex x_k kept, J = |n_k . w_y| / |n_k . w_x| * |x_k - x_{k-1}|^2 /
 * |x_k - y_{k-1}|^2, the light pick at x_{k+1} independent of the shift).  DESIGN.md §GI
 * states the rules; the HIP kernels of csrc/ptx_gi.hip are checked against these bit for
 * bit.
 *
 * Per pixel with G-buffer hit x1 (camera point x0, V1 = normalize(x0 - x1)), from the
 * stream seed = pcg(init_seed ^ SALT_GI):
 *   direct  = L_emit * BSDF(x1, V1, L) * |n1.L| / pdf_light * Visibility   (one NEE sample)
 *   L1      ~ gi_sample_dir(x1, V1) with its pdf1; trace -> x2 (or the environment)
 *   x2 hit:   NEE at x2 (V2 = normalize(x1 - x2)): lt = L_emit / pdf_light * Visibility,
 *             Lo(x2 -> V2) = BSDF(x2, V2, L2) * lt * |n2.L2|
 *   escape:   Lo = ENV (0.5), the sample is the direction L1
 *   f = BSDF(x1, V1, L1) * |n1.L1| * Lo, p_hat = Luminance(f), W = (p_hat / pdf1) / p_hat
 * The sample (x2 surface, L2, lt) is a reconnection vertex with a fixed outgoing light
 * path, so its value in another domain y re-evaluates only the two BSDFs and the geometry:
 *   q_y = |x2 - y1|^2 / |n2 . w_y|  (1 for an environment direction), J(x -> y) = q_x / q_y,
 * and its visibility in y is BINARY (the segment y1 -> x2 shortened by GI_VIS_SHORTEN, or the
 * escape of direction w from y1, is free of ANY hit): exactly the paths the canonical
 * technique can produce (its BSDF ray stops at the first surface, transmissive or not).
 *
 * GI reservoir, 16 words (64 B):
 *   [0..3]   x2 CompactSurface (bit 31 of word 0 set: surface sample; clear: environment)
 *   [4..6]   L2 (surface sample) or the escape direction (environment); [7] W (UCW)
 *   [8..10]  lt (surface sample; 0 for the environment);               [11] confidence C
 *   [12..14] f: the sample's contribution in the reservoir's own domain; [15] q there
 * C = 0 marks the empty reservoir (no G-buffer hit).  Temporal and spatial reuse use the
 * DI passes' confidence-weighted rules (pt_oracle.c temporal_pixel / spatial_pixel).
 */

#define SALT_GI 0x47494E49u          /* "GINI" */
#define SALT_GI_TEMPORAL 0x47495450u /* "GITP" */
#define SALT_GI_SPATIAL 0x47495350u  /* "GISP" */
#define GI_VIS_SHORTEN 0.999f
#define FLT_MAX_F 3.402823466e38f

static inline v3 gi_v3(const uint32_t *w) { return V3(f32_of(w[0]), f32_of(w[1]), f32_of(w[2])); }
static inline void gi_put3(uint32_t *w, v3 v) { w[0] = u32_of(v.x); w[1] = u32_of(v.y); w[2] = u32_of(v.z); }

/* q of a surface sample seen from y: |x2 - y|^2 / |n2 . normalize(x2 - y)| */
static inline float gi_q(v3 y, const surface *X2) {
    v3 r = vsub(X2->pos, y);
    return vdot(r, r) / fabsf(vdot(X2->nrm, vnormalize(r)));
}
/* Lo(x2 -> V2) of the stored light path: BSDF(x2, V2, L2) * lt * |n2 . L2| */
static inline v3 gi_lo(const surface *X2, v3 V2, v3 L2, v3 lt) {
    return vscale(vmul(bsdf(X2, V2, L2), lt), fabsf(vdot(X2->nrm, L2)));
}
static inline int gi_q_ok(float q) { return q > 0.0f && q <= FLT_MAX_F; }

/* The GI candidate direction at x: a cosine lobe (SampleCosineHemisphere + TBNMatrix,
 * PT_1:577-589,937-946) on V's side with probability 1 - T, on the far side with T.  Not
 * the reference's SampleBSDF: a reconnection shift is unbiased only when the candidate's
 * pdf is the sampler's TRUE density, and the reference's PDF_BSDF is not that of its
 * SampleBSDF (E[1/pdf] over its samples is ~2.5 pi-steradian off for a transmissive
 * material, 6 % for a rough metal: tests/test_gi_oracle.py).  This pdf is exact, positive
 * wherever BSDF(x, V, .) can be (BSDF = (1-T) BRDF on V's side, T BTDF across), so every
 * domain's target has the canonical technique's support.  3 Random() draws. */
static v3 gi_sample_dir(uint32_t *seed, const surface *X, v3 V, float *pdf) {
    const float T = X->mat.transmission;
    v3 N = vdot(V, X->nrm) >= 0.0f ? X->nrm : vneg(X->nrm);
    if (pto_random(seed) < T) N = vneg(N);
    v3 L = mat3_mul(tbn(N), sample_cosine(seed));
    const int same = vdot(L, X->nrm) * vdot(V, X->nrm) > 0.0f;
    *pdf = (same ? 1.0f - T : T) * fabsf(vdot(X->nrm, L)) / PI_F;
    return L;
}

/* GI candidate pass: the pixel's direct light and its one-candidate GI reservoir. */
static void gi_init_pixel(const ctx *c, const uint32_t *gbuffer, uint32_t x, uint32_t y, uint32_t *res,
                          float *direct) {
    const uint32_t W = c->U[U_W];
    compact x1 = decode_compact(gbuffer + 4u * (y * W + x));
    memset(res, 0, 4u * PTO_GI_WORDS);
    direct[0] = direct[1] = direct[2] = direct[3] = 0.0f;
    if (!x1.valid) return;
    uint32_t seed = pto_pcg(init_seed(c, x, y) ^ SALT_GI);
    surface X1 = get_surface(c, x1);
    v3 V1 = vnormalize(vsub(get_x0(c, x, y), X1.pos));
    /* direct light: one NEE sample (SampleNEE, PT_1:970-1025) */
    light_sample XL = sample_nee(c, &seed, &X1, V1);
    v3 L = direction_to_light(&X1, &XL);
    v3 u = vscale(vmul(l_emit(c, &XL, &X1), bsdf(&X1, V1, L)), fabsf(vdot(X1.nrm, L)));
    u = XL.pdf > 0.0f ? vdivs(u, XL.pdf) : V3(0.0f, 0.0f, 0.0f);
    v3 d = vscale(u, visibility(c, X1.pos, XL.pos));
    direct[0] = d.x; direct[1] = d.y; direct[2] = d.z;
    /* the indirect candidate: one BSDF sample at x1 */
    float pdf1;
    v3 L1 = gi_sample_dir(&seed, &X1, V1, &pdf1);
    v3 b1 = vscale(bsdf(&X1, V1, L1), fabsf(vdot(X1.nrm, L1)));
    ray r = {X1.pos, L1};
    hit h = trace_ray(c, r);
    v3 f;
    float q;
    if (!h.valid) { /* escapes: the environment in direction L1 */
        f = vscale(b1, ENV_C);
        q = 1.0f;
        gi_put3(res + 4, L1);
    } else {
        surface X2 = get_surface(c, h.s);
        v3 V2 = vnormalize(vsub(X1.pos, X2.pos));
        light_sample XL2 = sample_nee(c, &seed, &X2, V2);
        v3 L2 = direction_to_light(&X2, &XL2);
        v3 lt = l_emit(c, &XL2, &X2);
        lt = XL2.pdf > 0.0f ? vdivs(lt, XL2.pdf) : V3(0.0f, 0.0f, 0.0f);
        lt = vscale(lt, visibility(c, X2.pos, XL2.pos));
        f = vmul(b1, gi_lo(&X2, V2, L2, lt));
        q = gi_q(X1.pos, &X2);
        encode_compact(h.s, res);
        res[0] |= 0x80000000u;
        gi_put3(res + 4, L2);
        gi_put3(res + 8, lt);
    }
    /* one-candidate RIS (UpdateReservoir with C = 1) */
    const float p_hat = luminance(f);
    const float w_sum = pdf1 > 0.0f ? p_hat / pdf1 : 0.0f;
    const int ok = p_hat > 0.0f && gi_q_ok(q) && w_sum > 0.0f && w_sum <= FLT_MAX_F;
    res[7] = u32_of(ok ? w_sum / p_hat : 0.0f);
    res[11] = 1u;
    gi_put3(res + 12, f);
    res[15] = u32_of(q);
}

/* The sample of GI reservoir `s` in the domain of pixel (x, y) with G-buffer hit y1:
 * returns 0 when no such path exists there (else f = its contribution incl. the binary
 * visibility, q = its measure factor). */
static int gi_shift(const ctx *c, uint32_t x, uint32_t y, compact y1, const uint32_t *s, v3 *f_out, float *q_out) {
    *f_out = V3(0.0f, 0.0f, 0.0f);
    *q_out = 0.0f;
    if (!y1.valid || s[11] == 0u) return 0;
    surface Y = get_surface(c, y1);
    v3 Vy = vnormalize(vsub(get_x0(c, x, y), Y.pos));
    v3 f, dir;
    float q, remain;
    if (!(s[0] & 0x80000000u)) { /* environment direction */
        dir = gi_v3(s + 4);
        f = vscale(vscale(bsdf(&Y, Vy, dir), fabsf(vdot(Y.nrm, dir))), ENV_C);
        q = 1.0f;
        remain = FLT_MAX_F;
    } else {
        compact x2 = decode_compact(s);
        x2.valid = 1u;
        surface X2 = get_surface(c, x2);
        v3 r = vsub(X2.pos, Y.pos);
        const float dist = vlength(r);
        dir = vdivs(r, dist);
        v3 V2 = vnormalize(vsub(Y.pos, X2.pos));
        f = vmul(vscale(bsdf(&Y, Vy, dir), fabsf(vdot(Y.nrm, dir))), gi_lo(&X2, V2, gi_v3(s + 4), gi_v3(s + 8)));
        q = gi_q(Y.pos, &X2);
        remain = dist * GI_VIS_SHORTEN;
    }
    if (!gi_q_ok(q)) return 0;
    ray rr = {Y.pos, dir};
    hit h = trace_ray(c, rr);
    const float vis = (!h.valid || h.t > remain) ? 1.0f : 0.0f;
    *f_out = vscale(f, vis);
    *q_out = q;
    return 1;
}

/* Reservoir `src`'s sample with a new contribution f / q / W and confidence C. */
static void gi_write(uint32_t *out, const uint32_t *src, v3 f, float q, float w_sum, uint32_t C) {
    uint32_t tmp[11];
    memcpy(tmp, src, sizeof tmp); /* src may alias out */
    memcpy(out, tmp, sizeof tmp);
    const float p = luminance(f);
    out[7] = u32_of(p > 0.0f ? w_sum / p : 0.0f);
    out[11] = C;
    gi_put3(out + 12, f);
    out[15] = u32_of(q);
}

/* Temporal GI reuse: the pixel's candidate reservoir with last frame's spatial output at
 * the same pixel (static camera: same domain, identity shift). */
static void gi_temporal_pixel(const ctx *c, const uint32_t *gbuffer, uint32_t *cur, const uint32_t *hist,
                              const pto_reuse_params *prm, uint32_t x, uint32_t y) {
    const uint32_t W = c->U[U_W];
    if (!decode_compact(gbuffer + 4u * (y * W + x)).valid) return;
    uint32_t seed = reuse_seed(c, x, y, SALT_GI_TEMPORAL);
    const v3 fc = gi_v3(cur + 12), fh = gi_v3(hist + 12);
    const float pc = luminance(fc), ph = luminance(fh);
    const int canon_ok = cur[11] != 0u && pc > 0.0f;
    const uint32_t Cp = prm->hist_valid ? (hist[11] < prm->temporal_cap ? hist[11] : prm->temporal_cap) : 0u;
    const float cp = (float)Cp, tot = 1.0f + cp;
    const int hist_ok = Cp != 0u && ph > 0.0f;
    const float wc = canon_ok ? (1.0f / tot) * pc * f32_of(cur[7]) : 0.0f;
    const float wp = hist_ok ? (cp / tot) * ph * f32_of(hist[7]) : 0.0f;
    float w_sum = 0.0f;
    int from_hist = 0;
    if (wrs_update(&w_sum, wc, &seed)) from_hist = 0;
    if (wrs_update(&w_sum, wp, &seed)) from_hist = 1;
    const uint32_t *src = from_hist ? hist : cur;
    gi_write(cur, src, gi_v3(src + 12), f32_of(src[15]), w_sum, 1u + Cp);
}

/* Temporal GI reuse under camera motion (round 5; the DI pass's rules, temporal_motion_pixel in
 * pt_oracle.c): the history lives at the reprojection p' of the pixel's primary hit in the
 * previous frame's domain (its camera point x0' and hit x1'), so it is the spatial pass's pairwise
 * rule with M = 1 -- the history sample shifted here (gi_shift, one occlusion ray, J = q_h / q_here)
 * and the canonical sample shifted into the previous domain for its own weight; c_c = 1,
 * c_h = min(C_hist, cap); canonical draw first, then the history. */
static void gi_temporal_motion_pixel(const ctx *c, const ctx *cprev, const float *vp_prev, const uint32_t *gbuffer,
                                     uint32_t *cur, const uint32_t *hist_all, const uint32_t *gbuffer_prev,
                                     const pto_reuse_params *prm, uint32_t x, uint32_t y) {
    const uint32_t W = c->U[U_W];
    const compact x1 = decode_compact(gbuffer + 4u * (y * W + x));
    if (!x1.valid) return;
    uint32_t seed = reuse_seed(c, x, y, SALT_GI_TEMPORAL);
    const v3 fc = gi_v3(cur + 12);
    const float cc = 1.0f, pc = luminance(fc), qc = f32_of(cur[15]), Wc = f32_of(cur[7]);
    const int canon_ok = cur[11] != 0u && pc > 0.0f;
    uint32_t Cp = 0u, px = 0u, py = 0u;
    compact x1p = {0u, 0u, 0u, 0u, 0.0f, 0.0f};
    const uint32_t *h = NULL;
    if (prm->hist_valid) {
        const surface S1 = get_surface(c, x1);
        if (motion_lookup(c, cprev, vp_prev, &S1, y, gbuffer_prev, prm->radius, &px, &py, &x1p)) {
            h = hist_all + PTO_GI_WORDS * (py * W + px);
            Cp = h[11] < prm->temporal_cap ? h[11] : prm->temporal_cap;
        }
    }
    const float cp = (float)Cp;
    /* forward: the history sample in this pixel's domain */
    float wh = 0.0f, qf = 0.0f;
    v3 ff = V3(0.0f, 0.0f, 0.0f);
    if (Cp != 0u && luminance(gi_v3(h + 12)) > 0.0f) {
        const float ph = luminance(gi_v3(h + 12)), qh = f32_of(h[15]), Wh = f32_of(h[7]);
        v3 F;
        float qF;
        if (gi_shift(c, x, y, x1, h, &F, &qF)) {
            const float pF = luminance(F);
            const float J = qh / qF;
            const float pb = ph / J;
            const float den = cc * pF + cp * pb;
            const float m = den > 0.0f ? (cp * pb) / den : 0.0f;
            wh = m * pF * Wh * J;
            ff = F;
            qf = qF;
        }
    }
    /* backward: this pixel's sample in the previous domain (its weight) */
    float Q = 1.0f;
    if (canon_ok && Cp != 0u) {
        v3 B;
        float qB;
        if (gi_shift(cprev, px, py, x1p, cur, &B, &qB)) {
            const float pbc = luminance(B) * qc / qB;
            const float den = cc * pc + cp * pbc;
            Q = den > 0.0f ? (cc * pc) / den : 1.0f;
        }
    }
    const float wc = canon_ok ? Q * pc * Wc : 0.0f;
    float w_sum = 0.0f;
    const uint32_t *src = cur;
    v3 fsel = fc;
    float qsel = qc;
    if (wrs_update(&w_sum, wc, &seed)) { src = cur; fsel = fc; qsel = qc; }
    if (wrs_update(&w_sum, wh, &seed)) { src = h; fsel = ff; qsel = qf; }
    gi_write(cur, src, fsel, qsel, w_sum, 1u + Cp);
}

/* Spatial GI reuse with pairwise MIS (the rule of spatial_pixel, pt_oracle.c), the shift
 * being gi_shift: forward = neighbour sample into this pixel, backward = this pixel's
 * sample into the neighbour. */
static void gi_spatial_pixel(const ctx *c, const uint32_t *gbuffer, const uint32_t *cur, uint32_t *out,
                             const pto_reuse_params *prm, uint32_t x, uint32_t y) {
    const uint32_t W = c->U[U_W], H = c->U[U_H];
    const uint32_t p = y * W + x;
    compact x1 = decode_compact(gbuffer + 4u * p);
    uint32_t *o = out + PTO_GI_WORDS * p;
    if (!x1.valid) { memset(o, 0, 4u * PTO_GI_WORDS); return; }
    const uint32_t *rc = cur + PTO_GI_WORDS * p;
    uint32_t seed = reuse_seed(c, x, y, SALT_GI_SPATIAL);
    const uint32_t M = prm->neighbors;
    uint32_t nb[16];
    int present[16];
    for (uint32_t k = 0; k < M; ++k) {
        uint32_t nx = 0, ny = 0;
        present[k] = spatial_neighbor(&seed, prm->radius, x, y, W, H, &nx, &ny);
        nb[k] = ny * W + nx;
        if (present[k]) present[k] = decode_compact(gbuffer + 4u * nb[k]).valid;
    }
    const float Mf = (float)M, cc = (float)rc[11];
    const v3 fcv = gi_v3(rc + 12);
    const float pc = luminance(fcv), qc = f32_of(rc[15]), Wc = f32_of(rc[7]);
    const int canon_ok = rc[11] != 0u && pc > 0.0f;
    float wn[16], sumQ = 0.0f;
    v3 ff[16];
    float qf[16];
    uint32_t Csum = rc[11];
    for (uint32_t k = 0; k < M; ++k) {
        wn[k] = 0.0f; ff[k] = V3(0.0f, 0.0f, 0.0f); qf[k] = 0.0f;
        float Q = 1.0f;
        if (present[k]) {
            const uint32_t *rn = cur + PTO_GI_WORDS * nb[k];
            const uint32_t nx = nb[k] % W, ny = nb[k] / W;
            const float cn = (float)rn[11], pn = luminance(gi_v3(rn + 12)), qn = f32_of(rn[15]), Wn = f32_of(rn[7]);
            Csum += rn[11];
            if (pn > 0.0f) { /* forward */
                v3 F;
                float qF;
                if (gi_shift(c, x, y, x1, rn, &F, &qF)) {
                    const float pF = luminance(F);
                    const float J = qn / qF;
                    const float pb = pn / J;
                    const float den = cc * pF + Mf * cn * pb;
                    const float m = den > 0.0f ? (cn * pb) / den : 0.0f;
                    wn[k] = m * pF * Wn * J;
                    ff[k] = F;
                    qf[k] = qF;
                }
            }
            if (canon_ok) { /* backward */
                v3 B;
                float qB;
                if (gi_shift(c, nx, ny, decode_compact(gbuffer + 4u * nb[k]), rc, &B, &qB)) {
                    const float pbc = luminance(B) * qc / qB;
                    const float den = cc * pc + Mf * cn * pbc;
                    Q = den > 0.0f ? (cc * pc) / den : 1.0f;
                }
            }
        }
        sumQ += Q;
    }
    const float wc = canon_ok ? (sumQ / Mf) * pc * Wc : 0.0f;
    float w_sum = 0.0f;
    const uint32_t *src = rc;
    v3 fsel = fcv;
    float qsel = qc;
    if (wrs_update(&w_sum, wc, &seed)) { src = rc; fsel = fcv; qsel = qc; }
    for (uint32_t k = 0; k < M; ++k)
        if (wrs_update(&w_sum, wn[k], &seed)) { src = cur + PTO_GI_WORDS * nb[k]; fsel = ff[k]; qsel = qf[k]; }
    gi_write(o, src, fsel, qsel, w_sum, Csum);
}

/* GI shading: direct + f * W, accumulated like WriteColor (PT_4:599-606); a G-buffer miss
 * shows the environment (PT_4:1404-1408). */
static void gi_final_pixel(const ctx *c, const uint32_t *gbuffer, const uint32_t *res, const float *direct,
                           uint32_t x, uint32_t y, float *px) {
    const uint32_t W = c->U[U_W];
    if (!decode_compact(gbuffer + 4u * (y * W + x)).valid) { px[0] = px[1] = px[2] = ENV_C; px[3] = 1.0f; return; }
    v3 col = vadd(V3(direct[0], direct[1], direct[2]), vscale(gi_v3(res + 12), f32_of(res[7])));
    write_color(c, px, col);
}

void pto_gi_init(const pto_inputs *in, const uint32_t *gbuffer, int x0, int y0, int x1, int y1, uint32_t *res,
                 float *direct, pto_counters *cnt) {
    ctx c;
    ctx_init(&c, in, EPS_INIT, cnt);
    const uint32_t W = c.U[U_W];
    for (int y = y0; y < y1; ++y)
        for (int x = x0; x < x1; ++x) {
            const uint32_t p = (uint32_t)y * W + (uint32_t)x;
            gi_init_pixel(&c, gbuffer, (uint32_t)x, (uint32_t)y, res + PTO_GI_WORDS * p, direct + 4u * p);
        }
}

void pto_gi_temporal(const pto_inputs *in, const uint32_t *gbuffer, uint32_t *res_cur, const uint32_t *res_hist,
                     const pto_reuse_params *prm, int x0, int y0, int x1, int y1) {
    ctx c;
    ctx_init(&c, in, EPS_INIT, NULL);
    const uint32_t W = c.U[U_W];
    for (int y = y0; y < y1; ++y)
        for (int x = x0; x < x1; ++x) {
            const uint32_t p = (uint32_t)y * W + (uint32_t)x;
            gi_temporal_pixel(&c, gbuffer, res_cur + PTO_GI_WORDS * p, res_hist + PTO_GI_WORDS * p, prm, (uint32_t)x,
                              (uint32_t)y);
        }
}

void pto_gi_spatial(const pto_inputs *in, const uint32_t *gbuffer, const uint32_t *res_cur, uint32_t *res_out,
                    const pto_reuse_params *prm, int x0, int y0, int x1, int y1, pto_counters *cnt) {
    ctx c;
    ctx_init(&c, in, EPS_INIT, cnt);
    for (int y = y0; y < y1; ++y)
        for (int x = x0; x < x1; ++x) gi_spatial_pixel(&c, gbuffer, res_cur, res_out, prm, (uint32_t)x, (uint32_t)y);
}

void pto_gi_final(const pto_inputs *in, const uint32_t *gbuffer, const uint32_t *res, const float *direct, int x0,
                  int y0, int x1, int y1, float *accum) {
    ctx c;
    ctx_init(&c, in, EPS_INIT, NULL);
    const uint32_t W = c.U[U_W];
    for (int y = y0; y < y1; ++y)
        for (int x = x0; x < x1; ++x) {
            const uint32_t p = (uint32_t)y * W + (uint32_t)x;
            gi_final_pixel(&c, gbuffer, res + PTO_GI_WORDS * p, direct + 4u * p, (uint32_t)x, (uint32_t)y,
                           accum + 4u * p);
        }
}

void pto_gi_temporal_motion(const pto_inputs *in, const pto_motion *mot, const uint32_t *gbuffer, uint32_t *res_cur,
                            const uint32_t *res_hist, const pto_reuse_params *prm, int x0, int y0, int x1, int y1,
                            pto_counters *cnt) {
    ctx c, cprev;
    ctx_init(&c, in, EPS_INIT, cnt);
    pto_inputs pin = *in;
    pin.uniform = mot->prev_uniform;
    ctx_init(&cprev, &pin, EPS_INIT, cnt);
    float vp_prev[16];
    pto_mat4_inverse((const float *)(mot->prev_uniform + U_VPINV), vp_prev);
    const uint32_t W = c.U[U_W];
    for (int y = y0; y < y1; ++y)
        for (int x = x0; x < x1; ++x) {
            const uint32_t p = (uint32_t)y * W + (uint32_t)x;
            gi_temporal_motion_pixel(&c, &cprev, vp_prev, gbuffer, res_cur + PTO_GI_WORDS * p, res_hist,
                                     mot->gbuffer_prev, prm, (uint32_t)x, (uint32_t)y);
        }
}

/* Test helper: gi_shift of GI reservoir `s` into pixel (x, y); out = {valid, f.rgb, q}. */
void pto_gi_shift(const pto_inputs *in, const uint32_t *gbuffer, uint32_t x, uint32_t y, const uint32_t *s,
                  float out[5]) {
    ctx c;
    ctx_init(&c, in, EPS_INIT, NULL);
    v3 f;
    float q;
    out[0] = (float)gi_shift(&c, x, y, decode_compact(gbuffer + 4u * (y * c.U[U_W] + x)), s, &f, &q);
    out[1] = f.x; out[2] = f.y; out[3] = f.z; out[4] = q;
}

/* ------------------------------------------------------------------ threaded driver */
typedef struct gi_job {
    int pass, tid, nthreads, x0, y0, x1, y1;
    const pto_inputs *in;
    const uint32_t *gbuffer;
    uint32_t *res_cur, *res_hist;
    float *direct, *accum;
    const pto_reuse_params *prm;
    pto_counters cnt;
    const pto_motion *mot;
} gi_job;

static void *gi_worker(void *arg) {
    gi_job *j = (gi_job *)arg;
    for (int y = j->y0 + j->tid; y < j->y1; y += j->nthreads) {
        switch (j->pass) {
        case PTO_GI_PASS_INIT: pto_gi_init(j->in, j->gbuffer, j->x0, y, j->x1, y + 1, j->res_cur, j->direct, &j->cnt); break;
        case PTO_GI_PASS_TEMPORAL: pto_gi_temporal(j->in, j->gbuffer, j->res_cur, j->res_hist, j->prm, j->x0, y, j->x1, y + 1); break;
        case PTO_GI_PASS_SPATIAL: pto_gi_spatial(j->in, j->gbuffer, j->res_cur, j->res_hist, j->prm, j->x0, y, j->x1, y + 1, &j->cnt); break;
        case PTO_GI_PASS_FINAL: pto_gi_final(j->in, j->gbuffer, j->res_hist, j->direct, j->x0, y, j->x1, y + 1, j->accum); break;
        case PTO_GI_PASS_TEMPORAL_MOTION:
            pto_gi_temporal_motion(j->in, j->mot, j->gbuffer, j->res_cur, j->res_hist, j->prm, j->x0, y, j->x1, y + 1,
                                   &j->cnt);
            break;
        default: break;
        }
    }
    return NULL;
}

static int run_gi_m(int pass, int nthreads, const pto_inputs *in, int x0, int y0, int x1, int y1,
                    const uint32_t *gbuffer, uint32_t *res_cur, uint32_t *res_hist, float *direct, float *accum,
                    const pto_reuse_params *prm, pto_counters *cnt, const pto_motion *mot);
int pto_run_gi(int pass, int nthreads, const pto_inputs *in, int x0, int y0, int x1, int y1, const uint32_t *gbuffer,
               uint32_t *res_cur, uint32_t *res_hist, float *direct, float *accum, const pto_reuse_params *prm,
               pto_counters *cnt) {
    if (pass < PTO_GI_PASS_INIT || pass > PTO_GI_PASS_FINAL || !prm || prm->neighbors > 16u) return -2;
    return run_gi_m(pass, nthreads, in, x0, y0, x1, y1, gbuffer, res_cur, res_hist, direct, accum, prm, cnt, NULL);
}
int pto_run_gi_temporal_motion(int nthreads, const pto_inputs *in, int x0, int y0, int x1, int y1,
                               const uint32_t *gbuffer, uint32_t *res_cur, const uint32_t *res_hist,
                               const uint32_t *prev_uniform, const uint32_t *gbuffer_prev,
                               const pto_reuse_params *prm, pto_counters *cnt) {
    if (!prm || !prev_uniform || !gbuffer_prev) return -2;
    pto_motion mot = {prev_uniform, gbuffer_prev};
    return run_gi_m(PTO_GI_PASS_TEMPORAL_MOTION, nthreads, in, x0, y0, x1, y1, gbuffer, res_cur, (uint32_t *)res_hist,
                    NULL, NULL, prm, cnt, &mot);
}
static int run_gi_m(int pass, int nthreads, const pto_inputs *in, int x0, int y0, int x1, int y1,
                    const uint32_t *gbuffer, uint32_t *res_cur, uint32_t *res_hist, float *direct, float *accum,
                    const pto_reuse_params *prm, pto_counters *cnt, const pto_motion *mot) {
    if (nthreads < 1) nthreads = 1;
    gi_job *jobs = (gi_job *)calloc((size_t)nthreads, sizeof(gi_job));
    pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
    if (!jobs || !th) { free(jobs); free(th); return -1; }
    for (int t = 0; t < nthreads; ++t) {
        gi_job j = {pass, t, nthreads, x0, y0, x1, y1, in, gbuffer, res_cur, res_hist, direct, accum, prm,
                    {0, 0, 0, 0, 0}, mot};
        jobs[t] = j;
        if (nthreads > 1) pthread_create(&th[t], NULL, gi_worker, &jobs[t]);
    }
    if (nthreads == 1) gi_worker(&jobs[0]);
    for (int t = 0; t < nthreads; ++t) {
        if (nthreads > 1) pthread_join(th[t], NULL);
        if (cnt) {
            cnt->rays += jobs[t].cnt.rays;
            cnt->instance_xforms += jobs[t].cnt.instance_xforms;
            cnt->aabb_tests += jobs[t].cnt.aabb_tests;
            cnt->tri_tests += jobs[t].cnt.tri_tests;
            cnt->hits += jobs[t].cnt.hits;
        }
    }
    free(jobs);
    free(th);
    return 0;
}

/* KAT helper: gi_sample_dir on an explicit surface (mat as pto_bsdf's); returns the pdf. */
float pto_gi_sample_dir(const float n[3], const float mat[7], const float v[3], uint32_t *seed, float out_dir[3]) {
    surface s = kat_surface(n, mat);
    float pdf;
    v3 d = gi_sample_dir(seed, &s, V3(v[0], v[1], v[2]), &pdf);
    out_dir[0] = d.x; out_dir[1] = d.y; out_dir[2] = d.z;
    return pdf;
}
