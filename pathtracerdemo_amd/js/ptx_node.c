/*
 * ptx_node.c -- thin Node N-API addon over the C ABI of include/ptx.h (libptx.so).
 *
 * This is the binding a TypeScript maintainer adds behind the reference's Renderer
 * surface (apps/frontend/src/graphics-core/Renderer_TEST.ts): NativeRenderer.js calls
 * these functions where Renderer_TEST issues WebGPU calls.  Plain data only crosses the
 * boundary: typed arrays in, typed arrays / numbers / plain objects out.  Errors become
 * JS exceptions carrying ptx_last_error().  renderAsync runs ptx_render on the libuv
 * thread pool (napi_create_async_work) so the event loop never blocks; one render may be
 * in flight per handle.
 */
#define NAPI_VERSION 6
#include <node_api.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/ptx.h"

typedef struct {
    ptx_handle *h;
    int busy;             /* a renderAsync / renderBandsAsync is in flight */
    uint32_t width, band_h; /* image rows of this handle (ptx_render's output: band_h*W*4 f32) */
} Handle;

#define MAX_BANDS 64
typedef struct {
    napi_async_work work;
    napi_deferred deferred;
    napi_ref out_ref;             /* keeps the output Float32Array alive */
    napi_ref h_ref[MAX_BANDS];    /* keeps the handles alive while the job runs */
    Handle *H[MAX_BANDS];
    int n;                        /* handles: 1 (renderAsync) or the bands (renderBandsAsync) */
    int bands;                    /* ptx_render_bands instead of ptx_render */
    float *out;
    int rc;
    char err[512];
} RenderJob;

#define CHECK_NAPI(env, call)                                                    \
    do {                                                                         \
        if ((call) != napi_ok) {                                                 \
            napi_throw_error((env), NULL, "N-API call failed: " #call);          \
            return NULL;                                                         \
        }                                                                        \
    } while (0)

static int typed_view(napi_env env, napi_value v, void **data, size_t *count, size_t *elem,
                      napi_typedarray_type *type_out);

static napi_value throw_ptx(napi_env env, Handle *H, int rc, const char *what) {
    char msg[768];
    const char *detail = H && H->h ? ptx_last_error(H->h) : "";
    snprintf(msg, sizeof msg, "%s failed (%d)%s%s", what, rc, detail && *detail ? ": " : "", detail ? detail : "");
    napi_throw_error(env, NULL, msg);
    return NULL;
}

static void finalize_handle(napi_env env, void *data, void *hint) {
    (void)env;
    (void)hint;
    Handle *H = (Handle *)data;
    /* an async job holds a reference to its handles, so a busy handle is never collected;
       at environment teardown with a job still queued, leak rather than free under it */
    if (!H || H->busy) return;
    if (H->h) ptx_destroy(H->h);
    free(H);
}

/* The handle behind a JS external.  Every entry point that touches the ptx handle requires
 * it idle: a handle is single-threaded (include/ptx.h) and an async render owns it. */
static Handle *get_handle(napi_env env, napi_value v) {
    void *p = NULL;
    if (napi_get_value_external(env, v, &p) != napi_ok || !p) {
        napi_throw_type_error(env, NULL, "expected a ptx handle");
        return NULL;
    }
    Handle *H = (Handle *)p;
    if (!H->h) {
        napi_throw_error(env, NULL, "ptx handle already destroyed");
        return NULL;
    }
    if (H->busy) {
        napi_throw_error(env, NULL, "an async render is in flight on this handle");
        return NULL;
    }
    return H;
}

/* Optional Float32Array output of at least `need` floats (argv[i] absent / null -> NULL). */
static int get_out(napi_env env, size_t argc, napi_value *argv, size_t i, size_t need, float **out) {
    *out = NULL;
    if (argc <= i) return 0;
    napi_valuetype vt;
    napi_typeof(env, argv[i], &vt);
    if (vt == napi_undefined || vt == napi_null) return 0;
    void *p;
    size_t n, es;
    napi_typedarray_type t;
    if (typed_view(env, argv[i], &p, &n, &es, &t) || t != napi_float32_array) {
        napi_throw_type_error(env, NULL, "out must be a Float32Array");
        return -1;
    }
    if (n < need) {
        char msg[160];
        snprintf(msg, sizeof msg, "out holds %zu floats; the image needs %zu (rows * width * 4)", n, need);
        napi_throw_range_error(env, NULL, msg);
        return -1;
    }
    *out = (float *)p;
    return 0;
}

static int get_u32_prop(napi_env env, napi_value obj, const char *name, uint32_t dflt, uint32_t *out) {
    bool has = false;
    *out = dflt;
    if (napi_has_named_property(env, obj, name, &has) != napi_ok || !has) return 0;
    napi_value v;
    if (napi_get_named_property(env, obj, name, &v) != napi_ok) return -1;
    napi_valuetype t;
    napi_typeof(env, v, &t);
    if (t == napi_undefined || t == napi_null) return 0;
    int32_t i;
    if (napi_get_value_int32(env, v, &i) != napi_ok) return -1;
    *out = (uint32_t)i;
    return 0;
}

/* typed array view: data pointer, element count, element size */
static int typed_view(napi_env env, napi_value v, void **data, size_t *count, size_t *elem,
                      napi_typedarray_type *type_out) {
    bool is_ta = false;
    if (napi_is_typedarray(env, v, &is_ta) != napi_ok || !is_ta) return -1;
    napi_typedarray_type type;
    size_t length, offset;
    napi_value ab;
    if (napi_get_typedarray_info(env, v, &type, &length, data, &ab, &offset) != napi_ok) return -1;
    size_t es = 1;
    switch (type) {
    case napi_int8_array: case napi_uint8_array: case napi_uint8_clamped_array: es = 1; break;
    case napi_int16_array: case napi_uint16_array: es = 2; break;
    case napi_int32_array: case napi_uint32_array: case napi_float32_array: es = 4; break;
    case napi_float64_array: es = 8; break;
    default: es = 8; break;
    }
    *count = length;
    *elem = es;
    if (type_out) *type_out = type;
    return 0;
}

static napi_value js_abi_version(napi_env env, napi_callback_info info) {
    (void)info;
    napi_value r;
    CHECK_NAPI(env, napi_create_int32(env, ptx_abi_version(), &r));
    return r;
}

/* create({width, height, rowBegin, rowEnd, device, pipeline, flags, reuseRadius, reuseNeighbors,
 *         temporalCap}) -> handle */
static napi_value js_create(napi_env env, napi_callback_info info) {
    size_t argc = 1;
    napi_value argv[1];
    CHECK_NAPI(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    if (argc < 1) {
        napi_throw_type_error(env, NULL, "create(config) needs a config object");
        return NULL;
    }
    ptx_config cfg;
    memset(&cfg, 0, sizeof cfg);
    uint32_t dev = 0xffffffffu;
    if (get_u32_prop(env, argv[0], "width", 0, &cfg.width) || get_u32_prop(env, argv[0], "height", 0, &cfg.height) ||
        get_u32_prop(env, argv[0], "rowBegin", 0, &cfg.row_begin) ||
        get_u32_prop(env, argv[0], "rowEnd", 0, &cfg.row_end) || get_u32_prop(env, argv[0], "device", dev, &dev) ||
        get_u32_prop(env, argv[0], "pipeline", PTX_PIPELINE_RESTIR, &cfg.pipeline) ||
        get_u32_prop(env, argv[0], "flags", 0, &cfg.flags) ||
        get_u32_prop(env, argv[0], "reuseRadius", 0, &cfg.reuse_radius) ||
        get_u32_prop(env, argv[0], "reuseNeighbors", 0, &cfg.reuse_neighbors) ||
        get_u32_prop(env, argv[0], "temporalCap", 0, &cfg.temporal_cap)) {
        napi_throw_type_error(env, NULL, "create: config fields must be integers");
        return NULL;
    }
    cfg.device = (int32_t)dev;
    ptx_handle *h = NULL;
    int rc = ptx_create(&cfg, &h);
    if (rc != PTX_OK) return throw_ptx(env, NULL, rc, "ptx_create");
    Handle *H = (Handle *)calloc(1, sizeof(Handle));
    if (!H) {
        ptx_destroy(h);
        napi_throw_error(env, NULL, "out of memory");
        return NULL;
    }
    H->h = h;
    H->width = cfg.width;
    H->band_h = (cfg.row_begin == 0 && cfg.row_end == 0 ? cfg.height : cfg.row_end) - cfg.row_begin;
    napi_value ext;
    CHECK_NAPI(env, napi_create_external(env, H, finalize_handle, NULL, &ext));
    return ext;
}

/* uploadScene(h, Uint32Array scene, Uint32Array geometry, Uint32Array accel) */
static napi_value js_upload_scene(napi_env env, napi_callback_info info) {
    size_t argc = 4;
    napi_value argv[4];
    CHECK_NAPI(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    Handle *H = argc >= 1 ? get_handle(env, argv[0]) : NULL;
    if (!H) return NULL;
    void *p[3];
    size_t n[3], es;
    for (int i = 0; i < 3; ++i) {
        napi_typedarray_type t;
        if ((size_t)(i + 1) >= argc || typed_view(env, argv[i + 1], &p[i], &n[i], &es, &t) || t != napi_uint32_array) {
            napi_throw_type_error(env, NULL, "uploadScene(h, scene, geometry, accel) takes three Uint32Arrays");
            return NULL;
        }
    }
    int rc = ptx_upload_scene(H->h, (const uint32_t *)p[0], n[0], (const uint32_t *)p[1], n[1],
                              (const uint32_t *)p[2], n[2]);
    if (rc != PTX_OK) return throw_ptx(env, H, rc, "ptx_upload_scene");
    return NULL;
}

/* setFrame(h, Uint32Array(33)) */
static napi_value js_set_frame(napi_env env, napi_callback_info info) {
    size_t argc = 2;
    napi_value argv[2];
    CHECK_NAPI(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    Handle *H = argc >= 1 ? get_handle(env, argv[0]) : NULL;
    if (!H) return NULL;
    void *p;
    size_t n, es;
    napi_typedarray_type t;
    if (argc < 2 || typed_view(env, argv[1], &p, &n, &es, &t) || t != napi_uint32_array || n != PTX_UNIFORM_WORDS) {
        napi_throw_type_error(env, NULL, "setFrame(h, uniform) takes a Uint32Array of 33 words");
        return NULL;
    }
    int rc = ptx_set_frame(H->h, (const uint32_t *)p);
    if (rc != PTX_OK) return throw_ptx(env, H, rc, "ptx_set_frame");
    return NULL;
}

/* render(h [, Float32Array out]) -- blocking when out is given, else asynchronous on the GPU */
static napi_value js_render(napi_env env, napi_callback_info info) {
    size_t argc = 2;
    napi_value argv[2];
    CHECK_NAPI(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    Handle *H = argc >= 1 ? get_handle(env, argv[0]) : NULL;
    if (!H) return NULL;
    float *out = NULL;
    if (get_out(env, argc, argv, 1, (size_t)H->band_h * H->width * 4u, &out)) return NULL;
    int rc = ptx_render(H->h, out);
    if (rc != PTX_OK) return throw_ptx(env, H, rc, "ptx_render");
    return NULL;
}

static void render_execute(napi_env env, void *data) {
    (void)env;
    RenderJob *J = (RenderJob *)data;
    ptx_handle *hs[MAX_BANDS];
    for (int i = 0; i < J->n; ++i) hs[i] = J->H[i]->h;
    J->rc = J->bands ? ptx_render_bands(hs, J->n, J->out) : ptx_render(hs[0], J->out);
    for (int i = 0; i < J->n && J->rc == PTX_OK; ++i) J->rc = ptx_synchronize(hs[i]);
    if (J->rc != PTX_OK) {
        const char *m = "";
        for (int i = 0; i < J->n && !*m; ++i) m = ptx_last_error(hs[i]);
        snprintf(J->err, sizeof J->err, "render failed (%d): %s", J->rc, m);
    }
}

static void render_complete(napi_env env, napi_status status, void *data) {
    RenderJob *J = (RenderJob *)data;
    for (int i = 0; i < J->n; ++i) {
        J->H[i]->busy = 0;
        if (J->h_ref[i]) napi_delete_reference(env, J->h_ref[i]);
    }
    napi_value v;
    if (status == napi_ok && J->rc == PTX_OK) {
        napi_get_undefined(env, &v);
        napi_resolve_deferred(env, J->deferred, v);
    } else {
        napi_value msg;
        napi_create_string_utf8(env, J->err[0] ? J->err : "render cancelled", NAPI_AUTO_LENGTH, &msg);
        napi_create_error(env, NULL, msg, &v);
        napi_reject_deferred(env, J->deferred, v);
    }
    if (J->out_ref) napi_delete_reference(env, J->out_ref);
    napi_delete_async_work(env, J->work);
    free(J);
}

/* Queue a render job over handles argv_h[0..n) (already validated idle). */
static napi_value queue_render(napi_env env, napi_value *argv_h, Handle **H, int n, int bands, napi_value out_v,
                               float *out) {
    RenderJob *J = (RenderJob *)calloc(1, sizeof(RenderJob));
    if (!J) {
        napi_throw_error(env, NULL, "out of memory");
        return NULL;
    }
    J->n = n;
    J->bands = bands;
    J->out = out;
    if (out) CHECK_NAPI(env, napi_create_reference(env, out_v, 1, &J->out_ref));
    for (int i = 0; i < n; ++i) {
        J->H[i] = H[i];
        CHECK_NAPI(env, napi_create_reference(env, argv_h[i], 1, &J->h_ref[i]));
    }
    napi_value promise, name;
    CHECK_NAPI(env, napi_create_promise(env, &J->deferred, &promise));
    CHECK_NAPI(env, napi_create_string_utf8(env, bands ? "ptx_render_bands" : "ptx_render", NAPI_AUTO_LENGTH, &name));
    CHECK_NAPI(env, napi_create_async_work(env, NULL, name, render_execute, render_complete, J, &J->work));
    for (int i = 0; i < n; ++i) H[i]->busy = 1;
    CHECK_NAPI(env, napi_queue_async_work(env, J->work));
    return promise;
}

/* renderAsync(h [, Float32Array out]) -> Promise: ptx_render + synchronize off the event loop;
 * the handle stays busy (every other call on it throws) until the promise settles */
static napi_value js_render_async(napi_env env, napi_callback_info info) {
    size_t argc = 2;
    napi_value argv[2];
    CHECK_NAPI(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    Handle *H = argc >= 1 ? get_handle(env, argv[0]) : NULL;
    if (!H) return NULL;
    float *out = NULL;
    if (get_out(env, argc, argv, 1, (size_t)H->band_h * H->width * 4u, &out)) return NULL;
    return queue_render(env, argv, &H, 1, 0, argc >= 2 ? argv[1] : NULL, out);
}

/* The band handles of an array argument (idle, distinct, at most MAX_BANDS). */
static int band_handles(napi_env env, napi_value arr, napi_value *hv, Handle **H, uint32_t *n, size_t *rows,
                        uint32_t *width) {
    bool is_array = false;
    if (napi_is_array(env, arr, &is_array) != napi_ok || !is_array || napi_get_array_length(env, arr, n) != napi_ok ||
        *n < 1 || *n > MAX_BANDS) {
        napi_throw_type_error(env, NULL, "expected an array of 1..64 band handles");
        return -1;
    }
    *rows = 0;
    for (uint32_t i = 0; i < *n; ++i) {
        if (napi_get_element(env, arr, i, &hv[i]) != napi_ok || !(H[i] = get_handle(env, hv[i]))) return -1;
        for (uint32_t k = 0; k < i; ++k)
            if (H[k] == H[i]) {
                napi_throw_error(env, NULL, "a band handle appears twice");
                return -1;
            }
        *rows += H[i]->band_h;
        *width = H[i]->width;
    }
    return 0;
}

/* renderBands([h...] [, Float32Array out]) -- one frame over the band handles of this process
 * (ptx_render_bands: halo over their communicators or peer copies); blocking */
static napi_value js_render_bands(napi_env env, napi_callback_info info) {
    size_t argc = 2;
    napi_value argv[2], hv[MAX_BANDS];
    CHECK_NAPI(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    Handle *H[MAX_BANDS];
    uint32_t n = 0, width = 0;
    size_t rows = 0;
    if (argc < 1 || band_handles(env, argv[0], hv, H, &n, &rows, &width)) return NULL;
    float *out = NULL;
    if (get_out(env, argc, argv, 1, rows * width * 4u, &out)) return NULL;
    ptx_handle *hs[MAX_BANDS];
    for (uint32_t i = 0; i < n; ++i) hs[i] = H[i]->h;
    int rc = ptx_render_bands(hs, (int)n, out);
    if (rc != PTX_OK) {
        for (uint32_t i = 0; i < n; ++i)
            if (*ptx_last_error(H[i]->h)) return throw_ptx(env, H[i], rc, "ptx_render_bands");
        return throw_ptx(env, H[0], rc, "ptx_render_bands");
    }
    return NULL;
}

/* renderBandsAsync([h...] [, Float32Array out]) -> Promise */
static napi_value js_render_bands_async(napi_env env, napi_callback_info info) {
    size_t argc = 2;
    napi_value argv[2], hv[MAX_BANDS];
    CHECK_NAPI(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    Handle *H[MAX_BANDS];
    uint32_t n = 0, width = 0;
    size_t rows = 0;
    if (argc < 1 || band_handles(env, argv[0], hv, H, &n, &rows, &width)) return NULL;
    float *out = NULL;
    if (get_out(env, argc, argv, 1, rows * width * 4u, &out)) return NULL;
    return queue_render(env, hv, H, (int)n, 1, argc >= 2 ? argv[1] : NULL, out);
}

/* commUniqueId() -> Uint8Array(128): ncclGetUniqueId, to ship to the other ranks */
static napi_value js_comm_unique_id(napi_env env, napi_callback_info info) {
    (void)info;
    napi_value ab, arr;
    void *p = NULL;
    CHECK_NAPI(env, napi_create_arraybuffer(env, PTX_COMM_ID_BYTES, &p, &ab));
    int rc = ptx_comm_unique_id(p, PTX_COMM_ID_BYTES);
    if (rc != PTX_OK) return throw_ptx(env, NULL, rc, "ptx_comm_unique_id (is RCCL installed?)");
    CHECK_NAPI(env, napi_create_typedarray(env, napi_uint8_array, PTX_COMM_ID_BYTES, ab, 0, &arr));
    return arr;
}

/* commInit(h, Uint8Array(128) id, rank, world): the handle's own RCCL communicator */
static napi_value js_comm_init(napi_env env, napi_callback_info info) {
    size_t argc = 4;
    napi_value argv[4];
    CHECK_NAPI(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    Handle *H = argc >= 1 ? get_handle(env, argv[0]) : NULL;
    if (!H) return NULL;
    void *p;
    size_t n, es;
    int32_t rank = -1, world = 0;
    if (argc < 4 || typed_view(env, argv[1], &p, &n, &es, NULL) || n * es != PTX_COMM_ID_BYTES ||
        napi_get_value_int32(env, argv[2], &rank) != napi_ok || napi_get_value_int32(env, argv[3], &world) != napi_ok) {
        napi_throw_type_error(env, NULL, "commInit(h, id: Uint8Array(128), rank, world)");
        return NULL;
    }
    int rc = ptx_comm_init(H->h, p, PTX_COMM_ID_BYTES, rank, world);
    if (rc != PTX_OK) return throw_ptx(env, H, rc, "ptx_comm_init");
    return NULL;
}

/* commInitAll([h...]): ncclCommInitAll over the band handles of this process (one per GPU) */
static napi_value js_comm_init_all(napi_env env, napi_callback_info info) {
    size_t argc = 1;
    napi_value argv[1], hv[MAX_BANDS];
    CHECK_NAPI(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    Handle *H[MAX_BANDS];
    uint32_t n = 0, width = 0;
    size_t rows = 0;
    if (argc < 1 || band_handles(env, argv[0], hv, H, &n, &rows, &width)) return NULL;
    ptx_handle *hs[MAX_BANDS];
    for (uint32_t i = 0; i < n; ++i) hs[i] = H[i]->h;
    int rc = ptx_comm_init_all(hs, (int)n);
    if (rc != PTX_OK) return throw_ptx(env, H[0], rc, "ptx_comm_init_all");
    return NULL;
}

/* rowCensus(h, BigUint64Array(tileRows * 5)) -- PTX_FLAG_ROW_CENSUS handles */
static napi_value js_row_census(napi_env env, napi_callback_info info) {
    size_t argc = 2;
    napi_value argv[2];
    CHECK_NAPI(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    Handle *H = argc >= 1 ? get_handle(env, argv[0]) : NULL;
    if (!H) return NULL;
    void *p;
    size_t n, es;
    napi_typedarray_type t;
    if (argc < 2 || typed_view(env, argv[1], &p, &n, &es, &t) || t != napi_biguint64_array || n % 5) {
        napi_throw_type_error(env, NULL, "rowCensus(h, out: BigUint64Array(tileRows * 5))");
        return NULL;
    }
    int rc = ptx_row_census(H->h, (uint64_t *)p, n / 5);
    if (rc != PTX_OK) return throw_ptx(env, H, rc, "ptx_row_census");
    return NULL;
}

static napi_value simple_call(napi_env env, napi_callback_info info, int (*fn)(ptx_handle *), const char *what) {
    size_t argc = 1;
    napi_value argv[1];
    CHECK_NAPI(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    Handle *H = argc >= 1 ? get_handle(env, argv[0]) : NULL;
    if (!H) return NULL;
    int rc = fn(H->h);
    if (rc != PTX_OK) return throw_ptx(env, H, rc, what);
    return NULL;
}
static napi_value js_reset_accumulation(napi_env env, napi_callback_info info) {
    return simple_call(env, info, ptx_reset_accumulation, "ptx_reset_accumulation");
}
static napi_value js_synchronize(napi_env env, napi_callback_info info) {
    return simple_call(env, info, ptx_synchronize, "ptx_synchronize");
}
static napi_value js_reset_stats(napi_env env, napi_callback_info info) {
    return simple_call(env, info, ptx_reset_stats, "ptx_reset_stats");
}

/* runPass(h, pass) */
static napi_value js_run_pass(napi_env env, napi_callback_info info) {
    size_t argc = 2;
    napi_value argv[2];
    CHECK_NAPI(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    Handle *H = argc >= 1 ? get_handle(env, argv[0]) : NULL;
    if (!H) return NULL;
    int32_t pass = -1;
    if (argc < 2 || napi_get_value_int32(env, argv[1], &pass) != napi_ok) {
        napi_throw_type_error(env, NULL, "runPass(h, pass) needs an integer pass");
        return NULL;
    }
    int rc = ptx_run_pass(H->h, pass);
    if (rc != PTX_OK) return throw_ptx(env, H, rc, "ptx_run_pass");
    return NULL;
}

/* runPasses(h, [pass, ...]) -- one overlapped launch sequence (ptx_run_passes) */
static napi_value js_run_passes(napi_env env, napi_callback_info info) {
    size_t argc = 2;
    napi_value argv[2];
    CHECK_NAPI(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    Handle *H = argc >= 1 ? get_handle(env, argv[0]) : NULL;
    if (!H) return NULL;
    bool is_array = false;
    uint32_t n = 0;
    if (argc < 2 || napi_is_array(env, argv[1], &is_array) != napi_ok || !is_array ||
        napi_get_array_length(env, argv[1], &n) != napi_ok || n > 8) {
        napi_throw_type_error(env, NULL, "runPasses(h, passes) needs an array of at most 8 passes");
        return NULL;
    }
    int passes[8];
    for (uint32_t i = 0; i < n; ++i) {
        napi_value e;
        int32_t p = -1;
        if (napi_get_element(env, argv[1], i, &e) != napi_ok || napi_get_value_int32(env, e, &p) != napi_ok) {
            napi_throw_type_error(env, NULL, "runPasses: passes must be integers");
            return NULL;
        }
        passes[i] = p;
    }
    int rc = ptx_run_passes(H->h, passes, (int)n);
    if (rc != PTX_OK) return throw_ptx(env, H, rc, "ptx_run_passes");
    return NULL;
}

/* read/writeBuffer(h, which, TypedArray) -- byte count = the array's byte length */
static napi_value buffer_io(napi_env env, napi_callback_info info, int write) {
    size_t argc = 3;
    napi_value argv[3];
    CHECK_NAPI(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    Handle *H = argc >= 1 ? get_handle(env, argv[0]) : NULL;
    if (!H) return NULL;
    int32_t which = -1;
    void *p;
    size_t n, es;
    if (argc < 3 || napi_get_value_int32(env, argv[1], &which) != napi_ok ||
        typed_view(env, argv[2], &p, &n, &es, NULL)) {
        napi_throw_type_error(env, NULL, "read/writeBuffer(h, which, typedArray)");
        return NULL;
    }
    int rc = write ? ptx_write_buffer(H->h, which, p, n * es) : ptx_read_buffer(H->h, which, p, n * es);
    if (rc != PTX_OK) return throw_ptx(env, H, rc, write ? "ptx_write_buffer" : "ptx_read_buffer");
    return NULL;
}
static napi_value js_read_buffer(napi_env env, napi_callback_info info) { return buffer_io(env, info, 0); }
static napi_value js_write_buffer(napi_env env, napi_callback_info info) { return buffer_io(env, info, 1); }

/* trace(h, Float32Array rays (n*8), Float32Array hits (n*8), epsMode) */
static napi_value js_trace(napi_env env, napi_callback_info info) {
    size_t argc = 4;
    napi_value argv[4];
    CHECK_NAPI(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    Handle *H = argc >= 1 ? get_handle(env, argv[0]) : NULL;
    if (!H) return NULL;
    void *pr, *ph;
    size_t nr, nh, es;
    napi_typedarray_type tr, th;
    int32_t eps = 1;
    if (argc < 3 || typed_view(env, argv[1], &pr, &nr, &es, &tr) || typed_view(env, argv[2], &ph, &nh, &es, &th) ||
        tr != napi_float32_array || th != napi_float32_array || nr % 8 || nh < nr) {
        napi_throw_type_error(env, NULL, "trace(h, rays: Float32Array n*8, hits: Float32Array n*8, epsMode)");
        return NULL;
    }
    if (argc >= 4) napi_get_value_int32(env, argv[3], &eps);
    int rc = ptx_trace(H->h, (const float *)pr, (float *)ph, nr / 8, eps);
    if (rc != PTX_OK) return throw_ptx(env, H, rc, "ptx_trace");
    return NULL;
}

/* getStats(h) -> {frames, kernelMsTotal[16], kernelLaunches[16], triangles, bvhNodes, instances, maxBvhDepth,
 *                 deviceBytes} */
static napi_value js_get_stats(napi_env env, napi_callback_info info) {
    size_t argc = 1;
    napi_value argv[1];
    CHECK_NAPI(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    Handle *H = argc >= 1 ? get_handle(env, argv[0]) : NULL;
    if (!H) return NULL;
    ptx_stats st;
    int rc = ptx_get_stats(H->h, &st);
    if (rc != PTX_OK) return throw_ptx(env, H, rc, "ptx_get_stats");
    napi_value o, v, ms, la;
    CHECK_NAPI(env, napi_create_object(env, &o));
    const uint32_t nslots = (uint32_t)(sizeof st.kernel_launches / sizeof st.kernel_launches[0]);
    CHECK_NAPI(env, napi_create_array_with_length(env, nslots, &ms));
    CHECK_NAPI(env, napi_create_array_with_length(env, nslots, &la));
    for (uint32_t i = 0; i < nslots; ++i) {
        napi_create_double(env, st.kernel_ms_total[i], &v);
        napi_set_element(env, ms, i, v);
        napi_create_double(env, (double)st.kernel_launches[i], &v);
        napi_set_element(env, la, i, v);
    }
    napi_set_named_property(env, o, "kernelMsTotal", ms);
    napi_set_named_property(env, o, "kernelLaunches", la);
    napi_create_double(env, (double)st.frames, &v);
    napi_set_named_property(env, o, "frames", v);
    napi_create_uint32(env, st.triangles, &v);
    napi_set_named_property(env, o, "triangles", v);
    napi_create_uint32(env, st.bvh_nodes, &v);
    napi_set_named_property(env, o, "bvhNodes", v);
    napi_create_uint32(env, st.instances, &v);
    napi_set_named_property(env, o, "instances", v);
    napi_create_uint32(env, st.max_bvh_depth, &v);
    napi_set_named_property(env, o, "maxBvhDepth", v);
    napi_create_double(env, (double)st.device_bytes, &v);
    napi_set_named_property(env, o, "deviceBytes", v);
    return o;
}

/* destroy(h) -- idempotent; the GC finalizer also releases an undestroyed handle */
static napi_value js_destroy(napi_env env, napi_callback_info info) {
    size_t argc = 1;
    napi_value argv[1];
    CHECK_NAPI(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    void *p = NULL;
    if (argc < 1 || napi_get_value_external(env, argv[0], &p) != napi_ok || !p) {
        napi_throw_type_error(env, NULL, "destroy(h) needs a ptx handle");
        return NULL;
    }
    Handle *H = (Handle *)p;
    if (H->busy) {
        napi_throw_error(env, NULL, "destroy: a renderAsync is in flight");
        return NULL;
    }
    if (H->h) ptx_destroy(H->h);
    H->h = NULL;
    return NULL;
}

static napi_value js_last_error(napi_env env, napi_callback_info info) {
    size_t argc = 1;
    napi_value argv[1], s;
    CHECK_NAPI(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    Handle *H = argc >= 1 ? get_handle(env, argv[0]) : NULL;
    if (!H) return NULL;
    CHECK_NAPI(env, napi_create_string_utf8(env, ptx_last_error(H->h), NAPI_AUTO_LENGTH, &s));
    return s;
}

/* present(handle, canvasW, canvasH, bgra, out: Uint8Array | Uint8ClampedArray of canvasW * canvasH * 4):
 * the reference's render pass onto the canvas (ptx_present, include/ptx.h) */
static napi_value js_present(napi_env env, napi_callback_info info) {
    size_t argc = 5;
    napi_value argv[5];
    CHECK_NAPI(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    Handle *H = argc >= 1 ? get_handle(env, argv[0]) : NULL;
    if (!H) return NULL;
    if (argc < 5) {
        napi_throw_type_error(env, NULL, "present(handle, canvasW, canvasH, bgra, out)");
        return NULL;
    }
    uint32_t cw = 0, ch = 0;
    bool bgra = false;
    CHECK_NAPI(env, napi_get_value_uint32(env, argv[1], &cw));
    CHECK_NAPI(env, napi_get_value_uint32(env, argv[2], &ch));
    CHECK_NAPI(env, napi_get_value_bool(env, argv[3], &bgra));
    void *p;
    size_t n, es;
    napi_typedarray_type t;
    if (typed_view(env, argv[4], &p, &n, &es, &t) || (t != napi_uint8_array && t != napi_uint8_clamped_array)) {
        napi_throw_type_error(env, NULL, "out must be a Uint8Array or Uint8ClampedArray");
        return NULL;
    }
    if (n < (size_t)cw * ch * 4u) {
        napi_throw_range_error(env, NULL, "out holds fewer than canvasW * canvasH * 4 bytes");
        return NULL;
    }
    int rc = ptx_present(H->h, cw, ch, bgra ? 1 : 0, (uint8_t *)p);
    if (rc != PTX_OK) return throw_ptx(env, H, rc, "ptx_present");
    return NULL;
}

/* presentAsync(handle, canvasW, canvasH, bgra): enqueue the render pass for the frame last rendered
 * without waiting (ptx_present_async); presentPoll fetches the bytes */
static napi_value js_present_async(napi_env env, napi_callback_info info) {
    size_t argc = 4;
    napi_value argv[4];
    CHECK_NAPI(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    Handle *H = argc >= 1 ? get_handle(env, argv[0]) : NULL;
    if (!H) return NULL;
    if (argc < 4) {
        napi_throw_type_error(env, NULL, "presentAsync(handle, canvasW, canvasH, bgra)");
        return NULL;
    }
    uint32_t cw = 0, ch = 0;
    bool bgra = false;
    CHECK_NAPI(env, napi_get_value_uint32(env, argv[1], &cw));
    CHECK_NAPI(env, napi_get_value_uint32(env, argv[2], &ch));
    CHECK_NAPI(env, napi_get_value_bool(env, argv[3], &bgra));
    int rc = ptx_present_async(H->h, cw, ch, bgra ? 1 : 0);
    if (rc != PTX_OK) return throw_ptx(env, H, rc, "ptx_present_async");
    return NULL;
}

/* presentPoll(handle, out: Uint8Array | Uint8ClampedArray) -> true once the bytes are in `out`,
 * false while the present is in flight (ptx_present_poll: never waits) */
static napi_value js_present_poll(napi_env env, napi_callback_info info) {
    size_t argc = 2;
    napi_value argv[2];
    CHECK_NAPI(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    Handle *H = argc >= 1 ? get_handle(env, argv[0]) : NULL;
    if (!H) return NULL;
    void *p;
    size_t n, es;
    napi_typedarray_type t;
    if (argc < 2 || typed_view(env, argv[1], &p, &n, &es, &t) || (t != napi_uint8_array && t != napi_uint8_clamped_array)) {
        napi_throw_type_error(env, NULL, "presentPoll(handle, out: Uint8Array | Uint8ClampedArray)");
        return NULL;
    }
    int rc = ptx_present_poll(H->h, (uint8_t *)p, n);
    if (rc != PTX_OK && rc != PTX_E_PENDING) return throw_ptx(env, H, rc, "ptx_present_poll");
    napi_value r;
    CHECK_NAPI(env, napi_get_boolean(env, rc == PTX_OK, &r));
    return r;
}

/* buildInfo() -> the JSON string of ptx_build_info (which libptx.so build is loaded) */
static napi_value js_build_info(napi_env env, napi_callback_info info) {
    (void)info;
    char buf[2048];
    ptx_build_info(buf, sizeof buf);
    napi_value s;
    CHECK_NAPI(env, napi_create_string_utf8(env, buf, NAPI_AUTO_LENGTH, &s));
    return s;
}

static napi_value init(napi_env env, napi_value exports) {
    static const struct {
        const char *name;
        napi_callback fn;
    } fns[] = {
        {"abiVersion", js_abi_version},     {"create", js_create},
        {"uploadScene", js_upload_scene},   {"setFrame", js_set_frame},
        {"render", js_render},              {"renderAsync", js_render_async},
        {"runPass", js_run_pass},           {"runPasses", js_run_passes},           {"resetAccumulation", js_reset_accumulation},
        {"synchronize", js_synchronize},    {"getStats", js_get_stats},
        {"resetStats", js_reset_stats},     {"readBuffer", js_read_buffer},
        {"writeBuffer", js_write_buffer},   {"trace", js_trace},
        {"destroy", js_destroy},            {"lastError", js_last_error},
        {"renderBands", js_render_bands},   {"renderBandsAsync", js_render_bands_async},
        {"commUniqueId", js_comm_unique_id}, {"commInit", js_comm_init},
        {"commInitAll", js_comm_init_all},  {"rowCensus", js_row_census},
        {"present", js_present},            {"presentAsync", js_present_async},
        {"presentPoll", js_present_poll},   {"buildInfo", js_build_info},
    };
    for (size_t i = 0; i < sizeof fns / sizeof fns[0]; ++i) {
        napi_value f;
        if (napi_create_function(env, fns[i].name, NAPI_AUTO_LENGTH, fns[i].fn, NULL, &f) != napi_ok ||
            napi_set_named_property(env, exports, fns[i].name, f) != napi_ok)
            return NULL;
    }
    return exports;
}

NAPI_MODULE(NODE_GYP_MODULE_NAME, init)
