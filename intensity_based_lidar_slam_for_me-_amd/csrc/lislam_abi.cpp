// C ABI of liblislam (include/lislam.h): contexts, device-resident batches, the single-scan
// scanRegistration / laserOdometry drop-ins and the batched functor evaluation.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/lislam.h"
#include "lislam_batch.hpp"
#include "lislam_ctx.hpp"
#include "lislam_internal.hpp"

using namespace lislam;


namespace {

int fail(lislam_ctx* c, int code, const char* fmt, ...) {
  if (c) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    c->err = buf;
  }
  return code;
}

#define HIPCHK(ctx, x)                                                                  \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess) return fail(ctx, LISLAM_ERR_DEVICE, "%s: %s", #x, hipGetErrorString(e_)); \
  } while (0)

template <typename T>
int dalloc(lislam_batch* b, T** p, size_t count) {
  void* q = nullptr;
  hipError_t e = hipMalloc(&q, std::max<size_t>(count, 1) * sizeof(T));
  if (e != hipSuccess) return fail(b->ctx, LISLAM_ERR_DEVICE, "hipMalloc(%zu): %s", count * sizeof(T), hipGetErrorString(e));
  b->allocs.push_back(q);
  *p = static_cast<T*>(q);
  // developer: LISLAM_POISON=<byte> fills every new batch buffer with that byte (a read-before-write
  // hunt: 255 = NaN doubles / -1 ints); LISLAM_POISON_LO / _HI: only buffers lo .. hi (1-based order)
  if (const char* e = getenv("LISLAM_POISON")) {
    const int lo = getenv("LISLAM_POISON_LO") ? atoi(getenv("LISLAM_POISON_LO")) : 0;
    const int hi = getenv("LISLAM_POISON_HI") ? atoi(getenv("LISLAM_POISON_HI")) : 1 << 30;
    const int i = (int)b->allocs.size();
    if (i >= lo && i <= hi) (void)hipMemset(q, atoi(e), std::max<size_t>(count, 1) * sizeof(T));
  }
  return LISLAM_OK;
}

bool valid_lines(int n) { return n == 16 || n == 32 || n == 64 || n == 128; }

bool is_packed(const lislam_point_layout* L) {
  return !L || (L->point_step == 16 && L->off_x == 0 && L->off_y == 4 && L->off_z == 8 && L->off_intensity == 12);
}

}  // namespace

namespace lislam {

static hipEvent_t g_epoch[64] = {};

void timeline_epoch(int dev, hipStream_t s) {
  if (!getenv("LISLAM_TIMELINE") || dev < 0 || dev >= 64 || g_epoch[dev]) return;
  if (hipEventCreate(&g_epoch[dev]) == hipSuccess) (void)hipEventRecord(g_epoch[dev], s);
}

void timeline_print(int dev, const char* who, const void* obj, int kernel, hipEvent_t b, hipEvent_t e) {
  if (dev < 0 || dev >= 64 || !g_epoch[dev]) return;
  float t0 = 0, t1 = 0;
  if (hipEventElapsedTime(&t0, g_epoch[dev], b) != hipSuccess || hipEventElapsedTime(&t1, g_epoch[dev], e) != hipSuccess) return;
  fprintf(stderr, "timeline %s %p %d %.3f %.3f\n", who, obj, kernel, t0, t1);
}

}  // namespace lislam

extern "C" {

// live contexts per device: the device's shared engine streams go with the last one
static std::atomic<int> g_ctx_count[64];

int lislam_ctx_create(const lislam_config* cfg, int32_t device, lislam_ctx** out) {
  if (!cfg || !out) return LISLAM_ERR_ARG;
  *out = nullptr;
  if (!valid_lines(cfg->n_scans) || cfg->width <= 0 || cfg->max_iterations < 0) return LISLAM_ERR_ARG;
  lislam_ctx* c = new lislam_ctx();
  c->cfg = *cfg;
  c->device = device;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0 || device < 0 || device >= ndev) {
    delete c;
    return LISLAM_ERR_DEVICE;
  }
  if (hipSetDevice(device) != hipSuccess || !lislam::work_stream(device, &c->own_stream)) {
    delete c;
    return LISLAM_ERR_DEVICE;
  }
  c->stream = c->own_stream;
  timeline_epoch(device, c->stream);
  // LISLAM_ENGINE (0 off, 1 auto, 2 on) seeds the odometry schedule; lislam_set_odometry_schedule
  // changes it per context
  if (const char* e = getenv("LISLAM_ENGINE")) {
    const int m = atoi(e);
    if (m >= LISLAM_ENGINE_OFF && m <= LISLAM_ENGINE_ON) c->odom_engine = m;
  }
  // LISLAM_ENGINE_QPW / LISLAM_ENGINE_DEPTH seed the engine's shape (lislam_set_engine_shape)
  if (const char* e = getenv("LISLAM_ENGINE_QPW")) c->eng_qpw = std::min(4, std::max(1, atoi(e)));
  if (const char* e = getenv("LISLAM_ENGINE_DEPTH")) c->eng_depth = std::min(lislam::kMaxEngineDepth, std::max(1, atoi(e)));
  if (device < 64) ++g_ctx_count[device];
  *out = c;
  return LISLAM_OK;
}

int lislam_ctx_destroy(lislam_ctx* c) {
  if (!c) return LISLAM_OK;
  hipSetDevice(c->device);
  if (c->single) lislam_batch_destroy(c->single);
  if (c->map_scratch) {
    (void)hipStreamSynchronize(c->stream);
    lislam_free_map_scratch(c->map_scratch);
  }
  if (c->factor_buf) {
    (void)hipStreamSynchronize(c->stream);
    (void)hipFree(c->factor_buf);
  }
  if (c->own_stream) lislam::destroy_stream(c->own_stream);
  const int dev = c->device;
  delete c;
  if (dev >= 0 && dev < 64 && --g_ctx_count[dev] == 0) lislam::release_engine_streams(dev);
  return LISLAM_OK;
}

const char* lislam_last_error(const lislam_ctx* c) { return c ? c->err.c_str() : "null context"; }

static int engine_settle(lislam_batch* b);

// The per-round schedule's chain groups: 2 streams, so one group's solves overlap another's
// association (a solve occupies one workgroup per chain, far from filling the device).  Group 0
// runs on the context stream; the other groups' streams belong to the device (lislam::round_stream,
// made when that schedule first runs, shared by every batch): running that schedule adds one
// hardware queue to the process, not one per batch.
static int round_streams(lislam_batch* b) {
  lislam_ctx* c = b->ctx;
  b->odo_stream[0] = c->stream;
  for (int g = 1; g < lislam_batch::kGroups; g++) {
    if (!b->odo_stream[g] && !(b->odo_stream[g] = lislam::round_stream(c->device, g)))
      return fail(c, LISLAM_ERR_DEVICE, "stream");
    if (!b->odo_join[g]) HIPCHK(c, hipEventCreateWithFlags(&b->odo_join[g], hipEventDisableTiming));
  }
  if (lislam_batch::kGroups > 1 && !b->odo_fork) HIPCHK(c, hipEventCreateWithFlags(&b->odo_fork, hipEventDisableTiming));
  return LISLAM_OK;
}

int lislam_synchronize(lislam_ctx* c) {
  if (!c) return LISLAM_ERR_ARG;
  hipSetDevice(c->device);
  for (lislam_batch* b : c->batches) {
    const int rc = engine_settle(b);
    if (rc != LISLAM_OK) return rc;
  }
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return LISLAM_OK;
}

int lislam_set_stream(lislam_ctx* c, void* s) {
  if (!c) return LISLAM_ERR_ARG;
  c->stream = s ? static_cast<hipStream_t>(s) : c->own_stream;
  return LISLAM_OK;
}

int lislam_get_stream(lislam_ctx* c, void** s) {
  if (!c || !s) return LISLAM_ERR_ARG;
  *s = c->stream;
  return LISLAM_OK;
}

// ------------------------------------------------------------------------------ batch
// The context stream waits for the batch's split engine launch, if one is pending, and the outcome of
// the last engine launch is resolved (lislam_batch.hpp): an aborted launch is re-run on the per-round
// schedule, queued on the context stream ahead of whatever the calling batch function queues next.
static int engine_settle(lislam_batch* b) {
  if (!b->eng_pending && !b->eng_check) return LISLAM_OK;
  lislam_ctx* c = b->ctx;
  hipSetDevice(c->device);
  if (b->eng_pending) {
    lislam::wait_engine_launched(&b->eng_req);  // the dispatcher has recorded the join events
    HIPCHK(c, hipStreamWaitEvent(c->stream, b->eng_join_r, 0));
    HIPCHK(c, hipStreamWaitEvent(c->stream, b->eng_join_i, 0));
    b->eng_pending = false;
  }
  if (!b->eng_check) return LISLAM_OK;
  // the host waits for the engine itself (not the context stream, which may hold later work)
  HIPCHK(c, hipEventSynchronize(b->eng_done));
  // h_abort: the engine's error word (which wait gave up) and its sticky abort word
  if (b->h_abort[1] == 0) {
    b->eng_check = false;
    return LISLAM_OK;
  }
  // eng_check stays set until the re-run is queued: a failure below leaves the recovery to the
  // batch's next call instead of losing it
  HIPCHK(c, hipMemsetAsync(b->oa.eng_ctl + 3, 0, sizeof(unsigned), c->stream));
  // the per-round schedule has no device waits: it cannot abort
  if (round_streams(b) != LISLAM_OK) return LISLAM_ERR_DEVICE;
  lislam::launch_odometry(b->eng_args, b->odo_stream, lislam_batch::kGroups, b->odo_fork, b->odo_join, nullptr,
                          &lislam_batch::event_cb, b);
  HIPCHK(c, hipGetLastError());
  b->eng_abort_code = b->h_abort[0];
  b->h_abort[0] = b->h_abort[1] = 0;
  b->eng_fallbacks++;
  b->eng_check = false;
  return LISLAM_OK;
}
#define SETTLE(b)                           \
  do {                                      \
    const int rc_ = engine_settle(b);       \
    if (rc_ != LISLAM_OK) return rc_;       \
  } while (0)

int lislam_batch_create(lislam_ctx* c, int32_t max_scans, lislam_batch** out) {
  if (!c || !out || max_scans < 1) return LISLAM_ERR_ARG;
  hipSetDevice(c->device);
  lislam_batch* b = new lislam_batch();
  b->ctx = c;
  hipEventCreateWithFlags(&b->ev_images, hipEventDisableTiming);
  hipEventCreateWithFlags(&b->eng_ready, hipEventDisableTiming);
  c->batches.push_back(b);
  const int S = max_scans, H = c->cfg.n_scans, W = c->cfg.width, N = H * W;
  b->max_scans = S; b->H = H; b->W = W; b->N = N;
  b->cap_sharp = kCapSharpPerLine * H;
  b->cap_less_sharp = kCapLessSharpPerLine * H;
  b->cap_flat = kCapFlatPerLine * H;
  FeatureArgs& f = b->fa;
  f.S = S; f.H = H; f.W = W; f.N = N; f.min_range = c->cfg.min_range;
  const size_t SN = (size_t)S * N;
  int rc = LISLAM_OK;
  P4* pts = nullptr;
  rc |= dalloc(b, &pts, SN);
  f.pts = pts;
  if (c->cfg.want_images) {
    rc |= dalloc(b, &f.img_range, SN);
    rc |= dalloc(b, &f.img_int, SN);
    rc |= dalloc(b, &f.track, SN);
  }
  rc |= dalloc(b, &f.cloud, SN);
  rc |= dalloc(b, &f.n_cloud, S);
  rc |= dalloc(b, &f.line_off, (size_t)S * (H + 1));
  rc |= dalloc(b, &f.curv, SN);
  rc |= dalloc(b, &f.label, SN);
  rc |= dalloc(b, &f.stg_sharp, (size_t)S * H * kCapSharpPerLine);
  rc |= dalloc(b, &f.stg_less_sharp, (size_t)S * H * kCapLessSharpPerLine);
  rc |= dalloc(b, &f.stg_flat, (size_t)S * H * kCapFlatPerLine);
  rc |= dalloc(b, &f.stg_less_flat, SN);
  rc |= dalloc(b, &f.line_counts, (size_t)S * H * 4);
  f.fr_R = (N + 1023) / 1024;
  rc |= dalloc(b, &f.fr_hist, (size_t)S * f.fr_R * H);
  rc |= dalloc(b, &f.fr_flip, (size_t)S * f.fr_R);
  rc |= dalloc(b, &f.fr_ori, (size_t)S * 2);
  rc |= dalloc(b, &f.scr_picked, SN);
  rc |= dalloc(b, &f.scr_keys, 2 * SN);
  rc |= dalloc(b, &f.scr_list, SN);
  rc |= dalloc(b, &f.scr_link, SN);
  rc |= dalloc(b, &f.sharp, (size_t)S * b->cap_sharp);
  rc |= dalloc(b, &f.less_sharp, (size_t)S * b->cap_less_sharp);
  rc |= dalloc(b, &f.flat, (size_t)S * b->cap_flat);
  rc |= dalloc(b, &f.less_flat, SN);
  rc |= dalloc(b, &f.n_feat, (size_t)S * 4);
  rc |= dalloc(b, &f.feat_loff, (size_t)S * 2 * (H + 1));
  f.cap_sharp = b->cap_sharp; f.cap_less_sharp = b->cap_less_sharp; f.cap_flat = b->cap_flat;
  OdomArgs& o = b->oa;
  o.S = S; o.N = N; o.H = H;
  o.sharp = f.sharp; o.less_sharp = f.less_sharp; o.flat = f.flat; o.less_flat = f.less_flat;
  o.n_feat = f.n_feat;
  o.feat_loff = f.feat_loff;
  o.idx_ls.nchunk = (b->cap_less_sharp + kChunk - 1) / kChunk;
  o.idx_ls.nsuper = (o.idx_ls.nchunk + kChunk - 1) / kChunk;
  o.idx_lf.nchunk = (N + kChunk - 1) / kChunk;
  o.idx_lf.nsuper = (o.idx_lf.nchunk + kChunk - 1) / kChunk;
  o.idx_ls.cap = b->cap_less_sharp;
  o.idx_lf.cap = N;
  for (TargetIndex* ti : {&o.idx_ls, &o.idx_lf}) {
    rc |= dalloc(b, &ti->chunk, (size_t)S * ti->nchunk * 2);
    rc |= dalloc(b, &ti->super, (size_t)S * ti->nsuper * 2);
    rc |= dalloc(b, &ti->nn_chunk, (size_t)S * ti->nchunk * 2);
    rc |= dalloc(b, &ti->nn_super, (size_t)S * ti->nsuper * 2);
    rc |= dalloc(b, &ti->sorted, (size_t)S * ti->cap);
    rc |= dalloc(b, &ti->keys, (size_t)S * 2 * ti->cap);
  }
  rc |= dalloc(b, &o.qpts_sharp, (size_t)S * b->cap_sharp);
  rc |= dalloc(b, &o.qpts_flat, (size_t)S * b->cap_flat);
  rc |= dalloc(b, &o.state, (size_t)S * 16);
  o.cap_sharp = b->cap_sharp; o.cap_less_sharp = b->cap_less_sharp; o.cap_flat = b->cap_flat;
  o.max_iterations = c->cfg.max_iterations;
  rc |= dalloc(b, &o.blk, (size_t)S * (b->cap_sharp + b->cap_flat) * 9);
  rc |= dalloc(b, &o.blk_kind, (size_t)S * (b->cap_sharp + b->cap_flat));
  rc |= dalloc(b, &o.para, (size_t)S * 7);
  rc |= dalloc(b, &o.pose, (size_t)S * 7);
  rc |= dalloc(b, &o.stats, (size_t)S * 8);
  rc |= dalloc(b, &o.eng_ctl, (size_t)8 + 10 * (size_t)S);
  rc |= dalloc(b, &o.warm, (size_t)S * (b->cap_sharp + b->cap_flat) * 4);
  rc |= dalloc(b, &o.eng_part, (size_t)S * lislam::engine_part_rows(b->cap_sharp + b->cap_flat) * 32);  // [chains][rows][32]
  rc |= dalloc(b, &b->d_init, (size_t)S * 14);
  rc |= dalloc(b, &b->d_gate, (size_t)S);
  if (rc != LISLAM_OK) {
    lislam_batch_destroy(b);
    return LISLAM_ERR_DEVICE;
  }
  // the engine's control words (its sticky abort word is never cleared by a launch)
  if (hipMemset(o.eng_ctl, 0, sizeof(unsigned) * ((size_t)8 + 10 * (size_t)S)) != hipSuccess) {
    lislam_batch_destroy(b);
    return LISLAM_ERR_DEVICE;
  }
  *out = b;
  return LISLAM_OK;
}

int lislam_batch_destroy(lislam_batch* b) {
  if (!b) return LISLAM_OK;
  hipSetDevice(b->ctx->device);
  if (b->eng_pending) {  // the batch's last engine launch (its streams are the device's, shared)
    lislam::wait_engine_launched(&b->eng_req);
    hipEventSynchronize(b->eng_join_r);
    hipEventSynchronize(b->eng_join_i);
  }
  hipStreamSynchronize(b->ctx->stream);
  {
    auto& v = b->ctx->batches;
    for (size_t i = 0; i < v.size(); i++)
      if (v[i] == b) { v.erase(v.begin() + i); break; }
  }
  for (void* p : b->allocs) hipFree(p);
  for (auto& v : b->ext_ev) for (hipEvent_t e : v) hipEventDestroy(e);
  for (auto& v : b->odo_ev) for (auto& t : v) { hipEventDestroy(t.b); hipEventDestroy(t.e); }
  for (int g = 1; g < lislam_batch::kMaxGroups; g++) {
    // odo_stream[g]: the device's (lislam::round_stream), joined into the context stream synchronized above
    if (b->odo_join[g]) hipEventDestroy(b->odo_join[g]);
  }
  if (b->odo_fork) hipEventDestroy(b->odo_fork);
  for (hipEvent_t e : {b->eng_fork, b->eng_join_r, b->eng_join_i}) if (e) hipEventDestroy(e);
  for (hipEvent_t e : b->pool) hipEventDestroy(e);
  if (b->orb) lislam_free_orb(b->orb);
  if (b->ground) lislam_free_ground(b->ground);
  if (b->wire) hipFree(b->wire);
  if (b->ev_images) hipEventDestroy(b->ev_images);
  if (b->eng_ready) hipEventDestroy(b->eng_ready);
  if (b->eng_done) hipEventDestroy(b->eng_done);
  if (b->h_abort) hipHostFree(b->h_abort);
  if (b->stage_ev) hipEventDestroy(b->stage_ev);
  if (b->copy_stream) {
    hipStreamSynchronize(b->copy_stream);
    hipStreamDestroy(b->copy_stream);
  }
  for (hipEvent_t e : b->chunk_landed) hipEventDestroy(e);
  for (hipEvent_t e : b->chunk_parsed) hipEventDestroy(e);
  if (b->ring) hipFree(b->ring);
  if (b->h_stage) hipHostFree(b->h_stage);
  delete b;
  return LISLAM_OK;
}

// device staging buffer of at least `bytes` for PointCloud2 bytes
static int rc_wire(lislam_batch* b, size_t bytes) {
  if (b->wire_bytes >= bytes) return LISLAM_OK;
  if (b->wire) hipFree(b->wire);
  b->wire = nullptr;
  b->wire_bytes = 0;
  if (hipMalloc(&b->wire, bytes) != hipSuccess) return LISLAM_ERR_DEVICE;
  b->wire_bytes = bytes;
  return LISLAM_OK;
}

static int batch_output_source(lislam_batch* b, int what, int scan, const void** src, int* cnt);
static int output_source(lislam_batch* b, int what, int scan, const void** src_out, int* cnt_out, size_t* esz_out);

int lislam_batch_upload(lislam_batch* b, const void* points, int32_t n_scans, const lislam_point_layout* layout) {
  if (!b || !points || n_scans < 1 || n_scans > b->max_scans) return LISLAM_ERR_ARG;
  // no engine settle: the chain engine (and its per-round re-run) reads the features, never the
  // points, so the next batch's bytes move while the engine runs
  lislam_ctx* c = b->ctx;
  hipSetDevice(c->device);
  const size_t n = (size_t)n_scans * b->N;
  if (is_packed(layout)) {
    HIPCHK(c, hipMemcpyAsync((void*)b->fa.pts, points, n * 16, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
  } else {  // the message bytes go to the device scan by scan, the fields are parsed there
    if (layout->point_step < 4 || std::max({layout->off_x, layout->off_y, layout->off_z, layout->off_intensity}) + 4 > layout->point_step)
      return fail(c, LISLAM_ERR_ARG, "bad point layout");
    const size_t scan_bytes = (size_t)b->N * layout->point_step;
    if ((rc_wire(b, scan_bytes)) != LISLAM_OK) return fail(c, LISLAM_ERR_DEVICE, "staging allocation failed");
    const lislam::WireLayout L{layout->point_step, layout->off_x, layout->off_y, layout->off_z, layout->off_intensity};
    for (int s = 0; s < n_scans; s++) {
      HIPCHK(c, hipMemcpyAsync(b->wire, static_cast<const uint8_t*>(points) + s * scan_bytes, scan_bytes, hipMemcpyDefault,
                               c->stream));
      lislam::launch_unpack_layout(static_cast<const uint8_t*>(b->wire), b->N, L,
                                   const_cast<lislam::P4*>(b->fa.pts) + (size_t)s * b->N, c->stream);
    }
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipStreamSynchronize(c->stream));
  }
  return LISLAM_OK;
}

int lislam_batch_upload_async(lislam_batch* b, const void* points, int32_t n_scans, const lislam_point_layout* layout) {
  if (!b || !points || n_scans < 1 || n_scans > b->max_scans) return LISLAM_ERR_ARG;
  // no engine settle: the chain engine (and its per-round re-run) reads the features, never the
  // points, so the next batch's bytes move while the engine runs
  lislam_ctx* c = b->ctx;
  hipSetDevice(c->device);
  static const lislam_point_layout kPacked{16, 0, 4, 8, 12};
  const lislam_point_layout* lay = (!layout || is_packed(layout)) ? &kPacked : layout;
  if (lay->point_step < 4 || std::max({lay->off_x, lay->off_y, lay->off_z, lay->off_intensity}) + 4 > lay->point_step)
    return fail(c, LISLAM_ERR_ARG, "bad point layout");
  const size_t scan_bytes = (size_t)b->N * lay->point_step;
  const size_t need = (size_t)b->max_scans * scan_bytes;
  if (b->ring_bytes < need) {
    // a new staging area: everything queued on either stream may still use the old one
    if (b->copy_stream) HIPCHK(c, hipStreamSynchronize(b->copy_stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (b->ring) hipFree(b->ring);
    b->ring = nullptr;
    b->ring_bytes = 0;
    if (hipMalloc(&b->ring, need) != hipSuccess) return fail(c, LISLAM_ERR_DEVICE, "staging allocation failed");
    b->ring_bytes = need;
    std::fill(b->chunk_used.begin(), b->chunk_used.end(), 0);
  }
  if (!b->copy_stream) HIPCHK(c, hipStreamCreateWithFlags(&b->copy_stream, hipStreamNonBlocking));
  constexpr int kChunk = 16;
  const int nchunks = (n_scans + kChunk - 1) / kChunk;
  while ((int)b->chunk_landed.size() < nchunks) {
    hipEvent_t e1 = nullptr, e2 = nullptr;
    HIPCHK(c, hipEventCreateWithFlags(&e1, hipEventDisableTiming));
    HIPCHK(c, hipEventCreateWithFlags(&e2, hipEventDisableTiming));
    b->chunk_landed.push_back(e1);
    b->chunk_parsed.push_back(e2);
    b->chunk_used.push_back(0);
  }
  const lislam::WireLayout L{lay->point_step, lay->off_x, lay->off_y, lay->off_z, lay->off_intensity};
  for (int k = 0; k < nchunks; k++) {
    const int s0 = k * kChunk, ns = std::min(kChunk, n_scans - s0);
    uint8_t* dst = static_cast<uint8_t*>(b->ring) + (size_t)s0 * scan_bytes;
    // the chunk's staging bytes are free once the previous upload's parse of them has run
    if (b->chunk_used[k]) HIPCHK(c, hipStreamWaitEvent(b->copy_stream, b->chunk_parsed[k], 0));
    HIPCHK(c, hipMemcpyAsync(dst, static_cast<const uint8_t*>(points) + (size_t)s0 * scan_bytes, (size_t)ns * scan_bytes,
                             hipMemcpyHostToDevice, b->copy_stream));
    HIPCHK(c, hipEventRecord(b->chunk_landed[k], b->copy_stream));
    HIPCHK(c, hipStreamWaitEvent(c->stream, b->chunk_landed[k], 0));
    lislam::launch_unpack_layout(dst, ns * b->N, L, const_cast<lislam::P4*>(b->fa.pts) + (size_t)s0 * b->N, c->stream);
    HIPCHK(c, hipEventRecord(b->chunk_parsed[k], c->stream));
    b->chunk_used[k] = 1;
  }
  HIPCHK(c, hipGetLastError());
  return LISLAM_OK;
}

// mapOptimizationCallback's input assembly (mapOptimization.cpp:136-150): GroundPointOut of the
// scan (lislam_batch_ground) followed by its less-flat cloud (the plane cloud), concatenated on the
// device (the 4th field is not read by the ground-map stage), then lislam_mapopt_step.
int lislam_batch_mapopt(lislam_batch* b, lislam_map* m, int32_t scan, const double* odom, double* state,
                        double* out_pose, int32_t* summary) {
  return lislam_batch_mapopt_corner(b, m, nullptr, scan, odom, state, out_pose, summary);
}

// With the corner ikd-Tree: pc_corner is the scan's less-sharp cloud (/laser_cloud_less_sharp,
// mapOptimizationNode.cpp:63), staged behind the plane cloud in the same device buffer.
int lislam_batch_mapopt_corner(lislam_batch* b, lislam_map* m, lislam_map* cm, int32_t scan, const double* odom,
                               double* state, double* out_pose, int32_t* summary) {
  if (!b || !m || !odom || !state || scan < 0 || scan >= b->max_scans) return LISLAM_ERR_ARG;
  SETTLE(b);
  lislam_ctx* c = b->ctx;
  hipSetDevice(c->device);
  const void *g = nullptr, *lf = nullptr;
  int ng = 0, nlf = 0;
  size_t eg = 0, elf = 0;
  const void* ls = nullptr;
  int nls = 0;
  size_t els = 0;
  int rc = output_source(b, LISLAM_OUT_GROUND, scan, &g, &ng, &eg);
  if (rc) return rc;
  if ((rc = output_source(b, LISLAM_OUT_LESS_FLAT, scan, &lf, &nlf, &elf))) return rc;
  if (cm && (rc = output_source(b, LISLAM_OUT_LESS_SHARP, scan, &ls, &nls, &els))) return rc;
  const size_t bytes = (size_t)(ng + nlf + nls) * 16;
  if ((rc = rc_wire(b, std::max<size_t>(bytes, 16)))) return fail(c, rc, "lislam_batch_mapopt: staging allocation");
  uint8_t* dst = static_cast<uint8_t*>(b->wire);
  if (ng) HIPCHK(c, hipMemcpyAsync(dst, g, (size_t)ng * 16, hipMemcpyDeviceToDevice, c->stream));
  if (nlf) HIPCHK(c, hipMemcpyAsync(dst + (size_t)ng * 16, lf, (size_t)nlf * 16, hipMemcpyDeviceToDevice, c->stream));
  if (nls)
    HIPCHK(c, hipMemcpyAsync(dst + (size_t)(ng + nlf) * 16, ls, (size_t)nls * 16, hipMemcpyDeviceToDevice, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return lislam_mapopt_step_corner(m, cm, reinterpret_cast<const float*>(dst), ng + nlf,
                                   reinterpret_cast<const float*>(dst + (size_t)(ng + nlf) * 16), nls, odom, state,
                                   out_pose, summary);
}

int lislam_batch_download_cloud(lislam_batch* b, int32_t what, int32_t scan, void* dst, const lislam_point_layout* layout,
                                int32_t cap, int32_t* n) {
  if (!b || !dst || !layout || scan < 0 || scan >= b->max_scans) return LISLAM_ERR_ARG;
  SETTLE(b);
  lislam_ctx* c = b->ctx;
  if (layout->point_step < 4 || std::max({layout->off_x, layout->off_y, layout->off_z, layout->off_intensity}) + 4 > layout->point_step)
    return fail(c, LISLAM_ERR_ARG, "bad point layout");
  const bool cloud4 = what == LISLAM_OUT_LASER_CLOUD || what == LISLAM_OUT_SHARP || what == LISLAM_OUT_LESS_SHARP ||
                      what == LISLAM_OUT_FLAT || what == LISLAM_OUT_LESS_FLAT || what == LISLAM_OUT_CLOUD_TRACK ||
                      what == LISLAM_OUT_GROUND || what == LISLAM_OUT_ORB_POINTS;
  if (!cloud4) return fail(c, LISLAM_ERR_ARG, "output %d is not a point cloud", what);
  hipSetDevice(c->device);
  // the device source of the cloud: lislam_batch_download with a null copy (cap 0) gives the count
  int cnt = 0;
  const void* src = nullptr;
  int rc = batch_output_source(b, what, scan, &src, &cnt);
  if (rc) return rc;
  if (n) *n = cnt;
  if (cnt > cap) return fail(c, LISLAM_ERR_CAPACITY, "cloud %d needs %d points, cap %d", what, cnt, cap);
  if (cnt == 0) return LISLAM_OK;
  const size_t bytes = (size_t)cnt * layout->point_step;
  if (rc_wire(b, bytes) != LISLAM_OK) return fail(c, LISLAM_ERR_DEVICE, "staging allocation failed");
  const lislam::WireLayout L{layout->point_step, layout->off_x, layout->off_y, layout->off_z, layout->off_intensity};
  lislam::launch_pack_layout(static_cast<const lislam::P4*>(src), cnt, L, static_cast<uint8_t*>(b->wire), c->stream);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipMemcpyAsync(dst, b->wire, bytes, hipMemcpyDefault, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return LISLAM_OK;
}

int lislam_batch_input_device_ptr(lislam_batch* b, void** dptr) {
  if (!b || !dptr) return LISLAM_ERR_ARG;
  // no engine settle: the chain engine (and its per-round re-run) reads the features, never the
  // points, so the next batch's bytes move while the engine runs
  *dptr = (void*)b->fa.pts;
  return LISLAM_OK;
}

int lislam_batch_set_timing(lislam_batch* b, int32_t enable) {
  if (!b) return LISLAM_ERR_ARG;
  b->timing = enable != 0;
  return LISLAM_OK;
}

int lislam_batch_extract(lislam_batch* b, int32_t n_scans) {
  if (!b || n_scans < 1 || n_scans > b->max_scans) return LISLAM_ERR_ARG;
  SETTLE(b);
  lislam_ctx* c = b->ctx;
  hipSetDevice(c->device);
  // a pending ORB cascade may still need the current images (its host-round redo): settle it
  // before they are overwritten
  if (b->orb) {
    const int rc = orb_settle(b);
    if (rc != LISLAM_OK) return rc;
  }
  FeatureArgs f = b->fa;
  f.S = n_scans;
  f.ties = c->ties;
  hipEvent_t* ev = nullptr;
  if (b->timing) {
    b->ext_ev.emplace_back();
    for (int i = 0; i < 5; i++) b->ext_ev.back().push_back(b->get_event());
    ev = b->ext_ev.back().data();
  }
  launch_features(f, c->stream, ev, b->ev_images);
  launch_target_index(b->oa, n_scans, c->stream);  // spatial index of the clouds odometry searches
  if (ev) HIPCHK(c, hipEventRecord(ev[4], c->stream));
  HIPCHK(c, hipEventRecord(b->eng_ready, c->stream));  // the chain engine's inputs
  HIPCHK(c, hipGetLastError());
  b->extracted = n_scans;
  return LISLAM_OK;
}

static int run_odometry(lislam_batch* b, int n_scans, int chain_len, const double* init_host,
                        const int32_t* use_aloam = nullptr) {
  SETTLE(b);
  lislam_ctx* c = b->ctx;
  OdomArgs o = b->oa;
  o.gate = nullptr;
  o.S = n_scans;
  o.chain_len = chain_len;
  o.n_chains = n_scans > 1 ? (n_scans - 1 + chain_len - 1) / chain_len : 0;
  o.init_state = nullptr;
  if (use_aloam || init_host) {
    // the caller's arrays -> pinned staging -> device, so they may be freed on return
    const size_t init_bytes = sizeof(double) * 14 * (size_t)b->max_scans;
    if (!b->h_stage) {
      HIPCHK(c, hipHostMalloc(&b->h_stage, init_bytes + sizeof(int) * (size_t)b->max_scans, hipHostMallocDefault));
      HIPCHK(c, hipEventCreateWithFlags(&b->stage_ev, hipEventDisableTiming));
    }
    if (b->stage_busy) HIPCHK(c, hipEventSynchronize(b->stage_ev));  // the previous upload has been read
    double* hi = static_cast<double*>(b->h_stage);
    int* hg = reinterpret_cast<int*>(static_cast<char*>(b->h_stage) + init_bytes);
    if (use_aloam) {
      hipPointerAttribute_t attr{};
      const bool on_device = hipPointerGetAttributes(&attr, use_aloam) == hipSuccess && attr.type == hipMemoryTypeDevice;
      (void)hipGetLastError();  // an unregistered host pointer reports an error here
      if (on_device) {
        HIPCHK(c, hipMemcpyAsync(b->d_gate, use_aloam, sizeof(int) * n_scans, hipMemcpyDeviceToDevice, c->stream));
      } else {
        std::memcpy(hg, use_aloam, sizeof(int) * n_scans);
        HIPCHK(c, hipMemcpyAsync(b->d_gate, hg, sizeof(int) * n_scans, hipMemcpyHostToDevice, c->stream));
      }
      o.gate = b->d_gate;
    }
    if (init_host) {
      std::memcpy(hi, init_host, sizeof(double) * 14 * o.n_chains);
      HIPCHK(c, hipMemcpyAsync(b->d_init, hi, sizeof(double) * 14 * o.n_chains, hipMemcpyHostToDevice, c->stream));
      o.init_state = b->d_init;
    }
    HIPCHK(c, hipEventRecord(b->stage_ev, c->stream));
    b->stage_busy = true;
  }
  const int G = lislam_batch::kGroups;
  std::vector<lislam::OdoTimed>* ev = nullptr;
  if (b->timing) {
    b->odo_ev.emplace_back();
    ev = &b->odo_ev.back();
  }
  o.c0 = 0;
  o.cn = o.n_chains;
  o.eng_qpw = c->eng_qpw;
  o.eng_depth = c->eng_depth;
  if (lislam::use_chain_engine(o, c->odom_engine)) {
    // few long chains: one persistent launch sequences every round on the device
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (b->eng_split < 0) {  // the engine's streams, once per batch
      // LISLAM_ENGINE_SINGLE=1: the single-launch engine (k_odom_chain) even where CU masks exist
      // (read once per batch: the tests run both engines in one process)
      const bool single = getenv("LISLAM_ENGINE_SINGLE") && atoi(getenv("LISLAM_ENGINE_SINGLE")) == 1;
      b->eng_split = !single && lislam::engine_streams_available(c->device) ? 1 : 0;
      if (b->eng_split) {
        HIPCHK(c, hipEventCreateWithFlags(&b->eng_fork, hipEventDisableTiming));
        HIPCHK(c, hipEventCreateWithFlags(&b->eng_join_r, hipEventDisableTiming));
        HIPCHK(c, hipEventCreateWithFlags(&b->eng_join_i, hipEventDisableTiming));
      }
      HIPCHK(c, hipEventCreateWithFlags(&b->eng_done, hipEventDisableTiming));
      HIPCHK(c, hipHostMalloc((void**)&b->h_abort, 2 * sizeof(unsigned), hipHostMallocDefault));
      b->h_abort[0] = b->h_abort[1] = 0;
    }
    if (ev) { e0 = b->get_event(); e1 = b->get_event(); }
    bool queued = false;
    if (b->eng_split) {
      // the inputs: everything queued on the context stream so far (the last extract, any per-round
      // odometry queued after it, the staging copies just queued); the launch copies its abort words
      // to h_abort and records eng_done on its own stream
      HIPCHK(c, hipEventRecord(b->eng_ready, c->stream));
      if (o.eng_depth > 1 && lislam::engine_dispatch_enabled()) {
        // to the device's dispatcher: launched on the first free engine slot once the inputs exist.
        // Depth 1 keeps the direct gate: one engine at a time has no slot to choose, and the host
        // hop costs a single sequence ~2% (profiles/r06q_dispatch_ab.txt)
        lislam::EngineRequest& r = b->eng_req;
        r.a = o;
        r.ready = b->eng_ready; r.fork = b->eng_fork; r.join_r = b->eng_join_r; r.join_i = b->eng_join_i;
        r.t0 = e0; r.t1 = e1; r.h_abort = b->h_abort; r.done = b->eng_done;
        queued = lislam::submit_odometry_chain_split(&r) > 0;
      } else {
        queued = lislam::launch_odometry_chain_split(o, b->eng_ready, b->eng_fork, b->eng_join_r, b->eng_join_i, e0, e1,
                                                     b->h_abort, b->eng_done) > 0;
      }
      if (queued) b->eng_pending = true;
      else b->eng_split = 0;  // no engine streams on this device after all: the single launch below
    }
    if (!queued) {
      if (ev) HIPCHK(c, hipEventRecord(e0, c->stream));
      lislam::launch_odometry_chain(o, c->stream);
      if (ev) HIPCHK(c, hipEventRecord(e1, c->stream));
      HIPCHK(c, hipMemcpyAsync(b->h_abort, b->oa.eng_ctl + 2, 2 * sizeof(unsigned), hipMemcpyDeviceToHost, c->stream));
      HIPCHK(c, hipEventRecord(b->eng_done, c->stream));
    }
    b->eng_args = o;
    b->eng_check = true;
    b->engine_ran = true;
    if (ev) ev->push_back({6, e0, e1});
    HIPCHK(c, hipGetLastError());
    return LISLAM_OK;
  }
  b->engine_ran = false;
  if (round_streams(b) != LISLAM_OK) return LISLAM_ERR_DEVICE;
  launch_odometry(o, b->odo_stream, G, b->odo_fork, b->odo_join, ev, &lislam_batch::event_cb, b);
  HIPCHK(c, hipGetLastError());
  return LISLAM_OK;
}

int lislam_batch_odometry(lislam_batch* b, int32_t n_scans, int32_t chain_len) {
  if (!b || n_scans < 1 || n_scans > b->max_scans || chain_len < 1) return LISLAM_ERR_ARG;
  if (b->extracted < n_scans) return fail(b->ctx, LISLAM_ERR_STATE, "extract %d scans before odometry", n_scans);
  hipSetDevice(b->ctx->device);
  return run_odometry(b, n_scans, chain_len, nullptr);
}

int lislam_batch_odometry_gated(lislam_batch* b, int32_t n_scans, int32_t chain_len, const int32_t* use_aloam) {
  if (!b || n_scans < 1 || n_scans > b->max_scans || chain_len < 1 || !use_aloam) return LISLAM_ERR_ARG;
  if (b->extracted < n_scans) return fail(b->ctx, LISLAM_ERR_STATE, "extract %d scans before odometry", n_scans);
  hipSetDevice(b->ctx->device);
  return run_odometry(b, n_scans, chain_len, nullptr, use_aloam);
}

int lislam_batch_odometry_status(lislam_batch* b, int32_t* status) {
  if (!b || !status) return LISLAM_ERR_ARG;
  // engine launches that gave up (a bounded device wait expired) since the last status call or the
  // batch's creation; each was re-run on the per-round schedule when it settled, so the outputs are
  // valid.  Reading the count clears it.
  SETTLE(b);
  *status = b->eng_fallbacks;
  b->eng_fallbacks = 0;
  return LISLAM_OK;
}

int lislam_batch_odometry_abort_code(lislam_batch* b, int32_t* code) {
  if (!b || !code) return LISLAM_ERR_ARG;
  SETTLE(b);
  *code = (int32_t)b->eng_abort_code;
  return LISLAM_OK;
}

int lislam_device_queue_count(int32_t device, int32_t* masked_queues) {
  if (!masked_queues || device < 0) return LISLAM_ERR_ARG;
  *masked_queues = lislam::masked_queue_count(device);
  return LISLAM_OK;
}

int lislam_batch_odometry_engine(lislam_batch* b, int32_t* kind) {
  if (!b || !kind) return LISLAM_ERR_ARG;
  *kind = !b->engine_ran ? 0 : b->eng_split == 1 ? 2 : 1;
  return LISLAM_OK;
}

int lislam_batch_kernel_times(lislam_batch* b, float* ms_per_call, int32_t* launches_per_call, int32_t* calls) {
  if (!b || !ms_per_call) return LISLAM_ERR_ARG;
  SETTLE(b);
  lislam_ctx* c = b->ctx;
  hipSetDevice(c->device);
  HIPCHK(c, hipStreamSynchronize(c->stream));
  double acc[LISLAM_NUM_KERNELS] = {0};
  int launches[LISLAM_NUM_KERNELS] = {0};
  auto el = [&](hipEvent_t a0, hipEvent_t a1) -> double {
    float ms = 0;
    if (hipEventElapsedTime(&ms, a0, a1) != hipSuccess) return 0.0;
    return ms;
  };
  for (auto& v : b->ext_ev) {
    timeline_print(c->device, "extract", b, 0, v[0], v[4]);
    for (int i = 0; i < 4; i++) { acc[i] += el(v[i], v[i + 1]); launches[i] += i == 3 ? 2 : i == 0 ? 3 : 1; }  // front: 3 launches, k_target_index: 2
    for (hipEvent_t e : v) b->pool.push_back(e);
  }
  for (auto& v : b->odo_ev) {
    for (auto& t : v) {  // every launch bracketed on its own stream
      timeline_print(c->device, "odometry", b, t.kernel, t.b, t.e);
      acc[t.kernel] += el(t.b, t.e);
      launches[t.kernel] += 1;
      b->pool.push_back(t.b);
      b->pool.push_back(t.e);
    }
  }
  const int ne = (int)b->ext_ev.size(), no = (int)b->odo_ev.size();
  for (int k = 0; k < LISLAM_NUM_KERNELS; k++) {
    const int ncall = k < 4 ? ne : no;
    ms_per_call[k] = ncall ? (float)(acc[k] / ncall) : 0.f;
    if (launches_per_call) launches_per_call[k] = ncall ? launches[k] / ncall : 0;
  }
  if (calls) { calls[0] = ne; calls[1] = no; }
  b->ext_ev.clear();
  b->odo_ev.clear();
  return LISLAM_OK;
}

}  // extern "C"

// Device source, element count and element size of one output of one scan (synchronizes).
static int output_source(lislam_batch* b, int what, int scan, const void** src_out, int* cnt_out, size_t* esz_out) {
  lislam_ctx* c = b->ctx;
  hipSetDevice(c->device);
  HIPCHK(c, hipStreamSynchronize(c->stream));
  const size_t N = b->N;
  const FeatureArgs& f = b->fa;
  const OdomArgs& o = b->oa;
  int cnt = 0;
  const void* src = nullptr;
  size_t esz = 0;
  auto devint = [&](const int* p, int* v) -> int {
    HIPCHK(c, hipMemcpy(v, p, sizeof(int), hipMemcpyDeviceToHost));
    return LISLAM_OK;
  };
  int ncloud = 0;
  switch (what) {
    case LISLAM_OUT_IMAGE_RANGE: src = f.img_range ? f.img_range + scan * N : nullptr; cnt = (int)N; esz = 1; break;
    case LISLAM_OUT_IMAGE_INTENSITY: src = f.img_int ? f.img_int + scan * N : nullptr; cnt = (int)N; esz = 1; break;
    case LISLAM_OUT_CLOUD_TRACK: src = f.track ? f.track + scan * N : nullptr; cnt = (int)N; esz = 16; break;
    case LISLAM_OUT_LASER_CLOUD:
    case LISLAM_OUT_CURVATURE:
    case LISLAM_OUT_LABEL:
      if (devint(f.n_cloud + scan, &ncloud) != LISLAM_OK) return LISLAM_ERR_DEVICE;
      cnt = ncloud;
      if (what == LISLAM_OUT_LASER_CLOUD) { src = f.cloud + scan * N; esz = 16; }
      else if (what == LISLAM_OUT_CURVATURE) { src = f.curv + scan * N; esz = 4; }
      else { src = f.label + scan * N; esz = 1; }
      break;
    case LISLAM_OUT_LINE_OFFSETS: src = f.line_off + (size_t)scan * (b->H + 1); cnt = b->H + 1; esz = 4; break;
    case LISLAM_OUT_SHARP:
    case LISLAM_OUT_LESS_SHARP:
    case LISLAM_OUT_FLAT:
    case LISLAM_OUT_LESS_FLAT: {
      const int k = what - LISLAM_OUT_SHARP;
      if (devint(f.n_feat + scan * 4 + k, &cnt) != LISLAM_OK) return LISLAM_ERR_DEVICE;
      esz = 16;
      src = k == 0 ? (const void*)(f.sharp + (size_t)scan * b->cap_sharp)
          : k == 1 ? (const void*)(f.less_sharp + (size_t)scan * b->cap_less_sharp)
          : k == 2 ? (const void*)(f.flat + (size_t)scan * b->cap_flat)
                   : (const void*)(f.less_flat + scan * N);
      break;
    }
    case LISLAM_OUT_PARA:
    case LISLAM_OUT_POSE:
    case LISLAM_OUT_STATS: {
      // (an aborted engine launch has been re-run by the caller's SETTLE before this point)
      if (what == LISLAM_OUT_PARA) { src = o.para + (size_t)scan * 7; cnt = 7; esz = 8; }
      else if (what == LISLAM_OUT_POSE) { src = o.pose + (size_t)scan * 7; cnt = 7; esz = 8; }
      else { src = o.stats + (size_t)scan * 8; cnt = 8; esz = 4; }
      break;
    }
    case LISLAM_OUT_ORB_T:
    case LISLAM_OUT_ORB_STATS:
    case LISLAM_OUT_ORB_KEYPOINTS:
    case LISLAM_OUT_ORB_POINTS:
    case LISLAM_OUT_ORB_DESCRIPTORS: {
      const int rc = lislam_orb_batch_output(b, what, scan, &src, &cnt, &esz);
      if (rc) return fail(c, rc, "ORB output %d unavailable (run lislam_batch_intensity_odometry first)", what);
      break;
    }
    case LISLAM_OUT_GROUND:
    case LISLAM_OUT_GROUND_PLANE:
    case LISLAM_OUT_GROUND_INFO: {
      const int rc = lislam_ground_batch_output(b, what, scan, &src, &cnt, &esz);
      if (rc) return fail(c, rc, "ground output %d unavailable (run lislam_batch_ground first)", what);
      break;
    }
    default: return fail(c, LISLAM_ERR_ARG, "unknown output %d", what);
  }
  if (!src) return fail(c, LISLAM_ERR_STATE, "output %d not materialized (want_images=0?)", what);
  *src_out = src;
  *cnt_out = cnt;
  *esz_out = esz;
  return LISLAM_OK;
}

static int batch_output_source(lislam_batch* b, int what, int scan, const void** src, int* cnt) {
  size_t esz = 0;
  return output_source(b, what, scan, src, cnt, &esz);
}

extern "C" {

int lislam_batch_download(lislam_batch* b, int32_t what, int32_t scan, void* dst, int32_t cap, int32_t* n) {
  if (!b || (!dst && !n) || scan < 0 || scan >= b->max_scans) return LISLAM_ERR_ARG;
  SETTLE(b);
  lislam_ctx* c = b->ctx;
  int cnt = 0;
  const void* src = nullptr;
  size_t esz = 0;
  const int rc = output_source(b, what, scan, &src, &cnt, &esz);
  if (rc) return rc;
  if (n) *n = cnt;
  if (!dst) return LISLAM_OK;  // count only
  if (cnt > cap) return fail(c, LISLAM_ERR_CAPACITY, "output %d needs %d elements, cap %d", what, cnt, cap);
  if (cnt > 0) HIPCHK(c, hipMemcpy(dst, src, (size_t)cnt * esz, hipMemcpyDeviceToHost));
  return LISLAM_OK;
}

// ------------------------------------------------------------------------------ single scan
static int ensure_single(lislam_ctx* c) {
  if (c->single) return LISLAM_OK;
  return lislam_batch_create(c, 2, &c->single);
}

int lislam_scan_registration(lislam_ctx* c, const void* points, const lislam_point_layout* layout, lislam_scan_out* out) {
  if (!c || !points || !out) return LISLAM_ERR_ARG;
  hipSetDevice(c->device);
  int rc = ensure_single(c);
  if (rc) return rc;
  lislam_batch* b = c->single;
  if ((rc = lislam_batch_upload(b, points, 1, layout))) return rc;
  if ((rc = lislam_batch_extract(b, 1))) return rc;
  // every output of the scan in one pass: the counts once, then the copies, one wait at the end
  const FeatureArgs& f = b->fa;
  const int N = b->N;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  int ncloud = 0, nfeat[4] = {0, 0, 0, 0};
  HIPCHK(c, hipMemcpy(&ncloud, f.n_cloud, sizeof(int), hipMemcpyDeviceToHost));
  HIPCHK(c, hipMemcpy(nfeat, f.n_feat, sizeof(nfeat), hipMemcpyDeviceToHost));
  struct Item { const void* src; int cnt; size_t esz; void* dst; int cap; int* n; const char* name; };
  const Item items[] = {
      {f.cloud, ncloud, 16, out->laser_cloud, out->cap_laser_cloud, &out->n_laser_cloud, "laser_cloud"},
      {f.sharp, nfeat[0], 16, out->sharp, out->cap_sharp, &out->n_sharp, "sharp"},
      {f.less_sharp, nfeat[1], 16, out->less_sharp, out->cap_less_sharp, &out->n_less_sharp, "less_sharp"},
      {f.flat, nfeat[2], 16, out->flat, out->cap_flat, &out->n_flat, "flat"},
      {f.less_flat, nfeat[3], 16, out->less_flat, out->cap_less_flat, &out->n_less_flat, "less_flat"},
      {f.img_range, N, 1, out->image_range, N, nullptr, "image_range"},
      {f.img_int, N, 1, out->image_intensity, N, nullptr, "image_intensity"},
      {f.track, N, 16, out->cloud_track, N, nullptr, "cloud_track"}};
  for (const Item& it : items) {
    if (!it.dst) continue;
    if (!it.src) return fail(c, LISLAM_ERR_STATE, "%s unavailable (context created without images)", it.name);
    if (it.cnt > it.cap) return fail(c, LISLAM_ERR_CAPACITY, "%s needs %d elements, cap %d", it.name, it.cnt, it.cap);
    if (it.n) *it.n = it.cnt;
    if (it.cnt > 0) HIPCHK(c, hipMemcpyAsync(it.dst, it.src, (size_t)it.cnt * it.esz, hipMemcpyDeviceToHost, c->stream));
  }
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return LISLAM_OK;
}

int lislam_ground_extract(lislam_ctx* c, const void* points, const lislam_point_layout* layout, float* out,
                          int32_t cap, int32_t* n_out, float* plane, int32_t* info) {
  if (!c || !points) return LISLAM_ERR_ARG;
  hipSetDevice(c->device);
  int rc = ensure_single(c);
  if (rc) return rc;
  lislam_batch* b = c->single;
  if ((rc = lislam_batch_upload(b, points, 1, layout))) return rc;
  if ((rc = lislam_batch_ground(b, 1))) return rc;
  int n = 0;
  if (plane && (rc = lislam_batch_download(b, LISLAM_OUT_GROUND_PLANE, 0, plane, 4, &n))) return rc;
  if (info && (rc = lislam_batch_download(b, LISLAM_OUT_GROUND_INFO, 0, info, 4, &n))) return rc;
  if (out) {
    if ((rc = lislam_batch_download(b, LISLAM_OUT_GROUND, 0, out, cap, &n))) return rc;
    if (n_out) *n_out = n;
  }
  return LISLAM_OK;
}

// ------------------------------------------------------------------------------ odometry node
int lislam_odom_create(lislam_ctx* c, lislam_odom** out) {
  if (!c || !out) return LISLAM_ERR_ARG;
  hipSetDevice(c->device);
  int rc = ensure_single(c);
  if (rc) return rc;
  *out = new lislam_odom();
  (*out)->ctx = c;
  return LISLAM_OK;
}

int lislam_odom_destroy(lislam_odom* od) {
  delete od;
  return LISLAM_OK;
}

static int put_frame(lislam_batch* b, int slot, const lislam_frame* fr) {
  lislam_ctx* c = b->ctx;
  if (fr->n_sharp > b->cap_sharp || fr->n_less_sharp > b->cap_less_sharp || fr->n_flat > b->cap_flat ||
      fr->n_less_flat > b->N || fr->n_sharp < 0 || fr->n_less_sharp < 0 || fr->n_flat < 0 || fr->n_less_flat < 0)
    return fail(c, LISLAM_ERR_CAPACITY, "frame exceeds feature capacities");
  const FeatureArgs& f = b->fa;
  auto cp = [&](P4* dst, const float* src, int n) -> int {
    if (n > 0) HIPCHK(c, hipMemcpyAsync(dst, src, (size_t)n * 16, hipMemcpyHostToDevice, c->stream));
    return LISLAM_OK;
  };
  int rc = 0;
  rc |= cp(f.sharp + (size_t)slot * b->cap_sharp, fr->sharp, fr->n_sharp);
  rc |= cp(f.less_sharp + (size_t)slot * b->cap_less_sharp, fr->less_sharp, fr->n_less_sharp);
  rc |= cp(f.flat + (size_t)slot * b->cap_flat, fr->flat, fr->n_flat);
  rc |= cp(f.less_flat + (size_t)slot * b->N, fr->less_flat, fr->n_less_flat);
  const int cnt[4] = {fr->n_sharp, fr->n_less_sharp, fr->n_flat, fr->n_less_flat};
  HIPCHK(c, hipMemcpyAsync(f.n_feat + slot * 4, cnt, sizeof(cnt), hipMemcpyHostToDevice, c->stream));
  // per-line offsets of less_sharp / less_flat (first index whose int(intensity) >= line); they
  // only seed the 1-NN bound, so any non-decreasing array within [0, n] keeps results exact
  const int H = b->H;
  std::vector<int> loff(2 * (H + 1));
  const float* src[2] = {fr->less_sharp, fr->less_flat};
  const int nsrc[2] = {fr->n_less_sharp, fr->n_less_flat};
  for (int w = 0; w < 2; w++) {
    int j = 0;
    for (int l = 0; l <= H; l++) {
      while (j < nsrc[w] && (l == H || (int)src[w][4 * j + 3] < l)) j++;
      loff[w * (H + 1) + l] = j;
    }
  }
  HIPCHK(c, hipMemcpyAsync(f.feat_loff + (size_t)slot * 2 * (H + 1), loff.data(), loff.size() * sizeof(int),
                           hipMemcpyHostToDevice, c->stream));
  OdomArgs o = b->oa;
  o.less_sharp = f.less_sharp + (size_t)slot * b->cap_less_sharp;
  o.less_flat = f.less_flat + (size_t)slot * b->N;
  o.sharp = f.sharp + (size_t)slot * b->cap_sharp;
  o.flat = f.flat + (size_t)slot * b->cap_flat;
  o.qpts_sharp += (size_t)slot * b->cap_sharp;
  o.qpts_flat += (size_t)slot * b->cap_flat;
  o.n_feat = f.n_feat + slot * 4;
  for (TargetIndex* ti : {&o.idx_ls, &o.idx_lf}) {
    ti->chunk += (size_t)slot * ti->nchunk * 2;
    ti->super += (size_t)slot * ti->nsuper * 2;
    ti->nn_chunk += (size_t)slot * ti->nchunk * 2;
    ti->nn_super += (size_t)slot * ti->nsuper * 2;
    ti->sorted += (size_t)slot * ti->cap;
    ti->keys += (size_t)slot * 2 * ti->cap;
  }
  launch_target_index(o, 1, c->stream);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return rc ? LISLAM_ERR_DEVICE : LISLAM_OK;
}

// Slot `from` of the node batch becomes slot `to` on the device (the frame's clouds, counts, line
// offsets and its target index): the current frame turns into the last frame without a second
// upload and index build.
static int copy_slot(lislam_batch* b, int from, int to) {
  lislam_ctx* c = b->ctx;
  const hipStream_t st = c->stream;
  auto cp = [&](const void* base, size_t per_slot) -> int {
    const char* p = static_cast<const char*>(base);
    HIPCHK(c, hipMemcpyAsync(const_cast<char*>(p) + (size_t)to * per_slot, p + (size_t)from * per_slot, per_slot,
                             hipMemcpyDeviceToDevice, st));
    return LISLAM_OK;
  };
  const FeatureArgs& f = b->fa;
  const OdomArgs& o = b->oa;
  int rc = 0;
  rc |= cp(f.sharp, (size_t)b->cap_sharp * 16);
  rc |= cp(f.less_sharp, (size_t)b->cap_less_sharp * 16);
  rc |= cp(f.flat, (size_t)b->cap_flat * 16);
  rc |= cp(f.less_flat, (size_t)b->N * 16);
  rc |= cp(f.n_feat, 4 * sizeof(int));
  rc |= cp(f.feat_loff, (size_t)2 * (b->H + 1) * sizeof(int));
  for (const TargetIndex* ti : {&o.idx_ls, &o.idx_lf}) {
    rc |= cp(ti->chunk, (size_t)ti->nchunk * 2 * 16);
    rc |= cp(ti->super, (size_t)ti->nsuper * 2 * 16);
    rc |= cp(ti->nn_chunk, (size_t)ti->nchunk * 2 * 16);
    rc |= cp(ti->nn_super, (size_t)ti->nsuper * 2 * 16);
    rc |= cp(ti->sorted, (size_t)ti->cap * 16);
  }
  return rc ? LISLAM_ERR_DEVICE : LISLAM_OK;
}

static int odom_step(lislam_odom* od, const lislam_frame* fr, int use_aloam, double* para_out, double* pose_out,
                     int32_t* stats_out) {
  if (!od || !fr) return LISLAM_ERR_ARG;
  lislam_ctx* c = od->ctx;
  hipSetDevice(c->device);
  lislam_batch* b = c->single;
  int rc;
  int32_t st[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (!od->have_last) {  // first frame: initialization only (laserOdometry.cpp:382-389)
    if ((rc = put_frame(b, 0, fr))) return rc;
    od->have_last = true;
  } else {
    if ((rc = put_frame(b, 1, fr))) return rc;
    b->extracted = 2;
    od->gate[1] = use_aloam != 0;
    if ((rc = run_odometry(b, 2, 1, od->state, use_aloam < 0 ? nullptr : od->gate))) return rc;
    // para, pose and stats of the pair: three copies on the context stream, one wait
    SETTLE(b);
    const struct { int what; void* dst; int cap; } outs[3] = {
        {LISLAM_OUT_PARA, od->state, 7}, {LISLAM_OUT_POSE, od->state + 7, 7}, {LISLAM_OUT_STATS, st, 8}};
    for (const auto& o : outs) {
      const void* src = nullptr;
      int cnt = 0;
      size_t esz = 0;
      if ((rc = output_source(b, o.what, 1, &src, &cnt, &esz))) return rc;
      if (cnt > o.cap) return fail(c, LISLAM_ERR_CAPACITY, "output %d needs %d elements", o.what, cnt);
      if (cnt > 0) HIPCHK(c, hipMemcpyAsync(o.dst, src, (size_t)cnt * esz, hipMemcpyDeviceToHost, c->stream));
    }
    HIPCHK(c, hipStreamSynchronize(c->stream));
    // the current frame becomes the last frame (laserOdometry.cpp:793-808), on the device
    if ((rc = copy_slot(b, 1, 0))) return rc;
  }
  od->frames++;
  if (para_out) std::memcpy(para_out, od->state, 7 * sizeof(double));
  if (pose_out) std::memcpy(pose_out, od->state + 7, 7 * sizeof(double));
  if (stats_out) std::memcpy(stats_out, st, sizeof(st));
  return LISLAM_OK;
}

int lislam_odom_step(lislam_odom* od, const lislam_frame* fr, double* para_out, double* pose_out, int32_t* stats_out) {
  return odom_step(od, fr, -1, para_out, pose_out, stats_out);
}

int lislam_odom_step_gated(lislam_odom* od, const lislam_frame* fr, int32_t use_aloam, double* para_out,
                           double* pose_out, int32_t* stats_out) {
  return odom_step(od, fr, use_aloam ? 1 : 0, para_out, pose_out, stats_out);
}

// ------------------------------------------------------------------------------ functors
// The context's factor scratch, at least `bytes` (caller holds c->factor_mu).
static int factor_scratch(lislam_ctx* c, size_t bytes, uint8_t** out) {
  if (c->factor_bytes < bytes) {
    if (c->factor_buf) {
      (void)hipStreamSynchronize(c->stream);
      (void)hipFree(c->factor_buf);
      c->factor_buf = nullptr;
      c->factor_bytes = 0;
    }
    const size_t want = std::max(bytes, (size_t)1 << 20);
    if (hipMalloc(&c->factor_buf, want) != hipSuccess) return fail(c, LISLAM_ERR_DEVICE, "factor scratch allocation failed");
    c->factor_bytes = want;
  }
  *out = static_cast<uint8_t*>(c->factor_buf);
  return LISLAM_OK;
}

int lislam_eval_factors(lislam_ctx* c, int32_t n, const int32_t* kind, const double* pts, const double* q,
                        const double* t, double* residuals, double* jac) {
  if (!c || n < 0 || (n > 0 && (!kind || !pts)) || !q || !t) return LISLAM_ERR_ARG;
  if (n == 0) return LISLAM_OK;
  hipSetDevice(c->device);
  std::lock_guard<std::mutex> lock(c->factor_mu);
  // [x 7][pts n*12][res n*3][jac n*18] doubles, then kinds
  const size_t nd = 7 + (size_t)n * (12 + 3 + 18);
  uint8_t* base = nullptr;
  int rc = factor_scratch(c, nd * 8 + (size_t)n * 4, &base);
  if (rc) return rc;
  double* dx = reinterpret_cast<double*>(base);
  double* dp = dx + 7;
  double* dr = dp + (size_t)n * 12;
  double* dj = dr + (size_t)n * 3;
  int* dk = reinterpret_cast<int*>(dj + (size_t)n * 18);
  const double x[7] = {q[0], q[1], q[2], q[3], t[0], t[1], t[2]};
  hipError_t e = hipMemcpyAsync(dk, kind, n * sizeof(int), hipMemcpyDefault, c->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(dp, pts, (size_t)n * 12 * sizeof(double), hipMemcpyDefault, c->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(dx, x, sizeof(x), hipMemcpyHostToDevice, c->stream);
  if (e == hipSuccess) {
    FactorArgs a{n, dk, dp, dx, dr, dj};
    launch_factors(a, c->stream);
    e = hipGetLastError();
  }
  if (e == hipSuccess && residuals) e = hipMemcpyAsync(residuals, dr, (size_t)n * 3 * sizeof(double), hipMemcpyDefault, c->stream);
  if (e == hipSuccess && jac) e = hipMemcpyAsync(jac, dj, (size_t)n * 18 * sizeof(double), hipMemcpyDefault, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  if (e != hipSuccess) return fail(c, LISLAM_ERR_DEVICE, "lislam_eval_factors: %s", hipGetErrorString(e));
  return LISLAM_OK;
}

int lislam_set_odometry_schedule(lislam_ctx* c, int32_t mode) {
  if (!c || mode < LISLAM_ENGINE_OFF || mode > LISLAM_ENGINE_ON) return LISLAM_ERR_ARG;
  c->odom_engine = mode;
  return LISLAM_OK;
}

int lislam_set_engine_shape(lislam_ctx* c, int32_t queries_per_wave, int32_t depth) {
  if (!c || queries_per_wave < 0 || queries_per_wave > 4 || depth < 0 || depth > lislam::kMaxEngineDepth)
    return LISLAM_ERR_ARG;
  if (queries_per_wave) c->eng_qpw = queries_per_wave;
  if (depth) c->eng_depth = depth;
  return LISLAM_OK;
}

int lislam_set_tie_order(lislam_ctx* c, int32_t order) {
  if (!c || (order != LISLAM_TIES_REFERENCE && order != LISLAM_TIES_INDEX)) return LISLAM_ERR_ARG;
  c->ties = order;
  return LISLAM_OK;
}

int lislam_eval_factors_raw(lislam_ctx* c, int32_t n, const int32_t* kind, const double* pts, const double* q,
                            const double* t, double* residuals, double* jac_q, double* jac_t) {
  if (!c || n < 0 || (n > 0 && (!kind || !pts)) || !q || !t) return LISLAM_ERR_ARG;
  for (int32_t i = 0; i < n; i++)
    if (kind[i] < 0 || kind[i] > 6) return fail(c, LISLAM_ERR_ARG, "lislam_eval_factors_raw: block %d has kind %d", i, kind[i]);
  if (n == 0) return LISLAM_OK;
  hipSetDevice(c->device);
  std::lock_guard<std::mutex> lock(c->factor_mu);
  // [x 7][pts n*12][res n*3][jq n*12][jt n*9] doubles, then kinds
  const size_t nd = 7 + (size_t)n * (12 + 3 + 12 + 9);
  uint8_t* base = nullptr;
  const int rc = factor_scratch(c, nd * 8 + (size_t)n * 4, &base);
  if (rc) return rc;
  double* dx = reinterpret_cast<double*>(base);
  double* dp = dx + 7;
  double* dr = dp + (size_t)n * 12;
  double* djq = dr + (size_t)n * 3;
  double* djt = djq + (size_t)n * 12;
  int* dk = reinterpret_cast<int*>(djt + (size_t)n * 9);
  const double x[7] = {q[0], q[1], q[2], q[3], t[0], t[1], t[2]};
  hipError_t e = hipMemcpyAsync(dk, kind, n * sizeof(int), hipMemcpyDefault, c->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(dp, pts, (size_t)n * 12 * sizeof(double), hipMemcpyDefault, c->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(dx, x, sizeof(x), hipMemcpyHostToDevice, c->stream);
  if (e == hipSuccess) {
    RawFactorArgs a{n, dk, dp, dx, dr, djq, djt};
    launch_factors_raw(a, c->stream);
    e = hipGetLastError();
  }
  if (e == hipSuccess && residuals) e = hipMemcpyAsync(residuals, dr, (size_t)n * 3 * sizeof(double), hipMemcpyDefault, c->stream);
  if (e == hipSuccess && jac_q) e = hipMemcpyAsync(jac_q, djq, (size_t)n * 12 * sizeof(double), hipMemcpyDefault, c->stream);
  if (e == hipSuccess && jac_t) e = hipMemcpyAsync(jac_t, djt, (size_t)n * 9 * sizeof(double), hipMemcpyDefault, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  if (e != hipSuccess) return fail(c, LISLAM_ERR_DEVICE, "lislam_eval_factors_raw: %s", hipGetErrorString(e));
  return LISLAM_OK;
}

}  // extern "C"
