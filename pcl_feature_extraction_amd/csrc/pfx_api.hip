// pfx_api.hip -- the extern "C" boundary (include/pfx.h).  Host-pointer entry points stage
// through ctx-owned device buffers and call the stream-ordered *_dev implementations.
#include <cstring>

#include "pfx_internal.h"

using pfx::Error;

#define PFX_API_BEGIN try {
#define PFX_API_END(ctx)                                            \
  }                                                                 \
  catch (const pfx::Error& e) {                                     \
    if (ctx) (ctx)->last_error = e.what();                          \
    return e.code;                                                  \
  }                                                                 \
  catch (const std::exception& e) {                                 \
    if (ctx) (ctx)->last_error = e.what();                          \
    return PFX_ERR_DEVICE;                                          \
  }                                                                 \
  return PFX_OK;

namespace {

void harvest_timing(pfx_ctx* ctx) {
  if (ctx->timer.pending.empty()) return;
  PFX_HIP(hipStreamSynchronize(ctx->stream));
  for (auto& p : ctx->timer.pending) {
    float ms = 0.f;
    PFX_HIP(hipEventElapsedTime(&ms, p.a, p.b));
    auto& acc = ctx->timer.acc[p.name];
    acc.first += ms;
    acc.second += 1;
    ctx->timer.pool.push_back(p.a);
    ctx->timer.pool.push_back(p.b);
  }
  ctx->timer.pending.clear();
}

float* stage_in(pfx_ctx* ctx, const char* name, const float* host, int64_t count) {
  float* d = ctx->buf(name).as<float>(count > 0 ? count : 1);
  if (count > 0) PFX_HIP(hipMemcpyAsync(d, host, sizeof(float) * count, hipMemcpyHostToDevice, ctx->stream));
  return d;
}

void check_ctx(pfx_ctx* ctx) {
  if (!ctx) throw Error(PFX_ERR_INVALID, "null pfx_ctx");
  PFX_HIP(hipSetDevice(ctx->device));
  // the ctx-owned stream exists only once a call runs on it: a ctx re-pointed at the caller's
  // stream right after creation (the torch pipeline, the batch driver) never holds one, so it
  // takes no hardware queue (GPU_MAX_HW_QUEUES = 4 per process)
  if (ctx->on_own_stream && !ctx->own_stream) {
    PFX_HIP(hipStreamCreateWithFlags(&ctx->own_stream, hipStreamNonBlocking));
    ctx->stream = ctx->own_stream;
  }
}

}  // namespace

extern "C" {

void pfx_narf_params_default(pfx_narf_params* p) {
  if (!p) return;
  p->support_size = -1.0f;
  p->max_no_of_interest_points = -1;
  p->min_distance_between_interest_points = 0.25f;
  p->optimal_distance_to_high_surface_change = 0.25f;
  p->min_interest_value = 0.45f;
  p->min_surface_change_score = 0.2f;
  p->do_non_maximum_suppression = 1;
  p->calculate_sparse_interest_image = 1;
  p->no_of_polynomial_approximations_per_point = 0;
  p->add_points_on_straight_edges = 0;
  p->pixel_radius_borders = 3;
  p->pixel_radius_plane_extraction = 2;
  p->pixel_radius_border_direction = 2;
  p->minimum_border_probability = 0.8f;
  p->pixel_radius_principal_curvature = 2;
}

void pfx_camera_default(pfx_camera* c) {
  if (!c) return;
  c->width = 640;
  c->height = 480;
  c->center_x = 640.0f / 2.0f;
  c->center_y = 480.0f / 2.0f;
  c->focal_length_x = 525.0f;
  c->focal_length_y = 525.0f;
  for (int i = 0; i < 16; ++i) c->sensor_pose[i] = (i % 5 == 0) ? 1.0f : 0.0f;
  c->coordinate_frame = 0;
  c->noise_level = 0.0f;
  c->min_range = 0.0f;
}

pfx_status pfx_ctx_create(int device, pfx_ctx** out) {
  if (!out) return PFX_ERR_INVALID;
  *out = nullptr;
  pfx_ctx* ctx = nullptr;
  try {
    int count = 0;
    hipError_t e = hipGetDeviceCount(&count);
    if (e != hipSuccess || count == 0)
      throw Error(PFX_ERR_DEVICE, std::string("no HIP device available: ") + hipGetErrorString(e));
    if (device < 0 || device >= count) throw Error(PFX_ERR_INVALID, "device ordinal out of range");
    ctx = new pfx_ctx();
    ctx->device = device;
    PFX_HIP(hipSetDevice(device));
    ctx->on_own_stream = true;  // created on first use (check_ctx)
    *out = ctx;
    return PFX_OK;
  } catch (const Error& e) {
    delete ctx;
    return e.code;
  }
}

void pfx_ctx_destroy(pfx_ctx* ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  (void)hipStreamSynchronize(ctx->stream);
  pfx::narf_release(ctx);
  pfx::normals_release(ctx);
  pfx::keypoints_release(ctx);
  ctx->grid_a.release();
  ctx->grid_b.release();
  for (auto& kv : ctx->bufs) kv.second.release();
  for (auto& p : ctx->timer.pending) { (void)hipEventDestroy(p.a); (void)hipEventDestroy(p.b); }
  for (auto e : ctx->timer.pool) (void)hipEventDestroy(e);
  if (ctx->own_stream) (void)hipStreamDestroy(ctx->own_stream);
  if (ctx->side) (void)hipStreamDestroy(ctx->side);
  for (auto& e : ctx->fork_ev)
    if (e) (void)hipEventDestroy(e);
  if (ctx->spin_ev) (void)hipEventDestroy(ctx->spin_ev);
  if (ctx->host_rb) (void)hipHostFree(ctx->host_rb);
  if (ctx->host_scratch) (void)hipHostFree(ctx->host_scratch);
  if (ctx->fpfh_rb_mem) (void)hipHostFree(ctx->fpfh_rb_mem);
  delete ctx;
}

const char* pfx_last_error(const pfx_ctx* ctx) { return ctx ? ctx->last_error.c_str() : "null pfx_ctx"; }

pfx_status pfx_ctx_set_stream(pfx_ctx* ctx, void* hip_stream) {
  PFX_API_BEGIN
  check_ctx(ctx);
  harvest_timing(ctx);
  ctx->on_own_stream = false;
  ctx->stream = static_cast<hipStream_t>(hip_stream);  // NULL = HIP's null (legacy default) stream
  PFX_API_END(ctx)
}

pfx_status pfx_ctx_use_own_stream(pfx_ctx* ctx) {
  PFX_API_BEGIN
  check_ctx(ctx);
  harvest_timing(ctx);
  ctx->on_own_stream = true;
  check_ctx(ctx);
  ctx->stream = ctx->own_stream;
  PFX_API_END(ctx)
}

void* pfx_ctx_get_stream(pfx_ctx* ctx) {
  if (!ctx) return nullptr;
  try {
    check_ctx(ctx);
  } catch (const pfx::Error& e) {
    ctx->last_error = e.what();
    return nullptr;
  }
  return (void*)ctx->stream;
}

pfx_status pfx_ctx_trim(pfx_ctx* ctx) {
  PFX_API_BEGIN
  check_ctx(ctx);
  // a split estimation still owes its lists check (normals_launch_dev): conclude it first, so
  // the outputs it launched are validated (and rerun if needed) before its state goes
  pfx::normals_finish_dev(ctx);
  ctx->lists_gate = nullptr;  // a borrowed event the next call must not wait on
  PFX_HIP(hipStreamSynchronize(ctx->stream));
  pfx::fpfh_resolve(ctx);
  pfx::narf_release(ctx);
  pfx::normals_release(ctx);
  pfx::keypoints_release(ctx);
  ctx->grid_a.release();
  ctx->grid_b.release();
  for (auto& kv : ctx->bufs) kv.second.release();
  ctx->prep_x = nullptr;
  ctx->prep_n = -1;
  ctx->prep_qx = nullptr;
  ctx->prep_nq = -1;
  ctx->fpfh_support = nullptr;
  PFX_API_END(ctx)
}

pfx_status pfx_ctx_synchronize(pfx_ctx* ctx) {
  PFX_API_BEGIN
  check_ctx(ctx);
  PFX_HIP(hipStreamSynchronize(ctx->stream));
  pfx::fpfh_resolve(ctx);  // deferred statistics / capacity errors of the stream-ordered calls
  PFX_API_END(ctx)
}

pfx_status pfx_ctx_set_timing(pfx_ctx* ctx, int enable) {
  PFX_API_BEGIN
  check_ctx(ctx);
  harvest_timing(ctx);
  ctx->timer.enabled = enable != 0;
  ctx->timer.stages_only = enable == 2;
  PFX_API_END(ctx)
}

pfx_status pfx_ctx_set_shared(pfx_ctx* ctx, int shared) {
  PFX_API_BEGIN
  check_ctx(ctx);
  ctx->shared_device = shared != 0;
  PFX_API_END(ctx)
}

pfx_status pfx_ctx_reset_timing(pfx_ctx* ctx) {
  PFX_API_BEGIN
  check_ctx(ctx);
  harvest_timing(ctx);
  ctx->timer.acc.clear();
  PFX_API_END(ctx)
}

pfx_status pfx_ctx_kernel_time(pfx_ctx* ctx, const char* name, double* total_ms, int64_t* launches) {
  PFX_API_BEGIN
  check_ctx(ctx);
  if (!name || !total_ms || !launches) throw Error(PFX_ERR_INVALID, "null argument");
  harvest_timing(ctx);
  auto it = ctx->timer.acc.find(name);
  *total_ms = it == ctx->timer.acc.end() ? 0.0 : it->second.first;
  *launches = it == ctx->timer.acc.end() ? 0 : it->second.second;
  PFX_API_END(ctx)
}

pfx_status pfx_ctx_last_stats(pfx_ctx* ctx, const char* what, int64_t* value) {
  PFX_API_BEGIN
  if (!ctx || !what || !value) throw Error(PFX_ERR_INVALID, "null argument");
  if (ctx->fpfh_pending) {
    PFX_HIP(hipStreamSynchronize(ctx->stream));
    pfx::fpfh_resolve(ctx);
  }
  auto it = ctx->stats.find(what);
  if (it == ctx->stats.end()) throw Error(PFX_ERR_INVALID, std::string("unknown stat ") + what);
  *value = it->second;
  PFX_API_END(ctx)
}

pfx_status pfx_radius_search(pfx_ctx* ctx, const float* x, const float* y, const float* z, int64_t n,
                             const float* qx, const float* qy, const float* qz, int64_t nq, double radius,
                             int64_t* counts, int32_t* idx, float* d2, int64_t cap) {
  PFX_API_BEGIN
  check_ctx(ctx);
  if (n < 0 || nq < 0 || (n && (!x || !y || !z)) || (nq && (!qx || !qy || !qz || !counts)))
    throw Error(PFX_ERR_INVALID, "radius_search: invalid arguments");
  if (idx && (cap <= 0 || !d2)) throw Error(PFX_ERR_INVALID, "radius_search: idx needs cap > 0 and d2");
  float* dx = stage_in(ctx, "in_x", x, n);
  float* dy = stage_in(ctx, "in_y", y, n);
  float* dz = stage_in(ctx, "in_z", z, n);
  float* dqx = stage_in(ctx, "in_qx", qx, nq);
  float* dqy = stage_in(ctx, "in_qy", qy, nq);
  float* dqz = stage_in(ctx, "in_qz", qz, nq);
  int64_t* dc = ctx->buf("out_counts").as<int64_t>(nq + 1);
  int32_t* di = idx ? ctx->buf("out_idx").as<int32_t>(nq * cap + 1) : nullptr;
  float* dd = idx ? ctx->buf("out_d2").as<float>(nq * cap + 1) : nullptr;
  pfx::radius_search_dev(ctx, dx, dy, dz, n, dqx, dqy, dqz, nq, radius, dc, di, dd, cap);
  if (nq) PFX_HIP(hipMemcpyAsync(counts, dc, sizeof(int64_t) * nq, hipMemcpyDeviceToHost, ctx->stream));
  if (idx && nq) {
    PFX_HIP(hipMemcpyAsync(idx, di, sizeof(int32_t) * nq * cap, hipMemcpyDeviceToHost, ctx->stream));
    PFX_HIP(hipMemcpyAsync(d2, dd, sizeof(float) * nq * cap, hipMemcpyDeviceToHost, ctx->stream));
  }
  PFX_HIP(hipStreamSynchronize(ctx->stream));
  PFX_API_END(ctx)
}

pfx_status pfx_normals_dev(pfx_ctx* ctx, const float* d_x, const float* d_y, const float* d_z, int64_t n,
                           double radius, const float viewpoint[3], float* d_nx, float* d_ny, float* d_nz,
                           float* d_curvature) {
  PFX_API_BEGIN
  check_ctx(ctx);
  if (n < 0 || (n && (!d_x || !d_y || !d_z || !d_nx || !d_ny || !d_nz || !d_curvature)))
    throw Error(PFX_ERR_INVALID, "normals: invalid arguments");
  const float vp0[3] = {0.f, 0.f, 0.f};
  pfx::normals_dev(ctx, d_x, d_y, d_z, n, radius, viewpoint ? viewpoint : vp0, d_nx, d_ny, d_nz, d_curvature);
  PFX_API_END(ctx)
}

pfx_status pfx_normals_fast_dev(pfx_ctx* ctx, const float* d_x, const float* d_y, const float* d_z, int64_t n,
                                double radius, const float viewpoint[3], float* d_nx, float* d_ny, float* d_nz,
                                float* d_curvature) {
  PFX_API_BEGIN
  check_ctx(ctx);
  if (n < 0 || (n && (!d_x || !d_y || !d_z || !d_nx || !d_ny || !d_nz || !d_curvature)))
    throw Error(PFX_ERR_INVALID, "normals_fast: invalid arguments");
  const float vp0[3] = {0.f, 0.f, 0.f};
  pfx::normals_fast_dev(ctx, d_x, d_y, d_z, n, radius, viewpoint ? viewpoint : vp0, d_nx, d_ny, d_nz, d_curvature);
  PFX_API_END(ctx)
}

pfx_status pfx_normals_fast(pfx_ctx* ctx, const float* x, const float* y, const float* z, int64_t n, double radius,
                            const float viewpoint[3], float* nx, float* ny, float* nz, float* curvature) {
  PFX_API_BEGIN
  check_ctx(ctx);
  if (n < 0 || (n && (!x || !y || !z || !nx || !ny || !nz || !curvature)))
    throw Error(PFX_ERR_INVALID, "normals_fast: invalid arguments");
  float* dx = stage_in(ctx, "in_x", x, n);
  float* dy = stage_in(ctx, "in_y", y, n);
  float* dz = stage_in(ctx, "in_z", z, n);
  float* o = ctx->buf("out_normals").as<float>(4 * n + 4);
  const float vp0[3] = {0.f, 0.f, 0.f};
  pfx::normals_fast_dev(ctx, dx, dy, dz, n, radius, viewpoint ? viewpoint : vp0, o, o + n, o + 2 * n, o + 3 * n);
  if (n) {
    PFX_HIP(hipMemcpyAsync(nx, o, sizeof(float) * n, hipMemcpyDeviceToHost, ctx->stream));
    PFX_HIP(hipMemcpyAsync(ny, o + n, sizeof(float) * n, hipMemcpyDeviceToHost, ctx->stream));
    PFX_HIP(hipMemcpyAsync(nz, o + 2 * n, sizeof(float) * n, hipMemcpyDeviceToHost, ctx->stream));
    PFX_HIP(hipMemcpyAsync(curvature, o + 3 * n, sizeof(float) * n, hipMemcpyDeviceToHost, ctx->stream));
  }
  PFX_HIP(hipStreamSynchronize(ctx->stream));
  PFX_API_END(ctx)
}

pfx_status pfx_normals_launch_dev(pfx_ctx* ctx, const float* d_x, const float* d_y, const float* d_z, int64_t n,
                                  double radius, const float viewpoint[3], float* d_nx, float* d_ny, float* d_nz,
                                  float* d_curvature) {
  PFX_API_BEGIN
  check_ctx(ctx);
  if (n < 0 || (n && (!d_x || !d_y || !d_z || !d_nx || !d_ny || !d_nz || !d_curvature)))
    throw Error(PFX_ERR_INVALID, "normals: invalid arguments");
  const float vp0[3] = {0.f, 0.f, 0.f};
  pfx::normals_launch_dev(ctx, d_x, d_y, d_z, n, radius, viewpoint ? viewpoint : vp0, d_nx, d_ny, d_nz, d_curvature);
  PFX_API_END(ctx)
}

pfx_status pfx_normals_grid_launch_dev(pfx_ctx* ctx, const float* d_x, const float* d_y, const float* d_z, int64_t n,
                                       double radius) {
  PFX_API_BEGIN
  check_ctx(ctx);
  if (n < 0 || (n && (!d_x || !d_y || !d_z))) throw Error(PFX_ERR_INVALID, "normals grid: invalid arguments");
  pfx::normals_grid_launch_dev(ctx, d_x, d_y, d_z, n, radius);
  PFX_API_END(ctx)
}

pfx_status pfx_normals_gate_dev(pfx_ctx* ctx, void* hip_event) {
  PFX_API_BEGIN
  check_ctx(ctx);
  ctx->lists_gate = static_cast<hipEvent_t>(hip_event);
  PFX_API_END(ctx)
}

pfx_status pfx_normals_finish_dev(pfx_ctx* ctx, int32_t* rerun) {
  PFX_API_BEGIN
  check_ctx(ctx);
  const bool stood = pfx::normals_finish_dev(ctx);
  if (rerun) *rerun = stood ? 0 : 1;
  PFX_API_END(ctx)
}

pfx_status pfx_normals_prepare_dev(pfx_ctx* ctx, const float* d_x, const float* d_y, const float* d_z, int64_t n,
                                   double radius) {
  PFX_API_BEGIN
  check_ctx(ctx);
  if (n < 0 || (n && (!d_x || !d_y || !d_z)))
    throw Error(PFX_ERR_INVALID, "normals prepare: invalid arguments");
  pfx::normals_prepare_dev(ctx, d_x, d_y, d_z, n, radius);
  PFX_API_END(ctx)
}

pfx_status pfx_normals_subset_dev(pfx_ctx* ctx, const float* d_x, const float* d_y, const float* d_z, int64_t n,
                                  double radius, const uint8_t* d_mask, int32_t want, const float viewpoint[3],
                                  float* d_nx, float* d_ny, float* d_nz, float* d_curvature) {
  PFX_API_BEGIN
  check_ctx(ctx);
  if (n < 0 || (n && (!d_x || !d_y || !d_z || !d_mask || !d_nx || !d_ny || !d_nz || !d_curvature)))
    throw Error(PFX_ERR_INVALID, "normals subset: invalid arguments");
  const float vp0[3] = {0.f, 0.f, 0.f};
  pfx::normals_subset_dev(ctx, d_x, d_y, d_z, n, radius, d_mask, want, viewpoint ? viewpoint : vp0, d_nx, d_ny, d_nz,
                          d_curvature);
  PFX_API_END(ctx)
}

pfx_status pfx_normals_lists_dev(pfx_ctx* ctx, const float* d_x, const float* d_y, const float* d_z, int64_t n,
                                 double radius, float* d_nx, float* d_ny, float* d_nz, float* d_curvature) {
  PFX_API_BEGIN
  check_ctx(ctx);
  if (n < 0 || (n && (!d_x || !d_y || !d_z || !d_nx || !d_ny || !d_nz || !d_curvature)))
    throw Error(PFX_ERR_INVALID, "normals lists: invalid arguments");
  pfx::normals_lists_dev(ctx, d_x, d_y, d_z, n, radius, d_nx, d_ny, d_nz, d_curvature);
  PFX_API_END(ctx)
}

pfx_status pfx_normals_chains_dev(pfx_ctx* ctx, pfx_ctx* lists_ctx, const uint8_t* d_mask, int32_t want,
                                  const float viewpoint[3], float* d_nx, float* d_ny, float* d_nz,
                                  float* d_curvature) {
  PFX_API_BEGIN
  check_ctx(ctx);
  if (!lists_ctx || lists_ctx->device != ctx->device || !d_nx || !d_ny || !d_nz || !d_curvature)
    throw Error(PFX_ERR_INVALID, "normals chains: invalid arguments");
  const float vp0[3] = {0.f, 0.f, 0.f};
  pfx::normals_chains_dev(ctx, lists_ctx, d_mask, want, viewpoint ? viewpoint : vp0, d_nx, d_ny, d_nz, d_curvature);
  PFX_API_END(ctx)
}

pfx_status pfx_normals(pfx_ctx* ctx, const float* x, const float* y, const float* z, int64_t n, double radius,
                       const float viewpoint[3], float* nx, float* ny, float* nz, float* curvature) {
  PFX_API_BEGIN
  check_ctx(ctx);
  if (n < 0 || (n && (!x || !y || !z || !nx || !ny || !nz || !curvature)))
    throw Error(PFX_ERR_INVALID, "normals: invalid arguments");
  float* dx = stage_in(ctx, "in_x", x, n);
  float* dy = stage_in(ctx, "in_y", y, n);
  float* dz = stage_in(ctx, "in_z", z, n);
  float* out = ctx->buf("out_normals").as<float>(4 * n + 4);
  const float vp0[3] = {0.f, 0.f, 0.f};
  pfx::normals_dev(ctx, dx, dy, dz, n, radius, viewpoint ? viewpoint : vp0, out, out + n, out + 2 * n, out + 3 * n);
  if (n) {
    PFX_HIP(hipMemcpyAsync(nx, out, sizeof(float) * n, hipMemcpyDeviceToHost, ctx->stream));
    PFX_HIP(hipMemcpyAsync(ny, out + n, sizeof(float) * n, hipMemcpyDeviceToHost, ctx->stream));
    PFX_HIP(hipMemcpyAsync(nz, out + 2 * n, sizeof(float) * n, hipMemcpyDeviceToHost, ctx->stream));
    PFX_HIP(hipMemcpyAsync(curvature, out + 3 * n, sizeof(float) * n, hipMemcpyDeviceToHost, ctx->stream));
  }
  PFX_HIP(hipStreamSynchronize(ctx->stream));
  PFX_API_END(ctx)
}

static void fpfh_dev_checked(pfx_ctx* ctx, const float* d_sx, const float* d_sy, const float* d_sz,
                             const float* d_snx, const float* d_sny, const float* d_snz, int64_t n_surface,
                             const float* d_qx, const float* d_qy, const float* d_qz, int64_t nq,
                             int same_as_surface, double radius, float* d_out, bool after_normals) {
  check_ctx(ctx);
  if (n_surface < 0 || nq < 0 || (nq && !d_out) ||
      (n_surface && (!d_sx || !d_sy || !d_sz || !d_snx || !d_sny || !d_snz)) ||
      (nq && (!d_qx || !d_qy || !d_qz)))
    throw Error(PFX_ERR_INVALID, "fpfh: invalid arguments");
  if (same_as_surface && nq != n_surface)
    throw Error(PFX_ERR_INVALID, "fpfh: same_as_surface requires nq == n_surface");
  pfx::fpfh_dev(ctx, d_sx, d_sy, d_sz, d_snx, d_sny, d_snz, n_surface, d_qx, d_qy, d_qz, nq, same_as_surface,
                radius, d_out, after_normals);
}

pfx_status pfx_fpfh_dev(pfx_ctx* ctx, const float* d_sx, const float* d_sy, const float* d_sz,
                        const float* d_snx, const float* d_sny, const float* d_snz, int64_t n_surface,
                        const float* d_qx, const float* d_qy, const float* d_qz, int64_t nq,
                        int same_as_surface, double radius, float* d_out) {
  PFX_API_BEGIN
  fpfh_dev_checked(ctx, d_sx, d_sy, d_sz, d_snx, d_sny, d_snz, n_surface, d_qx, d_qy, d_qz, nq, same_as_surface,
                   radius, d_out, false);
  PFX_API_END(ctx)
}

pfx_status pfx_fpfh_after_normals_dev(pfx_ctx* ctx, const float* d_sx, const float* d_sy, const float* d_sz,
                                      const float* d_snx, const float* d_sny, const float* d_snz,
                                      int64_t n_surface, const float* d_qx, const float* d_qy,
                                      const float* d_qz, int64_t nq, int same_as_surface, double radius,
                                      float* d_out) {
  PFX_API_BEGIN
  fpfh_dev_checked(ctx, d_sx, d_sy, d_sz, d_snx, d_sny, d_snz, n_surface, d_qx, d_qy, d_qz, nq, same_as_surface,
                   radius, d_out, true);
  PFX_API_END(ctx)
}

pfx_status pfx_fpfh_prepare_dev(pfx_ctx* ctx, const float* d_sx, const float* d_sy, const float* d_sz,
                                int64_t n_surface, double radius) {
  PFX_API_BEGIN
  check_ctx(ctx);
  if (n_surface < 0 || !(radius > 0.0) || (n_surface && (!d_sx || !d_sy || !d_sz)))
    throw Error(PFX_ERR_INVALID, "fpfh_prepare: invalid arguments");
  pfx::fpfh_prepare_dev(ctx, d_sx, d_sy, d_sz, n_surface, radius);
  PFX_API_END(ctx)
}

pfx_status pfx_fpfh_prepare_queries_dev(pfx_ctx* ctx, const float* d_sx, const float* d_sy, const float* d_sz,
                                        int64_t n_surface, const float* d_qx, const float* d_qy,
                                        const float* d_qz, int64_t nq, double radius) {
  PFX_API_BEGIN
  check_ctx(ctx);
  if (n_surface < 0 || nq < 0 || !(radius > 0.0) || (n_surface && (!d_sx || !d_sy || !d_sz)) ||
      (nq && (!d_qx || !d_qy || !d_qz)))
    throw Error(PFX_ERR_INVALID, "fpfh_prepare_queries: invalid arguments");
  pfx::fpfh_prepare_queries_dev(ctx, d_sx, d_sy, d_sz, n_surface, d_qx, d_qy, d_qz, nq, radius);
  PFX_API_END(ctx)
}

pfx_status pfx_fpfh(pfx_ctx* ctx, const float* sx, const float* sy, const float* sz, const float* snx,
                    const float* sny, const float* snz, int64_t n_surface, const float* qx, const float* qy,
                    const float* qz, int64_t nq, int same_as_surface, double radius, float* out) {
  PFX_API_BEGIN
  check_ctx(ctx);
  if (n_surface < 0 || nq < 0 || (nq && !out)) throw Error(PFX_ERR_INVALID, "fpfh: invalid arguments");
  if (same_as_surface && nq != n_surface)
    throw Error(PFX_ERR_INVALID, "fpfh: same_as_surface requires nq == n_surface");
  float* dsx = stage_in(ctx, "in_x", sx, n_surface);
  float* dsy = stage_in(ctx, "in_y", sy, n_surface);
  float* dsz = stage_in(ctx, "in_z", sz, n_surface);
  float* dnx = stage_in(ctx, "in_nx", snx, n_surface);
  float* dny = stage_in(ctx, "in_ny", sny, n_surface);
  float* dnz = stage_in(ctx, "in_nz", snz, n_surface);
  float *dqx = dsx, *dqy = dsy, *dqz = dsz;
  if (!same_as_surface) {
    dqx = stage_in(ctx, "in_qx", qx, nq);
    dqy = stage_in(ctx, "in_qy", qy, nq);
    dqz = stage_in(ctx, "in_qz", qz, nq);
  }
  float* dout = ctx->buf("out_fpfh").as<float>(nq * 33 + 1);
  pfx::fpfh_dev(ctx, dsx, dsy, dsz, dnx, dny, dnz, n_surface, dqx, dqy, dqz, nq, same_as_surface, radius, dout);
  if (nq) PFX_HIP(hipMemcpyAsync(out, dout, sizeof(float) * nq * 33, hipMemcpyDeviceToHost, ctx->stream));
  PFX_HIP(hipStreamSynchronize(ctx->stream));
  pfx::fpfh_resolve(ctx);  // the host API reports at once
  PFX_API_END(ctx)
}

pfx_status pfx_fpfh_support_mask_dev(pfx_ctx* ctx, const float* d_sx, const float* d_sy, const float* d_sz,
                                     int64_t n_surface, const float* d_qx, const float* d_qy, const float* d_qz,
                                     int64_t nq, double radius, uint8_t* d_mask) {
  PFX_API_BEGIN
  check_ctx(ctx);
  if (n_surface < 0 || nq < 0 || (n_surface && (!d_sx || !d_sy || !d_sz || !d_mask)) ||
      (nq && (!d_qx || !d_qy || !d_qz)))
    throw Error(PFX_ERR_INVALID, "fpfh support mask: invalid arguments");
  pfx::fpfh_support_mask_dev(ctx, d_sx, d_sy, d_sz, n_surface, d_qx, d_qy, d_qz, nq, radius, d_mask);
  PFX_API_END(ctx)
}

pfx_status pfx_fpfh_support_ball_dev(pfx_ctx* ctx, const float* d_sx, const float* d_sy, const float* d_sz,
                                     int64_t n_surface, const float* d_qx, const float* d_qy, const float* d_qz,
                                     int64_t nq, double radius, uint8_t* d_mask) {
  PFX_API_BEGIN
  check_ctx(ctx);
  if (n_surface < 0 || nq < 0 || (n_surface && (!d_sx || !d_sy || !d_sz || !d_mask)) ||
      (nq && (!d_qx || !d_qy || !d_qz)))
    throw Error(PFX_ERR_INVALID, "fpfh support ball: invalid arguments");
  pfx::fpfh_support_ball_dev(ctx, d_sx, d_sy, d_sz, n_surface, d_qx, d_qy, d_qz, nq, radius, d_mask);
  PFX_API_END(ctx)
}

pfx_status pfx_shot_dev(pfx_ctx* ctx, const float* d_sx, const float* d_sy, const float* d_sz,
                        const float* d_snx, const float* d_sny, const float* d_snz, int64_t n_surface,
                        const float* d_qx, const float* d_qy, const float* d_qz, int64_t nq, double radius,
                        float* d_desc, float* d_rf) {
  PFX_API_BEGIN
  check_ctx(ctx);
  if (n_surface < 0 || nq < 0 || (nq && (!d_desc || !d_rf || !d_qx || !d_qy || !d_qz)))
    throw Error(PFX_ERR_INVALID, "shot: invalid arguments");
  pfx::shot_dev(ctx, d_sx, d_sy, d_sz, d_snx, d_sny, d_snz, n_surface, d_qx, d_qy, d_qz, nq, radius, d_desc, d_rf);
  PFX_API_END(ctx)
}

pfx_status pfx_shot(pfx_ctx* ctx, const float* sx, const float* sy, const float* sz, const float* snx,
                    const float* sny, const float* snz, int64_t n_surface, const float* qx, const float* qy,
                    const float* qz, int64_t nq, double radius, float* desc, float* rf) {
  PFX_API_BEGIN
  check_ctx(ctx);
  if (n_surface < 0 || nq < 0 || (nq && (!desc || !rf))) throw Error(PFX_ERR_INVALID, "shot: invalid arguments");
  float* dsx = stage_in(ctx, "in_x", sx, n_surface);
  float* dsy = stage_in(ctx, "in_y", sy, n_surface);
  float* dsz = stage_in(ctx, "in_z", sz, n_surface);
  float* dnx = stage_in(ctx, "in_nx", snx, n_surface);
  float* dny = stage_in(ctx, "in_ny", sny, n_surface);
  float* dnz = stage_in(ctx, "in_nz", snz, n_surface);
  float* dqx = stage_in(ctx, "in_qx", qx, nq);
  float* dqy = stage_in(ctx, "in_qy", qy, nq);
  float* dqz = stage_in(ctx, "in_qz", qz, nq);
  float* ddesc = ctx->buf("out_shot").as<float>(nq * 352 + 1);
  float* drf = ctx->buf("out_rf").as<float>(nq * 9 + 1);
  pfx::shot_dev(ctx, dsx, dsy, dsz, dnx, dny, dnz, n_surface, dqx, dqy, dqz, nq, radius, ddesc, drf);
  if (nq) {
    PFX_HIP(hipMemcpyAsync(desc, ddesc, sizeof(float) * nq * 352, hipMemcpyDeviceToHost, ctx->stream));
    PFX_HIP(hipMemcpyAsync(rf, drf, sizeof(float) * nq * 9, hipMemcpyDeviceToHost, ctx->stream));
  }
  PFX_HIP(hipStreamSynchronize(ctx->stream));
  PFX_API_END(ctx)
}

pfx_status pfx_range_image_planar(pfx_ctx* ctx, const float* x, const float* y, const float* z, int64_t n,
                                  const pfx_camera* cam, float* out_points) {
  PFX_API_BEGIN
  check_ctx(ctx);
  if (!cam || !out_points || n < 0 || cam->width <= 0 || cam->height <= 0)
    throw Error(PFX_ERR_INVALID, "range_image: invalid arguments");
  float* dx = stage_in(ctx, "in_x", x, n);
  float* dy = stage_in(ctx, "in_y", y, n);
  float* dz = stage_in(ctx, "in_z", z, n);
  int64_t npx = (int64_t)cam->width * cam->height;
  float4* d = ctx->buf("out_ri").as<float4>(npx);
  pfx::range_image_dev(ctx, dx, dy, dz, n, *cam, d);
  PFX_HIP(hipMemcpyAsync(out_points, d, sizeof(float4) * npx, hipMemcpyDeviceToHost, ctx->stream));
  PFX_HIP(hipStreamSynchronize(ctx->stream));
  PFX_API_END(ctx)
}

pfx_status pfx_narf_keypoints_dev(pfx_ctx* ctx, const float* d_x, const float* d_y, const float* d_z, int64_t n,
                                  const pfx_camera* cam, const pfx_narf_params* params, int32_t* out, int64_t cap,
                                  int64_t* n_out) {
  PFX_API_BEGIN
  check_ctx(ctx);
  if (!cam || !params || !n_out || n < 0 || (cap > 0 && !out))
    throw Error(PFX_ERR_INVALID, "narf: invalid arguments");
  std::vector<int32_t> kp;
  pfx::narf_dev(ctx, d_x, d_y, d_z, n, *cam, *params, kp);
  *n_out = (int64_t)kp.size();
  if ((int64_t)kp.size() > cap) throw Error(PFX_ERR_CAPACITY, "narf: output capacity too small");
  if (!kp.empty()) std::memcpy(out, kp.data(), sizeof(int32_t) * kp.size());
  PFX_API_END(ctx)
}

pfx_status pfx_narf_keypoints(pfx_ctx* ctx, const float* x, const float* y, const float* z, int64_t n,
                              const pfx_camera* cam, const pfx_narf_params* params, int32_t* out, int64_t cap,
                              int64_t* n_out) {
  PFX_API_BEGIN
  check_ctx(ctx);
  if (n < 0) throw Error(PFX_ERR_INVALID, "narf: invalid arguments");
  float* dx = stage_in(ctx, "in_x", x, n);
  float* dy = stage_in(ctx, "in_y", y, n);
  float* dz = stage_in(ctx, "in_z", z, n);
  pfx_status s = pfx_narf_keypoints_dev(ctx, dx, dy, dz, n, cam, params, out, cap, n_out);
  if (s != PFX_OK) return s;
  PFX_API_END(ctx)
}

pfx_status pfx_narf_debug_image(pfx_ctx* ctx, const char* which, void* out, int64_t count) {
  PFX_API_BEGIN
  check_ctx(ctx);
  if (!which || !out) throw Error(PFX_ERR_INVALID, "narf_debug: null argument");
  pfx::narf_debug(ctx, which, out, count);
  PFX_API_END(ctx)
}

}  // extern "C"

// ---- keypoints.h:227-229: cloud_keypoints->points.push_back(cloud->points[keypoints[i]]) ----
namespace {
__global__ void k_gather_points(const float* __restrict__ x, const float* __restrict__ y, const float* __restrict__ z,
                                int64_t n, const int32_t* __restrict__ idx, int64_t k, float* __restrict__ kx,
                                float* __restrict__ ky, float* __restrict__ kz) {
  int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= k) return;
  int32_t p = idx[i];
  kx[i] = x[p];
  ky[i] = y[p];
  kz[i] = z[p];
}
}  // namespace

extern "C" pfx_status pfx_gather_points_dev(pfx_ctx* ctx, const float* d_x, const float* d_y, const float* d_z,
                                            int64_t n, const int32_t* idx, int64_t k, float* d_kx, float* d_ky,
                                            float* d_kz, int64_t cap, int64_t* n_out) {
  PFX_API_BEGIN
  check_ctx(ctx);
  if (!n_out || k < 0 || cap < 0 || (k && !idx)) throw Error(PFX_ERR_INVALID, "gather_points: invalid arguments");
  // the reference reads cloud->points[pixel_index] unchecked (out of bounds when the index is
  // >= cloud size); the guarded mapping keeps only in-range indices, in order
  std::vector<int32_t> keep;
  keep.reserve((size_t)k);
  for (int64_t i = 0; i < k; ++i)
    if (idx[i] >= 0 && idx[i] < n) keep.push_back(idx[i]);
  if ((int64_t)keep.size() > cap)
    throw Error(PFX_ERR_CAPACITY, "gather_points: " + std::to_string(keep.size()) + " in-range keypoints, output holds " +
                                      std::to_string(cap));
  *n_out = (int64_t)keep.size();
  if (keep.empty()) return PFX_OK;
  int32_t* d_idx = ctx->buf("gather_idx").as<int32_t>(keep.size());
  // through the context's pinned block (an async DMA copy; the stream is synchronised first, so
  // a previous call's copy out of that block has completed)
  PFX_HIP(hipStreamSynchronize(ctx->stream));
  int32_t* h_idx = static_cast<int32_t*>(ctx->pinned(sizeof(int32_t) * keep.size()));
  std::memcpy(h_idx, keep.data(), sizeof(int32_t) * keep.size());
  PFX_HIP(hipMemcpyAsync(d_idx, h_idx, sizeof(int32_t) * keep.size(), hipMemcpyHostToDevice, ctx->stream));
  k_gather_points<<<(unsigned)pfx::ceil_div((int64_t)keep.size(), 256), 256, 0, ctx->stream>>>(
      d_x, d_y, d_z, n, d_idx, (int64_t)keep.size(), d_kx, d_ky, d_kz);
  pfx::check_launch("k_gather_points");
  PFX_API_END(ctx)
}

namespace {
void check_match_args(const float* src, int64_t ns, int64_t ss, const float* tgt, int64_t nt, int64_t ts,
                      int32_t dim) {
  if (dim <= 0 || ns < 0 || nt < 0 || ss < dim || ts < dim || (ns && !src) || (nt && !tgt))
    throw Error(PFX_ERR_INVALID, "correspondences: invalid arguments");
}
}  // namespace

extern "C" pfx_status pfx_nearest_descriptors_dev(pfx_ctx* ctx, const float* d_src, int64_t n_src,
                                                  int64_t src_stride, const float* d_tgt, int64_t n_tgt,
                                                  int64_t tgt_stride, int32_t dim, int32_t* d_s2t,
                                                  float* d_s2t_dist, int32_t* d_t2s, float* d_t2s_dist) {
  PFX_API_BEGIN
  check_ctx(ctx);
  check_match_args(d_src, n_src, src_stride, d_tgt, n_tgt, tgt_stride, dim);
  if (n_src && !d_s2t) throw Error(PFX_ERR_INVALID, "nearest_descriptors: null output");
  pfx::match_nearest_dev(ctx, d_src, n_src, src_stride, d_tgt, n_tgt, tgt_stride, dim, d_s2t, d_s2t_dist, d_t2s,
                         d_t2s_dist);
  PFX_API_END(ctx)
}

extern "C" pfx_status pfx_nearest_descriptors(pfx_ctx* ctx, const float* src, int64_t n_src, int64_t src_stride,
                                              const float* tgt, int64_t n_tgt, int64_t tgt_stride, int32_t dim,
                                              int32_t* s2t, float* s2t_dist) {
  PFX_API_BEGIN
  check_ctx(ctx);
  check_match_args(src, n_src, src_stride, tgt, n_tgt, tgt_stride, dim);
  if (n_src && !s2t) throw Error(PFX_ERR_INVALID, "nearest_descriptors: null output");
  const int64_t cs = n_src ? (n_src - 1) * src_stride + dim : 0, ct = n_tgt ? (n_tgt - 1) * tgt_stride + dim : 0;
  float* ds = stage_in(ctx, "in_match_src", src, cs);
  float* dt = stage_in(ctx, "in_match_tgt", tgt, ct);
  int32_t* di = ctx->buf("out_match_i").as<int32_t>(n_src + 1);
  float* dd = ctx->buf("out_match_d").as<float>(n_src + 1);
  pfx::match_nearest_dev(ctx, ds, n_src, src_stride, dt, n_tgt, tgt_stride, dim, di, dd, nullptr, nullptr);
  if (n_src) {
    PFX_HIP(hipMemcpyAsync(s2t, di, sizeof(int32_t) * n_src, hipMemcpyDeviceToHost, ctx->stream));
    if (s2t_dist) PFX_HIP(hipMemcpyAsync(s2t_dist, dd, sizeof(float) * n_src, hipMemcpyDeviceToHost, ctx->stream));
  }
  PFX_HIP(hipStreamSynchronize(ctx->stream));
  PFX_API_END(ctx)
}

extern "C" pfx_status pfx_correspondences_dev(pfx_ctx* ctx, const float* d_src, int64_t n_src, int64_t src_stride,
                                              const float* d_tgt, int64_t n_tgt, int64_t tgt_stride, int32_t dim,
                                              int32_t* d_query, int32_t* d_match, int64_t cap, int64_t* n_out) {
  PFX_API_BEGIN
  check_ctx(ctx);
  check_match_args(d_src, n_src, src_stride, d_tgt, n_tgt, tgt_stride, dim);
  if (!n_out || cap < 0 || (cap && (!d_query || !d_match)))
    throw Error(PFX_ERR_INVALID, "correspondences: invalid output arguments");
  const int64_t n = pfx::correspondences_dev(ctx, d_src, n_src, src_stride, d_tgt, n_tgt, tgt_stride, dim, d_query,
                                             d_match, cap);
  *n_out = n;
  if (n > cap) throw Error(PFX_ERR_CAPACITY, "correspondences: " + std::to_string(n) + " pairs > cap");
  PFX_API_END(ctx)
}

extern "C" pfx_status pfx_correspondences(pfx_ctx* ctx, const float* src, int64_t n_src, int64_t src_stride,
                                          const float* tgt, int64_t n_tgt, int64_t tgt_stride, int32_t dim,
                                          int32_t* query, int32_t* match, int64_t cap, int64_t* n_out) {
  PFX_API_BEGIN
  check_ctx(ctx);
  check_match_args(src, n_src, src_stride, tgt, n_tgt, tgt_stride, dim);
  if (!n_out || cap < 0 || (cap && (!query || !match)))
    throw Error(PFX_ERR_INVALID, "correspondences: invalid output arguments");
  // the last row needs only `dim` floats of its stride
  const int64_t cs = n_src ? (n_src - 1) * src_stride + dim : 0, ct = n_tgt ? (n_tgt - 1) * tgt_stride + dim : 0;
  float* ds = stage_in(ctx, "in_match_src", src, cs);
  float* dt = stage_in(ctx, "in_match_tgt", tgt, ct);
  int32_t* dq = ctx->buf("out_match_q").as<int32_t>(n_src + 1);
  int32_t* dm = ctx->buf("out_match_m").as<int32_t>(n_src + 1);
  const int64_t n = pfx::correspondences_dev(ctx, ds, n_src, src_stride, dt, n_tgt, tgt_stride, dim, dq, dm, n_src);
  *n_out = n;
  if (n > cap) throw Error(PFX_ERR_CAPACITY, "correspondences: " + std::to_string(n) + " pairs > cap");
  if (n) {
    PFX_HIP(hipMemcpyAsync(query, dq, sizeof(int32_t) * n, hipMemcpyDeviceToHost, ctx->stream));
    PFX_HIP(hipMemcpyAsync(match, dm, sizeof(int32_t) * n, hipMemcpyDeviceToHost, ctx->stream));
  }
  PFX_HIP(hipStreamSynchronize(ctx->stream));
  PFX_API_END(ctx)
}

extern "C" pfx_status pfx_pcd_read_header(const char* path, pfx_pcd_header* out) {
  if (!path || !out) return PFX_ERR_INVALID;
  std::string err;
  try {
    return pfx::pcd_read_header(path, out, err);
  } catch (...) {
    return PFX_ERR_INVALID;
  }
}

extern "C" pfx_status pfx_pcd_load_xyz_dev(pfx_ctx* ctx, const char* path, float* d_x, float* d_y, float* d_z,
                                           int64_t cap, int64_t* n_out, pfx_pcd_header* hdr) {
  PFX_API_BEGIN
  check_ctx(ctx);
  if (!path || !n_out || cap < 0 || (cap && (!d_x || !d_y || !d_z)))
    throw Error(PFX_ERR_INVALID, "pcd load: invalid arguments");
  const int64_t n = pfx::pcd_load_xyz_dev(ctx, path, d_x, d_y, d_z, cap, hdr);
  *n_out = n;
  if (n > cap) throw Error(PFX_ERR_CAPACITY, "pcd load: " + std::to_string(n) + " points > cap");
  PFX_API_END(ctx)
}

namespace {
void check_points(const float* x, const float* y, const float* z, int64_t n, const char* what) {
  if (n < 0 || (n && (!x || !y || !z))) throw Error(PFX_ERR_INVALID, std::string(what) + ": invalid point arrays");
}
void check_iss(double sal, double nm, int32_t min_nb, double t21, double t32) {
  if (!(sal > 0.0) || !(nm > 0.0) || min_nb <= 0 || !(t21 > 0.0) || !(t32 > 0.0))
    throw Error(PFX_ERR_INVALID, "iss: radii, thresholds and min neighbours must be > 0 (ISSKeypoint3D::initCompute)");
}
}  // namespace

extern "C" pfx_status pfx_cloud_resolution_dev(pfx_ctx* ctx, const float* d_x, const float* d_y, const float* d_z,
                                               int64_t n, double* resolution) {
  PFX_API_BEGIN
  check_ctx(ctx);
  check_points(d_x, d_y, d_z, n, "cloud_resolution");
  if (!resolution) throw Error(PFX_ERR_INVALID, "cloud_resolution: null output");
  *resolution = pfx::cloud_resolution_dev(ctx, d_x, d_y, d_z, n);
  PFX_API_END(ctx)
}

extern "C" pfx_status pfx_cloud_resolution(pfx_ctx* ctx, const float* x, const float* y, const float* z, int64_t n,
                                           double* resolution) {
  PFX_API_BEGIN
  check_ctx(ctx);
  check_points(x, y, z, n, "cloud_resolution");
  if (!resolution) throw Error(PFX_ERR_INVALID, "cloud_resolution: null output");
  float* dx = stage_in(ctx, "in_x", x, n);
  float* dy = stage_in(ctx, "in_y", y, n);
  float* dz = stage_in(ctx, "in_z", z, n);
  *resolution = pfx::cloud_resolution_dev(ctx, dx, dy, dz, n);
  PFX_API_END(ctx)
}

extern "C" pfx_status pfx_iss_keypoints_dev(pfx_ctx* ctx, const float* d_x, const float* d_y, const float* d_z,
                                            int64_t n, double salient_radius, double non_max_radius,
                                            int32_t min_neighbors, double threshold21, double threshold32,
                                            int32_t* d_idx, int64_t cap, int64_t* n_out, double* d_third) {
  PFX_API_BEGIN
  check_ctx(ctx);
  check_points(d_x, d_y, d_z, n, "iss");
  check_iss(salient_radius, non_max_radius, min_neighbors, threshold21, threshold32);
  if (!n_out || cap < 0 || (cap && !d_idx)) throw Error(PFX_ERR_INVALID, "iss: invalid output arguments");
  const int64_t k = pfx::iss_keypoints_dev(ctx, d_x, d_y, d_z, n, salient_radius, non_max_radius, min_neighbors,
                                           threshold21, threshold32, d_idx, cap, d_third);
  *n_out = k;
  if (k > cap) throw Error(PFX_ERR_CAPACITY, "iss: " + std::to_string(k) + " keypoints > cap");
  PFX_API_END(ctx)
}

extern "C" pfx_status pfx_iss_keypoints(pfx_ctx* ctx, const float* x, const float* y, const float* z, int64_t n,
                                        double salient_radius, double non_max_radius, int32_t min_neighbors,
                                        double threshold21, double threshold32, int32_t* idx, int64_t cap,
                                        int64_t* n_out, double* third) {
  PFX_API_BEGIN
  check_ctx(ctx);
  check_points(x, y, z, n, "iss");
  check_iss(salient_radius, non_max_radius, min_neighbors, threshold21, threshold32);
  if (!n_out || cap < 0 || (cap && !idx)) throw Error(PFX_ERR_INVALID, "iss: invalid output arguments");
  float* dx = stage_in(ctx, "in_x", x, n);
  float* dy = stage_in(ctx, "in_y", y, n);
  float* dz = stage_in(ctx, "in_z", z, n);
  int32_t* di = ctx->buf("out_iss_idx").as<int32_t>(n + 1);
  double* dt = third ? ctx->buf("out_iss_third").as<double>(n + 1) : nullptr;
  const int64_t k = pfx::iss_keypoints_dev(ctx, dx, dy, dz, n, salient_radius, non_max_radius, min_neighbors,
                                           threshold21, threshold32, di, n, dt);
  *n_out = k;
  if (k > cap) throw Error(PFX_ERR_CAPACITY, "iss: " + std::to_string(k) + " keypoints > cap");
  if (k) PFX_HIP(hipMemcpyAsync(idx, di, sizeof(int32_t) * k, hipMemcpyDeviceToHost, ctx->stream));
  if (third && n) PFX_HIP(hipMemcpyAsync(third, dt, sizeof(double) * n, hipMemcpyDeviceToHost, ctx->stream));
  PFX_HIP(hipStreamSynchronize(ctx->stream));
  PFX_API_END(ctx)
}

namespace {
void check_harris(double radius, int32_t non_max) {
  if (!(radius > 0.0)) throw Error(PFX_ERR_INVALID, "harris3d: radius must be > 0");
  if (!non_max) throw Error(PFX_ERR_UNSUPPORTED, "harris3d: only non-maximum suppression is on the accelerated path");
}
}  // namespace

extern "C" pfx_status pfx_harris3d_keypoints_dev(pfx_ctx* ctx, const float* d_x, const float* d_y, const float* d_z,
                                                 int64_t n, double radius, float threshold, int32_t non_max,
                                                 int32_t refine, int32_t* d_idx, int64_t cap, int64_t* n_out,
                                                 float* d_response, float* d_corners, int64_t* n_corners,
                                                 int32_t* d_corner_idx) {
  PFX_API_BEGIN
  check_ctx(ctx);
  check_points(d_x, d_y, d_z, n, "harris3d");
  check_harris(radius, non_max);
  if (!n_out || cap < 0 || (cap && !d_idx)) throw Error(PFX_ERR_INVALID, "harris3d: invalid output arguments");
  int64_t nc = 0;
  const int64_t k = pfx::harris3d_dev(ctx, d_x, d_y, d_z, n, radius, threshold, refine, d_idx, cap, d_response,
                                      d_corners, &nc, d_corner_idx);
  *n_out = k;
  if (n_corners) *n_corners = nc;
  if (k > cap || (d_corners && nc > cap))
    throw Error(PFX_ERR_CAPACITY, "harris3d: " + std::to_string(std::max(k, nc)) + " keypoints/corners > cap");
  PFX_API_END(ctx)
}

extern "C" pfx_status pfx_harris3d_keypoints(pfx_ctx* ctx, const float* x, const float* y, const float* z, int64_t n,
                                             double radius, float threshold, int32_t non_max, int32_t refine,
                                             int32_t* idx, int64_t cap, int64_t* n_out, float* response,
                                             float* corners, int64_t* n_corners, int32_t* corner_idx) {
  PFX_API_BEGIN
  check_ctx(ctx);
  check_points(x, y, z, n, "harris3d");
  check_harris(radius, non_max);
  if (!n_out || cap < 0 || (cap && !idx)) throw Error(PFX_ERR_INVALID, "harris3d: invalid output arguments");
  float* dx = stage_in(ctx, "in_x", x, n);
  float* dy = stage_in(ctx, "in_y", y, n);
  float* dz = stage_in(ctx, "in_z", z, n);
  int32_t* di = ctx->buf("out_h3_idx").as<int32_t>(n + 1);
  float* dr = response ? ctx->buf("out_h3_resp").as<float>(n + 1) : nullptr;
  float* dc = corners ? ctx->buf("out_h3_corners").as<float>(3 * (n + 1)) : nullptr;
  int32_t* dci = corner_idx ? ctx->buf("out_h3_cidx").as<int32_t>(n + 1) : nullptr;
  int64_t nc = 0;
  const int64_t k = pfx::harris3d_dev(ctx, dx, dy, dz, n, radius, threshold, refine, di, n, dr, dc, &nc, dci);
  *n_out = k;
  if (n_corners) *n_corners = nc;
  if (k > cap || (corners && nc > cap))
    throw Error(PFX_ERR_CAPACITY, "harris3d: " + std::to_string(std::max(k, nc)) + " keypoints/corners > cap");
  if (k) PFX_HIP(hipMemcpyAsync(idx, di, sizeof(int32_t) * k, hipMemcpyDeviceToHost, ctx->stream));
  if (response && n) PFX_HIP(hipMemcpyAsync(response, dr, sizeof(float) * n, hipMemcpyDeviceToHost, ctx->stream));
  if (corners && nc) PFX_HIP(hipMemcpyAsync(corners, dc, sizeof(float) * 3 * nc, hipMemcpyDeviceToHost, ctx->stream));
  if (corner_idx && nc)
    PFX_HIP(hipMemcpyAsync(corner_idx, dci, sizeof(int32_t) * nc, hipMemcpyDeviceToHost, ctx->stream));
  PFX_HIP(hipStreamSynchronize(ctx->stream));
  PFX_API_END(ctx)
}

extern "C" pfx_status pfx_harris6d_keypoints_dev(pfx_ctx* ctx, const float* d_x, const float* d_y, const float* d_z,
                                                 const uint32_t* d_rgb, int64_t n, double radius, float threshold,
                                                 int32_t non_max, int32_t refine, int32_t* d_idx, int64_t cap,
                                                 int64_t* n_out, float* d_response, float* d_corners,
                                                 int64_t* n_corners, float* d_grad, int32_t* d_corner_idx) {
  PFX_API_BEGIN
  check_ctx(ctx);
  check_points(d_x, d_y, d_z, n, "harris6d");
  if (n && !d_rgb) throw Error(PFX_ERR_INVALID, "harris6d: null rgb");
  check_harris(radius, non_max);
  if (!n_out || cap < 0 || (cap && !d_idx)) throw Error(PFX_ERR_INVALID, "harris6d: invalid output arguments");
  int64_t nc = 0;
  const int64_t k = pfx::harris6d_dev(ctx, d_x, d_y, d_z, d_rgb, n, radius, threshold, refine, d_idx, cap, d_response,
                                      d_corners, &nc, d_grad, d_corner_idx);
  *n_out = k;
  if (n_corners) *n_corners = nc;
  if (k > cap || (d_corners && nc > cap))
    throw Error(PFX_ERR_CAPACITY, "harris6d: " + std::to_string(std::max(k, nc)) + " keypoints/corners > cap");
  PFX_API_END(ctx)
}

extern "C" pfx_status pfx_harris6d_keypoints(pfx_ctx* ctx, const float* x, const float* y, const float* z,
                                             const uint32_t* rgb, int64_t n, double radius, float threshold,
                                             int32_t non_max, int32_t refine, int32_t* idx, int64_t cap,
                                             int64_t* n_out, float* response, float* corners, int64_t* n_corners,
                                             float* grad, int32_t* corner_idx) {
  PFX_API_BEGIN
  check_ctx(ctx);
  check_points(x, y, z, n, "harris6d");
  if (n && !rgb) throw Error(PFX_ERR_INVALID, "harris6d: null rgb");
  check_harris(radius, non_max);
  if (!n_out || cap < 0 || (cap && !idx)) throw Error(PFX_ERR_INVALID, "harris6d: invalid output arguments");
  float* dx = stage_in(ctx, "in_x", x, n);
  float* dy = stage_in(ctx, "in_y", y, n);
  float* dz = stage_in(ctx, "in_z", z, n);
  uint32_t* dc_rgb = ctx->buf("in_rgb").as<uint32_t>(n + 1);
  if (n) PFX_HIP(hipMemcpyAsync(dc_rgb, rgb, sizeof(uint32_t) * n, hipMemcpyHostToDevice, ctx->stream));
  int32_t* di = ctx->buf("out_h3_idx").as<int32_t>(n + 1);
  float* dr = response ? ctx->buf("out_h3_resp").as<float>(n + 1) : nullptr;
  float* dc = corners ? ctx->buf("out_h3_corners").as<float>(3 * (n + 1)) : nullptr;
  float* dg = grad ? ctx->buf("out_h6_grad").as<float>(3 * (n + 1)) : nullptr;
  int32_t* dci = corner_idx ? ctx->buf("out_h3_cidx").as<int32_t>(n + 1) : nullptr;
  int64_t nc = 0;
  const int64_t k = pfx::harris6d_dev(ctx, dx, dy, dz, dc_rgb, n, radius, threshold, refine, di, n, dr, dc, &nc, dg, dci);
  *n_out = k;
  if (n_corners) *n_corners = nc;
  if (k > cap || (corners && nc > cap))
    throw Error(PFX_ERR_CAPACITY, "harris6d: " + std::to_string(std::max(k, nc)) + " keypoints/corners > cap");
  if (k) PFX_HIP(hipMemcpyAsync(idx, di, sizeof(int32_t) * k, hipMemcpyDeviceToHost, ctx->stream));
  if (response && n) PFX_HIP(hipMemcpyAsync(response, dr, sizeof(float) * n, hipMemcpyDeviceToHost, ctx->stream));
  if (corners && nc) PFX_HIP(hipMemcpyAsync(corners, dc, sizeof(float) * 3 * nc, hipMemcpyDeviceToHost, ctx->stream));
  if (grad && n) PFX_HIP(hipMemcpyAsync(grad, dg, sizeof(float) * 3 * n, hipMemcpyDeviceToHost, ctx->stream));
  if (corner_idx && nc)
    PFX_HIP(hipMemcpyAsync(corner_idx, dci, sizeof(int32_t) * nc, hipMemcpyDeviceToHost, ctx->stream));
  PFX_HIP(hipStreamSynchronize(ctx->stream));
  PFX_API_END(ctx)
}

extern "C" pfx_status pfx_ransac_rejector(pfx_ctx* ctx, const float* sx, const float* sy, const float* sz, int64_t ns,
                                          const float* tx, const float* ty, const float* tz, int64_t nt,
                                          const int32_t* query, const int32_t* match, int64_t n, double threshold,
                                          int32_t max_iterations, int32_t* keep, int64_t* n_keep,
                                          float* transformation) {
  PFX_API_BEGIN
  check_ctx(ctx);
  check_points(sx, sy, sz, ns, "ransac");
  check_points(tx, ty, tz, nt, "ransac");
  if (n < 0 || (n && (!query || !match || !keep)) || !n_keep || !transformation || !(threshold > 0.0) ||
      max_iterations < 0)
    throw Error(PFX_ERR_INVALID, "ransac: invalid arguments");
  int64_t iters = 0;
  *n_keep = pfx::ransac_rejector(ctx, sx, sy, sz, ns, tx, ty, tz, nt, query, match, n, threshold, max_iterations,
                                 keep, transformation, &iters);
  ctx->stats["ransac_iterations"] = iters;
  PFX_API_END(ctx)
}
