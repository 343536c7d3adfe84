// pfx_internal.h -- host-side context, error and workspace plumbing of libpfx (HIP, gfx950).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <cstdlib>

#include <map>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/pfx.h"

namespace pfx {

struct Error : std::runtime_error {
  pfx_status code;
  Error(pfx_status c, const std::string& m) : std::runtime_error(m), code(c) {}
};

#define PFX_HIP(expr)                                                                   \
  do {                                                                                  \
    hipError_t _e = (expr);                                                             \
    if (_e != hipSuccess)                                                               \
      throw ::pfx::Error(PFX_ERR_DEVICE, std::string(#expr) + ": " + hipGetErrorString(_e)); \
  } while (0)

#define PFX_CHECK(cond, msg)                                                \
  do {                                                                      \
    if (!(cond)) throw ::pfx::Error(PFX_ERR_INVALID, std::string(msg));     \
  } while (0)

// Device scratch that only grows (one per purpose, reused across calls; no hipMalloc inside
// a steady-state call once sizes have been seen).
struct DevBuf {
  void* ptr = nullptr;
  size_t bytes = 0;
  void* get(size_t need) {
    if (need > bytes) {
      if (ptr) PFX_HIP(hipFree(ptr));
      size_t nb = need + need / 4 + 256;
      PFX_HIP(hipMalloc(&ptr, nb));
      bytes = nb;
    }
    return ptr;
  }
  template <class T> T* as(size_t count) { return static_cast<T*>(get(count * sizeof(T))); }
  void release() { if (ptr) (void)hipFree(ptr); ptr = nullptr; bytes = 0; }
};

struct KernelTimer {
  struct Pending { hipEvent_t a, b; std::string name; };
  bool enabled = false;
  bool stages_only = false;  // pfx_ctx_set_timing(ctx, 2): only the stage scopes (2 events per stage)
  std::vector<Pending> pending;
  std::vector<hipEvent_t> pool;
  std::map<std::string, std::pair<double, int64_t> > acc;
  hipEvent_t take() {
    if (!pool.empty()) { hipEvent_t e = pool.back(); pool.pop_back(); return e; }
    hipEvent_t e;
    PFX_HIP(hipEventCreate(&e));
    return e;
  }
};

// Uniform-grid spatial index over a point set (see pfx_grid.hip).
struct Grid {
  int64_t n = 0;
  float cell = 0.f, inv = 0.f, ox = 0.f, oy = 0.f, oz = 0.f;
  double dinv = 0.0, dox = 0.0, doy = 0.0, doz = 0.0;  // exact cell mapping (builder == queries)
  int32_t nx = 0, ny = 0, nz = 0;
  int64_t ncells = 0;
  // device arrays
  float *sx = nullptr, *sy = nullptr, *sz = nullptr;  // sorted-by-cell SoA coordinates
  float4* sp = nullptr;                               // the same, packed (x, y, z, 0)
  const float *ux = nullptr, *uy = nullptr, *uz = nullptr;  // the caller's arrays (not owned)
  int32_t* perm = nullptr;                            // sorted position -> caller index
  int32_t* cell_start = nullptr;                      // ncells + 1 prefix (by linear cell key)
  const uint32_t* skeys = nullptr;                    // cell key of each sorted position
  DevBuf b_sx, b_sy, b_sz, b_sp, b_perm, b_start, b_keys, b_keys2, b_vals, b_tmp, b_minmax, b_oob;
  // Speculative bounds (build_grid with use_hint): the last exact bounds of this grid, widened;
  // when a build uses them, `oob` (device int) counts the finite points outside, and the grid is
  // valid only if it stays 0 -- the caller checks it at its next readback and rebuilds exactly
  bool have_hint = false;
  double hint_lo[3] = {0, 0, 0}, hint_hi[3] = {0, 0, 0};
  int* oob = nullptr;  // non-null iff the current build is speculative
  uint64_t gen = 0;    // incremented by every build (consumers holding a grid check it)
  void release() {
    b_sx.release(); b_sy.release(); b_sz.release(); b_sp.release(); b_perm.release(); b_start.release();
    b_keys.release(); b_keys2.release(); b_vals.release(); b_tmp.release(); b_minmax.release(); b_oob.release();
    have_hint = false;
    oob = nullptr;
    ++gen;
  }
};

// Per-query view of a grid handed to kernels by value.
struct GridView {
  const float *sx, *sy, *sz;
  const float4* sp;
  const float *ux, *uy, *uz;  // caller-order (unsorted) coordinates, indexed by perm values
  const int32_t* perm;
  const int32_t* cell_start;
  double inv, ox, oy, oz;
  int32_t nx, ny, nz;
};

struct FpfhReadback {  // pfx_fpfh.hip
  int h[10];
  int64_t count;
  unsigned slow_cap;
};

struct NarfState;     // pfx_narf.hip
struct NormalsState;  // pfx_normals.hip
struct KeypointState;  // pfx_iss.hip

}  // namespace pfx

struct pfx_ctx {
  int device = 0;
  hipStream_t own_stream = nullptr;
  hipStream_t stream = nullptr;
  bool on_own_stream = true;  // stream == own_stream, created lazily (pfx_api.hip check_ctx)
  std::string last_error;
  // another stream runs latency-critical work on this device concurrently (pfx_ctx_set_shared):
  // throughput kernels whose grid is free (work queues) launch narrower
  bool shared_device = false;
  pfx::KernelTimer timer;
  std::map<std::string, int64_t> stats;
  pfx::Grid grid_a, grid_b;          // normal-radius grid, feature-radius grid
  // grid_b built ahead by pfx_fpfh_prepare_dev for (surface x pointer, n, radius)
  const float* prep_x = nullptr;
  int64_t prep_n = -1;
  double prep_r = 0.0;
  // ... and its SPFH point set for these queries (pfx_fpfh_prepare_queries_dev)
  const float* prep_qx = nullptr;
  int64_t prep_nq = -1;
  const uint8_t* fpfh_support = nullptr;  // pfx_fpfh_support_mask_dev -> next pfx_fpfh_dev
  // a speculative grid_b (pfx_fpfh_prepare_dev on the previous scan's widened bounds): its
  // out-of-bounds count, copied to pinned memory in stream order, checked by the first consumer
  int* grid_b_hoob = nullptr;
  hipEvent_t grid_b_oob_ev = nullptr;
  std::map<std::string, pfx::DevBuf> bufs;  // named scratch
  pfx::NarfState* narf = nullptr;
  pfx::NormalsState* normals = nullptr;  // neighbour lists between the two normal phases
  hipEvent_t lists_gate = nullptr;       // pfx_normals_gate_dev: waited for before the next list kernels
  bool normals_fork_hint = true;         // long-list chains on the side stream (last decision)
  pfx::KeypointState* kp = nullptr;      // grids + lists of the keypoint detectors
  pfx::DevBuf& buf(const char* name) { return bufs[name]; }
  // fpfh_dev's statistics / sticky error word, copied to pinned memory in stream order and read
  // after the next synchronisation (pfx::fpfh_resolve)
  void* fpfh_rb_mem = nullptr;
  bool fpfh_pending = false;
  pfx::FpfhReadback* fpfh_rb() {
    if (!fpfh_rb_mem) PFX_HIP(hipHostMalloc(&fpfh_rb_mem, sizeof(pfx::FpfhReadback), hipHostMallocDefault));
    return static_cast<pfx::FpfhReadback*>(fpfh_rb_mem);
  }
  // one side stream + fork/join events (normal estimation's long-list chains), created on first use
  hipStream_t side = nullptr;
  hipEvent_t fork_ev[2] = {nullptr, nullptr};
  // host wait for a stream on the critical path of a call (a readback that sizes the next
  // launches): an event polled with hipEventQuery instead of hipStreamSynchronize's blocking
  // wait, whose wake-up left ~150 us idle on the stream per readback
  hipEvent_t spin_ev = nullptr;
  void sync_spin(hipStream_t st) {
    if (!spin_ev) PFX_HIP(hipEventCreateWithFlags(&spin_ev, hipEventDisableTiming));
    PFX_HIP(hipEventRecord(spin_ev, st));
    hipError_t e;
    while ((e = hipEventQuery(spin_ev)) == hipErrorNotReady) {
    }
    PFX_HIP(e);
  }
  void ensure_side() {
    if (side) return;
    // the forked work runs at the priority of the stream the ctx was driven on when it forked
    // first (the overlapped step's normal estimation runs on a high-priority stream; measured
    // neutral on the headline, 167.7 vs 167.8 Mpoints/s, kept so a caller's priority holds)
    int prio = 0;
    if (stream) PFX_HIP(hipStreamGetPriority(stream, &prio));
    PFX_HIP(hipStreamCreateWithPriority(&side, hipStreamNonBlocking, prio));
    for (auto& e : fork_ev) PFX_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  }
  // small pinned host block for the per-call readbacks (counters, cursors): one D2H copy of
  // pinned memory per synchronisation instead of staged pageable copies
  void* host_rb = nullptr;
  template <class T> T* readback() {
    if (!host_rb) PFX_HIP(hipHostMalloc(&host_rb, 4096, hipHostMallocDefault));
    return static_cast<T*>(host_rb);
  }
  // grow-only pinned host block for larger per-call transfers (H2D of host-built index lists):
  // pageable copies are staged through blit kernels that wait for CU slots on a busy device
  void* host_scratch = nullptr;
  size_t host_scratch_bytes = 0;
  void* pinned(size_t need) {
    if (need > host_scratch_bytes) {
      if (host_scratch) {
        PFX_HIP(hipStreamSynchronize(stream));  // a pending copy may still read the old block
        PFX_HIP(hipHostFree(host_scratch));
      }
      host_scratch_bytes = need + need / 2 + 4096;
      PFX_HIP(hipHostMalloc(&host_scratch, host_scratch_bytes, hipHostMallocDefault));
    }
    return host_scratch;
  }
};

namespace pfx {

// RAII timing scope around kernel launches on ctx->stream
struct TimeScope {
  pfx_ctx* ctx;
  hipEvent_t a = nullptr, b = nullptr;
  std::string name;
  TimeScope(pfx_ctx* c, std::string n, bool stage = false) : ctx(c), name(std::move(n)) {
    if (ctx->timer.enabled && (stage || !ctx->timer.stages_only)) {
      a = ctx->timer.take();
      b = ctx->timer.take();
      PFX_HIP(hipEventRecord(a, ctx->stream));
    }
  }
  ~TimeScope() {
    if (a) {
      (void)hipEventRecord(b, ctx->stream);
      ctx->timer.pending.push_back(KernelTimer::Pending{a, b, name});
    }
  }
};

inline void check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess)
    throw Error(PFX_ERR_DEVICE, std::string("launch ") + what + ": " + hipGetErrorString(e));
}

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

// grid building (pfx_grid.hip)
void build_grid(pfx_ctx* ctx, Grid& g, const float* d_x, const float* d_y, const float* d_z,
                int64_t n, double radius, bool use_hint = false);
// bounding box of the finite points (0 when there are none), synchronous
void points_bbox(pfx_ctx* ctx, Grid& g, const float* d_x, const float* d_y, const float* d_z, int64_t n,
                 double lo[3], double hi[3]);
inline GridView view(const Grid& g) {
  GridView v;
  v.sx = g.sx; v.sy = g.sy; v.sz = g.sz; v.sp = g.sp; v.perm = g.perm; v.cell_start = g.cell_start;
  v.ux = g.ux; v.uy = g.uy; v.uz = g.uz;
  v.inv = g.dinv; v.ox = g.dox; v.oy = g.doy; v.oz = g.doz; v.nx = g.nx; v.ny = g.ny; v.nz = g.nz;
  return v;
}

// implemented in pfx_normals.hip / pfx_fpfh.hip / pfx_shot.hip / pfx_narf.hip
void normals_dev(pfx_ctx* ctx, const float* x, const float* y, const float* z, int64_t n,
                 double r, const float vp[3], float* nx, float* ny, float* nz, float* curv);
void normals_lists_dev(pfx_ctx* ctx, const float* x, const float* y, const float* z, int64_t n, double r,
                       float* nx, float* ny, float* nz, float* curv);
void normals_chains_dev(pfx_ctx* ctx, pfx_ctx* owner, const uint8_t* mask, int want, const float vp[3], float* nx,
                        float* ny, float* nz, float* curv);
void normals_release(pfx_ctx* ctx);
void normals_grid_launch_dev(pfx_ctx* ctx, const float* x, const float* y, const float* z, int64_t n, double r);
void normals_launch_dev(pfx_ctx* ctx, const float* x, const float* y, const float* z, int64_t n, double r,
                        const float vp[3], float* nx, float* ny, float* nz, float* curv);
bool normals_finish_dev(pfx_ctx* ctx);
void normals_prepare_dev(pfx_ctx* ctx, const float* x, const float* y, const float* z, int64_t n, double r);
void normals_subset_dev(pfx_ctx* ctx, const float* x, const float* y, const float* z, int64_t n, double r,
                        const uint8_t* mask, int want, const float vp[3], float* nx, float* ny, float* nz,
                        float* curv);
// opt-in MFMA covariance (pfx_normals_fast.hip): not parity-exact
void normals_fast_dev(pfx_ctx* ctx, const float* x, const float* y, const float* z, int64_t n, double r,
                      const float vp[3], float* nx, float* ny, float* nz, float* curv);
double cloud_resolution_dev(pfx_ctx* ctx, const float* x, const float* y, const float* z, int64_t n);
int64_t iss_keypoints_dev(pfx_ctx* ctx, const float* x, const float* y, const float* z, int64_t n, double salient,
                          double non_max, int min_nb, double g21, double g32, int32_t* out, int64_t cap,
                          double* third_out);
void keypoints_release(pfx_ctx* ctx);
int64_t ransac_rejector(pfx_ctx* ctx, const float* sx, const float* sy, const float* sz, int64_t ns,
                        const float* tx, const float* ty, const float* tz, int64_t nt, const int32_t* query,
                        const int32_t* match, int64_t n, double threshold, int max_iterations, int32_t* keep_out,
                        float* T_out, int64_t* iters_out);
int64_t harris3d_dev(pfx_ctx* ctx, const float* x, const float* y, const float* z, int64_t n, double radius,
                     float threshold, int refine, int32_t* out, int64_t cap, float* resp_out, float* corners_out,
                     int64_t* n_corners, int32_t* corner_idx_out = nullptr);
// Harris6D (keypoints.h:164-176): rgb packed 0x00RRGGBB; grad_out (nullable, 3 n floats): the
// normalised intensity gradients (x, y, z per point)
int64_t harris6d_dev(pfx_ctx* ctx, const float* x, const float* y, const float* z, const uint32_t* rgb, int64_t n,
                     double radius, float threshold, int refine, int32_t* out, int64_t cap, float* resp_out,
                     float* corners_out, int64_t* n_corners, float* grad_out, int32_t* corner_idx_out = nullptr);
void fpfh_support_mask_dev(pfx_ctx* ctx, const float* sx, const float* sy, const float* sz, int64_t ns,
                           const float* qx, const float* qy, const float* qz, int64_t nq, double r, uint8_t* mask);
void fpfh_support_ball_dev(pfx_ctx* ctx, const float* sx, const float* sy, const float* sz, int64_t ns,
                           const float* qx, const float* qy, const float* qz, int64_t nq, double r, uint8_t* mask);
void radius_search_dev(pfx_ctx* ctx, const float* x, const float* y, const float* z, int64_t n,
                       const float* qx, const float* qy, const float* qz, int64_t nq, double r,
                       int64_t* d_counts, int32_t* d_idx, float* d_d2, int64_t cap);
// after a synchronisation of ctx->stream: the last fpfh_dev's statistics and capacity check
void fpfh_resolve(pfx_ctx* ctx);
void fpfh_dev(pfx_ctx* ctx, const float* sx, const float* sy, const float* sz, const float* snx,
              const float* sny, const float* snz, int64_t ns, const float* qx, const float* qy,
              const float* qz, int64_t nq, int same, double r, float* out,
              bool reuse_normal_lists = false);
void fpfh_prepare_dev(pfx_ctx* ctx, const float* sx, const float* sy, const float* sz, int64_t ns, double r);
// a prepared speculative grid_b checked (one pinned read, normally long complete) and rebuilt
// exactly when a point fell outside its bounds; true when it was rebuilt
bool fpfh_validate_grid(pfx_ctx* ctx);
void fpfh_prepare_queries_dev(pfx_ctx* ctx, const float* sx, const float* sy, const float* sz, int64_t ns,
                              const float* qx, const float* qy, const float* qz, int64_t nq, double r);
void shot_dev(pfx_ctx* ctx, const float* sx, const float* sy, const float* sz, const float* snx,
              const float* sny, const float* snz, int64_t ns, const float* qx, const float* qy,
              const float* qz, int64_t nq, double r, float* desc, float* rf);
void range_image_dev(pfx_ctx* ctx, const float* x, const float* y, const float* z, int64_t n,
                     const pfx_camera& cam, float4* d_points);
int64_t narf_dev(pfx_ctx* ctx, const float* x, const float* y, const float* z, int64_t n,
                 const pfx_camera& cam, const pfx_narf_params& p, std::vector<int32_t>& out);
void narf_debug(pfx_ctx* ctx, const std::string& which, void* out, int64_t count);
void narf_release(pfx_ctx* ctx);
pfx_status pcd_read_header(const char* path, pfx_pcd_header* out, std::string& err);
int64_t pcd_load_xyz_dev(pfx_ctx* ctx, const char* path, float* d_x, float* d_y, float* d_z, int64_t cap,
                         pfx_pcd_header* hdr_out);
// mode 0: complete (one host round trip); 1: deferred -- returns true when the caller must, after
// its own stream synchronisation, call match_pairs_overflowed and rerun with mode 2 if it says so;
// 2: the two-contraction path (no pruned pair list)
bool match_nearest_dev(pfx_ctx* ctx, const float* src, int64_t ns, int64_t ss, const float* tgt, int64_t nt,
                       int64_t ts, int D, int32_t* s2t, float* ds2t, int32_t* t2s, float* dt2s, int mode = 0);
bool match_pairs_overflowed(pfx_ctx* ctx);
int64_t correspondences_dev(pfx_ctx* ctx, const float* src, int64_t ns, int64_t ss, const float* tgt, int64_t nt,
                            int64_t ts, int D, int32_t* query, int32_t* match, int64_t cap);

}  // namespace pfx
