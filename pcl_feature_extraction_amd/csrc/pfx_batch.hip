// pfx_batch.hip -- the multi-GPU scan batch behind the C-ABI (SURVEY 8(e), configs[4]).
//
// The reference runs its (keypoint, descriptor) pass scan by scan in one process
// (evaluation.cpp:272-852: Keypoints::compute, keypoints.h:199-231, then Features<T>::compute,
// features.h:175-196).  pfx_batch_narf_fpfh replaces that loop for a C++ host: one process, G
// devices, scan s on device s % G.  Per device one host thread drives two contexts on two streams
// -- a second thread issues every owned scan's normal estimation back to back on the high-priority
// side stream (the critical path), while the device thread issues scan i's NARF, keypoint gather
// and FPFH preparation on the main stream and then scan i's FPFH behind an event on scan i's
// normals, so scan i's FPFH and scan i+1's NARF run under scan i+1's normal estimation.  After
// compute the K_s x 33 descriptor blocks and K_s cloud indices of every scan move to the first
// device over RCCL (communicator from ncclCommInitAll; one group of ncclSend / ncclRecv; the K_s
// are host-known in one process, so no count exchange), are laid out in scan order there and
// copied to the caller's host arrays.  Within a scan: replicas only (NARF's greedy selection is
// sequential, a spatial split of the normals would need an r-halo).
#include <rccl/rccl.h>

#include <algorithm>
#include <condition_variable>
#include <exception>
#include <mutex>
#include <thread>

#include "pfx_internal.h"

using pfx::DevBuf;
using pfx::Error;

namespace {

#define PFX_NCCL(expr)                                                                          \
  do {                                                                                          \
    ncclResult_t _r = (expr);                                                                   \
    if (_r != ncclSuccess) throw Error(PFX_ERR_DEVICE, std::string(#expr) + ": " + ncclGetErrorString(_r)); \
  } while (0)

void ok(pfx_ctx* ctx, pfx_status st) {
  if (st != PFX_OK) throw Error(st, pfx_last_error(ctx));
}

void plan_ok(pfx_status st) {
  if (st != PFX_OK) throw Error(st, "batch: invalid scan / device counts for the plan");
}

struct ScanSlot {
  int scan = -1;
  int64_t n = 0;
  DevBuf x, y, z, nx, ny, nz, curv, kx, ky, kz, desc, idx;
  int64_t rows = 0;
  std::vector<int32_t> host_rows;  // the in-range keypoint indices (source of the index upload)
  hipEvent_t normals_done = nullptr;
};

struct Device {
  int device = 0;
  pfx_ctx* main = nullptr;
  pfx_ctx* side = nullptr;
  hipStream_t s_main = nullptr, s_side = nullptr;
  std::vector<ScanSlot> slots;  // grow-only, reused across calls
  size_t active = 0;             // slots holding this call's scans
};

// Latch per scan: the normals thread signals, the device thread waits.
struct Latches {
  std::mutex m;
  std::condition_variable cv;
  std::vector<char> done;
  bool failed = false;
  void reset(size_t n) {
    std::lock_guard<std::mutex> g(m);
    done.assign(n, 0);
    failed = false;
  }
  void set(size_t i) {
    { std::lock_guard<std::mutex> g(m); done[i] = 1; }
    cv.notify_all();
  }
  void fail() {
    { std::lock_guard<std::mutex> g(m); failed = true; }
    cv.notify_all();
  }
  bool wait(size_t i) {  // false: the normals thread failed
    std::unique_lock<std::mutex> g(m);
    cv.wait(g, [&] { return done[i] || failed; });
    return done[i] != 0;
  }
};

}  // namespace

struct pfx_batch {
  std::vector<Device> devs;
  std::vector<ncclComm_t> comms;
  DevBuf gather_desc, gather_idx;  // on devs[0]
  std::string last_error;
};

namespace {

// One device's share of the batch: upload, the two-stream pipeline, deferred-error check.
void run_device(Device& D, const float* const* x, const float* const* y, const float* const* z,
                const int64_t* n, const pfx_narf_params* params, const pfx_camera* cam, double r_normal,
                double r_feature) {
  PFX_HIP(hipSetDevice(D.device));
  const size_t m = D.active;
  for (size_t i = 0; i < m; ++i) {
    ScanSlot& S = D.slots[i];
    const int s = S.scan;
    S.n = n[s];
    float* dx = S.x.as<float>(S.n + 1);
    float* dy = S.y.as<float>(S.n + 1);
    float* dz = S.z.as<float>(S.n + 1);
    if (S.n) {
      PFX_HIP(hipMemcpyAsync(dx, x[s], sizeof(float) * S.n, hipMemcpyHostToDevice, D.s_main));
      PFX_HIP(hipMemcpyAsync(dy, y[s], sizeof(float) * S.n, hipMemcpyHostToDevice, D.s_main));
      PFX_HIP(hipMemcpyAsync(dz, z[s], sizeof(float) * S.n, hipMemcpyHostToDevice, D.s_main));
    }
    S.nx.as<float>(S.n + 1);
    S.ny.as<float>(S.n + 1);
    S.nz.as<float>(S.n + 1);
    S.curv.as<float>(S.n + 1);
    if (!S.normals_done) PFX_HIP(hipEventCreateWithFlags(&S.normals_done, hipEventDisableTiming));
  }
  // the side stream starts after the uploads on the main stream
  hipEvent_t up = nullptr;
  PFX_HIP(hipEventCreateWithFlags(&up, hipEventDisableTiming));
  PFX_HIP(hipEventRecord(up, D.s_main));
  PFX_HIP(hipStreamWaitEvent(D.s_side, up, 0));
  PFX_HIP(hipEventDestroy(up));

  Latches L;
  L.reset(m);
  std::exception_ptr side_err;
  std::thread normals([&] {
    try {
      PFX_HIP(hipSetDevice(D.device));
      const float vp[3] = {0.f, 0.f, 0.f};
      for (size_t i = 0; i < m; ++i) {
        ScanSlot& S = D.slots[i];
        ok(D.side, pfx_normals_dev(D.side, S.x.as<float>(1), S.y.as<float>(1), S.z.as<float>(1), S.n, r_normal, vp,
                                   S.nx.as<float>(1), S.ny.as<float>(1), S.nz.as<float>(1), S.curv.as<float>(1)));
        PFX_HIP(hipEventRecord(S.normals_done, D.s_side));
        L.set(i);
      }
    } catch (...) {
      side_err = std::current_exception();
      L.fail();
    }
  });
  std::exception_ptr main_err;
  try {
    const int64_t npx = (int64_t)cam->width * cam->height;
    std::vector<int32_t> kp((size_t)std::max<int64_t>(npx, 1));
    for (size_t i = 0; i < m; ++i) {
      ScanSlot& S = D.slots[i];
      const float *dx = S.x.as<float>(1), *dy = S.y.as<float>(1), *dz = S.z.as<float>(1);
      int64_t nkp = 0;
      ok(D.main, pfx_narf_keypoints_dev(D.main, dx, dy, dz, S.n, cam, params, kp.data(), npx, &nkp));
      // keypoints.h:229 reads cloud->points[pixel index]: the in-range indices, in order
      std::vector<int32_t>& rows = S.host_rows;
      rows.clear();
      rows.reserve((size_t)nkp);
      for (int64_t j = 0; j < nkp; ++j)
        if (kp[(size_t)j] >= 0 && kp[(size_t)j] < S.n) rows.push_back(kp[(size_t)j]);
      const int64_t k = (int64_t)rows.size();
      float* kx = S.kx.as<float>(k + 1);
      float* ky = S.ky.as<float>(k + 1);
      float* kz = S.kz.as<float>(k + 1);
      int32_t* didx = S.idx.as<int32_t>(k + 1);
      float* desc = S.desc.as<float>(k * 33 + 1);
      int64_t kk = 0;
      ok(D.main, pfx_gather_points_dev(D.main, dx, dy, dz, S.n, rows.data(), k, kx, ky, kz, k, &kk));
      if (k) PFX_HIP(hipMemcpyAsync(didx, rows.data(), sizeof(int32_t) * k, hipMemcpyHostToDevice, D.s_main));
      ok(D.main, pfx_fpfh_prepare_dev(D.main, dx, dy, dz, S.n, r_feature));
      if (k) ok(D.main, pfx_fpfh_prepare_queries_dev(D.main, dx, dy, dz, S.n, kx, ky, kz, k, r_feature));
      if (!L.wait(i)) break;  // the normals thread failed: its error is reported below
      PFX_HIP(hipStreamWaitEvent(D.s_main, S.normals_done, 0));
      if (k)
        ok(D.main, pfx_fpfh_dev(D.main, dx, dy, dz, S.nx.as<float>(1), S.ny.as<float>(1), S.nz.as<float>(1), S.n,
                                kx, ky, kz, k, 0, r_feature, desc));
      S.rows = k;
    }
  } catch (...) {
    main_err = std::current_exception();
  }
  normals.join();
  if (side_err) std::rethrow_exception(side_err);
  if (main_err) std::rethrow_exception(main_err);
  ok(D.side, pfx_ctx_synchronize(D.side));
  ok(D.main, pfx_ctx_synchronize(D.main));  // deferred FPFH capacity errors surface here
}

void destroy(pfx_batch* b) {
  for (Device& D : b->devs) {
    (void)hipSetDevice(D.device);
    if (D.s_main) (void)hipStreamSynchronize(D.s_main);
    if (D.s_side) (void)hipStreamSynchronize(D.s_side);
    for (ScanSlot& S : D.slots) {
      for (DevBuf* p : {&S.x, &S.y, &S.z, &S.nx, &S.ny, &S.nz, &S.curv, &S.kx, &S.ky, &S.kz, &S.desc, &S.idx})
        p->release();
      if (S.normals_done) (void)hipEventDestroy(S.normals_done);
    }
    if (D.main) pfx_ctx_destroy(D.main);
    if (D.side) pfx_ctx_destroy(D.side);
    if (D.s_main) (void)hipStreamDestroy(D.s_main);
    if (D.s_side) (void)hipStreamDestroy(D.s_side);
  }
  if (!b->devs.empty()) {
    (void)hipSetDevice(b->devs[0].device);
    b->gather_desc.release();
    b->gather_idx.release();
  }
  for (ncclComm_t c : b->comms)
    if (c) (void)ncclCommDestroy(c);
  delete b;
}

}  // namespace

extern "C" {

pfx_status pfx_batch_plan(int n_scans, int n_devices, const int64_t* rows_per_scan, int32_t* device_of_scan,
                          int32_t* slot_of_scan, int64_t* row_offset) {
  if (n_scans < 0 || n_devices <= 0) return PFX_ERR_INVALID;
  int64_t acc = 0;
  if (row_offset) row_offset[0] = 0;
  for (int s = 0; s < n_scans; ++s) {
    if (device_of_scan) device_of_scan[s] = s % n_devices;  // round-robin deal
    if (slot_of_scan) slot_of_scan[s] = s / n_devices;
    if (rows_per_scan) {
      if (rows_per_scan[s] < 0) return PFX_ERR_INVALID;
      acc += rows_per_scan[s];
    }
    if (row_offset) row_offset[s + 1] = acc;  // scan-order layout of the gathered rows
  }
  return PFX_OK;
}

pfx_status pfx_batch_create(const int* devices, int n_devices, pfx_batch** out) {
  if (!out) return PFX_ERR_INVALID;
  *out = nullptr;
  pfx_batch* b = new pfx_batch();
  try {
    int count = 0;
    PFX_HIP(hipGetDeviceCount(&count));
    if (!devices || n_devices <= 0) throw Error(PFX_ERR_INVALID, "batch: need at least one device");
    for (int i = 0; i < n_devices; ++i) {
      if (devices[i] < 0 || devices[i] >= count) throw Error(PFX_ERR_INVALID, "batch: device ordinal out of range");
      for (int j = 0; j < i; ++j)
        if (devices[j] == devices[i]) throw Error(PFX_ERR_INVALID, "batch: a device is listed twice");
    }
    b->devs.resize((size_t)n_devices);
    for (int i = 0; i < n_devices; ++i) {
      Device& D = b->devs[(size_t)i];
      D.device = devices[i];
      PFX_HIP(hipSetDevice(D.device));
      int lo = 0, hi = 0;
      PFX_HIP(hipDeviceGetStreamPriorityRange(&lo, &hi));
      PFX_HIP(hipStreamCreateWithFlags(&D.s_main, hipStreamNonBlocking));
      // the normal estimation is the critical path: its stream gets the highest priority
      PFX_HIP(hipStreamCreateWithPriority(&D.s_side, hipStreamNonBlocking, hi));
      pfx_status st = pfx_ctx_create(D.device, &D.main);
      if (st == PFX_OK) st = pfx_ctx_create(D.device, &D.side);
      if (st != PFX_OK) throw Error(st, "batch: context creation failed");
      ok(D.main, pfx_ctx_set_stream(D.main, D.s_main));
      ok(D.side, pfx_ctx_set_stream(D.side, D.s_side));
      ok(D.main, pfx_ctx_set_shared(D.main, 1));  // NARF shares the device with the critical normals
    }
    b->comms.assign((size_t)n_devices, nullptr);
    PFX_NCCL(ncclCommInitAll(b->comms.data(), n_devices, devices));
    *out = b;
    return PFX_OK;
  } catch (const Error& e) {
    destroy(b);
    return e.code;
  } catch (...) {
    destroy(b);
    return PFX_ERR_DEVICE;
  }
}

void pfx_batch_destroy(pfx_batch* b) {
  if (b) destroy(b);
}

const char* pfx_batch_last_error(const pfx_batch* b) { return b ? b->last_error.c_str() : "null pfx_batch"; }

pfx_status pfx_batch_narf_fpfh(pfx_batch* b, int n_scans, const float* const* x, const float* const* y,
                               const float* const* z, const int64_t* n, const pfx_camera* cam,
                               const pfx_narf_params* params, double normal_radius, double feature_radius,
                               float* desc, int32_t* idx, int64_t cap_rows, int64_t* rows) {
  if (!b) return PFX_ERR_INVALID;
  try {
    if (n_scans < 0 || (n_scans && (!x || !y || !z || !n || !rows)) || !cam || !params || cap_rows < 0 ||
        (cap_rows && (!desc || !idx)) || !(normal_radius > 0.0) || !(feature_radius > 0.0))
      throw Error(PFX_ERR_INVALID, "batch_narf_fpfh: invalid arguments");
    for (int s = 0; s < n_scans; ++s)
      if (n[s] < 0 || (n[s] && (!x[s] || !y[s] || !z[s])))
        throw Error(PFX_ERR_INVALID, "batch_narf_fpfh: invalid scan " + std::to_string(s));
    const int G = (int)b->devs.size();
    // deal the scans (pfx_batch_plan: scan s on device s % G as its slot s / G), slots reused
    // across calls
    std::vector<int32_t> dev_of((size_t)n_scans), slot_of((size_t)n_scans);
    plan_ok(pfx_batch_plan(n_scans, G, nullptr, dev_of.data(), slot_of.data(), nullptr));
    for (Device& D : b->devs) D.active = 0;
    for (int s = 0; s < n_scans; ++s) {
      Device& D = b->devs[(size_t)dev_of[(size_t)s]];
      const size_t i = (size_t)slot_of[(size_t)s];
      if (D.slots.size() <= i) D.slots.resize(i + 1);
      D.active = std::max(D.active, i + 1);
      D.slots[i].scan = s;
      D.slots[i].rows = 0;
    }
    std::vector<std::exception_ptr> errs((size_t)G);
    std::vector<std::thread> th;
    for (int d = 0; d < G; ++d)
      th.emplace_back([&, d] {
        try {
          run_device(b->devs[(size_t)d], x, y, z, n, params, cam, normal_radius, feature_radius);
        } catch (...) {
          errs[(size_t)d] = std::current_exception();
        }
      });
    for (auto& t : th) t.join();
    for (auto& e : errs)
      if (e) std::rethrow_exception(e);
    // scan-order row offsets on the first device (pfx_batch_plan)
    std::vector<int64_t> off((size_t)n_scans + 1, 0), k((size_t)n_scans, 0);
    for (Device& D : b->devs)
      for (size_t i = 0; i < D.active; ++i) k[(size_t)D.slots[i].scan] = D.slots[i].rows;
    plan_ok(pfx_batch_plan(n_scans, G, k.data(), nullptr, nullptr, off.data()));
    const int64_t total = off[(size_t)n_scans];
    for (int s = 0; s < n_scans; ++s) rows[s] = k[(size_t)s];
    if (total > cap_rows)
      throw Error(PFX_ERR_CAPACITY, "batch_narf_fpfh: " + std::to_string(total) + " descriptor rows, output holds " +
                                        std::to_string(cap_rows));
    if (total == 0) return PFX_OK;
    Device& R = b->devs[0];
    PFX_HIP(hipSetDevice(R.device));
    float* gd = b->gather_desc.as<float>(total * 33);
    int32_t* gi = b->gather_idx.as<int32_t>(total);
    for (size_t i = 0; i < R.active; ++i)
      if (ScanSlot& S = R.slots[i]; S.rows) {
        PFX_HIP(hipMemcpyAsync(gd + off[(size_t)S.scan] * 33, S.desc.as<float>(1), sizeof(float) * S.rows * 33,
                               hipMemcpyDeviceToDevice, R.s_main));
        PFX_HIP(hipMemcpyAsync(gi + off[(size_t)S.scan], S.idx.as<int32_t>(1), sizeof(int32_t) * S.rows,
                               hipMemcpyDeviceToDevice, R.s_main));
      }
    if (G > 1) {
      // one group: every other device sends its scans' blocks, the first device receives them
      // straight into their scan-order slots (send / recv pairs matched in issue order per peer)
      PFX_NCCL(ncclGroupStart());
      for (int d = 1; d < G; ++d) {
        Device& D = b->devs[(size_t)d];
        for (size_t i = 0; i < D.active; ++i) {
          ScanSlot& S = D.slots[i];
          if (!S.rows) continue;
          PFX_NCCL(ncclSend(S.desc.as<float>(1), (size_t)S.rows * 33, ncclFloat, 0, b->comms[(size_t)d], D.s_main));
          PFX_NCCL(ncclSend(S.idx.as<int32_t>(1), (size_t)S.rows, ncclInt32, 0, b->comms[(size_t)d], D.s_main));
          PFX_NCCL(ncclRecv(gd + off[(size_t)S.scan] * 33, (size_t)S.rows * 33, ncclFloat, d, b->comms[0], R.s_main));
          PFX_NCCL(ncclRecv(gi + off[(size_t)S.scan], (size_t)S.rows, ncclInt32, d, b->comms[0], R.s_main));
        }
      }
      PFX_NCCL(ncclGroupEnd());
    }
    PFX_HIP(hipSetDevice(R.device));
    PFX_HIP(hipMemcpyAsync(desc, gd, sizeof(float) * total * 33, hipMemcpyDeviceToHost, R.s_main));
    PFX_HIP(hipMemcpyAsync(idx, gi, sizeof(int32_t) * total, hipMemcpyDeviceToHost, R.s_main));
    PFX_HIP(hipStreamSynchronize(R.s_main));
    for (int d = 1; d < G; ++d) {
      PFX_HIP(hipSetDevice(b->devs[(size_t)d].device));
      PFX_HIP(hipStreamSynchronize(b->devs[(size_t)d].s_main));
    }
    return PFX_OK;
  } catch (const Error& e) {
    b->last_error = e.what();
    return e.code;
  } catch (const std::exception& e) {
    b->last_error = e.what();
    return PFX_ERR_DEVICE;
  }
}

}  // extern "C"
