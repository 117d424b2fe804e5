// Host-side helpers shared by the libccsc translation units (engine.cpp, solve.cpp):
// error type and guards of the C-ABI, HIP/RCCL checks, device buffers, the context.
#pragma once

#include "../../include/ccsc.h"
#include "kernels.hpp"

#include <rccl/rccl.h>

#include <atomic>
#include <condition_variable>
#include <cstdio>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

namespace ccsc {

struct Err : std::runtime_error {
  int code;
  Err(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

#define HIPCHK(x)                                                                         \
  do {                                                                                    \
    hipError_t e_ = (x);                                                                  \
    if (e_ != hipSuccess)                                                                 \
      throw Err(CCSC_E_HIP, std::string(#x) + " failed: " + hipGetErrorString(e_));       \
  } while (0)
#define NCCLCHK(x)                                                                        \
  do {                                                                                    \
    ncclResult_t r_ = (x);                                                                \
    if (r_ != ncclSuccess)                                                                \
      throw Err(CCSC_E_RCCL, std::string(#x) + " failed: " + ncclGetErrorString(r_));     \
  } while (0)

inline void set_err(char* err, size_t errlen, const std::string& m) {
  if (err && errlen) {
    std::snprintf(err, errlen, "%s", m.c_str());
  }
}

template <typename F>
static int32_t guarded(char* err, size_t errlen, F&& f) {
  try {
    f();
    return CCSC_OK;
  } catch (const Err& e) {
    set_err(err, errlen, e.what());
    return e.code;
  } catch (const std::bad_alloc&) {
    set_err(err, errlen, "host allocation failed");
    return CCSC_E_NOMEM;
  } catch (const std::exception& e) {
    set_err(err, errlen, e.what());
    return CCSC_E_INVALID;
  }
}

// ---------------------------------------------------------------------------
// device memory helpers
// ---------------------------------------------------------------------------
struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  ~DevBuf() { release(); }
  void alloc(size_t b) {
    release();
    if (b == 0) return;
    HIPCHK(hipMalloc(&p, b));
    bytes = b;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
  }
  template <typename X> X* as() const { return reinterpret_cast<X*>(p); }
};

}  // namespace ccsc

namespace ccsc {
// In-process exchange between the device threads of a multi-device context whose
// device list repeats a device (RCCL needs distinct GPUs): every rank deposits its
// buffer, the last to arrive combines them in rank order (deterministic sums) and
// releases the others.  abort() wakes every waiter when one device thread failed.
struct HostGroup {
  int n;
  std::mutex mu;
  std::condition_variable cv;
  int arrived = 0;
  uint64_t gen = 0;
  bool aborted = false;
  std::vector<std::vector<double>> slot;
  std::vector<double> res;
  explicit HostGroup(int n_) : n(n_), slot(n_) {}
  int exchange(int rank, int op, double* buf, int64_t count) {
    std::unique_lock<std::mutex> lk(mu);
    if (aborted) return -1;
    const uint64_t g = gen;
    slot[rank].assign(buf, buf + count);
    if (++arrived == n) {
      if (op == CCSC_COMM_BCAST0) {
        res = slot[0];
      } else {
        res = slot[0];
        for (int r = 1; r < n; ++r)
          for (int64_t i = 0; i < count; ++i) res[i] += slot[r][i];
      }
      arrived = 0;
      ++gen;
      cv.notify_all();
    } else {
      cv.wait(lk, [&] { return gen != g || aborted; });
      if (aborted) return -1;
    }
    // the next exchange cannot complete (and replace res) before every rank has
    // arrived at it, i.e. has copied this result
    std::copy(res.begin(), res.begin() + count, buf);
    return 0;
  }
  void abort() {
    std::lock_guard<std::mutex> lk(mu);
    aborted = true;
    cv.notify_all();
  }
};
struct HostGroupRank {
  HostGroup* g;
  int rank;
};
static int32_t host_group_fn(void* user, int32_t op, double* buf, int64_t count) {
  auto* u = static_cast<HostGroupRank*>(user);
  return u->g->exchange(u->rank, op, buf, count);
}

// Failure state shared by the ranks of a multi-device context.  When one rank's
// thread fails, abort_group() (engine.cpp) marks the group aborted ONCE, wakes the
// in-process exchange and aborts every RCCL communicator, so the other ranks' blocked
// collectives return; every later collective of the group throws instead of touching
// a communicator.  `inflight` counts collectives between that check and their
// enqueue, so the abort does not free a communicator under them.  The next
// ccsc_learn on the context re-creates the communicators (reset_group).
struct CommGroup {
  std::mutex mu;
  std::atomic<bool> aborted{false};
  std::atomic<int> inflight{0};
};
}  // namespace ccsc

struct ccsc_ctx {
  int device = 0;
  int rank = 0;
  int nranks = 1;
  hipStream_t stream = nullptr;
  ncclComm_t comm = nullptr;       // RCCL over xGMI (production)
  ccsc_comm_fn hostfn = nullptr;   // host-staged transport (tests)
  void* hostuser = nullptr;
  std::vector<double> stage;
  // single-process multi-device context (ccsc_create_multi): one sub-context per
  // device, rank i of ndev, driven by one host thread each inside ccsc_learn
  std::vector<ccsc_ctx*> subs;
  std::unique_ptr<ccsc::HostGroup> hg;           // repeated devices: in-process exchange
  std::vector<ccsc::HostGroupRank> hg_ranks;
  std::vector<int32_t> devices;                  // the device list (ranks 0..ndev-1)
  std::shared_ptr<ccsc::CommGroup> grp;          // parent and subs of a multi-device context
  // test-only (CCSC_TEST_RCCL_SELF=1 on a one-device ccsc_create_multi): a 1-rank RCCL
  // communicator that every collective goes through, so the RCCL path (non-blocking init,
  // enqueue + wait_comm, abort / re-init) executes on a one-GPU box
  bool rccl_self = false;
};
