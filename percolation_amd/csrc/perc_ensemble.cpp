// perc_ensemble.cpp -- independent realisations over the GPUs of one node.
//
// The reference runs its trials one after another in one process
// (Fortran/Square/bond_cond.f:62-70 seeds, :123-498 trial loop, rows written
// at :481-482).  Trials are independent, so here trial ii (1-based) runs on
// device (ii-1) mod ndev: one host thread and one perc_ctx per device, every
// per-trial result written straight into the caller's arrays at index ii-1
// (so the rows come back in ii order whatever device ran them), and ONE
// collective -- an RCCL all-reduce (sum, fp64) of the per-grid-point
// statistics [count, sum G, sum G^2, #spanning, sum iter] -- over the
// communicator ncclCommInitAll builds across the devices (xGMI on MI355X).
// No data-path collective: every device solves its own lattices.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "perc_internal.h"

using namespace perc;

struct perc_ensemble {
  int ndev = 0;
  int workers = 1;  // contexts (host threads, streams) per device
  int lattice = 0, m = 0, n = 0, pbc = 0;
  std::vector<int> devices;
  std::vector<perc_ctx*> ctx;  // [d * workers + w]
  std::vector<ncclComm_t> comm;
  std::vector<hipStream_t> stream;
  std::vector<double*> d_buf;  // per device all-reduce buffer
  std::vector<long long> d_cap;
};

namespace {

int nccl_status(ncclResult_t r, const char* where) {
  if (r == ncclSuccess) return PERC_OK;
  set_error(std::string(where) + ": " + ncclGetErrorString(r));
  return PERC_EHIP;
}

// GNU Fortran rand/srand stream local to one trial (the process-global
// stream of perc_srand would interleave between device threads).  Same
// Park-Miller recurrence and REAL*4 mapping as libgfortran (perc_host.cpp).
struct LocalRand {
  unsigned long long s;
  explicit LocalRand(int seed) : s(seed ? (unsigned long long)seed : 123459876ULL) {}
  float next() {
    s = (16807ULL * s) % 2147483647ULL;
    const unsigned v = (unsigned)((int)s - 1) & (~0u << 9);
    return (float)v / (float)2147483646;
  }
};

}  // namespace

extern "C" {

// 1-based id permutation of srand(seed) + the REAL*4 Fisher-Yates of
// bondc.f:162-174 (H2 spill slot order[N] = 0), without the global stream.
void perc_shuffle_seeded(int seed, int N, int* order) {
  for (int k = 0; k < N; ++k) order[k] = k + 1;
  order[N] = 0;
  LocalRand r(seed);
  for (int i = 1; i <= N; ++i) {
    const float prod = (float)(N - i + 1) * r.next();
    int j = (int)((float)i + prod);
    j = std::min(std::max(j, 1), N + 1);
    std::swap(order[i - 1], order[j - 1]);
  }
}

int perc_ensemble_trials(int ntrials, int ndev, int dev, int* ii_out) {
  if (ntrials < 0 || ndev < 1 || dev < 0 || dev >= ndev) return PERC_EINVAL;
  int c = 0;
  for (int ii = dev + 1; ii <= ntrials; ii += ndev) {
    if (ii_out) ii_out[c] = ii;
    ++c;
  }
  return c;
}

int perc_ensemble_create(int ndev, const int* devices, int lattice, int m, int n, int pbc,
                         perc_ensemble** out) {
  if (!out || ndev < 1) return PERC_EINVAL;
  *out = nullptr;
  int have = 0;
  if (hipGetDeviceCount(&have) != hipSuccess || have == 0) {
    set_error("perc_ensemble_create: no HIP device");
    return PERC_ENODEV;
  }
  auto* e = new perc_ensemble();
  e->ndev = ndev;
  e->lattice = lattice;
  e->m = m;
  e->n = n;
  e->pbc = pbc;
  for (int d = 0; d < ndev; ++d) e->devices.push_back(devices ? devices[d] : d);
  for (int d : e->devices)
    if (d < 0 || d >= have) {
      set_error("perc_ensemble_create: device id out of range");
      delete e;
      return PERC_ENODEV;
    }
  e->ctx.assign(ndev, nullptr);
  e->stream.assign(ndev, nullptr);
  e->d_buf.assign(ndev, nullptr);
  e->d_cap.assign(ndev, 0);
  for (int d = 0; d < ndev; ++d) {
    int rc = perc_ctx_create(e->devices[d], lattice, m, n, pbc, &e->ctx[d]);
    if (rc) {
      perc_ensemble_destroy(e);
      return rc;
    }
    hipSetDevice(e->devices[d]);
    if (hipStreamCreateWithFlags(&e->stream[d], hipStreamNonBlocking) != hipSuccess) {
      perc_ensemble_destroy(e);
      return hip_status(hipErrorUnknown, "perc_ensemble_create stream");
    }
  }
  e->comm.assign(ndev, nullptr);
  int rc = nccl_status(ncclCommInitAll(e->comm.data(), ndev, e->devices.data()),
                       "ncclCommInitAll");
  if (rc) {
    e->comm.clear();
    perc_ensemble_destroy(e);
    return rc;
  }
  *out = e;
  return PERC_OK;
}

int perc_ensemble_destroy(perc_ensemble* e) {
  if (!e) return PERC_EINVAL;
  for (size_t d = 0; d < e->comm.size(); ++d)
    if (e->comm[d]) ncclCommDestroy(e->comm[d]);
  for (int d = 0; d < (int)e->stream.size(); ++d) {
    hipSetDevice(e->devices[d]);
    if (e->d_buf[d]) hipFree(e->d_buf[d]);
    if (e->stream[d]) hipStreamDestroy(e->stream[d]);
  }
  for (size_t i = 0; i < e->ctx.size(); ++i)
    if (e->ctx[i]) perc_ctx_destroy(e->ctx[i]);
  delete e;
  return PERC_OK;
}

int perc_ensemble_ndev(perc_ensemble* e) { return e ? e->ndev : PERC_EINVAL; }

perc_ctx* perc_ensemble_ctx(perc_ensemble* e, int dev) {
  return (e && dev >= 0 && dev < e->ndev) ? e->ctx[(size_t)dev * e->workers] : nullptr;
}

// W contexts (host threads, streams) per device: small lattices leave most
// of a device idle in one trial's chain of labelings and one-workgroup
// solves, and independent trials fill it (bond_cond L = 64 on one GPU, one
// context per Python thread: 3.2 / 6.3 / 6.5 / 8.9 trials/s at 1 / 2 / 4 / 8,
// profiles/r2_24_cond_workers.log)
int perc_ensemble_set_workers(perc_ensemble* e, int workers) {
  if (!e || workers < 1 || workers > 64) return PERC_EINVAL;
  if (workers == e->workers) return PERC_OK;
  std::vector<perc_ctx*> nctx((size_t)e->ndev * workers, nullptr);
  int rc = PERC_OK;
  for (int d = 0; d < e->ndev; ++d)
    for (int w = 0; w < workers; ++w) {
      perc_ctx*& c = nctx[(size_t)d * workers + w];
      if (w < e->workers) {
        std::swap(c, e->ctx[(size_t)d * e->workers + w]);
      } else if (!rc) {
        rc = perc_ctx_create(e->devices[d], e->lattice, e->m, e->n, e->pbc, &c);
      }
    }
  for (perc_ctx* c : e->ctx)  // the contexts beyond the new count
    if (c) perc_ctx_destroy(c);
  e->ctx.swap(nctx);
  e->workers = workers;
  if (rc) {  // keep a consistent ensemble: back to one worker per device
    perc_ensemble_set_workers(e, 1);
    return rc;
  }
  return PERC_OK;
}

int perc_ensemble_workers(perc_ensemble* e) { return e ? e->workers : PERC_EINVAL; }

// stats[d*k .. d*k+k) is device d's vector; on return every slice holds the
// element-wise sum over the devices (ncclAllReduce, sum, fp64).
int perc_ensemble_allreduce(perc_ensemble* e, double* stats, int k) {
  if (!e || !stats || k < 0) return PERC_EINVAL;
  if (k == 0) return PERC_OK;
  for (int d = 0; d < e->ndev; ++d) {
    hipSetDevice(e->devices[d]);
    if (e->d_cap[d] < k) {
      if (e->d_buf[d]) hipFree(e->d_buf[d]);
      e->d_buf[d] = nullptr;
      hipError_t he = hipMalloc(&e->d_buf[d], sizeof(double) * k);
      if (he != hipSuccess) return hip_status(he, "perc_ensemble_allreduce");
      e->d_cap[d] = k;
    }
    hipError_t he = hipMemcpyAsync(e->d_buf[d], stats + (size_t)d * k, sizeof(double) * k,
                                   hipMemcpyHostToDevice, e->stream[d]);
    if (he != hipSuccess) return hip_status(he, "perc_ensemble_allreduce");
  }
  int rc = nccl_status(ncclGroupStart(), "ncclGroupStart");
  for (int d = 0; d < e->ndev && !rc; ++d)
    rc = nccl_status(ncclAllReduce(e->d_buf[d], e->d_buf[d], k, ncclDouble, ncclSum, e->comm[d],
                                   e->stream[d]),
                     "ncclAllReduce");
  const int rc2 = nccl_status(ncclGroupEnd(), "ncclGroupEnd");
  if (rc) return rc;
  if (rc2) return rc2;
  for (int d = 0; d < e->ndev; ++d) {
    hipSetDevice(e->devices[d]);
    hipError_t he = hipMemcpyAsync(stats + (size_t)d * k, e->d_buf[d], sizeof(double) * k,
                                   hipMemcpyDeviceToHost, e->stream[d]);
    if (he == hipSuccess) he = hipStreamSynchronize(e->stream[d]);
    if (he != hipSuccess) return hip_status(he, "perc_ensemble_allreduce");
  }
  return PERC_OK;
}

int perc_ensemble_bond_cond(perc_ensemble* e, int ntrials, const int* tseed, int npts,
                            const int* nbarr, double Va, double g0, double tol, int itmax,
                            int* nrows, double* gbot, double* gtop, int* iters, int* bf_c,
                            int* perccln, double* stats) {
  if (!e || ntrials < 0 || !tseed || npts < 0 || (npts && !nbarr) || !nrows || !bf_c ||
      !perccln || (npts && (!gbot || !gtop || !iters)))
    return PERC_EINVAL;
  const int ndev = e->ndev, W = e->workers;
  const int nb = perc_nbonds(e->lattice, e->m, e->n, e->pbc);
  // per worker, then summed per device in worker order
  std::vector<double> wacc((size_t)ndev * W * npts * 5, 0.0);
  std::vector<double> acc((size_t)ndev * npts * 5, 0.0);
  std::atomic<int> status{PERC_OK};
  std::vector<std::string> errs((size_t)ndev * W);

  auto worker = [&](int d, int w) {
    const size_t dw = (size_t)d * W + w;
    perc_ctx* h = e->ctx[dw];
    hipSetDevice(e->devices[d]);
    std::vector<int> order(nb + 1);
    double* a = wacc.data() + dw * npts * 5;
    auto check = [&](int rc) {
      if (rc && status.load() == PERC_OK) {
        int expect = PERC_OK;
        if (status.compare_exchange_strong(expect, rc)) errs[dw] = perc_last_error();
      }
      return rc == PERC_OK && status.load() == PERC_OK;
    };
    // trial ii on device (ii-1) mod ndev; on the device, worker ((ii-1) / ndev) mod W
    for (int ii = d + 1 + w * ndev; ii <= ntrials; ii += ndev * W) {
      const int t = ii - 1;
      perc_shuffle_seeded(tseed[t], nb, order.data());  // bond_cond.f:181-193
      int jj = 0, lastbf = -1;
      for (; jj < npts; ++jj) {  // bond_cond.f:392-483; a repeated nbarr stalls (H3)
        const int bf = nbarr[jj];
        if (bf <= 0 || bf <= lastbf || bf > nb) break;
        perc_label_info li{};
        perc_cond_result res{};
        if (!check(perc_occupy(h, PERC_BOND, 0, nullptr, bf, order.data()))) return;
        if (!check(perc_label(h, &li, nullptr))) return;
        if (!check(perc_conductance(h, PERC_RULE_BOND, PERC_CUR_FORTRAN, Va, g0, 1.0e-12, 2, tol,
                                    itmax, &res, nullptr)))
          return;
        const size_t o = (size_t)t * npts + jj;
        gbot[o] = res.gbot;
        gtop[o] = res.gtop;
        iters[o] = res.iter;
        double* s = a + (size_t)jj * 5;
        s[0] += 1.0;
        s[1] += res.gtop;
        s[2] += res.gtop * res.gtop;
        s[3] += li.nspan > 0 ? 1.0 : 0.0;
        s[4] += res.iter;
        lastbf = bf;
      }
      nrows[t] = jj;
      // pc and the final lowest spanning label (bond_cond.f:353-389, 486-496)
      perc_label_info li{};
      if (!check(perc_occupy(h, PERC_BOND, 0, nullptr, nb, order.data()))) return;
      if (!check(perc_label(h, &li, nullptr))) return;
      int pl = 0, first = 0;
      if (li.nspan > 0) {
        int st[4] = {0, 0, 0, 0};
        if (!check(perc_label_numbers(h, nullptr, nullptr, nullptr, 0, st))) return;
        pl = st[3];
        if (!check(perc_first_spanning(h, PERC_BOND, order.data(), nb, 0, &first))) return;
      }
      perccln[t] = pl;
      bf_c[t] = first;
    }
  };

  std::vector<std::thread> th;
  for (int d = 0; d < ndev; ++d)
    for (int w = 0; w < W; ++w) th.emplace_back(worker, d, w);
  for (auto& x : th) x.join();
  for (int d = 0; d < ndev; ++d)
    for (int w = 0; w < W; ++w)
      for (int k = 0; k < npts * 5; ++k)
        acc[(size_t)d * npts * 5 + k] += wacc[((size_t)d * W + w) * npts * 5 + k];
  if (status.load() != PERC_OK) {
    for (auto& s : errs)
      if (!s.empty()) set_error("perc_ensemble_bond_cond: " + s);
    return status.load();
  }
  const int rc = perc_ensemble_allreduce(e, acc.data(), npts * 5);
  if (rc) return rc;
  if (stats) std::memcpy(stats, acc.data(), sizeof(double) * npts * 5);
  return PERC_OK;
}

}  // extern "C"
