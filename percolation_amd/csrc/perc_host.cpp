// perc_host.cpp -- libperc C-ABI (include/perc.h): contexts, the
// gfortran-compatible RNG, orchestration of the labeling and conductance
// kernels, and the Numerical-Recipes-compatible F77 entry points.
//
// There is no CPU fallback for any compute step: a missing device is an
// error (PERC_ENODEV), never a silent host path.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "perc_internal.h"

namespace perc {

static thread_local std::string g_last_error = "ok";

void set_error(const std::string& msg) { g_last_error = msg; }

int hip_status(hipError_t e, const char* where) {
  if (e == hipSuccess) return PERC_OK;
  set_error(std::string(where) + ": " + hipGetErrorString(e));
  if (e == hipErrorOutOfMemory) return PERC_ENOMEM;
  if (e == hipErrorNoDevice || e == hipErrorInvalidDevice) return PERC_ENODEV;
  return PERC_EHIP;
}

// ---------------------------------------------------------------------------
// GNU Fortran runtime rand/srand (libgfortran intrinsics/rand.c): Park-Miller
// minimal standard, seed 0 -> 123459876, REAL*4 result ((x-1) & ~0x1FF)/2^31.
static unsigned long long g_rand_seed = 1ULL;
static std::mutex g_rand_mu;

static void srand_locked(long long i) { g_rand_seed = i ? (unsigned long long)i : 123459876ULL; }

static float rand_locked(int i) {
  if (i == 1) srand_locked(0);
  else if (i != 0) srand_locked(i);
  g_rand_seed = (16807ULL * g_rand_seed) % 2147483647ULL;
  const unsigned v = (unsigned)((int)g_rand_seed - 1) & (~0u << 9);
  return (float)v / (float)2147483646;
}

// Fisher-Yates index j = i + (N-i+1)*rand(0) in REAL*4 (bondc.f:167, H2)
static inline int fy_index(int i, int N) {
  const float r = rand_locked(0);
  const float prod = (float)(N - i + 1) * r;
  const float s = (float)i + prod;
  return (int)s;
}

static double now_ms() {
  using namespace std::chrono;
  return duration<double, std::milli>(steady_clock::now().time_since_epoch()).count();
}

static float event_ms(perc_ctx* h, int a, int b) {
  float t = 0.f;
  hipEventElapsedTime(&t, h->ev[a], h->ev[b]);
  return t;
}

// lowest-label spanning component via the host replay (hazard H4)
static int resolve_lowest_label(perc_ctx* h, int* span_root, int* perccln) {
  const Geom& g = h->g;
  const int kind = h->last.kind;
  std::vector<int> stats(4, 0);
  int lowest = 0, rep_site = 0;
  if (kind == PERC_BOND) {
    const long long nb = h->nb;
    std::vector<int> label(nb), c(nb + 2);
    int rc = replay_bonds(g, h->h_bond_first, h->last.bonds.data(), (int)h->last.bonds.size(),
                          label.data(), c.data(), (int)c.size(), stats.data());
    if (rc) return rc;
    const int cln = stats[0];
    std::vector<uint8_t> bot(cln + 1, 0), top(cln + 1, 0);
    std::vector<int> site_of(cln + 1, 0);
    for (int s = 1; s < g.t; ++s) {
      int nn[6];
      nearestn(g, s, nn);
      int k = h->h_bond_first[s];
      for (int j = 0; j < g.scn; ++j)
        if (nn[j] > s) {
          const int lab = label[k];
          if (lab > 0 && lab < cln) {
            if (s <= g.m) bot[lab] = 1;
            if (nn[j] > g.t - g.m) top[lab] = 1;
            if (!site_of[lab]) site_of[lab] = s;
          }
          ++k;
        }
    }
    for (int l = 1; l < cln; ++l)  // bondc.f:413-456
      if (c[l] >= g.n - 1 && bot[l] && top[l]) { lowest = l; break; }
    rep_site = lowest ? site_of[lowest] : 0;
  } else {
    std::vector<int> slab(g.t), c;
    int rc;
    if (kind == PERC_SITE) {
      c.assign(g.t + 2, 0);
      rc = replay_sites(g, h->last.sites.data(), (int)h->last.sites.size(), slab.data(), c.data(),
                        (int)c.size(), stats.data());
    } else {
      c.assign(g.t + h->nb + 2, 0);
      rc = replay_sitebond(g, h->h_bond_first, h->last.sites.data(), (int)h->last.sites.size(),
                           h->last.bonds.data(), (int)h->last.bonds.size(), slab.data(), nullptr,
                           c.data(), (int)c.size(), stats.data());
    }
    if (rc) return rc;
    const int cln = stats[0];
    const int minsize = kind == PERC_SITE ? g.n : 2 * g.n - 1;  // site.f:316 / sitebond.f:426
    std::vector<uint8_t> bot(cln + 1, 0), top(cln + 1, 0);
    std::vector<int> site_of(cln + 1, 0);
    for (int s = 1; s <= g.t; ++s) {
      const int lab = slab[s - 1];
      if (lab <= 0 || lab >= cln) continue;
      if (s <= g.m) bot[lab] = 1;
      if (s > g.t - g.m) top[lab] = 1;
      if (!site_of[lab]) site_of[lab] = s;
    }
    for (int l = 1; l < cln; ++l)
      if (c[l] >= minsize && bot[l] && top[l]) { lowest = l; break; }
    rep_site = lowest ? site_of[lowest] : 0;
  }
  *perccln = lowest;
  *span_root = 0;
  if (rep_site) {
    int root = 0;
    hipError_t e = dev_flatten(h);
    if (e == hipSuccess) e = hipMemcpyAsync(&root, h->d.parent + rep_site, sizeof(int), hipMemcpyDeviceToHost, h->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
    if (e != hipSuccess) return hip_status(e, "resolve_lowest_label");
    *span_root = root;
  }
  return PERC_OK;
}

void dev_free_all(perc_ctx* h);
static void free_buffers(perc_ctx* h) { dev_free_all(h); }

}  // namespace perc

using namespace perc;

// ===========================================================================
extern "C" {

void perc_srand(int seed) {
  std::lock_guard<std::mutex> lk(g_rand_mu);
  srand_locked(seed);
}

float perc_rand(int i) {
  std::lock_guard<std::mutex> lk(g_rand_mu);
  return rand_locked(i);
}

void perc_trial_seeds_scaled(int master, int k, int scale, int* tseed) {
  std::lock_guard<std::mutex> lk(g_rand_mu);
  srand_locked(master);
  for (int i = 0; i < k; ++i) {
    const float v = rand_locked(0) * (float)scale;  // REAL*4 product, then int()
    tseed[i] = (int)v + 1;
  }
}

void perc_trial_seeds(int master, int k, int* tseed) {
  perc_trial_seeds_scaled(master, k, 10000000, tseed);
}

int perc_nbonds(int lattice, int m, int n, int pbc) {
  return (int)nbonds(make_geom(lattice, m, n, pbc));
}

int perc_nearestn(int lattice, int m, int n, int pbc, int rn, int* nn) {
  const Geom g = make_geom(lattice, m, n, pbc);
  int tmp[6];
  nearestn(g, rn, tmp);
  for (int k = 0; k < 6; ++k) nn[k] = k < g.scn ? tmp[k] : 0;
  return g.scn;
}

int perc_bond_list(int lattice, int m, int n, int pbc, int* b1, int* b2) {
  const Geom g = make_geom(lattice, m, n, pbc);
  int rc = 0;
  for (int i = 1; i <= g.t - 1; ++i) {  // bondc.f:139-154
    int nn[6];
    nearestn(g, i, nn);
    for (int j = 0; j < g.scn; ++j)
      if (nn[j] > i) {
        b1[rc] = i;
        b2[rc] = nn[j];
        ++rc;
      }
  }
  return rc;
}

void perc_shuffle(int N, int* order) {
  std::lock_guard<std::mutex> lk(g_rand_mu);
  for (int i = 1; i <= N; ++i) {
    int j = fy_index(i, N);
    j = std::min(std::max(j, 1), N + 1);
    std::swap(order[i - 1], order[j - 1]);
  }
}

const char* perc_last_error(void) { return g_last_error.c_str(); }

int perc_ctx_create(int device, int lattice, int m, int n, int pbc, perc_ctx** out) {
  if (!out) return PERC_EINVAL;
  *out = nullptr;
  if ((lattice != PERC_SQUARE && lattice != PERC_TRIANGULAR) || m < 3 || n < 3 ||
      (long long)m * n >= (1LL << 31) - 16) {
    set_error("perc_ctx_create: lattice must be 0/1 and m,n >= 3");
    return PERC_EINVAL;
  }
  if (lattice == PERC_TRIANGULAR && (m % 2) == 1) {
    // Triangular/bond_cond.f:586-616: the top/bottom rows ignore row parity
    // for odd m, so the neighbour relation is asymmetric (hazard H7); the
    // reference itself documents even m (Triangular/bondc.f:72-73).
    set_error("perc_ctx_create: triangular lattice needs even m (H7)");
    return PERC_EINVAL;
  }
  {
    char rt[2048];
    if (perc_hip_runtimes(rt, (int)sizeof(rt)) > 1) {
      set_error(std::string("perc_ctx_create: two HIP runtimes in one process (") + rt +
                "): load libperc after the framework that brings its own (e.g. import torch first)");
      return PERC_ESTATE;
    }
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
    set_error("perc_ctx_create: no HIP device");
    return PERC_ENODEV;
  }
  if (device < 0 || device >= ndev) return PERC_EINVAL;
  perc_ctx* h = new perc_ctx();
  h->device = device;
  h->g = make_geom(lattice, m, n, pbc);
  h->nb = nbonds(h->g);
  h->N = h->g.t - 2 * m;
  hipError_t e = hipSetDevice(device);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking);
  for (int i = 0; i < 8 && e == hipSuccess; ++i) e = hipEventCreate(&h->ev[i]);
  if (e == hipSuccess) e = dev_build_lattice(h);
  if (e != hipSuccess) {
    const int st = hip_status(e, "perc_ctx_create");
    perc_ctx_destroy(h);
    return st;
  }
  // the bond list produced by nearestn must match the reference count
  if (h->h_bond_first[h->g.t + 1] != h->nb) {
    set_error("perc_ctx_create: bond count mismatch");
    perc_ctx_destroy(h);
    return PERC_EINVAL;
  }
  *out = h;
  return PERC_OK;
}

int perc_ctx_destroy(perc_ctx* h) {
  if (!h) return PERC_EINVAL;
  hipSetDevice(h->device);
  if (h->stream) hipStreamSynchronize(h->stream);
  if (h->dslab) dev_dslab_end(h, false);
  dslab_comm_release(h);
  free_buffers(h);
  for (int i = 0; i < 8; ++i)
    if (h->ev[i]) hipEventDestroy(h->ev[i]);
  for (hipEvent_t e : h->timing.ev) hipEventDestroy(e);
  if (h->pin) hipHostFree(h->pin);
  if (h->stream) hipStreamDestroy(h->stream);
  delete h;
  return PERC_OK;
}

static int occupy_impl(perc_ctx* h, int kind, int nsites, const int* site_order, int nbonds,
                       const int* bond_order, bool on_device) {
  if (!h || kind < PERC_BOND || kind > PERC_SITEBOND) return PERC_EINVAL;
  if (kind == PERC_SITE) nbonds = 0;
  if (kind == PERC_BOND) nsites = 0;
  if (nbonds < 0 || nbonds > h->nb || (nbonds && !bond_order)) return PERC_EINVAL;
  if (nsites < 0 || nsites > h->g.t || (nsites && !site_order)) return PERC_EINVAL;
  hipSetDevice(h->device);
  ReplayOrder& L = h->last;
  L.kind = kind;
  L.sites.clear();
  L.bonds.clear();
  L.random = false;
  L.d_sites = on_device ? site_order : nullptr;
  L.d_bonds = on_device ? bond_order : nullptr;
  L.n_sites = nsites;
  L.n_bonds = nbonds;
  L.host_valid = !on_device;
  if (!on_device) {
    L.sites.assign(site_order, site_order + nsites);
    L.bonds.assign(bond_order, bond_order + nbonds);
  }
  hipError_t e = dev_occupy(h, kind, nsites, site_order, nbonds, bond_order, on_device);
  if (e != hipSuccess) return hip_status(e, "perc_occupy");
  h->occupied = true;
  h->labeled = false;
  h->assembled = false;
  return PERC_OK;
}

// the first `count` ids of the permutation "ids 1..n in ascending
// perc_rand_key(seed, id) order" (the occupancy perc_occupy_random selects)
static void random_order(long long n, long long count, unsigned long long seed, int* out) {
  std::vector<unsigned long long> keys((size_t)n);
  const RandKeyCtx kc = perc_rand_key_ctx(seed);  // (the device draw's arithmetic; = perc_rand_key)
  for (long long i = 0; i < n; ++i) {
    const unsigned id = (unsigned)(i + 1);
    keys[(size_t)i] = (unsigned long long)perc_rand_hash32(kc, id) << 32 | id;
  }
  if (count < n) std::nth_element(keys.begin(), keys.begin() + count, keys.end());
  std::sort(keys.begin(), keys.begin() + count);
  for (long long i = 0; i < count; ++i) out[i] = (int)(keys[(size_t)i] & 0xFFFFFFFFull);
}

int perc_random_order(long long n, int count, unsigned long long seed, int kind, int* order_out) {
  if (n <= 0 || n > 0x7FFFFFFFll || count < 0 || count > n || (count && !order_out) ||
      (kind != PERC_BOND && kind != PERC_SITE))
    return PERC_EINVAL;
  random_order(n, count, kind == PERC_BOND ? perc_mix64(seed ^ 0x5DEECE66Dull) : seed, order_out);
  return PERC_OK;
}

int perc_occupy_random(perc_ctx* h, int kind, int nsites, int nbonds, unsigned long long seed) {
  if (!h || kind < PERC_BOND || kind > PERC_SITEBOND) return PERC_EINVAL;
  if (kind == PERC_SITE) nbonds = 0;
  if (kind == PERC_BOND) nsites = 0;
  if (nbonds < 0 || nbonds > h->nb || nsites < 0 || nsites > h->g.t) return PERC_EINVAL;
  hipSetDevice(h->device);
  ReplayOrder& L = h->last;
  L.kind = kind;
  L.sites.clear();
  L.bonds.clear();
  L.d_sites = L.d_bonds = nullptr;
  L.n_sites = nsites;
  L.n_bonds = nbonds;
  L.host_valid = false;
  L.random = true;
  L.seed = seed;
  hipError_t e = dev_occupy_random(h, kind, nsites, nbonds, seed);
  if (e != hipSuccess) return hip_status(e, "perc_occupy_random");
  h->occupied = true;
  h->labeled = false;
  h->assembled = false;
  return PERC_OK;
}

// host copies of a device-resident occupancy, fetched only for a replay
// (random occupancies: the order regenerated from the keys on the host)
static int ensure_host_order(perc_ctx* h) {
  ReplayOrder& L = h->last;
  if (L.host_valid) return PERC_OK;
  if (L.random) {
    L.sites.resize(L.n_sites);
    L.bonds.resize(L.n_bonds);
    if (L.n_sites) random_order(h->g.t, L.n_sites, L.seed, L.sites.data());
    if (L.n_bonds) random_order(h->nb, L.n_bonds, perc_mix64(L.seed ^ 0x5DEECE66Dull), L.bonds.data());
    L.host_valid = true;
    return PERC_OK;
  }
  L.sites.resize(L.n_sites);
  L.bonds.resize(L.n_bonds);
  hipError_t e = hipSuccess;
  if (L.n_sites) e = hipMemcpy(L.sites.data(), L.d_sites, sizeof(int) * L.n_sites, hipMemcpyDeviceToHost);
  if (e == hipSuccess && L.n_bonds)
    e = hipMemcpy(L.bonds.data(), L.d_bonds, sizeof(int) * L.n_bonds, hipMemcpyDeviceToHost);
  if (e != hipSuccess) return hip_status(e, "ensure_host_order");
  L.host_valid = true;
  return PERC_OK;
}

int perc_occupy(perc_ctx* h, int kind, int nsites, const int* site_order, int nbonds,
                const int* bond_order) {
  return occupy_impl(h, kind, nsites, site_order, nbonds, bond_order, false);
}

int perc_occupy_device(perc_ctx* h, int kind, int nsites, const int* d_site_order, int nbonds,
                       const int* d_bond_order) {
  return occupy_impl(h, kind, nsites, d_site_order, nbonds, d_bond_order, true);
}

int perc_set_kernel_timing(perc_ctx* h, int enable) {
  if (!h) return PERC_EINVAL;
  h->timing.enabled = enable != 0;
  return PERC_OK;
}

int perc_kernel_stats(perc_ctx* h, double* stats, int reset) {
  if (!h || !stats) return PERC_EINVAL;
  stats[0] = h->timing.spmv_ms;
  stats[1] = (double)h->timing.spmv_n;
  stats[2] = h->timing.update_ms;
  stats[3] = (double)h->timing.update_n;
  stats[4] = h->timing.p_ms;
  stats[5] = (double)h->timing.p_n;
  if (reset) {
    h->timing.spmv_ms = h->timing.update_ms = h->timing.p_ms = 0.0;
    h->timing.spmv_n = h->timing.update_n = h->timing.p_n = 0;
  }
  return PERC_OK;
}

int perc_system_size(perc_ctx* h, long long* out) {
  if (!h || !out) return PERC_EINVAL;
  out[0] = h->N;
  out[1] = h->nnz;
  return PERC_OK;
}

int perc_occupancy(perc_ctx* h, uint8_t* site_occ, uint8_t* bond_occ) {
  if (!h) return PERC_EINVAL;
  if (!h->occupied) return PERC_ESTATE;
  hipSetDevice(h->device);
  hipStream_t st = h->stream;
  hipError_t e = hipSuccess;
  if (site_occ) e = hipMemcpyAsync(site_occ, h->d.socc + 1, (size_t)h->g.t, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess && bond_occ) e = hipMemcpyAsync(bond_occ, h->d.bocc, (size_t)h->nb, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  return e == hipSuccess ? PERC_OK : hip_status(e, "perc_occupancy");
}

int perc_label(perc_ctx* h, perc_label_info* info, int* canon_out) {
  if (!h) return PERC_EINVAL;
  if (!h->occupied) return PERC_ESTATE;
  hipSetDevice(h->device);
  int nspan = 0, nclus = 0, list[kMaxSpanList];
  hipError_t e = dev_label(h, &nspan, list, &nclus, h->span_guess);
  if (e != hipSuccess) return hip_status(e, "perc_label");
  h->span_guess = nspan > 0;
  perc_label_info li{};
  li.nclusters = nclus;
  li.nspan = nspan;
  li.perccln = -1;  // unknown unless replayed
  if (nspan == 1) {
    li.span_root = list[0];
  } else if (nspan > 1) {
    int root = 0, pl = 0;
    int rc = ensure_host_order(h);
    if (rc) return rc;
    rc = resolve_lowest_label(h, &root, &pl);
    if (rc) return rc;
    li.span_root = root;
    li.perccln = pl;
    li.replayed = 1;
  } else {
    li.perccln = 0;
  }
  if (li.span_root && nspan == 1 && h->span_count >= 0) {
    li.span_sites = h->span_count;  // (counted with the labeling: its root is list[0])
  } else if (li.span_root) {
    e = dev_span_sites(h, li.span_root, &li.span_sites);
    if (e != hipSuccess) return hip_status(e, "perc_label");
  }
  if (canon_out) {
    e = dev_canon(h, canon_out);
    if (e != hipSuccess) return hip_status(e, "perc_label");
  }
  h->span_root = li.span_root;
  h->perccln = li.perccln;
  h->labeled = true;
  h->assembled = false;
  if (info) *info = li;
  return PERC_OK;
}

int perc_cluster_sizes(perc_ctx* h, int* maxcs, int* span_size) {
  if (!h || !maxcs || !span_size) return PERC_EINVAL;
  if (!h->labeled) return PERC_ESTATE;
  if (h->last.kind != PERC_BOND && h->last.kind != PERC_SITE) {
    set_error("perc_cluster_sizes: bond or site occupancy only");
    return PERC_EINVAL;
  }
  hipSetDevice(h->device);
  return hip_status(dev_cluster_sizes(h, h->last.kind, h->span_root, maxcs, span_size),
                    "perc_cluster_sizes");
}

static int label_numbers_impl(const Geom& g, const std::vector<int>& bond_first, int kind,
                              const int* sites, int nsites, const int* bonds, int nbond,
                              int* bond_label, int* site_label, int* csize, int cap,
                              int* stats) {
  const long long nb = nbonds(g);
  int st[4] = {0, 0, 0, 0};
  int rc;
  std::vector<int> c;
  std::vector<int> sl, bl;
  if (kind == PERC_BOND) {
    c.assign(nb + 2, 0);
    bl.assign(nb, 0);
    rc = replay_bonds(g, bond_first, bonds, nbond, bl.data(), c.data(), (int)c.size(), st);
  } else if (kind == PERC_SITE) {
    c.assign(g.t + 2, 0);
    sl.assign(g.t, 0);
    rc = replay_sites(g, sites, nsites, sl.data(), c.data(), (int)c.size(), st);
  } else if (kind == PERC_BONDSITE) {
    c.assign(g.t + nb + 2, 0);
    sl.assign(g.t, 0);
    bl.assign(nb, 0);
    rc = replay_bondsite(g, bond_first, sites, nsites, bonds, nbond, sl.data(), bl.data(),
                         c.data(), (int)c.size(), st);
  } else {
    c.assign(g.t + nb + 2, 0);
    sl.assign(g.t, 0);
    bl.assign(nb, 0);
    rc = replay_sitebond(g, bond_first, sites, nsites, bonds, nbond, sl.data(), bl.data(),
                         c.data(), (int)c.size(), st);
  }
  if (rc) return rc;
  // lowest spanning label by the reference rule (bondc.f:413-456, site.f:309-344,
  // sitebond.f:423-458)
  const int cln = st[0];
  std::vector<uint8_t> bot(cln + 1, 0), top(cln + 1, 0);
  int minsize;
  if (kind == PERC_BOND) {
    minsize = g.n - 1;
    for (int s = 1; s < g.t; ++s) {
      int nn[6];
      nearestn(g, s, nn);
      int k = bond_first[s];
      for (int j = 0; j < g.scn; ++j)
        if (nn[j] > s) {
          const int lab = bl[k++];
          if (lab <= 0 || lab >= cln) continue;
          if (s <= g.m) bot[lab] = 1;
          if (nn[j] > g.t - g.m) top[lab] = 1;
        }
    }
  } else {
    minsize = kind == PERC_SITE ? g.n : 2 * g.n - 1;
    for (int s = 1; s <= g.t; ++s) {
      const int lab = sl[s - 1];
      if (lab <= 0 || lab >= cln) continue;
      if (s <= g.m) bot[lab] = 1;
      if (s > g.t - g.m) top[lab] = 1;
    }
  }
  int perccln = 0;
  for (int l = 1; l < cln; ++l)
    if (c[l] >= minsize && bot[l] && top[l]) { perccln = l; break; }
  st[3] = perccln;
  if (bond_label && !bl.empty()) std::memcpy(bond_label, bl.data(), sizeof(int) * bl.size());
  if (site_label && !sl.empty()) std::memcpy(site_label, sl.data(), sizeof(int) * sl.size());
  if (csize) {
    if (cap < (int)c.size()) return PERC_EINVAL;
    std::memcpy(csize, c.data(), sizeof(int) * c.size());
  }
  if (stats) std::memcpy(stats, st, sizeof(st));
  return PERC_OK;
}

int perc_first_spanning(perc_ctx* h, int kind, const int* order, int n, int on_device,
                        int* first) {
  if (!h || !first || (kind != PERC_BOND && kind != PERC_SITE)) return PERC_EINVAL;
  const long long cap = kind == PERC_BOND ? h->nb : h->g.t;
  if (n < 0 || n > cap || (n && !order)) return PERC_EINVAL;
  hipSetDevice(h->device);
  const int* d = order;
  if (!on_device && n) {  // one upload; every probe occupies a prefix of it
    hipError_t e = hipMemcpy(h->d.order, order, sizeof(int) * n, hipMemcpyHostToDevice);
    if (e != hipSuccess) return hip_status(e, "perc_first_spanning");
    d = h->d.order;
  }
  auto occupy = [&](int c) {
    return occupy_impl(h, kind, kind == PERC_SITE ? c : 0, d, kind == PERC_BOND ? c : 0, d, true);
  };
  auto spans = [&](int c, bool* out) -> int {
    int rc = occupy(c);
    if (rc) return rc;
    int nspan = 0, nclus = 0, list[kMaxSpanList];
    hipError_t e = dev_label(h, &nspan, list, &nclus);
    if (e != hipSuccess) return hip_status(e, "perc_first_spanning");
    *out = nspan > 0;
    return PERC_OK;
  };
  // spanning only appears as elements are added (monotone in the count)
  bool s = false;
  int rc = spans(n, &s);
  if (rc) return rc;
  int lo = 0, hi = s ? n : 0;
  while (s && hi - lo > 1) {
    const int mid = lo + (hi - lo) / 2;
    bool sm = false;
    rc = spans(mid, &sm);
    if (rc) return rc;
    if (sm) hi = mid;
    else lo = mid;
  }
  *first = hi;
  rc = occupy(hi ? hi : n);  // leave the context at the first spanning count (or n)
  if (rc) return rc;
  return perc_label(h, nullptr, nullptr);
}

int perc_bs_perc_replay(int lattice, int m, int n, int pbc, const int* site_order, int nsites,
                        const int* bond_order, int nbond, int c0_overflow, int* first) {
  if ((lattice != PERC_SQUARE && lattice != PERC_TRIANGULAR) || m < 2 || n < 2 || !first)
    return PERC_EINVAL;
  const Geom g = make_geom(lattice, m, n, pbc);
  std::vector<int> bf(g.t + 2, 0);
  for (int s = 1; s <= g.t + 1; ++s)
    bf[s] = bf[s - 1] + ((s - 1 >= 1 && s - 1 <= g.t - 1) ? forward_count(g, s - 1) : 0);
  if (nsites < 0 || nsites > g.t || nbond < 0 || nbond > bf[g.t + 1] || (nsites && !site_order) ||
      (nbond && !bond_order))
    return PERC_EINVAL;
  *first = replay_bs_scan(g, bf, site_order, nsites, bond_order, nbond, c0_overflow != 0);
  return PERC_OK;
}

int perc_first_spanning_mixed(perc_ctx* h, int scan, const int* site_order, int nsites,
                              const int* bond_order, int nbonds, int on_device, int* first) {
  if (!h || !first || (scan != PERC_BOND && scan != PERC_SITE)) return PERC_EINVAL;
  if (nsites < 0 || nsites > h->g.t || nbonds < 0 || nbonds > h->nb) return PERC_EINVAL;
  if ((nsites && !site_order) || (nbonds && !bond_order)) return PERC_EINVAL;
  hipSetDevice(h->device);
  // both lists on the device: the bond list in the context's upload buffer,
  // the site list in a scratch buffer (host inputs are copied once)
  const int* ds = site_order;
  const int* db = bond_order;
  int* tmp = nullptr;
  hipError_t e = hipSuccess;
  if (!on_device) {
    e = hipMalloc(reinterpret_cast<void**>(&tmp), sizeof(int) * (nsites + 1));
    if (e == hipSuccess && nsites)
      e = hipMemcpy(tmp, site_order, sizeof(int) * nsites, hipMemcpyHostToDevice);
    if (e == hipSuccess && nbonds)
      e = hipMemcpy(h->d.order, bond_order, sizeof(int) * nbonds, hipMemcpyHostToDevice);
    if (e != hipSuccess) {
      if (tmp) hipFree(tmp);
      return hip_status(e, "perc_first_spanning_mixed");
    }
    ds = tmp;
    db = h->d.order;
  }
  auto occupy = [&](int c) {
    return scan == PERC_BOND ? occupy_impl(h, PERC_SITEBOND, nsites, ds, c, db, true)
                             : occupy_impl(h, PERC_SITEBOND, c, ds, nbonds, db, true);
  };
  auto spans = [&](int c, bool* out) -> int {
    int rc = occupy(c);
    if (rc) return rc;
    int nspan = 0, nclus = 0, list[kMaxSpanList];
    hipError_t err = dev_label(h, &nspan, list, &nclus);
    if (err != hipSuccess) return hip_status(err, "perc_first_spanning_mixed");
    *out = nspan > 0;
    return PERC_OK;
  };
  const int n = scan == PERC_BOND ? nbonds : nsites;
  bool s = false;
  int rc = spans(n, &s);
  int lo = 0, hi = s ? n : 0;
  while (!rc && s && hi - lo > 1) {  // monotone in the scanned count
    const int mid = lo + (hi - lo) / 2;
    bool sm = false;
    rc = spans(mid, &sm);
    if (sm) hi = mid;
    else lo = mid;
  }
  if (!rc) *first = hi;
  // the device lists are not kept: the context is left unoccupied
  h->occupied = h->labeled = h->assembled = false;
  hipError_t e2 = hipDeviceSynchronize();
  if (tmp) hipFree(tmp);
  if (rc) return rc;
  return hip_status(e2, "perc_first_spanning_mixed");
}

int perc_label_numbers(perc_ctx* h, int* bond_label, int* site_label, int* csize, int cap,
                       int* stats) {
  if (!h) return PERC_EINVAL;
  if (!h->occupied) return PERC_ESTATE;
  const int rc = ensure_host_order(h);
  if (rc) return rc;
  return label_numbers_impl(h->g, h->h_bond_first, h->last.kind, h->last.sites.data(),
                            (int)h->last.sites.size(), h->last.bonds.data(),
                            (int)h->last.bonds.size(), bond_label, site_label, csize, cap, stats);
}

int perc_replay_labels(int lattice, int m, int n, int pbc, int kind, int nsites,
                       const int* site_order, int nbond, const int* bond_order, int* bond_label,
                       int* site_label, int* csize, int cap, int* stats) {
  if ((lattice != PERC_SQUARE && lattice != PERC_TRIANGULAR) || m < 2 || n < 2 ||
      kind < PERC_BOND || kind > PERC_BONDSITE)
    return PERC_EINVAL;
  const Geom g = make_geom(lattice, m, n, pbc);
  std::vector<int> bf(g.t + 2, 0);
  for (int s = 1; s <= g.t + 1; ++s)
    bf[s] = bf[s - 1] + ((s - 1 >= 1 && s - 1 <= g.t - 1) ? forward_count(g, s - 1) : 0);
  if (kind != PERC_SITE && (nbond < 0 || nbond > bf[g.t + 1] || (nbond && !bond_order)))
    return PERC_EINVAL;
  if (kind != PERC_BOND && (nsites < 0 || nsites > g.t || (nsites && !site_order)))
    return PERC_EINVAL;
  return label_numbers_impl(g, bf, kind, site_order, kind == PERC_BOND ? 0 : nsites, bond_order,
                            kind == PERC_SITE ? 0 : nbond, bond_label, site_label, csize, cap,
                            stats);
}

int perc_replay_bond_trace(int lattice, int m, int n, int pbc, int nbond, const int* bond_order,
                           int* trace) {
  if ((lattice != PERC_SQUARE && lattice != PERC_TRIANGULAR) || m < 2 || n < 2 || nbond < 0 ||
      (nbond && (!bond_order || !trace)))
    return PERC_EINVAL;
  const Geom g = make_geom(lattice, m, n, pbc);
  std::vector<int> bf(g.t + 2, 0);
  for (int s = 1; s <= g.t + 1; ++s)
    bf[s] = bf[s - 1] + ((s - 1 >= 1 && s - 1 <= g.t - 1) ? forward_count(g, s - 1) : 0);
  if (nbond > bf[g.t + 1] + 1) return PERC_EINVAL;
  const long long nb = nbonds(g);
  std::vector<int> c(nb + 2, 0), bl(nb, 0);
  int st[4] = {0, 0, 0, 0};
  return replay_bonds(g, bf, bond_order, nbond, bl.data(), c.data(), (int)c.size(), st, trace);
}

int perc_replay_site_trace(int lattice, int m, int n, int pbc, int nsite, const int* site_order,
                           int* trace) {
  if ((lattice != PERC_SQUARE && lattice != PERC_TRIANGULAR) || m < 2 || n < 2 || nsite < 0 ||
      (nsite && (!site_order || !trace)))
    return PERC_EINVAL;
  static_assert(PERC_SITE_TRACE == kSiteTrace, "trace record size");
  const Geom g = make_geom(lattice, m, n, pbc);
  if (nsite > g.t) return PERC_EINVAL;
  for (int i = 0; i < nsite; ++i)
    if (site_order[i] < 1 || site_order[i] > g.t) {
      set_error("perc_replay_site_trace: site id outside 1..m*n");
      return PERC_EREPLAY;
    }
  std::vector<int> c(g.t + 2, 0), sl(g.t, 0);
  int st[4] = {0, 0, 0, 0};
  return replay_sites(g, site_order, nsite, sl.data(), c.data(), (int)c.size(), st, trace);
}

int perc_replay_mixed_trace(int lattice, int m, int n, int pbc, int kind, int nsites,
                            const int* site_order, int nbond, const int* bond_order, int* trace,
                            long long cap, long long* len) {
  if ((lattice != PERC_SQUARE && lattice != PERC_TRIANGULAR) || m < 2 || n < 2 || !len ||
      (kind != PERC_SITEBOND && kind != PERC_BONDSITE) || nsites < 0 || nbond < 0 ||
      (nsites && !site_order) || (nbond && !bond_order))
    return PERC_EINVAL;
  const Geom g = make_geom(lattice, m, n, pbc);
  std::vector<int> bf(g.t + 2, 0);
  for (int s = 1; s <= g.t + 1; ++s)
    bf[s] = bf[s - 1] + ((s - 1 >= 1 && s - 1 <= g.t - 1) ? forward_count(g, s - 1) : 0);
  if (nsites > g.t + 1 || nbond > bf[g.t + 1] + 1) return PERC_EINVAL;
  const long long nb = nbonds(g);
  std::vector<int> c(g.t + nb + 2, 0), sl(g.t, 0), bl(nb, 0), ev;
  int st[4] = {0, 0, 0, 0};
  const int rc = kind == PERC_SITEBOND
                     ? replay_sitebond(g, bf, site_order, nsites, bond_order, nbond, sl.data(),
                                       bl.data(), c.data(), (int)c.size(), st, &ev)
                     : replay_bondsite(g, bf, site_order, nsites, bond_order, nbond, sl.data(),
                                       bl.data(), c.data(), (int)c.size(), st, &ev);
  if (rc) return rc;
  *len = (long long)ev.size();
  if (!trace) return PERC_OK;
  if (cap < *len) return PERC_EINVAL;
  std::memcpy(trace, ev.data(), sizeof(int) * ev.size());
  return PERC_OK;
}

// the spanning cluster's Kirchhoff system (perc_conductance / perc_assemble)
static int assemble_impl(perc_ctx* h, int rule, double g0, double leak, double Va, const char* who) {
  hipError_t e = dev_assemble(h, rule, g0, leak, Va, h->span_root);
  if (e != hipSuccess) return hip_status(e, who);
  if (((h->fmt_req == PERC_FMT_STENCIL || h->fmt_req == PERC_FMT_STENCIL_TILED) && !h->tiled_ok) ||
      (h->fmt_req == PERC_FMT_STENCIL_SPLIT && !h->stencil_ok)) {
    set_error(std::string(who) + ": requested stencil operator not available for this system");
    return PERC_EINVAL;
  }
  h->assembled = true;
  h->rule = rule;
  return PERC_OK;
}

// terminal currents of the context's x -> Gtop, Gbot (bondc.f:554-592)
static int currents_impl(perc_ctx* h, int rule, int cur_rule, double Va, double g0, double leak,
                         perc_cond_result* res, const char* who);

int perc_conductance(perc_ctx* h, int rule, int cur_rule, double Va, double g0, double leak,
                     int itol, double tol, int itmax, perc_cond_result* res, double* vint_out) {
  if (!h || !res) return PERC_EINVAL;
  if (!h->labeled) return PERC_ESTATE;
  if (itol < 1 || itol > 4) {
    set_error("perc_conductance: illegal itol (1..4)");
    return PERC_EITOL;
  }
  if (rule < PERC_RULE_BOND || rule > PERC_RULE_MIXED || itmax < 0) return PERC_EINVAL;
  hipSetDevice(h->device);
  std::memset(res, 0, sizeof(*res));
  if (h->span_root == 0) {  // bond_cond.f:484-487: no spanning cluster -> G = 0
    res->status = 1;
    return PERC_OK;
  }
  hipStream_t st = h->stream;
  hipEventRecord(h->ev[0], st);
  int rc = assemble_impl(h, rule, g0, leak, Va, "perc_conductance/assemble");
  if (rc) return rc;
  hipEventRecord(h->ev[1], st);
  int iter = 0;
  double err = 0.0;
  hipError_t e = dev_solve(h, itol, tol, itmax, true, h->full_voltages || vint_out != nullptr, &iter, &err);
  if (e != hipSuccess) return hip_status(e, "perc_conductance/solve");
  hipEventRecord(h->ev[2], st);
  rc = currents_impl(h, rule, cur_rule, Va, g0, leak, res, "perc_conductance/currents");
  if (rc) return rc;
  res->iter = iter;
  res->err = err;
  res->t_assemble_ms = event_ms(h, 0, 1);
  res->t_solve_ms = event_ms(h, 1, 2);
  res->t_currents_ms = event_ms(h, 2, 3);
  if (vint_out) {
    e = hipMemcpy(vint_out, h->d.x, sizeof(double) * h->N, hipMemcpyDeviceToHost);
    if (e != hipSuccess) return hip_status(e, "perc_conductance/vint");
  }
  return PERC_OK;
}

static int currents_impl(perc_ctx* h, int rule, int cur_rule, double Va, double g0, double leak,
                         perc_cond_result* res, const char* who) {
  std::vector<double> iout(2 * (size_t)h->g.m);
  const double thresh = cur_rule == PERC_CUR_FORTRAN ? 1.0e-10 : 0.0;
  hipError_t e = dev_currents(h, rule, cur_rule, g0, leak, Va, h->span_root, thresh, iout.data());
  if (e != hipSuccess) return hip_status(e, who);
  hipEventRecord(h->ev[3], h->stream);
  hipEventSynchronize(h->ev[3]);
  const int m = h->g.m;
  double Ibot = 0.0, Itop = 0.0;
  if (cur_rule == PERC_CUR_FORTRAN) {  // bondc.f:587-590
    for (int i = 0; i < m; ++i) {
      Ibot = Ibot + iout[i];
      Itop = Itop + iout[m + i];
    }
  } else {  // ConductCalc.m:191-194
    for (int i = 0; i < m; ++i) {
      Ibot = iout[i] + Ibot;
      Itop = iout[2 * m - 1 - i] + Itop;
    }
  }
  res->gtop = Itop / Va;
  res->gbot = std::fabs(Ibot) / Va;
  return PERC_OK;
}

int perc_assemble(perc_ctx* h, int rule, double g0, double leak, double Va, int* spanning) {
  if (!h || !spanning) return PERC_EINVAL;
  if (!h->labeled) return PERC_ESTATE;
  if (rule < PERC_RULE_BOND || rule > PERC_RULE_MIXED) return PERC_EINVAL;
  hipSetDevice(h->device);
  *spanning = h->span_root != 0;
  if (!*spanning) return PERC_OK;
  return assemble_impl(h, rule, g0, leak, Va, "perc_assemble");
}

int perc_currents(perc_ctx* h, int rule, int cur_rule, double Va, double g0, double leak,
                  perc_cond_result* res) {
  if (!h || !res) return PERC_EINVAL;
  if (!h->assembled) return PERC_ESTATE;
  hipSetDevice(h->device);
  std::memset(res, 0, sizeof(*res));
  return currents_impl(h, rule, cur_rule, Va, g0, leak, res, "perc_currents");
}

int perc_dslab_begin(perc_ctx* h, int K, int s, int itol, double tol, int itmax, int full_x,
                     const perc_dslab_bufs* bufs) {
  if (!h || !bufs || itmax < 0) return PERC_EINVAL;
  if (!h->assembled) return PERC_ESTATE;
  if (itol != 1 && itol != 2) return PERC_EITOL;
  hipSetDevice(h->device);
  return hip_status(dev_dslab_begin(h, K, s, itol, tol, itmax, full_x != 0, *bufs), "perc_dslab_begin");
}

int perc_dslab_step(perc_ctx* h, int op) {
  if (!h || !h->dslab || op < PERC_DSLAB_COMBINE_INIT || op > PERC_DSLAB_GHOSTS) return PERC_EINVAL;
  hipSetDevice(h->device);
  return hip_status(dev_dslab_step(h, op), "perc_dslab_step");
}

int perc_dslab_status(perc_ctx* h, int* iter, double* err, int* done) {
  if (!h || !h->dslab || !iter || !err || !done) return PERC_EINVAL;
  hipSetDevice(h->device);
  return hip_status(dev_dslab_status(h, iter, err, done), "perc_dslab_status");
}

int perc_dslab_end(perc_ctx* h) {
  if (!h || !h->dslab) return PERC_EINVAL;
  hipSetDevice(h->device);
  return hip_status(dev_dslab_end(h, true), "perc_dslab_end");
}

int perc_x_row(perc_ctx* h, int row, double* dev_buf, int to_ctx) {
  if (!h || !dev_buf || row < 0 || row >= h->g.n - 2) return PERC_EINVAL;
  hipSetDevice(h->device);
  return hip_status(dev_x_row(h, row, dev_buf, to_ctx != 0), "perc_x_row");
}

void* perc_stream(perc_ctx* h) { return h ? (void*)h->stream : nullptr; }

int perc_get_system(perc_ctx* h, int* rowptr, int* col, double* val, double* diag, double* rhs,
                    int* n_out, int* nnz_out) {
  if (!h) return PERC_EINVAL;
  hipSetDevice(h->device);
  hipError_t e = ensure_csr(h);
  hipStreamSynchronize(h->stream);
  const size_t N = h->N, nnz = h->nnz;
  if (rowptr && e == hipSuccess) e = hipMemcpy(rowptr, h->d.rowptr, sizeof(int) * (N + 1), hipMemcpyDeviceToHost);
  if (col && e == hipSuccess) e = hipMemcpy(col, h->d.col, sizeof(int) * nnz, hipMemcpyDeviceToHost);
  if (val && e == hipSuccess) e = hipMemcpy(val, h->d.val, sizeof(double) * nnz, hipMemcpyDeviceToHost);
  if (diag && e == hipSuccess) e = hipMemcpy(diag, h->d.diag, sizeof(double) * N, hipMemcpyDeviceToHost);
  if (rhs && e == hipSuccess) e = hipMemcpy(rhs, h->d.rhs, sizeof(double) * N, hipMemcpyDeviceToHost);
  if (n_out) *n_out = (int)N;
  if (nnz_out) *nnz_out = (int)nnz;
  return hip_status(e, "perc_get_system");
}

int perc_spmv_host(perc_ctx* h, const double* x, double* y) {
  if (!h || !x || !y) return PERC_EINVAL;
  if (!h->assembled) return PERC_ESTATE;
  hipSetDevice(h->device);
  return hip_status(dev_spmv(h, x, y), "perc_spmv_host");
}

int perc_set_matrix_format(perc_ctx* h, int fmt) {
  if (!h || fmt < PERC_FMT_AUTO || fmt > PERC_FMT_STENCIL_TILED) return PERC_EINVAL;
  if (h->assembled && (fmt == PERC_FMT_STENCIL || fmt == PERC_FMT_STENCIL_TILED) && !h->tiled_ok)
    return PERC_EINVAL;
  if (h->assembled && fmt == PERC_FMT_STENCIL_SPLIT && !h->stencil_ok) return PERC_EINVAL;
  h->fmt_req = fmt;
  if (h->assembled) select_format(h);
  return PERC_OK;
}

int perc_set_full_voltages(perc_ctx* h, int enable) {
  if (!h) return PERC_EINVAL;
  h->full_voltages = enable != 0;
  return PERC_OK;
}

int perc_set_slabs(perc_ctx* h, int nslab) {
  if (!h || nslab < 1 || (h->g.n > 2 && nslab > h->g.n - 2)) return PERC_EINVAL;
  h->nslab = nslab;
  return PERC_OK;
}

int perc_set_march_rows(perc_ctx* h, int rows) {
  if (!h || rows < 0 || rows > 1024) return PERC_EINVAL;
  h->march_rows_req = rows;
  march_geometry(h);
  return PERC_OK;
}

int perc_set_march_mode(perc_ctx* h, int mode) {
  constexpr int kAll = PERC_MARCH_QFREE | PERC_MARCH_ALT | PERC_SOLVE_RESIDENT | PERC_MARCH_STRIPS |
                       PERC_MARCH_SLOTS | PERC_MARCH_TAG | PERC_MARCH_NIBBLE;
  if (!h || (mode & ~kAll) != 0) return PERC_EINVAL;
  h->march_mode = mode;
  march_geometry(h);  // band heights depend on PERC_MARCH_SLOTS
  if (h->assembled) select_format(h);
  return PERC_OK;
}

int perc_set_band_weights(perc_ctx* h, int which, int n, const int* w) {
  if (!h || n < 0 || n > 4 || (n && (!w || which < 0 || which > 2))) return PERC_EINVAL;
  for (int i = 0; i < n; ++i)
    if (w[i] <= 0) return PERC_EINVAL;
  if (n == 0) {
    h->slot_w_set = false;
  } else {
    if (!h->slot_w_set) {  // start from the defaults
      const int def[3][4] = {{100, 76, 48, 40}, {100, 78, 55, 50}, {100, 100, 100, 100}};  // (kSlotW)
      std::memcpy(h->slot_w, def, sizeof(def));
    }
    for (int i = 0; i < 4; ++i) h->slot_w[which][i] = i < n ? w[i] : h->slot_w[which][i];
    h->slot_w_set = true;
  }
  march_geometry(h);
  if (h->assembled) select_format(h);
  return PERC_OK;
}

int perc_set_dot_order(perc_ctx* h, int order) {
  if (!h || (order != PERC_DOT_FAST && order != PERC_DOT_LITERAL && order != PERC_DOT_LITERAL_HOST))
    return PERC_EINVAL;
  h->dot_order = order;
  if (h->assembled) select_format(h);
  return PERC_OK;
}

int perc_err_history(perc_ctx* h, double* out, int cap) {
  if (!h || cap < 0 || (cap && !out)) return PERC_EINVAL;
  if (!h->assembled) return PERC_ESTATE;
  CGScalars hs{};
  hipSetDevice(h->device);
  hipError_t e = hipMemcpy(&hs, h->d.scal, sizeof(hs), hipMemcpyDeviceToHost);
  if (e != hipSuccess) return hip_status(e, "perc_err_history");
  const int n = std::min(std::min(hs.iter, cap), h->d.err_hist_cap);
  if (n > 0 && h->d.err_hist) {
    e = hipMemcpy(out, h->d.err_hist, sizeof(double) * n, hipMemcpyDeviceToHost);
    if (e != hipSuccess) return hip_status(e, "perc_err_history");
  }
  return hs.iter;
}

int perc_set_bond_weights(perc_ctx* h, const double* w, long long n) {
  if (!h || (w && n != h->nb)) return PERC_EINVAL;
  hipSetDevice(h->device);
  return hip_status(dev_set_bond_weights(h, w), "perc_set_bond_weights");
}

// MT19937 (Matsumoto & Nishimura): init_genrand + genrand_int32, and the
// 53-bit doubles of genrand_res53 -- MATLAB's rand('twister', seed)
// (ConductCalc.m:38-47), also numpy.random.RandomState(seed).random_sample
namespace {
struct Twister {
  uint32_t mt[624];
  int mti = 625;
  explicit Twister(uint32_t seed) {
    mt[0] = seed;
    for (mti = 1; mti < 624; ++mti) mt[mti] = 1812433253u * (mt[mti - 1] ^ (mt[mti - 1] >> 30)) + (uint32_t)mti;
  }
  uint32_t next() {
    if (mti >= 624) {
      for (int k = 0; k < 624; ++k) {
        const uint32_t y = (mt[k] & 0x80000000u) | (mt[(k + 1) % 624] & 0x7fffffffu);
        mt[k] = mt[(k + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
      }
      mti = 0;
    }
    uint32_t y = mt[mti++];
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
  }
  double res53() {
    const uint32_t a = next() >> 5, b = next() >> 6;
    return (a * 67108864.0 + b) * (1.0 / 9007199254740992.0);
  }
};
}  // namespace

int perc_twister_uniform(unsigned int seed, long long n, double* out) {
  if (n < 0 || (n && !out)) return PERC_EINVAL;
  Twister t(seed);
  for (long long k = 0; k < n; ++k) out[k] = t.res53();
  return PERC_OK;
}

int perc_set_conductcalc_weights(perc_ctx* h, int rule, unsigned int seed) {
  if (!h || (rule != PERC_RULE_BOND && rule != PERC_RULE_SITE && rule != PERC_RULE_MIXED)) return PERC_EINVAL;
  if (!h->labeled) return PERC_ESTATE;
  hipSetDevice(h->device);
  if (!h->span_root) return hip_status(dev_set_bond_weights(h, nullptr), "perc_set_conductcalc_weights");
  std::vector<uint8_t> mask((size_t)h->nb);
  int rc = hip_status(dev_bond_mask(h, rule, mask.data()), "perc_set_conductcalc_weights");
  if (rc) return rc;
  std::vector<double> w((size_t)h->nb, 1.0);
  Twister t(seed);
  for (size_t id = 0; id < mask.size(); ++id)
    if (mask[id]) w[id] = t.res53();  // one rand per -g0 bond, bond-list order (ConductCalc.m:94-97)
  return hip_status(dev_set_bond_weights(h, w.data()), "perc_set_conductcalc_weights");
}

int perc_march_info(perc_ctx* h, int* out5) {
  if (!h || !out5) return PERC_EINVAL;
  if (!h->assembled) return PERC_ESTATE;
  out5[0] = h->small ? 4 : (h->resident && h->stencil ? 3 : (h->march ? 1 : 0));
  out5[1] = (h->qfree ? 1 : 0) | (h->strips ? 2 : 0) | (h->march_slots ? 8 : 0) |
            (h->march_tag ? 16 : 0) | (h->nib_used && out5[0] == 1 ? 32 : 0);
  out5[2] = h->march_alt ? 1 : 0;
  out5[3] = h->resident ? h->res_H : (h->march ? h->march_h : 0);
  out5[4] = h->resident ? h->g.m : (h->march ? 128 : 0);
  return PERC_OK;
}

int perc_last_solve(perc_ctx* h, int* out4) {
  if (!h || !out4) return PERC_EINVAL;
  if (h->last_iter < 0) return PERC_ESTATE;
  out4[0] = h->last_kernel;
  out4[1] = h->last_flags;
  out4[2] = h->last_iter;
  out4[3] = 0;
  return PERC_OK;
}

int perc_matrix_format(perc_ctx* h) {
  if (!h) return PERC_EINVAL;
  if (!h->assembled) return PERC_ESTATE;
  if (!h->stencil) return PERC_FMT_CSR;
  if (!h->fused) return PERC_FMT_STENCIL_SPLIT;
  return h->march ? PERC_FMT_STENCIL : PERC_FMT_STENCIL_TILED;
}

int perc_selftest_division(long long n, unsigned long long seed, unsigned long long* out3) {
  if (n < 0 || !out3) return PERC_EINVAL;
  return hip_status(dev_selftest_division(n, seed, out3), "perc_selftest_division");
}

int perc_bench_kernel(perc_ctx* h, int which, int reps, double* ms) {
  if (!h || !ms || reps <= 0 || which < 0 || which > 6) return PERC_EINVAL;
  if (!h->assembled && which != 4) return PERC_ESTATE;  // the copy needs no system
  hipSetDevice(h->device);
  // the CG kernels clobber the solver vectors (x, r, p, q), not the system
  return hip_status(dev_bench(h, which, reps, ms), "perc_bench_kernel");
}

int perc_bondc_realisation(perc_ctx* h, int tbonds, const int* bond_order, int on_device,
                           double Va, double g0, double tol, int itmax, perc_realisation* out) {
  if (!h || !out) return PERC_EINVAL;
  std::memset(out, 0, sizeof(*out));
  const double t0 = now_ms();
  int rc = occupy_impl(h, PERC_BOND, 0, nullptr, tbonds, bond_order, on_device != 0);
  if (rc) return rc;
  if (on_device) hipStreamSynchronize(h->stream);
  const double t1 = now_ms();
  rc = perc_label(h, &out->label, nullptr);
  if (rc) return rc;
  const double t2 = now_ms();
  rc = perc_conductance(h, PERC_RULE_BOND, PERC_CUR_FORTRAN, Va, g0, 1.0e-12, 2, tol, itmax,
                        &out->cond, nullptr);
  if (rc) return rc;
  const double t3 = now_ms();
  out->t_upload_ms = t1 - t0;
  out->t_label_ms = t2 - t1;
  out->t_total_ms = t3 - t0;
  return PERC_OK;
}

void perc_stats_accumulate(double* acc, int point, double g, int spanning, int iter) {
  double* a = acc + 5 * (size_t)point;
  a[0] += 1.0;
  a[1] += g;
  a[2] += g * g;
  a[3] += spanning ? 1.0 : 0.0;
  a[4] += iter;
}

}  // extern "C"
