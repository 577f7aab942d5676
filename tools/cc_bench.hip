// cc_bench.hip -- stand-alone A/B harness for the labeling kernels of
// percolation_amd/csrc/perc_cc.h: one L x L square-lattice bond occupancy
// (p, a fixed hash), the production k_cc_tile / k_cc_merge / k_cc_compress
// timed with HIP events, and candidate tile kernels defined here checked
// against the production tile kernel's output (parent and member arrays,
// element by element) before they are timed.
//
//   make -C tools cc_bench && ./tools/cc_bench 4096 0.6 20
#include "perc_cc.h"

#include <cstdio>
#include <cstdlib>
#include <type_traits>
#include <vector>

using namespace perc;

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(2);                                                                \
    }                                                                              \
  } while (0)

namespace {

unsigned hash32(unsigned long long x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return (unsigned)x;
}

struct Run {
  Geom g;
  int *bf, *parent, *parent_ref;
  uint8_t *bocc, *socc, *member, *member_ref;
  int* counters;
  int tiles;
};

template <typename F>
double time_ms(F f, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  f();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a, 0));
  for (int i = 0; i < reps; ++i) f();
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return ms / reps;
}

bool same(const Run& R, const char* what) {
  const size_t t = (size_t)R.g.t + 2;
  std::vector<int> p(t), q(t);
  std::vector<uint8_t> m(t), n(t);
  CK(hipMemcpy(p.data(), R.parent, t * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(q.data(), R.parent_ref, t * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(m.data(), R.member, t, hipMemcpyDeviceToHost));
  CK(hipMemcpy(n.data(), R.member_ref, t, hipMemcpyDeviceToHost));
  long long bad = 0, first = -1;
  for (size_t s = 1; s <= (size_t)R.g.t; ++s)
    if (p[s] != q[s] || m[s] != n[s]) {
      if (first < 0) first = (long long)s;
      ++bad;
    }
  std::printf("  %-28s %s", what, bad ? "MISMATCH" : "matches the production tile kernel");
  if (bad) std::printf(" (%lld sites, first %lld: parent %d vs %d, member %d vs %d)", bad, first, p[first],
                       q[first], m[first], n[first]);
  std::printf("\n");
  return bad == 0;
}


// Candidate: one wave per tile, rows walked bottom to top.  Lane l owns the
// tile's columns l and l + 64.  Per row: the row's links (right, up), its
// horizontal runs by ballots (a run's node = its first site), the vertical
// links down into the previous row united in an LDS union-find over run
// nodes (larger root -> smaller, so a root is its component's minimum site;
// a lane whose (run, run below) pair equals the column to its left skips
// its union), the run node written as the provisional parent; a last pass
// writes every site's root.  Square lattice, no pbc; kind as cc_link (bond:
// member = any incident occupied bond; site / mixed: the occupied site).
template <int H>
__global__ __launch_bounds__(64) void k_cc_tile_w(Geom g, int kind, const int* bond_first, const uint8_t* bocc,
                                                  const uint8_t* socc, int* parent, uint8_t* member,
                                                  int bf_closed) {
  __shared__ int uf[kCcW * H];
  const int ntx = cdiv(g.m, kCcW);
  const int tb = xcd_logical_block(blockIdx.x, gridDim.x);
  const int tx = tb % ntx, ty = tb / ntx;
  const int c0 = tx * kCcW, r0 = ty * H;
  const int tw = min(kCcW, g.m - c0), th = min(H, g.n - r0);
  const int lane = threadIdx.x;
  // R / U: the link right / up of each of the lane's two sites; O: the site occupied (site kinds)
  auto load_row = [&](int r, unsigned (&R)[2], unsigned (&U)[2], unsigned (&O)[2]) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int lc = lane + 64 * h, col = c0 + lc, row = r0 + r;
      const bool v = lc < tw && r < th;
      const int s = row * g.m + col + 1;
      const bool hr = v && col < g.m - 1, hu = v && row < g.n - 1;
      if (kind == PERC_SITE) {
        const unsigned o = v ? socc[s] : 0u;
        O[h] = o;
        R[h] = o && hr ? socc[s + 1] : 0u;
        U[h] = o && hu ? socc[s + g.m] : 0u;
        continue;
      }
      const int fb = !v ? 0 : bf_closed && row <= g.n - 2 ? bf_square(g, row, col) : bond_first[s];
      R[h] = hr ? bocc[fb] : 0u;
      U[h] = hu ? bocc[fb + (col < g.m - 1 ? 1 : 0)] : 0u;
      O[h] = 1u;
      if (kind != PERC_BOND) {  // mixed: the bond and both sites
        const unsigned o = v ? socc[s] : 0u;
        O[h] = o;
        R[h] = R[h] && o && socc[s + 1];
        U[h] = U[h] && o && socc[s + g.m];
      }
    }
  };
  unsigned R[2], U[2], O[2], Rn[2], Un[2], On[2], Up[2] = {0u, 0u};
  int labp[2] = {0, 0};
  load_row(0, R, U, O);
  const unsigned long long le = lane == 63 ? ~0ull : ((2ull << lane) - 1ull);
  for (int r = 0; r < th; ++r) {
    load_row(r + 1, Rn, Un, On);  // (past th: nothing loaded)
    // runs: column c has a left link iff c - 1 links right
    const unsigned rl0 = __shfl(R[0], (lane + 63) & 63, 64), rl1 = __shfl(R[1], (lane + 63) & 63, 64);
    const bool left0 = lane > 0 && rl0, left1 = lane > 0 ? rl1 != 0u : rl0 != 0u;  // (lane 0, half 1: column 63)
    const bool v0 = lane < tw, v1 = lane + 64 < tw;
    const unsigned long long lo = __ballot(!left0 || !v0), hi = __ballot(!left1 || !v1);
    int node[2];
    node[0] = r * kCcW + 63 - __clzll((long long)(lo & le));
    const unsigned long long hm = hi & le;
    node[1] = r * kCcW + (hm ? 64 + 63 - __clzll((long long)hm) : 63 - __clzll((long long)lo));
    if (v0 && !left0) uf[node[0]] = node[0];
    if (v1 && !left1) uf[node[1]] = node[1];
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // vertical links down into row r - 1 (that row's up links)
    const bool w0 = r > 0 && v0 && Up[0], w1 = r > 0 && v1 && Up[1];
    const int a0 = w0 ? node[0] : -1, b0 = w0 ? labp[0] : -1, a1 = w1 ? node[1] : -1, b1 = w1 ? labp[1] : -1;
    const int pa0 = __shfl(a0, (lane + 63) & 63, 64), pb0 = __shfl(b0, (lane + 63) & 63, 64);
    const int pa1 = __shfl(a1, (lane + 63) & 63, 64), pb1 = __shfl(b1, (lane + 63) & 63, 64);
    const bool sk0 = lane > 0 && pa0 == a0 && pb0 == b0;
    const bool sk1 = lane > 0 ? (pa1 == a1 && pb1 == b1) : (pa0 == a1 && pb0 == b1);
    // (lane 0, half 1: the column to the left is column 63 = lane 63, half 0: its pa0/pb0 came
    // from lane 63 through the same shuffle)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const bool w = h ? w1 && !sk1 : w0 && !sk0;
      if (!w) continue;
      int a = h ? a1 : a0, b = h ? b1 : b0;
      while (true) {
        a = find_root(uf, a);
        b = find_root(uf, b);
        if (a == b) break;
        if (a < b) { const int t = a; a = b; b = t; }
        const int old = atomicCAS(&uf[a], a, b);
        if (old == a) break;
        a = old;
      }
    }
    // provisional parents (run nodes) and member flags
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const bool v = h ? v1 : v0;
      if (!v) continue;
      const int lc = lane + 64 * h, s = (r0 + r) * g.m + c0 + lc + 1;
      const bool lft = h ? left1 : left0;
      parent[s] = node[h];
      member[s] = kind == PERC_BOND ? ((R[h] | U[h] | (lft ? 1u : 0u) | (r > 0 ? Up[h] : 0u)) ? 1 : 0)
                                    : (O[h] ? 1 : 0);
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      labp[h] = node[h];
      Up[h] = U[h];
      R[h] = Rn[h];
      U[h] = Un[h];
      O[h] = On[h];
    }
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  for (int r = 0; r < th; ++r) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int lc = lane + 64 * h;
      if (lc >= tw) continue;
      const int s = (r0 + r) * g.m + c0 + lc + 1;
      int x = parent[s], p = uf[x];
      while (p != x) {
        x = p;
        p = uf[x];
      }
      parent[s] = (r0 + x / kCcW) * g.m + c0 + x % kCcW + 1;
    }
  }
}

}  // namespace

int main(int argc, char** argv) {
  const int L = argc > 1 ? std::atoi(argv[1]) : 4096;
  const double p = argc > 2 ? std::atof(argv[2]) : 0.6;
  const int reps = argc > 3 ? std::atoi(argv[3]) : 20;
  Run R;
  R.g = make_geom(kSquare, L, L, 0);
  const Geom& g = R.g;
  const long long nb = nbonds(g);
  std::vector<int> bf((size_t)g.t + 2, 0);
  long long acc = 0;
  for (int s = 0; s <= g.t + 1; ++s) {
    bf[s] = (int)acc;
    acc += (s >= 1 && s <= g.t - 1) ? forward_count(g, s) : 0;
  }
  std::vector<uint8_t> occ((size_t)nb + 8, 0);
  const unsigned thr = (unsigned)(p * 4294967296.0);
  long long nocc = 0;
  for (long long b = 0; b < nb; ++b) {
    occ[b] = hash32((unsigned long long)b * 0x9E3779B97F4A7C15ull + 12345) < thr;
    nocc += occ[b];
  }
  CK(hipMalloc(&R.bf, bf.size() * 4));
  CK(hipMemcpy(R.bf, bf.data(), bf.size() * 4, hipMemcpyHostToDevice));
  CK(hipMalloc(&R.bocc, occ.size()));
  CK(hipMemcpy(R.bocc, occ.data(), occ.size(), hipMemcpyHostToDevice));
  CK(hipMalloc(&R.socc, (size_t)g.t + 2));
  CK(hipMemset(R.socc, 1, (size_t)g.t + 2));
  for (int** q : {&R.parent, &R.parent_ref}) CK(hipMalloc(q, ((size_t)g.t + 2) * 4));
  for (uint8_t** q : {&R.member, &R.member_ref}) CK(hipMalloc(q, (size_t)g.t + 2));
  CK(hipMalloc(&R.counters, 64));
  R.tiles = cdiv(g.m, kCcW) * cdiv(g.n, kCcH);
  std::printf("L = %d, p = %.3f: %lld of %lld bonds occupied, %d tiles of %d x %d\n", L, p, nocc, nb, R.tiles,
              kCcW, kCcH);
  auto tile = [&](int* par, uint8_t* mem) {
    k_cc_tile<<<R.tiles, kCcThreads>>>(g, PERC_BOND, R.bf, R.bocc, R.socc, par, mem, 1, nullptr);
  };
  // the production tile kernel vs a candidate of the same block height, element by element
  tile(R.parent_ref, R.member_ref);
  CK(hipDeviceSynchronize());
  const double t_tile = time_ms([&]() { tile(R.parent, R.member); }, reps);
  same(R, "k_cc_tile (production)");
  auto tw32 = [&]() { k_cc_tile_w<kCcH><<<R.tiles, 64>>>(g, PERC_BOND, R.bf, R.bocc, R.socc, R.parent, R.member, 1); };
  CK(hipMemset(R.parent, 0, ((size_t)g.t + 2) * 4));
  tw32();
  CK(hipDeviceSynchronize());
  if (same(R, "k_cc_tile_w (same blocks)"))
    std::printf("  tile: production %.1f us, k_cc_tile_w %.1f us\n", t_tile * 1e3, time_ms(tw32, reps) * 1e3);
  // whole chains (tile, merge, compress): the final parents are the partition's
  // minimum sites whatever the blocks, so chains of other block heights compare too
  hipEvent_t e[4];
  for (auto& x : e) CK(hipEventCreate(&x));
  auto chain = [&](const char* what, auto tilef, auto mergef, bool ref) {
    double t[3] = {0, 0, 0};
    for (int i = 0; i < reps; ++i) {
      CK(hipEventRecord(e[0], 0));
      tilef();
      CK(hipEventRecord(e[1], 0));
      mergef();
      CK(hipEventRecord(e[2], 0));
      k_cc_compress<<<std::min(cdiv(g.t, kCcThreads), 1024), kCcThreads>>>(g.t, R.parent, R.member, R.counters);
      CK(hipEventRecord(e[3], 0));
      CK(hipEventSynchronize(e[3]));
      for (int k = 0; k < 3; ++k) {
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e[k], e[k + 1]));
        t[k] += ms * 1e3 / reps;
      }
    }
    if (ref) {
      CK(hipMemcpy(R.parent_ref, R.parent, ((size_t)g.t + 2) * 4, hipMemcpyDeviceToDevice));
      CK(hipMemcpy(R.member_ref, R.member, (size_t)g.t + 2, hipMemcpyDeviceToDevice));
      std::printf("  chain %-24s tile %.1f + merge %.1f + compress %.1f = %.1f us\n", what, t[0], t[1], t[2],
                  t[0] + t[1] + t[2]);
    } else if (same(R, what)) {
      std::printf("  chain %-24s tile %.1f + merge %.1f + compress %.1f = %.1f us\n", what, t[0], t[1], t[2],
                  t[0] + t[1] + t[2]);
    }
  };
  auto merge_for = [&](auto hconst) {
    constexpr int H = decltype(hconst)::value;
    const int nseg = cdiv(g.m, kCcThreads), nfull = g.n / H, ncand = 2 * cdiv(g.m, kCcW) + 1;
    return [&, nseg, nfull, ncand]() {
      k_cc_merge<H><<<nfull * nseg + ncand * cdiv(g.n, kCcThreads), kCcThreads>>>(
          g, PERC_BOND, R.bf, R.bocc, R.socc, R.parent, R.member, nseg, nfull);
    };
  };
  chain("production", [&]() { tile(R.parent, R.member); }, merge_for(std::integral_constant<int, kCcH>{}), true);
  chain("tile_w<32>", [&]() { k_cc_tile_w<32><<<cdiv(g.m, kCcW) * cdiv(g.n, 32), 64>>>(g, PERC_BOND, R.bf, R.bocc, R.socc,
                                                                                       R.parent, R.member, 1); },
        merge_for(std::integral_constant<int, 32>{}), false);
  chain("tile_w<16>", [&]() { k_cc_tile_w<16><<<cdiv(g.m, kCcW) * cdiv(g.n, 16), 64>>>(g, PERC_BOND, R.bf, R.bocc, R.socc,
                                                                                       R.parent, R.member, 1); },
        merge_for(std::integral_constant<int, 16>{}), false);
  chain("tile_w<64>", [&]() { k_cc_tile_w<64><<<cdiv(g.m, kCcW) * cdiv(g.n, 64), 64>>>(g, PERC_BOND, R.bf, R.bocc, R.socc,
                                                                                       R.parent, R.member, 1); },
        merge_for(std::integral_constant<int, 64>{}), false);
  // site and mixed kinds (sites occupied at 0.8 by another hash): the production tile kernel vs the candidate
  {
    std::vector<uint8_t> so((size_t)g.t + 2, 0);
    for (int st = 1; st <= g.t; ++st) so[st] = hash32((unsigned long long)st * 0xD1B54A32D192ED03ull + 777) < 0xCCCCCCCCu;
    CK(hipMemcpy(R.socc, so.data(), so.size(), hipMemcpyHostToDevice));
    for (int kind : {PERC_SITE, PERC_SITEBOND}) {
      k_cc_tile<<<R.tiles, kCcThreads>>>(g, kind, R.bf, R.bocc, R.socc, R.parent_ref, R.member_ref, 1, nullptr);
      k_cc_tile_w<kCcH><<<R.tiles, 64>>>(g, kind, R.bf, R.bocc, R.socc, R.parent, R.member, 1);
      CK(hipDeviceSynchronize());
      same(R, kind == PERC_SITE ? "k_cc_tile_w, site kind" : "k_cc_tile_w, mixed kind");
    }
  }
  return 0;
}
