// cc_bench.hip -- stand-alone A/B harness for the labeling kernels of
// percolation_amd/csrc/perc_cc.h: one L x L square-lattice bond occupancy
// (p, a fixed hash): the LDS union-find tiles (k_cc_tile, the triangular
// and pbc lattices' labeling), the wave tiles (k_cc_tile_w, the open square
// lattice's) at several shapes and the merge / compress variants, timed
// with HIP events phase by phase; every chain's final parents and members
// checked element by element against the LDS union-find chain's.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -Iinclude -Ipercolation_amd/csrc \
//     tools/cc_bench.hip -o tools/cc_bench && ./tools/cc_bench 4096 0.6 20
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
  // the wave tiles at the production kernel's block height, element by element
  auto tw32 = [&]() {
    k_cc_tile_w<kCcH, PERC_BOND><<<R.tiles, 64>>>(g, R.bocc, R.socc, R.parent, R.member, (unsigned)nb + 8u);
  };
  CK(hipMemset(R.parent, 0, ((size_t)g.t + 2) * 4));
  tw32();
  CK(hipDeviceSynchronize());
  if (same(R, "k_cc_tile_w (same blocks)"))
    std::printf("  tile: LDS union-find %.1f us, k_cc_tile_w %.1f us\n", t_tile * 1e3, time_ms(tw32, reps) * 1e3);
  // whole chains (tile, merge, compress): the final parents are the partition's
  // minimum sites whatever the blocks, so chains of other block heights compare too
  hipEvent_t e[4];
  for (auto& x : e) CK(hipEventCreate(&x));
  auto compress0 = [&]() {
    k_cc_compress<<<std::min(cdiv(g.t, kCcThreads * kCcCompressU), kReduceGrid), kCcThreads>>>(
        g.t, R.parent, R.member, 0, R.counters);
  };
  auto chain_c = [&](const char* what, auto tilef, auto mergef, auto compressf, bool ref) {
    double t[3] = {0, 0, 0};
    for (int i = 0; i < reps; ++i) {
      CK(hipEventRecord(e[0], 0));
      tilef();
      CK(hipEventRecord(e[1], 0));
      mergef();
      CK(hipEventRecord(e[2], 0));
      compressf();
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
  auto chain = [&](const char* what, auto tilef, auto mergef, bool ref) { chain_c(what, tilef, mergef, compress0, ref); };
  auto merge_for = [&](auto hconst) {
    constexpr int H = decltype(hconst)::value;
    const int nseg = cdiv(g.m, kCcThreads), nfull = g.n / H, ncand = 2 * cdiv(g.m, kCcW) + 1;
    return [&, nseg, nfull, ncand]() {
      k_cc_merge<H><<<nfull * nseg + ncand * cdiv(g.n, kCcThreads), kCcThreads>>>(
          g, PERC_BOND, R.bf, R.bocc, R.socc, R.parent, R.member, nseg, nfull);
    };
  };
  chain("LDS union-find 128 x 32", [&]() { tile(R.parent, R.member); }, merge_for(std::integral_constant<int, kCcH>{}),
        true);
  auto wave = [&](auto hconst, auto dconst) {
    constexpr int H = decltype(hconst)::value, D = decltype(dconst)::value;
    return [&]() {
      k_cc_tile_w<H, PERC_BOND, D><<<cdiv(g.m, kCcW) * cdiv(g.n, H), 64>>>(g, R.bocc, R.socc, R.parent, R.member,
                                                                          (unsigned)nb + 8u);
    };
  };
  using I16 = std::integral_constant<int, 16>;
  chain("wave 128 x 16 (production)", wave(I16{}, std::integral_constant<int, 2>{}), merge_for(I16{}), false);
  {
    const int nseg = cdiv(g.m, kCcThreads), nfull = g.n / 16, ntx = cdiv(g.m, kCcW);
    const int GMs = nfull * nseg + (ntx - 1) * cdiv(g.n, kCcThreads);
    chain("wave 16 + square merge", wave(I16{}, std::integral_constant<int, 2>{}), [&, nseg, nfull, GMs]() {
      k_cc_merge_sq<16, PERC_BOND><<<GMs, kCcThreads>>>(g, R.bocc, R.socc, R.parent, R.member, nseg, nfull, nullptr);
    }, false);
  }
  chain("wave 16, ballots", [&]() {
    k_cc_tile_w<16, PERC_BOND, 2, true><<<cdiv(g.m, kCcW) * cdiv(g.n, 16), 64>>>(g, R.bocc, R.socc, R.parent,
                                                                                 R.member, (unsigned)nb + 8u);
  }, merge_for(I16{}), false);
  chain("wave 128 x 16, 4 rows in flight", wave(I16{}, std::integral_constant<int, 4>{}), merge_for(I16{}), false);
  // the merge's unions deduplicated only against the previous lane (WD = false)
  {
    const int nseg = cdiv(g.m, kCcThreads), nfull = g.n / 16, ncand = 2 * cdiv(g.m, kCcW) + 1;
    chain("wave 16 + merge lane-pair dedup", wave(I16{}, std::integral_constant<int, 2>{}),
          [&, nseg, nfull, ncand]() { k_cc_merge<16, false><<<nfull * nseg + ncand * cdiv(g.n, kCcThreads), kCcThreads>>>(
                                          g, PERC_BOND, R.bf, R.bocc, R.socc, R.parent, R.member, nseg, nfull); }, false);
  }
  // compress: U sites per thread chased in lockstep (production: kCcCompressU), one site per thread
  chain_c("wave 16 + compress<1>", wave(I16{}, std::integral_constant<int, 2>{}), merge_for(I16{}),
          [&]() { k_cc_compress<1><<<std::min(cdiv(g.t, kCcThreads), kReduceGrid), kCcThreads>>>(
                      g.t, R.parent, R.member, 0, R.counters); }, false);
  chain_c("wave 16 + compress<4>", wave(I16{}, std::integral_constant<int, 2>{}), merge_for(I16{}),
          [&]() { k_cc_compress<4><<<std::min(cdiv(g.t, kCcThreads * 4), kReduceGrid), kCcThreads>>>(
                      g.t, R.parent, R.member, 0, R.counters); }, false);
  // site and mixed kinds (sites occupied at 0.8 by another hash): the production tile kernel vs the candidate
  {
    std::vector<uint8_t> so((size_t)g.t + 2, 0);
    for (int st = 1; st <= g.t; ++st) so[st] = hash32((unsigned long long)st * 0xD1B54A32D192ED03ull + 777) < 0xCCCCCCCCu;
    CK(hipMemcpy(R.socc, so.data(), so.size(), hipMemcpyHostToDevice));
    // the 16-row wave tiles of each kind (the production; ballots), element
    // by element against the production tile and timed alone
    const int G16 = cdiv(g.m, kCcW) * cdiv(g.n, 16);
    auto wk = [&](auto kc, auto wl) {
      constexpr int K = decltype(kc)::value;
      constexpr bool W = decltype(wl)::value;
      return [&, G16]() {
        k_cc_tile_w<16, K, 2, W><<<G16, 64>>>(g, R.bocc, R.socc, R.parent, R.member, (unsigned)nb + 8u);
      };
    };
    using KS = std::integral_constant<int, PERC_SITE>;
    using KM = std::integral_constant<int, PERC_SITEBOND>;
    using WF = std::false_type;
    using WT = std::true_type;
    for (int kind : {PERC_SITE, PERC_SITEBOND}) {
      k_cc_tile<<<R.tiles, kCcThreads>>>(g, kind, R.bf, R.bocc, R.socc, R.parent_ref, R.member_ref, 1, nullptr);
      if (kind == PERC_SITE)
        k_cc_tile_w<kCcH, PERC_SITE><<<R.tiles, 64>>>(g, R.bocc, R.socc, R.parent, R.member, (unsigned)nb + 8u);
      else
        k_cc_tile_w<kCcH, PERC_SITEBOND><<<R.tiles, 64>>>(g, R.bocc, R.socc, R.parent, R.member, (unsigned)nb + 8u);
      CK(hipDeviceSynchronize());
      same(R, kind == PERC_SITE ? "k_cc_tile_w, site kind" : "k_cc_tile_w, mixed kind");
      // 16-row references: the production wave tile of that height
      if (kind == PERC_SITE) wk(KS{}, WF{})();
      else wk(KM{}, WF{})();
      CK(hipDeviceSynchronize());
      CK(hipMemcpy(R.parent_ref, R.parent, ((size_t)g.t + 2) * 4, hipMemcpyDeviceToDevice));
      CK(hipMemcpy(R.member_ref, R.member, (size_t)g.t + 2, hipMemcpyDeviceToDevice));
      const double tb = kind == PERC_SITE ? time_ms(wk(KS{}, WF{}), reps) : time_ms(wk(KM{}, WF{}), reps);
      CK(hipMemset(R.parent, 0, ((size_t)g.t + 2) * 4));
      const double tw = kind == PERC_SITE ? time_ms(wk(KS{}, WT{}), reps) : time_ms(wk(KM{}, WT{}), reps);
      if (same(R, kind == PERC_SITE ? "wave 16 ballots, site" : "wave 16 ballots, mixed"))
        std::printf("  tile 16 rows, %s kind: production %.1f us, ballots %.1f us\n",
                    kind == PERC_SITE ? "site" : "mixed", tb * 1e3, tw * 1e3);
      // the merges of that kind after the ballot tile: the generic one, then
      // the square lattice's (k_cc_merge_sq), whole chains compared
      const int nseg = cdiv(g.m, kCcThreads), nfull = g.n / 16, ntx = cdiv(g.m, kCcW);
      const int GMg = nfull * nseg + (2 * ntx + 1) * cdiv(g.n, kCcThreads);
      const int GMs = nfull * nseg + (ntx - 1) * cdiv(g.n, kCcThreads);
      auto tilek = [&]() {
        if (kind == PERC_SITE) wk(KS{}, WT{})();
        else wk(KM{}, WT{})();
      };
      auto mgen = [&]() {
        k_cc_merge<16><<<GMg, kCcThreads>>>(g, kind, R.bf, R.bocc, R.socc, R.parent, R.member, nseg, nfull);
      };
      auto msq = [&]() {
        if (kind == PERC_SITE)
          k_cc_merge_sq<16, PERC_SITE><<<GMs, kCcThreads>>>(g, R.bocc, R.socc, R.parent, R.member, nseg, nfull,
                                                             nullptr);
        else
          k_cc_merge_sq<16, PERC_SITEBOND><<<GMs, kCcThreads>>>(g, R.bocc, R.socc, R.parent, R.member, nseg,
                                                                 nfull, nullptr);
      };
      chain(kind == PERC_SITE ? "site: generic merge" : "mixed: generic merge", tilek, mgen, true);
      chain(kind == PERC_SITE ? "site: square merge" : "mixed: square merge", tilek, msq, false);
      // tile height (16 in production) against 8 and 32: the merge's
      // block-top rows scale as 1/H, the tile's per-row work does not
      auto by_h = [&](auto hconst, const char* what) {
        constexpr int HH = decltype(hconst)::value;
        const int GH = cdiv(g.m, kCcW) * cdiv(g.n, HH), nfh = g.n / HH;
        const int GMh = nfh * nseg + (ntx - 1) * cdiv(g.n, kCcThreads);
        chain(what, [&, GH]() {
          if (kind == PERC_SITE)
            k_cc_tile_w<HH, PERC_SITE, 2, true><<<GH, 64>>>(g, R.bocc, R.socc, R.parent, R.member, (unsigned)nb + 8u);
          else
            k_cc_tile_w<HH, PERC_SITEBOND, 2, true><<<GH, 64>>>(g, R.bocc, R.socc, R.parent, R.member,
                                                                (unsigned)nb + 8u);
        }, [&, nfh, GMh]() {
          if (kind == PERC_SITE)
            k_cc_merge_sq<HH, PERC_SITE><<<GMh, kCcThreads>>>(g, R.bocc, R.socc, R.parent, R.member, nseg, nfh,
                                                               nullptr);
          else
            k_cc_merge_sq<HH, PERC_SITEBOND><<<GMh, kCcThreads>>>(g, R.bocc, R.socc, R.parent, R.member, nseg,
                                                                   nfh, nullptr);
        }, false);
      };
      by_h(std::integral_constant<int, 8>{}, kind == PERC_SITE ? "site: 8-row tiles" : "mixed: 8-row tiles");
      by_h(std::integral_constant<int, 32>{}, kind == PERC_SITE ? "site: 32-row tiles" : "mixed: 32-row tiles");
    }
  }
  // rows in flight (the ring depth D) of the 16-row wave tiles, each kind:
  // element by element against D = 2 and timed alone (socc as above: sites
  // 0.8; the bond kind ignores it)
  {
    const int G16 = cdiv(g.m, kCcW) * cdiv(g.n, 16);
    auto tk = [&](auto kc, auto dc) {
      constexpr int K = decltype(kc)::value, D = decltype(dc)::value;
      return [&, G16]() {
        k_cc_tile_w<16, K, D, K != PERC_BOND><<<G16, 64>>>(g, R.bocc, R.socc, R.parent, R.member, (unsigned)nb + 8u);
      };
    };
    auto depth = [&](auto kc, const char* what) {
      using D2 = std::integral_constant<int, 2>;
      using D3 = std::integral_constant<int, 3>;
      using D4 = std::integral_constant<int, 4>;
      tk(kc, D2{})();
      CK(hipDeviceSynchronize());
      CK(hipMemcpy(R.parent_ref, R.parent, ((size_t)g.t + 2) * 4, hipMemcpyDeviceToDevice));
      CK(hipMemcpy(R.member_ref, R.member, (size_t)g.t + 2, hipMemcpyDeviceToDevice));
      double t[3];
      t[0] = time_ms(tk(kc, D2{}), reps);
      bool ok = true;
      CK(hipMemset(R.parent, 0, ((size_t)g.t + 2) * 4));
      t[1] = time_ms(tk(kc, D3{}), reps);
      ok = same(R, "D 3") && ok;
      CK(hipMemset(R.parent, 0, ((size_t)g.t + 2) * 4));
      t[2] = time_ms(tk(kc, D4{}), reps);
      ok = same(R, "D 4") && ok;
      // (again, interleaved: D 2, 4)
      const double t2b = time_ms(tk(kc, D2{}), reps), t4b = time_ms(tk(kc, D4{}), reps);
      std::printf("  tile depth, %s kind: D 2 %.1f / %.1f us, D 3 %.1f us, D 4 %.1f / %.1f us%s\n", what,
                  t[0] * 1e3, t2b * 1e3, t[1] * 1e3, t[2] * 1e3, t4b * 1e3, ok ? "" : " (MISMATCH)");
    };
    depth(std::integral_constant<int, PERC_BOND>{}, "bond");
    depth(std::integral_constant<int, PERC_SITE>{}, "site");
    depth(std::integral_constant<int, PERC_SITEBOND>{}, "mixed");
  }
  return 0;
}
