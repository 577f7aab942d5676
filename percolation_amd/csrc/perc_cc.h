// perc_cc.h -- the connected-component labeling kernels of libperc
// (k_cc_tile, k_cc_merge, k_cc_compress), included by perc_label.hip and by
// tools/cc_bench.hip (the kernels' stand-alone A/B harness).  Definitions in
// an anonymous namespace, like the other device headers.
#pragma once
#include "perc_common.h"

#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Wunused-function"
namespace perc {
namespace {

__device__ __forceinline__ int wave_sum_int(int v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// ---------------------------------------------------------------------------
// Connected components (the partition of bondc.f:194-393, site.f:167-289,
// sitebond.f:190-400).  Roots are always linked larger -> smaller, so the
// final root of a component is its minimum site id: a canonical,
// schedule-independent partition.  Three passes:
//
//  k_cc_tile      one workgroup per kCcW x kCcH block of sites.  The links
//                 inside the block are united in an LDS union-find (local
//                 index order = site order inside a block, so the local root
//                 is the block-local minimum site); then every site's parent
//                 (that root's global id) and member flag are written once,
//                 coalesced.  No global atomics.
//  k_cc_merge     only the links that cross a block edge (sites on the top
//                 row or the edge columns of a block: ~1/32 + 2/128 of them)
//                 are united in the global array (lock-free CAS, same rule;
//                 neighbouring lanes with the same pair of parents unite once).
//  k_cc_compress  parent[s] = final root; cluster count reduced per
//                 workgroup (one atomic per workgroup of a fixed grid).
//
// Path halving (LDS and global): stale reads only cost retries, parents only
// ever move to smaller ancestors, and only roots are CASed.
#ifndef PERC_CC_H
#define PERC_CC_H 32  // tile height (probe builds: -DPERC_CC_H=64)
#endif
constexpr int kCcW = 128, kCcH = PERC_CC_H, kCcSites = kCcW * kCcH, kCcThreads = 256;
constexpr int kReduceGrid = 1024;  // fixed grid of the counting passes
constexpr int kCcWaveH = 16;       // block height of k_cc_tile_w (the open square lattice)
// rows whose loads the bond kind's k_cc_tile_w keeps in flight: 3 -- tile
// 92.6 vs 114.8 (D = 2) and 116 us (D = 4) at L = 4096, 292.7 vs 322.6 /
// 328.5 at 8192 (profiles/r6_31_cc_depth.txt); labels per realisation at
// L = 4096 0.2467 vs 0.2664 ms (r6_32).  The site and mixed kinds keep D = 2
// (D = 3 within 1 %: config 5's labels 0.332 vs 0.329 ms).  PERC_CC_TILE_D:
// A/B probe builds only
// sites per thread of the square lattice's merge (k_cc_merge_squ; 0: one
// per thread, k_cc_merge_sq -- PERC_MERGE_U, A/B probe builds only): 2 --
// config 5's labels 0.3188 vs 0.3287 ms (one per thread), L = 4096 bond
// 0.2395 vs 0.2412; 4: 0.332 / 0.271 (profiles/r6_35_*)
#ifdef PERC_MERGE_U
constexpr int kMergeU = PERC_MERGE_U;
#else
constexpr int kMergeU = 2;
#endif
#ifdef PERC_CC_TILE_D
constexpr int kCcWaveDBond = PERC_CC_TILE_D;
#else
constexpr int kCcWaveDBond = 3;
#endif


__device__ __forceinline__ int find_root(int* parent, int x) {
  int p = parent[x];
  while (p != x) {
    const int gp = parent[p];
    if (gp != p) parent[x] = gp;
    x = gp;
    p = parent[x];
  }
  return x;
}

// true when this call joined two sets (its CAS hooked a root): the
// successful hooks of a pass count the components it merged
__device__ __forceinline__ bool unite(int* parent, int a, int b) {
  while (true) {
    a = find_root(parent, a);
    b = find_root(parent, b);
    if (a == b) return false;
    if (a < b) { const int tmp = a; a = b; b = tmp; }
    const int old = atomicCAS(&parent[a], a, b);
    if (old == a) return true;
    a = old;
  }
}

// link predicate of the forward bond id = (s, q), s < q (bondc.f:194-393:
// occupied bond; site.f: both sites occupied; sitebond.f / the mixed
// conductance rule: bond and both sites)
__device__ __forceinline__ bool cc_link(int kind, const uint8_t* bocc, const uint8_t* socc,
                                        long long id, int s, int q) {
  if (kind == PERC_BOND) return bocc[id];
  if (kind == PERC_SITE) return socc[s] && socc[q];
  return bocc[id] && socc[s] && socc[q];
}

__global__ __launch_bounds__(kCcThreads) void k_cc_tile(Geom g, int kind, const int* bond_first,
                                                        const uint8_t* bocc,
                                                        const uint8_t* socc, int* parent,
                                                        uint8_t* member, int bf_closed,
                                                        unsigned long long* trace) {
  unsigned long long tr0 = trace ? wall_clock64() : 0ull;
  static_assert(kCcW % 64 == 0 && kCcThreads % kCcW == 0, "a wave covers 64 columns of a tile row");
  constexpr int kPer = kCcSites / kCcThreads;
  __shared__ int lp[kCcSites];
  // lk: bits 0-5 the forward links, bit 7 membership (one byte per site:
  // 20 KB of LDS, 8 workgroups per CU).  During phase 2 the link bits are
  // fixed and bit 7 only ever set, so a plain byte read-or-write is exact.
  __shared__ uint8_t lk[kCcSites];
  const int ntx = cdiv(g.m, kCcW);
  // XCD-contiguous tiles (the edge-column tiles, every ntx-th, would share an XCD)
  const int tb = xcd_logical_block(blockIdx.x, gridDim.x);
  const int tx = tb % ntx, ty = tb / ntx;
  const int c0 = tx * kCcW, r0 = ty * kCcH;
  const int tw = min(kCcW, g.m - c0), th = min(kCcH, g.n - r0);
  const bool sq = g.lattice == kSquare;
  // phase 1: each site's forward links (bit r: the r-th forward bond in
  // nearestn order).  Square lattice, interior column, not the top row: the
  // forward links are (s, s+1), (s, s+m), bond ids fb, fb+1 (nearestn_square
  // lists +1 before +m in every such case).  All bond_first loads first,
  // then all link loads: two memory latencies per thread, not 2 per site.
  constexpr int kG = 4;  // sites per batch: loads of a batch in flight together (8: no faster)
  static_assert(kPer % kG == 0, "batches");
  for (int k0 = 0; k0 < kPer; k0 += kG) {
    int fbv[kG];
    bool occv[kG];
#pragma unroll
    for (int u = 0; u < kG; ++u) {
      const int li = threadIdx.x + (k0 + u) * kCcThreads, lr = li / kCcW, lc = li % kCcW;
      const int s = (r0 + lr) * g.m + c0 + lc + 1;
      const bool in = lr < th && lc < tw;
      occv[u] = in && (kind == PERC_BOND || socc[s]);
      const int row = r0 + lr;
      fbv[u] = !in || s > g.t - 1 ? 0
               : bf_closed && row <= g.n - 2 ? bf_square(g, row, c0 + lc)
                                             : bond_first[s];
    }
#pragma unroll
    for (int u = 0; u < kG; ++u) {
      const int li = threadIdx.x + (k0 + u) * kCcThreads, lr = li / kCcW, lc = li % kCcW;
      const int row = r0 + lr, col = c0 + lc;
      const int s = row * g.m + col + 1;
      unsigned mask = 0;
      if (occv[u] && s <= g.t - 1) {
        const int fb = fbv[u];
        if (sq && col >= 1 && col <= g.m - 2 && row <= g.n - 2) {
          mask = (unsigned)cc_link(kind, bocc, socc, fb, s, s + 1) |
                 (unsigned)cc_link(kind, bocc, socc, fb + 1, s, s + g.m) << 1;
        } else {
          int nn[6];
          nearestn_rc(g, s, row, col, nn);
          int r = 0;
          for (int kk = 0; kk < g.scn; ++kk) {
            const int q = nn[kk];
            if (q <= s) continue;
            if (cc_link(kind, bocc, socc, fb + r, s, q)) mask |= 1u << r;
            ++r;
          }
        }
      }
      const bool mem = (kind != PERC_BOND && occv[u]) || (kind == PERC_BOND && mask);
      lk[li] = (uint8_t)(mask | (mem ? 0x80u : 0u));
    }
  }
  __syncthreads();
  unsigned long long tr1 = trace ? wall_clock64() : 0ull;
  // phase 1b: the square lattice's horizontal runs.  Its first forward
  // neighbour is s+1 whenever col < m-1 (every nearestn_square case), so bit
  // 0 is the link to the right; a run's sites point at its first site (the
  // run's minimum: larger -> smaller as every union), the second 64-column
  // half of a row at the first half's last site when the run crosses.
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    const int li = threadIdx.x + k * kCcThreads, lc = li % kCcW;
    int par = li;
    if (sq) {
      const bool right = lc + 1 < tw && (lk[li] & 1u);
      const unsigned long long rb = __ballot(right);
      const bool left =
          lc > 0 && lc < tw && (lane > 0 ? (rb >> (lane - 1) & 1ull) : (lk[li - 1] & 1u));
      const unsigned long long starts = __ballot(!left);
      const unsigned long long upto = starts & (lane == 63 ? ~0ull : ((2ull << lane) - 1ull));
      par = upto ? li - lane + (63 - __clzll((long long)upto)) : li - lane - 1;
      if (left && kind == PERC_BOND) lk[li] |= 0x80u;
    }
    lp[li] = par;
  }
  __syncthreads();
  unsigned long long tr2 = trace ? wall_clock64() : 0ull;
  // phase 2: the other links inside the tile, LDS union-find (crossing
  // links: k_cc_merge).  (Measured: bottom-up order beats top-down -- finds
  // 23 vs 28 us per tile, flatten 5 vs 12 us.)
  for (int li = threadIdx.x; li < kCcSites; li += kCcThreads) {
    unsigned mask = lk[li] & 0x3Fu;
    const int lr = li / kCcW, lc = li % kCcW;
    if (sq && lc + 1 < tw) mask &= ~1u;  // in the run
    // square interior: the link up from s is redundant when s-1 links up
    // too and both s-1 -> s and s-1+m -> s+m are run links (a closed
    // plaquette: the union of s-1 already joined the two runs)
    if (sq && (mask & 2u) && lc >= 1 && lr + 1 < th && c0 + lc <= g.m - 2 && c0 + lc >= 1) {
      const unsigned lft = lk[li - 1], lup = lk[li - 1 + kCcW];
      if ((lft & 3u) == 3u && (lup & 1u) && c0 + lc - 1 >= 1) mask &= ~2u;
    }
    if (!mask) continue;
    const int row = r0 + lr, col = c0 + lc;
    const int s = row * g.m + col + 1;
    int qs[6], nq = 0;
    if (sq && col >= 1 && col <= g.m - 2 && row <= g.n - 2) {
      qs[0] = s + 1;
      qs[1] = s + g.m;
      nq = 2;
    } else {
      int nn[6];
      nearestn_rc(g, s, row, col, nn);
      for (int kk = 0; kk < g.scn; ++kk)
        if (nn[kk] > s) qs[nq++] = nn[kk];
    }
    for (int r = 0; r < nq; ++r) {
      if (!(mask >> r & 1u)) continue;
      const int q = qs[r];
      const int qrow = div_m(g, q - 1);
      const int qr = qrow - r0, qc = q - 1 - qrow * g.m - c0;
      if (qr < 0 || qr >= th || qc < 0 || qc >= tw) continue;  // crossing: k_cc_merge
      const int lq = qr * kCcW + qc;
      if (kind == PERC_BOND) lk[lq] |= 0x80u;
      // LDS union (larger local root -> smaller)
      int a = li, b = lq;
      while (true) {
        a = find_root(lp, a);
        b = find_root(lp, b);
        if (a == b) break;
        if (a < b) { const int tmp = a; a = b; b = tmp; }
        const int old = atomicCAS(&lp[a], a, b);
        if (old == a) break;
        a = old;
      }
    }
  }
  __syncthreads();
  unsigned long long tr3 = trace ? wall_clock64() : 0ull;
  for (int li = threadIdx.x; li < kCcSites; li += kCcThreads) {
    const int lr = li / kCcW, lc = li % kCcW;
    if (lr >= th || lc >= tw) continue;
    int x = li, p = lp[x];
    while (p != x) {
      x = p;
      p = lp[x];
    }
    const int s = (r0 + lr) * g.m + c0 + lc + 1;
    parent[s] = (r0 + x / kCcW) * g.m + c0 + x % kCcW + 1;
    member[s] = lk[li] >> 7;
  }
  if (trace && threadIdx.x == 0) {
    unsigned long long* o = trace + 5 * (size_t)blockIdx.x;
    o[0] = tr0;
    o[1] = tr1;
    o[2] = tr2;
    o[3] = tr3;
    o[4] = wall_clock64();
  }
}

// k_cc_tile_w (below): one wave per 128 x H tile of the open square lattice,
// rows walked bottom to top.  Lane l owns the tile's columns l and l + 64.
// Per row: the row's links (right, up), its horizontal runs by ballots (a
// run's node = its first site), the vertical links down into the previous
// row united in an LDS union-find over run nodes (larger root -> smaller, so
// a root is its component's minimum site; a lane whose (run, run below) pair
// equals the column to its left skips its union); a last pass writes every
// site's root.  Kind as cc_link (bond: member = any incident occupied bond;
// site / mixed: the occupied site).
// LDS union-find over tile nodes: 32-bit entries, or 16-bit ones (P16: half
// the LDS, so twice the waves per CU; the root CAS is a 32-bit CAS on the
// entry's word that leaves the other half as it finds it)
template <bool P16>
struct TileUF {
  int* w;  // P16: kCcW * H / 2 words holding two entries each
  // relaxed wavefront-scope atomic accesses: every access is performed (other
  // lanes move entries under a find), and none waits for the wave's global
  // loads in flight (a volatile access waited for vmcnt(0) and lgkmcnt(0))
  __device__ int get(int x) const {
    if (P16) return __hip_atomic_load(reinterpret_cast<unsigned short*>(w) + x, __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_WAVEFRONT);
    return __hip_atomic_load(w + x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
  }
  __device__ void set(int x, int v) const {
    if (P16) __hip_atomic_store(reinterpret_cast<unsigned short*>(w) + x, (unsigned short)v, __ATOMIC_RELAXED,
                                __HIP_MEMORY_SCOPE_WAVEFRONT);
    else __hip_atomic_store(w + x, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
  }
  // set x's parent to b if it is still a; returns what it found (a: done)
  __device__ int cas(int a, int b) const {
    if (!P16) return atomicCAS(&w[a], a, b);
    unsigned* word = reinterpret_cast<unsigned*>(w) + (a >> 1);
    const int sh = (a & 1) * 16;
    while (true) {
      const unsigned old = __hip_atomic_load(word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
      const int cur = (int)((old >> sh) & 0xffffu);
      if (cur != a) return cur;
      const unsigned nw = (old & ~(0xffffu << sh)) | ((unsigned)b << sh);
      if (atomicCAS(word, old, nw) == old) return a;
    }
  }
  __device__ int find(int x) const {  // path halving
    int p = get(x);
    while (p != x) {
      const int gp = get(p);
      if (gp != p) set(x, gp);
      x = gp;
      p = get(x);
    }
    return x;
  }
};

// wave-level LDS order: a wave's LDS instructions execute in program order,
// so lanes see each other's earlier LDS stores once the compiler keeps the
// order -- no memory fence (a release fence would also wait for the
// prefetched global loads, vmcnt(0), every row)
__device__ __forceinline__ void wave_lds_order() {
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
}

// forward bond id of site (row, col) of the open square lattice in the
// reference's bond order (bondc.f:137-154): rows 0..n-2 bf_square, the top
// row's right links after them (perc_ctx::bf_closed checks both)
__device__ __forceinline__ int bf_open_square(const Geom& g, int row, int col) {
  return row <= g.n - 2 ? bf_square(g, row, col) : (g.n - 1) * (2 * g.m - 1) + col;
}

// Row loads: the occupancy kind a template parameter, every load of a row
// unconditional (buffer loads, out-of-range offsets where a link does not
// exist), D rows in flight (a ring refilled as rows are consumed); no
// fences in the walk (wave_lds_order); the run nodes and member flags of
// the block's rows kept in registers, so the last pass writes every site's
// root without reading a provisional parent back.  Against the round-4
// version with branchy per-row loads (each waited for at once), volatile
// LDS entries, fences and provisional parents: tile 91.7 vs 123.8 us at
// L = 4096 (profiles/r4_13_cc_bench_L4096.txt).
// BAL: the left-link and deduplication tests from ballots of the row's
// right links and vertical unions -- 64-bit scalar masks (a lane's left
// neighbour in the row is bit lane - 1; lane 0's h = 1 site follows lane
// 63's h = 0 one) instead of LDS shuffles -- and each lane's (up to two)
// unions in one loop.  A lane skips its union when its column and the one
// to its left share their run in this row (a right link) and in the row
// below, and that column unites too: the same pair of runs.
// ncl: the block's member roots written to ncl[block]; the merge's hooks
// subtract from that count (k_span_top sums both), so no pass over every
// parent counts the clusters.  The bond kind's member flag of a block-edge
// site also depends on the links that cross into the block from the left
// (lane 0's first column: the right link of the site left of it) and from
// below (the block's first row: the up links of the row below); the tile
// reads those two link kinds for the flags only (their unions are the
// merge's), so the bond kind counts this way too and k_cc_count_roots is
// not run.
template <int H, int KIND, int D = 2, bool BAL = false>  // D: rows whose loads are in flight
__global__ __launch_bounds__(64) void k_cc_tile_w(Geom g, const uint8_t* bocc, const uint8_t* socc, int* parent,
                                                  uint8_t* member, unsigned nb_bytes, int* ncl = nullptr) {
  static_assert(H <= 32, "member flags: a row per bit of one word");
  __shared__ int uf_mem[kCcW * H / 2];
  const TileUF<true> uf{uf_mem};
  const int ntx = cdiv(g.m, kCcW);
  const int tb = xcd_logical_block(blockIdx.x, gridDim.x);
  const int tx = tb % ntx, ty = tb / ntx;
  const int c0 = tx * kCcW, r0 = ty * H;
  const int tw = min(kCcW, g.m - c0), th = min(H, g.n - r0);
  const int lane = threadIdx.x;
  // NBO (site / mixed kinds with BAL): a row's loads are the sites' own
  // occupancies (and bonds); the occupancy of the site a link leads to is
  // the right neighbour's (a ballot) or the next row's own load, applied
  // where the link is used -- 2 / 6 byte loads per lane and row, not 6 / 10
  constexpr bool NBO = BAL && KIND != PERC_BOND;
  const __amdgpu_buffer_rsrc_t rb = rsrc(bocc, nb_bytes), rs = rsrc(socc, (unsigned)g.t + 8u);
  auto ld8 = [](__amdgpu_buffer_rsrc_t r, bool ok, unsigned off) {
    return (unsigned)__builtin_amdgcn_raw_buffer_load_b8(r, (int)(ok ? off : kOOB), 0, 0);
  };
  // R / U: the link right / up of the lane's two sites; O: the site occupied
  auto load_row = [&](int r, unsigned (&R)[2], unsigned (&U)[2], unsigned (&O)[2]) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int lc = lane + 64 * h, col = c0 + lc, row = r0 + r;
      const bool v = lc < tw && r < th;
      const int s = row * g.m + col + 1;
      const bool hr = v && col < g.m - 1, hu = v && row < g.n - 1;
      if constexpr (KIND == PERC_SITE) {
        O[h] = ld8(rs, v, (unsigned)s);
        if constexpr (NBO) {
          R[h] = hr ? 1u : 0u;
          U[h] = hu ? 1u : 0u;
        } else {
          R[h] = ld8(rs, hr, (unsigned)s + 1u);
          U[h] = ld8(rs, hu, (unsigned)(s + g.m));
        }
      } else {
        const int fb = bf_open_square(g, row, col);
        R[h] = ld8(rb, hr, (unsigned)fb);
        U[h] = ld8(rb, hu, (unsigned)fb + (col < g.m - 1 ? 1u : 0u));
        O[h] = 1u;
        if constexpr (KIND != PERC_BOND) {
          O[h] = ld8(rs, v, (unsigned)s);
          if constexpr (!NBO) {
            R[h] &= ld8(rs, hr, (unsigned)s + 1u);
            U[h] &= ld8(rs, hu, (unsigned)(s + g.m));
          }
        }
      }
    }
  };
  auto finish = [&](unsigned (&R)[2], unsigned (&U)[2], unsigned (&O)[2]) {
    if constexpr (KIND != PERC_BOND) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        R[h] = O[h] ? R[h] : 0u;
        U[h] = O[h] ? U[h] : 0u;
      }
    }
  };
  unsigned Rq[D][2], Uq[D][2], Oq[D][2], R[2], U[2], O[2], Up[2] = {0u, 0u};
  int labp[2] = {0, 0};
  unsigned nodes[H], Mb[2] = {0u, 0u};
  // bond kind, the links crossing into the block's edge sites (member flags
  // only): Xl -- lane r holds the left block's link into row r's column 0
  // (one load for the block, read back per row with a readlane); Up of the
  // first row -- the row below's up links
  unsigned Xl = 0u;
  if constexpr (KIND == PERC_BOND) {
    const bool hx = c0 > 0 && lane < th;
    Xl = ld8(rb, hx, (unsigned)bf_open_square(g, hx ? r0 + lane : 0, hx ? c0 - 1 : 0));
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int lc = lane + 64 * h, col = c0 + lc;
      const bool hd = r0 > 0 && lc < tw;
      Up[h] = ld8(rb, hd, (unsigned)(hd ? bf_open_square(g, r0 - 1, col) + (col < g.m - 1 ? 1 : 0) : 0));
    }
  }
#pragma unroll
  for (int d = 0; d < D; ++d) load_row(d, Rq[d], Uq[d], Oq[d]);
  const unsigned long long le = lane == 63 ? ~0ull : ((2ull << lane) - 1ull);
  const bool v0 = lane < tw, v1 = lane + 64 < tw;
  const unsigned long long vm0 = __ballot(v0), vm1 = __ballot(v1);
  unsigned long long lmp0 = 0, lmp1 = 0;  // BAL: the row below's left-link masks
#pragma unroll
  for (int r = 0; r < H; ++r) {
    nodes[r] = 0u;
    if (r >= th) continue;  // (uniform)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      R[h] = Rq[r % D][h];
      U[h] = Uq[r % D][h];
      O[h] = Oq[r % D][h];
    }
    finish(R, U, O);
    load_row(r + D, Rq[r % D], Uq[r % D], Oq[r % D]);  // (past th: nothing loaded)
    const unsigned X = KIND == PERC_BOND && lane == 0 ? (unsigned)__builtin_amdgcn_readlane((int)Xl, r) : 0u;
    bool left0, left1;
    unsigned long long lo, hi, lm0 = 0, lm1 = 0;
    if constexpr (BAL) {
      // the columns whose left neighbour links to them in this row
      const unsigned long long rb0 = __ballot(R[0] != 0u), rb1 = __ballot(R[1] != 0u);
      lm0 = rb0 << 1;
      lm1 = rb1 << 1 | rb0 >> 63;
      if constexpr (NBO) {  // the linked-to site occupied too
        lm0 &= __ballot(O[0] != 0u);
        lm1 &= __ballot(O[1] != 0u);
      }
      left0 = (lm0 >> lane) & 1ull;
      left1 = (lm1 >> lane) & 1ull;
      lo = ~(lm0 & vm0);
      hi = ~(lm1 & vm1);
    } else {
      const unsigned rl0 = __shfl(R[0], (lane + 63) & 63, 64), rl1 = __shfl(R[1], (lane + 63) & 63, 64);
      left0 = lane > 0 && rl0;
      left1 = lane > 0 ? rl1 != 0u : rl0 != 0u;
      lo = __ballot(!left0 || !v0);
      hi = __ballot(!left1 || !v1);
    }
    int node[2];
    node[0] = r * kCcW + 63 - __clzll((long long)(lo & le));
    const unsigned long long hm = hi & le;
    node[1] = r * kCcW + (hm ? 64 + 63 - __clzll((long long)hm) : 63 - __clzll((long long)lo));
    if (v0 && !left0) uf.set(node[0], node[0]);
    if (v1 && !left1) uf.set(node[1], node[1]);
    wave_lds_order();
    const bool w0 = r > 0 && v0 && Up[0] && (!NBO || O[0]), w1 = r > 0 && v1 && Up[1] && (!NBO || O[1]);
    const int a0 = w0 ? node[0] : -1, b0 = w0 ? labp[0] : -1, a1 = w1 ? node[1] : -1, b1 = w1 ? labp[1] : -1;
    if constexpr (BAL) {
      const unsigned long long wb0 = __ballot(w0), wb1 = __ballot(w1);
      const unsigned long long sm0 = lm0 & lmp0 & wb0 << 1, sm1 = lm1 & lmp1 & (wb1 << 1 | wb0 >> 63);
      bool more = w1 && !((sm1 >> lane) & 1ull);
      bool act = w0 && !((sm0 >> lane) & 1ull);
      int a = a0, b = b0;
      if (!act && more) {
        a = a1;
        b = b1;
        act = true;
        more = false;
      }
#if defined(PERC_TILE_PROBE_NOUNION)  // (cost probes only: wrong partitions)
      act = false;
#endif
      while (act) {  // the lane's unions, one after the other, in one loop
        a = uf.find(a);
        b = uf.find(b);
        bool done = a == b;
        if (!done) {
          if (a < b) { const int t = a; a = b; b = t; }
          const int old = uf.cas(a, b);
          done = old == a;
          a = old;
        }
        if (done) {
          act = more;
          more = false;
          a = a1;
          b = b1;
        }
      }
      lmp0 = lm0;
      lmp1 = lm1;
    } else {
      const int pa0 = __shfl(a0, (lane + 63) & 63, 64), pb0 = __shfl(b0, (lane + 63) & 63, 64);
      const int pa1 = __shfl(a1, (lane + 63) & 63, 64), pb1 = __shfl(b1, (lane + 63) & 63, 64);
      const bool sk0 = lane > 0 && pa0 == a0 && pb0 == b0;
      const bool sk1 = lane > 0 ? (pa1 == a1 && pb1 == b1) : (pa0 == a1 && pb0 == b1);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const bool w = h ? w1 && !sk1 : w0 && !sk0;
        if (!w) continue;
        int a = h ? a1 : a0, b = h ? b1 : b0;
        while (true) {
          a = uf.find(a);
          b = uf.find(b);
          if (a == b) break;
          if (a < b) { const int t = a; a = b; b = t; }
          const int old = uf.cas(a, b);
          if (old == a) break;
          a = old;
        }
      }
    }
    wave_lds_order();
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const bool lft = h ? left1 : left0;
      // (bond kind: Up of the first row = the row below the block's up
      // links, X = the left block's link into column 0)
      const bool mem = KIND == PERC_BOND ? (R[h] | U[h] | (lft ? 1u : 0u) | Up[h] | (h == 0 ? X : 0u)) != 0u
                                         : O[h] != 0u;
      Mb[h] |= (mem ? 1u : 0u) << r;
    }
    nodes[r] = (unsigned)node[0] | (unsigned)node[1] << 16;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      labp[h] = node[h];
      Up[h] = U[h];
    }
  }
  wave_lds_order();
  int nroot = 0;
#pragma unroll
  for (int r = 0; r < H; ++r) {
    if (r >= th) continue;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int lc = lane + 64 * h;
      if (lc >= tw) continue;
      const int s = (r0 + r) * g.m + c0 + lc + 1;
      int x = (int)(nodes[r] >> (16 * h) & 0xffffu), p = uf.get(x);
#if defined(PERC_TILE_PROBE_NOFINAL)  // (cost probes only: wrong partitions)
      p = x;
#endif
      while (p != x) {
        x = p;
        p = uf.get(x);
      }
      const int root = (r0 + x / kCcW) * g.m + c0 + x % kCcW + 1;
      parent[s] = root;
      member[s] = (uint8_t)(Mb[h] >> r & 1u);
      nroot += root == s && (Mb[h] >> r & 1u);
    }
  }
  if (ncl) {  // (uniform)
    nroot = wave_sum_int(nroot);
    if (lane == 0) ncl[blockIdx.x] = nroot;
  }
}

// The links that cross a block edge, with neighbouring lanes on neighbouring
// sites of the same edge: part A, the blocks' top rows (every column: the
// links up into the next block row), one workgroup per kCcThreads columns;
// part B, the other rows' candidate columns (the block edge columns and the
// last column), one workgroup per candidate column and kCcThreads rows.
// Before any union a lane reads the parents of its link's two sites (after
// k_cc_tile: the block-local roots, or ancestors of them); a lane whose pair
// equals the previous lane's skips its union -- that lane's union joins the
// same two sets (by induction down to the first lane of the run).  Along an
// edge most crossing links join the same two block components, so most
// unions drop out; the rest start one hop closer to the roots.  (Against
// the round-3 mapping, one workgroup per lattice row: labels 0.435 vs
// 0.512 ms per realisation at L = 4096, profiles/r4_4_label_ab_L4096.json.)
// WD: the wave's unions deduplicated over all its lanes, the pairs taken as
// (min, max) -- one union per distinct pair of parents in the wave, by the
// pair's first lane (one ballot round per distinct pair); else only a lane
// whose pair equals the previous lane's skips.  Along a block edge most
// crossing links join the same few block components, so most lanes drop out:
// merge 47.4 vs 83.6 us at L = 4096 (profiles/r4_11_cc_bench_L4096.txt)
// nhook (with the tiles' ncl): minus the workgroup's successful hooks,
// written to nhook[blockIdx.x]
template <int TH = kCcH, bool WD = true>  // TH: block height of the tile kernel that ran before
__global__ __launch_bounds__(kCcThreads) void k_cc_merge(Geom g, int kind, const int* bond_first,
                                                         const uint8_t* bocc,
                                                         const uint8_t* socc, int* parent,
                                                         uint8_t* member, int nseg, int nfull,
                                                         int* nhook = nullptr) {
  const int ntx = cdiv(g.m, kCcW), lane = threadIdx.x & 63;
  int row, c;
  if ((int)blockIdx.x < nfull * nseg) {  // A: block-top row, columns of segment
    row = (blockIdx.x / nseg) * TH + TH - 1;
    c = (blockIdx.x % nseg) * kCcThreads + threadIdx.x;
  } else {  // B: candidate column j, rows of block rb (block-top rows are A's)
    const int e = blockIdx.x - nfull * nseg, nrb = cdiv(g.n, kCcThreads);
    const int j = e / nrb;
    row = (e % nrb) * kCcThreads + threadIdx.x;
    c = j == 2 * ntx ? g.m - 1 : min((j >> 1) * kCcW + (j & 1) * (kCcW - 1), g.m - 1);
    if (row % TH == TH - 1) row = g.n;  // (part A's)
  }
  const int s = row * g.m + c + 1;
  bool site = row < g.n && c < g.m && s <= g.t - 1 && (kind == PERC_BOND || socc[s]);
  int nn[6] = {0, 0, 0, 0, 0, 0}, fb = 0;
  if (site) {
    nearestn_rc(g, s, row, c, nn);
    fb = bond_first[s];
  }
  int r = 0, hooks = 0;
  for (int k = 0; k < g.scn; ++k) {  // (uniform trip count: the shuffles below)
    const int q = nn[k];
    const bool fwd = site && q > s;
    bool want = fwd && cc_link(kind, bocc, socc, fb + r, s, q);
    r += fwd ? 1 : 0;
    if (want) {
      const int qrow = div_m(g, q - 1), qcol = q - 1 - qrow * g.m;
      want = !(qrow / TH == row / TH && qcol / kCcW == c / kCcW);  // inside: k_cc_tile's
    }
    if (want && kind == PERC_BOND) member[q] = 1;
    const int a = want ? parent[s] : -1, b = want ? parent[q] : -1;
    if constexpr (WD) {
      const int lo = min(a, b), hi = max(a, b);
      bool lead = want && lo != hi;
      unsigned long long act = __ballot(lead);
      while (act) {
        const int l = __builtin_ctzll(act);
        const int la = __shfl(lo, l, 64), lh = __shfl(hi, l, 64);
        const bool same = lead && lo == la && hi == lh;
        act &= ~__ballot(same);
        if (same && lane != l) lead = false;
      }
      if (lead) hooks += unite(parent, lo, hi) ? 1 : 0;
    } else {
      const int pa = __shfl_up(a, 1, 64), pb = __shfl_up(b, 1, 64);
      if (want && !(lane > 0 && pa == a && pb == b)) hooks += unite(parent, a, b) ? 1 : 0;
    }
  }
  if (nhook) {  // (uniform)
    __shared__ int s_h[kCcThreads / 64];
    hooks = wave_sum_int(hooks);
    if (lane == 0) s_h[threadIdx.x >> 6] = hooks;
    __syncthreads();
    if (threadIdx.x == 0) {
      int tot = 0;
#pragma unroll
      for (int w = 0; w < kCcThreads / 64; ++w) tot += s_h[w];
      nhook[blockIdx.x] = -tot;
    }
  }
}

// The open square lattice's merge (after k_cc_tile_w<TH>): only its two
// crossing link kinds, bond ids in closed form (bf_open_square), no
// neighbour lists.  Part A, the block-top rows, one workgroup per kCcThreads
// columns: every column's up link, and a block's last column's right link;
// part B, the blocks' last columns (c = 128 k + 127 < m - 1) of the other
// rows: the right link (the generic merge also walked the blocks' first
// columns, which have no forward crossing link here).  Unions deduplicated
// over the wave as in k_cc_merge; nhook as there.
template <int TH, int KIND>
__global__ __launch_bounds__(kCcThreads) void k_cc_merge_sq(Geom g, const uint8_t* bocc, const uint8_t* socc,
                                                            int* parent, uint8_t* member, int nseg, int nfull,
                                                            int* nhook) {
  const int lane = threadIdx.x & 63;
  const bool partA = (int)blockIdx.x < nfull * nseg;
  int row, c;
  if (partA) {
    row = (blockIdx.x / nseg) * TH + TH - 1;
    c = (blockIdx.x % nseg) * kCcThreads + threadIdx.x;
  } else {
    const int e = blockIdx.x - nfull * nseg, nrb = cdiv(g.n, kCcThreads);
    c = (e / nrb) * kCcW + kCcW - 1;
    row = (e % nrb) * kCcThreads + threadIdx.x;
    if (row % TH == TH - 1) row = g.n;  // (part A's)
  }
  const bool site = row < g.n && c < g.m;
  const int s = row * g.m + c + 1;
  const bool so = site && (KIND == PERC_BOND || socc[s]);
  int hooks = 0;
  // link 0: up (part A); link 1: right (part B, and part A's block-last columns)
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    if (k == 0 && !partA) continue;  // (uniform)
    const bool exists = k == 0 ? row < g.n - 1 : (c % kCcW == kCcW - 1 && c < g.m - 1);
    const int q = k == 0 ? s + g.m : s + 1;
    bool want = so && exists;
    if (want) {
      const int fb = bf_open_square(g, row, c);
      const int id = k == 0 ? fb + (c < g.m - 1 ? 1 : 0) : fb;
      if constexpr (KIND == PERC_BOND) want = bocc[id] != 0;
      else if constexpr (KIND == PERC_SITE) want = socc[q] != 0;
      else want = bocc[id] != 0 && socc[q] != 0;
    }
    if (want && KIND == PERC_BOND) member[q] = 1;
    const int a = want ? parent[s] : -1, b = want ? parent[q] : -1;
    const int lo = min(a, b), hi = max(a, b);
    bool lead = want && lo != hi;
    unsigned long long act = __ballot(lead);
    while (act) {
      const int l = __builtin_ctzll(act);
      const int la = __shfl(lo, l, 64), lh = __shfl(hi, l, 64);
      const bool same = lead && lo == la && hi == lh;
      act &= ~__ballot(same);
      if (same && lane != l) lead = false;
    }
    if (lead) hooks += unite(parent, lo, hi) ? 1 : 0;
  }
  if (nhook) {  // (uniform)
    __shared__ int s_h[kCcThreads / 64];
    hooks = wave_sum_int(hooks);
    if (lane == 0) s_h[threadIdx.x >> 6] = hooks;
    __syncthreads();
    if (threadIdx.x == 0) {
      int tot = 0;
#pragma unroll
      for (int w = 0; w < kCcThreads / 64; ++w) tot += s_h[w];
      nhook[blockIdx.x] = -tot;
    }
  }
}

// k_cc_merge_sq with U sites per thread whose memory round trips overlap:
// the occupancy bytes of all U sites' links loaded together (buffer loads,
// out-of-range offsets where a link does not exist), then their parents,
// then each link deduplicated over the wave as in k_cc_merge_sq, then the
// thread's remaining unions in lockstep -- every hop of every chain and
// every CAS of the round issued before any is waited for (a chain's first
// node then points at the root it found).  A union that
// loses its CAS retries from the value it found, as in unite(): the
// partition, the hooks (one per merged pair of components) and, after the
// compress, every parent are the one-site-per-thread merge's.  Part A:
// kCcThreads * U columns of a block-top row per workgroup, part B:
// kCcThreads * U rows of a block-last column.
template <int TH, int KIND, int U>
__global__ __launch_bounds__(kCcThreads) void k_cc_merge_squ(Geom g, const uint8_t* bocc, const uint8_t* socc,
                                                             int* parent, uint8_t* member, unsigned nb_bytes,
                                                             int nsegu, int nfull, int* nhook) {
  const int lane = threadIdx.x & 63;
  const bool partA = (int)blockIdx.x < nfull * nsegu;
  const __amdgpu_buffer_rsrc_t rb = rsrc(bocc, nb_bytes), rs = rsrc(socc, (unsigned)g.t + 8u);
  const __amdgpu_buffer_rsrc_t rp = rsrc(parent, ((unsigned)g.t + 2u) * 4u);
  constexpr int M = 2 * U;  // (u, link kind k): k = 0 up (part A), 1 right
  int sq[M], pa[M], pb[M];
  bool want[M];
  unsigned ob[M], oq[M], os[U];
  int s[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    int row, c;
    if (partA) {
      row = (blockIdx.x / nsegu) * TH + TH - 1;
      c = (blockIdx.x % nsegu) * kCcThreads * U + u * kCcThreads + threadIdx.x;
    } else {
      const int e = blockIdx.x - nfull * nsegu, nrbu = cdiv(g.n, kCcThreads * U);
      c = (e / nrbu) * kCcW + kCcW - 1;
      row = (e % nrbu) * kCcThreads * U + u * kCcThreads + threadIdx.x;
      if (row % TH == TH - 1) row = g.n;  // (part A's)
    }
    const bool site = row < g.n && c < g.m;
    s[u] = row * g.m + c + 1;
    os[u] = KIND == PERC_BOND ? 1u : (unsigned)__builtin_amdgcn_raw_buffer_load_b8(rs, site ? s[u] : (int)kOOB, 0, 0);
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int j = 2 * u + k;
      const bool exists = site && (k == 0 ? partA && row < g.n - 1 : (c % kCcW == kCcW - 1 && c < g.m - 1));
      sq[j] = k == 0 ? s[u] + g.m : s[u] + 1;
      want[j] = exists;
      const int fb = exists ? bf_open_square(g, row, c) : 0;
      const int id = k == 0 ? fb + (c < g.m - 1 ? 1 : 0) : fb;
      ob[j] = KIND == PERC_SITE ? 1u : (unsigned)__builtin_amdgcn_raw_buffer_load_b8(rb, exists ? id : (int)kOOB, 0, 0);
      oq[j] = KIND == PERC_BOND ? 1u : (unsigned)__builtin_amdgcn_raw_buffer_load_b8(rs, exists ? sq[j] : (int)kOOB, 0, 0);
    }
  }
#pragma unroll
  for (int j = 0; j < M; ++j) {
    want[j] = want[j] && os[j / 2] && ob[j] && oq[j];
    if (KIND == PERC_BOND && want[j]) member[sq[j]] = 1;
    pa[j] = (int)__builtin_amdgcn_raw_buffer_load_b32(rp, want[j] ? s[j / 2] * 4 : (int)kOOB, 0, 0);
    pb[j] = (int)__builtin_amdgcn_raw_buffer_load_b32(rp, want[j] ? sq[j] * 4 : (int)kOOB, 0, 0);
  }
  // one union per distinct pair of parents in the wave, by its first lane
  int A[M], B[M];
  bool act[M];
#pragma unroll
  for (int j = 0; j < M; ++j) {
    const int lo = min(pa[j], pb[j]), hi = max(pa[j], pb[j]);
    bool lead = want[j] && lo != hi;
    if (j % 2 == 0 && !partA) lead = false;  // (no up links in part B)
    unsigned long long actm = __ballot(lead);
    while (actm) {
      const int l = __builtin_ctzll(actm);
      const int la = __shfl(lo, l, 64), lh = __shfl(hi, l, 64);
      const bool same = lead && lo == la && hi == lh;
      actm &= ~__ballot(same);
      if (same && lane != l) lead = false;
    }
    act[j] = lead;
    A[j] = lo;
    B[j] = hi;
  }
  int hooks = 0;
  while (true) {
    int A0[M], B0[M];
#pragma unroll
    for (int j = 0; j < M; ++j) {
      A0[j] = A[j];
      B0[j] = B[j];
    }
    // roots of every active pair: one hop of every chain per round
    while (true) {
      int na[M], nb2[M];
#pragma unroll
      for (int j = 0; j < M; ++j) {
        na[j] = act[j] ? parent[A[j]] : A[j];
        nb2[j] = act[j] ? parent[B[j]] : B[j];
      }
      bool more = false;
#pragma unroll
      for (int j = 0; j < M; ++j) {
        more |= na[j] != A[j] || nb2[j] != B[j];
        A[j] = na[j];
        B[j] = nb2[j];
      }
      if (!more) break;
    }
    // the chains' first nodes straight to the roots found (an ancestor: the
    // same set, a smaller index) -- the next chase from them is one hop
#pragma unroll
    for (int j = 0; j < M; ++j) {
      if (act[j] && A0[j] != A[j]) parent[A0[j]] = A[j];
      if (act[j] && B0[j] != B[j]) parent[B0[j]] = B[j];
    }
    bool any = false;
#pragma unroll
    for (int j = 0; j < M; ++j) {
      if (!act[j]) continue;
      if (A[j] == B[j]) {
        act[j] = false;
        continue;
      }
      int a = max(A[j], B[j]), b = min(A[j], B[j]);
      const int old = atomicCAS(&parent[a], a, b);
      if (old == a) {
        ++hooks;
        act[j] = false;
      } else {
        A[j] = old;  // a lost race: again from what the root became
        B[j] = b;
        any = true;
      }
    }
    if (!any) break;
  }
  if (nhook) {  // (uniform)
    __shared__ int s_h[kCcThreads / 64];
    hooks = wave_sum_int(hooks);
    if (lane == 0) s_h[threadIdx.x >> 6] = hooks;
    __syncthreads();
    if (threadIdx.x == 0) {
      int tot = 0;
#pragma unroll
      for (int w = 0; w < kCcThreads / 64; ++w) tot += s_h[w];
      nhook[blockIdx.x] = -tot;
    }
  }
}

// sum of v over the workgroup of kCcThreads, then one atomic add
__device__ __forceinline__ void block_count_add(int v, int* counter) {
  __shared__ int s_cnt[kCcThreads / 64];
  v = wave_sum_int(v);
  if ((threadIdx.x & 63) == 0) s_cnt[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    int tot = 0;
#pragma unroll
    for (int w = 0; w < kCcThreads / 64; ++w) tot += s_cnt[w];
    if (tot) atomicAdd(counter, tot);
  }
}

// member roots (parent[s] == s, member[s]): the cluster count, with or
// without the parents flattened; a thread's U sites loaded together
__global__ __launch_bounds__(kCcThreads) void k_cc_count_roots(int t, const int* parent, const uint8_t* member,
                                                               int* nclusters) {
  constexpr int U = 4;
  int cnt = 0;
  for (long long b = (long long)blockIdx.x * kCcThreads * U + threadIdx.x + 1; b <= t;
       b += (long long)gridDim.x * kCcThreads * U) {
    int p[U];
    uint8_t mb[U];
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const long long s = b + k * kCcThreads;
      p[k] = s <= t ? parent[s] : 0;
      mb[k] = s <= t ? member[s] : 0;
    }
#pragma unroll
    for (int k = 0; k < U; ++k) cnt += p[k] == (int)(b + k * kCcThreads) && mb[k];
  }
  block_count_add(cnt, nclusters);
}

// final flattening: read-only walks, then each thread writes only its own
// entries (path halving here would let one thread overwrite another's
// freshly written root with an intermediate ancestor); counts the clusters
// (member roots).  A thread's U sites are chased in lockstep: every hop
// issues their U parent loads together (one chain after another: compress
// 83.3 vs 55.3 us at L = 4096, profiles/r4_7_cc_bench_L4096.txt).
constexpr int kCcCompressU = 8;
// With root > 0 the member sites whose root is `root` are counted into
// *rcount (the spanning cluster's size, formerly a second pass, k_count_root:
// 30 us at L = 4096, profiles/r5_35_final_rocprof_kernel_stats.csv).
template <int U = kCcCompressU>
__global__ __launch_bounds__(kCcThreads) void k_cc_compress(int t, int* parent, const uint8_t* member, int root,
                                                            int* rcount) {
  int cnt = 0;
  for (long long b = (long long)blockIdx.x * kCcThreads * U + threadIdx.x + 1; b <= t;
       b += (long long)gridDim.x * kCcThreads * U) {
    int x[U], y[U];
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const long long s = b + k * kCcThreads;
      x[k] = s <= t ? parent[s] : 0;
    }
    while (true) {
#pragma unroll
      for (int k = 0; k < U; ++k) y[k] = b + k * kCcThreads <= t ? parent[x[k]] : 0;
      bool more = false;
#pragma unroll
      for (int k = 0; k < U; ++k) {
        more |= y[k] != x[k];
        x[k] = y[k];
      }
      if (!more) break;
    }
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const long long s = b + k * kCcThreads;
      if (s > t) continue;
      parent[s] = x[k];
      cnt += x[k] == root && member[s];
    }
  }
  if (root > 0) block_count_add(cnt, rcount);  // (uniform)
}

// k_cc_compress of a labeling whose spanning roots the host has not read
// yet (perc_label's one-synchronisation path): dcnt[0] the spanning count
// and dcnt[8] the first spanning root as k_span_top left them in device
// memory.  Nothing spans: every workgroup returns (nothing flattened, nothing
// counted).  Else every parent to its root and the member sites of that
// root counted; the last workgroup to finish (ticket and count in the
// 64-bit word at dcnt[4]) writes the total to hout[2] (the pinned read-back
// words).
template <int U = kCcCompressU>
__global__ __launch_bounds__(kCcThreads) void k_cc_compress_spec(int t, int* parent, const uint8_t* member,
                                                                 int* dcnt, int* hout) {
  if (dcnt[0] == 0) return;  // (uniform)
  const int root = dcnt[8];
  int cnt = 0;
  for (long long b = (long long)blockIdx.x * kCcThreads * U + threadIdx.x + 1; b <= t;
       b += (long long)gridDim.x * kCcThreads * U) {
    int x[U], y[U];
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const long long s = b + k * kCcThreads;
      x[k] = s <= t ? parent[s] : 0;
    }
    while (true) {
#pragma unroll
      for (int k = 0; k < U; ++k) y[k] = b + k * kCcThreads <= t ? parent[x[k]] : 0;
      bool more = false;
#pragma unroll
      for (int k = 0; k < U; ++k) {
        more |= y[k] != x[k];
        x[k] = y[k];
      }
      if (!more) break;
    }
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const long long s = b + k * kCcThreads;
      if (s > t) continue;
      parent[s] = x[k];
      cnt += x[k] == root && member[s];
    }
  }
  __shared__ int s_cnt[kCcThreads / 64];
  cnt = wave_sum_int(cnt);
  if ((threadIdx.x & 63) == 0) s_cnt[threadIdx.x >> 6] = cnt;
  __syncthreads();
  if (threadIdx.x == 0) {
    int tot = 0;
#pragma unroll
    for (int w = 0; w < kCcThreads / 64; ++w) tot += s_cnt[w];
    // one 64-bit atomic: the ticket in the high word, the count in the low
    // one -- the last workgroup's old value holds every other's count (no
    // fences: an acquire / release pair per workgroup cost 7 us at L = 4096)
    const unsigned long long old = __hip_atomic_fetch_add(reinterpret_cast<unsigned long long*>(&dcnt[4]),
                                                          (1ull << 32) | (unsigned)tot, __ATOMIC_RELAXED,
                                                          __HIP_MEMORY_SCOPE_AGENT);
    if ((old >> 32) == gridDim.x - 1) hout[2] = (int)(unsigned)old + tot;
  }
}

}  // namespace
}  // namespace perc
#pragma clang diagnostic pop
