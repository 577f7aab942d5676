// perc_label.hip -- occupancy and cluster labeling of libperc (gfx950):
// the occupation of sites / bonds (given orders or drawn on the device),
// the connected-component partition (Square/bondc.f:194-393,
// site.f:167-289), the spanning test, cluster sizes and canonical labels.
#include "perc_common.h"

namespace perc {
namespace {

// ---------------------------------------------------------------------------
// Occupancy
__global__ void k_occupy(const int* order, int count, long long limit, uint8_t* occ) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= count) return;
  const int id = order[k];
  if (id > 0 && id <= limit) occ[id - 1] = 1;
}
__device__ __forceinline__ int wave_sum_int(int v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// The `count`-th smallest key T of ids 1..n (perc_occupy_random) without a
// host round trip.  The 32-bit hashes are uniform, so T's hash lies, with
// overwhelming probability, in a window [lo, hi) a few binomial standard
// deviations around count/n * 2^32.  k_select_window counts the keys below
// the window and gathers the keys inside it (LDS staging, one global
// reservation per workgroup, at most kSelCap keys); k_select_final (one
// workgroup) bins the window keys by hash (kSelBins LDS bins), finds the bin
// holding the (count - below)-th smallest and ranks that bin's few keys.  A
// crowded bin falls back to an 8-pass radix select of the window keys, T
// outside the window (or an overflowing window) to the radix select of all n
// keys -- slow, exact: T is the exact order statistic on every path.
constexpr int kSelCap = 1 << 17, kSelThreads = 1024, kSelStage = 512, kSelBins = 4096;
constexpr int kSelBinCap = 1024;
__global__ __launch_bounds__(kBlock) void k_select_window(long long n, unsigned long long seed,
                                                          unsigned long long lo,
                                                          unsigned long long hi,
                                                          unsigned* cnt,
                                                          unsigned long long* cand) {
  __shared__ unsigned long long s_c[kSelStage];
  __shared__ unsigned s_n, s_base, s_b[kBlock / 64];
  if (threadIdx.x == 0) s_n = 0;
  __syncthreads();
  unsigned below = 0;
  const int lane = threadIdx.x & 63;
  for (long long i = (long long)blockIdx.x * kBlock + threadIdx.x; i < n;
       i += (long long)gridDim.x * kBlock) {
    const unsigned long long key = perc_rand_key(seed, (unsigned)(i + 1));
    const unsigned long long hsh = key >> 32;
    below += hsh < lo;
    if (hsh >= lo && hsh < hi) {
      const unsigned slot = atomicAdd(&s_n, 1u);
      if (slot < (unsigned)kSelStage) {
        s_c[slot] = key;
      } else {  // a crowded workgroup: straight to the global list
        const unsigned idx = atomicAdd(&cnt[1], 1u);
        if (idx < (unsigned)kSelCap) cand[1 + idx] = key;
      }
    }
  }
  below = (unsigned)wave_sum_int((int)below);
  if (lane == 0) s_b[threadIdx.x >> 6] = below;
  __syncthreads();
  const unsigned nst = min(s_n, (unsigned)kSelStage);
  if (threadIdx.x == 0) {
    unsigned tot = 0;
    for (int w = 0; w < kBlock / 64; ++w) tot += s_b[w];
    if (tot) atomicAdd(&cnt[0], tot);
    s_base = nst ? atomicAdd(&cnt[1], nst) : 0u;
  }
  __syncthreads();
  for (unsigned j = threadIdx.x; j < nst; j += kBlock)
    if (s_base + j < (unsigned)kSelCap) cand[1 + s_base + j] = s_c[j];
}

__global__ __launch_bounds__(kSelThreads) void k_select_final(long long n,
                                                              unsigned long long seed,
                                                              long long count,
                                                              unsigned long long lo,
                                                              unsigned long long hi,
                                                              const unsigned* cnt,
                                                              unsigned long long* cand) {
  __shared__ unsigned s_h[kSelBins];
  __shared__ unsigned long long s_k[kSelBinCap];
  __shared__ unsigned long long s_sel[2];  // prefix, need
  __shared__ int s_bin, s_nb;
  unsigned long long* tr = cand + 1 + kSelCap;  // PERC_SELECT_TRACE stamps
  if (threadIdx.x == 0) tr[0] = wall_clock64();
  const long long below = cnt[0], nin = cnt[1];
  const bool win = count > below && count - below <= nin && nin <= kSelCap;
  if (win) {
    // bins of the window's hash range: (hash - lo) >> sh < kSelBins
    const unsigned long long range = hi - lo;
    const int bits = range > 1 ? 64 - __clzll((long long)(range - 1)) : 0;
    const int sh = max(0, bits - 12);
    for (int j = threadIdx.x; j < kSelBins; j += kSelThreads) s_h[j] = 0;
    if (threadIdx.x == 0) s_nb = 0;
    __syncthreads();
    constexpr int kU = 8;  // loads in flight per thread
    for (long long i0 = threadIdx.x; i0 < nin; i0 += kSelThreads * kU) {
      unsigned long long kk[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u) kk[u] = i0 + u * kSelThreads < nin ? cand[1 + i0 + u * kSelThreads] : 0;
#pragma unroll
      for (int u = 0; u < kU; ++u)
        if (i0 + u * kSelThreads < nin) atomicAdd(&s_h[((kk[u] >> 32) - lo) >> sh], 1u);
    }
    __syncthreads();
    if (threadIdx.x == 0) tr[1] = wall_clock64();
    {  // the bin of the (count - below)-th window key: a block scan of the
       // bin counts, kPerT consecutive bins per thread (a serial scan of
       // 4096 LDS words by one thread costs ~70 us)
      constexpr int kPerT = kSelBins / kSelThreads;
      static_assert(kSelBins % kSelThreads == 0, "bins per thread");
      __shared__ unsigned s_w[kSelThreads / 64];
      const unsigned need = (unsigned)(count - below);
      unsigned loc[kPerT], sum = 0;
#pragma unroll
      for (int u = 0; u < kPerT; ++u) {
        loc[u] = s_h[threadIdx.x * kPerT + u];
        sum += loc[u];
      }
      const int ln = threadIdx.x & 63, wv = threadIdx.x >> 6;
      unsigned inc = sum;
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        const unsigned y = __shfl_up(inc, off, 64);
        if (ln >= off) inc += y;
      }
      if (ln == 63) s_w[wv] = inc;
      __syncthreads();
      unsigned before = inc - sum;
      for (int w2 = 0; w2 < wv; ++w2) before += s_w[w2];
      if (before < need && before + sum >= need) {  // exactly one thread
        unsigned cum = before;
        int u = 0;
        for (; u < kPerT - 1; ++u) {
          if (cum + loc[u] >= need) break;
          cum += loc[u];
        }
        s_bin = threadIdx.x * kPerT + u;
        s_sel[1] = need - cum;
      }
    }
    __syncthreads();
    const int bin = s_bin;
    if (s_h[bin] <= (unsigned)kSelBinCap) {
      constexpr int kU = 8;
      for (long long i0 = threadIdx.x; i0 < nin; i0 += kSelThreads * kU) {
        unsigned long long kk[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u)
          kk[u] = i0 + u * kSelThreads < nin ? cand[1 + i0 + u * kSelThreads] : ~0ull;
#pragma unroll
        for (int u = 0; u < kU; ++u)
          if (i0 + u * kSelThreads < nin && (int)(((kk[u] >> 32) - lo) >> sh) == bin)
            s_k[atomicAdd(&s_nb, 1)] = kk[u];
      }
      __syncthreads();
      if (threadIdx.x == 0) tr[2] = wall_clock64();
      const int nb = s_nb;
      const unsigned long long want = s_sel[1] - 1;  // 0-based rank in the bin
      for (int j = threadIdx.x; j < nb; j += kSelThreads) {
        const unsigned long long kj = s_k[j];
        unsigned long long r = 0;
        for (int u = 0; u < nb; ++u) r += s_k[u] < kj;
        if (r == want) cand[0] = kj;  // keys are unique (id in the low bits)
      }
      if (threadIdx.x == 0) {
        tr[3] = wall_clock64();
        tr[4] = (unsigned long long)nin;
        tr[5] = (unsigned long long)s_h[bin];
      }
      return;
    }
    __syncthreads();
  }
  // radix select, 8 passes of one key byte: of the window keys (a crowded
  // bin) or of all n keys (T outside the window)
  const long long nk = win ? nin : n;
  if (threadIdx.x == 0) {
    s_sel[0] = 0;
    s_sel[1] = (unsigned long long)(win ? count - below : count);
  }
  unsigned long long mask = 0;
  for (int pass = 0; pass < 8; ++pass) {
    const int shift = 56 - 8 * pass;
    if (threadIdx.x < 256) s_h[threadIdx.x] = 0;
    __syncthreads();
    const unsigned long long prefix = s_sel[0];
    for (long long i = threadIdx.x; i < nk; i += kSelThreads) {
      const unsigned long long key = win ? cand[1 + i] : perc_rand_key(seed, (unsigned)(i + 1));
      if ((key & mask) == prefix) atomicAdd(&s_h[(key >> shift) & 255u], 1u);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      unsigned long long need = s_sel[1], cum = 0;
      int b = 0;
      for (; b < 255; ++b) {
        if (cum + s_h[b] >= need) break;
        cum += s_h[b];
      }
      s_sel[1] = need - cum;
      s_sel[0] = prefix | (unsigned long long)b << shift;
    }
    mask |= 0xFFull << shift;
    __syncthreads();
  }
  if (threadIdx.x == 0) cand[0] = s_sel[0];
}

// occupy every id whose key is <= T (T = the count-th smallest key);
// occ[id - 1 + base] (bonds: base 0, 0-based; sites: base 1, socc[id])
// (Tp: the threshold in device memory, k_select_final's; null: all n)
__global__ __launch_bounds__(kBlock) void k_occupy_rand(long long n, unsigned long long seed,
                                                         const unsigned long long* Tp, int base,
                                                         uint8_t* occ) {
  const long long i = (long long)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const unsigned long long T = Tp ? *Tp : ~0ull;
  occ[i + base] = perc_rand_key(seed, (unsigned)(i + 1)) <= T ? 1 : 0;
}

__global__ void k_occupy_sites(const int* order, int count, int t, uint8_t* socc) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= count) return;
  const int id = order[k];
  if (id > 0 && id <= t) socc[id] = 1;
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

__device__ __forceinline__ void unite(int* parent, int a, int b) {
  while (true) {
    a = find_root(parent, a);
    b = find_root(parent, b);
    if (a == b) return;
    if (a < b) { const int tmp = a; a = b; b = tmp; }
    const int old = atomicCAS(&parent[a], a, b);
    if (old == a) return;
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
__global__ __launch_bounds__(kCcThreads) void k_cc_merge(Geom g, int kind, const int* bond_first,
                                                         const uint8_t* bocc,
                                                         const uint8_t* socc, int* parent,
                                                         uint8_t* member, int nseg, int nfull) {
  const int ntx = cdiv(g.m, kCcW), lane = threadIdx.x & 63;
  int row, c;
  if ((int)blockIdx.x < nfull * nseg) {  // A: block-top row, columns of segment
    row = (blockIdx.x / nseg) * kCcH + kCcH - 1;
    c = (blockIdx.x % nseg) * kCcThreads + threadIdx.x;
  } else {  // B: candidate column j, rows of block rb (block-top rows are A's)
    const int e = blockIdx.x - nfull * nseg, nrb = cdiv(g.n, kCcThreads);
    const int j = e / nrb;
    row = (e % nrb) * kCcThreads + threadIdx.x;
    c = j == 2 * ntx ? g.m - 1 : min((j >> 1) * kCcW + (j & 1) * (kCcW - 1), g.m - 1);
    if (row % kCcH == kCcH - 1) row = g.n;  // (part A's)
  }
  const int s = row * g.m + c + 1;
  bool site = row < g.n && c < g.m && s <= g.t - 1 && (kind == PERC_BOND || socc[s]);
  int nn[6] = {0, 0, 0, 0, 0, 0}, fb = 0;
  if (site) {
    nearestn_rc(g, s, row, c, nn);
    fb = bond_first[s];
  }
  int r = 0;
  for (int k = 0; k < g.scn; ++k) {  // (uniform trip count: the shuffles below)
    const int q = nn[k];
    const bool fwd = site && q > s;
    bool want = fwd && cc_link(kind, bocc, socc, fb + r, s, q);
    r += fwd ? 1 : 0;
    if (want) {
      const int qrow = div_m(g, q - 1), qcol = q - 1 - qrow * g.m;
      want = !(qrow / kCcH == row / kCcH && qcol / kCcW == c / kCcW);  // inside: k_cc_tile's
    }
    if (want && kind == PERC_BOND) member[q] = 1;
    const int a = want ? parent[s] : -1, b = want ? parent[q] : -1;
    const int pa = __shfl_up(a, 1, 64), pb = __shfl_up(b, 1, 64);
    if (want && !(lane > 0 && pa == a && pb == b)) unite(parent, a, b);
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

// final flattening: a read-only walk, then each thread writes only its own
// entry (path halving here would let one thread overwrite another's freshly
// written root with an intermediate ancestor); counts the clusters (member
// roots)
__global__ __launch_bounds__(kCcThreads) void k_cc_compress(int t, int* parent,
                                                            const uint8_t* member,
                                                            int* nclusters) {
  // four sites per thread and step, their first parent loads issued together
  constexpr int kU = 4;
  int cnt = 0;
  for (long long b = (long long)blockIdx.x * kCcThreads * kU + threadIdx.x + 1; b <= t;
       b += (long long)gridDim.x * kCcThreads * kU) {
    int p0[kU];
#pragma unroll
    for (int k = 0; k < kU; ++k) {
      const long long s = b + k * kCcThreads;
      p0[k] = s <= t ? parent[s] : 0;
    }
#pragma unroll
    for (int k = 0; k < kU; ++k) {
      const long long s = b + k * kCcThreads;
      if (s > t) continue;
      int x = (int)s, p = p0[k];
      while (p != x) {
        x = p;
        p = parent[x];
      }
      parent[s] = x;
      cnt += x == s && member[s];
    }
  }
  block_count_add(cnt, nclusters);
}

// Spanning clusters (bondc.f:413-456, site.f:309-344, sitebond.f:423-458).
// The root is the component's minimum site, so a component reaches the
// bottom row (bond: a bond with b1 <= m; site / mixed: an occupied site
// there) iff its root is <= m; it reaches the top row (bond: b2 > t-m; site:
// an occupied site) iff one of the m top-row sites is a member of it.  One
// workgroup: flag[root] for the top-row members whose root is <= m, then the
// flagged roots in ascending order (ballot compaction) -> counters[0] =
// count, counters[8..] = the first kMaxSpanList roots.
__global__ __launch_bounds__(1024) void k_span_top(Geom g, const int* parent,
                                                   const uint8_t* member, uint8_t* flag,
                                                   int* counters) {
  __shared__ int s_w[16];
  __shared__ int s_base;
  const int m = g.m;
  for (int c = threadIdx.x; c <= m; c += 1024) flag[c] = 0;
  if (threadIdx.x == 0) s_base = 0;
  __syncthreads();
  for (int c = threadIdx.x; c < m; c += 1024) {
    const int s = g.t - m + 1 + c;
    if (member[s]) {
      const int root = parent[s];
      if (root <= m) flag[root] = 1;
    }
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (int base = 1; base <= m; base += 1024) {
    const int c = base + threadIdx.x;
    const bool f = c <= m && flag[c];
    const unsigned long long b = __ballot(f);
    if (lane == 0) s_w[wid] = __popcll(b);
    __syncthreads();
    int off = s_base;
    for (int w = 0; w < wid; ++w) off += s_w[w];
    off += __popcll(b & ((1ull << lane) - 1ull));
    if (f && off < kMaxSpanList) counters[8 + off] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
      int tot = 0;
      for (int w = 0; w < 16; ++w) tot += s_w[w];
      s_base += tot;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) counters[0] = s_base;
}

// member sites of the component rooted at root (fixed grid, one atomic per
// workgroup)
__global__ __launch_bounds__(kCcThreads) void k_count_root(int t, const int* parent,
                                                           const uint8_t* member, int root,
                                                           int* counter) {
  constexpr int kU = 4;  // loads in flight per thread
  int cnt = 0;
  for (long long b = (long long)blockIdx.x * kCcThreads * kU + threadIdx.x + 1; b <= t;
       b += (long long)gridDim.x * kCcThreads * kU) {
    int pv[kU];
    uint8_t mv[kU];
#pragma unroll
    for (int k = 0; k < kU; ++k) {
      const long long s = b + k * kCcThreads;
      pv[k] = s <= t ? parent[s] : 0;
      mv[k] = s <= t ? member[s] : 0;
    }
#pragma unroll
    for (int k = 0; k < kU; ++k) cnt += mv[k] && pv[k] == root;
  }
  block_count_add(cnt, counter);
}

// cluster sizes c(label) of the reference (bond_perc.f:296-322: bonds of
// the cluster; site_perc.f: sites): each site adds its occupied forward
// bonds (bond) or itself (site) to its root's count, one atomic per site
// that contributes
__global__ __launch_bounds__(kCcThreads) void k_cluster_sizes(Geom g, int kind,
                                                              const int* bond_first,
                                                              const uint8_t* bocc,
                                                              const uint8_t* member,
                                                              const int* parent, int* size) {
  for (int s = blockIdx.x * kCcThreads + threadIdx.x + 1; s <= g.t; s += gridDim.x * kCcThreads) {
    int c = 0;
    if (kind == PERC_BOND) {
      for (int j = bond_first[s]; j < bond_first[s + 1]; ++j) c += bocc[j];
    } else {
      c = member[s];
    }
    if (c) atomicAdd(&size[parent[s]], c);
  }
}

// largest entry of size[1..t] (wave max, workgroup max, one atomicMax per
// workgroup)
__global__ __launch_bounds__(kCcThreads) void k_max_size(int t, const int* size, int* out) {
  __shared__ int s_m[kCcThreads / 64];
  int v = 0;
  for (int s = blockIdx.x * kCcThreads + threadIdx.x + 1; s <= t; s += gridDim.x * kCcThreads)
    v = max(v, size[s]);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = max(v, __shfl_xor(v, off, 64));
  if ((threadIdx.x & 63) == 0) s_m[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < kCcThreads / 64; ++w) v = max(v, s_m[w]);
    if (v) atomicMax(out, v);
  }
}

__global__ void k_canon(int t, const int* parent, const uint8_t* member, int* canon) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x + 1;
  if (s > t) return;
  canon[s - 1] = member[s] ? parent[s] : 0;
}

}  // namespace

hipError_t dev_occupy(perc_ctx* h, int kind, int nsites, const int* site_order, int nbonds,
                      const int* bond_order, bool device_src) {
  hipStream_t st = h->stream;
  DeviceBuffers& d = h->d;
  HIP_TRY(hipMemsetAsync(d.bocc, 0, (size_t)h->nb + 8, st));
  HIP_TRY(hipMemsetAsync(d.socc, 0, h->g.t + 8, st));
  if (kind != PERC_BOND && nsites > 0) {
    const int* src = site_order;
    if (!device_src) {
      HIP_TRY(hipMemcpyAsync(d.order, site_order, sizeof(int) * nsites, hipMemcpyHostToDevice, st));
      src = d.order;
    }
    k_occupy_sites<<<blocks_for(nsites), kBlock, 0, st>>>(src, nsites, h->g.t, d.socc);
    HIP_TRY(hipGetLastError());
  }
  if (kind != PERC_SITE && nbonds > 0) {
    const int* src = bond_order;
    if (!device_src) {
      HIP_TRY(hipMemcpyAsync(d.order, bond_order, sizeof(int) * nbonds, hipMemcpyHostToDevice, st));
      src = d.order;
    }
    k_occupy<<<blocks_for(nbonds), kBlock, 0, st>>>(src, nbonds, h->nb, d.bocc);
    HIP_TRY(hipGetLastError());
  }
  return hipSuccess;
}

// the count smallest keys of ids 1..n occupied: window count + one-workgroup
// select (k_select_window / k_select_final), then the occupation pass; no
// host synchronisation
static hipError_t occupy_rand_one(perc_ctx* h, long long n, long long count,
                                  unsigned long long seed, int base, uint8_t* occ) {
  hipStream_t st = h->stream;
  if (count <= 0) return hipSuccess;  // occ is zeroed by the caller
  const unsigned long long* Tp = nullptr;
  if (count < n) {
    if (!h->d.sel_hist) HIP_TRY(dmalloc(&h->d.sel_hist, 2));
    if (!h->d.sel_cand) HIP_TRY(dmalloc(&h->d.sel_cand, (size_t)kSelCap + 1 + 16));
    // window: T's hash is count/n * 2^32 give or take the binomial spread
    // sqrt(n q (1-q)) keys; +-(8 sigma + 256) keys of hash width
    const double q = (double)count / (double)n;
    const double wkeys = 8.0 * std::sqrt((double)n * q * (1.0 - q)) + 256.0;
    const double two32 = 4294967296.0, c = q * two32, w = wkeys / (double)n * two32;
    unsigned long long lo = c - w <= 0.0 ? 0ull : (unsigned long long)(c - w);
    unsigned long long hi = c + w >= two32 ? (1ull << 32) : (unsigned long long)(c + w) + 1;
    const char* full = std::getenv("PERC_SELECT_FULL");  // tests: the exact slow path
    if (full && full[0] == '1') lo = hi = 0;
    HIP_TRY(hipMemsetAsync(h->d.sel_hist, 0, 2 * sizeof(unsigned), st));
    const int G = (int)std::min<long long>(cdiv(n, kBlock), 2048);
    k_select_window<<<G, kBlock, 0, st>>>(n, seed, lo, hi, h->d.sel_hist, h->d.sel_cand);
    HIP_TRY(dbg_sync(st, "k_select_window"));
    k_select_final<<<1, kSelThreads, 0, st>>>(n, seed, count, lo, hi, h->d.sel_hist,
                                              h->d.sel_cand);
    HIP_TRY(dbg_sync(st, "k_select_final"));
    Tp = h->d.sel_cand;
    if (std::getenv("PERC_SELECT_TRACE")) {
      unsigned long long tr[6];
      HIP_TRY(hipMemcpyAsync(tr, h->d.sel_cand + 1 + kSelCap, sizeof(tr), hipMemcpyDeviceToHost, st));
      HIP_TRY(hipStreamSynchronize(st));
      std::fprintf(stderr, "select trace: hist %llu bin %llu rank %llu ticks; nin %llu bin %llu\n",
                   tr[1] - tr[0], tr[2] - tr[1], tr[3] - tr[2], tr[4], tr[5]);
    }
  }
  k_occupy_rand<<<cdiv(n, kBlock), kBlock, 0, st>>>(n, seed, Tp, base, occ);
  return hipGetLastError();
}

hipError_t dev_occupy_random(perc_ctx* h, int kind, int nsites, int nbonds,
                             unsigned long long seed) {
  hipStream_t st = h->stream;
  DeviceBuffers& d = h->d;
  HIP_TRY(hipMemsetAsync(d.bocc, 0, (size_t)h->nb + 8, st));
  HIP_TRY(hipMemsetAsync(d.socc, 0, h->g.t + 8, st));
  if (kind != PERC_BOND) HIP_TRY(occupy_rand_one(h, h->g.t, nsites, seed, 1, d.socc));
  if (kind != PERC_SITE)
    HIP_TRY(occupy_rand_one(h, h->nb, nbonds, perc_mix64(seed ^ 0x5DEECE66Dull), 0, d.bocc));
  return hipSuccess;
}

hipError_t dev_label(perc_ctx* h, int* nspan, int* span_list, int* nclusters) {
  const Geom& g = h->g;
  hipStream_t st = h->stream;
  DeviceBuffers& d = h->d;
  const int kind = h->last.kind;
  HIP_TRY(hipMemsetAsync(d.counters, 0, sizeof(int) * (8 + kMaxSpanList), st));
  const int tiles = cdiv(g.m, kCcW) * cdiv(g.n, kCcH);
  unsigned long long* ttr = nullptr;  // PERC_TILE_TRACE: per-workgroup phase stamps
  static const bool ttrace = std::getenv("PERC_TILE_TRACE") != nullptr;
  if (ttrace) HIP_TRY(dmalloc(&ttr, (size_t)tiles * 5));
  k_cc_tile<<<tiles, kCcThreads, 0, st>>>(g, kind, d.bond_first, d.bocc, d.socc, d.parent,
                                          d.member, (int)h->bf_closed, ttr);
  if (ttrace) {
    std::vector<unsigned long long> v((size_t)tiles * 5);
    HIP_TRY(hipMemcpyAsync(v.data(), ttr, v.size() * 8, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    HIP_TRY(hipFree(ttr));
    unsigned long long lo = ~0ull, hi = 0;
    double ph[4] = {0, 0, 0, 0};
    for (int b = 0; b < tiles; ++b) {
      lo = std::min(lo, v[5 * b]);
      hi = std::max(hi, v[5 * b + 4]);
      for (int j = 0; j < 4; ++j) ph[j] += (double)(v[5 * b + j + 1] - v[5 * b + j]);
    }
    std::fprintf(stderr, "tile trace: span %llu ticks; per-WG avg phase1 %.1f runs %.1f unions %.1f flatten %.1f\n",
                 hi - lo, ph[0] / tiles, ph[1] / tiles, ph[2] / tiles, ph[3] / tiles);
  }
  HIP_TRY(dbg_sync(st, "k_cc_tile"));
  const int nseg = cdiv(g.m, kCcThreads);
  const int nfull = g.n / kCcH;  // rows kCcH-1, 2kCcH-1, ... (< n)
  const int ncand = 2 * cdiv(g.m, kCcW) + 1;
  k_cc_merge<<<nfull * nseg + ncand * cdiv(g.n, kCcThreads), kCcThreads, 0, st>>>(
      g, kind, d.bond_first, d.bocc, d.socc, d.parent, d.member, nseg, nfull);
  HIP_TRY(dbg_sync(st, "k_cc_merge"));
  k_cc_compress<<<std::min(cdiv(g.t, kCcThreads), kReduceGrid), kCcThreads, 0, st>>>(
      g.t, d.parent, d.member, d.counters + 1);
  HIP_TRY(dbg_sync(st, "k_cc_compress"));
  k_span_top<<<1, 1024, 0, st>>>(g, d.parent, d.member, d.top, d.counters);
  HIP_TRY(dbg_sync(st, "k_span_top"));
  int hc[8 + kMaxSpanList];
  HIP_TRY(hipMemcpyAsync(hc, d.counters, sizeof(hc), hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  *nspan = hc[0];
  *nclusters = hc[1];
  for (int i = 0; i < std::min(hc[0], kMaxSpanList); ++i) span_list[i] = hc[8 + i];
  return hipSuccess;
}

hipError_t dev_span_sites(perc_ctx* h, int root, int* count) {
  hipStream_t st = h->stream;
  HIP_TRY(hipMemsetAsync(h->d.counters + 2, 0, sizeof(int), st));
  k_count_root<<<std::min(cdiv(h->g.t, kCcThreads), kReduceGrid), kCcThreads, 0, st>>>(
      h->g.t, h->d.parent, h->d.member, root, h->d.counters + 2);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(count, h->d.counters + 2, sizeof(int), hipMemcpyDeviceToHost, st));
  return hipStreamSynchronize(st);
}

hipError_t dev_cluster_sizes(perc_ctx* h, int kind, int root, int* maxcs, int* rootsize) {
  DeviceBuffers& d = h->d;
  hipStream_t st = h->stream;
  const Geom& g = h->g;
  if (!d.csize) HIP_TRY(dmalloc(&d.csize, (size_t)g.t + 2));
  HIP_TRY(hipMemsetAsync(d.csize, 0, sizeof(int) * ((size_t)g.t + 2), st));
  HIP_TRY(hipMemsetAsync(d.counters + 3, 0, sizeof(int), st));
  const int G = std::min(cdiv(g.t, kCcThreads), kReduceGrid * 4);
  k_cluster_sizes<<<G, kCcThreads, 0, st>>>(g, kind, d.bond_first, d.bocc, d.member, d.parent,
                                            d.csize);
  HIP_TRY(dbg_sync(st, "k_cluster_sizes"));
  k_max_size<<<std::min(cdiv(g.t, kCcThreads), kReduceGrid), kCcThreads, 0, st>>>(g.t, d.csize,
                                                                                  d.counters + 3);
  HIP_TRY(dbg_sync(st, "k_max_size"));
  HIP_TRY(hipMemcpyAsync(maxcs, d.counters + 3, sizeof(int), hipMemcpyDeviceToHost, st));
  *rootsize = 0;
  if (root > 0 && root <= g.t)
    HIP_TRY(hipMemcpyAsync(rootsize, d.csize + root, sizeof(int), hipMemcpyDeviceToHost, st));
  return hipStreamSynchronize(st);
}

hipError_t dev_canon(perc_ctx* h, int* canon_out) {
  hipStream_t st = h->stream;
  int* tmp = nullptr;
  HIP_TRY(dmalloc(&tmp, h->g.t));
  k_canon<<<blocks_for(h->g.t), kBlock, 0, st>>>(h->g.t, h->d.parent, h->d.member, tmp);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(canon_out, tmp, sizeof(int) * h->g.t, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  return hipFree(tmp);
}

}  // namespace perc
