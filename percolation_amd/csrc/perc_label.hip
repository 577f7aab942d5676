// perc_label.hip -- occupancy and cluster labeling of libperc (gfx950):
// the occupation of sites / bonds (given orders or drawn on the device),
// the connected-component partition (Square/bondc.f:194-393,
// site.f:167-289), the spanning test, cluster sizes and canonical labels.
#include "perc_cc.h"

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
// workgroups per draw of k_select_final: the window keys of T's bin are
// picked out by kSelParts workgroups (a share each, appended to a list after
// the window keys), the last one to finish ranks them (one workgroup walked
// the ~93 K window keys of a 2^27-bond draw in 12 dependent rounds, 14 of its
// 19 us, PERC_SELECT_TRACE; PERC_SEL_PARTS, A/B probe builds only)
#ifdef PERC_SEL_PARTS
constexpr int kSelParts = PERC_SEL_PARTS;
#else
constexpr int kSelParts = 16;
#endif
// cand[] layout per draw: [0] T, [1 .. kSelCap] the window keys, then 16
// words (PERC_SELECT_TRACE stamps [0 .. 5], the bin list's count [8] and the
// parts' ticket [9]), then the bin's keys (kSelBinCap)
constexpr int kSelAux = 1 + kSelCap;
constexpr int kSelList = kSelAux + 16;
constexpr size_t kSelCand = (size_t)kSelList + kSelBinCap;
// occupancy bytes per thread and trip of k_select_window (one store of a
// kSelV-byte word; PERC_SEL_V: A/B probe builds only)
#ifdef PERC_SEL_V
constexpr int kSelV = PERC_SEL_V;
#else
constexpr int kSelV = 4;
#endif
template <int V> struct SelWord;
template <> struct SelWord<1> { using T = uint8_t; };
template <> struct SelWord<2> { using T = unsigned short; };
template <> struct SelWord<4> { using T = unsigned; };
template <> struct SelWord<8> { using T = unsigned long long; };
constexpr int kSelCnt = 4 + kSelBins;  // unsigned words per draw (cnt)
// bins of the window's hash range: (hash - lo) >> sh < kSelBins
__host__ __device__ inline int sel_shift(unsigned long long lo, unsigned long long hi) {
  const unsigned long long range = hi - lo;
  int bits = 0;
  while (bits < 64 && range > 1 && (range - 1) >> bits) ++bits;
  return bits > 12 ? bits - 12 : 0;
}
// One draw of perc_occupy_random: n ids, the count smallest keys occupied
// in occ[base .. base + n); the window [lo, hi) of T's hash; cnt: [0] keys
// below the window, [1] keys in it, [2] window valid, [3] unused, [4 ..]
// kSelBins bin counts of the window keys by hash; cand: [0] T, then the
// window's keys; the pad bytes occ[0 .. base) and npad at padp.  The
// site and bond draws of a mixed occupation run in one launch of each
// kernel: draw k owns the workgroups [g0, g0 + gn) (the select: workgroup
// k), so neither draw's tail or one-workgroup select idles the device alone.
struct SelDraw {
  long long n, count;
  unsigned long long seed, lo, hi;
  RandKeyCtx kc;
  int sh, base, npad, g0, gn;
  unsigned* cnt;
  unsigned long long* cand;
  uint8_t* occ;
  uint8_t* padp;
};
struct SelDraws {
  SelDraw d[2];
  int nd;
};
// the draw of workgroup b (a draw's range starts at its g0)
__device__ __forceinline__ SelDraw sel_draw(const SelDraws& D, int b) {
  return D.nd == 2 && b >= D.d[1].g0 ? D.d[1] : D.d[0];
}

__global__ __launch_bounds__(kBlock) void k_select_window(SelDraws D) {
  const SelDraw w = sel_draw(D, blockIdx.x);
  const long long n = w.n;
  const RandKeyCtx kc = w.kc;
  const unsigned long long lo = w.lo, hi = w.hi;
  const int sh = w.sh, base = w.base, npad = w.npad, bid = blockIdx.x - w.g0;
  unsigned* cnt = w.cnt;
  unsigned long long* cand = w.cand;
  uint8_t* occ = w.occ;
  if (bid == 0) {  // the pads: occ[0 .. base) and npad bytes at padp
    uint8_t* padp = w.padp;
    if ((int)threadIdx.x < npad) padp[threadIdx.x] = 0;
    if ((int)threadIdx.x < base) occ[threadIdx.x] = 0;
    if (threadIdx.x < 2) cand[kSelAux + 8 + threadIdx.x] = 0;  // k_select_final's list count and ticket
  }
  __shared__ unsigned long long s_c[kSelStage];
  __shared__ unsigned s_n, s_base, s_b[kBlock / 64];
  if (threadIdx.x == 0) s_n = 0;
  __syncthreads();
  unsigned below = 0;
  const int lane = threadIdx.x & 63;
  // a thread's kSelV bytes of one aligned word of occ per trip (one store
  // instead of kSelV byte stores): byte o is id o - base + 1, the bytes
  // outside ids 1..n are pads (written 0 here and by the pad stores above)
  const long long nw = cdiv(n + base, (long long)kSelV);
  for (long long j = (long long)bid * kBlock + threadIdx.x; j < nw; j += (long long)w.gn * kBlock) {
    using Word = typename SelWord<kSelV>::T;
    Word word = 0;
#pragma unroll
    for (int k = 0; k < kSelV; ++k) {
      const long long i = j * kSelV + k - base;
      const bool v = i >= 0 && i < n;
      const unsigned id = (unsigned)(i + 1);
      const unsigned long long hsh = perc_rand_hash32(kc, id);  // = perc_rand_key(seed, id) >> 32
      const unsigned long long key = hsh << 32 | id;
      // every key below the window is occupied, every key above it is not;
      // the window's keys (0 here) are decided by k_occupy_cand once T is known
      const bool b = v && hsh < lo;
      below += b;
      word |= (Word)(b ? 1u : 0u) << (8 * k);
      if (v && hsh >= lo && hsh < hi) {
        atomicAdd(&cnt[4 + (int)((hsh - lo) >> sh)], 1u);
        const unsigned slot = atomicAdd(&s_n, 1u);
        if (slot < (unsigned)kSelStage) {
          s_c[slot] = key;
        } else {  // a crowded workgroup: straight to the global list
          const unsigned idx = atomicAdd(&cnt[1], 1u);
          if (idx < (unsigned)kSelCap) cand[1 + idx] = key;
        }
      }
    }
    reinterpret_cast<Word*>(occ)[j] = word;
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

__global__ __launch_bounds__(kSelThreads) void k_select_final(SelDraws D) {
  const int part = blockIdx.x % kSelParts;
  const SelDraw w = blockIdx.x >= kSelParts ? D.d[1] : D.d[0];
  const long long n = w.n, count = w.count;
  const unsigned long long seed = w.seed, lo = w.lo, hi = w.hi;
  unsigned* cnt = w.cnt;
  unsigned long long* cand = w.cand;
  __shared__ unsigned s_h[kSelBins];
  __shared__ unsigned long long s_k[kSelBinCap];
  __shared__ unsigned long long s_sel[2];  // prefix, need
  __shared__ int s_bin, s_nb;
  unsigned long long* tr = cand + kSelAux;  // PERC_SELECT_TRACE stamps
  const bool p0 = part == 0;
  if (p0 && threadIdx.x == 0) tr[0] = wall_clock64();
  const long long below = cnt[0], nin = cnt[1];
  const bool win = count > below && count - below <= nin && nin <= kSelCap;
  // T inside the window and every window key gathered: k_select_window's
  // occupation stands and k_occupy_cand completes it; else k_occupy_cand
  // rewrites the whole occupation from T
  if (p0 && threadIdx.x == 0) cnt[2] = win ? 1u : 0u;
  if (win) {
    // bins of the window's hash range: (hash - lo) >> sh < kSelBins
    const int sh = sel_shift(lo, hi);
    // the bin counts k_select_window kept (a block-wide LDS histogram of the
    // window keys here cost ~15 us per draw of conflicting LDS atomics)
    for (int j = threadIdx.x; j < kSelBins; j += kSelThreads) s_h[j] = cnt[4 + j];
    if (threadIdx.x == 0) s_nb = 0;
    __syncthreads();
    if (p0 && threadIdx.x == 0) tr[1] = wall_clock64();
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
      // this part's share of the window keys: those of T's bin appended to
      // the bin list (their count is s_h[bin] over all parts)
      unsigned long long* list = cand + kSelList;
      unsigned long long* aux = cand + kSelAux;
      const long long per = (nin + kSelParts - 1) / kSelParts, i0 = part * per, i1 = min(nin, i0 + per);
      constexpr int kU = 8;
      for (long long ib = i0 + threadIdx.x; ib < i1; ib += kSelThreads * kU) {
        unsigned long long kk[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u)
          kk[u] = ib + u * kSelThreads < i1 ? cand[1 + ib + u * kSelThreads] : ~0ull;
#pragma unroll
        for (int u = 0; u < kU; ++u)
          if (ib + u * kSelThreads < i1 && (int)(((kk[u] >> 32) - lo) >> sh) == bin) {
            const unsigned long long at =
                __hip_atomic_fetch_add(&aux[8], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&list[at], kk[u], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
      }
      __syncthreads();
      if (threadIdx.x == 0) {  // the last part to finish ranks the bin's keys
        const unsigned long long tk =
            __hip_atomic_fetch_add(&aux[9], 1ull, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        s_nb = tk == (unsigned long long)(kSelParts - 1) ? 1 : 0;
      }
      __syncthreads();
      if (!s_nb) return;  // (uniform)
      const int nb = (int)s_h[bin];
      for (int j = threadIdx.x; j < nb; j += kSelThreads)
        s_k[j] = __hip_atomic_load(&list[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __syncthreads();
      if (threadIdx.x == 0) tr[2] = wall_clock64();
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
  // bin) or of all n keys (T outside the window) -- by the draw's first
  // part alone
  if (!p0) return;  // (uniform)
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

// the window's keys (cand[1 ..], id in the low 32 bits) at or below T; when
// T fell outside the window (cnt[2] == 0, rare) the whole occupation is
// rewritten from T instead, grid-stride over all n ids (one launch either
// way: an empty second launch cost ~5 us per draw)
__global__ __launch_bounds__(kBlock) void k_occupy_cand(SelDraws D) {
  const SelDraw w = sel_draw(D, blockIdx.x);
  const unsigned* cnt = w.cnt;
  const unsigned long long* cand = w.cand;
  const int base = w.base, bid = blockIdx.x - w.g0;
  uint8_t* occ = w.occ;
  const long long n = w.n;
  const RandKeyCtx kc = w.kc;
  const unsigned long long T = cand[0];
  if (!cnt[2]) {
    for (long long i = (long long)bid * kBlock + threadIdx.x; i < n; i += (long long)w.gn * kBlock) {
      const unsigned id = (unsigned)(i + 1);
      occ[i + base] = ((unsigned long long)perc_rand_hash32(kc, id) << 32 | id) <= T ? 1 : 0;
    }
    return;
  }
  const unsigned nin = cnt[1];
  for (unsigned j = bid * kBlock + threadIdx.x; j < nin; j += w.gn * kBlock) {
    const unsigned long long key = cand[1 + j];
    if (key <= T) occ[(long long)(key & 0xFFFFFFFFull) - 1 + base] = 1;
  }
}

__global__ void k_occupy_sites(const int* order, int count, int t, uint8_t* socc) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= count) return;
  const int id = order[k];
  if (id > 0 && id <= t) socc[id] = 1;
}

// Spanning clusters (bondc.f:413-456, site.f:309-344, sitebond.f:423-458).
// The root is the component's minimum site, so a component reaches the
// bottom row (bond: a bond with b1 <= m; site / mixed: an occupied site
// there) iff its root is <= m; it reaches the top row (bond: b2 > t-m; site:
// an occupied site) iff one of the m top-row sites is a member of it.  One
// workgroup: flag[root] for the top-row members whose root is <= m (flags in
// LDS where m < kSpanLds), then the flagged roots in ascending order -- each
// thread counts its own run of consecutive flags, one workgroup scan ->
// counters[0] = count, counters[8..] = the first kMaxSpanList roots.  (The
// ballot compaction over 1024-flag windows in global memory, three
// barriers a window, cost ~10 us at m = 8192.)
// part (npart > 0): the cluster count as the sum of the wave tiles' member
// roots and the merge's negated hooks -> counters[1]
constexpr int kSpanLds = 32768;
template <bool LF>
__global__ __launch_bounds__(1024) void k_span_top(Geom g, const int* parent,
                                                   const uint8_t* member, uint8_t* gflag,
                                                   int* counters, const int* part, int npart,
                                                   int* dcopy = nullptr) {
  __shared__ uint8_t s_fl[LF ? kSpanLds : 1];
  __shared__ int s_w[16];
  uint8_t* flag = LF ? s_fl : gflag;
  const int m = g.m;
  for (int c = threadIdx.x; c <= m; c += 1024) flag[c] = 0;
  // the cluster count's partials (npart > 0) loaded first, in flight
  // while the chains below are walked: up to kPartU per thread
  constexpr int kPartU = 64;
  int pv[kPartU];
#pragma unroll
  for (int u = 0; u < kPartU; ++u) {
    const int i = (int)threadIdx.x + 1024 * u;
    pv[u] = i < npart ? part[i] : 0;
  }
  __syncthreads();
  // the top row's chains (parents may not be flattened yet: dev_flatten),
  // a thread's U sites chased in lockstep: every hop issues their U parent
  // loads together (one site after another: 33 us per labeling at m = 8192)
  constexpr int U = 8;
  for (int c0 = threadIdx.x; c0 < m; c0 += 1024 * U) {
    int x[U];
    bool act[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int c = c0 + 1024 * u, s = g.t - m + 1 + c;
      act[u] = c < m && member[s];
      x[u] = act[u] ? parent[s] : 0;
    }
    while (true) {
      int y[U];
#pragma unroll
      for (int u = 0; u < U; ++u) y[u] = act[u] ? parent[x[u]] : x[u];
      bool more = false;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        more |= y[u] != x[u];
        x[u] = y[u];
      }
      if (!more) break;
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (act[u] && x[u] <= m) flag[x[u]] = 1;
  }
  __syncthreads();
  // thread t's run of flags: roots c0 .. c0 + K - 1 (1-based, <= m)
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int K = cdiv(m, 1024), c0 = 1 + (int)threadIdx.x * K;
  int cnt = 0;
  for (int k = 0; k < K; ++k) cnt += c0 + k <= m && flag[c0 + k];
  int inc = cnt;  // inclusive scan over the wave, then over the waves
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int y = __shfl_up(inc, off, 64);
    if (lane >= off) inc += y;
  }
  if (lane == 63) s_w[wid] = inc;
  __syncthreads();
  int off = inc - cnt, tot = 0;
  for (int w = 0; w < 16; ++w) {
    off += w < wid ? s_w[w] : 0;
    tot += s_w[w];
  }
  for (int k = 0; k < K && off < kMaxSpanList; ++k)
    if (c0 + k <= m && flag[c0 + k]) {
      if (dcopy && off == 0) dcopy[8] = c0 + k;  // (the first spanning root)
      counters[8 + off++] = c0 + k;
    }
  if (threadIdx.x == 0) {
    counters[0] = tot;
    if (dcopy) {  // device copies for k_cc_compress_spec: the count; its ticket and sum zeroed
      dcopy[0] = tot;
      dcopy[4] = 0;
      dcopy[5] = 0;
    }
  }
  if (npart > 0) {  // (uniform)
    int v = 0;
#pragma unroll
    for (int u = 0; u < kPartU; ++u) v += pv[u];
    for (int i = (int)threadIdx.x + 1024 * kPartU; i < npart; i += 1024) v += part[i];  // (past 64 K partials)
    v = wave_sum_int(v);
    __syncthreads();
    if (lane == 0) s_w[wid] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
      int t2 = 0;
      for (int w = 0; w < 16; ++w) t2 += s_w[w];
      counters[1] = t2;
    }
  }
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

// the count smallest keys of ids 1..n occupied, occ[base .. base + n):
// k_select_window (every key hashed once: the keys below the window
// occupied, the others not, the window's keys gathered), the one-workgroup
// select of T (k_select_final), then the window's keys at or below T
// (k_occupy_cand); when T fell outside the window k_occupy_cand rewrites the
// whole occupation from T instead.  No host synchronisation.  A draw with
// nothing to select (count <= 0 or >= n) is a memset.
static hipError_t sel_prepare(perc_ctx* h, long long n, long long count, unsigned long long seed, int base,
                              uint8_t* occ, unsigned* cnt, unsigned long long* cand, uint8_t* padp, int npad,
                              SelDraws& D) {
  hipStream_t st = h->stream;
  if (count <= 0 || count >= n) {
    HIP_TRY(hipMemsetAsync(occ + base, count <= 0 ? 0 : 1, (size_t)n, st));
    if (base) HIP_TRY(hipMemsetAsync(occ, 0, (size_t)base, st));
    return npad ? hipMemsetAsync(padp, 0, (size_t)npad, st) : hipSuccess;
  }
  // window: T's hash is count/n * 2^32 give or take the binomial spread
  // sqrt(n q (1-q)) keys; +-(8 sigma + 256) keys of hash width
  const double q = (double)count / (double)n;
  const double wkeys = 8.0 * std::sqrt((double)n * q * (1.0 - q)) + 256.0;
  const double two32 = 4294967296.0, c = q * two32, w = wkeys / (double)n * two32;
  unsigned long long lo = c - w <= 0.0 ? 0ull : (unsigned long long)(c - w);
  unsigned long long hi = c + w >= two32 ? (1ull << 32) : (unsigned long long)(c + w) + 1;
  const char* full = std::getenv("PERC_SELECT_FULL");  // tests: the exact slow path
  if (full && full[0] == '1') lo = hi = 0;
  SelDraw& x = D.d[D.nd++];
  x.n = n;
  x.count = count;
  x.seed = seed;
  x.lo = lo;
  x.hi = hi;
  x.kc = perc_rand_key_ctx(seed);
  x.sh = sel_shift(lo, hi);
  x.base = base;
  x.npad = npad;
  x.cnt = cnt;
  x.cand = cand;
  x.occ = occ;
  x.padp = padp;
  return hipSuccess;
}

hipError_t dev_occupy_random(perc_ctx* h, int kind, int nsites, int nbonds,
                             unsigned long long seed) {
  hipStream_t st = h->stream;
  DeviceBuffers& d = h->d;
  // one memset: both draws' counters and bin counts; the drawn ranges are
  // written whole and their pad bytes by the draw (socc[0] and socc[t+1 ..
  // t+8) with the sites, bocc[nb .. nb+8) with the bonds); an undrawn kind
  // is zeroed whole
  constexpr size_t kCand = kSelCand;  // per draw: T, the window keys, stamps / list count / ticket, the bin list
  if (!d.sel_hist) HIP_TRY(dmalloc(&d.sel_hist, 2 * kSelCnt));
  if (!d.sel_cand) HIP_TRY(dmalloc(&d.sel_cand, 2 * kCand));
  HIP_TRY(hipMemsetAsync(d.sel_hist, 0, sizeof(unsigned) * 2 * kSelCnt, st));
  if (kind == PERC_SITE) HIP_TRY(hipMemsetAsync(d.bocc, 0, (size_t)h->nb + 8, st));
  if (kind == PERC_BOND) HIP_TRY(hipMemsetAsync(d.socc, 0, h->g.t + 8, st));
  SelDraws D{};
  if (kind != PERC_BOND)
    HIP_TRY(sel_prepare(h, h->g.t, nsites, seed, 1, d.socc, d.sel_hist, d.sel_cand, d.socc + h->g.t + 1, 7, D));
  if (kind != PERC_SITE)
    HIP_TRY(sel_prepare(h, h->nb, nbonds, perc_mix64(seed ^ 0x5DEECE66Dull), 0, d.bocc, d.sel_hist + kSelCnt,
                        d.sel_cand + kCand, d.bocc + h->nb, 8, D));
  if (D.nd == 0) return hipSuccess;
  // the window pass: a draw's share of 2048 workgroups by its size (>= 1);
  // the window-key pass: kSelCap / kBlock workgroups a draw
  long long tot = 0;
  for (int k = 0; k < D.nd; ++k) tot += D.d[k].n;
  int G = 0;
  for (int k = 0; k < D.nd; ++k) {
    const long long share = D.nd == 1 ? 2048 : std::max<long long>(1, 2048 * D.d[k].n / tot);
    D.d[k].g0 = G;
    D.d[k].gn = (int)std::min<long long>(cdiv(D.d[k].n, kBlock), share);
    G += D.d[k].gn;
  }
  k_select_window<<<G, kBlock, 0, st>>>(D);
  HIP_TRY(dbg_sync(st, "k_select_window"));
  k_select_final<<<D.nd * kSelParts, kSelThreads, 0, st>>>(D);
  HIP_TRY(dbg_sync(st, "k_select_final"));
  if (std::getenv("PERC_SELECT_TRACE")) {
    for (int k = 0; k < D.nd; ++k) {
      unsigned long long tr[6];
      HIP_TRY(hipMemcpyAsync(tr, D.d[k].cand + 1 + kSelCap, sizeof(tr), hipMemcpyDeviceToHost, st));
      HIP_TRY(hipStreamSynchronize(st));
      std::fprintf(stderr, "select trace (draw %d): hist %llu bin %llu rank %llu ticks; nin %llu bin %llu\n", k,
                   tr[1] - tr[0], tr[2] - tr[1], tr[3] - tr[2], tr[4], tr[5]);
    }
  }
  const int GC = cdiv(kSelCap, kBlock);
  for (int k = 0; k < D.nd; ++k) {
    D.d[k].g0 = k * GC;
    D.d[k].gn = GC;
  }
  k_occupy_cand<<<GC * D.nd, kBlock, 0, st>>>(D);
  return dbg_sync(st, "k_occupy_cand");
}

static hipError_t label_finish(perc_ctx* h, int* nspan, int* span_list, int* nclusters,
                                const int* part = nullptr, int npart = 0, bool spec_span = false);

hipError_t dev_label(perc_ctx* h, int* nspan, int* span_list, int* nclusters, bool spec_span) {
  const Geom& g = h->g;
  hipStream_t st = h->stream;
  DeviceBuffers& d = h->d;
  const int kind = h->last.kind;
  // (the open square lattice, every kind -- the tiles' partials count the
  // clusters: k_span_top writes every counter the labeling reads, no memset)
  const bool wave = g.lattice == kSquare && !g.pbc && h->bf_open_sq && !std::getenv("PERC_TILE_TRACE");
#if defined(PERC_LABEL_COPYBACK)  // (A/B probe builds only: round 6's memset for the bond kind)
  if (!wave || kind == PERC_BOND) HIP_TRY(hipMemsetAsync(d.counters, 0, sizeof(int) * (8 + kMaxSpanList), st));
#else
  if (!wave) HIP_TRY(hipMemsetAsync(d.counters, 0, sizeof(int) * (8 + kMaxSpanList), st));
#endif
  // the open square lattice: one wave per 128 x 16 block walking its rows
  // (k_cc_tile_w; tile 91.7 vs 190.6 us for the 128 x 32 LDS union-find
  // blocks at L = 4096, profiles/r4_13_cc_bench_L4096.txt); else the LDS
  // union-find blocks
  if (wave) {
    constexpr int H = kCcWaveH;
    const int G = cdiv(g.m, kCcW) * cdiv(g.n, H);
    const unsigned nbb = (unsigned)h->nb + 8u;
    const int nseg = cdiv(g.m, kCcThreads), nfull = g.n / H;
    // (the merge's grid: kMergeU sites per thread)
    constexpr int MU = kMergeU > 0 ? kMergeU : 1;
    const int nsegu = cdiv(g.m, kCcThreads * MU);
    const int GM = nfull * nsegu + (cdiv(g.m, kCcW) - 1) * cdiv(g.n, kCcThreads * MU);
    // the cluster count from the tiles' member roots and the merge's hooks
    // (every kind: the bond tile reads the links that cross into its edge
    // sites for their member flags), no pass over the parents
    if (!d.ccpart) HIP_TRY(dmalloc(&d.ccpart, (size_t)G + GM));
    int* part = d.ccpart;
    if (kind == PERC_BOND)
      k_cc_tile_w<H, PERC_BOND, kCcWaveDBond><<<G, 64, 0, st>>>(g, d.bocc, d.socc, d.parent, d.member, nbb, part);
    // (site and mixed kinds: the ballot-mask walk, 95.6 vs 103.8 us mixed at
    // L = 4096, 273.7 vs 298.5 at 8192; the bond kind's is 2 % slower with
    // it, profiles/r5_10_cc_bench_L*.txt)
    else if (kind == PERC_SITE)
      k_cc_tile_w<H, PERC_SITE, 2, true><<<G, 64, 0, st>>>(g, d.bocc, d.socc, d.parent, d.member, nbb, part);
    else k_cc_tile_w<H, PERC_SITEBOND, 2, true><<<G, 64, 0, st>>>(g, d.bocc, d.socc, d.parent, d.member, nbb, part);
    HIP_TRY(dbg_sync(st, "k_cc_tile_w"));
    // the square lattice's merge: 107 vs 163 us mixed, 153 vs 191 bond at
    // L = 8192 (profiles/r5_11_cc_bench_L8192.txt)
    int* hk = part + G;
    if (GM == 0) {  // one block: nothing crosses a block edge
    } else if constexpr (kMergeU > 0) {
      if (kind == PERC_BOND)
        k_cc_merge_squ<H, PERC_BOND, MU><<<GM, kCcThreads, 0, st>>>(g, d.bocc, d.socc, d.parent, d.member, nbb,
                                                                    nsegu, nfull, hk);
      else if (kind == PERC_SITE)
        k_cc_merge_squ<H, PERC_SITE, MU><<<GM, kCcThreads, 0, st>>>(g, d.bocc, d.socc, d.parent, d.member, nbb,
                                                                    nsegu, nfull, hk);
      else
        k_cc_merge_squ<H, PERC_SITEBOND, MU><<<GM, kCcThreads, 0, st>>>(g, d.bocc, d.socc, d.parent, d.member,
                                                                        nbb, nsegu, nfull, hk);
    } else if (kind == PERC_BOND)
      k_cc_merge_sq<H, PERC_BOND><<<GM, kCcThreads, 0, st>>>(g, d.bocc, d.socc, d.parent, d.member, nseg, nfull, hk);
    else if (kind == PERC_SITE)
      k_cc_merge_sq<H, PERC_SITE><<<GM, kCcThreads, 0, st>>>(g, d.bocc, d.socc, d.parent, d.member, nseg, nfull, hk);
    else
      k_cc_merge_sq<H, PERC_SITEBOND><<<GM, kCcThreads, 0, st>>>(g, d.bocc, d.socc, d.parent, d.member, nseg, nfull,
                                                                 hk);
    HIP_TRY(dbg_sync(st, "k_cc_merge_sq"));
    return label_finish(h, nspan, span_list, nclusters, part, G + GM, spec_span);
  }
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
  k_cc_merge<kCcH><<<nfull * nseg + ncand * cdiv(g.n, kCcThreads), kCcThreads, 0, st>>>(
      g, kind, d.bond_first, d.bocc, d.socc, d.parent, d.member, nseg, nfull);
  HIP_TRY(dbg_sync(st, "k_cc_merge"));
  return label_finish(h, nspan, span_list, nclusters);
}

// every parent to its root, cluster count, spanning roots, read-back
static hipError_t label_finish(perc_ctx* h, int* nspan, int* span_list, int* nclusters, const int* part,
                               int npart, bool spec_span) {
  const Geom& g = h->g;
  hipStream_t st = h->stream;
  DeviceBuffers& d = h->d;
  // the clusters are the member roots, countable before the parents are
  // flattened; k_cc_compress runs when a consumer of the roots needs it
  // (dev_flatten: assembly, bond masks, span sizes, cluster sizes, canonical
  // labels) -- a labeling that spans nothing (config 5 as stated, the
  // threshold scans' probes) does without it
  h->flat = false;
  h->span_count = -1;
  if (npart == 0) {
    k_cc_count_roots<<<std::min(cdiv(g.t, kCcThreads * 4), kReduceGrid), kCcThreads, 0, st>>>(
        g.t, d.parent, d.member, d.counters + 1);
    HIP_TRY(dbg_sync(st, "k_cc_count_roots"));
  }
  constexpr int kHc = 8 + kMaxSpanList;
#if defined(PERC_LABEL_PAGEABLE)  // (A/B probe builds only: a stack array)
  int hcs[kHc];
  const int* hc = hcs;
  int* out = d.counters;
  const bool direct = false;
#else
  if (!h->pin) HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&h->pin), sizeof(int) * kHc, hipHostMallocCoherent));
  const int* hc = h->pin;
  // with the cluster count from the partials (npart > 0) k_span_top writes
  // every word the host reads: straight into the pinned words (coherent
  // host memory, visible once the stream is synchronised) -- no copy after
  // it.  (k_cc_count_roots' count is in device memory: copied back.)
#if defined(PERC_LABEL_COPYBACK)  // (A/B probe builds only)
  const bool direct = false;
#else
  const bool direct = npart > 0;
#endif
  int* out = d.counters;
  if (direct) HIP_TRY(hipHostGetDevicePointer(reinterpret_cast<void**>(&out), h->pin, 0));
#endif
  // (perc_label, when the previous labeling spanned: the spanning cluster's
  // flatten and site count enqueued behind the spanning test, read back in
  // the same synchronisation -- k_cc_compress_spec does nothing if nothing
  // spans)
#if defined(PERC_LABEL_NOSPEC)  // (A/B probe builds only: the count after a second synchronisation)
  const bool spec = false && spec_span;
#else
  const bool spec = direct && spec_span;
#endif
  int* dcopy = spec ? d.counters : nullptr;
  if (g.m < kSpanLds) k_span_top<true><<<1, 1024, 0, st>>>(g, d.parent, d.member, d.top, out, part, npart, dcopy);
  else k_span_top<false><<<1, 1024, 0, st>>>(g, d.parent, d.member, d.top, out, part, npart, dcopy);
  HIP_TRY(dbg_sync(st, "k_span_top"));
  if (spec) {
    k_cc_compress_spec<<<std::min(cdiv(g.t, kCcThreads * kCcCompressU), kReduceGrid), kCcThreads, 0, st>>>(
        g.t, d.parent, d.member, d.counters, out);
    HIP_TRY(dbg_sync(st, "k_cc_compress_spec"));
  }
#if defined(PERC_LABEL_PAGEABLE)
  HIP_TRY(hipMemcpyAsync(hcs, d.counters, sizeof(hcs), hipMemcpyDeviceToHost, st));
#else
  if (!direct) HIP_TRY(hipMemcpyAsync(h->pin, d.counters, sizeof(int) * kHc, hipMemcpyDeviceToHost, st));
#endif
  HIP_TRY(hipStreamSynchronize(st));
  *nspan = hc[0];
  *nclusters = hc[1];
  if (spec && hc[0] > 0) {
    h->flat = true;
    h->span_count = hc[2];
  }
  for (int i = 0; i < std::min(hc[0], kMaxSpanList); ++i) span_list[i] = hc[8 + i];
  return hipSuccess;
}

// every parent to its root; with root > 0 the member sites of that root's
// cluster counted into *count (device) in the same pass
static hipError_t flatten_count(perc_ctx* h, int root, int* count) {
  const Geom& g = h->g;
  k_cc_compress<<<std::min(cdiv(g.t, kCcThreads * kCcCompressU), kReduceGrid), kCcThreads, 0, h->stream>>>(
      g.t, h->d.parent, h->d.member, root, count);
  HIP_TRY(dbg_sync(h->stream, "k_cc_compress"));
  h->flat = true;
  return hipSuccess;
}

hipError_t dev_flatten(perc_ctx* h) {
  if (h->flat) return hipSuccess;
  return flatten_count(h, 0, nullptr);
}

hipError_t dev_span_sites(perc_ctx* h, int root, int* count) {
  hipStream_t st = h->stream;
  HIP_TRY(hipMemsetAsync(h->d.counters + 2, 0, sizeof(int), st));
  if (!h->flat) {  // the spanning cluster's sites counted by the compress pass itself
    HIP_TRY(flatten_count(h, root, h->d.counters + 2));
  } else {
    k_count_root<<<std::min(cdiv(h->g.t, kCcThreads), kReduceGrid), kCcThreads, 0, st>>>(
        h->g.t, h->d.parent, h->d.member, root, h->d.counters + 2);
  }
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(count, h->d.counters + 2, sizeof(int), hipMemcpyDeviceToHost, st));
  return hipStreamSynchronize(st);
}

hipError_t dev_cluster_sizes(perc_ctx* h, int kind, int root, int* maxcs, int* rootsize) {
  HIP_TRY(dev_flatten(h));
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
  HIP_TRY(dev_flatten(h));
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
