// perc_march.h -- the register-march P / B kernels.
//
// Device code of libperc, included by perc_solve.hip and perc_slabs.hip (every definition sits in an
// anonymous namespace: each translation unit keeps its own copy of what it
// launches).
#pragma once
#include "perc_cg.h"

// (each TU launches a subset of these internal-linkage helpers)
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Wunused-function"
namespace perc {
namespace {

// ---------------------------------------------------------------------------
// Register-march fused P(k)+S(k) (stencil operator, m a multiple of 128).
// A wave owns a strip of 128 columns (a column pair per lane, 16-B
// accesses) and walks down a band of H rows.  Rows are prefetched D steps
// ahead into registers; p(k) of the rows above, at and below the current
// row live in a three-row register window, the column neighbours come from
// the adjacent lanes (lanes 0 / 63 also form p(k) of the halo column left
// / right of the strip).  No LDS tile, no barrier between loading and the
// SpMV: every wave streams like the B kernel.  Per row and element the
// arithmetic is k_cg_ps's (z = r/d, p = bk p + z, x += ak p, q in slot
// order), so every value is bitwise the other kernels'; only the q.p
// association differs (rows summed per lane).
// Buffer access with a hardware range check: a byte offset at or past the
// buffer's size makes a load return 0 and drops a store.  The row-march
// keeps every memory instruction of a step unconditional this way (rows
// outside the lattice or the band, halo columns of non-halo threads, q of
// the steps without a finished row), so hipcc's
// s_waitcnt bookkeeping stays exact across the loop: with loads and stores
// under branches it waited for vmcnt(0) -- every prefetched row and every
// store in flight -- once per step.
__device__ __forceinline__ double2 bld2(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0));
}
__device__ __forceinline__ double bld1(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, (int)off, 0, 0));
}
// sc1 (agent-coherent) load: data another workgroup stored with sc1
__device__ __forceinline__ double bld1s(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, (int)off, 0, 16));
}
// the march's p / q / r stores are nontemporal (write-through sc1 stores,
// which leave no dirty L2 line for the end-of-kernel write-back, measured
// no faster: solve 0.1441 / 0.1427 (sc0 sc1) vs 0.1422 ms per iteration,
// profiles/r4_4_store_policy_ab_L4096.json)
constexpr int kStAux = kNT;

template <int AUX>
__device__ __forceinline__ void bst2(__amdgpu_buffer_rsrc_t r, unsigned off, double2 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, (int)off, 0, AUX);
}
// one double (the edge z stores)
__device__ __forceinline__ void bst2e(__amdgpu_buffer_rsrc_t r, unsigned off, double v) {
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), r, (int)off, 0, 0);
}

// publish_and_reduce with tagged granules (the march kernels, TAG): every
// partial travels as one 16-B write-through {value, tag} store (untorn), so
// the workgroup that publishes it need not drain its stores before taking
// its ticket -- the reader polls the tags instead.  At the end of a march
// launch the last workgroup to arrive waited twice for s_waitcnt vmcnt(0)
// (its last rows' stores, then its group partial's) before the totals could
// be formed.  Association, and so the totals, are publish_and_reduce's term
// for term.  tag: unique per launch and solve; a reader that polls for ~0.5 s
// without seeing it sets *err and uses what it has (the host reports it).
__device__ __forceinline__ double2 gran_poll(__amdgpu_buffer_rsrc_t rg, int off, double tag, int* err) {
  double2 g2 = __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(rg, off, 0, 16));
  for (unsigned spin = 0; g2.y != tag; ++spin) {
    if (spin > (1u << 22)) {
      *err = 1;
      break;
    }
    __builtin_amdgcn_s_sleep(1);
    g2 = __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(rg, off, 0, 16));
  }
  return g2;
}

// NV granules polled together: every load is issued before any tag is
// checked, so the NV values cost one round trip, not NV (the march B's two
// sums waited for two, at both reduction levels: its tail ran 5.2 us after
// the last walk against P's 2.9, profiles/r5_3_mtrace_summary_L4096.txt)
template <int NV>
__device__ __forceinline__ void gran_poll_n(__amdgpu_buffer_rsrc_t rg, const int (&off)[NV], double tag,
                                            int* err, double (&out)[NV]) {
  for (unsigned spin = 0;; ++spin) {
    double2 g2[NV];
#pragma unroll
    for (int j = 0; j < NV; ++j)
      g2[j] = __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(rg, off[j], 0, 16));
    bool ok = true;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      ok = ok && g2[j].y == tag;
      out[j] = g2[j].x;
    }
    if (ok) return;
    if (spin > (1u << 22)) {
      *err = 1;
      return;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

constexpr int kDefGroups = 12;  // groups of kGroup workgroups a deferred total takes (grid <= 768)

// One-hop collector (grids of <= kDefGroups groups, the default; the
// two-level collectors below with PERC_MARCH_GROUPCOL, A/B probe builds
// only): the last logical workgroup polls every workgroup granule itself --
// wave w the granules of groups w, w + 4, w + 8, each lane re-polling only
// the granules it has not yet seen -- and forms the totals by the two-level
// association: a group's granules summed by one wave_sum over its lanes in
// order (the group collector's sum), the group sums thread-strided and
// block-summed (the last collector's).  Every total is the two-level one
// bitwise; the hop through the group granules (a write-through store and
// the last collector's poll of it) leaves the tail.
template <int NV>
__device__ __forceinline__ void flat_collect(__amdgpu_buffer_rsrc_t rg, int nwg, int ngroups, double tag, int* err,
                                             double (&tot)[NV], double* s_red) {
  __shared__ double s_grp[NV * kDefGroups];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  constexpr int kPer = kDefGroups / 4;  // groups per wave (4 waves per workgroup)
  double val[kPer][NV];
  bool need[kPer][NV];
#pragma unroll
  for (int i = 0; i < kPer; ++i) {
    const int g = wid + 4 * i, gn = g < ngroups ? min(kGroup, nwg - g * kGroup) : 0;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      val[i][j] = 0.0;
      need[i][j] = lane < gn;
    }
  }
  for (unsigned spin = 0;; ++spin) {
    double2 g2[kPer][NV];
#pragma unroll
    for (int i = 0; i < kPer; ++i) {  // every load issued before any tag is checked
      const int g0 = (wid + 4 * i) * kGroup;
#pragma unroll
      for (int j = 0; j < NV; ++j)
        g2[i][j] = __builtin_bit_cast(
            double2, __builtin_amdgcn_raw_buffer_load_b128(
                         rg, need[i][j] ? (j * nwg + g0 + lane) * 16 : (int)kOOB, 0, 16));
    }
    bool more = false;
#pragma unroll
    for (int i = 0; i < kPer; ++i)
#pragma unroll
      for (int j = 0; j < NV; ++j)
        if (need[i][j]) {
          if (g2[i][j].y == tag) {
            val[i][j] = g2[i][j].x;
            need[i][j] = false;
          } else {
            more = true;
          }
        }
    if (!__any(more)) break;
    if (spin > (1u << 22)) {  // (uniform)
      if (more) *err = 1;
      break;
    }
    __builtin_amdgcn_s_sleep(1);
  }
#pragma unroll
  for (int i = 0; i < kPer; ++i) {
    const int g = wid + 4 * i;
    if (g < ngroups) {  // (wave-uniform)
#pragma unroll
      for (int j = 0; j < NV; ++j) {
        const double w = wave_sum(val[i][j]);  // the group collector's sum
        if (lane == 0) s_grp[j * kDefGroups + g] = w;
      }
    }
  }
  __syncthreads();
  double acc[NV];
#pragma unroll
  for (int j = 0; j < NV; ++j) {  // the last collector's thread-strided group sums
    acc[j] = 0.0;
    if ((int)threadIdx.x < ngroups) acc[j] = acc[j] + s_grp[j * kDefGroups + threadIdx.x];
  }
  block_sum<NV>(acc, s_red);
  if (threadIdx.x == 0)
#pragma unroll
    for (int j = 0; j < NV; ++j) s_red[16 + j] = acc[j];
  __syncthreads();
#pragma unroll
  for (int j = 0; j < NV; ++j) tot[j] = s_red[16 + j];
}

// Fixed collectors instead of tickets (the default; PERC_MARCH_TICKETS, A/B
// probe builds only: the ticket form below): a group's LAST logical
// workgroup (lb = g0 + gn - 1, dispatched late: logical blocks of an XCD are
// consecutive) sums its group's granules as they arrive and publishes the
// group's granule; the last group's collector sums the group granules.  The
// association is the ticket form's term for term (the group's lanes in
// order + butterfly; the groups thread-strided + block sum), so every value
// is bitwise the same; what goes is the two agent-scope ticket atomics (and
// their resets) on the tail's critical path: the collectors only poll.
template <int NV>
__device__ bool publish_and_reduce_tagged(double (&v)[NV], double* gran, unsigned* tickets, int lb,
                                          int nwg, double tag, int* err, double (&tot)[NV],
                                          double* s_red, int* s_flag) {
#if !defined(PERC_MARCH_TICKETS)
  (void)tickets;
  (void)s_flag;
  block_sum<NV>(v, s_red);
  const int ngroups = red_groups(nwg);
  const int grp = lb / kGroup, g0 = grp * kGroup, gn = min(kGroup, nwg - g0);
  const __amdgpu_buffer_rsrc_t rg = rsrc(gran, (unsigned)(NV * (nwg + ngroups) * 16));
  const int goff = NV * nwg;
  if (threadIdx.x == 0) {
#pragma unroll
    for (int j = 0; j < NV; ++j)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, make_double2(v[j], tag)), rg,
                                             (j * nwg + lb) * 16, 0, 16);
  }
#if !defined(PERC_MARCH_GROUPCOL)
  if (ngroups <= kDefGroups) {  // (uniform) the one-hop collector
    if (lb != nwg - 1) return false;
    flat_collect<NV>(rg, nwg, ngroups, tag, err, tot, s_red);
    return true;
  }
#endif
  if (lb != g0 + gn - 1) return false;  // (uniform) not a collector
  if (threadIdx.x < 64) {  // the group's collector: wave 0 sums the group's partials
    const int lane = threadIdx.x;
    double w[NV];
    if (lane < gn) {
      int off[NV];
#pragma unroll
      for (int j = 0; j < NV; ++j) off[j] = (j * nwg + g0 + lane) * 16;
      gran_poll_n<NV>(rg, off, tag, err, w);
    } else {
#pragma unroll
      for (int j = 0; j < NV; ++j) w[j] = 0.0;
    }
#pragma unroll
    for (int j = 0; j < NV; ++j) w[j] = wave_sum(w[j]);
    if (lane == 0)
#pragma unroll
      for (int j = 0; j < NV; ++j)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, make_double2(w[j], tag)), rg,
                                               (goff + j * ngroups + grp) * 16, 0, 16);
  }
  if (grp != ngroups - 1) return false;  // (uniform)
  double acc[NV];
#pragma unroll
  for (int j = 0; j < NV; ++j) acc[j] = 0.0;
  for (int i = threadIdx.x; i < ngroups; i += blockDim.x) {
    int off[NV];
    double gv[NV];
#pragma unroll
    for (int j = 0; j < NV; ++j) off[j] = (goff + j * ngroups + i) * 16;
    gran_poll_n<NV>(rg, off, tag, err, gv);
#pragma unroll
    for (int j = 0; j < NV; ++j) acc[j] = acc[j] + gv[j];
  }
  __syncthreads();  // s_red reuse
  block_sum<NV>(acc, s_red);
  if (threadIdx.x == 0)
#pragma unroll
    for (int j = 0; j < NV; ++j) s_red[16 + j] = acc[j];
  __syncthreads();
#pragma unroll
  for (int j = 0; j < NV; ++j) tot[j] = s_red[16 + j];
  return true;
#else
  block_sum<NV>(v, s_red);
  const int ngroups = red_groups(nwg);
  const int grp = lb / kGroup, g0 = grp * kGroup, gn = min(kGroup, nwg - g0);
  // granules: [j][workgroup] then [j][group]
  const __amdgpu_buffer_rsrc_t rg = rsrc(gran, (unsigned)(NV * (nwg + ngroups) * 16));
  const int goff = NV * nwg;
  if (threadIdx.x == 0) {
#pragma unroll
    for (int j = 0; j < NV; ++j)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, make_double2(v[j], tag)), rg,
                                             (j * nwg + lb) * 16, 0, 16);
    const unsigned tk = __hip_atomic_fetch_add(&tickets[grp * kTicketStride], 1u,
                                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_flag[0] = tk == (unsigned)(gn - 1);
  }
  __syncthreads();
  if (!s_flag[0]) return false;
  if (threadIdx.x < 64) {  // last of its group: wave 0 sums the group's partials
    const int lane = threadIdx.x;
    double w[NV];
    if (lane < gn) {
      int off[NV];
#pragma unroll
      for (int j = 0; j < NV; ++j) off[j] = (j * nwg + g0 + lane) * 16;
      gran_poll_n<NV>(rg, off, tag, err, w);
    } else {
#pragma unroll
      for (int j = 0; j < NV; ++j) w[j] = 0.0;
    }
#pragma unroll
    for (int j = 0; j < NV; ++j) w[j] = wave_sum(w[j]);
    if (lane == 0) {
#pragma unroll
      for (int j = 0; j < NV; ++j)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, make_double2(w[j], tag)), rg,
                                               (goff + j * ngroups + grp) * 16, 0, 16);
      __hip_atomic_store(&tickets[grp * kTicketStride], 0u, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
      const unsigned tk = __hip_atomic_fetch_add(&tickets[ngroups * kTicketStride], 1u,
                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_flag[1] = tk == (unsigned)(ngroups - 1);
    }
  }
  __syncthreads();
  if (!s_flag[1]) return false;
  double acc[NV];
#pragma unroll
  for (int j = 0; j < NV; ++j) acc[j] = 0.0;
  for (int i = threadIdx.x; i < ngroups; i += blockDim.x) {
    int off[NV];
    double v[NV];
#pragma unroll
    for (int j = 0; j < NV; ++j) off[j] = (goff + j * ngroups + i) * 16;
    gran_poll_n<NV>(rg, off, tag, err, v);
#pragma unroll
    for (int j = 0; j < NV; ++j) acc[j] = acc[j] + v[j];
  }
  __syncthreads();  // s_red reuse
  block_sum<NV>(acc, s_red);
  if (threadIdx.x == 0) {
#pragma unroll
    for (int j = 0; j < NV; ++j) s_red[16 + j] = acc[j];
    __hip_atomic_store(&tickets[ngroups * kTicketStride], 0u, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < NV; ++j) tot[j] = s_red[16 + j];
  return true;
#endif
}

// Deferred reductions (DEF, an opt-in variant of the strip-major tagged
// march, PERC_MARCH_DEF; measured and not the default, perc_solve.hip
// setup_granules): a launch ends once its workgroups have published their
// granules -- no collector waits on the slowest workgroup's granule and no
// second hop follows (the march trace put the exits 2.9 us (P) and 4.4 us
// (B) past the last walk, profiles/r5_4_mtrace_summary_L4096.txt; the
// launch times moved by 1.4 and 2.3 us).  The NEXT launch forms the totals
// in every workgroup, after its first rows' loads are issued: the group
// sums by the same lanes-in-order wave_sum the group collectors formed and
// the group totals by the same thread-strided block_sum the last collector
// formed, so every total is the collector form's bitwise in every
// workgroup (tagged = ticket = deferred: test_tagged_reduction_is_bitwise_
// the_ticket_one).  The granules are complete when a launch starts (the
// previous one has ended); their tags are checked, not polled.
// CGArgs::mdef bits: kDefP -- P publishes only, B forms q.p (ak) at its
// start; kDefB -- B publishes only, the next P (and k_march_epi) forms z.r,
// r.r (bk, err, stop); kDefBench -- perc_bench_kernel's fixed iteration (no
// stop, no scalars but bkn)
constexpr int kDefP = 1, kDefB = 2, kDefBench = 4;
template <int NV>
__device__ __forceinline__ void def_totals(const double* gran, int nwg, double tag, int* err,
                                           double (&tot)[NV], double* s_red, double* s_grp, bool sc1) {
  const int ngroups = red_groups(nwg);
  const __amdgpu_buffer_rsrc_t rg = rsrc(gran, (unsigned)(NV * (nwg + ngroups) * 16));
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  constexpr int kPer = kDefGroups / 4;  // groups per wave (4 waves per workgroup)
  double2 g2[kPer][NV];
#pragma unroll
  for (int i = 0; i < kPer; ++i) {  // every load issued before any is used
    const int g = wid + 4 * i, g0 = g * kGroup, gn = g < ngroups ? min(kGroup, nwg - g0) : 0;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const int off = (int)(lane < gn ? (j * nwg + g0 + lane) * 16 : kOOB);
      // (sc1: past this XCD's L2; plain: the XCD's workgroups share one L2
      // fill -- the previous launch's write-through granules are in memory
      // when this launch starts, and a stale line would fail the tag check)
      g2[i][j] = __builtin_bit_cast(double2, sc1 ? __builtin_amdgcn_raw_buffer_load_b128(rg, off, 0, 16)
                                                 : __builtin_amdgcn_raw_buffer_load_b128(rg, off, 0, 0));
    }
  }
  bool bad = false;
#pragma unroll
  for (int i = 0; i < kPer; ++i) {
    const int g = wid + 4 * i;
    if (g < ngroups) {  // (wave-uniform)
      const int gn = min(kGroup, nwg - g * kGroup);
#pragma unroll
      for (int j = 0; j < NV; ++j) {
        bad = bad || (lane < gn && g2[i][j].y != tag);
        const double w = wave_sum(lane < gn ? g2[i][j].x : 0.0);  // the group collector's sum
        if (lane == 0) s_grp[j * kDefGroups + g] = w;
      }
    }
  }
  if (err && __any(bad) && lane == 0) *err = 1;
  __syncthreads();
  double acc[NV];
#pragma unroll
  for (int j = 0; j < NV; ++j) {  // the last collector's thread-strided group sums
    acc[j] = 0.0;
    if ((int)threadIdx.x < ngroups) acc[j] = acc[j] + s_grp[j * kDefGroups + threadIdx.x];
  }
  block_sum<NV>(acc, s_red);
  if (threadIdx.x == 0)
#pragma unroll
    for (int j = 0; j < NV; ++j) s_red[16 + j] = acc[j];
  __syncthreads();
#pragma unroll
  for (int j = 0; j < NV; ++j) tot[j] = s_red[16 + j];
  __syncthreads();  // s_red / s_grp reuse
}

// a workgroup-uniform double held in SGPRs (values read back from LDS land
// in VGPRs: 2 more for the whole walk -- P's 169 instead of 167, 2 waves
// per SIMD instead of 3)
__device__ __forceinline__ double sgpr_double(double v) {
  const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)u), hi = __builtin_amdgcn_readfirstlane((unsigned)(u >> 32));
  return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}

// B(kk)'s epilogue, deferred to the next P (or k_march_epi): the z.r and
// r.r totals -> bk, err, the stop test (k_cg_b's epilogue; linbcg
// bondc.f:785-787, 834).  Every workgroup forms the same values; `writer`
// stores them.  bkn is parity-buffered: the writer stores bknum(kk) while
// the others read bknum(kk - 1).  Returns the stop decision.
__device__ __forceinline__ bool march_def_epilogue(const CGArgs& a, int kk, const double (&tb)[2], bool writer,
                                                   double& bk) {
  CGScalars* S = a.S;
  const double old = kk == 1 ? S->bknum : S->bkn[(kk - 1) & 1];
  const double err = sqrt(tb[1]) / S->bnrm;
  bk = tb[0] / old;
  const bool live = !(a.mdef & kDefBench);
  const bool dn = live && (!(err > S->tol) || kk >= S->itmax + 1);
  if (writer) {
    S->bkn[kk & 1] = tb[0];
    if (live) {
      S->bk = bk;
      S->err = err;
      if (kk - 1 < a.err_hist_cap) a.err_hist[kk - 1] = err;
      S->iter = kk;
      if (dn) S->done = 1;
    }
  }
  return dn;
}

constexpr int kMarchW = 128;     // columns per wave strip
constexpr int kEdgeRows = 64;    // band rows whose edge pairs B can stage in LDS (ES)
constexpr int kMarchWaves = 4;   // waves (strips) per workgroup
// A/B probe builds only: the column-class path in the row-major march too
// (PERC_MARCH_RM_SQ), optionally held to 4 waves per SIMD (PERC_MARCH_RM_SQ4)
#if defined(PERC_MARCH_RM_SQ) || defined(PERC_MARCH_RM_SQ4)
constexpr bool kMarchRmSq = true;
#else
constexpr bool kMarchRmSq = false;
#endif
// the row-major march's nibble codes (on unless PERC_MARCH_RM_U16, A/B probe
// builds only)
#ifdef PERC_MARCH_RM_U16
constexpr bool kMarchRmNib = false;
#else
constexpr bool kMarchRmNib = true;
#endif
// waves per SIMD the row-major nibble march (B) is held to (its column-class
// path would take 132-134 VGPRs: 3 waves; 128 without spills when held;
// the u16 march has 123-126)
#if defined(PERC_MARCH_RM_SQ4)
#define PERC_MARCH_MINW(SM, MODE, PK) ((SM) || (MODE) == 0 ? 1 : 4)
#elif defined(PERC_MARCH_RM_NOBOUND)  // (A/B probe builds only)
#define PERC_MARCH_MINW(SM, MODE, PK) 1
#else
#define PERC_MARCH_MINW(SM, MODE, PK) (!(SM) && (PK) && (MODE) != 0 ? 4 : 1)
#endif

struct MRow {       // one prefetched row of the lane's pair (+ halo column)
  double2 p, r;     // p(k-1), r
  unsigned c;       // the pair's codes
  double hp, hr;    // halo column (lanes 0 and 63)
  unsigned hc;
};
struct MWin {       // p(k) at columns col-1, col, col+1, col+2 of one row
  double l, e0, e1, rr;
};

// neighbour value at raster position kp (0..7: (-1,-1) (-1,0) (-1,1) (0,-1)
// (0,1) (1,-1) (1,0) (1,1)) of element E (0: column col, 1: col+1)
template <int E>
__device__ __forceinline__ double mwin_at(int kp, const MWin& U, const MWin& C, const MWin& D) {
  const MWin& W = kp < 3 ? U : (kp < 5 ? C : D);
  const int dc = kp < 3 ? kp - 1 : (kp == 3 ? -1 : (kp == 4 ? 1 : kp - 6));
  const int s = E + 1 + dc;  // 0: l, 1: e0, 2: e1, 3: rr
  return s == 0 ? W.l : (s == 1 ? W.e0 : (s == 2 ? W.e1 : W.rr));
}

// q of element E: d x + sum over the form's slots (slot order) of g x_nb,
// when the wave's rows all share one regular form (slot order = raster
// order) with used-position bits `mask` (wave-uniform: scalar branches)
template <int E>
__device__ __forceinline__ double march_q(unsigned c, double d, double xi, unsigned mask,
                                          const MWin& U, const MWin& C, const MWin& D,
                                          double ng0, double nleak) {
  double acc = d * xi;
  int j = 0;
#pragma unroll
  for (int kp = 0; kp < 8; ++kp) {
    if (mask & (1u << kp)) {
      const double gv = ((c >> j) & 1u) ? ng0 : nleak;
      acc = acc + gv * mwin_at<E>(kp, U, C, D);
      ++j;
    }
  }
  return acc;
}

// general path (rows whose wave mixes forms, or wrapped-column forms): the
// lane's 12 window values are in the wave's LDS scratch s_w[v * 64 + lane]
// (v = row * 4 + {l, e0, e1, rr}); slot j reads value kvi(kp_j) + E
template <int E>
__device__ __forceinline__ double march_q_gen(unsigned c, double d, double xi, unsigned pos,
                                              const double* s_w, int lane, double ng0,
                                              double nleak) {
  // raster position -> window value index (row * 4 + 1 + dc), 4 bits each
  constexpr unsigned kVi = 0xA9864210u;
  double acc = d * xi;
  const int cnt = (c >> 8) & 7;
#pragma unroll
  for (int j = 0; j < kMaxSlots; ++j) {
    if (j < cnt) {
      const int kp = (pos >> (3 * j)) & 7;
      const int v = ((kVi >> (4 * kp)) & 15u) + E;
      const double gv = ((c >> j) & 1u) ? ng0 : nleak;
      acc = acc + gv * s_w[v * 64 + lane];
    }
  }
  return acc;
}

// q of element E for a wave whose rows are all regular (slot order = raster
// order) but not one form: lane-private raster -> slot map (rmap), so edge
// strips (columns 0 and m-1 lack a neighbour) take this register path too.
// Positions a row lacks read an exact 0 from the window (outside the
// lattice or the interior system) or are skipped by the select.
template <int E>
__device__ __forceinline__ double march_q_map(unsigned c, double d, double xi, unsigned map,
                                              unsigned umask, const MWin& U, const MWin& C,
                                              const MWin& D, double ng0, double nleak) {
  double acc = d * xi;
#pragma unroll
  for (int kp = 0; kp < 8; ++kp) {
    if (umask & (1u << kp)) {
      const unsigned j = (map >> (4 * kp)) & 15u;
      const double gv = ((c >> j) & 1u) ? ng0 : nleak;
      const double pr = gv * mwin_at<E>(kp, U, C, D);
      acc = j != 15u ? acc + pr : acc;
    }
  }
  return acc;
}

// Rows prefetched ahead (template D).  The P+S kernel of the solve runs
// D = 3 (strip-major: 162 VGPRs, 3 waves per SIMD, one round of 43-row
// bands at L = 4096): 0.106-0.107 ms vs D = 4 / 5 at 2 waves per SIMD
// 0.114-0.116 (profiles/r2_12_strips_depth_rows_probe.log,
// r2_14_march_depth5.log): waves per SIMD, not rows in flight, decide.  Before the memory instructions were
// made unconditional (MBuf) every step waited for vmcnt(0) and deeper
// prefetch could not help.  The opt-in variants (q-free P and B, strip-
// major) keep D = 2.
constexpr int kMarchDepth = 2;

// Register march, three kernels of one loop (MODE):
//   kMarchPQ: P(k)+S(k), stores q for the streaming B (k_cg_b)
//   kMarchP:  P(k)+S(k) without the q store
//   kMarchB:  B(k) rebuilding q = A p(k) from p(k) (+ halo) instead of
//             reading it: r -= ak q, z = r/d, z.r, r.r, bk, err, stop
// With kMarchP + kMarchB an iteration moves 52N bytes instead of 60N.
// Direction: a wave walks its band down (increasing rows) or up.  With
// a.march_alt, odd bands walk up in P and even bands walk up in B, so the
// halo rows two neighbouring bands share are read by both waves at the
// same moment (start or end of the walk: the second read hits L2 / the
// Infinity Cache), and B starts each band on the rows P wrote last.
constexpr int kMarchPQ = 0, kMarchP = 1, kMarchB = 2;

struct MGeom {
  int r0, rend, col, hcol;
  bool hok;
  // strip-major edge {p, z} (CGArgs::ez), pair bases: ezh -- the halo
  // column's (P's lanes 0 and 63), ezo -- the lane's own edge column (B's
  // lanes 0 and 63 store there)
  int ezh, ezo;
  unsigned cb0, cb1, cbh;  // nibble codes (PK): count / form bits of col, col+1, hcol
  // open square lattice with nibble codes (PK): the slot bits of element 0 /
  // 1 in the INTERIOR form's slot numbering, c' = (c & lo) | ((c & hi) << 1)
  // -- the identity inside, a gap at the absent neighbour of column 0 (lo 1,
  // hi 6) and column m-1 (lo 3, hi 4); see march_step
  unsigned lo0, hi0, lo1, hi1;
};

// Buffer views of the rows one march wave touches, [lo, hi) = its band plus
// the halo rows, clipped to the loadable rows [glo, ghi): every load and
// store of a step is issued unconditionally with a byte offset that is out
// of range (kOOB, or a row outside the view) where the row-major kernel had
// a branch -- a row outside the lattice, a halo column of a non-halo lane,
// p(k-1) of the first iteration, q / p of a row the wave does not own.
// With memory instructions under branches hipcc's waitcnt pass put
// s_waitcnt vmcnt(0) at the top of every step (every prefetched row and
// every store drained once per step: ~3.5 read requests in flight per wave,
// TCC_EA0_RDREQ_LEVEL, profiles/r2_3_*); unconditional, the waits count
// exactly and the prefetch ring keeps its rows in flight.
struct MBuf {
  __amdgpu_buffer_rsrc_t p, r, c, pn, q;  // p(k-1), r, codes, p(k): rows [lo, hi); q: own rows
  __amdgpu_buffer_rsrc_t t;  // literal dot terms (a.lit, row-major; size 0 in the fast order)
  __amdgpu_buffer_rsrc_t ez;  // strip-major: the edge z array (CGArgs::ez)
  int lo, hi;
};

// strip-major solve (SM): whole-array views (vectors < 2 GB there), element
// offsets through sm_at; row-major: the band's views, offsets from row lo
template <int MODE, bool SM, bool PK = false>
__device__ __forceinline__ MBuf march_bufs(const CGArgs& a, const MGeom& g, const double* psrc,
                                           double* pnew) {
  const int m = a.T.m;
  MBuf B;
  B.lo = max(g.r0 - 1, a.glo);
  B.hi = max(min(g.rend + 1, a.ghi), B.lo);
  // (dev_solve sets a.lit only where 3 N doubles stay below 2 GB; only the
  // LIT instantiation stores through this view)
  B.t = rsrc(a.lit, a.lit ? (unsigned)a.St.N * 24u : 0u);
  if constexpr (SM) {
    const unsigned nall = (unsigned)a.T.nrows * (unsigned)m;
    B.p = rsrc(psrc, nall * 8u);
    B.r = rsrc(a.r, nall * 8u);
    B.c = PK ? rsrc(a.nib, nall / 2u) : rsrc(a.St.code, nall * 2u);
    B.pn = rsrc(pnew, nall * 8u);
    B.q = rsrc(a.q, MODE == kMarchPQ ? nall * 8u : 0u);
    B.ez = rsrc(a.ez, a.ez ? (unsigned)(2 * (m / kMarchW) * a.T.nrows) * 16u : 0u);
    return B;
  }
  B.ez = rsrc(nullptr, 0u);
  // (the row-major nibble march: edge pairs too)
  if (PK) B.ez = rsrc(a.ez, a.ez ? (unsigned)(2 * (m / kMarchW) * a.T.nrows) * 16u : 0u);
  const long long base = (long long)B.lo * m;
  const unsigned n = (unsigned)(B.hi - B.lo) * (unsigned)m;
  const unsigned nown = (unsigned)max(g.rend - g.r0, 0) * (unsigned)m;
  B.p = rsrc(psrc + base, n * 8u);
  B.r = rsrc(a.r + base, n * 8u);
  B.c = PK ? rsrc(a.nib + base / 2, n / 2u) : rsrc(a.St.code + base, n * 2u);
  B.pn = rsrc(pnew + base, n * 8u);
  B.q = rsrc(MODE == kMarchPQ ? a.q + (long long)g.r0 * m : a.r, MODE == kMarchPQ ? nown * 8u : 0u);
  return B;
}

// element offset (in elements) of (row gr, column col) in a view of MBuf
template <bool SM>
__device__ __forceinline__ unsigned melem(const CGArgs& a, const MBuf& B, int gr, int col) {
  return SM ? (unsigned)sm_at(a.T, gr, col) : (unsigned)((gr - B.lo) * a.T.m + col);
}

// count / form bits of column c on the open square lattice (interior, first,
// last column): the row-major nibble march forms them per access instead of
// holding them in MGeom (7 VGPRs: its P spilled 6 at the 4-wave bound, 128
// VGPRs; the strip-major march keeps them in registers)
__device__ __forceinline__ unsigned col_cls(const CGArgs& a, int c) {
  return c == 0 ? a.ncls[1] : (c == a.T.m - 1 ? a.ncls[2] : a.ncls[0]);
}

template <int MODE, bool SM, int PAUX = 0, bool PK = false>
__device__ __forceinline__ void march_load(const CGArgs& a, const MGeom& g, const MBuf& B, int gr,
                                           bool first, const double* __restrict__ psrc, MRow& R) {
  {
    const bool rowok = (unsigned)(gr - B.lo) < (unsigned)(B.hi - B.lo);
    const unsigned e = rowok ? melem<SM>(a, B, gr, g.col) : 0u;
    const unsigned eh = rowok ? melem<SM>(a, B, gr, g.hcol) : 0u;
    const unsigned o8 = rowok ? e * 8u : kOOB;
    const bool rown = MODE != kMarchB || (gr >= g.r0 && gr < g.rend);
#if defined(PERC_PROBE_NO_PHALO)  // (A/B probe builds only: P's halo-column loads' cost, wrong values)
    const bool hk = rowok && g.hok && MODE == kMarchB;
#else
    const bool hk = rowok && g.hok;
#endif
    const unsigned h8 = hk ? eh * 8u : kOOB;
    if constexpr (PK) {
      // the pair's two slot nibbles in one byte (element e even); the count
      // and form bits come from the columns (g.cb0 / cb1): the u16 codes
      const unsigned b = __builtin_amdgcn_raw_buffer_load_b8(B.c, (int)(rowok ? e / 2u : kOOB), 0, 0);
      const unsigned cb0 = SM ? g.cb0 : col_cls(a, g.col), cb1 = SM ? g.cb1 : col_cls(a, g.col + 1);
      R.c = ((b & 0xFu) | cb0) | (((b >> 4) | cb1) << 16);
    } else {
      R.c = __builtin_amdgcn_raw_buffer_load_b32(B.c, (int)(rowok ? e * 2u : kOOB), 0, 0);
    }
    // PAUX on the loads that read a value for the last time: P's p(k-1)
    // (dead once p(k) is formed), B's r(k) (overwritten by r(k+1))
    constexpr int kRAux = MODE == kMarchB ? PAUX : 0;
    constexpr int kPAux = MODE == kMarchP ? PAUX : 0;
    R.r = __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(B.r, (int)(rown ? o8 : kOOB), 0, kRAux));
    R.p = __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(B.p, (int)(first ? kOOB : o8), 0, kPAux));
    if (MODE != kMarchB && (SM || PK)) {
      // strip-major, and the row-major nibble march: the halo column's p(k-1) and z = r/d as the last B
      // stored them (edge {p, z}): one 16-B load instead of its code, r and
      // p, and no division -- the three halo loads held P 2.5 us (71.4 vs
      // 73.9 us without them, profiles/r6_13_ab_p.json)
      const double2 e = bld2(B.ez, hk ? (unsigned)(g.ezh + gr) * 16u : kOOB);
      R.hc = 0u;
      R.hr = e.y;  // z
      R.hp = e.x;  // p(k-1)
    } else if (MODE != kMarchB) {
      if constexpr (PK) {
        const unsigned b = __builtin_amdgcn_raw_buffer_load_b8(B.c, (int)(hk ? eh / 2u : kOOB), 0, 0);
        R.hc = ((b >> (4u * (eh & 1u))) & 0xFu) | (SM ? g.cbh : col_cls(a, g.hcol));
      } else {
        R.hc = __builtin_amdgcn_raw_buffer_load_b16(B.c, (int)(hk ? eh * 2u : kOOB), 0, 0);
      }
      R.hr = bld1(B.r, h8);
    } else {
      R.hc = 0u;
      R.hr = 0.0;
    }
    if (MODE == kMarchB || !(SM || PK)) R.hp = bld1(B.p, first ? kOOB : h8);
  }
}

struct MState {
  MWin U, C, Dn;
  unsigned cN, cM;        // codes of the newest / middle window rows
  double2 rN, rM;         // r of the newest / middle rows (kMarchB)
};

// one step: row gr enters the window, then the middle row (gr -+ 1) is
// finished when it is one of the band's own rows
template <int MODE, bool UP, bool SM, bool LIT = false, bool PK = false, int ESR = 0>
__device__ __forceinline__ void march_step(const CGArgs& a, const MGeom& g, const MBuf& B,
                                           const MRow& R, int gr,
                                           bool first, double bk, double ak,
                                           double* __restrict__ pnew, const double2* s_dt,
                                           const unsigned* s_rpos, const unsigned* s_rmap,
                                           double* s_w, MState& W, double (&acc)[2],
                                           double2* s_ed = nullptr) {
  const int lane = threadIdx.x & 63;
  const int nrows = a.T.nrows;
  const double ng0 = a.St.ng0, nleak = a.St.nleak;
  double2 pn = make_double2(0.0, 0.0);
  double hpn = 0.0;
  double2 d0 = make_double2(1.0, 1.0), d1 = d0;  // {d, 1/d}
  if (gr >= a.glo && gr < a.ghi) {
    d0 = s_dt[diag_idx(R.c & 0xffffu)];
    d1 = s_dt[diag_idx(R.c >> 16)];
    if (MODE == kMarchB) {
      pn = R.p;
      hpn = R.hp;
    } else {
      const double z0 = div_tab(R.r.x, d0), z1 = div_tab(R.r.y, d1);
      if (first) {
        pn.x = z0;
        pn.y = z1;
      } else {
        pn.x = bk * R.p.x + z0;
        pn.y = bk * R.p.y + z1;
      }
      if (g.hok) {
        const double zh = SM || PK ? R.hr : div_tab(R.hr, s_dt[diag_idx(R.hc)]);  // (the edge z)
        hpn = first ? zh : bk * R.hp + zh;
      }
    }
  }
  if (MODE != kMarchB) {
    // own row; in a slab also the ghost rows, so the next iteration's
    // halo p(k) is at hand (bitwise the neighbour slab's own value)
    const bool own = gr >= g.r0 && gr < g.rend;
    const bool pst = (unsigned)(gr - B.lo) < (unsigned)(B.hi - B.lo) &&
                     (own || (a.slab && (gr < 0 || gr >= nrows)));
    bst2<kStAux>(B.pn, pst ? melem<SM>(a, B, gr, g.col) * 8u : kOOB, pn);
  }
  MWin Nw;
  Nw.e0 = pn.x;
  Nw.e1 = pn.y;
  const double up = __shfl_up(pn.y, 1);
  const double dn = __shfl_down(pn.x, 1);
  Nw.l = lane == 0 ? hpn : up;
  Nw.rr = lane == 63 ? hpn : dn;
  if (UP) {
    W.Dn = W.C;
    W.C = W.U;
    W.U = Nw;
  } else {
    W.U = W.C;
    W.C = W.Dn;
    W.Dn = Nw;
  }
  W.cM = W.cN;
  W.cN = R.c;
  if (MODE == kMarchB) {
    W.rM = W.rN;
    W.rN = R.r;
  }
  const int mid = UP ? gr + 1 : gr - 1;
  const bool mown = mid >= g.r0 && mid < g.rend;  // wave-uniform
  double2 mq = make_double2(0.0, 0.0), mr = mq;   // q / r(k+1) of the middle row
  // the middle row's dot terms (P: q.p; B: z.r, r.r), summed into acc and
  // stored for the literal folds
  double2 t0 = mq, t1 = mq;
  if (mown) {
    const unsigned c0w = W.cM & 0xffffu, c1w = W.cM >> 16;
    const unsigned f0 = c0w >> 11, f1 = c1w >> 11;
    const double2 dM0 = s_dt[diag_idx(c0w)], dM1 = s_dt[diag_idx(c1w)];
    const unsigned ff = __builtin_amdgcn_readfirstlane(f0);
    const bool uni = !__any(f0 != ff || f1 != ff) && a.St.F.regular[ff];
    double q0, q1;
    // u16 codes (the row-major march past the Infinity Cache): the same
    // path where the lattice is the open square one (a.sqcls) and every
    // row of the step carries its column class's count / form bits
    bool sqp;
    // (strip-major u16 codes only: in the row-major march past the Infinity
    // Cache the path's 6 VGPRs cost a wave per SIMD -- 133 vs 127, P 0.394
    // vs 0.314 ms at L = 8192, profiles/r5_6_l8192_probe_bond.json)
    // (the row-major nibble march runs on the open square lattice only --
    // the host takes the u16 codes with pbc -- so the other paths are not
    // compiled into it: their registers spilled it at the 4-wave bound)
    if constexpr (PK && !SM) sqp = true;
    else if constexpr (PK) sqp = !a.T.pbc;
    else if constexpr (SM || kMarchRmSq) sqp = a.sqcls && !__any((((c0w ^ g.cb0) | (c1w ^ g.cb1)) >> 8) != 0u);
    else sqp = false;
    if (sqp) {
      // Open square lattice, nibble codes: every row is interior, column 0
      // or column m-1 (k_pack_nib checked it), so EVERY wave -- the edge
      // strips too -- takes the interior form's scalar path.  A row of
      // column 0 (m-1) lacks its left (right) neighbour: its slot bits are
      // spread into the interior numbering with a gap there (MGeom lo/hi),
      // whose term is leak x (+0.0) -- the window holds an exact +0 for the
      // absent column (hok false: hpn = 0 / an out-of-range load) -- i.e.
      // -0.0, and acc + (-0.0) == acc for every acc: the row's sum is
      // bitwise the form's own (the first / last interior rows rely on the
      // same identity for their electrode neighbours).  Before, one lane's
      // edge form sent the whole edge-strip wave to march_q_map: edge
      // strips walked 69.8 vs 65.9 us (P, iteration 20000) and set the
      // kernel's end (profiles/r5_2_mtrace_summary_it20000_L4096.txt)
      const unsigned mask = a.St.F.rmask[a.ncls[0] >> 11];
      unsigned e0, e1;
      if constexpr (SM) {
        e0 = (c0w & g.lo0) | ((c0w & g.hi0) << 1);
        e1 = (c1w & g.lo1) | ((c1w & g.hi1) << 1);
      } else {  // (the same spreads, formed from the column)
        e0 = g.col == 0 ? (c0w & 1u) | ((c0w & 6u) << 1) : c0w & 0xFu;
        e1 = g.col + 1 == a.T.m - 1 ? (c1w & 3u) | ((c1w & 4u) << 1) : c1w & 0xFu;
      }
      q0 = march_q<0>(e0, dM0.x, W.C.e0, mask, W.U, W.C, W.Dn, ng0, nleak);
      q1 = march_q<1>(e1, dM1.x, W.C.e1, mask, W.U, W.C, W.Dn, ng0, nleak);
    } else if (uni) {
      const unsigned mask = a.St.F.rmask[ff];
      q0 = march_q<0>(c0w, dM0.x, W.C.e0, mask, W.U, W.C, W.Dn, ng0, nleak);
      q1 = march_q<1>(c1w, dM1.x, W.C.e1, mask, W.U, W.C, W.Dn, ng0, nleak);
    } else {
      const unsigned mp0 = s_rmap[f0], mp1 = s_rmap[f1];
      if (!__any(mp0 == kRmapIrregular || mp1 == kRmapIrregular)) {
        const unsigned um = a.St.F.umask;
        q0 = march_q_map<0>(c0w, dM0.x, W.C.e0, mp0, um, W.U, W.C, W.Dn, ng0, nleak);
        q1 = march_q_map<1>(c1w, dM1.x, W.C.e1, mp1, um, W.U, W.C, W.Dn, ng0, nleak);
      } else {
        const MWin* rows[3] = {&W.U, &W.C, &W.Dn};
#pragma unroll
        for (int rr = 0; rr < 3; ++rr) {
          s_w[(4 * rr + 0) * 64 + lane] = rows[rr]->l;
          s_w[(4 * rr + 1) * 64 + lane] = rows[rr]->e0;
          s_w[(4 * rr + 2) * 64 + lane] = rows[rr]->e1;
          s_w[(4 * rr + 3) * 64 + lane] = rows[rr]->rr;
        }
        // lane-private slots: no cross-lane hazard, only the wave's own
        // LDS write -> read order (lgkmcnt, inserted by the compiler)
        q0 = march_q_gen<0>(c0w, dM0.x, W.C.e0, s_rpos[f0], s_w, lane, ng0, nleak);
        q1 = march_q_gen<1>(c1w, dM1.x, W.C.e1, s_rpos[f1], s_w, lane, ng0, nleak);
      }
    }
    if (MODE == kMarchB) {
      // k_cg_b's per-pair arithmetic
      double2 rn;
      rn.x = W.rM.x - ak * q0;
      rn.y = W.rM.y - ak * q1;
      mr = rn;
      const double z0 = div_tab(rn.x, dM0), z1 = div_tab(rn.y, dM1);
      if constexpr (SM || PK) {  // {p(k), z} of the edge columns: the next P's halo (lanes 0 and 63)
        const bool ed = mown && (lane == 0 || lane == 63);
        if constexpr (ESR > 0) {
          // staged in the wave's LDS rows (k_cg_march ESR): one store per
          // lane after the walk instead of one store instruction per step
          if (ed) s_ed[(lane == 63 ? ESR : 0) + (mid - g.r0)] = lane == 0 ? make_double2(W.C.e0, z0)
                                                                          : make_double2(W.C.e1, z1);
        } else {
          // (issued by every lane, the others' offsets out of range: under a
          // divergent branch with two active lanes B took 0.7 us longer,
          // profiles/r6_16_ab_edgestore.json)
          bst2<0>(B.ez, ed ? (unsigned)(g.ezo + mid) * 16u : kOOB,
                  lane == 0 ? make_double2(W.C.e0, z0) : make_double2(W.C.e1, z1));
        }
      }
      t0 = make_double2(z0 * rn.x, z1 * rn.y);  // bknum's terms (bondc.f:785-787)
      t1 = make_double2(rn.x * rn.x, rn.y * rn.y);  // snrm's (:872-875)
      acc[0] = acc[0] + t0.x;
      acc[0] = acc[0] + t0.y;
      acc[1] = acc[1] + t1.x;
      acc[1] = acc[1] + t1.y;
    } else {
      mq = make_double2(q0, q1);
      t0 = make_double2(q0 * W.C.e0, q1 * W.C.e1);  // akden's terms (:803-805)
      acc[0] = acc[0] + t0.x;
      acc[0] = acc[0] + t0.y;
    }
  }
  {
    const int m = a.T.m;
    const unsigned eq = SM ? (unsigned)sm_at(a.T, mid, g.col) : (unsigned)((mid - g.r0) * m + g.col);
    if (MODE == kMarchPQ) bst2<kStAux>(B.q, mown ? eq * 8u : kOOB, mq);
    if (MODE == kMarchB) bst2<kStAux>(B.r, mown ? melem<SM>(a, B, mid, g.col) * 8u : kOOB, mr);
    // literal dot terms at the row-major index (the LIT instantiation only:
    // as a runtime-dropped store in the fast order it cost P ~1.7 us)
    if constexpr (LIT) {
      const unsigned to = mown ? (unsigned)(mid * m + g.col) * 8u : kOOB;
      if (MODE != kMarchB) {
        bst2<kNT>(B.t, to, t0);
      } else {
        const unsigned n8 = (unsigned)a.St.N * 8u;
        bst2<kNT>(B.t, mown ? to + n8 : kOOB, t0);
        bst2<kNT>(B.t, mown ? to + 2u * n8 : kOOB, t1);
      }
    }
  }
}

template <int MODE, int D, bool UP, bool SM, int PAUX = 0, bool PK = false, bool LIT = false, int ESR = 0>
__device__ __forceinline__ void march_walk(const CGArgs& a, const MGeom& g, const MBuf& B,
                                           MRow (&ring)[D],
                                           bool first, double bk, double ak,
                                           const double* __restrict__ psrc,
                                           double* __restrict__ pnew, const double2* s_dt,
                                           const unsigned* s_rpos, const unsigned* s_rmap,
                                           double* s_w, double (&acc)[2], double2* s_ed = nullptr) {
  MState W;
  W.U = MWin{0.0, 0.0, 0.0, 0.0};
  W.C = W.U;
  W.Dn = W.U;
  W.cN = W.cM = 0u;
  W.rN = W.rM = make_double2(0.0, 0.0);
  const int nsteps = g.rend - g.r0 + 2;  // rows r0-1 .. rend
  for (int j0 = 0; j0 < nsteps; j0 += D) {
#pragma unroll
    for (int u = 0; u < D; ++u) {
      const int j = j0 + u;
      // no branches around memory instructions: a step past the walk (odd
      // step count) and the prefetch past its end address rows outside the
      // view (loads return 0, stores are dropped) and finish no row
      const MRow R = ring[u];
      march_load<MODE, SM, PAUX, PK>(a, g, B, UP ? g.rend - (j + D) : g.r0 - 1 + j + D, first, psrc, ring[u]);
      march_step<MODE, UP, SM, LIT, PK, ESR>(a, g, B, R, UP ? g.rend - j : g.r0 - 1 + j, first, bk, ak, pnew, s_dt,
                                            s_rpos, s_rmap, s_w, W, acc, s_ed);
    }
  }
}

// PAUX: cache policy of the last-use loads (P: p(k-1); B: r(k)).
// TR: phase probe -- lane 0 of every wave stores {kernel entry, walk end,
// exit, hardware id} wall-clock stamps (100 MHz) into a.mtrace[4 w ..]
// TAG: the epilogue reductions by tagged granules (publish_and_reduce_tagged)
// DEF: deferred reductions (with TAG, strip-major, fast order; see def_totals)
// ESR > 0: B's edge pairs staged in LDS (ESR rows per side) and stored
// after the walk -- bands of <= ESR rows: kEdgeRows strip-major, 16 on the
// row-major march's 8-row bands (the host picks it, CGArgs::mes)
template <int MODE, bool SM = false, int D = kMarchDepth, int PAUX = 0, bool TR = false,
          bool TAG = false, bool PK = false, bool LIT = false, bool DEF = false, int ESR = 0>
// (the deferred instantiations are held to 3 waves per SIMD -- 168 VGPRs:
// the strip-major march's slot-weighted bands assume 3 resident workgroups
// per CU, and their totals code left P at 169 without the bound)
__global__ __launch_bounds__(64 * kMarchWaves, DEF ? 3 : PERC_MARCH_MINW(SM, MODE, PK)) void k_cg_march(CGArgs a) {
  static_assert(!DEF || (TAG && SM && !LIT), "deferred reductions: the tagged strip-major fast march");
  static_assert(ESR == 0 || (MODE == kMarchB && (SM || PK)), "staged edge pairs: the march B with edge pairs");
  const unsigned long long tr_t0 = TR ? wall_clock64() : 0ull;
  unsigned long long tr_t1 = 0ull;
  CGScalars* S = a.S;
  __shared__ double s_red[32];
  __shared__ int s_flag[2];
  __shared__ unsigned s_rpos[kMaxForms], s_rmap[kMaxForms];
  __shared__ double2 s_dt[kDiagTab];
  __shared__ double s_win[kMarchWaves][12 * 64];  // general-path window scratch
  // the launch's iteration comes from the host (launch j of a solve is
  // iteration j + 1 until the stop; later launches return below), so the
  // first rows' loads go out before any device scalar is read
  const int k = a.kiter;
  const bool first = MODE != kMarchB && k == 1;
  // P reads p(k-1) and writes p(k); B reads p(k)
  const double* __restrict__ psrc = a.pb[(MODE == kMarchB ? k : k - 1) & 1];
  double* __restrict__ pnew = a.pb[k & 1];
  const int m = a.T.m, nrows = a.T.nrows, H = a.T.bh;
  const int lb = xcd_logical_block(blockIdx.x, gridDim.x);
  const int lane = threadIdx.x & 63;
  // wave-uniform in SGPRs (the buffer views below must be: a resource
  // the compiler cannot prove uniform gets a readfirstlane loop per access)
  const int w = __builtin_amdgcn_readfirstlane(lb * kMarchWaves + (threadIdx.x >> 6));
  const int spr = m / kMarchW;
  int band, strip;
  MGeom g;
  if (a.wslots > 0) {
    // slot-weighted bands (PERC_MARCH_SLOTS).  Workgroups are dealt one per
    // CU per round: blockIdx / CUs is the round -- the CU slot -- a
    // workgroup runs in (observed on MI355X, speed only: any placement
    // gives the same rows and results).  The waves of the first round get
    // memory requests served first and stream fastest (L = 4096, equal
    // bands: 49 / 56 / 66 us per walk for rounds 0 / 1 / 2,
    // profiles/r3_2_mtrace_static_summary.txt), so the rows of every cycle
    // of wslots neighbouring bands are split by per-round weights: all
    // waves finish together instead of the CU idling while its last round
    // drains.  Band b = q * wslots + round, so neighbouring bands still
    // alternate walk directions.
    const int ns = a.wslots, ncu = gridDim.x / ns;
    // (round 5: the round's workgroups taken in XCD-contiguous order, so a
    // band's neighbouring strips share an L2 for their halo columns,
    // measured no faster: P 76.75 vs 77.04 us, solve 0.1533 vs 0.1526 ms
    // per iteration, profiles/r5_2_ab_L4096.json)
    const int sl = blockIdx.x / ncu, i = blockIdx.x - sl * ncu;
    const int v = __builtin_amdgcn_readfirstlane(i * kMarchWaves + (threadIdx.x >> 6));
    const int Q = ncu * kMarchWaves / spr;  // cycles per strip
    const int q = v / spr;
    strip = v - q * spr;
    band = q * ns + sl;
    const int c0 = (int)((long long)q * nrows / Q), hc = (int)((long long)(q + 1) * nrows / Q) - c0;
    const int* wc = a.wcum[MODE == kMarchB ? 1 : 0];
    g.r0 = c0 + hc * wc[sl] / wc[ns];
    g.rend = c0 + hc * wc[sl + 1] / wc[ns];
  } else {
    band = w / spr;
    strip = w - band * spr;
    g.r0 = band * H;
    g.rend = min(g.r0 + H, nrows);
  }
  const bool active = g.r0 < nrows;  // wave-uniform
  const int c0 = strip * kMarchW;
  g.col = c0 + 2 * lane;
  g.hcol = lane == 0 ? c0 - 1 : c0 + kMarchW;
  g.hok = lane == 0 || lane == 63;
  if (g.hcol < 0 || g.hcol >= m) {
    if (a.T.pbc) g.hcol += g.hcol < 0 ? m : -m;
    else g.hok = false;
  }
  {
    const int hs = g.hcol / kMarchW, hside = g.hcol % kMarchW == kMarchW - 1 ? 1 : 0;
    g.ezh = (2 * hs + hside) * nrows;
    g.ezo = (2 * strip + (lane == 63 ? 1 : 0)) * nrows;
  }
  const bool up = (a.march_alt && (band & 1)) != (MODE == kMarchB);
  const int nsteps = g.rend - g.r0 + 2;
  // (the square lattice's three column classes: nibble codes, and the u16
  // codes of the open square lattice)
  g.cb0 = g.cb1 = g.cbh = 0u;
  g.lo0 = g.lo1 = 0xFu;
  g.hi0 = g.hi1 = 0u;
  if ((PK || a.sqcls) && (SM || kMarchRmSq)) {
    auto cls = [&](int c) { return c == 0 ? a.ncls[1] : (c == m - 1 ? a.ncls[2] : a.ncls[0]); };
    g.cb0 = cls(g.col);
    g.cb1 = cls(g.col + 1);
    g.cbh = cls(g.hcol);
    g.lo0 = g.col == 0 ? 1u : 0xFu;
    g.hi0 = g.col == 0 ? 6u : 0u;
    g.lo1 = g.col + 1 == m - 1 ? 3u : 0xFu;
    g.hi1 = g.col + 1 == m - 1 ? 4u : 0u;
  }
  const MBuf B = march_bufs<MODE, SM, PK>(a, g, psrc, pnew);
  MRow ring[D];
  if (active) {
#pragma unroll
    for (int u = 0; u < D; ++u)
      if (u < nsteps) march_load<MODE, SM, PAUX, PK>(a, g, B, up ? g.rend - u : g.r0 - 1 + u, first, psrc, ring[u]);
  }
  // (B, strip-major, fast order, x on the electrode-side rows: iteration
  // k - 1's x update of those rows, its loads issued behind the ring's)
  constexpr bool kXin = MODE == kMarchB && SM && !LIT && !DEF;
  const bool xin = kXin && a.mxin && k > 1 && active;
  double2 xo[2], po[2];
  if constexpr (kXin) {
    const __amdgpu_buffer_rsrc_t rx = rsrc(a.x, (unsigned)a.St.N * 8u);
    const __amdgpu_buffer_rsrc_t rp = rsrc(a.pb[(k - 1) & 1], (unsigned)a.St.N * 8u);
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int xr = e ? nrows - 1 : 0;  // the rows next to the electrodes
      const bool own = xin && xr >= g.r0 && xr < g.rend && (e == 0 || nrows > 1);
      xo[e] = bld2(rx, own ? (unsigned)(xr * m + g.col) * 8u : kOOB);
      po[e] = bld2(rp, own ? (unsigned)sm_at(a.T, xr, g.col) * 8u : kOOB);
    }
  }
  if (S->done) return;
  if constexpr (kXin) {
    // x(k-1) += ak(k-1) p(k-1): the same per-element expression as the
    // update after the walk it replaces (bitwise the same voltages), whose
    // reload held the bands of those rows 2.2 us past their walk (B 73.9 vs
    // 71.7 us without any x update, profiles/r6_10_ab_nobx.json)
    const double akp = S->akprev;
    const __amdgpu_buffer_rsrc_t rx = rsrc(a.x, (unsigned)a.St.N * 8u);
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int xr = e ? nrows - 1 : 0;
      const bool own = xin && xr >= g.r0 && xr < g.rend && (e == 0 || nrows > 1);
      bst2<0>(rx, own ? (unsigned)(xr * m + g.col) * 8u : kOOB,
              make_double2(xo[e].x + akp * po[e].x, xo[e].y + akp * po[e].y));
    }
  }
  if (threadIdx.x < kMaxForms) {
    s_rpos[threadIdx.x] = a.St.F.rpos[threadIdx.x];
    s_rmap[threadIdx.x] = a.St.F.rmap[threadIdx.x];
  }
  load_dtab(a.St, s_dt);
  __syncthreads();
  double bk = S->bk, ak = S->ak;
  // bknum of this iteration's ak (P's collector epilogue): the scalar, or
  // with kDefB the total this launch formed from B(k-1)'s granules
  double bkn_it = S->bknum;
  if constexpr (DEF) {
    // the previous launch's totals, formed here (its first rows' loads are
    // in flight): B takes P(k)'s q.p -> ak (kDefP); P takes B(k-1)'s z.r and
    // r.r -> bk, err and the stop test (kDefB)
    __shared__ double s_grp[2 * kDefGroups];
    const bool live = !(a.mdef & kDefBench);
    int* derr = live ? a.merr : nullptr;
    if (MODE == kMarchB) {
      if (a.mdef & kDefP) {
        double tp[1];
        def_totals<1>(a.mgran, gridDim.x, a.mtag, derr, tp, s_red, s_grp, a.mdsc1 != 0);
        const double bknum = (a.mdef & kDefB) && k > 1 ? S->bkn[(k - 1) & 1] : S->bknum;
        ak = sgpr_double(bknum / tp[0]);
        if (lb == 0 && threadIdx.x == 0 && live) {
          S->akden = tp[0];
          S->ak = ak;
        }
      }
    } else if (!first && (a.mdef & kDefB)) {
      double tb[2];
      def_totals<2>(a.mgran_b, gridDim.x, a.mtag - 1.0, derr, tb, s_red, s_grp, a.mdsc1 != 0);
      if (march_def_epilogue(a, k - 1, tb, lb == 0 && threadIdx.x == 0, bk)) return;  // (uniform)
      bk = sgpr_double(bk);
      bkn_it = sgpr_double(tb[0]);
    }
  }
  double acc[2] = {0.0, 0.0};
  if (active) {
    double* s_w = s_win[threadIdx.x >> 6];
    double2* s_ed = nullptr;
    if constexpr (ESR > 0) {
      __shared__ double2 s_edge[kMarchWaves][2 * (ESR > 0 ? ESR : 1)];
      s_ed = s_edge[threadIdx.x >> 6];
    }
    if (up)
      march_walk<MODE, D, true, SM, PAUX, PK, LIT, ESR>(a, g, B, ring, first, bk, ak, psrc, pnew, s_dt, s_rpos,
                                                       s_rmap, s_w, acc, s_ed);
    else
      march_walk<MODE, D, false, SM, PAUX, PK, LIT, ESR>(a, g, B, ring, first, bk, ak, psrc, pnew, s_dt, s_rpos,
                                                        s_rmap, s_w, acc, s_ed);
    if constexpr (ESR > 0) {
      // the band's staged edge pairs: lane l stores row r0 + l of side
      // l / ESR (the wave's own LDS writes, in program order: no barrier)
      __builtin_amdgcn_wave_barrier();
      asm volatile("" ::: "memory");
      const int h = g.rend - g.r0, base = 2 * strip * nrows + g.r0;
#pragma unroll
      for (int sd = 0; sd < (2 * ESR + 63) / 64; ++sd) {
        const int e = sd * 64 + lane, side = e / ESR, row = e % ESR;
        bst2<0>(B.ez, e < 2 * ESR && row < h ? (unsigned)(base + side * nrows + row) * 16u : kOOB,
                s_ed[e < 2 * ESR ? e : 0]);
      }
    }
    if (MODE == kMarchP && !SM && !first && !a.bx) {
      // row-major q-free solve: x += ak p(k-1) on the band's x rows, after
      // the walk.  Inside it the x load feeding the x store made every step
      // wait for vmcnt(0), draining the prefetched rows (L = 8192: 2 684
      // read requests in flight vs B's 3 229, profiles/r4_5_*level*)
      const int N = a.St.N;
      for (int gr = g.r0; gr < g.rend; ++gr) {
        const int i = gr * m + g.col;
        if (a.xrows != 0 && i >= a.xrows && i < N - a.xrows) continue;
        const double2 pv = *reinterpret_cast<const double2*>(psrc + i);
        double2 xv = *reinterpret_cast<const double2*>(a.x + i);
        xv.x = xv.x + ak * pv.x;
        xv.y = xv.y + ak * pv.y;
        *reinterpret_cast<double2*>(a.x + i) = xv;
      }
    }
    if (MODE == kMarchB && SM && !(kXin && a.mxin)) {
      // strip-major q-free solve: x (row-major) += ak p(k) on the band's x
      // rows, after the walk (loads and stores inside it would put a
      // vmcnt(0) in every step); k_cg_b's x update of the q-storing solve
      const int N = a.St.N;
      for (int gr = g.r0; gr < g.rend; ++gr) {
        const int i = gr * m + g.col;  // m is a multiple of the strip width
        if (a.xrows != 0 && i >= a.xrows && i < N - a.xrows) continue;
        const double2 pv = *reinterpret_cast<const double2*>(psrc + sm_at(a.T, gr, g.col));
        double2 xv = *reinterpret_cast<const double2*>(a.x + i);
        xv.x = xv.x + ak * pv.x;
        xv.y = xv.y + ak * pv.y;
        *reinterpret_cast<double2*>(a.x + i) = xv;
      }
    }
  }
  if constexpr (TR) {
    tr_t1 = wall_clock64();
    if (lane == 0) {
      unsigned hw;
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
      unsigned xcc;
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
      a.mtrace[4 * (size_t)w + 0] = tr_t0;
      a.mtrace[4 * (size_t)w + 1] = tr_t1;
      a.mtrace[4 * (size_t)w + 3] = ((unsigned long long)xcc << 32) | hw;
    }
  }
  bool pub_only = false;
  if constexpr (DEF) pub_only = (a.mdef & (MODE == kMarchB ? kDefB : kDefP)) != 0;
  if (pub_only) {
    // publish only: this launch's workgroup partials, {value, tag} granules
    // written through; the next launch (or k_march_epi) forms the totals
    constexpr int NV = MODE == kMarchB ? 2 : 1;
    double v[NV];
#pragma unroll
    for (int j = 0; j < NV; ++j) v[j] = acc[j];
    block_sum<NV>(v, s_red);
    if (threadIdx.x == 0) {
      const int ngroups = red_groups(gridDim.x);
      double* gran = MODE == kMarchB ? a.mgran_b : a.mgran;
      const __amdgpu_buffer_rsrc_t rg = rsrc(gran, (unsigned)(NV * ((int)gridDim.x + ngroups) * 16));
#pragma unroll
      for (int j = 0; j < NV; ++j)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, make_double2(v[j], a.mtag)), rg,
                                               (j * (int)gridDim.x + lb) * 16, 0, 16);
    }
  } else if (MODE != kMarchB) {
    double v[1] = {acc[0]}, tot[1];
    const bool last = TAG ? publish_and_reduce_tagged<1>(v, a.mgran, a.tickets, lb, gridDim.x, a.mtag,
                                                         a.merr, tot, s_red, s_flag)
                          : publish_and_reduce<1>(v, a.partials, a.tickets, lb, gridDim.x, tot, s_red, s_flag);
    if (last) {
      if (threadIdx.x == 0) {
        if (a.slab) {
          S->part[0] = tot[0];
          if (a.pub) a.pub[0] = tot[0];
        } else {
          S->akprev = S->ak;
          S->akden = tot[0];
          S->ak = bkn_it / tot[0];
        }
      }
    }
  } else {
    double tot[2];
    const bool last =
        TAG ? publish_and_reduce_tagged<2>(acc, a.mgran_b, a.tickets + a.tstride, lb, gridDim.x, a.mtag, a.merr, tot,
                                           s_red, s_flag)
            : publish_and_reduce<2>(acc, a.partials + a.pstride, a.tickets + a.tstride, lb, gridDim.x,
                                    tot, s_red, s_flag);
    if (last) {
      if (threadIdx.x == 0) {  // k_cg_b's epilogue
        const int kk = S->iter + 1;
        const double err = sqrt(tot[1]) / S->bnrm;
        S->bk = tot[0] / S->bknum;
        S->bknum = tot[0];
        S->err = err;
        if (kk - 1 < a.err_hist_cap) a.err_hist[kk - 1] = err;
        S->iter = kk;
        if (!(err > S->tol) || kk >= S->itmax + 1) S->done = 1;
      }
    }
  }
  if constexpr (TR) {
    if (lane == 0) a.mtrace[4 * (size_t)w + 2] = wall_clock64();
  }
}


// the edge {p, z} of the first P: z = r0/d of every strip's first and last
// column (B stores both later), the same division the march forms; p(0) is
// not read (the first P takes p = z)
__global__ __launch_bounds__(kBlock) void k_edge_init(CGArgs a) {
  const int nrows = a.T.nrows, spr = a.T.m / kMarchW;
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= 2 * spr * nrows) return;
  const int row = e % nrows, ss = e / nrows, strip = ss / 2, side = ss % 2;
  const int col = strip * kMarchW + (side ? kMarchW - 1 : 0);
  const int i = a.sm ? sm_at(a.T, row, col) : row * a.T.m + col;  // (r and the u16 codes in the march's layout)
  reinterpret_cast<double2*>(a.ez)[e] = make_double2(0.0, div_tab(a.r[i], a.St.dtab[diag_idx(a.St.code[i])]));
}

// The last iteration's x update of the electrode-side rows (CGArgs::mxin):
// x += ak(K) p(K), p(K) strip-major in pb[K & 1]; m threads per row
__global__ __launch_bounds__(kBlock) void k_march_xpend(CGArgs a) {
  const CGScalars* S = a.S;
  const int m = a.T.m, nrows = a.T.nrows, K = S->iter;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (K < 1 || i >= 2 * m || (i >= m && nrows < 2)) return;
  const int row = i < m ? 0 : nrows - 1, col = i < m ? i : i - m;
  const double* __restrict__ p = a.pb[K & 1];
  a.x[row * m + col] = a.x[row * m + col] + S->ak * p[sm_at(a.T, row, col)];
}

// The deferred epilogue of a chunk's last B (DEF): one workgroup of the
// march's shape forms the z.r and r.r totals as the next P would and stores
// iter, err, bk, the stop flag -- the host reads them after each chunk.  The
// next P forms the same values again (every store idempotent).
__global__ __launch_bounds__(64 * kMarchWaves) void k_march_epi(CGArgs a) {
  __shared__ double s_red[32];
  __shared__ double s_grp[2 * kDefGroups];
  if (a.S->done) return;
  double tb[2], bk;
  def_totals<2>(a.mgran_b, a.mnwg, a.mtag, a.merr, tb, s_red, s_grp, true);
  march_def_epilogue(a, a.kiter, tb, threadIdx.x == 0, bk);
}

}  // namespace
}  // namespace perc
#pragma clang diagnostic pop
