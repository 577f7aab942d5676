// sync_bench.hip -- the resident solve's per-iteration synchronisation
// (two block sums + two all-reductions of 1 and 2 fp64 partials per
// workgroup, as k_cg_res) in isolation, by transport variant, on one
// cooperative grid of G workgroups of NT threads:
//   flat  res_gather's all-gather: every workgroup publishes 16-B {value,
//         tag} granules write-through and wave 0 of every workgroup sweeps
//         all G of them until every tag is this epoch's
//   miss  the same, but a re-poll reloads only the granules not yet seen
//   xcc   two levels by the XCD a workgroup runs on (HW_REG_XCC_ID): the
//         granules of one XCD are read by that XCD's leader only (L2-local
//         traffic), the leaders publish 8 XCD totals, which every workgroup
//         polls (8 granules instead of G)
//   xcc1  the same with write-through level-1 stores
// Prints us per iteration and the number of wrong totals (the partials are
// small integers: every association gives the exact total).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/sync_bench.hip -o sync_bench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                 \
    }                                                                               \
  } while (0)

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
constexpr int kMaxG = 1024;
constexpr unsigned kSpin = 1u << 24;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, bytes, 0x00020000);
}
__device__ __forceinline__ double2 ld16(__amdgpu_buffer_rsrc_t r, int off) {
  return __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 16));
}
template <int AUX>
__device__ __forceinline__ void st16(__amdgpu_buffer_rsrc_t r, int off, double v, double tag) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, make_double2(v, tag)), r, off, 0, AUX);
}
__device__ __forceinline__ double wsum(double v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
template <int NV>
__device__ __forceinline__ void block_sum(double (&v)[NV], double* s) {
  const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const double t = wsum(v[j]);
    if ((threadIdx.x & 63) == 0) s[j * 16 + w] = t;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    double t = 0.0;
    for (int i = 0; i < nw; ++i) t += s[j * 16 + i];
    v[j] = t;
  }
  __syncthreads();
}

struct Args {
  double* gran;      // flat: [2 kinds][NVmax][G]; xcc: level 1 [2][NV][8][128]
  double* gran2;     // xcc: level 2 [2 kinds][2 parity][NV][8]
  unsigned* reg;     // xcc registration: [8] counters, then [G] ranks
  int G, iters;
  int* bad;
  int* timeout;
};

// ---- flat / miss -----------------------------------------------------------
template <int NV, bool MISS>
__device__ bool gather_flat(const Args& a, double* gran, double tag, const double (&v)[NV],
                            double (&tot)[NV], double* s_red) {
  __syncthreads();
  const int G = a.G;
  const __amdgpu_buffer_rsrc_t rg = rsrc(gran, (unsigned)(NV * G * 16));
  if (threadIdx.x == 0)
    for (int j = 0; j < NV; ++j) st16<16>(rg, (j * G + blockIdx.x) * 16, v[j], tag);
  bool ok = true;
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    constexpr int kPer = kMaxG / 64;
    double val[NV][kPer];
    unsigned seen = 0;  // MISS: bit (j * kPer + s) once granule seen
    const int per = (G + 63) / 64;
    for (unsigned spin = 0;; ++spin) {
      bool all = true;
#pragma unroll
      for (int j = 0; j < NV; ++j)
        for (int s = 0; s < per; ++s) {
          const int i = lane + 64 * s;
          if (i >= G) continue;
          const unsigned bit = 1u << (j * kPer + s);
          if (MISS && (seen & bit)) continue;
          const double2 g = ld16(rg, (j * G + i) * 16);
          if (g.y == tag) {
            val[j][s] = g.x;
            seen |= bit;
          } else {
            all = false;
          }
        }
      if (__builtin_amdgcn_readfirstlane(__all(all))) break;
      if (spin > kSpin) {
        ok = false;
        break;
      }
      if (!MISS) seen = 0;
      __builtin_amdgcn_s_sleep(1);
    }
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      double acc = 0.0;
      for (int s = 0; s < per; ++s)
        if (lane + 64 * s < G) acc += val[j][s];
      const double t = wsum(acc);
      if (lane == 0) s_red[24 + j] = t;
    }
    if (lane == 0) s_red[30] = ok ? 1.0 : 0.0;
  }
  __syncthreads();
  for (int j = 0; j < NV; ++j) tot[j] = s_red[24 + j];
  ok = s_red[30] != 0.0;
  __syncthreads();
  return ok;
}

// ---- xcc -------------------------------------------------------------------
struct XccInfo {
  int xcc, rank, nx;
};
template <int NV, int L1AUX>
__device__ bool gather_xcc(const Args& a, int kind, unsigned epoch, const XccInfo& X,
                           const double (&v)[NV], double (&tot)[NV], double* s_red) {
  __syncthreads();
  const double tag = (double)epoch;
  const int par = epoch & 1;
  // level 1: [kind][j][xcc][rank]
  const __amdgpu_buffer_rsrc_t r1 = rsrc(a.gran, (unsigned)(2 * 2 * 8 * 128 * 16));
  const __amdgpu_buffer_rsrc_t r2 = rsrc(a.gran2, (unsigned)(2 * 2 * 2 * 8 * 16));
  auto o1 = [&](int j, int x, int r) { return (((kind * 2 + j) * 8 + x) * 128 + r) * 16; };
  auto o2 = [&](int j, int x) { return (((kind * 2 + par) * 2 + j) * 8 + x) * 16; };
  if (threadIdx.x == 0)
    for (int j = 0; j < NV; ++j) st16<L1AUX>(r1, o1(j, X.xcc, X.rank), v[j], tag);
  bool ok = true;
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    if (X.rank == 0) {  // the XCD's leader: its XCD's granules, then publish
      double acc[NV];
      for (unsigned spin = 0;; ++spin) {
        bool all = true;
#pragma unroll
        for (int j = 0; j < NV; ++j) {
          acc[j] = 0.0;
          for (int r = lane; r < X.nx; r += 64) {
            const double2 g = ld16(r1, o1(j, X.xcc, r));
            all = all && g.y == tag;
            acc[j] += g.x;
          }
        }
        if (__builtin_amdgcn_readfirstlane(__all(all))) break;
        if (spin > kSpin) {
          ok = false;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
#pragma unroll
      for (int j = 0; j < NV; ++j) {
        const double t = wsum(acc[j]);
        if (lane == 0) st16<16>(r2, o2(j, X.xcc), t, tag);
      }
    }
    // level 2: the 8 XCD totals (lanes 0..7)
    double acc[NV];
    for (unsigned spin = 0;; ++spin) {
      bool all = true;
#pragma unroll
      for (int j = 0; j < NV; ++j) {
        acc[j] = 0.0;
        if (lane < 8) {
          const double2 g = ld16(r2, o2(j, lane));
          all = all && g.y == tag;
          acc[j] = g.x;
        }
      }
      if (__builtin_amdgcn_readfirstlane(__all(all))) break;
      if (spin > kSpin) {
        ok = false;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const double t = wsum(acc[j]);
      if (lane == 0) s_red[24 + j] = t;
    }
    if (lane == 0) s_red[30] = ok ? 1.0 : 0.0;
  }
  __syncthreads();
  for (int j = 0; j < NV; ++j) tot[j] = s_red[24 + j];
  ok = s_red[30] != 0.0;
  __syncthreads();
  return ok;
}

// VAR: 0 flat, 1 miss, 2 xcc (plain level 1), 3 xcc1 (write-through level 1)
template <int VAR>
__global__ void k_sync(Args a) {
  __shared__ double s_red[64];
  __shared__ int s_x[3];
  XccInfo X{0, 0, 0};
  if constexpr (VAR >= 2) {
    if (threadIdx.x == 0) {
      const int x = __builtin_amdgcn_s_getreg((3 << 11) | 20) & 7;
      const unsigned r = __hip_atomic_fetch_add(&a.reg[x * 32], 1u, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
      // every workgroup has registered: the grid's arrival count
      __hip_atomic_fetch_add(&a.reg[8 * 32], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      for (unsigned spin = 0; __hip_atomic_load(&a.reg[8 * 32], __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT) < (unsigned)a.G; ++spin) {
        if (spin > kSpin) {
          *a.timeout = 1;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      s_x[0] = x;
      s_x[1] = (int)r;
      s_x[2] = (int)__hip_atomic_load(&a.reg[x * 32], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    X = XccInfo{s_x[0], s_x[1], s_x[2]};
  }
  const int G = a.G;
  unsigned epoch = 0;
  int bad = 0;
  for (int it = 0; it < a.iters; ++it) {
    double v1[1] = {threadIdx.x == 0 ? (double)(blockIdx.x + 1 + it) : 0.0}, t1[1];
    block_sum<1>(v1, s_red);
    ++epoch;
    bool ok;
    if constexpr (VAR == 0) ok = gather_flat<1, false>(a, a.gran, (double)epoch, v1, t1, s_red);
    else if constexpr (VAR == 1) ok = gather_flat<1, true>(a, a.gran, (double)epoch, v1, t1, s_red);
    else ok = gather_xcc<1, VAR == 2 ? 0 : 16>(a, 0, epoch, X, v1, t1, s_red);
    if (!ok) break;
    double v2[2] = {threadIdx.x == 0 ? (double)blockIdx.x : 0.0, threadIdx.x == 0 ? 2.0 : 0.0}, t2[2];
    block_sum<2>(v2, s_red);
    ++epoch;
    if constexpr (VAR == 0)
      ok = gather_flat<2, false>(a, a.gran + 2 * kMaxG * 2, (double)epoch, v2, t2, s_red);
    else if constexpr (VAR == 1)
      ok = gather_flat<2, true>(a, a.gran + 2 * kMaxG * 2, (double)epoch, v2, t2, s_red);
    else ok = gather_xcc<2, VAR == 2 ? 0 : 16>(a, 1, epoch, X, v2, t2, s_red);
    if (!ok) break;
    const double want1 = (double)G * (G + 1) / 2 + (double)G * it, want20 = (double)G * (G - 1) / 2;
    bad += (t1[0] != want1) + (t2[0] != want20) + (t2[1] != 2.0 * G);
  }
  if (threadIdx.x == 0 && bad) atomicAdd(a.bad, bad);
}

template <int VAR>
double run(int G, int NT, int iters, int* bad_out) {
  Args a{};
  a.G = G;
  a.iters = iters;
  CK(hipMalloc(&a.gran, sizeof(double) * 2 * 2 * 8 * 128 * 2 + sizeof(double) * 4 * kMaxG * 4));
  CK(hipMalloc(&a.gran2, sizeof(double) * 2 * 2 * 2 * 8 * 2));
  CK(hipMalloc(&a.reg, sizeof(unsigned) * 9 * 32));
  CK(hipMalloc(&a.bad, sizeof(int) * 2));
  a.timeout = a.bad + 1;
  double best = 1e30;
  for (int rep = 0; rep < 4; ++rep) {
    CK(hipMemset(a.gran, 0, sizeof(double) * 2 * 2 * 8 * 128 * 2 + sizeof(double) * 4 * kMaxG * 4));
    CK(hipMemset(a.gran2, 0, sizeof(double) * 2 * 2 * 2 * 8 * 2));
    CK(hipMemset(a.reg, 0, sizeof(unsigned) * 9 * 32));
    CK(hipMemset(a.bad, 0, sizeof(int) * 2));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    void* args[] = {&a};
    CK(hipEventRecord(e0));
    CK(hipLaunchCooperativeKernel((const void*)k_sync<VAR>, dim3(G), dim3(NT), args, 0, 0));
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, e0, e1));
    int hb[2];
    CK(hipMemcpy(hb, a.bad, sizeof(hb), hipMemcpyDeviceToHost));
    *bad_out = hb[0] + (hb[1] ? 1000000 : 0);
    if (ms * 1e3 / iters < best) best = ms * 1e3 / iters;
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
  }
  CK(hipFree(a.gran));
  CK(hipFree(a.gran2));
  CK(hipFree(a.reg));
  CK(hipFree(a.bad));
  return best;
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? std::atoi(argv[1]) : 2000;
  const char* names[] = {"flat", "miss", "xcc", "xcc1"};
  for (int G : {256, 128}) {
    for (int NT : {1024, 256}) {
      for (int v = 0; v < 4; ++v) {
        int bad = 0;
        double us = v == 0 ? run<0>(G, NT, iters, &bad)
                    : v == 1 ? run<1>(G, NT, iters, &bad)
                    : v == 2 ? run<2>(G, NT, iters, &bad)
                             : run<3>(G, NT, iters, &bad);
        std::printf("G %4d NT %4d %-5s %7.3f us per iteration (2 reductions)  wrong %d\n", G, NT,
                    names[v], us, bad);
        std::fflush(stdout);
      }
    }
  }
  return 0;
}
