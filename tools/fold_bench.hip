// fold_bench.hip -- ns per term of the literal dot order's serial fold
// (linbcg's ascending-j sums, Square/bondc.f:785-787, 803-805, 872-875) on
// one wave, by the way the terms reach the adding lane:
//   0  LDS broadcast per 64-term chunk (fold_chunk, round 4-5: perc_cg.h)
//   1  scalar loads: every lane adds the same uniform term from SGPRs
//      (s_load, no LDS; safe across a kernel boundary, where the scalar
//      cache starts cold)
//   2  LDS broadcast, 16 terms per chain read as one batch ahead of the adds
// Each variant folds NC = 2 chains of N terms and checks the sums bitwise
// against a host sequential fold.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/fold_bench.hip -o tools/fold_bench
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                \
    }                                                                         \
  } while (0)

__device__ __forceinline__ void lds_order() {
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
}

// variant 0: the library's fold (ring of 8 chunks in registers, LDS broadcast)
__global__ __launch_bounds__(64) void k_fold0(const double* __restrict__ t0, const double* __restrict__ t1,
                                              int N, double* out) {
  __shared__ double s_t[2][64];
  const int lane = threadIdx.x;
  constexpr int D = 8;
  double r0[D], r1[D];
  const int nch = (N + 63) / 64;
#pragma unroll
  for (int u = 0; u < D; ++u) {
    const int j = min(u * 64 + lane, N - 1);
    r0[u] = t0[j];
    r1[u] = t1[j];
  }
  double a0 = 0.0, a1 = 0.0;
  for (int c0 = 0; c0 < nch; c0 += D) {
#pragma unroll
    for (int u = 0; u < D; ++u) {
      const int c = c0 + u;
      s_t[0][lane] = r0[u];
      s_t[1][lane] = r1[u];
      const int j = min((c + D) * 64 + lane, N - 1);
      r0[u] = t0[j];
      r1[u] = t1[j];
      lds_order();
      const int cnt = max(0, min(64, N - c * 64));
      if (cnt == 64) {
#pragma unroll
        for (int l = 0; l < 64; ++l) {
          a0 = a0 + s_t[0][l];
          a1 = a1 + s_t[1][l];
        }
      } else {
        for (int l = 0; l < cnt; ++l) {
          a0 = a0 + s_t[0][l];
          a1 = a1 + s_t[1][l];
        }
      }
      lds_order();
    }
  }
  if (lane == 0) {
    out[0] = a0;
    out[1] = a1;
  }
}

// variant 1: uniform (scalar) loads, U terms per chain per step
template <int U>
__global__ __launch_bounds__(64) void k_fold1(const double* __restrict__ t0, const double* __restrict__ t1,
                                              int N, double* out) {
  double a0 = 0.0, a1 = 0.0;
  int j = 0;
  for (; j + U <= N; j += U) {
    double v0[U], v1[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      v0[u] = t0[j + u];
      v1[u] = t1[j + u];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      a0 = a0 + v0[u];
      a1 = a1 + v1[u];
    }
  }
  for (; j < N; ++j) {
    a0 = a0 + t0[j];
    a1 = a1 + t1[j];
  }
  if (threadIdx.x == 0) {
    out[0] = a0;
    out[1] = a1;
  }
}

// variant 3: uniform loads double-buffered -- the next U terms per chain are
// requested before the current U are added (2 x 2 x U doubles of SGPRs)
template <int U>
__global__ __launch_bounds__(64) void k_fold3(const double* __restrict__ t0, const double* __restrict__ t1,
                                              int N, double* out) {
  double a0 = 0.0, a1 = 0.0;
  const int nfull = N / U * U;
  double c0[U], c1[U];
  if (nfull > 0) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      c0[u] = t0[u];
      c1[u] = t1[u];
    }
  }
  for (int j = 0; j < nfull; j += U) {
    const int jn = j + U < nfull ? j + U : j;  // (the last batch re-reads itself)
    double n0[U], n1[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      n0[u] = t0[jn + u];
      n1[u] = t1[jn + u];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      a0 = a0 + c0[u];
      a1 = a1 + c1[u];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      c0[u] = n0[u];
      c1[u] = n1[u];
    }
  }
  for (int j = nfull; j < N; ++j) {
    a0 = a0 + t0[j];
    a1 = a1 + t1[j];
  }
  if (threadIdx.x == 0) {
    out[0] = a0;
    out[1] = a1;
  }
}

// variant 2: LDS broadcast, the chunk's 64 terms read in batches of B ahead
template <int B>
__global__ __launch_bounds__(64) void k_fold2(const double* __restrict__ t0, const double* __restrict__ t1,
                                              int N, double* out) {
  __shared__ __attribute__((aligned(16))) double s_t[2][64];
  const int lane = threadIdx.x;
  constexpr int D = 8;
  double r0[D], r1[D];
  const int nch = (N + 63) / 64;
#pragma unroll
  for (int u = 0; u < D; ++u) {
    const int j = min(u * 64 + lane, N - 1);
    r0[u] = t0[j];
    r1[u] = t1[j];
  }
  double a0 = 0.0, a1 = 0.0;
  for (int c0 = 0; c0 < nch; c0 += D) {
#pragma unroll
    for (int u = 0; u < D; ++u) {
      const int c = c0 + u;
      s_t[0][lane] = r0[u];
      s_t[1][lane] = r1[u];
      const int j = min((c + D) * 64 + lane, N - 1);
      r0[u] = t0[j];
      r1[u] = t1[j];
      lds_order();
      const int cnt = max(0, min(64, N - c * 64));
      if (cnt == 64) {
        const double2* p0 = reinterpret_cast<const double2*>(s_t[0]);
        const double2* p1 = reinterpret_cast<const double2*>(s_t[1]);
#pragma unroll
        for (int b = 0; b < 32; b += B / 2) {
          double2 x0[B / 2], x1[B / 2];
#pragma unroll
          for (int i = 0; i < B / 2; ++i) {
            x0[i] = p0[b + i];
            x1[i] = p1[b + i];
          }
#pragma unroll
          for (int i = 0; i < B / 2; ++i) {
            a0 = a0 + x0[i].x;
            a1 = a1 + x1[i].x;
            a0 = a0 + x0[i].y;
            a1 = a1 + x1[i].y;
          }
        }
      } else {
        for (int l = 0; l < cnt; ++l) {
          a0 = a0 + s_t[0][l];
          a1 = a1 + s_t[1][l];
        }
      }
      lds_order();
    }
  }
  if (lane == 0) {
    out[0] = a0;
    out[1] = a1;
  }
}

int main(int argc, char** argv) {
  const int N = argc > 1 ? atoi(argv[1]) : (4 << 20);
  std::vector<double> h0(N), h1(N);
  unsigned long long s = 12345;
  for (int i = 0; i < N; ++i) {
    s = s * 6364136223846793005ull + 1442695040888963407ull;
    h0[i] = (double)(s >> 11) * 1e-10 * ((s & 1) ? 1.0 : -1.0);
    s = s * 6364136223846793005ull + 1442695040888963407ull;
    h1[i] = (double)(s >> 11) * 1e-12;
  }
  double w0 = 0.0, w1 = 0.0;
  for (int i = 0; i < N; ++i) {
    w0 = w0 + h0[i];
    w1 = w1 + h1[i];
  }
  double *d0, *d1, *dout;
  CK(hipMalloc(&d0, N * 8));
  CK(hipMalloc(&d1, N * 8));
  CK(hipMalloc(&dout, 16));
  CK(hipMemcpy(d0, h0.data(), N * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(d1, h1.data(), N * 8, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto run = [&](const char* name, auto kern) {
    kern();
    CK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < 3; ++r) {
      CK(hipEventRecord(e0));
      kern();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      best = ms < best ? ms : best;
    }
    double o[2];
    CK(hipMemcpy(o, dout, 16, hipMemcpyDeviceToHost));
    printf("{\"variant\": \"%s\", \"N\": %d, \"ms\": %.3f, \"ns_per_term\": %.3f, \"bitwise\": %s}\n", name, N,
           best, best * 1e6 / N, (o[0] == w0 && o[1] == w1) ? "true" : "false");
    fflush(stdout);
  };
  run("lds_chunk", [&] { k_fold0<<<1, 64>>>(d0, d1, N, dout); });
  run("scalar_u8", [&] { k_fold1<8><<<1, 64>>>(d0, d1, N, dout); });
  run("scalar_u16", [&] { k_fold1<16><<<1, 64>>>(d0, d1, N, dout); });
  run("scalar_u32", [&] { k_fold1<32><<<1, 64>>>(d0, d1, N, dout); });
  run("scalar_db4", [&] { k_fold3<4><<<1, 64>>>(d0, d1, N, dout); });
  run("scalar_db8", [&] { k_fold3<8><<<1, 64>>>(d0, d1, N, dout); });
  run("lds_batch8", [&] { k_fold2<8><<<1, 64>>>(d0, d1, N, dout); });
  run("lds_batch16", [&] { k_fold2<16><<<1, 64>>>(d0, d1, N, dout); });
  return 0;
}
