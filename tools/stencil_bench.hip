// stencil_bench.hip -- variants of the stencil-coded SpMV (perc_device.hip
// "Stencil-coded operator") on the L x L square interior system, timed with
// HIP events; all variants are checked bitwise against variant A.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/stencil_bench.hip -o tools/stencil_bench
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CHK(x)                                                                  \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

constexpr int kBlock = 256;
constexpr int kForms = 8, kSlots = 6;
struct Forms { int off[kForms][kSlots]; };
struct View { int N; const uint16_t* code; double ng0, nleak; Forms F; };

__device__ __forceinline__ int cdiv(int a, int b) { return (a + b - 1) / b; }

template <int S>
__device__ __forceinline__ double combine(unsigned c, const double* xv, const bool* use, double xi,
                                          double ng0, double nleak) {
  const int cnt = (c >> 8) & 7;
  double gv[S], rs = 0.0;
#pragma unroll
  for (int j = 0; j < S; ++j) {
    gv[j] = ((c >> j) & 1u) ? ng0 : nleak;
    if (j < cnt) rs = rs + gv[j];
  }
  double acc = (-rs) * xi;
#pragma unroll
  for (int j = 0; j < S; ++j) {
    const double pr = gv[j] * xv[j];
    acc = use[j] ? acc + pr : acc;
  }
  return acc;
}

// A: thread-row, stride kBlock, batch R, chunk ALIGN-rounded
template <int S, int R, int ALIGN>
__global__ __launch_bounds__(kBlock) void kA(View A, const double* __restrict__ x,
                                             double* __restrict__ y) {
  __shared__ int s_off[kForms * kSlots];
  if (threadIdx.x < kForms * kSlots) s_off[threadIdx.x] = A.F.off[threadIdx.x / kSlots][threadIdx.x % kSlots];
  __syncthreads();
  const int chunk = (cdiv(A.N, gridDim.x) + ALIGN - 1) / ALIGN * ALIGN;
  const int i0 = blockIdx.x * chunk, i1 = min(i0 + chunk, A.N);
  for (int base = i0 + threadIdx.x; base < i1; base += kBlock * R) {
    unsigned c[R];
#pragma unroll
    for (int k = 0; k < R; ++k) {
      const int i = base + k * kBlock;
      c[k] = i < i1 ? A.code[i] : 0u;
    }
    double xv[R][S], xi[R];
    bool use[R][S];
#pragma unroll
    for (int k = 0; k < R; ++k) {
      const int i = base + k * kBlock;
      const int ii = i < i1 ? i : base;
      const int f = c[k] >> 11, cnt = (c[k] >> 8) & 7;
#pragma unroll
      for (int j = 0; j < S; ++j) {
        const int col = ii + s_off[f * kSlots + j];
        use[k][j] = j < cnt && (unsigned)col < (unsigned)A.N;
        xv[k][j] = x[use[k][j] ? col : ii];
      }
      xi[k] = x[ii];
    }
#pragma unroll
    for (int k = 0; k < R; ++k) {
      const int i = base + k * kBlock;
      if (i < i1) y[i] = combine<S>(c[k], xv[k], use[k], xi[k], A.ng0, A.nleak);
    }
  }
}

// B: square, two consecutive rows per thread (i even): centre window as three
// 16-B loads, rows +-m as 16-B loads (m even), code pair as one u32; rows whose
// form is not the interior form (edges) re-gather through the form table.
template <int R>
__global__ __launch_bounds__(kBlock) void kB(View A, int m, const double* __restrict__ x,
                                             double* __restrict__ y) {
  __shared__ int s_off[kForms * kSlots];
  if (threadIdx.x < kForms * kSlots) s_off[threadIdx.x] = A.F.off[threadIdx.x / kSlots][threadIdx.x % kSlots];
  __syncthreads();
  const int np = A.N / 2;  // N even here
  const int chunk = (cdiv(np, gridDim.x) + 127) / 128 * 128;
  const int q0 = blockIdx.x * chunk, q1 = min(q0 + chunk, np);
  for (int base = q0 + threadIdx.x; base < q1; base += kBlock * R) {
    unsigned cc[R];
    double2 xl[R], xc[R], xr[R], xu[R], xd[R];
#pragma unroll
    for (int k = 0; k < R; ++k) {
      const int q = base + k * kBlock;
      const int qq = q < q1 ? q : base;
      const int i = 2 * qq;
      cc[k] = *reinterpret_cast<const unsigned*>(A.code + i);
      xl[k] = i >= 2 ? *reinterpret_cast<const double2*>(x + i - 2) : make_double2(0, 0);
      xc[k] = *reinterpret_cast<const double2*>(x + i);
      xr[k] = i + 2 < A.N ? *reinterpret_cast<const double2*>(x + i + 2) : make_double2(0, 0);
      xu[k] = i + m < A.N ? *reinterpret_cast<const double2*>(x + i + m) : make_double2(0, 0);
      xd[k] = i >= m ? *reinterpret_cast<const double2*>(x + i - m) : make_double2(0, 0);
    }
#pragma unroll
    for (int k = 0; k < R; ++k) {
      const int q = base + k * kBlock;
      if (q >= q1) continue;
      const int i = 2 * q;
      double2 out;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int r = i + h;
        const unsigned c = h ? cc[k] >> 16 : cc[k] & 0xffffu;
        const int f = c >> 11, cnt = (c >> 8) & 7;
        double xv[4];
        bool use[4];
        const double xi = h ? xc[k].y : xc[k].x;
        if (f == 0) {  // interior form: -m, -1, +1, +m
          xv[0] = h ? xd[k].y : xd[k].x;
          xv[1] = h ? xc[k].x : xl[k].y;
          xv[2] = h ? xr[k].x : xc[k].y;
          xv[3] = h ? xu[k].y : xu[k].x;
          use[0] = r >= m;
          use[1] = true;
          use[2] = true;
          use[3] = r + m < A.N;
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int col = r + s_off[f * kSlots + j];
            use[j] = j < cnt && (unsigned)col < (unsigned)A.N;
            xv[j] = x[use[j] ? col : r];
          }
        }
        const double v = combine<4>(c, xv, use, xi, A.ng0, A.nleak);
        if (h) out.y = v; else out.x = v;
      }
      *reinterpret_cast<double2*>(y + i) = out;
    }
  }
}

__global__ __launch_bounds__(kBlock) void k_copy(const double2* __restrict__ a,
                                                 double2* __restrict__ b, int n2) {
  const int chunk = (cdiv(n2, gridDim.x) + 255) / 256 * 256;
  const int i0 = blockIdx.x * chunk, i1 = min(i0 + chunk, n2);
#pragma unroll 4
  for (int i = i0 + threadIdx.x; i < i1; i += kBlock) b[i] = a[i];
}

int main(int argc, char** argv) {
  const int L = argc > 1 ? atoi(argv[1]) : 4096;
  const int reps = argc > 2 ? atoi(argv[2]) : 20;
  const int m = L, n = L, N = m * (n - 2);
  // forms of the square non-periodic lattice: 0 interior, 1 left, 2 right
  Forms F{};
  const int fo[3][4] = {{-m, -1, 1, m}, {-m, 1, m, 0}, {-m, -1, m, 0}};
  const int fc[3] = {4, 3, 3};
  for (int f = 0; f < 3; ++f)
    for (int j = 0; j < 4; ++j) F.off[f][j] = fo[f][j];
  std::vector<uint16_t> code(N + 8);
  unsigned s = 12345;
  for (int i = 0; i < N; ++i) {
    const int cx = i % m;
    const int f = cx == 0 ? 1 : cx == m - 1 ? 2 : 0;
    s = s * 1103515245u + 12345u;
    code[i] = (uint16_t)(((s >> 16) & 15u) | (unsigned)fc[f] << 8 | (unsigned)f << 11);
  }
  std::vector<double> x(N + 8);
  for (int i = 0; i < N; ++i) x[i] = 1.0 + (i % 977) * 1e-3;
  uint16_t* d_code;
  double *d_x, *d_y, *d_y2;
  CHK(hipMalloc(&d_code, 2 * (N + 8)));
  CHK(hipMalloc(&d_x, 8 * (N + 8)));
  CHK(hipMalloc(&d_y, 8 * (N + 8)));
  CHK(hipMalloc(&d_y2, 8 * (N + 8)));
  CHK(hipMemcpy(d_code, code.data(), 2 * (N + 8), hipMemcpyHostToDevice));
  CHK(hipMemcpy(d_x, x.data(), 8 * (N + 8), hipMemcpyHostToDevice));
  View A{N, d_code, -1.0, -1e-12, F};
  const double bytes = 18.0 * N;
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  struct V { const char* name; int kind, grid; double bytes; };
  std::vector<V> vs;
  for (int g : {1024, 2048, 4096, 8192, 16384}) {
    static char buf[64][40];
    static int nb = 0;
    snprintf(buf[nb], 40, "A_r4_al1_g%d", g); vs.push_back({buf[nb++], 0, g, bytes});
    snprintf(buf[nb], 40, "A_r4_al256_g%d", g); vs.push_back({buf[nb++], 1, g, bytes});
    snprintf(buf[nb], 40, "A_r2_al256_g%d", g); vs.push_back({buf[nb++], 2, g, bytes});
    snprintf(buf[nb], 40, "A_r8_al256_g%d", g); vs.push_back({buf[nb++], 3, g, bytes});
    snprintf(buf[nb], 40, "B_r2_g%d", g); vs.push_back({buf[nb++], 4, g, bytes});
    snprintf(buf[nb], 40, "B_r4_g%d", g); vs.push_back({buf[nb++], 5, g, bytes});
    snprintf(buf[nb], 40, "copy_g%d", g); vs.push_back({buf[nb++], 6, g, 16.0 * N});
  }
  auto launch = [&](const V& v, double* y) {
    switch (v.kind) {
      case 0: kA<4, 4, 1><<<v.grid, kBlock>>>(A, d_x, y); break;
      case 1: kA<4, 4, 256><<<v.grid, kBlock>>>(A, d_x, y); break;
      case 2: kA<4, 2, 256><<<v.grid, kBlock>>>(A, d_x, y); break;
      case 3: kA<4, 8, 256><<<v.grid, kBlock>>>(A, d_x, y); break;
      case 4: kB<2><<<v.grid, kBlock>>>(A, m, d_x, y); break;
      case 5: kB<4><<<v.grid, kBlock>>>(A, m, d_x, y); break;
      case 6: k_copy<<<v.grid, kBlock>>>((const double2*)d_x, (double2*)y, N / 2); break;
    }
  };
  // reference result
  kA<4, 4, 1><<<8192, kBlock>>>(A, d_x, d_y);
  CHK(hipDeviceSynchronize());
  std::vector<double> ref(N), got(N);
  CHK(hipMemcpy(ref.data(), d_y, 8 * N, hipMemcpyDeviceToHost));
  for (auto& v : vs) {
    if (v.kind == 6) continue;
    CHK(hipMemset(d_y2, 0, 8 * N));
    launch(v, d_y2);
    CHK(hipDeviceSynchronize());
    CHK(hipMemcpy(got.data(), d_y2, 8 * N, hipMemcpyDeviceToHost));
    if (memcmp(got.data(), ref.data(), 8 * (size_t)N) != 0) printf("MISMATCH %s\n", v.name);
  }
  std::vector<double> best(vs.size(), 1e30);
  for (int round = 0; round < 3; ++round)
    for (size_t k = 0; k < vs.size(); ++k) {
      CHK(hipEventRecord(e0));
      for (int i = 0; i < reps; ++i) launch(vs[k], d_y2);
      CHK(hipEventRecord(e1));
      CHK(hipEventSynchronize(e1));
      float t;
      CHK(hipEventElapsedTime(&t, e0, e1));
      best[k] = std::min(best[k], (double)t / reps);
    }
  printf("L=%d N=%d stencil bytes=%.0f\n", L, N, bytes);
  for (size_t k = 0; k < vs.size(); ++k)
    printf("%-20s %8.4f ms %7.1f GB/s\n", vs[k].name, best[k], vs[k].bytes / (best[k] * 1e-3) / 1e9);
  return 0;
}
