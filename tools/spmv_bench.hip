// spmv_bench.hip -- microbenchmark of SpMV / streaming kernel variants on the
// L x L square-lattice interior CSR (the CG system's pattern) plus STREAM-like
// copy references, all timed with HIP events, interleaved in one process.
//
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/spmv_bench.hip -o spmv_bench
//   ./spmv_bench [L=4096] [reps=20]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHK(x)                                                                      \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));     \
      exit(1);                                                                      \
    }                                                                               \
  } while (0)

constexpr int kBlock = 256;
constexpr int kSlots = 6;

struct Csr {
  int N;
  const int* rowptr;
  const int* col;
  const double* val;
  const double* diag;
};

__device__ __forceinline__ int cdiv(int a, int b) { return (a + b - 1) / b; }

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ void tile(const Csr& A, const double* __restrict__ x,
                                     double* __restrict__ y, int r0, int a, int b,
                                     double* s_prod) {
  const int lane = threadIdx.x & 63;
  const int r = r0 + lane;
  const bool valid = r < A.N;
  const int last = min(63, A.N - 1 - r0);
  const int e0 = __shfl(a, 0, 64);
  const int ne = __shfl(b, last, 64) - e0;
  const double xi = valid ? x[r] : 0.0;
  const double di = valid ? A.diag[r] : 0.0;
  const int jmax = max(ne - 1, 0);
  int c[kSlots];
  double v[kSlots], xv[kSlots];
#pragma unroll
  for (int s = 0; s < kSlots; ++s) {
    const int j = min(lane + 64 * s, jmax);
    c[s] = A.col[e0 + j];
    v[s] = A.val[e0 + j];
  }
#pragma unroll
  for (int s = 0; s < kSlots; ++s) xv[s] = x[c[s]];
#pragma unroll
  for (int s = 0; s < kSlots; ++s) s_prod[lane + 64 * s] = v[s] * xv[s];
  wave_sync();
  if (valid) {
    double acc = di * xi;
    for (int k = a - e0; k < b - e0; ++k) acc = acc + s_prod[k];
    y[r] = acc;
  }
  wave_sync();
}

// variant 0: contiguous tile chunk per block (current libperc)
// variant 1: tiles interleaved over all waves of the grid
template <int MODE>
__global__ __launch_bounds__(kBlock) void k_spmv_wave(Csr A, const double* __restrict__ x,
                                                      double* __restrict__ y) {
  __shared__ double s_prod[4][64 * kSlots];
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int ntile = cdiv(A.N, 64);
  int t, t1, stride;
  if (MODE == 0) {
    const int chunk = cdiv(ntile, gridDim.x);
    t = blockIdx.x * chunk + wid;
    t1 = min((int)blockIdx.x * chunk + chunk, ntile);
    stride = 4;
  } else {
    t = blockIdx.x * 4 + wid;
    t1 = ntile;
    stride = gridDim.x * 4;
  }
  int a = 0, b = 0;
  if (t < t1 && t * 64 + lane < A.N) { a = A.rowptr[t * 64 + lane]; b = A.rowptr[t * 64 + lane + 1]; }
  for (; t < t1; t += stride) {
    int an = 0, bn = 0;
    const int nt = t + stride;
    if (nt < t1 && nt * 64 + lane < A.N) { an = A.rowptr[nt * 64 + lane]; bn = A.rowptr[nt * 64 + lane + 1]; }
    tile(A, x, y, t * 64, a, b, s_prod[wid]);
    a = an;
    b = bn;
  }
}

// variant 2: thread per row, direct loads (no LDS), grid-stride
__global__ __launch_bounds__(kBlock) void k_spmv_row(Csr A, const double* __restrict__ x,
                                                     double* __restrict__ y) {
  for (int r = blockIdx.x * blockDim.x + threadIdx.x; r < A.N; r += gridDim.x * blockDim.x) {
    const int a = A.rowptr[r], b = A.rowptr[r + 1];
    double acc = A.diag[r] * x[r];
    double pr[kSlots];
#pragma unroll
    for (int s = 0; s < kSlots; ++s) {
      const int k = min(a + s, b - 1);
      pr[s] = A.val[k] * x[A.col[k]];
    }
#pragma unroll
    for (int s = 0; s < kSlots; ++s)
      if (a + s < b) acc = acc + pr[s];
    y[r] = acc;
  }
}

// streaming references
__global__ __launch_bounds__(kBlock) void k_copy(const double2* __restrict__ a,
                                                 double2* __restrict__ b, long long n2) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n2;
       i += (long long)gridDim.x * blockDim.x)
    b[i] = a[i];
}
__global__ __launch_bounds__(kBlock) void k_copy_chunk(const double2* __restrict__ a,
                                                       double2* __restrict__ b, long long n2) {
  const long long chunk = (n2 + gridDim.x - 1) / gridDim.x;
  const long long i0 = blockIdx.x * chunk, i1 = min(i0 + chunk, n2);
#pragma unroll 4
  for (long long i = i0 + threadIdx.x; i < i1; i += blockDim.x) b[i] = a[i];
}
// B-like: 3 streams in, 1 out (r -= ak q; z = r/d; sums discarded into r)
__global__ __launch_bounds__(kBlock) void k_resid(const double2* __restrict__ q,
                                                  const double2* __restrict__ d,
                                                  double2* __restrict__ r, long long n2,
                                                  double ak, double* sink) {
  double acc = 0.0;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n2;
       i += (long long)gridDim.x * blockDim.x) {
    const double2 qv = q[i], dv = d[i];
    double2 rv = r[i];
    rv.x = rv.x - ak * qv.x;
    rv.y = rv.y - ak * qv.y;
    r[i] = rv;
    acc = acc + (rv.x / dv.x) * rv.x + (rv.y / dv.y) * rv.y;
  }
  if (acc == 12345.0) *sink = acc;
}

int main(int argc, char** argv) {
  const int L = argc > 1 ? atoi(argv[1]) : 4096;
  const int reps = argc > 2 ? atoi(argv[2]) : 20;
  const int m = L, n = L, N = m * (n - 2);
  // interior CSR of the square lattice: neighbours i-m, i-1, i+1, i+m (row
  // edges drop i-1 / i+1; first / last interior rows drop i-m / i+m)
  std::vector<int> rowptr(N + 1);
  std::vector<int> col;
  col.reserve((size_t)N * 4);
  for (int i = 0; i < N; ++i) {
    rowptr[i] = (int)col.size();
    const int cx = i % m;
    if (i - m >= 0) col.push_back(i - m);
    if (cx > 0) col.push_back(i - 1);
    if (cx < m - 1) col.push_back(i + 1);
    if (i + m < N) col.push_back(i + m);
  }
  rowptr[N] = (int)col.size();
  const long long nnz = (long long)col.size();
  std::vector<double> val(nnz + 8, -1.0), diag(N, 4.0), x(N + 2, 1.0);
  for (long long k = 0; k < nnz; k += 3) val[k] = -1e-12;
  int *d_rp, *d_col;
  double *d_val, *d_diag, *d_x, *d_y, *d_a, *d_b, *d_c, *sink;
  CHK(hipMalloc(&d_rp, sizeof(int) * (N + 1)));
  CHK(hipMalloc(&d_col, sizeof(int) * (nnz + 8)));
  CHK(hipMalloc(&d_val, sizeof(double) * (nnz + 8)));
  CHK(hipMalloc(&d_diag, sizeof(double) * N));
  CHK(hipMalloc(&d_x, sizeof(double) * (N + 2)));
  CHK(hipMalloc(&d_y, sizeof(double) * (N + 2)));
  CHK(hipMalloc(&d_a, sizeof(double) * (N + 2)));
  CHK(hipMalloc(&d_b, sizeof(double) * (N + 2)));
  CHK(hipMalloc(&d_c, sizeof(double) * (N + 2)));
  CHK(hipMalloc(&sink, 64));
  CHK(hipMemcpy(d_rp, rowptr.data(), sizeof(int) * (N + 1), hipMemcpyHostToDevice));
  CHK(hipMemcpy(d_col, col.data(), sizeof(int) * nnz, hipMemcpyHostToDevice));
  CHK(hipMemset(d_col + nnz, 0, sizeof(int) * 8));
  CHK(hipMemcpy(d_val, val.data(), sizeof(double) * (nnz + 8), hipMemcpyHostToDevice));
  CHK(hipMemcpy(d_diag, diag.data(), sizeof(double) * N, hipMemcpyHostToDevice));
  CHK(hipMemcpy(d_x, x.data(), sizeof(double) * (N + 2), hipMemcpyHostToDevice));
  CHK(hipMemcpy(d_a, x.data(), sizeof(double) * (N + 2), hipMemcpyHostToDevice));
  CHK(hipMemcpy(d_b, x.data(), sizeof(double) * (N + 2), hipMemcpyHostToDevice));
  CHK(hipMemcpy(d_c, x.data(), sizeof(double) * (N + 2), hipMemcpyHostToDevice));
  Csr A{N, d_rp, d_col, d_val, d_diag};
  const double spmv_bytes = 8.0 * (N + nnz) + 4.0 * nnz + 4.0 * (N + 1) + 16.0 * N;
  printf("L=%d N=%d nnz=%lld spmv bytes=%.0f\n", L, N, nnz, spmv_bytes);
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  const int ntile = (N + 63) / 64;
  struct V { const char* name; int grid; int kind; double bytes; };
  std::vector<V> vs = {
      {"wave_chunk_g2048", 2048, 0, spmv_bytes}, {"wave_inter_g2048", 2048, 1, spmv_bytes},
      {"wave_inter_g1024", 1024, 1, spmv_bytes}, {"wave_inter_g4096", 4096, 1, spmv_bytes},
      {"wave_inter_full", (ntile + 3) / 4, 1, spmv_bytes},
      {"row_g2048", 2048, 2, spmv_bytes},        {"row_full", (N + 255) / 256, 2, spmv_bytes},
      {"copy_gs_g2048", 2048, 3, 16.0 * N},      {"copy_chunk_g2048", 2048, 4, 16.0 * N},
      {"copy_gs_g8192", 8192, 3, 16.0 * N},      {"resid_gs_g2048", 2048, 5, 32.0 * N},
  };
  std::vector<double> best(vs.size(), 1e30), sum(vs.size(), 0.0);
  auto launch = [&](const V& v) {
    switch (v.kind) {
      case 0: k_spmv_wave<0><<<v.grid, kBlock>>>(A, d_x, d_y); break;
      case 1: k_spmv_wave<1><<<v.grid, kBlock>>>(A, d_x, d_y); break;
      case 2: k_spmv_row<<<v.grid, kBlock>>>(A, d_x, d_y); break;
      case 3: k_copy<<<v.grid, kBlock>>>((const double2*)d_a, (double2*)d_b, N / 2); break;
      case 4: k_copy_chunk<<<v.grid, kBlock>>>((const double2*)d_a, (double2*)d_b, N / 2); break;
      case 5: k_resid<<<v.grid, kBlock>>>((const double2*)d_a, (const double2*)d_b,
                                          (double2*)d_c, N / 2, 1e-30, sink); break;
    }
  };
  for (auto& v : vs) launch(v);
  CHK(hipDeviceSynchronize());
  for (int round = 0; round < 3; ++round)
    for (size_t k = 0; k < vs.size(); ++k) {
      CHK(hipEventRecord(e0));
      for (int i = 0; i < reps; ++i) launch(vs[k]);
      CHK(hipEventRecord(e1));
      CHK(hipEventSynchronize(e1));
      float t;
      CHK(hipEventElapsedTime(&t, e0, e1));
      const double ms = t / reps;
      best[k] = std::min(best[k], ms);
      sum[k] += ms;
    }
  // correctness cross-check of the SpMV variants
  std::vector<double> y(N);
  for (int kind : {0, 1, 2}) {
    V v{"", 2048, kind, 0};
    CHK(hipMemset(d_y, 0, sizeof(double) * N));
    launch(v);
    CHK(hipMemcpy(y.data(), d_y, sizeof(double) * N, hipMemcpyDeviceToHost));
    double s = 0;
    for (int i = 0; i < N; ++i) s += y[i];
    printf("check kind %d: sum y = %.17g\n", kind, s);
  }
  for (size_t k = 0; k < vs.size(); ++k)
    printf("%-20s grid %6d  best %8.4f ms  mean %8.4f ms  %7.1f GB/s (best)\n", vs[k].name,
           vs[k].grid, best[k], sum[k] / 3, vs[k].bytes / (best[k] * 1e-3) / 1e9);
  return 0;
}
