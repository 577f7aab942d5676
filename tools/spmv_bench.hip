// spmv_bench.hip -- stand-alone A/B harness for the CSR SpMV (dsprsax order,
// percolation_amd/csrc/perc_csr.h): the interior Kirchhoff pattern of an
// L x L square lattice (diagonal first, then the off-diagonals in ascending
// column order, 2-4 per row; values from a fixed hash), the production
// k_spmv timed with HIP events on one resident round of workgroups, and
// candidate kernels defined here checked bitwise against it.  Bytes per
// launch on SURVEY §8(d)'s model: rowptr 4 + diag 8 + x 8 + y 8 B per row,
// col 4 + val 8 B per entry.
//
//   hipcc ... tools/spmv_bench.hip -o tools/spmv_bench && ./tools/spmv_bench 4096 20
#include "perc_csr.h"

#include <cstdio>
#include <cstdlib>
#include <cstring>
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

double hval(unsigned long long k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdull;
  k ^= k >> 33;
  return -1.0 - (double)(k >> 11) * 0x1.0p-53;
}

// Candidate 1: one row per lane (scalar CSR), the row's <= NS entries
// loaded unconditionally (clamped to the row's last entry, selects), all
// gathers in flight together; no LDS.
template <int NS>
__global__ __launch_bounds__(kBlock) void k_spmv_row(CsrView A, const double* __restrict__ x,
                                                     double* __restrict__ y) {
  const int stride = gridDim.x * kBlock;
  for (int i = blockIdx.x * kBlock + threadIdx.x; i < A.N; i += stride) {
    const int a = A.rowptr[i], b = A.rowptr[i + 1];
    int c[NS];
    double v[NS], xv[NS];
#pragma unroll
    for (int j = 0; j < NS; ++j) {
      const int k = min(a + j, b - 1 < a ? a : b - 1);
      c[j] = A.col[k];
      v[j] = A.val[k];
    }
    const double xi = x[i], di = A.diag[i];
#pragma unroll
    for (int j = 0; j < NS; ++j) xv[j] = x[c[j]];
    double acc = di * xi;
#pragma unroll
    for (int j = 0; j < NS; ++j) acc = j < b - a ? acc + v[j] * xv[j] : acc;
    y[i] = acc;
  }
}

// Candidate 2: the same, two rows per lane per step (rows i and i + stride)
template <int NS>
__global__ __launch_bounds__(kBlock) void k_spmv_row2(CsrView A, const double* __restrict__ x,
                                                      double* __restrict__ y) {
  const int stride = gridDim.x * kBlock;
  for (int i0 = blockIdx.x * kBlock + threadIdx.x; i0 < A.N; i0 += 2 * stride) {
    int a[2], b[2], c[2][NS];
    double v[2][NS], xv[2][NS], xi[2], di[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int i = min(i0 + u * stride, A.N - 1);
      a[u] = A.rowptr[i];
      b[u] = A.rowptr[i + 1];
    }
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int j = 0; j < NS; ++j) {
        const int k = min(a[u] + j, b[u] - 1 < a[u] ? a[u] : b[u] - 1);
        c[u][j] = A.col[k];
        v[u][j] = A.val[k];
      }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int i = min(i0 + u * stride, A.N - 1);
      xi[u] = x[i];
      di[u] = A.diag[i];
#pragma unroll
      for (int j = 0; j < NS; ++j) xv[u][j] = x[c[u][j]];
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int i = i0 + u * stride;
      double acc = di[u] * xi[u];
#pragma unroll
      for (int j = 0; j < NS; ++j) acc = j < b[u] - a[u] ? acc + v[u][j] * xv[u][j] : acc;
      if (i < A.N) y[i] = acc;
    }
  }
}

// Candidate 3: one row per thread, the once-read streams (col, val, diag)
// loaded nontemporal and y stored nontemporal; x (gathered, re-read by the
// neighbouring rows) and rowptr keep the default policy
template <int NS>
__global__ __launch_bounds__(kBlock) void k_spmv_nt(CsrView A, const double* __restrict__ x,
                                                    double* __restrict__ y) {
  const int i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= A.N) return;
  const int a = A.rowptr[i], b = A.rowptr[i + 1];
  int c[NS];
  double v[NS], xv[NS];
  const int last = b - 1 < a ? a : b - 1;
#pragma unroll
  for (int j = 0; j < NS; ++j) {
    const int k = min(a + j, last);
    c[j] = __builtin_nontemporal_load(A.col + k);
    v[j] = __builtin_nontemporal_load(A.val + k);
  }
  const double xi = x[i], di = __builtin_nontemporal_load(A.diag + i);
#pragma unroll
  for (int j = 0; j < NS; ++j) xv[j] = x[c[j]];
  double acc = di * xi;
#pragma unroll
  for (int j = 0; j < NS; ++j) acc = j < b - a ? acc + v[j] * xv[j] : acc;
  __builtin_nontemporal_store(acc, y + i);
}

// Candidate 4: 4 aligned slots per row (ELL: cols int4, vals 2 x double2, a
// per-row count byte; padding slots never added) -- 16-B loads, no rowptr
struct Ell {
  const int4* col;
  const double2* val;
  const unsigned char* cnt;
  const double* diag;
  int N;
};
template <bool NT>
__global__ __launch_bounds__(kBlock) void k_spmv_ell(Ell E, const double* __restrict__ x, double* __restrict__ y) {
  const int i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= E.N) return;
  int4 c;
  double2 v0, v1;
  double di;
  if (NT) {
    typedef int iv4 __attribute__((ext_vector_type(4)));
    typedef double dv2 __attribute__((ext_vector_type(2)));
    const iv4 cc = __builtin_nontemporal_load(reinterpret_cast<const iv4*>(E.col) + i);
    const dv2 a0 = __builtin_nontemporal_load(reinterpret_cast<const dv2*>(E.val) + 2 * i);
    const dv2 a1 = __builtin_nontemporal_load(reinterpret_cast<const dv2*>(E.val) + 2 * i + 1);
    c = make_int4(cc.x, cc.y, cc.z, cc.w);
    v0 = make_double2(a0.x, a0.y);
    v1 = make_double2(a1.x, a1.y);
    di = __builtin_nontemporal_load(E.diag + i);
  } else {
    c = E.col[i];
    v0 = E.val[2 * i];
    v1 = E.val[2 * i + 1];
    di = E.diag[i];
  }
  const int n = E.cnt[i];
  const double xi = x[i];
  const double x0 = x[c.x], x1 = x[c.y], x2 = x[c.z], x3 = x[c.w];
  double acc = di * xi;
  acc = 0 < n ? acc + v0.x * x0 : acc;
  acc = 1 < n ? acc + v0.y * x1 : acc;
  acc = 2 < n ? acc + v1.x * x2 : acc;
  acc = 3 < n ? acc + v1.y * x3 : acc;
  if (NT) __builtin_nontemporal_store(acc, y + i);
  else y[i] = acc;
}

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
  return ms / reps;
}

}  // namespace

int main(int argc, char** argv) {
  const int L = argc > 1 ? std::atoi(argv[1]) : 4096;
  const int reps = argc > 2 ? std::atoi(argv[2]) : 20;
  const int m = L, nrows = L - 2, N = m * nrows;
  std::vector<int> rowptr(N + 1), col;
  std::vector<double> val, diag(N), x(N);
  col.reserve((size_t)4 * N);
  val.reserve((size_t)4 * N);
  for (int i = 0; i < N; ++i) {
    rowptr[i] = (int)col.size();
    const int r = i / m, c = i % m;
    const int nb[4] = {r > 0 ? i - m : -1, c > 0 ? i - 1 : -1, c < m - 1 ? i + 1 : -1, r < nrows - 1 ? i + m : -1};
    double d = 0;
    for (int k = 0; k < 4; ++k)
      if (nb[k] >= 0) {
        col.push_back(nb[k]);
        const double v = hval((unsigned long long)i * 8 + k);
        val.push_back(v);
        d -= v;
      }
    diag[i] = d + 1.0;
    x[i] = hval(0x12345ull + (unsigned long long)i) + 2.0;
  }
  rowptr[N] = (int)col.size();
  const long long nnz = rowptr[N];
  for (int k = 0; k < 8; ++k) {  // padding (the production kernel's clamped loads)
    col.push_back(0);
    val.push_back(0.0);
  }
  int *drp, *dcol;
  double *dval, *ddiag, *dx, *dy, *dy2;
  CK(hipMalloc(&drp, (N + 1) * 4));
  CK(hipMalloc(&dcol, col.size() * 4));
  CK(hipMalloc(&dval, val.size() * 8));
  CK(hipMalloc(&ddiag, (size_t)N * 8));
  CK(hipMalloc(&dx, (size_t)N * 8));
  CK(hipMalloc(&dy, (size_t)N * 8));
  CK(hipMalloc(&dy2, (size_t)N * 8));
  CK(hipMemcpy(drp, rowptr.data(), (N + 1) * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dcol, col.data(), col.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dval, val.data(), val.size() * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(ddiag, diag.data(), (size_t)N * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(dx, x.data(), (size_t)N * 8, hipMemcpyHostToDevice));
  CsrView A{N, drp, dcol, dval, ddiag, 4};
  const double bytes = 28.0 * N + 12.0 * (double)nnz;
  perc_ctx h{};
  h.device = 0;
  auto prod = [&]() { spmv_launch(&h, A, dx, dy, 0); };
  const double tp = time_ms(prod, reps);
  std::printf("L = %d: N = %d rows, nnz = %lld, %.1f MB per launch\n", L, N, nnz, bytes / 1e6);
  std::printf("  production k_spmv<4> (one row per thread): %.4f ms = %.1f GB/s\n", tp, bytes / tp / 1e6);
  std::vector<double> y1(N), y2(N);
  CK(hipMemcpy(y1.data(), dy, (size_t)N * 8, hipMemcpyDeviceToHost));
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  auto check = [&](const char* what, double ms) {
    CK(hipMemcpy(y2.data(), dy2, (size_t)N * 8, hipMemcpyDeviceToHost));
    const bool ok = std::memcmp(y1.data(), y2.data(), (size_t)N * 8) == 0;
    std::printf("  %-34s %.4f ms = %.1f GB/s %s\n", what, ms, bytes / ms / 1e6, ok ? "(bitwise)" : "MISMATCH");
  };
  for (int per : {4, 8, 16}) {
    const int G = cus * per;
    char name[64];
    std::snprintf(name, sizeof name, "row per lane, grid %d", G);
    check(name, time_ms([&]() { k_spmv_row<4><<<G, kBlock>>>(A, dx, dy2); }, reps));
    std::snprintf(name, sizeof name, "two rows per lane, grid %d", G);
    check(name, time_ms([&]() { k_spmv_row2<4><<<G, kBlock>>>(A, dx, dy2); }, reps));
  }
  const int Gf = cdiv(N, kBlock);
  check("row per lane, one row per thread", time_ms([&]() { k_spmv_row<4><<<Gf, kBlock>>>(A, dx, dy2); }, reps));
  check("one row per thread, nt streams", time_ms([&]() { k_spmv_nt<4><<<Gf, kBlock>>>(A, dx, dy2); }, reps));
  // the same system in 4 aligned slots per row
  std::vector<int> ec((size_t)4 * N, 0);
  std::vector<double> ev((size_t)4 * N, 0.0);
  std::vector<unsigned char> en(N);
  for (int i = 0; i < N; ++i) {
    en[i] = (unsigned char)(rowptr[i + 1] - rowptr[i]);
    for (int k = rowptr[i]; k < rowptr[i + 1]; ++k) {
      ec[(size_t)4 * i + (k - rowptr[i])] = col[k];
      ev[(size_t)4 * i + (k - rowptr[i])] = val[k];
    }
    for (int k = rowptr[i + 1] - rowptr[i]; k < 4; ++k) ec[(size_t)4 * i + k] = i;  // (never added)
  }
  int* dec;
  double* dev;
  unsigned char* den;
  CK(hipMalloc(&dec, ec.size() * 4));
  CK(hipMalloc(&dev, ev.size() * 8));
  CK(hipMalloc(&den, (size_t)N));
  CK(hipMemcpy(dec, ec.data(), ec.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dev, ev.data(), ev.size() * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(den, en.data(), (size_t)N, hipMemcpyHostToDevice));
  Ell E{reinterpret_cast<const int4*>(dec), reinterpret_cast<const double2*>(dev), den, ddiag, N};
  check("4-slot rows (ELL), 16-B loads", time_ms([&]() { k_spmv_ell<false><<<Gf, kBlock>>>(E, dx, dy2); }, reps));
  check("4-slot rows (ELL), nt streams", time_ms([&]() { k_spmv_ell<true><<<Gf, kBlock>>>(E, dx, dy2); }, reps));
  CsrView AE = A;  // the production launcher given the assembly's ELL copy
  AE.ecol = E.col;
  AE.eval = E.val;
  AE.ecnt = den;
  check("production, ELL copy (spmv_launch)", time_ms([&]() { spmv_launch(&h, AE, dx, dy2, 0); }, reps));
  std::printf("  (ELL moves %.1f MB per launch: 4 slots x 12 B + count 1 B + diag, x, y 24 B per row)\n",
              (49.0 + 24.0) * N / 1e6);
  return 0;
}
