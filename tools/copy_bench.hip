// copy_bench.hip -- which streaming shape reaches the HBM ceiling on this
// chip: 512 MB -> 512 MB copies (past the 256 MB Infinity Cache) with
// chunked vs grid-stride work, 1-8 x 16 B in flight per thread,
// nontemporal or plain accesses, several grids and block sizes.
//   hipcc --offload-arch=gfx950 -O3 tools/copy_bench.hip -o tools/copy_bench
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHK(x)                                                                  \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

typedef double dvec2 __attribute__((ext_vector_type(2)));

template <int U, bool NT, bool CHUNK>
__global__ void k_copy(const dvec2* __restrict__ a, dvec2* __restrict__ b, long long n) {
  const long long nthreads = (long long)gridDim.x * blockDim.x;
  if (CHUNK) {
    const long long chunk = ((n + gridDim.x - 1) / gridDim.x + blockDim.x * U - 1) /
                            (blockDim.x * U) * (blockDim.x * U);
    const long long i0 = blockIdx.x * chunk, i1 = std::min(i0 + chunk, n);
    for (long long base = i0 + threadIdx.x; base < i1; base += (long long)blockDim.x * U) {
      dvec2 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const long long i = base + (long long)u * blockDim.x;
        if (i < i1) v[u] = NT ? __builtin_nontemporal_load(a + i) : a[i];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const long long i = base + (long long)u * blockDim.x;
        if (i < i1) {
          if (NT) __builtin_nontemporal_store(v[u], b + i);
          else b[i] = v[u];
        }
      }
    }
  } else {
    for (long long base = blockIdx.x * (long long)blockDim.x + threadIdx.x; base < n;
         base += nthreads * U) {
      dvec2 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const long long i = base + u * nthreads;
        if (i < n) v[u] = NT ? __builtin_nontemporal_load(a + i) : a[i];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const long long i = base + u * nthreads;
        if (i < n) {
          if (NT) __builtin_nontemporal_store(v[u], b + i);
          else b[i] = v[u];
        }
      }
    }
  }
}

struct V {
  char name[48];
  void (*k)(const dvec2*, dvec2*, long long);
  int grid, block;
};

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 20;
  const long long n = (512ll << 20) / 16;  // double2 elements in 512 MB
  dvec2 *a, *b;
  CHK(hipMalloc(&a, n * 16));
  CHK(hipMalloc(&b, n * 16));
  CHK(hipMemset(a, 0, n * 16));
  std::vector<V> vs;
  auto add = [&](const char* tag, void (*k)(const dvec2*, dvec2*, long long), int g, int bl) {
    V v;
    snprintf(v.name, sizeof v.name, "%s_g%d_b%d", tag, g, bl);
    v.k = k;
    v.grid = g;
    v.block = bl;
    vs.push_back(v);
  };
  for (int g : {1024, 2048, 4096, 8192, 16384, 65536}) {
    add("chunk_u1", k_copy<1, false, true>, g, 256);
    add("chunk_u4", k_copy<4, false, true>, g, 256);
    add("chunk_u4_nt", k_copy<4, true, true>, g, 256);
    add("gs_u1", k_copy<1, false, false>, g, 256);
    add("gs_u4", k_copy<4, false, false>, g, 256);
    add("gs_u4_nt", k_copy<4, true, false>, g, 256);
    add("gs_u8", k_copy<8, false, false>, g, 256);
  }
  for (int g : {1024, 2048, 4096}) {
    add("gs_u4", k_copy<4, false, false>, g, 512);
    add("gs_u4", k_copy<4, false, false>, g, 1024);
    add("chunk_u4", k_copy<4, false, true>, g, 1024);
  }
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  for (auto& v : vs) v.k<<<v.grid, v.block>>>(a, b, n);
  CHK(hipDeviceSynchronize());
  std::vector<double> best(vs.size(), 1e30);
  for (int round = 0; round < 3; ++round)
    for (size_t i = 0; i < vs.size(); ++i) {
      CHK(hipEventRecord(e0));
      for (int r = 0; r < reps; ++r) vs[i].k<<<vs[i].grid, vs[i].block>>>(a, b, n);
      CHK(hipEventRecord(e1));
      CHK(hipEventSynchronize(e1));
      float t;
      CHK(hipEventElapsedTime(&t, e0, e1));
      best[i] = std::min(best[i], (double)t / reps);
    }
  for (size_t i = 0; i < vs.size(); ++i)
    printf("%-28s %8.4f ms %7.1f GB/s\n", vs[i].name, best[i],
           2.0 * n * 16 / (best[i] * 1e-3) / 1e9);
  return 0;
}
