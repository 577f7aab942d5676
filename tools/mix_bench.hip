// mix_bench.hip -- streaming HBM throughput for the read/write mixes of the
// CG kernels at L = 4096 (N = 4094 * 4096 rows, fp64 vectors + u16 codes):
//   ps:  read p, r, code; write p', q      (34 B / row, 47 % writes)
//   b:   read q, r, code; write r in place (26 B / row, 31 % writes)
//   r2w2, r2w1, r3w0, copy: plain mixes for reference
// Pure streams, no stencil: the ceiling the fused kernels could reach with
// their byte counts.  Also nontemporal variants of the stores.
//   hipcc --offload-arch=gfx950 -O3 tools/mix_bench.hip -o tools/mix_bench
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

struct Bufs {
  dvec2 *a, *b, *c, *d;
  const unsigned* code;
  long long n;  // pairs
};

template <int NR, int NW, bool CODE, bool INPLACE, bool NT, int U>
__global__ void k_mix(Bufs B) {
  const long long n = B.n;
  const long long chunk = ((n + gridDim.x - 1) / gridDim.x + blockDim.x * U - 1) /
                          (blockDim.x * U) * (blockDim.x * U);
  const long long i0 = blockIdx.x * chunk, i1 = std::min(i0 + chunk, n);
  for (long long base = i0 + threadIdx.x; base < i1; base += (long long)blockDim.x * U) {
    dvec2 va[U], vb[U];
    unsigned vc[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long i = base + (long long)u * blockDim.x;
      if (i < i1) {
        va[u] = B.a[i];
        if (NR > 1) vb[u] = B.b[i];
        if (NR > 2) va[u] += B.d[i];
        if (CODE) vc[u] = B.code[i];
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long i = base + (long long)u * blockDim.x;
      if (i < i1) {
        dvec2 o1 = va[u] * 0.5;
        if (NR > 1) o1 += vb[u];
        if (CODE) o1 += (double)(vc[u] & 7);
        if (NW >= 1) {
          dvec2* dst = INPLACE ? B.b : B.c;
          if (NT) __builtin_nontemporal_store(o1, dst + i);
          else dst[i] = o1;
        }
        if (NW >= 2) {
          dvec2 o2 = va[u] - 1.0;
          if (NT) __builtin_nontemporal_store(o2, B.d + i);
          else B.d[i] = o2;
        }
        if (NW == 0 && o1.x == 12345.0) B.c[i] = o1;
      }
    }
  }
}

// the CG iteration's real sequence on the solver's buffers: PS-like
// (read pold, r, code; write pnew, q) then B-like (read q, r, code; write r),
// p ping-pong; B optionally walks its chunks in reverse (as k_cg_b does)
template <bool NT, bool REV>
__global__ void k_b_seq(const dvec2* __restrict__ q, dvec2* __restrict__ r,
                        const unsigned* __restrict__ code, long long n) {
  const int lb = REV ? (int)gridDim.x - 1 - (int)blockIdx.x : (int)blockIdx.x;
  const long long chunk = ((n + gridDim.x - 1) / gridDim.x + blockDim.x * 4 - 1) /
                          (blockDim.x * 4) * (blockDim.x * 4);
  const long long i0 = lb * chunk, i1 = std::min(i0 + chunk, n);
  for (long long base = i0 + threadIdx.x; base < i1; base += (long long)blockDim.x * 4) {
    dvec2 vq[4], vr[4];
    unsigned vc[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const long long i = base + (long long)u * blockDim.x;
      if (i < i1) {
        vq[u] = q[i];
        vr[u] = r[i];
        vc[u] = code[i];
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const long long i = base + (long long)u * blockDim.x;
      if (i < i1) {
        const dvec2 o = vr[u] - 0.5 * vq[u] + (double)(vc[u] & 1);
        if (NT) __builtin_nontemporal_store(o, r + i);
        else r[i] = o;
      }
    }
  }
}
template <bool NT>
__global__ void k_ps_seq(const dvec2* __restrict__ pold, const dvec2* __restrict__ r,
                         const unsigned* __restrict__ code, dvec2* __restrict__ pnew,
                         dvec2* __restrict__ q, long long n) {
  const long long chunk = ((n + gridDim.x - 1) / gridDim.x + blockDim.x * 4 - 1) /
                          (blockDim.x * 4) * (blockDim.x * 4);
  const long long i0 = blockIdx.x * chunk, i1 = std::min(i0 + chunk, n);
  for (long long base = i0 + threadIdx.x; base < i1; base += (long long)blockDim.x * 4) {
    dvec2 vp[4], vr[4];
    unsigned vc[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const long long i = base + (long long)u * blockDim.x;
      if (i < i1) {
        vp[u] = pold[i];
        vr[u] = r[i];
        vc[u] = code[i];
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const long long i = base + (long long)u * blockDim.x;
      if (i < i1) {
        const dvec2 pn = 0.5 * vp[u] + vr[u];
        const dvec2 qq = pn * (double)(vc[u] & 3);
        if (NT) {
          __builtin_nontemporal_store(pn, pnew + i);
          __builtin_nontemporal_store(qq, q + i);
        } else {
          pnew[i] = pn;
          q[i] = qq;
        }
      }
    }
  }
}

// march-shaped pure stream: the register-march kernel's access pattern
// (wave = 128-column strip x H-row band, rows r0-1 .. r0+H read, rows
// r0 .. r0+H-1 written, D rows prefetched) with trivial arithmetic
// (row-major: strip stride 128*PPL, row pitch m; strip-major: strip stride
// nrows*128*PPL, row pitch 128*PPL -- every wave then walks one contiguous
// stream; HALO adds the halo-column scalar loads of lanes 0 and 63)
template <int D, int PPL, bool HALO>
__global__ __launch_bounds__(256) void k_march_stream(const double* __restrict__ pold,
                                                      const double* __restrict__ r,
                                                      const unsigned short* __restrict__ code,
                                                      double* __restrict__ pnew,
                                                      double* __restrict__ q, int m, int pitch,
                                                      long long spitch, int nrows, int H) {
  const int lane = threadIdx.x & 63;
  const int w = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int spr = m / (128 * PPL);
  const int band = w / spr, strip = w - band * spr;
  const int r0 = band * H;
  if (r0 >= nrows) return;
  const long long col = strip * spitch + 2 * lane;
  const int rend = min(r0 + H, nrows), nsteps = rend - r0 + 2;
  const long long hcol = lane == 0 ? (strip > 0 ? col - 2 - spitch + 128 * PPL : col)
                                   : (strip + 1 < spr ? col - 126 + spitch : col);
  const bool hok = HALO && (lane == 0 || lane == 63);
  struct Row {
    dvec2 p[PPL], rr[PPL];
    unsigned c[PPL];
    double hp, hr;
    unsigned hc;
  };
  auto load = [&](int gr, Row& R) {
#pragma unroll
    for (int k = 0; k < PPL; ++k) {
      R.p[k] = R.rr[k] = dvec2{0.0, 0.0};
      R.c[k] = 0;
    }
    if (gr >= 0 && gr < nrows) {
#pragma unroll
      for (int k = 0; k < PPL; ++k) {
        const long long i = (long long)gr * pitch + col + 128 * k;
        R.p[k] = *reinterpret_cast<const dvec2*>(pold + i);
        R.rr[k] = *reinterpret_cast<const dvec2*>(r + i);
        R.c[k] = *reinterpret_cast<const unsigned*>(code + i);
      }
      R.hp = R.hr = 0.0;
      R.hc = 0;
      if (hok) {
        const long long hi = (long long)gr * pitch + hcol;
        R.hp = pold[hi];
        R.hr = r[hi];
        R.hc = code[hi];
      }
    }
  };
  dvec2 prev[PPL];
#pragma unroll
  for (int k = 0; k < PPL; ++k) prev[k] = dvec2{0.0, 0.0};
  Row ring[D];
#pragma unroll
  for (int u = 0; u < D; ++u) load(r0 - 1 + u, ring[u]);
  for (int j0 = 0; j0 < nsteps; j0 += D) {
#pragma unroll
    for (int u = 0; u < D; ++u) {
      const int j = j0 + u;
      if (j < nsteps) {
        const Row R = ring[u];
        if (j + D < nsteps) load(r0 - 1 + j + D, ring[u]);
        const int gr = r0 - 1 + j;
#pragma unroll
        for (int k = 0; k < PPL; ++k) {
          dvec2 pn = 0.5 * R.p[k] + R.rr[k] + (double)(R.c[k] & 3);
          if (HALO && k == 0) pn.x += R.hp * R.hr + (double)(R.hc & 1);
          if (gr >= r0 && gr < rend) {
            const long long i = (long long)gr * pitch + col + 128 * k;
            __builtin_nontemporal_store(pn, reinterpret_cast<dvec2*>(pnew + i));
          }
          if (gr - 1 >= r0) {
            const long long i = (long long)(gr - 1) * pitch + col + 128 * k;
            __builtin_nontemporal_store(prev[k] + pn, reinterpret_cast<dvec2*>(q + i));
          }
          prev[k] = pn;
        }
      }
    }
  }
}


// workgroup row-march: a workgroup owns a strip of W columns (W/4 threads,
// column pairs 2t and 2t + W/2) and an H-row band; each step loads one row
// of the strip (p, r, code; D rows ahead in registers), forms the new p row
// into a 4-slot LDS ring, one barrier, then the previous row's neighbour sum
// from LDS.  UPALT: odd bands walk up (shared halo rows read together).
template <int D, int W, bool UPALT>
__global__ __launch_bounds__(W / 4) void k_rowmarch(const double* __restrict__ pold,
                                                     const double* __restrict__ r,
                                                     const unsigned short* __restrict__ code,
                                                     double* __restrict__ pnew,
                                                     double* __restrict__ q, int m, int nrows,
                                                     int H) {
  extern __shared__ double s_ring[];  // 4 slots x (W + 2)
  constexpr int T = W / 4, SL = W + 2;
  const int t = threadIdx.x;
  const int spr = m / W;
  const int band = blockIdx.x / spr, strip = blockIdx.x - band * spr;
  const int r0 = band * H;
  if (r0 >= nrows) return;
  const int rend = min(r0 + H, nrows), nsteps = rend - r0 + 2;
  const bool up = UPALT && (band & 1);
  const int cA = strip * W + 2 * t, cB = cA + W / 2;
  struct Row {
    dvec2 pa, pb, ra, rb;
    unsigned ca, cb;
  };
  auto rowof = [&](int j) { return up ? rend - j : r0 - 1 + j; };
  auto load = [&](int gr, Row& R) {
    R.pa = R.pb = R.ra = R.rb = dvec2{0.0, 0.0};
    R.ca = R.cb = 0;
    if (gr >= 0 && gr < nrows) {
      const long long i = (long long)gr * m;
      R.pa = *reinterpret_cast<const dvec2*>(pold + i + cA);
      R.pb = *reinterpret_cast<const dvec2*>(pold + i + cB);
      R.ra = *reinterpret_cast<const dvec2*>(r + i + cA);
      R.rb = *reinterpret_cast<const dvec2*>(r + i + cB);
      R.ca = *reinterpret_cast<const unsigned*>(code + i + cA);
      R.cb = *reinterpret_cast<const unsigned*>(code + i + cB);
    }
  };
  Row ring[D];
#pragma unroll
  for (int u = 0; u < D; ++u) load(rowof(u), ring[u]);
  if (t < 4) {  // zero halo columns of every slot
    s_ring[t * SL] = 0.0;
    s_ring[t * SL + W + 1] = 0.0;
  }
  for (int j0 = 0; j0 < nsteps; j0 += D) {
#pragma unroll
    for (int u = 0; u < D; ++u) {
      const int j = j0 + u;
      if (j < nsteps) {
        const Row R = ring[u];
        if (j + D < nsteps) load(rowof(j + D), ring[u]);
        const int gr = rowof(j);
        const dvec2 pa = 0.5 * R.pa + R.ra + (double)(R.ca & 3);
        const dvec2 pb = 0.5 * R.pb + R.rb + (double)(R.cb & 3);
        double* sl = s_ring + (j & 3) * SL + 1;
        *reinterpret_cast<dvec2*>(sl + 2 * t) = pa;
        *reinterpret_cast<dvec2*>(sl + 2 * t + W / 2) = pb;
        if (gr >= r0 && gr < rend) {
          const long long i = (long long)gr * m;
          __builtin_nontemporal_store(pa, reinterpret_cast<dvec2*>(pnew + i + cA));
          __builtin_nontemporal_store(pb, reinterpret_cast<dvec2*>(pnew + i + cB));
        }
        __syncthreads();
        const int mid = up ? gr + 1 : gr - 1;
        if (j >= 2 && mid >= r0 && mid < rend) {
          const double* sm = s_ring + ((j - 1) & 3) * SL + 1;
          const double* su = s_ring + ((j - 2) & 3) * SL + 1;
          const double* sn = sl;
          dvec2 qa, qb;
          qa.x = sm[2 * t] * 4.0 - sm[2 * t - 1] - sm[2 * t + 1] - su[2 * t] - sn[2 * t];
          qa.y = sm[2 * t + 1] * 4.0 - sm[2 * t] - sm[2 * t + 2] - su[2 * t + 1] - sn[2 * t + 1];
          const int b = 2 * t + W / 2;
          qb.x = sm[b] * 4.0 - sm[b - 1] - sm[b + 1] - su[b] - sn[b];
          qb.y = sm[b + 1] * 4.0 - sm[b] - sm[b + 2] - su[b + 1] - sn[b + 1];
          const long long i = (long long)mid * m;
          __builtin_nontemporal_store(qa, reinterpret_cast<dvec2*>(q + i + cA));
          __builtin_nontemporal_store(qb, reinterpret_cast<dvec2*>(q + i + cB));
        }
      }
    }
  }
}

struct V {
  const char* name;
  void (*k)(Bufs);
  double bytes_per_pair;
};

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 20;
  const long long rows = 4094ll * 4096, n = rows / 2;
  const long long nalloc = 4094ll * 4160 / 2;  // room for a padded row pitch
  Bufs B;
  CHK(hipMalloc(&B.a, nalloc * 16));
  CHK(hipMalloc(&B.b, nalloc * 16));
  CHK(hipMalloc(&B.c, nalloc * 16));
  CHK(hipMalloc(&B.d, nalloc * 16));
  unsigned* code;
  CHK(hipMalloc(&code, nalloc * 4));
  B.code = code;
  B.n = n;
  CHK(hipMemset(B.a, 0, nalloc * 16));
  CHK(hipMemset(B.b, 0, nalloc * 16));
  CHK(hipMemset(B.d, 0, nalloc * 16));
  CHK(hipMemset(code, 0, nalloc * 4));
  std::vector<V> vs = {
      {"ps   r2+code w2", k_mix<2, 2, true, false, false, 4>, 68},
      {"ps   r2+code w2 nt", k_mix<2, 2, true, false, true, 4>, 68},
      {"ps   r2+code w2 u2", k_mix<2, 2, true, false, false, 2>, 68},
      {"b    r2+code w1 inpl", k_mix<2, 1, true, true, false, 4>, 52},
      {"b    r2+code w1 inpl nt", k_mix<2, 1, true, true, true, 4>, 52},
      {"r2w2", k_mix<2, 2, false, false, false, 4>, 64},
      {"r2w1", k_mix<2, 1, false, false, false, 4>, 48},
      {"r3w0", k_mix<3, 0, false, false, false, 4>, 48},
      {"r1w1 copy", k_mix<1, 1, false, false, false, 4>, 32},
      {"r1w1 copy nt", k_mix<1, 1, false, false, true, 4>, 32},
  };
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  for (int g : {8192}) {
    for (auto& v : vs) v.k<<<g, 256>>>(B);
    CHK(hipDeviceSynchronize());
    for (auto& v : vs) {
      double best = 1e30;
      for (int round = 0; round < 3; ++round) {
        CHK(hipEventRecord(e0));
        for (int r = 0; r < reps; ++r) v.k<<<g, 256>>>(B);
        CHK(hipEventRecord(e1));
        CHK(hipEventSynchronize(e1));
        float t;
        CHK(hipEventElapsedTime(&t, e0, e1));
        best = std::min(best, (double)t / reps);
      }
      printf("g%-6d %-26s %8.4f ms %7.1f GB/s\n", g, v.name, best,
             v.bytes_per_pair * n / (best * 1e-3) / 1e9);
    }
  }
  // march-shaped stream in the CG sequence with the b-like stream:
  // strip width 128 * PPL columns, row pitch 4096 (or padded)
  {
    const int m = 4096, nrows = 4094;
    const unsigned short* code16 = reinterpret_cast<const unsigned short*>(code);
    struct MV {
      const char* name;
      void (*k)(const double*, const double*, const unsigned short*, double*, double*, int, int,
                long long, int, int);
      int ppl, pitch;
      long long spitch;
      int H;
    };
    const long long sm = (long long)nrows * 128;  // strip-major strip stride (PPL 1)
    std::vector<MV> mvs = {
        {"rowmaj D2 H32", k_march_stream<2, 1, false>, 1, 4096, 128, 32},
        {"rowmaj D2 H32 halo", k_march_stream<2, 1, true>, 1, 4096, 128, 32},
        {"rowmaj D3 H32 halo", k_march_stream<3, 1, true>, 1, 4096, 128, 32},
        {"rowmaj D4 H32 halo", k_march_stream<4, 1, true>, 1, 4096, 128, 32},
        {"stripmaj D2 H32", k_march_stream<2, 1, false>, 1, 128, sm, 32},
        {"stripmaj D2 H32 halo", k_march_stream<2, 1, true>, 1, 128, sm, 32},
        {"stripmaj D3 H32 halo", k_march_stream<3, 1, true>, 1, 128, sm, 32},
        {"stripmaj D4 H32 halo", k_march_stream<4, 1, true>, 1, 128, sm, 32},
        {"stripmaj D2 H64 halo", k_march_stream<2, 1, true>, 1, 128, sm, 64},
        {"stripmaj D4 H64 halo", k_march_stream<4, 1, true>, 1, 128, sm, 64},
        {"rowmaj ppl2 D2 H16 halo", k_march_stream<2, 2, true>, 2, 4096, 256, 16},
        {"stripmaj ppl2 D2 H16 halo", k_march_stream<2, 2, true>, 2, 256, 2 * sm, 16}};
    for (auto& mv : mvs) {
      const int waves = (m / (128 * mv.ppl)) * ((nrows + mv.H - 1) / mv.H), grid = (waves + 3) / 4;
      std::vector<hipEvent_t> ev(3);
      for (auto& e : ev) CHK(hipEventCreate(&e));
      double tps = 0, tb = 0;
      for (int k = 0; k < 2 * reps + 4; ++k) {
        const double* po = (const double*)((k & 1) ? B.c : B.a);
        double* pn = (double*)((k & 1) ? B.a : B.c);
        CHK(hipEventRecord(ev[0]));
        mv.k<<<grid, 256>>>(po, (const double*)B.b, code16, pn, (double*)B.d, m, mv.pitch,
                             mv.spitch, nrows, mv.H);
        CHK(hipEventRecord(ev[1]));
        k_b_seq<true, false><<<8192, 256>>>(B.d, B.b, code, n);
        CHK(hipEventRecord(ev[2]));
        CHK(hipEventSynchronize(ev[2]));
        float a1, a2;
        CHK(hipEventElapsedTime(&a1, ev[0], ev[1]));
        CHK(hipEventElapsedTime(&a2, ev[1], ev[2]));
        if (k >= 4) {
          tps += a1;
          tb += a2;
        }
      }
      printf("march-stream %-20s in sequence: march %.4f ms  b-like %.4f ms\n", mv.name,
             tps / (2 * reps), tb / (2 * reps));
    }
  }
  {
    const int m = 4096, nrows = 4094;
    const unsigned short* code16 = reinterpret_cast<const unsigned short*>(code);
    struct RV {
      const char* name;
      void (*k)(const double*, const double*, const unsigned short*, double*, double*, int, int,
                int);
      int W, H;
    };
    std::vector<RV> rvs = {{"rowmarch W4096 D2 H16", k_rowmarch<2, 4096, false>, 4096, 16},
                           {"rowmarch W4096 D2 H16 alt", k_rowmarch<2, 4096, true>, 4096, 16},
                           {"rowmarch W4096 D3 H16 alt", k_rowmarch<3, 4096, true>, 4096, 16},
                           {"rowmarch W2048 D2 H16 alt", k_rowmarch<2, 2048, true>, 2048, 16},
                           {"rowmarch W2048 D3 H16 alt", k_rowmarch<3, 2048, true>, 2048, 16},
                           {"rowmarch W2048 D2 H32 alt", k_rowmarch<2, 2048, true>, 2048, 32},
                           {"rowmarch W1024 D3 H16 alt", k_rowmarch<3, 1024, true>, 1024, 16},
                           {"rowmarch W1024 D3 H32 alt", k_rowmarch<3, 1024, true>, 1024, 32}};
    for (auto& rv : rvs) {
      const int grid = (m / rv.W) * ((nrows + rv.H - 1) / rv.H);
      const size_t lds = 4 * (rv.W + 2) * sizeof(double);
      CHK(hipFuncSetAttribute((const void*)rv.k, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lds));
      std::vector<hipEvent_t> ev(3);
      for (auto& e : ev) CHK(hipEventCreate(&e));
      double tps = 0, tb = 0;
      for (int k = 0; k < 2 * reps + 4; ++k) {
        const double* po = (const double*)((k & 1) ? B.c : B.a);
        double* pn = (double*)((k & 1) ? B.a : B.c);
        CHK(hipEventRecord(ev[0]));
        rv.k<<<grid, rv.W / 4, lds>>>(po, (const double*)B.b, code16, pn, (double*)B.d, m, nrows,
                                      rv.H);
        CHK(hipEventRecord(ev[1]));
        k_b_seq<true, false><<<8192, 256>>>(B.d, B.b, code, n);
        CHK(hipEventRecord(ev[2]));
        CHK(hipEventSynchronize(ev[2]));
        float a1, a2;
        CHK(hipEventElapsedTime(&a1, ev[0], ev[1]));
        CHK(hipEventElapsedTime(&a2, ev[1], ev[2]));
        if (k >= 4) {
          tps += a1;
          tb += a2;
        }
      }
      CHK(hipGetLastError());
      printf("%-28s grid %5d in sequence: march %.4f ms  b-like %.4f ms\n", rv.name, grid,
             tps / (2 * reps), tb / (2 * reps));
    }
  }
  // real sequence: PS(p0 -> p1), B, PS(p1 -> p0), B ...
  for (int mode = 0; mode < 4; ++mode) {
    const bool nt = mode & 1, rev = mode & 2;
    const int g = 8192;
    auto iter = [&](int k) {
      dvec2* po = (k & 1) ? B.c : B.a;
      dvec2* pn = (k & 1) ? B.a : B.c;
      if (nt) k_ps_seq<true><<<g, 256>>>(po, B.b, code, pn, B.d, n);
      else k_ps_seq<false><<<g, 256>>>(po, B.b, code, pn, B.d, n);
      if (nt && rev) k_b_seq<true, true><<<g, 256>>>(B.d, B.b, code, n);
      else if (nt) k_b_seq<true, false><<<g, 256>>>(B.d, B.b, code, n);
      else if (rev) k_b_seq<false, true><<<g, 256>>>(B.d, B.b, code, n);
      else k_b_seq<false, false><<<g, 256>>>(B.d, B.b, code, n);
    };
    for (int k = 0; k < 4; ++k) iter(k);
    CHK(hipDeviceSynchronize());
    // per-kernel split (events between the launches)
    {
      std::vector<hipEvent_t> ev(3);
      for (auto& e : ev) CHK(hipEventCreate(&e));
      double tps = 0, tb = 0;
      for (int k = 0; k < 2 * reps; ++k) {
        dvec2* po = (k & 1) ? B.c : B.a;
        dvec2* pn = (k & 1) ? B.a : B.c;
        CHK(hipEventRecord(ev[0]));
        if (nt) k_ps_seq<true><<<g, 256>>>(po, B.b, code, pn, B.d, n);
        else k_ps_seq<false><<<g, 256>>>(po, B.b, code, pn, B.d, n);
        CHK(hipEventRecord(ev[1]));
        if (nt) k_b_seq<true, false><<<g, 256>>>(B.d, B.b, code, n);
        else k_b_seq<false, false><<<g, 256>>>(B.d, B.b, code, n);
        CHK(hipEventRecord(ev[2]));
        CHK(hipEventSynchronize(ev[2]));
        float a1, a2;
        CHK(hipEventElapsedTime(&a1, ev[0], ev[1]));
        CHK(hipEventElapsedTime(&a2, ev[1], ev[2]));
        tps += a1;
        tb += a2;
      }
      printf("cg-iter split nt=%d: ps-like %.4f ms  b-like %.4f ms\n", nt, tps / (2 * reps),
             tb / (2 * reps));
    }
    double best = 1e30;
    for (int round = 0; round < 3; ++round) {
      CHK(hipEventRecord(e0));
      for (int k = 0; k < 2 * reps; ++k) iter(k);
      CHK(hipEventRecord(e1));
      CHK(hipEventSynchronize(e1));
      float t;
      CHK(hipEventElapsedTime(&t, e0, e1));
      best = std::min(best, (double)t / (2 * reps));
    }
    printf("cg-iter seq nt=%d b_reverse=%d: %8.4f ms / iteration  %7.1f GB/s (60 B/row)\n", nt,
           rev, best, 60.0 * rows / (best * 1e-3) / 1e9);
  }
  return 0;
}
