// perc_nr.cpp -- Numerical-Recipes-compatible F77 entry points.
//
// Drop-in replacements for the routines embedded in every reference
// conductance program (Fortran/Square/bondc.f:723-917): same symbol names
// (F77 ABI, trailing underscore, arguments by reference), same argument
// meaning, same NR row-indexed storage (sa(1..n) diagonal, ija(1) = n+2,
// ija(i+1) = end+1 of row i, off-diagonals in ascending column order).
// linbcg_ and dsprsax_/dsprstx_ run on the GPU (device 0); the matrix is read
// from COMMON /mat/ sa(NMAX), ija(NMAX) (symbol mat_, NMAX = 20000 as in the
// reference, bondc.f:753) unless perc_nr_bind() supplies other storage.
// Where the reference `pause`s, the status is kept for perc_nr_status().
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <vector>

#include "perc_internal.h"

using namespace perc;

namespace {

constexpr int kNmaxDefault = 20000;  // bondc.f:753

struct MatCommon {
  double sa[kNmaxDefault];
  int ija[kNmaxDefault];
};

std::mutex g_nr_mu;
double* g_sa = nullptr;
int* g_ija = nullptr;
int g_nmax = kNmaxDefault;
int g_status = PERC_OK;
perc_ctx* g_nr = nullptr;  // matrix-only device context
int g_nr_dot = PERC_DOT_LITERAL;  // perc_nr_set_dot_order

}  // namespace

extern "C" {
// COMMON /mat/ of the calling Fortran program (weak: absent in non-Fortran hosts)
extern MatCommon mat_ __attribute__((weak));
// the calling program's blank COMMON m, n, t, pbc, nn(10), scn (Square/bondc.f:58,
// Triangular/bondc.f; flang and gfortran name it __BLNK__)
struct BlankCommon {
  int m, n, t, pbc, nn[10], scn;
};
extern BlankCommon __BLNK__ __attribute__((weak));
}

namespace {

bool bound(double** sa, int** ija) {
  if (g_sa) {
    *sa = g_sa;
    *ija = g_ija;
    return true;
  }
  if (&mat_ != nullptr) {
    *sa = mat_.sa;
    *ija = mat_.ija;
    return true;
  }
  return false;
}

// NR (1-based, in 0-based arrays) -> 0-based CSR of the off-diagonals
int nr_to_csr(const double* sa, const int* ija, int n, std::vector<int>& rowptr,
              std::vector<int>& col, std::vector<double>& val, std::vector<double>& diag) {
  if (ija[0] != n + 2) return PERC_EMISMATCH;  // bondc.f:891
  const int base = n + 2;
  rowptr.resize(n + 1);
  for (int i = 0; i <= n; ++i) rowptr[i] = ija[i] - base;
  const int nnz = rowptr[n];
  if (nnz < 0) return PERC_EMISMATCH;
  col.resize(nnz);
  val.resize(nnz);
  for (int k = 0; k < nnz; ++k) {
    col[k] = ija[base - 1 + k] - 1;
    val[k] = sa[base - 1 + k];
    if (col[k] < 0 || col[k] >= n) return PERC_EMISMATCH;
  }
  diag.assign(sa, sa + n);
  return PERC_OK;
}

bool is_symmetric(int n, const std::vector<int>& rowptr, const std::vector<int>& col,
                  const std::vector<double>& val) {
  for (int i = 0; i < n; ++i)
    for (int k = rowptr[i]; k < rowptr[i + 1]; ++k) {
      const int j = col[k];
      bool found = false;
      for (int kk = rowptr[j]; kk < rowptr[j + 1]; ++kk)
        if (col[kk] == i) {
          found = val[kk] == val[k];
          break;
        }
      if (!found) return false;
    }
  return true;
}

int upload(int n, const std::vector<int>& rowptr, const std::vector<int>& col,
           const std::vector<double>& val, const std::vector<double>& diag) {
  if (!g_nr) {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
      set_error("no HIP device (the NR routines run on the GPU; there is no CPU fallback)");
      return PERC_ENODEV;
    }
    g_nr = new perc_ctx();
    g_nr->device = 0;
    hipSetDevice(0);
    if (hipStreamCreateWithFlags(&g_nr->stream, hipStreamNonBlocking) != hipSuccess)
      return PERC_EHIP;
    for (int i = 0; i < 8; ++i) hipEventCreate(&g_nr->ev[i]);
  }
  hipSetDevice(g_nr->device);
  if (g_nr->N != n || g_nr->nnz < (long long)col.size()) {
    dev_free_all(g_nr);
    hipError_t e = dev_alloc_matrix(g_nr, n, (long long)col.size());
    if (e != hipSuccess) return hip_status(e, "nr upload");
  }
  g_nr->nnz = (long long)col.size();
  int mr = 0;
  for (int i = 0; i < n; ++i) mr = std::max(mr, rowptr[i + 1] - rowptr[i]);
  g_nr->csr_maxrow = mr;
  g_nr->dot_order = g_nr_dot;
  hipError_t e = hipMemcpy(g_nr->d.rowptr, rowptr.data(), sizeof(int) * (n + 1),
                           hipMemcpyHostToDevice);
  if (e == hipSuccess && !col.empty())
    e = hipMemcpy(g_nr->d.col, col.data(), sizeof(int) * col.size(), hipMemcpyHostToDevice);
  if (e == hipSuccess && !val.empty())
    e = hipMemcpy(g_nr->d.val, val.data(), sizeof(double) * val.size(), hipMemcpyHostToDevice);
  if (e == hipSuccess)
    e = hipMemcpy(g_nr->d.diag, diag.data(), sizeof(double) * n, hipMemcpyHostToDevice);
  return hip_status(e, "nr upload");
}

// The reference `pause`s with a message where these routines fail
// (bondc.f:737, 777, 891, 906); a caller that never reads perc_nr_status()
// still sees the failure on stderr instead of a silent zero result.
void nr_report(const char* who) {
  if (g_status == PERC_OK) return;
  std::fprintf(stderr, "[perc] %s failed (status %d)%s%s\n", who, g_status,
               perc_last_error()[0] ? ": " : "", perc_last_error());
}

}  // namespace

extern "C" {

void perc_nr_bind(double* sa, int* ija, int nmax) {
  std::lock_guard<std::mutex> lk(g_nr_mu);
  g_sa = sa;
  g_ija = ija;
  g_nmax = nmax > 0 ? nmax : kNmaxDefault;
}

int perc_nr_status(void) { return g_status; }
int perc_nr_set_dot_order(int order) {
  if (order != PERC_DOT_FAST && order != PERC_DOT_LITERAL) return PERC_EINVAL;
  std::lock_guard<std::mutex> lk(g_nr_mu);
  g_nr_dot = order;
  return PERC_OK;
}
// the same for F77 callers (implicit interface: integer perc_nr_status)
int perc_nr_status_(void) { return g_status; }

// sprsin: dense (column-major np x np) -> NR row-indexed storage (bondc.f:723-746)
void sprsin_(double* a, int* n_, int* np_, double* thresh_, int* nmax_, double* sa, int* ija) {
  const int n = *n_, np = *np_, nmax = *nmax_;
  const double thresh = *thresh_;
  g_status = PERC_OK;
  for (int j = 1; j <= n; ++j) sa[j - 1] = a[(size_t)(j - 1) * np + (j - 1)];
  ija[0] = n + 2;
  int k = n + 1;
  for (int i = 1; i <= n; ++i) {
    for (int j = 1; j <= n; ++j) {
      const double v = a[(size_t)(j - 1) * np + (i - 1)];
      if (std::fabs(v) >= thresh && i != j) {
        ++k;
        if (k > nmax) {  // 'nmax too small in sprsin'
          g_status = PERC_ENMAX;
          nr_report("sprsin_ (nmax too small)");
          return;
        }
        sa[k - 1] = v;
        ija[k - 1] = j;
      }
    }
    ija[i] = k + 1;
  }
}

static void spmv_nr(double* sa, int* ija, double* x, double* b, int n, bool transpose) {
  std::lock_guard<std::mutex> lk(g_nr_mu);
  std::vector<int> rowptr, col;
  std::vector<double> val, diag;
  g_status = nr_to_csr(sa, ija, n, rowptr, col, val, diag);
  if (g_status) return;
  if (transpose && !is_symmetric(n, rowptr, col, val)) {
    // build the explicit transpose (host re-indexing only; product on device)
    std::vector<int> cnt(n + 1, 0), rp(n + 1, 0), cc(col.size());
    std::vector<double> vv(col.size());
    for (int c : col) cnt[c + 1]++;
    for (int i = 0; i < n; ++i) rp[i + 1] = rp[i] + cnt[i + 1];
    std::vector<int> fill(rp.begin(), rp.end() - 1);
    for (int i = 0; i < n; ++i)
      for (int k = rowptr[i]; k < rowptr[i + 1]; ++k) {
        const int j = col[k], at = fill[j]++;
        cc[at] = i;
        vv[at] = val[k];
      }
    rowptr.swap(rp);
    col.swap(cc);
    val.swap(vv);
  }
  g_status = upload(n, rowptr, col, val, diag);
  if (g_status) return;
  g_nr->assembled = true;
  g_status = hip_status(dev_spmv(g_nr, x, b), "dsprsax_");
}
static void spmv_nr_checked(double* sa, int* ija, double* x, double* b, int n, bool transpose) {
  spmv_nr(sa, ija, x, b, n, transpose);
  nr_report(transpose ? "dsprstx_" : "dsprsax_");
}

// b = A x (bondc.f:887-899)
void dsprsax_(double* sa, int* ija, double* x, double* b, int* n) {
  spmv_nr_checked(sa, ija, x, b, *n, false);
}
// b = A' x (bondc.f:902-917)
void dsprstx_(double* sa, int* ija, double* x, double* b, int* n) {
  spmv_nr_checked(sa, ija, x, b, *n, true);
}

void atimes_(int* n, double* x, double* r, int* itrnsp) {  // bondc.f:841-852
  double* sa;
  int* ija;
  if (!bound(&sa, &ija)) {
    g_status = PERC_ESTATE;
    return;
  }
  spmv_nr_checked(sa, ija, x, r, *n, *itrnsp != 0);
}

void asolve_(int* n, double* b, double* x, int* itrnsp) {  // bondc.f:855-864
  (void)itrnsp;
  double* sa;
  int* ija;
  if (!bound(&sa, &ija)) {
    g_status = PERC_ESTATE;
    return;
  }
  for (int i = 0; i < *n; ++i) x[i] = b[i] / sa[i];
}

double snrm_(int* n, double* sx, int* itol) {  // bondc.f:867-884
  if (*itol <= 3) {
    double s = 0.0;
    for (int i = 0; i < *n; ++i) s = s + sx[i] * sx[i];
    return std::sqrt(s);
  }
  int im = 0;
  for (int i = 1; i < *n; ++i)
    if (std::fabs(sx[i]) > std::fabs(sx[im])) im = i;
  return std::fabs(sx[im]);
}

// linbcg (bondc.f:750-838) on the device: the reference's BiCG with the
// Jacobi preconditioner reduces to PCG for the symmetric conductance matrix;
// rr/pp/zz and dsprstx are then bitwise equal to r/p/z and dsprsax.
static void linbcg_impl(int* n_, double* b, double* x, int* itol, double* tol, int* itmax,
                        int* iter, double* err);
void linbcg_(int* n_, double* b, double* x, int* itol, double* tol, int* itmax, int* iter,
             double* err) {
  linbcg_impl(n_, b, x, itol, tol, itmax, iter, err);
  nr_report("linbcg_");
}
static void linbcg_impl(int* n_, double* b, double* x, int* itol, double* tol, int* itmax,
                        int* iter, double* err) {
  std::lock_guard<std::mutex> lk(g_nr_mu);
  const int n = *n_;
  *iter = 0;
  double* sa;
  int* ija;
  if (!bound(&sa, &ija)) {
    g_status = PERC_ESTATE;
    return;
  }
  if (*itol < 1 || *itol > 4) {  // 'illegal itol in linbcg'
    g_status = PERC_EITOL;
    return;
  }
  std::vector<int> rowptr, col;
  std::vector<double> val, diag;
  g_status = nr_to_csr(sa, ija, n, rowptr, col, val, diag);
  if (g_status) return;
  if (!is_symmetric(n, rowptr, col, val)) {
    set_error("linbcg_: non-symmetric matrix; device path implements the symmetric case");
    g_status = PERC_EINVAL;
    return;
  }
  g_status = upload(n, rowptr, col, val, diag);
  if (g_status) return;
  hipError_t e = hipMemcpy(g_nr->d.rhs, b, sizeof(double) * n, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(g_nr->d.x, x, sizeof(double) * n, hipMemcpyHostToDevice);
  int it = 0;
  double er = 0.0;
  bool x0_zero = true;
  for (int i = 0; i < n && x0_zero; ++i) x0_zero = x[i] == 0.0 && !std::signbit(x[i]);
  if (e == hipSuccess) e = dev_solve(g_nr, *itol, *tol, *itmax, x0_zero, true, &it, &er);
  if (e == hipSuccess) e = hipMemcpy(x, g_nr->d.x, sizeof(double) * n, hipMemcpyDeviceToHost);
  g_status = hip_status(e, "linbcg_");
  *iter = it;
  *err = er;
  if (std::getenv("PERC_NR_VERBOSE") && g_nr->d.err_hist) {
    std::vector<double> h(it);
    hipMemcpy(h.data(), g_nr->d.err_hist, sizeof(double) * it, hipMemcpyDeviceToHost);
    for (int k = 0; k < it; ++k) std::printf("  iter= %d  err= %.17g\n", k + 1, h[k]);
  }
}

}  // extern "C"

extern "C" {
// call nearestn(rn) (Square/bondc.f:617-715, Triangular/bondc.f:619-804): the
// neighbours of site rn into the caller's blank COMMON nn(1..scn), zeros
// where a neighbour is missing, from its m, n, pbc and scn (4: square, 6:
// triangular).  Sets perc_nr_status to PERC_ESTATE without a blank COMMON.
void nearestn_(const int* rn) {
  if (&__BLNK__ == nullptr || (__BLNK__.scn != 4 && __BLNK__.scn != 6)) {
    g_status = PERC_ESTATE;
    return;
  }
  BlankCommon& c = __BLNK__;
  const perc::Geom g = perc::make_geom(c.scn == 4 ? perc::kSquare : perc::kTriangular, c.m, c.n, c.pbc);
  int nn[6] = {0, 0, 0, 0, 0, 0};
  if (*rn >= 1 && *rn <= g.t) perc::nearestn(g, *rn, nn);
  for (int z = 0; z < c.scn; ++z) c.nn[z] = nn[z];
  g_status = PERC_OK;
}
}  // extern "C"
