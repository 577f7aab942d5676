// perc_internal.h -- libperc internals shared by the host and device units.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

#include "../../include/perc.h"
#include "lattice.h"

namespace perc {

constexpr int kBlock = 256;       // threads per workgroup (4 wave64)
constexpr int kRowsPerTile = 256; // CSR rows staged per LDS tile
constexpr int kMaxSpanList = 64;  // spanning roots recorded per labeling
constexpr int kMaxForms = 8;      // stencil row forms per lattice
constexpr int kMaxSlots = 6;      // neighbour slots per row

// Sorted neighbour offsets (c - s) of each row form of the stencil operator
// (interior / edge columns, up / down triangles): row i's columns are
// i + off[f][j] for its form f (perc_stencil.h).
// dr/dc: the slot's neighbour in lattice (row, column) steps, column
// wrapped for pbc; always in {-1, 0, 1} (the LDS-tiled kernel's halo).
struct StencilForms {
  int nforms;
  int cnt[kMaxForms];
  int off[kMaxForms][kMaxSlots];
  int dr[kMaxForms][kMaxSlots];
  int dc[kMaxForms][kMaxSlots];
  // register-march kernel: slot j's raster position in the 3x3 block
  // around the row (0..7 row-major, centre skipped) as 3-bit fields of
  // rpos; rmask has a bit per used position; regular: slot order is
  // raster order (every non-wrapped form)
  unsigned rpos[kMaxForms];
  unsigned rmask[kMaxForms];
  int regular[kMaxForms];
  // inverse of rpos for regular forms: 4-bit field kp = slot index of
  // raster position kp, 0xF where the form has no neighbour there;
  // kRmapIrregular for forms whose slot order is not raster order
  unsigned rmap[kMaxForms];
  unsigned umask;  // union of rmask over the regular forms
};
constexpr unsigned kRmapIrregular = 0xEEEEEEEEu;

// Device-resident CG scalars (one cache line each group; written only by the
// last-arriving workgroup of a kernel, read by the next kernel).
struct CGScalars {
  double bknum;  // z.r for the coming iteration (linbcg bknum)
  double bkden;  // previous bknum
  double akden;  // q.p of the current iteration
  double ak;     // bknum / akden
  double bnrm;   // ||D^-1 b|| (itol 2) or ||b|| (itol 1)
  double err;    // last err
  double tol;
  double bk;     // bknum / bkden for the coming p update (linbcg :799)
  int iter;      // completed iterations
  int itmax;
  int done;      // set once err <= tol or iter > itmax
  int pad[3];
  double part[4];  // row slabs: this slab's raw partials (q.p, z.r, r.r, ||D^-1 b||^2)
  // deferred march reductions (CGArgs::mdef): bkn[j & 1] = bknum of
  // iteration j (j >= 1; iteration 0's is bknum above), parity-buffered so
  // a launch reads the previous value while its writer stores the new one
  double bkn[2];
  // ak of the previous iteration (the march P's collector keeps it when it
  // forms the new ak): B(k + 1) applies x += ak(k) p(k) at its start (CGArgs::mxin)
  double akprev;
};

struct AsmParams {
  bool valid = false;
  int rule = 0, span_root = 0;
  double g0 = 0.0, leak = 0.0, Va = 0.0;
};

struct DeviceBuffers {
  // lattice (1-based sites): bonds whose smaller end is s are
  // [bond_first[s], bond_first[s+1]) in bond-list order
  int* bond_first = nullptr;  // t+2
  // interior CSR, 0-based: off-diagonals only, ascending column
  int* rowptr = nullptr;  // N+1
  int* col = nullptr;     // nnz (+pad)
  double* val = nullptr;  // nnz (+pad)
  double* diag = nullptr; // N
  double* rhs = nullptr;  // N
  // stencil-coded operator: code[i] = slot bits (bit j: sorted neighbour
  // slot j carries -g0, else -leak) | count << 8 | form << 11; sflag[0] != 0
  // if some slot has no bond (1) or a row matches no form (2)
  uint16_t* code = nullptr;  // N (+pad)
  uint16_t* code_sm = nullptr;  // strip-major copy of code (PERC_MARCH_STRIPS solves)
  uint8_t* nib_sm = nullptr;    // strip-major nibble codes (PERC_MARCH_NIBBLE, square lattice)
  double* ez = nullptr;         // strip-major march: edge-column z per strip side and row (CGArgs::ez)
  double2* dtab = nullptr;    // 512: the diagonal of every code (see diag_idx)
  int* sflag = nullptr;      // 4
  // occupancy
  uint8_t* bocc = nullptr;  // nb
  uint8_t* socc = nullptr;  // t+1
  int* order = nullptr;     // upload buffer (max(nb,t)+1)
  // labeling
  int* parent = nullptr;     // t+1
  uint8_t* member = nullptr; // t+1 (site belongs to some cluster)
  uint8_t* top = nullptr;    // t+1 (spanning-root flags, m+1 used)
  int* counters = nullptr;   // [0]=nspan [1]=nclusters [2]=span_sites [3]=max size, then list
  int* csize = nullptr;      // t+2 per-root cluster sizes (perc_cluster_sizes)
  int4* ell_col = nullptr;     // N: the CSR rows in 4 aligned slots (rows of <= 4 off-diagonals)
  double2* ell_val = nullptr;  // 2N
  uint8_t* ell_cnt = nullptr;  // N
  int* ccpart = nullptr;     // the wave tiles' member roots per block, then minus the merge's hooks per workgroup
  StencilForms* forms_dev = nullptr;  // device copy of perc_ctx::forms (k_assemble)
  unsigned* sel_hist = nullptr;  // perc_occupy_random's select, per draw: [0] keys below, [1] in window, [2] window valid, [4 ..] bins
  unsigned long long* sel_cand = nullptr;  // [0] the threshold key, then the window's keys
  // CG
  double* x = nullptr;
  double* r = nullptr;
  double* p0 = nullptr;
  double* p1 = nullptr;
  double* q = nullptr;
  double* partials = nullptr;   // 4 * grid
  unsigned* tickets = nullptr;  // 8
  CGScalars* scal = nullptr;
  double* mgran = nullptr;      // march tagged-granule reductions
  size_t mgran_n = 0;
  double* err_hist = nullptr;   // itmax+2
  int err_hist_cap = 0;
  double* iout = nullptr;       // 2m (boundary-row currents)
  double* bw = nullptr;         // per-bond conductance multipliers (ConductCalc condtype 2)
  double* res_xch = nullptr;    // resident solve: exchange rows
  unsigned* res_bar = nullptr;
  double* res_gran = nullptr;   // resident solve: tagged partial granules
  unsigned* res_reg = nullptr;  // resident solve: XCD registration counters
  double* res_xg = nullptr;     // resident solve: XCD-grouped reduction granules
  double* lit = nullptr;        // literal dot order: the q.p, z.r, r.r terms (3 N) of the
                                // q-free march and the resident solve
};

struct ReplayOrder {
  int kind = PERC_BOND;
  std::vector<int> sites;  // occupied prefix of the site order (ids, 0 = sentinel)
  std::vector<int> bonds;  // occupied prefix of the bond order (1-based ids)
  // device-resident source (perc_occupy_device): copied to the host vectors
  // only if a host replay needs them
  const int* d_sites = nullptr;
  const int* d_bonds = nullptr;
  int n_sites = 0, n_bonds = 0;
  bool host_valid = true;
  // perc_occupy_random: no order array; the host order (ascending keys) is
  // generated only if a replay needs it
  bool random = false;
  unsigned long long seed = 0;
};

struct KernelTiming {
  bool enabled = false;
  std::vector<hipEvent_t> ev;  // 6 per iteration slot of a launch chunk
  double spmv_ms = 0.0, update_ms = 0.0, p_ms = 0.0;
  long long spmv_n = 0, update_n = 0, p_n = 0;
};

}  // namespace perc

namespace perc {
struct DSlab;
}

struct perc_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  // pinned host words for the labeling's read-back (a copy into pageable
  // memory is staged by the runtime)
  int* pin = nullptr;
  perc::Geom g{};
  long long nb = 0;
  int N = 0;       // interior rows t-2m
  long long nnz = 0;
  int csr_maxrow = 6;  // most off-diagonals in one CSR row (lattices: <= 6; NR matrices: measured)
  int grid = 0;    // fixed grid of the CG kernels (reduction order depends on it)
  perc::DeviceBuffers d;
  std::vector<int> h_bond_first;  // host copy, t+2
  perc::ReplayOrder last;          // last occupancy (for the host replay)
  bool occupied = false;
  bool labeled = false;
  bool assembled = false;
  bool bf_closed = false;  // h_bond_first == bf_square on rows 0..n-2 (square lattice)
  bool bf_open_sq = false; // and the open lattice's top row follows (bf_open_square)
  bool flat = true;        // parent[] holds final roots (dev_flatten after a labeling)
  // perc_label's spanning-cluster site count formed on the device in the
  // labeling's own launch sequence (k_cc_compress_spec) when the previous
  // labeling spanned: span_count >= 0 -- that count for the first spanning
  // root, read back with the spanning roots (one host synchronisation)
  bool span_guess = false;
  int span_count = -1;
  bool csr_ok = true;    // the CSR values / diagonal of the assembled system are written
  bool ell_ok = false;   // ... and their ELL copy (d.ell_*)
  perc::AsmParams asm_p; // the assembly's parameters (ensure_csr re-runs it)
  int span_root = 0;
  int perccln = 0;
  int rule = -1;
  int fmt_req = PERC_FMT_AUTO;  // perc_set_matrix_format
  bool stencil_ok = false;      // every stencil slot of the assembled system has a bond
  bool stencil = false;         // solver kernels use the stencil operator
  bool tiled_ok = false;        // every row's slots are (row, col) +-1 steps of its form
  bool fused = false;           // stencil P+S fused into the LDS-tiled kernel
  int tile_grid = 0;            // workgroups of the tiled kernel
  int tile_h = 32;              // its tile height (rows)
  bool march_ok = false;        // register-march kernel usable (m % 128 == 0, tileable)
  bool march = false;           // fused format runs the register-march kernel
  int march_h = 32;             // its band height (rows per wave)
  int march_slots = 0;          // q-free strip-major march: slot-weighted bands
  int march_tag = 0;            // q-free strip-major march: tagged-granule reductions
  unsigned solve_epoch = 0;     // tags of the granule reductions
  int wm_slots = 0;             // slot-weighted bands: workgroup rounds (0: not available)
  int wm_grid = 0;              // their grid (CUs x rounds)
  int wm_cum[3][5] = {};        // cumulative round weights (P, B, row-major P)
  bool slot_w_set = false;      // perc_set_band_weights: weights instead of the defaults
  int slot_w[3][4] = {};        // per round (P, B, row-major P)
  int dot_order = PERC_DOT_FAST;  // perc_set_dot_order
  bool nib_ok = false;          // square-lattice column classes known (nibble codes)
  bool nib_used = false;        // the last strip-major solve ran the nibble codes
  unsigned ncls[3] = {};        // their count / form bits: interior, first, last column
  int march_grid = 0;           // its workgroups
  int march_grid_max = 0;       // workgroups at band height 1 (reduction buffers)
  int row_grid = 0;             // one CSR row per thread: cdiv(N, kBlock) (k_cg_spmv_row)
  int march_rows_req = 0;       // perc_set_march_rows (0: auto)
  int march_mode = PERC_MARCH_DEFAULT;  // perc_set_march_mode
  bool qfree = false;           // march B rebuilds q (52N / iteration)
  bool march_alt = false;       // alternating walk directions
  bool strips = false;          // march solve in the strip-major layout
  int b_grid = 0;               // streaming B workgroups in the fused formats (dev_build_lattice)
  bool has_weights = false;     // perc_set_bond_weights: G = -g0 w for the spanning bonds
  bool resident = false;        // persistent resident solve (k_cg_res)
  bool small = false;           // one-workgroup solve of a small system (k_cg_small)
  int res_G = 0, res_H = 0, res_MT = 0, res_HMAX = 0;  // its grid, band height, template
  int res_NT = 1024;            // its threads per workgroup (m rounded up to 64 for m < 1024)
  bool res_uneven = false;      // a grouped resident launch found the XCD placement uneven
  // what the last dev_solve ran (perc_last_solve): kernel family (PERC_RAN_*)
  // and flags (PERC_RAN_* bits: q-free, strip-major, nibble codes, tagged
  // reductions, literal folds of kernel-stored terms)
  int last_kernel = 0, last_flags = 0, last_iter = -1;
  bool full_voltages = false;   // perc_set_full_voltages: keep x on every row
  int nslab = 1;                // perc_set_slabs: row slabs of the CG solve
  perc::DSlab* dslab = nullptr;  // perc_dslab_*: this process's slab of a distributed solve
  double st_ng0 = 0.0, st_nleak = 0.0;  // its two off-diagonal values
  perc::StencilForms forms{};            // row forms of this lattice
  hipEvent_t ev[8];
  hipEvent_t ev_next[2] = {nullptr, nullptr};  // klaunch: start/stop of the next CG launch
  perc::KernelTiming timing;
};

namespace perc {

// device entry points (perc_label.hip, perc_assemble.hip, perc_solve.hip, perc_slabs.hip)
hipError_t dev_build_lattice(perc_ctx* h);
hipError_t dev_alloc_matrix(perc_ctx* h, int N, long long nnz);
void dev_free_all(perc_ctx* h);
hipError_t dev_occupy(perc_ctx* h, int kind, int nsites, const int* site_order, int nbonds,
                      const int* bond_order, bool device_src);
hipError_t dev_label(perc_ctx* h, int* nspan, int* span_list, int* nclusters, bool spec_span = false);
hipError_t dev_occupy_random(perc_ctx* h, int kind, int nsites, int nbonds, unsigned long long seed);
hipError_t dev_span_sites(perc_ctx* h, int root, int* count);
hipError_t dev_flatten(perc_ctx* h);  // parent[s] = final root (k_cc_compress) once per labeling
hipError_t dev_canon(perc_ctx* h, int* canon_out);
hipError_t dev_cluster_sizes(perc_ctx* h, int kind, int root, int* maxcs, int* rootsize);
hipError_t dev_assemble(perc_ctx* h, int rule, double g0, double leak, double Va, int span_root);
hipError_t ensure_csr(perc_ctx* h);  // the CSR copy of the assembled system, on demand
void select_format(perc_ctx* h);  // stencil / fused flags from fmt_req + assembly checks
void march_geometry(perc_ctx* h); // band height + grid of the register-march kernel
void res_geometry(perc_ctx* h);   // grid + band height of the resident solve
// force_exchange: run the combines and publishes even at K = 1 (measures
// the exchange machinery; K = 1 otherwise takes the one-slab epilogues)
hipError_t dev_dslab_begin(perc_ctx* h, int K, int s, int itol, double tol, int itmax, bool full_x,
                           const perc_dslab_bufs& bufs, bool force_exchange = false);
hipError_t dev_dslab_step(perc_ctx* h, int op);
// perc_dslab_comm_init's communicator of the context, if any (perc_dslab.cpp)
void dslab_comm_release(perc_ctx* h);
hipError_t dev_dslab_status(perc_ctx* h, int* iter, double* err, int* done);
hipError_t dev_dslab_end(perc_ctx* h, bool to_ctx);
hipError_t dev_x_row(perc_ctx* h, int row, double* buf, bool to_ctx);
// row forms of the interior system (perc_assemble.hip); band height of the
// register march over nrows rows (perc_solve.hip)
StencilForms stencil_forms(const Geom& g);
int march_rows_for(const perc_ctx* h, int nrows);
hipError_t dev_solve_slabs(perc_ctx* h, int K, int itol, double tol, int itmax, bool full_x,
                           int* iter, double* err);
hipError_t dev_solve(perc_ctx* h, int itol, double tol, int itmax, bool x0_zero, bool full_x,
                     int* iter, double* err);
hipError_t dev_currents(perc_ctx* h, int rule, int cur_rule, double g0, double leak, double Va,
                        int span_root, double thresh, double* iout_host);
hipError_t dev_spmv(perc_ctx* h, const double* x, double* y);
hipError_t dev_selftest_division(long long n, unsigned long long seed, unsigned long long* out3);
hipError_t dev_set_bond_weights(perc_ctx* h, const double* w);
// 1 per bond the assembly gives -g0 under `rule` (spanning cluster h->span_root)
hipError_t dev_bond_mask(perc_ctx* h, int rule, uint8_t* mask_host);
hipError_t dev_bench(perc_ctx* h, int which, int reps, double* ms);

// host replay (perc_replay.cpp): reference label numbering
// trace (optional, 3 per order entry): bondc.f's per-bond case (0: no
// occupied neighbour bond, 1: joined the largest neighbouring cluster), the
// cluster number the bond got and that cluster's size after the step
int replay_bonds(const Geom& g, const std::vector<int>& bond_first, const int* order,
                 int count, int* label, int* csize, int cap, int* stats, int* trace = nullptr);
// trace (optional, kSiteTrace per order entry): site.f's per-site step
// (siteocc.txt, Square/site.f:167-272): sn, nn(1..6), nnlc, lcn, lcs, the
// number of absorbed clusters k, k pairs (size added, largest cluster's
// size after), the cluster the site joined and that cluster's size after
constexpr int kSiteTrace = 24;
int replay_sites(const Geom& g, const int* order, int count, int* label, int* csize, int cap,
                 int* stats, int* trace = nullptr);
// ev (optional): the debug log's event stream, one record per step of the
// second phase (sbdebug.txt / bsdebug.txt; record layout in include/perc.h,
// perc_replay_mixed_trace)
int replay_bondsite(const Geom& g, const std::vector<int>& bond_first, const int* sorder,
                    int nsites, const int* border, int nbond, int* site_label, int* bond_label,
                    int* csize, int cap, int* stats, std::vector<int>* ev = nullptr);
int replay_sitebond(const Geom& g, const std::vector<int>& bond_first, const int* sorder,
                    int nsites, const int* border, int nbonds, int* site_label,
                    int* bond_label, int* csize, int cap, int* stats,
                    std::vector<int>* ev = nullptr);

int replay_bs_scan(const Geom& g, const std::vector<int>& bond_first, const int* sorder,
                   int nsites, const int* border, int nbond, bool c0_overflow);

void set_error(const std::string& msg);
int hip_status(hipError_t e, const char* where);

}  // namespace perc
