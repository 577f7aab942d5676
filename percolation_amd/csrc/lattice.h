// lattice.h -- lattice topology for libperc, usable on host and gfx950.
//
// Neighbour order is part of the reference's semantics (it fixes label
// tie-breaks, bond-list order and the RHS summation order), so nearestn()
// reproduces Fortran/Square/bondc.f:617-715 and Fortran/Triangular/
// bondc.f:619-804 branch for branch.  Sites are 1-based, row-major from the
// bottom row; nn[k] == 0 means "no neighbour".
#pragma once

#include <hip/hip_runtime.h>

namespace perc {

enum Lattice : int { kSquare = 0, kTriangular = 1 };

struct Geom {
  int lattice;  // kSquare / kTriangular
  int m, n;     // width, height (sites)
  int pbc;      // left/right periodic
  int t;        // m*n
  int scn;      // site coordination number (4 / 6)
  int bcn;      // bond coordination number (6 / 10)
  unsigned long long mrecip;  // ceil(2^64 / m) for m > 1, else 0 (div_m)
};

__host__ __device__ inline Geom make_geom(int lattice, int m, int n, int pbc) {
  Geom g;
  g.lattice = lattice;
  g.m = m;
  g.n = n;
  g.pbc = pbc;
  g.t = m * n;
  g.scn = lattice == kSquare ? 4 : 6;
  g.bcn = lattice == kSquare ? 6 : 10;
  g.mrecip = m > 1 ? ~0ull / (unsigned long long)m + 1ull : 0ull;
  return g;
}

// Square/bondc.f:119-123, Triangular/bondc.f:121-125
__host__ __device__ inline long long nbonds(const Geom& g) {
  long long m = g.m, n = g.n;
  if (g.lattice == kSquare) return g.pbc ? m * (2 * n - 1) : 2 * m * n - m - n;
  return g.pbc ? m * (3 * n - 2) : 3 * m * n - 2 * m - 2 * n + 1;
}

// nearestn of site rn at (row r, column col) = ((rn-1)/m, (rn-1)%m): the
// reference's branches in the reference's order, each test on rn restated on
// (r, col) -- rn == 1 <=> r == 0 && col == 0, rn < m <=> r == 0 && col < m-1,
// rn > t-m <=> r == n-1, (rn-1)%m == 0 <=> col == 0, rn%m == 0 <=> col == m-1,
// and (rn/m)%2 == r%2 where it is asked (interior columns) -- so the device
// kernels divide once per site (div_m) instead of at every modulo.
__host__ __device__ inline void nearestn_square_rc(const Geom& g, int rn, int r, int col, int* nn) {
  const int m = g.m, t = g.t;
  const bool b0 = r == 0, bT = r == g.n - 1, cL = col == 0, cR = col == m - 1;
  nn[0] = nn[1] = nn[2] = nn[3] = 0;
  if (b0 && cL) { nn[0] = rn + 1; nn[1] = rn + m; if (g.pbc) nn[2] = m; return; }
  if (b0 && cR) { nn[0] = rn - 1; nn[1] = rn + m; if (g.pbc) nn[2] = 1; return; }
  if (bT && cL) { nn[0] = rn - m; nn[1] = rn + 1; if (g.pbc) nn[2] = t; return; }
  if (bT && cR) { nn[0] = rn - m; nn[1] = rn - 1; if (g.pbc) nn[2] = rn - (m - 1); return; }
  if (b0) { nn[0] = rn - 1; nn[1] = rn + 1; nn[2] = rn + m; return; }
  if (bT) { nn[0] = rn - m; nn[1] = rn - 1; nn[2] = rn + 1; return; }
  if (cL) {
    nn[0] = rn - m; nn[1] = rn + 1; nn[2] = rn + m;
    if (g.pbc) nn[3] = rn + (m - 1);
    return;
  }
  if (cR) {
    nn[0] = rn - m; nn[1] = rn - 1; nn[2] = rn + m;
    if (g.pbc) nn[3] = rn - (m - 1);
    return;
  }
  nn[0] = rn - m; nn[1] = rn - 1; nn[2] = rn + 1; nn[3] = rn + m;
}

__host__ __device__ inline void nearestn_tri_rc(const Geom& g, int rn, int r, int col, int* nn) {
  const int m = g.m, t = g.t;
  const bool odd_m = (m & 1) == 1, even_rn = (rn & 1) == 0;
  const bool b0 = r == 0, bT = r == g.n - 1, cL = col == 0, cR = col == m - 1;
  for (int z = 0; z < 6; ++z) nn[z] = 0;
  if (b0 && cL) {
    nn[0] = rn + 1; nn[1] = rn + m; nn[2] = rn + (m + 1);
    if (g.pbc) { nn[3] = rn + (m - 1); nn[4] = rn + (2 * m - 1); }
    return;
  }
  if (b0 && cR) {
    nn[0] = rn - 1; nn[1] = rn + m;
    if (odd_m) { nn[2] = rn + (m - 1); return; }
    if (g.pbc) nn[2] = 1;
    return;
  }
  if (bT && cL) {
    nn[0] = rn - m; nn[1] = rn + 1;
    if (g.pbc) nn[2] = t;
    return;
  }
  if (bT && cR) {
    if (odd_m) { nn[0] = rn - m; nn[1] = rn - 1; return; }
    nn[0] = rn - (m + 1); nn[1] = rn - m; nn[2] = rn - 1;
    if (g.pbc) { nn[3] = rn - (2 * m - 1); nn[4] = rn - (m - 1); }
    return;
  }
  if (b0) {  // bottom row
    if (even_rn) {
      nn[0] = rn - 1; nn[1] = rn + 1; nn[2] = rn + m;
    } else {
      nn[0] = rn - 1; nn[1] = rn + 1; nn[2] = rn + (m - 1); nn[3] = rn + m; nn[4] = rn + (m + 1);
    }
    return;
  }
  if (bT) {  // top row
    if (even_rn) {
      nn[0] = rn - (m + 1); nn[1] = rn - m; nn[2] = rn - (m - 1); nn[3] = rn - 1; nn[4] = rn + 1;
    } else {
      nn[0] = rn - m; nn[1] = rn - 1; nn[2] = rn + 1;
    }
    return;
  }
  if (cL) {  // left edge
    nn[0] = rn - m; nn[1] = rn + 1; nn[2] = rn + m; nn[3] = rn + (m + 1);
    if (g.pbc) { nn[4] = rn + (m - 1); nn[5] = rn + (2 * m - 1); }
    return;
  }
  if (cR) {  // right edge
    if (odd_m) {
      nn[0] = rn - m; nn[1] = rn - 1; nn[2] = rn + (m - 1); nn[3] = rn + m;
      return;
    }
    nn[0] = rn - (m + 1); nn[1] = rn - m; nn[2] = rn - 1; nn[3] = rn + m;
    if (g.pbc) { nn[4] = rn - (2 * m - 1); nn[5] = rn - (m - 1); }
    return;
  }
  // "up" form: rn-(m+1), rn-m, rn-(m-1), rn-1, rn+1, rn+m
  const bool up = odd_m ? (((r & 1) == 0) == even_rn) : even_rn;
  if (up) {
    nn[0] = rn - (m + 1); nn[1] = rn - m; nn[2] = rn - (m - 1);
    nn[3] = rn - 1; nn[4] = rn + 1; nn[5] = rn + m;
  } else {
    nn[0] = rn - m; nn[1] = rn - 1; nn[2] = rn + 1;
    nn[3] = rn + (m - 1); nn[4] = rn + m; nn[5] = rn + (m + 1);
  }
}

__host__ __device__ inline void nearestn_rc(const Geom& g, int rn, int r, int col, int* nn) {
  if (g.lattice == kSquare) nearestn_square_rc(g, rn, r, col, nn);
  else nearestn_tri_rc(g, rn, r, col, nn);
}

__host__ __device__ inline void nearestn(const Geom& g, int rn, int* nn) {
  const int r = (rn - 1) / g.m;
  nearestn_rc(g, rn, r, rn - 1 - r * g.m, nn);
}

// Neighbours of rn sorted ascending (the dense-row scan order of G, used for
// the diagonal row sum, Square/bondc.f:499-505, and by sprsin's column scan).
// Returns the count; out[] holds up to 6 sites.
__host__ __device__ inline int sorted_neighbours(const Geom& g, int rn, int* out) {
  int nn[6];
  nearestn(g, rn, nn);
  int c = 0;
  for (int k = 0; k < g.scn; ++k)
    if (nn[k] != 0) {
      int v = nn[k], j = c;
      while (j > 0 && out[j - 1] > v) { out[j] = out[j - 1]; --j; }
      out[j] = v;
      ++c;
    }
  return c;
}

// Neighbour c of site s in lattice steps: row difference and column
// difference, the column wrapped into {-1, 0, 1} for left/right pbc.
__host__ __device__ inline void lattice_delta(const Geom& g, int s, int c, int* dr, int* dc) {
  const int sr = (s - 1) / g.m, sc = (s - 1) % g.m;
  const int cr = (c - 1) / g.m, cc = (c - 1) % g.m;
  int d = cc - sc;
  if (d > 1) d -= g.m;
  else if (d < -1) d += g.m;
  *dr = cr - sr;
  *dc = d;
}

// bond_first of the square lattice's site (row r, column c), r <= n-2: rows
// 0..n-2 each hold 2m-1 (+1 with pbc) forward bonds -- 2 per site, +1 at
// column 0 with pbc (the wrap bond), -1 at column m-1 (no right neighbour).
// Used where perc_ctx::bf_closed says the built bond_first agrees.
__host__ __device__ inline int bf_square(const Geom& g, int r, int c) {
  const int pb = g.pbc ? 1 : 0;
  return r * (2 * g.m - 1 + pb) + 2 * c + (c > 0 ? pb : 0);
}

// Number of bonds whose smaller end is rn (bond list, Square/bondc.f:139-154)
__host__ __device__ inline int forward_count(const Geom& g, int rn) {
  int nn[6], c = 0;
  nearestn(g, rn, nn);
  for (int k = 0; k < g.scn; ++k) c += nn[k] > rn;
  return c;
}

// Random occupation without an order array (perc_occupy_random): element id
// (1-based) gets the key (hash32(seed, id) << 32) | id, unique per id; the
// `count` elements with the smallest keys are occupied, i.e. the first
// `count` of the permutation "ids in ascending key order" -- a uniform
// random permutation up to the order of equal 32-bit hashes (by id).
// Host and device compute the same keys (perc_random_order gives the order).
__host__ __device__ inline unsigned long long perc_mix64(unsigned long long x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
__host__ __device__ inline unsigned long long perc_rand_key(unsigned long long seed, unsigned id) {
  const unsigned long long h = perc_mix64(perc_mix64(seed) ^ (unsigned long long)id);
  return (h & 0xFFFFFFFF00000000ull) | (unsigned long long)id;
}

// perc_rand_key's hash word, hash32(seed, id) = perc_rand_key(seed, id) >> 32,
// in 32-bit arithmetic with the seed folded in once per draw: id only
// touches the low word of S ^ id (S = perc_mix64(seed)), so after the
// golden-ratio add the high word is Shi + Chi + carry -- one of two
// constants, and so are the terms of the first multiply it feeds; the last
// multiply needs only its high word.  5 32-bit multiplies per key instead
// of 6, and no 64-bit shifts (the occupancy draw is bound by this hash).
struct RandKeyCtx {
  unsigned slo;         // low word of S
  unsigned hs0, hs1;    // (high word of S + C + carry) << 2, carry 0 / 1
  unsigned t0, t1;      // (y's high word) * C1lo, carry 0 / 1
};
__host__ __device__ inline RandKeyCtx perc_rand_key_ctx(unsigned long long seed) {
  const unsigned long long S = perc_mix64(seed);
  RandKeyCtx k;
  k.slo = (unsigned)S;
  const unsigned h0 = (unsigned)(S >> 32) + 0x9E3779B9u, h1 = h0 + 1u;
  k.hs0 = h0 << 2;
  k.hs1 = h1 << 2;
  k.t0 = (h0 ^ (h0 >> 30)) * 0x1CE4E5B9u;
  k.t1 = (h1 ^ (h1 >> 30)) * 0x1CE4E5B9u;
  return k;
}
__host__ __device__ inline unsigned perc_rand_hash32(const RandKeyCtx& k, unsigned id) {
  const unsigned x0lo = (k.slo ^ id) + 0x7F4A7C15u;
  const bool c = x0lo < 0x7F4A7C15u;  // carry into the high word
  const unsigned ylo = x0lo ^ ((x0lo >> 30) | (c ? k.hs1 : k.hs0));
  const unsigned long long pz = (unsigned long long)ylo * 0x1CE4E5B9u;
  const unsigned zlo = (unsigned)pz;
  const unsigned zhi = (unsigned)(pz >> 32) + ylo * 0xBF58476Du + (c ? k.t1 : k.t0);
  const unsigned wlo = zlo ^ ((zlo >> 27) | (zhi << 5));
  const unsigned whi = zhi ^ (zhi >> 27);
  const unsigned vhi =
      (unsigned)(((unsigned long long)wlo * 0x133111EBu) >> 32) + wlo * 0x94D049BBu + whi * 0x133111EBu;
  return vhi ^ (vhi >> 31);
}

}  // namespace perc
