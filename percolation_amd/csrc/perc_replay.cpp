// perc_replay.cpp -- reference label numbering by O(N alpha) host replay.
//
// Cluster label numbers in the reference are history-dependent: a new
// cluster takes the counter `cln`, a merge keeps the label of the largest
// neighbouring cluster (ties: first in nearestn/nnb order) and zeroes the
// absorbed sizes (Fortran/Square/bondc.f:275-364, Square/site.f:184-254,
// Square/sitebond.f:230-389).  The GPU labeling produces the partition; these
// replays reproduce the numbers with a union-find over sites, in
// O(N alpha) instead of the reference's O(N^2) relabel scans.
#include <algorithm>
#include <cstring>
#include <numeric>
#include <vector>

#include "perc_internal.h"

namespace perc {
namespace {

struct DSU {
  std::vector<int> par, sz;
  explicit DSU(int n) : par(n), sz(n, 1) { std::iota(par.begin(), par.end(), 0); }
  int find(int x) {
    int r = x;
    while (par[r] != r) r = par[r];
    while (par[x] != r) {
      const int nx = par[x];
      par[x] = r;
      x = nx;
    }
    return r;
  }
  int unite(int a, int b) {
    a = find(a);
    b = find(b);
    if (a == b) return a;
    if (sz[a] < sz[b]) std::swap(a, b);
    par[b] = a;
    sz[a] += sz[b];
    return a;
  }
};

// bond-list index of (p<q) using the per-site forward neighbour rank
inline int bond_index(const Geom& g, const std::vector<int>& bond_first, int p, int q) {
  if (p < 1 || p > g.t) return -1;
  int nn[6];
  nearestn(g, p, nn);
  int r = 0;
  for (int k = 0; k < g.scn; ++k)
    if (nn[k] > p) {
      if (nn[k] == q) return bond_first[p] + r;
      ++r;
    }
  return -1;
}

// bond id (0-based) -> endpoints
inline void bond_ends(const Geom& g, const std::vector<int>& bond_first, int id, int* p, int* q) {
  const int s = int(std::upper_bound(bond_first.begin() + 1, bond_first.begin() + g.t + 1, id) -
                    bond_first.begin()) - 1;
  int nn[6];
  nearestn(g, s, nn);
  int r = bond_first[s];
  for (int k = 0; k < g.scn; ++k)
    if (nn[k] > s) {
      if (r == id) { *p = s; *q = nn[k]; return; }
      ++r;
    }
  *p = *q = 0;
}

inline void track_max(const std::vector<int>& c, int lcn, int lcs, int* maxcn, int* maxcs) {
  // bondc.f:382-391 / site.f:263-272
  if (c[lcn] > *maxcs) {
    *maxcs = c[lcn];
    *maxcn = lcn;
  } else if (lcs == 0 && *maxcs == 0) {
    *maxcs = 1;
    *maxcn = 1;
  }
}

}  // namespace

int replay_bonds(const Geom& g, const std::vector<int>& bond_first, const int* order, int count,
                 int* label, int* csize, int cap, int* stats, int* trace) {
  const long long nb = nbonds(g);
  if (cap < nb + 2) return PERC_EINVAL;
  std::vector<int> c(cap, 0);  // c(0) stays 0 (hazard H1)
  std::vector<int> clab(g.t + 1, 0);
  std::vector<uint8_t> occ(nb, 0);
  DSU dsu(g.t + 1);
  int cln = 1, maxcn = 0, maxcs = 0;
  for (int i = 0; i < count; ++i) {
    const int id = order[i];
    if (id <= 0 || id > nb) {
      // H2 sentinel (0,0): no nnb row or b row matches; the reference opens
      // a cluster number that no bond carries.
      c[cln] = 1;
      if (trace) { trace[3 * i] = 0; trace[3 * i + 1] = cln; trace[3 * i + 2] = 1; }
      ++cln;
      if (maxcs == 0) { maxcs = 1; maxcn = 1; }
      continue;
    }
    int a, b;
    bond_ends(g, bond_first, id - 1, &a, &b);
    // nnb rows: neighbours of a (except b), then of b (except a)
    int rs[10], rlab[10], rsz[10], rc = 0;
    int nn[6];
    nearestn(g, a, nn);
    for (int k = 0; k < g.scn; ++k)
      if (nn[k] != 0 && nn[k] != b) {
        const int lo = std::min(a, nn[k]), hi = std::max(a, nn[k]);
        const int q = bond_index(g, bond_first, lo, hi);
        rs[rc] = lo;
        rlab[rc] = (q >= 0 && occ[q]) ? clab[dsu.find(lo)] : 0;
        ++rc;
      }
    nearestn(g, b, nn);
    for (int k = 0; k < g.scn; ++k)
      if (nn[k] != 0 && nn[k] != a) {
        const int lo = std::min(b, nn[k]), hi = std::max(b, nn[k]);
        const int q = bond_index(g, bond_first, lo, hi);
        rs[rc] = lo;
        rlab[rc] = (q >= 0 && occ[q]) ? clab[dsu.find(lo)] : 0;
        ++rc;
      }
    for (int k = 0; k < rc; ++k) rsz[k] = c[rlab[k]];
    int lcn = rc ? rlab[0] : 0, lcs = rc ? rsz[0] : 0;
    for (int k = 1; k < rc; ++k)
      if (rlab[k] != 0 && rsz[k] > lcs) { lcn = rlab[k]; lcs = rsz[k]; }
    occ[id - 1] = 1;
    if (lcs == 0) {
      if (clab[dsu.find(a)] != 0 || clab[dsu.find(b)] != 0) return PERC_EREPLAY;  // H7
      const int r = dsu.unite(a, b);
      clab[r] = cln;
      c[cln] = 1;
      if (trace) { trace[3 * i] = 0; trace[3 * i + 1] = cln; trace[3 * i + 2] = 1; }
      ++cln;
    } else {
      int clsum = lcs;
      for (int k = 0; k < rc; ++k) {
        if (rlab[k] == 0) continue;
        if (rlab[k] != lcn) {
          bool dup = false;
          for (int l = 0; l < k; ++l) dup |= rlab[l] == rlab[k];
          if (!dup) clsum += rsz[k];
          c[rlab[k]] = 0;
        }
        dsu.unite(a, rs[k]);
      }
      const int r = dsu.unite(a, b);
      clab[r] = lcn;
      c[lcn] = clsum + 1;
      if (trace) { trace[3 * i] = 1; trace[3 * i + 1] = lcn; trace[3 * i + 2] = c[lcn]; }
    }
    track_max(c, lcn, lcs, &maxcn, &maxcs);
  }
  if (label) {
    for (int s = 1; s < g.t; ++s)
      for (int k = bond_first[s]; k < bond_first[s + 1]; ++k)
        label[k] = occ[k] ? clab[dsu.find(s)] : 0;
  }
  if (csize) std::memcpy(csize, c.data(), sizeof(int) * cap);
  if (stats) { stats[0] = cln; stats[1] = maxcn; stats[2] = maxcs; }
  return PERC_OK;
}

int replay_sites(const Geom& g, const int* order, int count, int* label, int* csize, int cap,
                 int* stats, int* trace) {
  if (cap < g.t + 2) return PERC_EINVAL;
  std::vector<int> c(cap, 0);
  std::vector<int> clab(g.t + 1, 0);
  std::vector<uint8_t> occ(g.t + 1, 0);
  DSU dsu(g.t + 1);
  int cln = 1, maxcn = 0, maxcs = 0;
  for (int i = 0; i < count; ++i) {
    const int sn = order[i];
    if (sn <= 0 || sn > g.t) continue;  // H2 sentinel: reference reads s(-1); skipped
    int nn[6], lab[6], siz[6];
    nearestn(g, sn, nn);
    for (int k = 0; k < g.scn; ++k) {
      lab[k] = (nn[k] > 0 && occ[nn[k]]) ? clab[dsu.find(nn[k])] : 0;
      siz[k] = c[lab[k]];
    }
    int lcn = lab[0], lcs = siz[0], nnlc = nn[0];
    for (int k = 1; k < g.scn; ++k)
      if (nn[k] != 0 && lab[k] != 0 && siz[k] > lcs) { lcn = lab[k]; lcs = siz[k]; nnlc = nn[k]; }
    int* tr = trace ? trace + (size_t)kSiteTrace * i : nullptr;
    if (tr) {
      std::memset(tr, 0, sizeof(int) * kSiteTrace);
      tr[0] = sn;
      for (int k = 0; k < g.scn; ++k) tr[1 + k] = nn[k];
      tr[7] = nnlc;
      tr[8] = lcn;
      tr[9] = lcs;
    }
    occ[sn] = 1;
    if (lcs == 0) {
      clab[sn] = cln;
      c[cln] = 1;
      if (tr) {
        tr[21] = cln;
        tr[22] = 1;
      }
      ++cln;
    } else {
      int clsum = lcs;
      for (int k = 0; k < g.scn; ++k) {
        if (nn[k] == 0 || lab[k] == 0) continue;
        if (lab[k] != lcn) {
          bool dup = false;
          for (int l = 0; l < k; ++l) dup |= lab[l] == lab[k];
          if (!dup) {
            clsum += siz[k];
            c[lab[k]] = 0;
            if (tr && tr[10] < 5) {  // "adding c(s(nn(k))) / largest cluster is now clsum"
              tr[11 + 2 * tr[10]] = siz[k];
              tr[12 + 2 * tr[10]] = clsum;
              ++tr[10];
            }
          }
        }
        dsu.unite(sn, nn[k]);
      }
      clab[dsu.find(sn)] = lcn;
      c[lcn] = clsum + 1;
      if (tr) {
        tr[21] = lcn;
        tr[22] = c[lcn];
      }
    }
    track_max(c, lcn, lcs, &maxcn, &maxcs);
  }
  if (label)
    for (int s = 1; s <= g.t; ++s) label[s - 1] = occ[s] ? clab[dsu.find(s)] : 0;
  if (csize) std::memcpy(csize, c.data(), sizeof(int) * cap);
  if (stats) { stats[0] = cln; stats[1] = maxcn; stats[2] = maxcs; }
  return PERC_OK;
}

int replay_sitebond(const Geom& g, const std::vector<int>& bond_first, const int* sorder,
                    int nsites, const int* border, int nbond, int* site_label, int* bond_label,
                    int* csize, int cap, int* stats, std::vector<int>* ev) {
  const long long nb = nbonds(g);
  if (cap < g.t + nb + 2) return PERC_EINVAL;
  std::vector<int> c(cap, 0);
  std::vector<int> clab(g.t + 1, 0);
  std::vector<uint8_t> socc(g.t + 1, 0);
  std::vector<int> battach(nb, 0);  // >0: site whose cluster the bond follows; <0: own label
  DSU dsu(g.t + 1);
  // log only: the sites and bonds (1-based list ids) each label holds, for
  // the relabel lines of a merge (sitebond.f:317-334), printed in index order
  std::vector<std::vector<int>> msite, mbond;
  if (ev) {
    msite.resize(cap);
    mbond.resize(cap);
  }
  int cln = 1;
  for (int i = 0; i < nsites; ++i) {  // sitebond.f:187-196
    const int sn = sorder[i];
    if (sn > 0 && sn <= g.t) {
      socc[sn] = 1;
      clab[sn] = cln;
      if (ev) msite[cln].push_back(sn);
    }
    c[cln] = 1;
    ++cln;
  }
  auto take = [&](std::vector<int>& v) {  // sorted member list, emptied
    std::sort(v.begin(), v.end());
    ev->push_back((int)v.size());
    ev->insert(ev->end(), v.begin(), v.end());
  };
  int maxcn = 1, maxcs = 1, lcn = 0;
  for (int i = 0; i < nbond; ++i) {  // sitebond.f:223-400
    const int id = border[i];
    if (id > 0 && id <= nb) {
      int a, b;
      bond_ends(g, bond_first, id - 1, &a, &b);
      const int la = socc[a] ? clab[dsu.find(a)] : 0;
      const int lb = socc[b] ? clab[dsu.find(b)] : 0;
      if (la == 0 && lb == 0) {
        battach[id - 1] = -cln;
        c[cln] = 1;
        if (ev) ev->insert(ev->end(), {0, cln});
        ++cln;
      } else if (la > 0 && lb == 0) {
        lcn = la;
        battach[id - 1] = a;
        c[la] += 1;
        if (ev) ev->insert(ev->end(), {1, a, lcn, c[lcn]});
      } else if (la == 0 && lb > 0) {
        lcn = lb;
        battach[id - 1] = b;
        c[lb] += 1;
        if (ev) ev->insert(ev->end(), {2, b, lcn, c[lcn]});
      } else if (la == lb) {
        lcn = la;
        battach[id - 1] = a;
        if (ev) ev->insert(ev->end(), {3, a, la, c[la], b, lb, c[lb], c[la] + 1});
        c[la] += 1;
      } else {
        int oldcn;
        const bool a_big = c[la] > c[lb];
        if (a_big) { lcn = la; oldcn = lb; }
        else { lcn = lb; oldcn = la; }
        const int clsum = c[lcn] + c[oldcn] + 1;
        if (ev) {
          ev->insert(ev->end(), {a_big ? 4 : 5, a, la, c[la], b, lb, c[lb]});
          take(msite[oldcn]);
          take(mbond[oldcn]);
          ev->insert(ev->end(), {lcn, clsum, oldcn});
          msite[lcn].insert(msite[lcn].end(), msite[oldcn].begin(), msite[oldcn].end());
          mbond[lcn].insert(mbond[lcn].end(), mbond[oldcn].begin(), mbond[oldcn].end());
          msite[oldcn].clear();
          mbond[oldcn].clear();
        }
        const int r = dsu.unite(a, b);
        clab[r] = lcn;
        battach[id - 1] = a;
        c[oldcn] = 0;
        c[lcn] = clsum;
      }
      if (ev && battach[id - 1] > 0) mbond[lcn].push_back(id);
    } else if (ev) {
      ev->push_back(6);  // the spill slot (0, 0): no list row matches
    }
    if (c[lcn] > maxcs) { maxcs = c[lcn]; maxcn = lcn; }  // sitebond.f:387-390
  }
  if (site_label)
    for (int s = 1; s <= g.t; ++s) site_label[s - 1] = socc[s] ? clab[dsu.find(s)] : 0;
  if (bond_label)
    for (long long k = 0; k < nb; ++k) {
      const int at = battach[k];
      bond_label[k] = at > 0 ? clab[dsu.find(at)] : (at < 0 ? -at : 0);
    }
  if (csize) std::memcpy(csize, c.data(), sizeof(int) * cap);
  if (stats) { stats[0] = cln; stats[1] = maxcn; stats[2] = maxcs; }
  return PERC_OK;
}

// bondsite (Square/bondsite.f:182-354, Triangular/bondsite.f the same with
// scn 6): bonds border[0..nbond) occupied first, each a cluster of size 1
// numbered in occupation order (an id of 0, the shuffle's spill slot H2,
// still takes a number); then sites in sorder, each joining the clusters of
// its occupied neighbour bonds: the largest (first in nearestn order on a
// tie, the first row's cluster kept unless a later one is strictly larger)
// keeps its number, the others merge into it and their sizes drop to 0, and
// the site counts 1.  A site with no occupied neighbour bond starts its own
// cluster.  Sizes count bonds and sites.  The reference reads c(0) for an
// unoccupied first neighbour bond; in its build that word is 0 (all five
// reference fixtures match with c(0) = 0), so the choice above is the
// intended one.  Union-find over bonds 0..nb-1 and sites nb+s.
int replay_bondsite(const Geom& g, const std::vector<int>& bond_first, const int* sorder,
                    int nsites, const int* border, int nbond, int* site_label, int* bond_label,
                    int* csize, int cap, int* stats, std::vector<int>* ev) {
  const int nb = (int)nbonds(g), t = g.t;
  if (cap < t + nb + 2) return PERC_EINVAL;
  std::vector<int> c(cap, 0);
  std::vector<int> lab(nb + t + 1, 0);  // label of a root element
  std::vector<char> bocc(nb, 0), socc(t + 1, 0);
  DSU u(nb + t + 1);
  int cln = 1;
  for (int i = 0; i < nbond; ++i) {  // bondsite.f:182-199
    const int id = border[i];
    if (id > 0 && id <= nb) {
      bocc[id - 1] = 1;
      lab[id - 1] = cln;
    }
    c[cln] = 1;
    ++cln;
  }
  int maxcn = 1, maxcs = 1;
  for (int i = 0; i < nsites; ++i) {  // bondsite.f:220-320
    const int sn = sorder[i];
    int lcn = 0;
    if (sn < 1 || sn > t) {  // spill slot: a one-site cluster with no site
      c[cln] = 1;
      if (ev) ev->insert(ev->end(), {0, cln});
      ++cln;
    } else {
      int nn[6];
      nearestn(g, sn, nn);
      int rl[6], re[6], nr = 0;  // row label, an element of its cluster
      for (int k = 0; k < g.scn; ++k) {
        if (nn[k] == 0) continue;
        const int id = bond_index(g, bond_first, std::min(sn, nn[k]), std::max(sn, nn[k]));
        rl[nr] = id >= 0 && bocc[id] ? lab[u.find(id)] : 0;
        re[nr] = id;
        ++nr;
      }
      lcn = nr ? rl[0] : 0;
      int lcs = nr ? c[lcn] : 0;
      int le = nr ? re[0] : -1;
      for (int k = 1; k < nr; ++k)
        if (rl[k] != 0 && c[rl[k]] > lcs) {
          lcn = rl[k];
          lcs = c[rl[k]];
          le = re[k];
        }
      const int node = nb + sn;
      socc[sn] = 1;
      if (lcs == 0) {  // bondsite.f:264-274
        lab[node] = cln;
        c[cln] = 1;
        if (ev) ev->insert(ev->end(), {0, cln});
        ++cln;
      } else {         // bondsite.f:278-313
        int clsum = lcs;
        int root = u.find(le);
        size_t at = 0;
        if (ev) {  // {1, k, k x (size added, largest cluster after), lcn, size}
          ev->push_back(1);
          at = ev->size();
          ev->push_back(0);
        }
        for (int k = 0; k < nr; ++k) {
          if (rl[k] == 0 || rl[k] == lcn) continue;
          bool dup = false;
          for (int l = 0; l < k; ++l) dup = dup || rl[l] == rl[k];
          if (!dup) {
            clsum += c[rl[k]];
            root = u.unite(root, re[k]);
            if (ev) {
              ev->insert(ev->end(), {c[rl[k]], clsum});
              ++(*ev)[at];
            }
          }
          c[rl[k]] = 0;
        }
        root = u.unite(root, node);
        lab[root] = lcn;
        c[lcn] = clsum + 1;
        if (ev) ev->insert(ev->end(), {lcn, c[lcn]});
      }
    }
    if (c[lcn] > maxcs) {  // bondsite.f:316-319
      maxcs = c[lcn];
      maxcn = lcn;
    }
  }
  if (site_label)
    for (int s = 1; s <= t; ++s) site_label[s - 1] = socc[s] ? lab[u.find(nb + s)] : 0;
  if (bond_label)
    for (int k = 0; k < nb; ++k) bond_label[k] = bocc[k] ? lab[u.find(k)] : 0;
  if (csize) std::memcpy(csize, c.data(), sizeof(int) * cap);
  if (stats) { stats[0] = cln; stats[1] = maxcn; stats[2] = maxcs; }
  return PERC_OK;
}

// bs_perc's site loop (Square/bs_perc.f:236-350): bonds border[0..nbonds)
// occupied first, each its own cluster of size 1; then sites are added in
// order, each joining the clusters of its occupied neighbour bonds (the
// largest one keeps its number, the others merge into it); returns the
// first site count at which a cluster of >= 2n-1 elements holds a bottom-
// and a top-row site, 0 if none.
//
// c0_overflow reproduces the reference as built (hazard H11): for an
// unoccupied neighbour bond the reference reads c(b(j,3)) = c(0), out of
// bounds, and in the flang build that word exceeds every cluster size. So
// when a site's FIRST neighbour bond (nearestn order) is unoccupied, cluster
// 0 wins the largest-cluster choice (bs_perc.f:271-285): the site and every
// cluster reached through its other occupied bonds are renumbered to 0 --
// they leave the lattice.  Without it (c(0) = 0, the intended rule) this is
// plain site+bond connectivity, what perc_first_spanning_mixed computes.
int replay_bs_scan(const Geom& g, const std::vector<int>& bond_first, const int* sorder,
                   int nsites, const int* border, int nbond, bool c0_overflow) {
  const int nbt = (int)nbonds(g), t = g.t;
  const long long kHuge = 1ll << 60;  // c(0) as read by the reference build
  DSU u(nbt + t + 1);                 // bonds 0..nbt-1, site s -> nbt + s
  std::vector<char> occ(nbt, 0), dead(nbt + t + 1, 0), bot(nbt + t + 1, 0), top(nbt + t + 1, 0);
  std::vector<long long> size(nbt + t + 1, 1);
  for (int i = 0; i < nbond; ++i) {
    const int id = border[i];
    if (id > 0 && id <= nbt) occ[id - 1] = 1;
  }
  struct Row {
    int root;        // -1: cluster 0 (unoccupied or removed bond)
    long long size;  // nnb(k,4)
  };
  for (int i = 1; i <= nsites; ++i) {
    const int s = sorder[i - 1];
    if (s < 1 || s > t) continue;  // H2 spill sentinel: a phantom one-site cluster
    int nn[6];
    nearestn(g, s, nn);
    Row rows[6];
    int nr = 0;
    for (int k = 0; k < g.scn; ++k) {
      if (nn[k] == 0) continue;
      const int lo = std::min(s, nn[k]), hi = std::max(s, nn[k]);
      const int id = bond_index(g, bond_first, lo, hi);
      Row r{-1, 0};
      if (id >= 0) {
        if (occ[id] && !dead[u.find(id)]) {
          r.root = u.find(id);
          r.size = size[r.root];
        } else {
          r.size = c0_overflow ? kHuge : 0;  // c(0)
        }
      }
      rows[nr++] = r;
    }
    int lcn = nr ? rows[0].root : -1;
    long long lcs = nr ? rows[0].size : 0;
    for (int k = 1; k < nr; ++k)
      if (rows[k].root >= 0 && rows[k].size > lcs) {
        lcn = rows[k].root;
        lcs = rows[k].size;
      }
    const int node = nbt + s;
    if (lcs == 0) {  // no occupied neighbour bond: a new one-site cluster
      bot[node] = s <= g.m;
      top[node] = s > t - g.m;
      continue;      // size 1 never spans (n >= 2)
    }
    if (lcn < 0) {  // merged into cluster 0: the site and those clusters leave
      dead[node] = 1;
      for (int k = 0; k < nr; ++k)
        if (rows[k].root >= 0) dead[u.find(rows[k].root)] = 1;
      continue;
    }
    long long tot = size[lcn];
    char b = bot[lcn], tp = top[lcn];
    int root = lcn;
    for (int k = 0; k < nr; ++k) {
      if (rows[k].root < 0) continue;
      const int r = u.find(rows[k].root);
      if (r == u.find(root)) continue;  // lcn itself, or a cluster already merged
      tot += size[r];
      b |= bot[r];
      tp |= top[r];
      root = u.unite(root, r);
    }
    root = u.unite(root, node);
    size[root] = tot + 1;
    bot[root] = b | (s <= g.m);
    top[root] = tp | (s > t - g.m);
    if (size[root] >= 2ll * g.n - 1 && bot[root] && top[root]) return i;
  }
  return 0;
}

}  // namespace perc
