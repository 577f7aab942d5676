"""ctypes binding of oracle/liboracle.so -- TEST INFRASTRUCTURE ONLY.

The oracle is the checker: tests, __graft_entry__.smoke() and bench.py's
cpu_baseline leg load it; the product (percolation_amd / libperc) never does.
"""
import ctypes as C
import os

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_SO = os.path.join(REPO, "oracle", "liboracle.so")

_I = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
_D = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")
_IP = C.POINTER(C.c_int)
_lib = None


class BondcResult(C.Structure):
    _fields_ = [(k, C.c_int) for k in
                ("nb", "tbonds", "cln", "maxcn", "maxcs", "perccln", "perccls", "iter")] + \
               [(k, C.c_double) for k in ("gtop", "gbot", "err")]


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(ORACLE_SO):
        import subprocess
        subprocess.check_call(["make", "-s", "-C", os.path.dirname(ORACLE_SO)])
    L = C.CDLL(ORACLE_SO)
    i, d = C.c_int, C.c_double
    sig = {
        "or_srand": (None, [i]),
        "or_rand": (C.c_float, [i]),
        "or_scn": (i, [i]),
        "or_bcn": (i, [i]),
        "or_nbonds": (i, [i, i, i, i]),
        "or_nearestn": (None, [i, i, i, i, i, _I]),
        "or_bond_list": (i, [i, i, i, i, _I, _I]),
        "or_shuffle_pairs": (None, [i, _I, _I]),
        "or_shuffle_ints": (None, [i, _I]),
        "or_trial_seeds": (None, [i, i, _I]),
        "or_label_bonds_literal": (i, [i, i, i, i, i, _I, _I, _I, _I, i, _I, _I, _IP, _IP]),
        "or_label_bonds_replay": (i, [i, i, i, i, i, _I, _I, _I, _I, i, _I, _I, _IP, _IP]),
        "or_label_sites_literal": (i, [i, i, i, i, _I, i, _I, _I, _IP, _IP]),
        "or_label_sites_replay": (i, [i, i, i, i, _I, i, _I, _I, _IP, _IP]),
        "or_label_sitebond": (i, [i, i, i, i, i, _I, _I, _I, i, _I, _I, i, _I, _I, _I, _IP, _IP]),
        "or_label_bondsite": (i, [i, i, i, i, i, _I, _I, _I, i, _I, i, _I, _I, _I, _IP, _IP]),
        "or_label_sitebond_replay": (i, [i, i, i, i, i, _I, _I, _I, i, _I, _I, i, _I, _I, _I, _IP,
                                         _IP]),
        "or_canon_sites": (None, [i, _I, i, _I]),
        "or_canon_bonds": (None, [i, i, _I, _I, _I, i, _I]),
        "or_span_bonds": (i, [i, i, i, _I, _I, _I, _I, i]),
        "or_span_sites": (i, [i, i, _I, _I, i, i]),
        "or_bond_values": (None, [i, i, _I, _I, _I, _I, i, d, d, _D]),
        "or_assemble": (i, [i, i, i, i, i, _I, _I, _D, d, d, i, i, _D, _I, _D, _D]),
        "or_dsprsax": (None, [_D, _I, _D, _D, i]),
        "or_dsprstx": (None, [_D, _I, _D, _D, i]),
        "or_linbcg": (None, [_D, _I, i, _D, _D, i, d, i, _IP, C.POINTER(d), C.c_void_p]),
        "or_linbcg_sym": (i, [_D, _I, i, _D, _D, i, i, i, _D, _D, _I, _D, _IP, C.POINTER(d),
                              C.c_void_p, i]),
        "or_currents": (None, [i, i, i, i, i, _I, _I, _D, _D, _D, d, d, i,
                               C.POINTER(d), C.POINTER(d)]),
        "or_bondc": (i, [i, i, i, i, d, i, d, d, i, d, i, C.c_void_p, C.c_void_p,
                         C.c_void_p, C.c_void_p, C.POINTER(BondcResult)]),
        "or_bond_cond_trial": (i, [i, i, i, i, i, d, d, i, d, _D, _D, _D, _I, _IP,
                                   C.POINTER(d)]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


def i32(n):
    return np.zeros(n, dtype=np.int32)


def f64(n):
    return np.zeros(n, dtype=np.float64)


# ---------------------------------------------------------------- helpers
def bond_list(lattice, m, n, pbc):
    L = lib()
    nb = L.or_nbonds(lattice, m, n, pbc)
    b1, b2 = i32(nb), i32(nb)
    cnt = L.or_bond_list(lattice, m, n, pbc, b1, b2)
    assert cnt == nb, (cnt, nb)
    return b1, b2


def bond_order(lattice, m, n, pbc, seed):
    b1, b2 = bond_list(lattice, m, n, pbc)
    nb = len(b1)
    o1, o2 = i32(nb + 1), i32(nb + 1)
    o1[:nb], o2[:nb] = b1, b2
    L = lib()
    L.or_srand(seed)
    L.or_shuffle_pairs(nb, o1, o2)
    return b1, b2, o1, o2


def site_order(t, seed):
    order = i32(t + 1)
    order[:t] = np.arange(1, t + 1, dtype=np.int32)
    L = lib()
    L.or_srand(seed)
    L.or_shuffle_ints(t, order)
    return order


def label_bonds(lattice, m, n, pbc, b1, b2, o1, o2, tbonds, literal=True):
    L = lib()
    nb = len(b1)
    label, csize = i32(nb), i32(nb + 2)
    mx, ms = C.c_int(), C.c_int()
    f = L.or_label_bonds_literal if literal else L.or_label_bonds_replay
    cln = f(lattice, m, n, pbc, nb, b1, b2, o1, o2, tbonds, label, csize,
            C.byref(mx), C.byref(ms))
    return label, csize, cln, mx.value, ms.value


def label_sites(lattice, m, n, pbc, order, tsites, literal=True):
    L = lib()
    t = m * n
    s, csize = i32(t), i32(t + 2)
    mx, ms = C.c_int(), C.c_int()
    f = L.or_label_sites_literal if literal else L.or_label_sites_replay
    cln = f(lattice, m, n, pbc, order, tsites, s, csize, C.byref(mx), C.byref(ms))
    return s, csize, cln, mx.value, ms.value


def label_sitebond(lattice, m, n, pbc, b1, b2, sorder, tsites, o1, o2, tbonds, literal=True):
    """mixed site-then-bond labels (sitebond.f:187-400): literal or O(N alpha) replay"""
    L = lib()
    t, nb = m * n, len(b1)
    s, bl, csize = i32(t), i32(nb), i32(t + nb + 2)
    mx, ms = C.c_int(), C.c_int()
    f = L.or_label_sitebond if literal else L.or_label_sitebond_replay
    cln = f(lattice, m, n, pbc, nb, b1, b2, sorder, tsites, o1, o2, tbonds, s, bl, csize,
            C.byref(mx), C.byref(ms))
    return s, bl, csize, cln, mx.value, ms.value


def canon_sites(s, maxlab):
    """canonical partition ids from site labels (min site of the cluster)"""
    out = i32(len(s))
    lib().or_canon_sites(len(s), np.ascontiguousarray(s, dtype=np.int32), int(maxlab), out)
    return out


def canon_bonds(t, b1, b2, label, maxlab):
    """canonical partition ids per site from bond labels"""
    out = i32(t)
    lib().or_canon_bonds(t, len(b1), b1, b2, np.ascontiguousarray(label, dtype=np.int32),
                         int(maxlab), out)
    return out


def conductance(lattice, m, n, pbc, b1, b2, gval, Va=1.0, itol=2, tol=1e-8,
                itmax=2500, rhs_rule=0, cur_rule=0, cur_thresh=1e-10):
    """assembly + linbcg + currents; returns dict (bondc.f:465-595)."""
    L = lib()
    t = m * n
    N = t - 2 * m
    nb = len(b1)
    nmax = N + 1 + 2 * nb + 8
    sa, ija = f64(nmax), i32(nmax)
    itemp, diag = f64(N), f64(t)
    k = L.or_assemble(lattice, m, n, pbc, nb, b1, b2, gval, Va, 1e-16, rhs_rule,
                      nmax, sa, ija, itemp, diag)
    assert k > 0
    vint = f64(N)
    it, err = C.c_int(), C.c_double()
    errs = f64(itmax + 2)
    L.or_linbcg(sa, ija, N, itemp, vint, itol, tol, itmax, C.byref(it), C.byref(err),
                errs.ctypes.data_as(C.c_void_p))
    gt, gb = C.c_double(), C.c_double()
    L.or_currents(lattice, m, n, pbc, nb, b1, b2, gval, diag, vint, Va, cur_thresh,
                  cur_rule, C.byref(gt), C.byref(gb))
    return dict(sa=sa[:k], ija=ija[:k], itemp=itemp, diag=diag, vint=vint,
                iter=it.value, err=err.value, errs=errs[:it.value],
                gtop=gt.value, gbot=gb.value, nnz=k)


def conductance_decades(lattice, m, n, pbc, b1, b2, gval, tols, Va=1.0, itmax=10 ** 7,
                        rhs_rule=0, cur_rule=0, cur_thresh=1e-10, threads=4, dot_order=0):
    """conductance() at several tolerances from one linbcg run
    (or_linbcg_sym: the literal iterates, threaded; tols descending).
    Returns a list of dicts (gtop, gbot, iter, err, true_res) per tolerance
    and the per-iteration err history.  true_res = ||b - A x||_2 / ||b/d||_2
    of the snapshot, recomputed in the same NR storage (diagnostic).
    dot_order 1: the dot products summed in descending order (not the
    reference's association; measures the solver's own association spread)."""
    L = lib()
    t = m * n
    N = t - 2 * m
    nb = len(b1)
    nmax = N + 1 + 2 * nb + 8
    sa, ija = f64(nmax), i32(nmax)
    itemp, diag = f64(N), f64(t)
    k = L.or_assemble(lattice, m, n, pbc, nb, b1, b2, gval, Va, 1e-16, rhs_rule,
                      nmax, sa, ija, itemp, diag)
    assert k > 0
    tols = np.ascontiguousarray(sorted(tols, reverse=True), dtype=np.float64)
    nc = len(tols)
    vint = f64(N)
    cx = f64(nc * N)
    citer, cerr = i32(nc), f64(nc)
    it, err = C.c_int(), C.c_double()
    errs = f64(itmax + 2)
    rc = L.or_linbcg_sym(sa, ija, N, itemp, vint, itmax, threads, nc, tols, cx, citer, cerr,
                         C.byref(it), C.byref(err), errs.ctypes.data_as(C.c_void_p), dot_order)
    assert rc == 0, "matrix not bitwise symmetric"
    bn = np.linalg.norm(itemp / sa[:N])
    out = []
    for c in range(nc):
        xs = np.ascontiguousarray(cx[c * N:(c + 1) * N])
        gt, gb = C.c_double(), C.c_double()
        L.or_currents(lattice, m, n, pbc, nb, b1, b2, gval, diag, xs, Va, cur_thresh,
                      cur_rule, C.byref(gt), C.byref(gb))
        ax = f64(N)
        L.or_dsprsax(sa, ija, xs, ax, N)
        out.append(dict(tol=float(tols[c]), gtop=gt.value, gbot=gb.value, iter=int(citer[c]),
                        err=float(cerr[c]),
                        true_res=float(np.linalg.norm(itemp - ax) / bn)))
    return out, errs[:it.value]


def bondc(lattice, m, n, pbc, pb, seed, Va=1.0, g0=1.0, itmax=2500, tol=1e-8,
          literal=False):
    L = lib()
    nb = L.or_nbonds(lattice, m, n, pbc)
    label, csize = i32(nb), i32(nb + 2)
    o1, o2 = i32(nb + 1), i32(nb + 1)
    res = BondcResult()
    rc = L.or_bondc(lattice, m, n, pbc, pb, seed, Va, g0, itmax, tol, int(literal),
                    label.ctypes.data_as(C.c_void_p), csize.ctypes.data_as(C.c_void_p),
                    o1.ctypes.data_as(C.c_void_p), o2.ctypes.data_as(C.c_void_p),
                    C.byref(res))
    assert rc == 0, rc
    out = {k: getattr(res, k) for k, _ in BondcResult._fields_}
    out.update(label=label, csize=csize, o1=o1, o2=o2)
    return out
