"""Host-side mirror of the reference drivers over the libperc C-ABI.

The drop-in host is Fortran (percolation_amd/fortran/); this module mirrors
the same programs for tests and the benchmark, with the reference's
parameter names and semantics:

  bondc      Fortran/Square/bondc.f, Fortran/Triangular/bondc.f
  site       Fortran/*/site.f (+ MATLAB/ConductCalc.m site rule)
  sitebond   Fortran/*/sitebond.f (+ ConductCalc.m mixed rule)
  bond_cond  Fortran/*/bond_cond.f grid-point conductances

Every compute step runs in libperc on the GPU; there is no fallback.
"""
import ctypes as C

import numpy as np

from . import _lib as L

LEAK = 1.0e-12  # bondc.f:487


def _i32(n):
    return np.zeros(n, dtype=np.int32)


def nbonds(lattice, m, n, pbc=0):
    return L.lib().perc_nbonds(lattice, m, n, pbc)


def bond_list(lattice, m, n, pbc=0):
    """(b1, b2) in reference order (bondc.f:137-154)."""
    nb = nbonds(lattice, m, n, pbc)
    b1, b2 = _i32(nb), _i32(nb)
    got = L.lib().perc_bond_list(lattice, m, n, pbc, b1, b2)
    assert got == nb
    return b1, b2


def nearestn(lattice, m, n, pbc, rn):
    nn = _i32(6)
    scn = L.lib().perc_nearestn(lattice, m, n, pbc, rn, nn)
    return nn[:scn]


def shuffled_ids(N, seed):
    """1-based id permutation after srand(seed) + REAL*4 Fisher-Yates;
    N+1 slots, slot N is the H2 spill slot (bondc.f:162-174)."""
    order = _i32(N + 1)
    order[:N] = np.arange(1, N + 1, dtype=np.int32)
    lib = L.lib()
    lib.perc_srand(seed)
    lib.perc_shuffle(N, order)
    return order


def random_order(n, count, seed, kind=L.BOND):
    """The order perc_occupy_random's occupancy is the prefix of: the first
    `count` ids (1-based) in ascending counter-based key order (host)."""
    out = _i32(max(count, 1))
    L.check(L.lib().perc_random_order(int(n), int(count), int(seed), int(kind), out),
            "perc_random_order")
    return out[:count]


def trial_seeds(master, k=1000, scale=10000000):
    """tseed(1..k) = int(rand(0)*scale)+1 after srand(master): scale 1e7 in
    bond_cond.f:65-70, 1e6 in bond_perc.f / site_perc.f:70-74."""
    ts = _i32(k)
    if scale == 10000000:
        L.lib().perc_trial_seeds(master, k, ts)
    else:
        L.lib().perc_trial_seeds_scaled(master, k, scale, ts)
    return ts


def replay_labels(lattice, m, n, pbc, kind, site_order=None, nsites=0, bond_order=None,
                  nbond=0):
    """Reference label numbering of an explicit occupancy (host replay, no
    device): dict(bond_label, site_label, csize, cln, maxcn, maxcs, perccln)."""
    t = m * n
    nb = nbonds(lattice, m, n, pbc)
    cap = {L.BOND: nb + 2, L.SITE: t + 2}.get(kind, t + nb + 2)
    bl = _i32(nb) if kind != L.SITE else None
    sl = _i32(t) if kind != L.BOND else None
    cs, st = _i32(cap), _i32(4)
    so = None if site_order is None else np.ascontiguousarray(site_order, dtype=np.int32)
    bo = None if bond_order is None else np.ascontiguousarray(bond_order, dtype=np.int32)
    L.check(L.lib().perc_replay_labels(lattice, m, n, pbc, kind, nsites, L.ptr(so), nbond,
                                       L.ptr(bo), L.ptr(bl), L.ptr(sl), L.ptr(cs), cap,
                                       L.ptr(st)), "perc_replay_labels")
    return dict(bond_label=bl, site_label=sl, csize=cs, cln=int(st[0]), maxcn=int(st[1]),
                maxcs=int(st[2]), perccln=int(st[3]))


class Context:
    """One libperc context (one lattice on one device)."""

    def __init__(self, lattice, m, n, pbc=0, device=0):
        self.lattice, self.m, self.n, self.pbc = lattice, m, n, pbc
        self.device = device
        self.t = m * n
        self.nb = nbonds(lattice, m, n, pbc)
        self.N = self.t - 2 * m
        h = C.c_void_p()
        L.check(L.lib().perc_ctx_create(device, lattice, m, n, pbc, C.byref(h)),
                "perc_ctx_create")
        self.h = h

    def close(self):
        if self.h:
            L.lib().perc_ctx_destroy(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- occupancy ---------------------------------------------------------
    def occupy(self, kind, site_order=None, nsites=0, bond_order=None, nbonds_=0):
        so = None if site_order is None else np.ascontiguousarray(site_order, dtype=np.int32)
        bo = None if bond_order is None else np.ascontiguousarray(bond_order, dtype=np.int32)
        L.check(L.lib().perc_occupy(self.h, kind, nsites, L.ptr(so), nbonds_, L.ptr(bo)),
                "perc_occupy")

    def occupy_random(self, kind, nsites=0, nbonds_=0, seed=1):
        """perc_occupy_random: the nsites / nbonds_ smallest counter-based
        keys occupied, drawn on the device (no order array)."""
        L.check(L.lib().perc_occupy_random(self.h, kind, int(nsites), int(nbonds_), int(seed)),
                "perc_occupy_random")

    def occupancy(self):
        """perc_occupancy: (site_occ[t], bond_occ[nb]) uint8 arrays of the
        device occupancy (site / bond ids 1.. at index 0..)."""
        so = np.zeros(self.t, dtype=np.uint8)
        bo = np.zeros(self.nb, dtype=np.uint8)
        L.check(L.lib().perc_occupancy(self.h, so.ctypes.data, bo.ctypes.data), "perc_occupancy")
        return so, bo

    def occupy_device(self, kind, site_ptr=None, nsites=0, bond_ptr=None, nbonds_=0):
        """perc_occupy_device: order lists already in device memory (int
        addresses of device int32 arrays on this context's device)."""
        sp = C.c_void_p(site_ptr) if site_ptr else None
        bp = C.c_void_p(bond_ptr) if bond_ptr else None
        L.check(L.lib().perc_occupy_device(self.h, kind, nsites, sp, nbonds_, bp),
                "perc_occupy_device")

    def label(self, canon=False):
        info = L.LabelInfo()
        out = _i32(self.t) if canon else None
        L.check(L.lib().perc_label(self.h, C.byref(info), L.ptr(out)), "perc_label")
        res = {k: getattr(info, k) for k, _ in L.LabelInfo._fields_}
        if canon:
            res["canon"] = out
        return res

    def label_numbers(self, kind):
        if kind == L.BOND:
            cap = self.nb + 2
        elif kind == L.SITE:
            cap = self.t + 2
        else:
            cap = self.t + self.nb + 2
        bl = _i32(self.nb) if kind != L.SITE else None
        sl = _i32(self.t) if kind != L.BOND else None
        cs, st = _i32(cap), _i32(4)
        L.check(L.lib().perc_label_numbers(self.h, L.ptr(bl), L.ptr(sl), L.ptr(cs), cap,
                                           L.ptr(st)), "perc_label_numbers")
        return dict(bond_label=bl, site_label=sl, csize=cs, cln=int(st[0]), maxcn=int(st[1]),
                    maxcs=int(st[2]), perccln=int(st[3]))

    # -- conductance -------------------------------------------------------
    def conductance(self, rule=L.RULE_BOND, cur_rule=L.CUR_FORTRAN, Va=1.0, g0=1.0, leak=LEAK,
                    itol=2, tol=1e-8, itmax=2500, vint=False):
        res = L.CondResult()
        v = np.zeros(self.N, dtype=np.float64) if vint else None
        L.check(L.lib().perc_conductance(self.h, rule, cur_rule, Va, g0, leak, itol, tol, itmax,
                                         C.byref(res), L.ptr(v)), "perc_conductance")
        out = {k: getattr(res, k) for k, _ in L.CondResult._fields_}
        if vint:
            out["vint"] = v
        return out

    def system(self):
        n, nnz = C.c_int(), C.c_int()
        L.check(L.lib().perc_get_system(self.h, None, None, None, None, None, C.byref(n),
                                        C.byref(nnz)), "perc_get_system")
        rp, col = _i32(n.value + 1), _i32(nnz.value)
        val, diag, rhs = (np.zeros(k, np.float64) for k in (nnz.value, n.value, n.value))
        L.check(L.lib().perc_get_system(self.h, L.ptr(rp), L.ptr(col), L.ptr(val), L.ptr(diag),
                                        L.ptr(rhs), C.byref(n), C.byref(nnz)),
                "perc_get_system")
        return dict(rowptr=rp, col=col, val=val, diag=diag, rhs=rhs)

    def spmv(self, x):
        x = np.ascontiguousarray(x, dtype=np.float64)
        y = np.zeros_like(x)
        L.check(L.lib().perc_spmv_host(self.h, x, y), "perc_spmv_host")
        return y

    def bench_kernel(self, which, reps):
        ms = C.c_double()
        L.check(L.lib().perc_bench_kernel(self.h, which, reps, C.byref(ms)), "perc_bench_kernel")
        return ms.value

    def set_kernel_timing(self, enable=True):
        L.check(L.lib().perc_set_kernel_timing(self.h, int(enable)), "perc_set_kernel_timing")

    def kernel_stats(self, reset=True):
        st = np.zeros(6)
        L.check(L.lib().perc_kernel_stats(self.h, st, int(reset)), "perc_kernel_stats")
        return dict(spmv_ms=st[0], spmv_n=int(st[1]), resid_ms=st[2], resid_n=int(st[3]),
                    xp_ms=st[4], xp_n=int(st[5]))

    def set_matrix_format(self, fmt):
        """PERC_FMT_AUTO / _CSR / _STENCIL (fused) / _STENCIL_SPLIT / _STENCIL_TILED (perc.h)."""
        L.check(L.lib().perc_set_matrix_format(self.h, int(fmt)), "perc_set_matrix_format")

    def set_full_voltages(self, enable=True):
        """Keep every interior voltage up to date during the solve (perc.h)."""
        L.check(L.lib().perc_set_full_voltages(self.h, int(enable)), "perc_set_full_voltages")

    def cluster_sizes(self):
        """(maxcs, span_size) of the labeled bond / site occupancy on the
        GPU (perc_cluster_sizes)."""
        mx, sp = C.c_int(), C.c_int()
        L.check(L.lib().perc_cluster_sizes(self.h, C.byref(mx), C.byref(sp)), "perc_cluster_sizes")
        return mx.value, sp.value

    def set_slabs(self, nslab=1):
        """Row-slab decomposition of the CG solve (perc_set_slabs)."""
        L.check(L.lib().perc_set_slabs(self.h, int(nslab)), "perc_set_slabs")

    def set_march_rows(self, rows=0):
        """Band height of the register-march kernel (0: auto; perc.h)."""
        L.check(L.lib().perc_set_march_rows(self.h, int(rows)), "perc_set_march_rows")

    def set_march_mode(self, mode):
        """PERC_MARCH_* bits of the register-march loop (perc.h)."""
        L.check(L.lib().perc_set_march_mode(self.h, int(mode)), "perc_set_march_mode")

    def set_band_weights(self, which=None, weights=None):
        """Per-round weights of the slot-weighted bands (perc_set_band_weights;
        which 0: strip-major P, 1: its B, 2: row-major P).  No arguments:
        the defaults."""
        if which is None:
            L.check(L.lib().perc_set_band_weights(self.h, 0, 0, None), "perc_set_band_weights")
            return
        w = np.ascontiguousarray(weights, dtype=np.int32)
        L.check(L.lib().perc_set_band_weights(self.h, int(which), len(w), w.ctypes.data),
                "perc_set_band_weights")

    def set_dot_order(self, order):
        """PERC_DOT_FAST / PERC_DOT_LITERAL: the association of linbcg's dot
        products (perc_set_dot_order; LITERAL reproduces the reference solver
        bitwise)."""
        L.check(L.lib().perc_set_dot_order(self.h, int(order)), "perc_set_dot_order")

    def err_history(self):
        """err of every iteration of the last solve (perc_err_history)."""
        n = L.lib().perc_err_history(self.h, None, 0)
        if n < 0:
            L.check(n, "perc_err_history")
        out = np.zeros(n, dtype=np.float64)
        m = L.lib().perc_err_history(self.h, out.ctypes.data, n)
        if m < 0:
            L.check(m, "perc_err_history")
        return out

    def set_conductcalc_weights(self, rule, seed=1838534):
        """ConductCalc.m condtype 2 inside libperc (perc_set_conductcalc_weights):
        the spanning cluster's -g0 bonds of the last labeling get
        -g0*rand('twister', seed), one draw per bond in bond-list order --
        conductcalc_weights + set_bond_weights without the host replay."""
        L.check(L.lib().perc_set_conductcalc_weights(self.h, rule, int(seed) & 0xFFFFFFFF),
                "perc_set_conductcalc_weights")

    def set_bond_weights(self, w=None):
        """Per-bond conductance multipliers for the spanning cluster's bonds
        (ConductCalc.m condtype 2; None: fixed g0).  perc_set_bond_weights."""
        if w is None:
            L.check(L.lib().perc_set_bond_weights(self.h, None, 0), "perc_set_bond_weights")
            return
        w = np.ascontiguousarray(w, dtype=np.float64)
        L.check(L.lib().perc_set_bond_weights(self.h, w.ctypes.data, len(w)),
                "perc_set_bond_weights")

    def march_info(self):
        """The solver loop of the assembled system (perc_march_info)."""
        out = np.zeros(5, dtype=np.int32)
        L.check(L.lib().perc_march_info(self.h, out.ctypes.data), "perc_march_info")
        return dict(kernel=("none", "wave", "", "resident", "small")[out[0]],
                    qfree=bool(out[1] & 1), strips=bool(out[1] & 2), slots=bool(out[1] & 8), tag=bool(out[1] & 16),
                    nibble=bool(out[1] & 32),
                    alt=bool(out[2]), band_rows=int(out[3]), strip_cols=int(out[4]))

    def last_solve(self):
        """What the last solve actually ran (perc_last_solve): the kernel
        family ('other', 'march', 'slabs', 'resident', 'small'), its flags and
        the iteration count.  lit_terms: the literal folds summed the terms
        the solve kernels themselves stored (the production kernels ran)."""
        out = np.zeros(4, dtype=np.int32)
        L.check(L.lib().perc_last_solve(self.h, out.ctypes.data), "perc_last_solve")
        f = int(out[1])
        return dict(kernel=("other", "march", "slabs", "resident", "small")[out[0]],
                    literal=bool(f & L.RAN_LITERAL), lit_terms=bool(f & L.RAN_LIT_TERMS),
                    qfree=bool(f & L.RAN_QFREE), strips=bool(f & L.RAN_STRIPS),
                    nibble=bool(f & L.RAN_NIBBLE), tag=bool(f & L.RAN_TAG),
                    host_fold=bool(f & L.RAN_HOST_FOLD), xcd_grouped=bool(f & L.RAN_XCD_GROUPED),
                    deferred=bool(f & L.RAN_DEFERRED),
                    iter=int(out[2]))

    def matrix_format(self):
        rc = L.lib().perc_matrix_format(self.h)
        if rc < 0:
            L.check(rc, "perc_matrix_format")
        return rc

    def system_size(self):
        out = np.zeros(2, dtype=np.int64)
        L.check(L.lib().perc_system_size(self.h, out), "perc_system_size")
        return int(out[0]), int(out[1])

    def bondc_realisation(self, order, tbonds, Va=1.0, g0=1.0, tol=1e-8, itmax=2500,
                          device_ptr=None):
        """occupy + label + conductance.  `order` is a host int32 array, or
        pass device_ptr (int address of a device int32 array) instead."""
        r = L.Realisation()
        if device_ptr is not None:
            src, on_dev = C.c_void_p(device_ptr), 1
        else:
            order = np.ascontiguousarray(order, dtype=np.int32)
            src, on_dev = L.ptr(order), 0
        L.check(L.lib().perc_bondc_realisation(self.h, tbonds, src, on_dev, Va, g0, tol, itmax,
                                               C.byref(r)), "perc_bondc_realisation")
        out = {k: getattr(r.label, k) for k, _ in L.LabelInfo._fields_}
        out.update({k: getattr(r.cond, k) for k, _ in L.CondResult._fields_})
        out.update(t_upload_ms=r.t_upload_ms, t_label_ms=r.t_label_ms,
                   t_total_ms=r.t_total_ms)
        return out


# ---------------------------------------------------------------- programs
def dslab_solve_group(ctxs, xport=L.XPORT_RCCL, rule=L.RULE_BOND, cur_rule=L.CUR_FORTRAN, Va=1.0,
                      g0=1.0, leak=LEAK, itol=2, tol=1e-8, itmax=2500, full_x=False):
    """One solve split over the labeled contexts `ctxs` (slab s on ctxs[s]),
    the whole loop inside libperc: perc_dslab_solve_group (RCCL over the
    contexts' devices, or staged through the host)."""
    K = len(ctxs)
    arr = (C.c_void_p * K)(*[c.h for c in ctxs])
    res = L.CondResult()
    L.check(L.lib().perc_dslab_solve_group(K, arr, int(xport), rule, cur_rule, Va, g0, leak, itol,
                                           tol, itmax, int(full_x), C.byref(res)),
            "perc_dslab_solve_group")
    return {k: getattr(res, k) for k, _ in L.CondResult._fields_}


def bondc(lattice=0, m=50, n=50, pbc=0, pb=0.50, seed=626504, Va=1.0, g0=1.0, tol=1e-8,
          itmax=2500, labels=True, ctx=None, device=0):
    """One bond realisation filled to pb, spanning test, conductance
    (Fortran/Square/bondc.f; triangular defaults pb=.35, seed=62703)."""
    own = ctx is None
    ctx = ctx or Context(lattice, m, n, pbc, device)
    try:
        nb = ctx.nb
        order = shuffled_ids(nb, seed)
        tbonds = int(pb * nb)  # bondc.f:191
        ctx.occupy(L.BOND, bond_order=order, nbonds_=tbonds)
        li = ctx.label()
        out = dict(nb=nb, tbonds=tbonds, order=order, nspan=li["nspan"],
                   span_root=li["span_root"], span_sites=li["span_sites"])
        if labels:
            ln = ctx.label_numbers(L.BOND)
            out.update(label=ln["bond_label"], csize=ln["csize"], cln=ln["cln"],
                       maxcn=ln["maxcn"], maxcs=ln["maxcs"], perccln=ln["perccln"],
                       perccls=int(ln["csize"][ln["perccln"]]) if ln["perccln"] else 0)
        c = ctx.conductance(L.RULE_BOND, L.CUR_FORTRAN, Va, g0, LEAK, 2, tol, itmax)
        out.update(gtop=c["gtop"], gbot=c["gbot"], iter=c["iter"], err=c["err"],
                   cond_status=c["status"])
        return out
    finally:
        if own:
            ctx.close()


def site(lattice=0, m=50, n=50, pbc=0, ps=0.60, seed=1080115, conductance=False, Va=1.0,
         g0=1.0, tol=1e-8, itmax=100000, cur_rule=L.CUR_MATLAB, ctx=None, device=0):
    """Site realisation (Fortran/Square/site.f) and, optionally, the
    ConductCalc.m site-rule conductance of its spanning cluster."""
    own = ctx is None
    ctx = ctx or Context(lattice, m, n, pbc, device)
    try:
        t = ctx.t
        order = shuffled_ids(t, seed)
        tsites = int(ps * t)
        ctx.occupy(L.SITE, site_order=order, nsites=tsites)
        li = ctx.label()
        ln = ctx.label_numbers(L.SITE)
        out = dict(order=order, tsites=tsites, site_label=ln["site_label"], csize=ln["csize"],
                   cln=ln["cln"], maxcn=ln["maxcn"], maxcs=ln["maxcs"], perccln=ln["perccln"],
                   nspan=li["nspan"], span_root=li["span_root"])
        if conductance:
            c = ctx.conductance(L.RULE_SITE, cur_rule, Va, g0, LEAK, 2, tol, itmax)
            out.update(gtop=c["gtop"], gbot=c["gbot"], iter=c["iter"], err=c["err"])
        return out
    finally:
        if own:
            ctx.close()


def sitebond(lattice=0, m=50, n=50, pbc=0, ps=0.50, pb=0.50, sseed=143285, bseed=43716,
             conductance=False, Va=1.0, g0=1.0, tol=1e-8, itmax=100000, cur_rule=L.CUR_MATLAB,
             ctx=None, device=0):
    """Mixed site-then-bond realisation (Fortran/Square/sitebond.f) and,
    optionally, the ConductCalc.m mixed-rule conductance."""
    own = ctx is None
    ctx = ctx or Context(lattice, m, n, pbc, device)
    try:
        t, nb = ctx.t, ctx.nb
        sorder = shuffled_ids(t, sseed)   # sitebond.f:129-143
        border = shuffled_ids(nb, bseed)  # sitebond.f:177-189
        ts, tb = int(ps * t), int(pb * nb)
        ctx.occupy(L.SITEBOND, site_order=sorder, nsites=ts, bond_order=border, nbonds_=tb)
        li = ctx.label()
        ln = ctx.label_numbers(L.SITEBOND)
        out = dict(sorder=sorder, border=border, site_label=ln["site_label"],
                   bond_label=ln["bond_label"], csize=ln["csize"], cln=ln["cln"],
                   maxcn=ln["maxcn"], maxcs=ln["maxcs"], perccln=ln["perccln"],
                   nspan=li["nspan"], span_root=li["span_root"])
        if conductance:
            c = ctx.conductance(L.RULE_MIXED, cur_rule, Va, g0, LEAK, 2, tol, itmax)
            out.update(gtop=c["gtop"], gbot=c["gbot"], iter=c["iter"], err=c["err"])
        return out
    finally:
        if own:
            ctx.close()


def bondsite(lattice=0, m=10, n=10, pbc=0, ps=0.50, pb=0.50, sseed=143285, bseed=43716):
    """Mixed bonds-then-sites realisation (Fortran/Square/bondsite.f): bonds
    to pb (seed bseed), each a size-1 cluster, then sites to ps (seed sseed)
    merging their neighbour bonds' clusters; reference numbering by host
    replay (perc_replay_labels, PERC_BONDSITE).  Also the drop-in text of
    bssite.txt / bsbond.txt (bondsite.f:420-430)."""
    t, nb = m * n, nbonds(lattice, m, n, pbc)
    sorder = shuffled_ids(t, sseed)   # bondsite.f:116-127
    border = shuffled_ids(nb, bseed)  # bondsite.f:153-166
    ts, tb = int(ps * t), int(pb * nb)
    r = replay_labels(lattice, m, n, pbc, L.BONDSITE, site_order=sorder, nsites=ts,
                      bond_order=border, nbond=tb)
    b1, b2 = bond_list(lattice, m, n, pbc)
    s_ext = np.zeros(nb + 1, dtype=np.int64)
    s_ext[1:min(t, nb) + 1] = r["site_label"][:min(t, nb)]
    c = r["csize"]
    r["bssite"] = fmt_i10(np.arange(1, nb + 1), s_ext[1:], c[1:nb + 1])
    r["bsbond"] = fmt_i10(b1, b2, r["bond_label"])
    r.update(sorder=sorder, border=border)
    return r


def twister_uniform(seed, n):
    """n draws of rand('twister', seed): MT19937 init_genrand(seed), 53-bit
    genrand_res53 doubles (perc_twister_uniform, host C)."""
    out = np.empty(max(int(n), 1))
    L.check(L.lib().perc_twister_uniform(int(seed) & 0xFFFFFFFF, int(n), out.ctypes.data),
            "perc_twister_uniform")
    return out[:n]


def conductcalc_weights(rule, b1, b2, bond_label, site_label, perccln, seed=1838534):
    """ConductCalc.m condtype 2 (MATLAB/ConductCalc.m:38-47, 94-97, 114-118,
    136-146): the bonds that get -g0 under the rule get -g0*rand instead,
    one rand per such bond in bond-list order from rand('twister', seed).
    MATLAB's 'twister' is MT19937 seeded by init_genrand(seed) with 53-bit
    doubles (genrand_res53) -- the generator numpy.random.RandomState(seed)
    .random_sample implements.  Parity with MATLAB itself is unpinned (no
    MATLAB here).  Returns w (1.0 for the other bonds)."""
    nb = len(b1)
    if rule == L.RULE_BOND:
        mask = bond_label == perccln
    else:
        both = (site_label[b1 - 1] == perccln) & (site_label[b2 - 1] == perccln)
        mask = both if rule == L.RULE_SITE else both & (bond_label == perccln)
    w = np.ones(nb)
    w[mask] = np.random.RandomState(seed).random_sample(int(mask.sum()))
    return w


def pb_grid(lattice, nb):
    """nbarr of bond_cond.f:84-97 (square 0.49.., triangular 0.35.., +5e-3)."""
    pbarr = np.zeros(250)
    pbarr[0] = 0.35 if lattice else 0.49
    npts = 131 if lattice else 103
    for i in range(1, npts):
        pbarr[i] = pbarr[i - 1] + 5.00e-03
    return (pbarr * nb).astype(np.int64).astype(np.int32)  # truncation (H3 repeats kept)


def first_spanning(ctx, order, kind=L.BOND, n=None):
    """Smallest count c such that occupying order[:c] spans (the pc step of
    bond_cond.f:381; bond_perc.f / site_perc.f), 0 if none: perc_first_spanning,
    a bisection with the GPU labeling.  The context is left occupied at c."""
    n = (ctx.nb if kind == L.BOND else ctx.t) if n is None else n
    o = np.ascontiguousarray(order[:n], dtype=np.int32)
    first = C.c_int()
    L.check(L.lib().perc_first_spanning(ctx.h, kind, L.ptr(o), n, 0, C.byref(first)),
            "perc_first_spanning")
    return first.value


def threshold_scan(lattice=0, m=50, n=50, pbc=0, kind=L.BOND, master=58302, numtrials=10,
                   ctx=None, device=0, replay=False):
    """bond_perc / site_perc (Fortran/Square/bond_perc.f, site_perc.f): per
    trial ii, seed tseed(ii) = int(rand(0)*1e6)+1, the reference shuffle,
    then the first occupation count that spans; the record is (tseed,
    fraction = REAL*4 count/N, largest cluster size, spanning cluster size)
    at that step (the whole order if nothing spans), sizes on the GPU
    (perc_cluster_sizes; replay=True: by the host label replay, which also
    gives the reference label number perccln)."""
    own = ctx is None
    ctx = ctx or Context(lattice, m, n, pbc, device)
    try:
        N = ctx.nb if kind == L.BOND else ctx.t
        seeds = trial_seeds(master, max(numtrials, 1), scale=1000000)
        out = []
        for ii in range(numtrials):
            order = shuffled_ids(N, int(seeds[ii]))
            first = first_spanning(ctx, order, kind, N)
            c = first if first else N
            if replay:  # reference label numbers too (host replay)
                r = ctx.label_numbers(kind)
                maxcs, perccln = r["maxcs"], r["perccln"]
                perccls = int(r["csize"][perccln]) if first and perccln else 0
            else:  # the two sizes the record needs, on the GPU
                maxcs, span = ctx.cluster_sizes()
                perccls, perccln = (span if first else 0), None
            out.append(dict(tseed=int(seeds[ii]), count=c,
                            f=float(np.float32(np.float32(c) / np.float32(N))),
                            maxcs=maxcs, perccls=perccls, perccln=perccln))
        return out
    finally:
        if own:
            ctx.close()


def first_spanning_mixed(ctx, scan, site_order, nsites, bond_order, nbonds):
    """perc_first_spanning_mixed: sites fixed and bonds scanned (scan=BOND,
    sb_perc) or bonds fixed and sites scanned (scan=SITE, bs_perc)."""
    so = np.ascontiguousarray(site_order[:max(nsites, 1)], dtype=np.int32)
    bo = np.ascontiguousarray(bond_order[:max(nbonds, 1)], dtype=np.int32)
    first = C.c_int()
    L.check(L.lib().perc_first_spanning_mixed(ctx.h, scan, L.ptr(so), nsites, L.ptr(bo), nbonds,
                                              0, C.byref(first)), "perc_first_spanning_mixed")
    return first.value


def bs_perc_replay(lattice, m, n, pbc, site_order, nsites, bond_order, nbond, c0_overflow=True):
    """perc_bs_perc_replay: bs_perc's site scan by host replay (first
    spanning site count); c0_overflow reproduces the reference build
    (hazard H11), False gives the intended site+bond connectivity."""
    so = np.ascontiguousarray(site_order[:max(nsites, 1)], dtype=np.int32)
    bo = np.ascontiguousarray(bond_order[:max(nbond, 1)], dtype=np.int32)
    first = C.c_int()
    L.check(L.lib().perc_bs_perc_replay(lattice, m, n, pbc, L.ptr(so), nsites, L.ptr(bo), nbond,
                                        int(c0_overflow), C.byref(first)), "perc_bs_perc_replay")
    return first.value


def paired_seeds(pseed, k=1000):
    """sseed(jj), bseed(jj) = int(rand(0)*1e7)+1 drawn alternately after
    srand(pseed) (sb_perc.f / bs_perc.f:106-111)."""
    lib = L.lib()
    lib.perc_srand(int(pseed))
    ss, bs = _i32(k), _i32(k)
    for j in range(k):
        ss[j] = int(np.float32(lib.perc_rand(0)) * np.float32(10000000)) + 1
        bs[j] = int(np.float32(lib.perc_rand(0)) * np.float32(10000000)) + 1
    return ss, bs


def mixed_scan(lattice=0, m=50, n=50, pbc=0, scan=L.BOND, master=8811064, points=None,
               iters=100, as_built=True, ctx=None, device=0):
    """sb_perc (scan=BOND: sites fixed at ps, bonds added until a mixed
    cluster spans; Square/sb_perc.f) / bs_perc (scan=SITE: bonds fixed at
    pb, sites added; Square/bs_perc.f).  points: the ps (sb) / pb (bs)
    values, default the reference's (square 0.59 + 0.01 i x 42, triangular
    0.50 + 0.01 i x 51) / 0.30 + 0.01 i x 71.  Records (sseed, bseed, ps,
    pb); the scanned fraction is 0 when nothing spans.  sb_perc's first
    spanning bond count is the GPU bisection (perc_first_spanning_mixed);
    bs_perc's is the host replay of the reference as built (as_built, hazard
    H11) or, with as_built=False, the GPU bisection of the intended rule."""
    own = ctx is None
    ctx = ctx or Context(lattice, m, n, pbc, device)
    try:
        t, nb = ctx.t, ctx.nb
        if points is None:
            if scan == L.BOND:
                points = ([0.59 + 0.01 * i for i in range(42)] if lattice == 0
                          else [0.50 + 0.01 * i for i in range(51)])
            else:
                points = [0.30 + 0.01 * i for i in range(71)]
        pseed = trial_seeds(master, 100)
        out = []
        for ii, pt in enumerate(points):
            ss, bs = paired_seeds(pseed[ii])
            for jj in range(iters):
                so = shuffled_ids(t, int(ss[jj]))
                bo = shuffled_ids(nb, int(bs[jj]))
                if scan == L.BOND:
                    ts = int(pt * t)  # sb_perc.f:210 (truncation)
                    first = first_spanning_mixed(ctx, L.BOND, so, ts, bo, nb)
                    ps = float(np.float32(ts) / np.float32(t))
                    pb = float(np.float32(first) / np.float32(nb)) if first else 0.0
                else:
                    tb = int(pt * nb)  # bs_perc.f:209
                    if as_built:
                        first = bs_perc_replay(lattice, m, n, pbc, so, t, bo, tb, True)
                    else:
                        first = first_spanning_mixed(ctx, L.SITE, so, t, bo, tb)
                    pb = float(np.float32(tb) / np.float32(nb))
                    ps = float(np.float32(first) / np.float32(t)) if first else 0.0
                out.append(dict(sseed=int(ss[jj]), bseed=int(bs[jj]), ps=ps, pb=pb, first=first))
        return out
    finally:
        if own:
            ctx.close()


def fmt_mixed_rows(rows):
    """sb_perc.txt / bs_perc.txt records: (i10,",",i10,",",f12.9,",",f12.9)."""
    return "".join("%10d,%10d,%12.9f,%12.9f\n" % (r["sseed"], r["bseed"], r["ps"], r["pb"])
                   for r in rows)


def fmt_perc_rows(rows):
    """bond_perc.txt / site_perc.txt records: (i10,",",f12.9,",",i10,",",i10)."""
    return "".join("%10d,%12.9f,%10d,%10d\n" % (r["tseed"], r["f"], r["maxcs"], r["perccls"])
                   for r in rows)


def bond_cond_grid(lattice=0, m=10, n=10, pbc=0, master=58302, numtrials=1, Va=1.0, g0=1.0,
                   tol=1e-8, itmax=2500, trials=None, with_labels=True, ctx=None, device=0):
    """bond_cond (Fortran/Square/bond_cond.f:123-498): per trial ii, seed
    tseed(ii), conductance of the lowest-label spanning cluster at each
    grid point nbarr(jj) until the sweep ends (or stalls on a repeated
    nbarr value, hazard H3), pc = first spanning fraction, and the final
    lowest spanning label."""
    own = ctx is None
    ctx = ctx or Context(lattice, m, n, pbc, device)
    try:
        nb = ctx.nb
        seeds = trial_seeds(master, 1000)
        nbarr = pb_grid(lattice, nb)
        out = []
        for ii in (trials if trials is not None else range(numtrials)):
            order = shuffled_ids(nb, int(seeds[ii]))
            rows = []
            jj = 0
            for bf in nbarr:
                if bf <= 0 or jj >= len(nbarr) or bf != nbarr[jj]:
                    break
                if rows and bf <= rows[-1]["bf"]:
                    break  # H3: repeated nbarr value stalls the sweep
                ctx.occupy(L.BOND, bond_order=order, nbonds_=int(bf))
                li = ctx.label()
                c = ctx.conductance(L.RULE_BOND, L.CUR_FORTRAN, Va, g0, LEAK, 2, tol, itmax)
                pbv = float(np.float32(np.float32(bf) / np.float32(nb)))
                rows.append(dict(bf=int(bf), pb=pbv, gbot=c["gbot"], gtop=c["gtop"],
                                 iter=c["iter"], spanning=li["nspan"] > 0))
                jj += 1
            bfc = first_spanning(ctx, order)
            pc = float(np.float32(np.float32(bfc) / np.float32(nb))) if bfc else 0.0
            tr = dict(ii=ii + 1, seed=int(seeds[ii]), rows=rows, pc=pc, bf_c=bfc)
            if with_labels:
                ctx.occupy(L.BOND, bond_order=order, nbonds_=nb)
                tr["perccln"] = ctx.label_numbers(L.BOND)["perccln"] if bfc else 0
            out.append(tr)
        return out
    finally:
        if own:
            ctx.close()


# ---------------------------------------------------------------- file output
def fmt_i10(*cols):
    """Records of (i10,",",i10,...) -- the reference's formatted writes."""
    n = len(cols[0])
    f = ",".join(["%10d"] * len(cols)) + "\n"
    return "".join(f % tuple(int(c[i]) for c in cols) for i in range(n))


# ---------------------------------------------------------------- multi-GPU ensemble
class Ensemble:
    """perc_ensemble: one context + host thread per device of this node,
    trials striped ii -> device (ii-1) mod ndev, one RCCL all-reduce of the
    per-grid-point statistics (include/perc.h; Square/bond_cond.f:123-498)."""

    def __init__(self, lattice, m, n, pbc=0, ndev=1, devices=None, workers=1):
        self.lattice, self.m, self.n, self.pbc = lattice, m, n, pbc
        self.nb = nbonds(lattice, m, n, pbc)
        h = C.c_void_p()
        dv = None if devices is None else np.ascontiguousarray(devices, dtype=np.int32)
        L.check(L.lib().perc_ensemble_create(ndev, L.ptr(dv), lattice, m, n, pbc, C.byref(h)),
                "perc_ensemble_create")
        self.h = h
        self.ndev = L.lib().perc_ensemble_ndev(h)
        self.workers = 1
        if workers != 1:
            self.set_workers(workers)

    def set_workers(self, workers):
        """contexts (host threads, streams) per device (perc_ensemble_set_workers)"""
        L.check(L.lib().perc_ensemble_set_workers(self.h, workers), "perc_ensemble_set_workers")
        self.workers = L.lib().perc_ensemble_workers(self.h)

    def close(self):
        if self.h:
            L.lib().perc_ensemble_destroy(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def allreduce(self, per_device):
        """per_device: (ndev, k) array; returns the sum over devices (RCCL)."""
        a = np.ascontiguousarray(per_device, dtype=np.float64).copy()
        k = a.shape[1]
        L.check(L.lib().perc_ensemble_allreduce(self.h, a.reshape(-1), k),
                "perc_ensemble_allreduce")
        return a

    def bond_cond(self, master=58302, numtrials=1, Va=1.0, g0=1.0, tol=1e-8, itmax=2500):
        """The bond_cond trial loop over the devices; same records as
        bond_cond_grid, plus the all-reduced statistics (npts, 5)."""
        if numtrials < 0:
            raise ValueError("numtrials < 0")
        # tseed(1..1000) as bond_cond.f:65-70, extended with the same stream past 1000
        # trials (perc_ensemble_bond_cond reads tseed[0..numtrials-1])
        seeds = trial_seeds(master, max(1000, numtrials))
        nbarr = pb_grid(self.lattice, self.nb)
        npts = len(nbarr)
        nrows, bfc, pl = _i32(numtrials), _i32(numtrials), _i32(numtrials)
        gbot, gtop = np.zeros(numtrials * npts), np.zeros(numtrials * npts)
        iters = _i32(numtrials * npts)
        stats = np.zeros(npts * 5)
        L.check(L.lib().perc_ensemble_bond_cond(self.h, numtrials, seeds, npts, nbarr, Va, g0,
                                                tol, itmax, nrows, gbot, gtop, iters, bfc, pl,
                                                stats.ctypes.data_as(C.c_void_p)),
                "perc_ensemble_bond_cond")
        out = []
        for t in range(numtrials):
            rows = []
            for j in range(nrows[t]):
                o = t * npts + j
                bf = int(nbarr[j])
                rows.append(dict(bf=bf, pb=float(np.float32(np.float32(bf) / np.float32(self.nb))),
                                 gbot=float(gbot[o]), gtop=float(gtop[o]), iter=int(iters[o])))
            b = int(bfc[t])
            out.append(dict(ii=t + 1, seed=int(seeds[t]), rows=rows, bf_c=b, perccln=int(pl[t]),
                            pc=float(np.float32(np.float32(b) / np.float32(self.nb))) if b else 0.0))
        return out, stats.reshape(npts, 5)


def ensemble_trials(ntrials, ndev, dev):
    """1-based trials device `dev` of `ndev` runs (perc_ensemble_trials)."""
    cnt = L.lib().perc_ensemble_trials(ntrials, ndev, dev, None)
    out = _i32(max(cnt, 0))
    L.lib().perc_ensemble_trials(ntrials, ndev, dev, L.ptr(out))
    return out
