"""ctypes binding of libperc.so (include/perc.h).

The library is built in-tree (percolation_amd/libperc.so, by
percolation_amd/build.py or `make -C percolation_amd/csrc`).  Loading fails
loudly when it is missing: there is no Python or CPU fallback for any
compute entry point.
"""
import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# (PERC_LIBPERC: a probe build of the same sources, e.g. another tile shape)
LIBPERC = os.environ.get("PERC_LIBPERC") or os.path.join(HERE, "libperc.so")

PERC_OK = 0
ERRORS = {
    -1: "PERC_EINVAL", -2: "PERC_ENOMEM", -3: "PERC_EHIP", -4: "PERC_ENMAX",
    -5: "PERC_EITOL", -6: "PERC_EMISMATCH", -7: "PERC_EREPLAY", -8: "PERC_ENODEV",
    -9: "PERC_ESTATE",
}
SQUARE, TRIANGULAR = 0, 1
BOND, SITE, SITEBOND, BONDSITE = 0, 1, 2, 3
RULE_BOND, RULE_SITE, RULE_MIXED = 0, 1, 2
CUR_FORTRAN, CUR_MATLAB = 0, 1
FMT_AUTO, FMT_CSR, FMT_STENCIL, FMT_STENCIL_SPLIT, FMT_STENCIL_TILED = 0, 1, 2, 3, 4
MARCH_QFREE, MARCH_ALT, SOLVE_RESIDENT, MARCH_STRIPS, MARCH_SLOTS, MARCH_TAG = 1, 2, 8, 16, 64, 128
MARCH_NIBBLE = 512
MARCH_DEFAULT = (MARCH_QFREE | MARCH_ALT | SOLVE_RESIDENT | MARCH_STRIPS | MARCH_SLOTS | MARCH_TAG
                 | MARCH_NIBBLE)
DOT_FAST, DOT_LITERAL, DOT_LITERAL_HOST = 0, 1, 2
# perc_last_solve: kernel family and flag bits of the last solve
RAN_OTHER, RAN_MARCH, RAN_SLABS, RAN_RESIDENT, RAN_SMALL = 0, 1, 2, 3, 4
RAN_LITERAL, RAN_LIT_TERMS, RAN_QFREE, RAN_STRIPS, RAN_NIBBLE, RAN_TAG, RAN_HOST_FOLD = 1, 2, 4, 8, 16, 32, 64
RAN_XCD_GROUPED, RAN_DEFERRED = 128, 256
XPORT_RCCL, XPORT_HOST, XPORT_EXCHANGE = 0, 1, 4
DSLAB_ID_BYTES = 128


class LabelInfo(C.Structure):
    _fields_ = [("nclusters", C.c_int), ("nspan", C.c_int), ("span_root", C.c_int),
                ("span_sites", C.c_int), ("replayed", C.c_int), ("perccln", C.c_int)]


class CondResult(C.Structure):
    _fields_ = [("gtop", C.c_double), ("gbot", C.c_double), ("err", C.c_double),
                ("iter", C.c_int), ("status", C.c_int), ("t_assemble_ms", C.c_double),
                ("t_solve_ms", C.c_double), ("t_currents_ms", C.c_double)]


class DslabBufs(C.Structure):
    _fields_ = [(k, C.c_void_p) for k in ("part_out", "part_all", "edge_lo", "edge_hi",
                                          "ghost_lo", "ghost_hi")]


DSLAB_COMBINE_INIT, DSLAB_PS, DSLAB_COMBINE_PS, DSLAB_B, DSLAB_COMBINE_B, DSLAB_GHOSTS = range(6)


class Realisation(C.Structure):
    _fields_ = [("label", LabelInfo), ("cond", CondResult), ("t_upload_ms", C.c_double),
                ("t_label_ms", C.c_double), ("t_total_ms", C.c_double)]


class PercError(RuntimeError):
    pass


_I = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
_D = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")
_VP = C.c_void_p
_lib = None

# name -> (restype, argtypes); every symbol declared in include/perc.h
SIGNATURES = {
    "perc_srand": (None, [C.c_int]),
    "perc_rand": (C.c_float, [C.c_int]),
    "perc_trial_seeds": (None, [C.c_int, C.c_int, _I]),
    "perc_nbonds": (C.c_int, [C.c_int] * 4),
    "perc_nearestn": (C.c_int, [C.c_int] * 5 + [_I]),
    "perc_bond_list": (C.c_int, [C.c_int] * 4 + [_I, _I]),
    "perc_shuffle": (None, [C.c_int, _I]),
    "perc_ctx_create": (C.c_int, [C.c_int] * 5 + [C.POINTER(C.c_void_p)]),
    "perc_ctx_destroy": (C.c_int, [_VP]),
    "perc_last_error": (C.c_char_p, []),
    "perc_hip_runtimes": (C.c_int, [C.c_char_p, C.c_int]),
    "perc_occupy": (C.c_int, [_VP, C.c_int, C.c_int, _VP, C.c_int, _VP]),
    "perc_label": (C.c_int, [_VP, C.POINTER(LabelInfo), _VP]),
    "perc_label_numbers": (C.c_int, [_VP, _VP, _VP, _VP, C.c_int, _VP]),
    "perc_replay_labels": (C.c_int, [C.c_int] * 6 + [_VP, C.c_int, _VP, _VP, _VP, _VP, C.c_int,
                                                      _VP]),
    "perc_conductance": (C.c_int, [_VP, C.c_int, C.c_int, C.c_double, C.c_double, C.c_double,
                                   C.c_int, C.c_double, C.c_int, C.POINTER(CondResult), _VP]),
    "perc_get_system": (C.c_int, [_VP, _VP, _VP, _VP, _VP, _VP, C.POINTER(C.c_int),
                                  C.POINTER(C.c_int)]),
    "perc_spmv_host": (C.c_int, [_VP, _D, _D]),
    "perc_bench_kernel": (C.c_int, [_VP, C.c_int, C.c_int, C.POINTER(C.c_double)]),
    "perc_bondc_realisation": (C.c_int, [_VP, C.c_int, _VP, C.c_int, C.c_double, C.c_double,
                                         C.c_double, C.c_int, C.POINTER(Realisation)]),
    "perc_occupy_device": (C.c_int, [_VP, C.c_int, C.c_int, _VP, C.c_int, _VP]),
    "perc_set_kernel_timing": (C.c_int, [_VP, C.c_int]),
    "perc_kernel_stats": (C.c_int, [_VP, _D, C.c_int]),
    "perc_system_size": (C.c_int, [_VP, np.ctypeslib.ndpointer(dtype=np.int64)]),
    "perc_set_matrix_format": (C.c_int, [_VP, C.c_int]),
    "perc_matrix_format": (C.c_int, [_VP]),
    "perc_first_spanning": (C.c_int, [_VP, C.c_int, _VP, C.c_int, C.c_int, _VP]),
    "perc_bs_perc_replay": (C.c_int, [C.c_int] * 4 + [_VP, C.c_int, _VP, C.c_int, C.c_int, _VP]),
    "perc_first_spanning_mixed": (C.c_int, [_VP, C.c_int, _VP, C.c_int, _VP, C.c_int, C.c_int,
                                            _VP]),
    "perc_trial_seeds_scaled": (None, [C.c_int, C.c_int, C.c_int, _I]),
    "perc_set_full_voltages": (C.c_int, [_VP, C.c_int]),
    "perc_set_march_rows": (C.c_int, [_VP, C.c_int]),
    "perc_set_slabs": (C.c_int, [_VP, C.c_int]),
    "perc_dslab_begin": (C.c_int, [_VP, C.c_int, C.c_int, C.c_int, C.c_double, C.c_int, C.c_int,
                                   C.POINTER(DslabBufs)]),
    "perc_dslab_step": (C.c_int, [_VP, C.c_int]),
    "perc_dslab_status": (C.c_int, [_VP, C.POINTER(C.c_int), C.POINTER(C.c_double),
                                    C.POINTER(C.c_int)]),
    "perc_dslab_end": (C.c_int, [_VP]),
    "perc_dslab_solve_group": (C.c_int, [C.c_int, _VP, C.c_int, C.c_int, C.c_int, C.c_double,
                                         C.c_double, C.c_double, C.c_int, C.c_double, C.c_int,
                                         C.c_int, _VP]),
    "perc_assemble": (C.c_int, [_VP, C.c_int, C.c_double, C.c_double, C.c_double,
                                C.POINTER(C.c_int)]),
    "perc_dslab_unique_id": (C.c_int, [_VP, C.c_int]),
    "perc_dslab_comm_init": (C.c_int, [_VP, C.c_int, C.c_int, _VP, C.c_int]),
    "perc_dslab_comm_free": (C.c_int, [_VP]),
    "perc_dslab_solve": (C.c_int, [_VP, C.c_int, C.c_int, C.c_double, C.c_double, C.c_double,
                                   C.c_int, C.c_double, C.c_int, C.c_int, C.POINTER(CondResult)]),
    "perc_set_conductcalc_weights": (C.c_int, [_VP, C.c_int, C.c_uint]),
    "perc_twister_uniform": (C.c_int, [C.c_uint, C.c_longlong, _VP]),
    "perc_replay_bond_trace": (C.c_int, [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, _VP, _VP]),
    "perc_replay_site_trace": (C.c_int, [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, _VP, _VP]),
    "perc_replay_mixed_trace": (C.c_int, [C.c_int] * 6 + [_VP, C.c_int, _VP, _VP, C.c_longlong,
                                                           C.POINTER(C.c_longlong)]),
    "perc_x_row": (C.c_int, [_VP, C.c_int, _VP, C.c_int]),
    "perc_currents": (C.c_int, [_VP, C.c_int, C.c_int, C.c_double, C.c_double, C.c_double,
                                C.POINTER(CondResult)]),
    "perc_stream": (C.c_void_p, [_VP]),
    "perc_cluster_sizes": (C.c_int, [_VP, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    "perc_occupy_random": (C.c_int, [_VP, C.c_int, C.c_int, C.c_int, C.c_ulonglong]),
    "perc_occupancy": (C.c_int, [_VP, _VP, _VP]),
    "perc_random_order": (C.c_int, [C.c_longlong, C.c_int, C.c_ulonglong, C.c_int, _I]),
    "perc_set_march_mode": (C.c_int, [_VP, C.c_int]),
    "perc_set_band_weights": (C.c_int, [_VP, C.c_int, C.c_int, _VP]),
    "perc_set_dot_order": (C.c_int, [_VP, C.c_int]),
    "perc_err_history": (C.c_int, [_VP, _VP, C.c_int]),
    "perc_march_info": (C.c_int, [_VP, _VP]),
    "perc_last_solve": (C.c_int, [_VP, _VP]),
    "perc_set_bond_weights": (C.c_int, [_VP, _VP, C.c_longlong]),
    "perc_selftest_division": (C.c_int, [C.c_longlong, C.c_ulonglong, _VP]),
    "perc_stats_accumulate": (None, [_D, C.c_int, C.c_double, C.c_int, C.c_int]),
    "sprsin_": (None, [_VP] * 7),
    "dsprsax_": (None, [_VP] * 5),
    "dsprstx_": (None, [_VP] * 5),
    "atimes_": (None, [_VP] * 4),
    "nearestn_": (None, [_VP]),
    "asolve_": (None, [_VP] * 4),
    "snrm_": (C.c_double, [_VP] * 3),
    "linbcg_": (None, [_VP] * 8),
    "perc_nr_bind": (None, [_VP, _VP, C.c_int]),
    "perc_nr_status": (C.c_int, []),
    "perc_nr_status_": (C.c_int, []),
    "perc_nr_set_dot_order": (C.c_int, [C.c_int]),
    "perc_shuffle_seeded": (None, [C.c_int, C.c_int, _I]),
    "perc_ensemble_create": (C.c_int, [C.c_int, _VP, C.c_int, C.c_int, C.c_int, C.c_int,
                                       C.POINTER(C.c_void_p)]),
    "perc_ensemble_destroy": (C.c_int, [_VP]),
    "perc_ensemble_ndev": (C.c_int, [_VP]),
    "perc_ensemble_set_workers": (C.c_int, [_VP, C.c_int]),
    "perc_ensemble_workers": (C.c_int, [_VP]),
    "perc_ensemble_ctx": (C.c_void_p, [_VP, C.c_int]),
    "perc_ensemble_trials": (C.c_int, [C.c_int, C.c_int, C.c_int, _VP]),
    "perc_ensemble_allreduce": (C.c_int, [_VP, _D, C.c_int]),
    "perc_ensemble_bond_cond": (C.c_int, [_VP, C.c_int, _I, C.c_int, _I, C.c_double, C.c_double,
                                          C.c_double, C.c_int, _I, _D, _D, _I, _I, _I, _VP]),
}


def _one_runtime():
    """One HIP / HSA / RCCL runtime per process.  torch ships its own copies
    (torch/lib/libamdhip64.so, libhsa-runtime64.so, librccl.so, sonames .so.7
    / .so.1 / .so.1) and names them unversioned in its NEEDED entries; libperc
    names the sonames.  Loaded after torch, libperc's sonames bind to torch's
    copies already in the process.  Loaded BEFORE torch, libperc brings
    /opt/rocm's copies and a later `import torch` loads torch's beside them:
    two HIP and two HSA runtimes on one device, a torch ExternalStream of a
    libperc stream names a handle of the other runtime, and interpreter exit
    aborts with glibc's "double free or corruption (!prev)" (round 4's
    teardown abort; reproduced without a GPU by tests/test_host_cpu.py).  So
    torch, where installed, is imported first (PERC_NO_TORCH=1 skips it for a
    process that will never import torch: /opt/rocm's runtime then)."""
    if os.environ.get("PERC_NO_TORCH") == "1":
        return
    try:
        import torch  # noqa: F401
    except ImportError:
        pass


def _torch_runtime():
    """the libamdhip64 torch would load (its bundled copy), found without
    importing torch; None if torch or its bundled runtime is absent"""
    import importlib.util
    try:
        spec = importlib.util.find_spec("torch")
    except (ImportError, ValueError):
        return None
    if spec is None or not spec.origin:
        return None
    p = os.path.join(os.path.dirname(spec.origin), "lib", "libamdhip64.so")
    return os.path.realpath(p) if os.path.exists(p) else None


class _SecondRuntimeGuard:
    """sys.meta_path entry installed when libperc was loaded on a HIP runtime
    other than torch's bundled one (PERC_NO_TORCH=1, or torch not importable
    then): a later `import torch` would map a second runtime into the
    process, so it raises PercError before torch's libraries load -- the
    invariant is checked, not left to the import order"""

    def __init__(self, ours, theirs):
        self.ours, self.theirs = ours, theirs

    def find_spec(self, name, path=None, target=None):
        if name == "torch":
            raise PercError("import torch after libperc would load a second HIP runtime (%s beside "
                            "libperc's %s; two runtimes corrupt the heap at exit): import torch before "
                            "percolation_amd, or leave PERC_NO_TORCH unset" % (self.theirs, self.ours))
        return None


def runtimes(L=None):
    """(count, paths) of the libamdhip64 copies mapped in this process
    (perc_hip_runtimes): the copy libperc binds to first"""
    L = L or lib()
    buf = C.create_string_buffer(8192)
    n = L.perc_hip_runtimes(buf, len(buf))
    paths = [p for p in buf.value.decode(errors="replace").split(";") if p]
    return n, paths


def _check_one_runtime(L):
    import sys
    if not hasattr(L, "perc_hip_runtimes"):
        return  # (an older probe build)
    n, paths = runtimes(L)
    if n > 1:
        raise PercError("two HIP runtimes in one process: %s -- import torch before percolation_amd"
                        % "; ".join(paths))
    if "torch" not in sys.modules and paths:
        theirs = _torch_runtime()
        if theirs and theirs != paths[0] and not any(isinstance(f, _SecondRuntimeGuard) for f in sys.meta_path):
            sys.meta_path.insert(0, _SecondRuntimeGuard(paths[0], theirs))


def lib():
    """Load libperc.so (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIBPERC):
        raise PercError("libperc.so not built: run `python -c 'import __graft_entry__ as g; "
                        "g.build()'` or `make -C percolation_amd/csrc` (%s missing)" % LIBPERC)
    _one_runtime()
    L = C.CDLL(LIBPERC, mode=C.RTLD_GLOBAL)
    probe = bool(os.environ.get("PERC_LIBPERC"))
    for name, (res, args) in SIGNATURES.items():
        if probe and not hasattr(L, name):
            continue  # (an older probe build: entry points added since are absent)
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _check_one_runtime(L)
    _lib = L
    return L


def check(rc, what=""):
    if rc != PERC_OK:
        msg = lib().perc_last_error().decode(errors="replace")
        raise PercError("%s failed: %s (%s)" % (what, ERRORS.get(rc, rc), msg))
    return rc


def ptr(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)
