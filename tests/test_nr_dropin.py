"""NR-level drop-in (INTEGRATION.md route 1): the reference's own bondc.f /
bond_cond.f with their embedded Numerical Recipes routines deleted and
linked against libperc.so (oracle/build_ref.sh, build_nr).  The programs'
calls to sprsin / linbcg / dsprsax then run libperc's F77 symbols -- linbcg_
is the HIP Jacobi-PCG -- on the programs' own COMMON /mat/.  Their output
files must equal the unmodified reference's (tests/golden).

These binaries are built only where /root/reference exists (this
container); they travel to the GPU box with oracle/_ref/.
"""
import os
import subprocess

import pytest

import golden_io as G

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.path.join(REPO, "oracle", "_ref")

BONDC = ["sq_bondc_p60", "sq_bondc_p60_pbc", "tri_bondc_p35"]
BOND_COND = ["sq_bond_cond_3t", "tri_bond_cond"]


def run(name, tmp_path):
    exe = os.path.join(REF, "nr_" + name)
    if not os.path.exists(exe):
        pytest.skip("NR drop-in binaries not built (oracle/build_ref.sh needs /root/reference)")
    r = subprocess.run([exe], cwd=tmp_path, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    return r


@pytest.mark.gpu
@pytest.mark.parametrize("v", BONDC)
def test_reference_bondc_on_libperc(v, tmp_path):
    r = run(v, tmp_path)
    md = G.meta(v)
    for f in ("bondorder.txt", "bond.txt"):
        assert (tmp_path / f).read_bytes() == G.text(v, f), f
    line = [l for l in r.stdout.splitlines() if "Conductance:" in l][-1]
    gtop, gbot = (float(x) for x in line.split(":")[1].split())
    assert abs(gtop - md["gtop"]) <= 1e-10 * md["gtop"]
    assert abs(gbot - md["gbot"]) <= 1e-6 * md["gbot"]


@pytest.mark.gpu
@pytest.mark.parametrize("v", BOND_COND)
def test_reference_bond_cond_on_libperc(v, tmp_path):
    run(v, tmp_path)
    got = (tmp_path / "bondcond.txt").read_text().splitlines()
    want = G.text(v, "bondcond.txt").decode().splitlines()
    assert len(got) == len(want)
    for a, b in zip(got, want):
        if b.count(",") == 3:
            assert a.split(",")[0] == b.split(",")[0]
            fa, fb = [float(x) for x in a.split(",")], [float(x) for x in b.split(",")]
            assert all(abs(x - y) <= 2e-9 for x, y in zip(fa[1:], fb[1:])), (a, b)
        else:
            assert a == b
