"""Multi-GPU ensemble inside libperc (perc_ensemble_*), exercised with the
devices of the box (ndev = 1 on a one-GPU box; the striping for 2-8
devices is covered on CPU by tests/test_ensemble_gloo.py):

* the RCCL communicator builds (ncclCommInitAll) and all-reduces;
* perc_ensemble_bond_cond gives the reference's bondcond.txt rows (goldens)
  and the single-context loop's numbers bitwise;
* the Fortran bond_cond driver with ndev = 1 writes the same bondcond.txt
  as with ndev = 0, and both match the goldens;
* torch.distributed's "nccl" backend (RCCL) all-reduces device tensors at
  world size 1 (the bench's path).
"""
import os
import socket
import subprocess

import numpy as np
import pytest

import golden_io as G
from percolation_amd import api

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(REPO, "percolation_amd", "fortran", "bin")
BOND_COND = [v for v in G.variants() if G.meta(v)["kind"] == "bond_cond"]


def golden_trials(v):
    want, cur = [], None
    for line in G.text(v, "bondcond.txt").decode().splitlines():
        if "Trial #" in line:
            cur = dict(rows=[])
            want.append(cur)
        elif cur is not None and line.count(",") == 3:
            cur["rows"].append([float(x) for x in line.split(",")])
        elif "lattice-spanning cluster:" in line:
            cur["perccln"] = int(line.split(":")[1])
        elif "pc =" in line:
            cur["pc"] = float(line.split("=")[1])
    return want


def test_ensemble_allreduce_rccl():
    with api.Ensemble(0, 16, 16, 0, ndev=1) as e:
        a = np.arange(12, dtype=np.float64).reshape(1, 12) * 0.5
        s = e.allreduce(a)
        assert np.array_equal(s, a)  # one device: the sum is its own vector


@pytest.mark.parametrize("v", BOND_COND)
def test_ensemble_bond_cond_equals_reference_and_serial(v):
    p = G.meta(v)["params"]
    with api.Ensemble(p["lattice"], p["m"], p["n"], p["pbc"], ndev=1) as e:
        res, stats = e.bond_cond(p["seed"], p["numtrials"])
    serial = api.bond_cond_grid(p["lattice"], p["m"], p["n"], p["pbc"], p["seed"], p["numtrials"])
    want = golden_trials(v)
    assert len(res) == len(want) == len(serial)
    for tr, w, s in zip(res, want, serial):
        assert len(tr["rows"]) == len(w["rows"]) == len(s["rows"])
        for r, wr, sr in zip(tr["rows"], w["rows"], s["rows"]):
            assert "%12.9f" % r["pb"] == "%12.9f" % wr[0]
            assert abs(r["gbot"] - wr[1]) <= 2e-9 and abs(r["gtop"] - wr[2]) <= 2e-9
            # same device kernels, same inputs: bitwise the single-context loop
            assert r["gtop"] == sr["gtop"] and r["gbot"] == sr["gbot"] and r["iter"] == sr["iter"]
        assert tr["pc"] == w["pc"] == s["pc"] and tr["perccln"] == w["perccln"]
    # statistics: count, sum G, sum G^2, spanning, sum iter per grid point
    rows = [r for tr in res for r in tr["rows"]]
    npts = max(len(tr["rows"]) for tr in res)
    for j in range(npts):
        rj = [tr["rows"][j] for tr in res if len(tr["rows"]) > j]
        assert stats[j, 0] == len(rj)
        assert stats[j, 1] == pytest.approx(sum(r["gtop"] for r in rj), rel=1e-15)
        assert stats[j, 4] == sum(r["iter"] for r in rj)
    assert stats[npts:, 0].sum() == 0 and len(rows) == stats[:, 0].sum()


@pytest.mark.parametrize("v", BOND_COND)
def test_fortran_bond_cond_ndev1_equals_single_context(v, tmp_path):
    p = G.meta(v)["params"]
    exe = os.path.join(BIN, "bond_cond_%s" % ("tri" if p["lattice"] else "sq"))
    if not os.path.exists(exe):
        pytest.skip("Fortran drivers not built")
    out = {}
    for ndev, workers in ((0, 1), (1, 1), (1, 3)):
        d = tmp_path / ("ndev%d_w%d" % (ndev, workers))
        d.mkdir()
        (d / "bond_cond.nml").write_text(
            "&bond_cond_nml lattice=%d, m=%d, n=%d, pbc=%d, numtrials=%d, seed=%d, ndev=%d, "
            "workers=%d /\n"
            % (p["lattice"], p["m"], p["n"], p["pbc"], p["numtrials"], p["seed"], ndev, workers))
        r = subprocess.run([exe], cwd=d, capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-2000:]
        out[ndev, workers] = (d / "bondcond.txt").read_bytes()
    # one device, one or three trials at a time: the serial loop's file
    assert out[1, 1] == out[0, 1] and out[1, 3] == out[0, 1]
    stats = (tmp_path / "ndev1_w1" / "bondcond_stats.txt").read_text().splitlines()
    assert stats[0] == "devices: 1" and len(stats) > 1
    want = G.text(v, "bondcond.txt").decode().splitlines()
    got = out[1, 1].decode().splitlines()
    assert len(got) == len(want)
    for a, b in zip(got, want):
        if b.count(",") == 3:
            fa, fb = [float(x) for x in a.split(",")], [float(x) for x in b.split(",")]
            assert a.split(",")[0] == b.split(",")[0]
            assert all(abs(x - y) <= 2e-9 for x, y in zip(fa[1:], fb[1:])), (a, b)
        else:
            assert a == b


def test_ensemble_workers_same_trials():
    """perc_ensemble_set_workers: W contexts per device run the trials
    concurrently; every trial's rows are bitwise those of one worker, the
    statistics the same sums up to their association over the workers."""
    out = {}
    for W in (1, 3, 4):
        with api.Ensemble(0, 24, 24, 0, ndev=1, workers=W) as e:
            assert e.workers == W
            out[W] = e.bond_cond(58302, 11)
    (r1, s1) = out[1]
    for W in (3, 4):
        rw, sw = out[W]
        assert len(rw) == len(r1) == 11
        for a, b in zip(rw, r1):
            assert a["rows"] == b["rows"] and a["bf_c"] == b["bf_c"] and a["perccln"] == b["perccln"]
        assert np.array_equal(sw[:, [0, 3, 4]], s1[:, [0, 3, 4]])
        assert np.allclose(sw[:, 1:3], s1[:, 1:3], rtol=1e-13, atol=0)


def test_torch_nccl_group_world1(tmp_path):
    """bench.py's collective: the "nccl" (RCCL) process group at world size 1
    all-reduces device tensors (run in a child process so the group does not
    outlive the test)."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    code = r"""
import os, torch, torch.distributed as dist
os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT="%d")
torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=0, world_size=1)
import sys; sys.path.insert(0, %r)
from percolation_amd import ensemble
st, el = ensemble.allreduce([1.0, 0.25, 0.0625, 1.0, 7.0], 3.5, device="cuda:0")
t = torch.arange(8, dtype=torch.float64, device="cuda:0")
dist.all_reduce(t)
assert t.cpu().tolist() == list(map(float, range(8)))
assert st.tolist() == [1.0, 0.25, 0.0625, 1.0, 7.0] and el == 3.5
dist.destroy_process_group()
print("NCCL_OK")
""" % (port, REPO)
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run(["python", "-c", code], capture_output=True, text=True, timeout=240,
                       env=env)
    assert r.returncode == 0 and "NCCL_OK" in r.stdout, r.stderr[-3000:]
