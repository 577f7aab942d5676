#!/usr/bin/env python3
"""Where does the literal dot order leave the oracle's literal linbcg at a
config size?  Runs the GPU literal solve of a config fixture's realisation
for a fixed number of iterations (tol 1e-300) and saves its per-iteration
err history (gpurun_out/literal_probe_<case>_<mode>.npy), electrode-row x
(default) and full voltages (vint); the CPU oracle's history of the same
system is compared off the GPU box.

  python tools/literal_probe.py c2_sq1024_bond_p50 4000
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

import numpy as np  # noqa: E402

from percolation_amd import _lib as PL  # noqa: E402
from percolation_amd import api  # noqa: E402
from test_config_goldens import occupation  # noqa: E402


def main():
    case, iters = sys.argv[1], int(sys.argv[2])
    doc = json.load(open(os.path.join(REPO, "tests", "golden", "configs", case + ".json")))
    rc = doc["recipe"]
    occ, rule, cur = occupation(rc)
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    with api.Context(rc["lattice"], rc["L"], rc["L"], 0) as ctx:
        ctx.occupy(**occ)
        assert ctx.label()["nspan"] > 0
        ctx.set_dot_order(PL.DOT_LITERAL)
        for mode, vint in (("rows", False), ("vint", True)):
            c = ctx.conductance(rule, cur, tol=1e-300, itmax=iters, vint=vint)
            h = ctx.err_history()[:c["iter"]]
            np.save(os.path.join(REPO, "gpurun_out", "literal_probe_%s_%s.npy" % (case, mode)), h)
            print(json.dumps(dict(mode=mode, iter=c["iter"], err=repr(c["err"]), gtop=repr(c["gtop"]),
                                  info=ctx.march_info())), flush=True)


if __name__ == "__main__":
    main()
