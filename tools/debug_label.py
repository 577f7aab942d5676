import sys, os, subprocess
sys.path.insert(0, '.'); sys.path.insert(0, 'tests')
if len(sys.argv) == 1:
    for v in ['0', '2', '3', '4']:
        env = dict(os.environ, PERC_CC_VARIANT=v)
        print('variant', v, flush=True)
        subprocess.run([sys.executable, __file__, 'x'], env=env)
    sys.exit()
import numpy as np
import percolation_amd as P
from percolation_amd import api, _lib as PL
from test_gpu_parity import oracle_canon_bonds
for (lat, m, n, pbc, p, seed) in [(0, 64, 64, 0, 0.5, 1), (0, 256, 256, 0, 0.6, 2)]:
    b1, b2 = api.bond_list(lat, m, n, pbc); nb = len(b1)
    order = api.shuffled_ids(nb, seed); tb = int(p * nb)
    with api.Context(lat, m, n, pbc) as ctx:
        ctx.occupy(PL.BOND, bond_order=order, nbonds_=tb)
        li = ctx.label(canon=True)
    ref = api.replay_labels(lat, m, n, pbc, PL.BOND, bond_order=order, nbond=tb)
    want = oracle_canon_bonds(b1, b2, ref["bond_label"], m * n)
    got = li["canon"].astype(np.int64)
    d = np.nonzero(got != want)[0]
    print((lat, m, n, p), li['nspan'], 'ndiff', len(d), flush=True)
