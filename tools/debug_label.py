import sys, os
sys.path.insert(0, '.'); sys.path.insert(0, 'tests')
import numpy as np
import percolation_amd as P
from percolation_amd import api, _lib as PL
from test_gpu_parity import oracle_canon_bonds
for (lat, m, n, pbc, p, seed) in [(0, 8, 8, 0, 1.0, 1), (0, 8, 8, 0, 0.5, 1), (0, 64, 64, 0, 0.5, 1)]:
    b1, b2 = api.bond_list(lat, m, n, pbc); nb = len(b1)
    order = api.shuffled_ids(nb, seed); tb = int(p * nb)
    with api.Context(lat, m, n, pbc) as ctx:
        ctx.occupy(PL.BOND, bond_order=order, nbonds_=tb)
        li = ctx.label(canon=True)
    ref = api.replay_labels(lat, m, n, pbc, PL.BOND, bond_order=order, nbond=tb)
    want = oracle_canon_bonds(b1, b2, ref["bond_label"], m * n)
    got = li["canon"].astype(np.int64)
    d = np.nonzero(got != want)[0]
    print((lat, m, n, p), {k: v for k, v in li.items() if k != 'canon'}, 'ndiff', len(d))
    if m <= 8:
        print(got.reshape(n, m)); print(want.reshape(n, m))
    else:
        print('first diffs (site, got, want):', [(int(i + 1), int(got[i]), int(want[i])) for i in d[:10]])
        print('unique got roots among diffs', np.unique(got[d])[:10], 'want', np.unique(want[d])[:10])
