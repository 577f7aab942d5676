import os, sys
sys.path.insert(0, '.'); sys.path.insert(0, 'tests')
import numpy as np
import percolation_amd as P
from percolation_amd import api, _lib as PL
lat, m, n, pbc, p, seed = 0, int(sys.argv[1]), int(sys.argv[1]), 0, 0.6, 1
b1, b2 = api.bond_list(lat, m, n, pbc); nb = len(b1)
order = api.shuffled_ids(nb, seed); tb = int(p * nb)
ctx = api.Context(lat, m, n, pbc)
ctx.occupy(PL.BOND, bond_order=order, nbonds_=tb)
li = ctx.label(); print('label', li, flush=True)
s = ctx.system(); print('pattern rowptr', s['rowptr'][:5], s['rowptr'][-1], 'col range', s['col'].min(), s['col'].max(), flush=True)
c = ctx.conductance(itmax=int(sys.argv[2]))
print('cond', c, flush=True)
s = ctx.system()
print('diag min/max', s['diag'].min(), s['diag'].max(), 'val uniq', np.unique(s['val'])[:5], 'rhs nz', np.count_nonzero(s['rhs']), flush=True)
