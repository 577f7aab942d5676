"""One conductance solve split over the processes of a torch.distributed
group: row slab s of K on process s (the linbcg loop
of Square/bondc.f:780-836).  libperc runs the slab's kernels
(perc_dslab_*, include/perc.h); this module moves the two things that cross
processes each iteration -- the slabs' dot partials (an all-gather of 4
doubles per slab, reduced in slab order on every process, so all take the
same stop decision) and the halo rows of r (one row each way per
neighbour).

With the "nccl" backend (RCCL over xGMI) the buffers stay in device memory
and the collectives run on the context's own stream
(torch.cuda.ExternalStream of perc_stream): kernels and collectives are
ordered by the stream, the host only enqueues and checks the stop flag
every `check_every` iterations.  With "gloo" (tests: several processes on
one GPU) the same buffers are staged through host memory.

Every process labels and assembles the whole lattice (a few ms at the
sizes that need several GPUs); the solve is what is split.  The per-slab
kernels and the combine order are those of perc_set_slabs(K) in one
process, so K processes give its numbers bitwise.

`solve` is the production path: libperc runs the whole loop itself
(perc_dslab_solve over an RCCL communicator of its own, made once per
context from rank 0's unique id; the group only carries that id), so no
Python runs per iteration.  `conductance` keeps the loop in Python over the
group's own backend -- the gloo test transport for several processes on one
GPU, which one RCCL communicator cannot hold.
"""
import ctypes as C

import torch
import torch.distributed as dist

from . import _lib as L

LEAK = 1.0e-12


class _Exchange:
    """all-gather of the partials and halo swap, on device (nccl) or staged
    through the host (gloo)"""

    def __init__(self, group, K, s, part_out, part_all, edges, ghosts):
        self.g, self.K, self.s = group, K, s
        self.nccl = dist.get_backend(group) == "nccl"
        self.part_out, self.part_all = part_out, part_all
        self.edges, self.ghosts = edges, ghosts  # (lo, hi) each; None past the ends
        self.ranks = [dist.get_global_rank(group, r) if group is not None else r for r in range(K)]

    def gather(self):
        if self.nccl:
            dist.all_gather_into_tensor(self.part_all, self.part_out, group=self.g)
            return
        po = self.part_out.cpu()
        parts = [torch.empty_like(po) for _ in range(self.K)]
        dist.all_gather(parts, po, group=self.g)
        self.part_all.copy_(torch.cat(parts))

    def halo(self):
        if self.K == 1:
            return
        nb = [(self.s - 1, 0), (self.s + 1, 1)]  # (neighbour slab, my side)
        if self.nccl:
            ops = []
            for q, side in nb:
                if 0 <= q < self.K:
                    ops.append(dist.P2POp(dist.isend, self.edges[side], self.ranks[q], self.g))
                    ops.append(dist.P2POp(dist.irecv, self.ghosts[side], self.ranks[q], self.g))
            for r in dist.batch_isend_irecv(ops):
                r.wait()
            return
        send = {side: self.edges[side].cpu() for q, side in nb if 0 <= q < self.K}
        recv = {side: torch.empty_like(send[side]) for side in send}
        reqs = []
        for q, side in nb:
            if 0 <= q < self.K:
                reqs.append(dist.isend(send[side], self.ranks[q], group=self.g))
                reqs.append(dist.irecv(recv[side], self.ranks[q], group=self.g))
        for r in reqs:
            r.wait()
        for side, t in recv.items():
            self.ghosts[side].copy_(t)


def conductance(ctx, rule=L.RULE_BOND, cur_rule=L.CUR_FORTRAN, Va=1.0, g0=1.0, leak=LEAK,
                itol=2, tol=1e-8, itmax=2500, full_x=False, group=None, check_every=64):
    """Gtop / Gbot of the labeled context's spanning cluster, the linbcg solve
    split over the group's processes (ctx labeled identically on every
    process, each on its own GPU).  Returns the perc_conductance fields on
    every process."""
    lib = L.lib()
    K, s = dist.get_world_size(group), dist.get_rank(group)
    span = C.c_int()
    L.check(lib.perc_assemble(ctx.h, rule, g0, leak, Va, C.byref(span)), "perc_assemble")
    if not span.value:
        return dict(gtop=0.0, gbot=0.0, err=0.0, iter=0, status=1)
    dev = torch.device("cuda", ctx.device)
    m, nrows = ctx.m, ctx.n - 2
    z = lambda n: torch.zeros(n, dtype=torch.float64, device=dev)  # noqa: E731
    part_out, part_all = z(4), z(4 * K)
    edges = (z(m) if s > 0 else None, z(m) if s < K - 1 else None)
    ghosts = (z(m) if s > 0 else None, z(m) if s < K - 1 else None)
    ptr = lambda t: None if t is None else t.data_ptr()  # noqa: E731
    bufs = L.DslabBufs(ptr(part_out), ptr(part_all), ptr(edges[0]), ptr(edges[1]),
                       ptr(ghosts[0]), ptr(ghosts[1]))
    ex = _Exchange(group, K, s, part_out, part_all, edges, ghosts)
    # every tensor the loop touches is allocated here, on the current stream:
    # a block the caching allocator assigned to the context's stream would
    # outlive that stream (perc_ctx_destroy) in the allocator's pools
    row = z(m) if K > 1 and s in (0, K - 1) else None
    out_dev = z(4)
    stream = torch.cuda.ExternalStream(lib.perc_stream(ctx.h), device=dev)
    step = lambda op: L.check(lib.perc_dslab_step(ctx.h, op), "perc_dslab_step")  # noqa: E731
    it, err, done = C.c_int(), C.c_double(), C.c_int()
    with torch.cuda.device(dev), torch.cuda.stream(stream):
        L.check(lib.perc_dslab_begin(ctx.h, K, s, itol, tol, itmax, int(full_x), C.byref(bufs)),
                "perc_dslab_begin")
        ex.gather()
        ex.halo()
        step(L.DSLAB_COMBINE_INIT)
        step(L.DSLAB_GHOSTS)
        k = 0
        while True:
            step(L.DSLAB_PS)
            ex.gather()
            step(L.DSLAB_COMBINE_PS)
            step(L.DSLAB_B)
            ex.gather()
            step(L.DSLAB_COMBINE_B)
            ex.halo()
            step(L.DSLAB_GHOSTS)
            k += 1
            if k % check_every == 0 or k > itmax:
                L.check(lib.perc_dslab_status(ctx.h, C.byref(it), C.byref(err), C.byref(done)),
                        "perc_dslab_status")
                if done.value:
                    break
        L.check(lib.perc_dslab_end(ctx.h), "perc_dslab_end")
        # the top electrode row's voltages to slab 0's process, which holds
        # the bottom one: the currents there
        out = torch.zeros(4, dtype=torch.float64)
        if K > 1 and s in (0, K - 1):
            if s == K - 1:
                L.check(lib.perc_x_row(ctx.h, nrows - 1, row.data_ptr(), 0), "perc_x_row")
                dist.send(row if ex.nccl else row.cpu(), ex.ranks[0], group=group)
            else:
                buf = row if ex.nccl else torch.empty(m, dtype=torch.float64)
                dist.recv(buf, ex.ranks[K - 1], group=group)
                row.copy_(buf)
                torch.cuda.current_stream().synchronize()
                L.check(lib.perc_x_row(ctx.h, nrows - 1, row.data_ptr(), 1), "perc_x_row")
        if s == 0:
            res = L.CondResult()
            L.check(lib.perc_currents(ctx.h, rule, cur_rule, Va, g0, leak, C.byref(res)),
                    "perc_currents")
            out[:] = torch.tensor([res.gtop, res.gbot, err.value, float(it.value)],
                                  dtype=torch.float64)
        if ex.nccl:
            out_dev.copy_(out)
            dist.broadcast(out_dev, ex.ranks[0], group=group)
            out = out_dev.cpu()
        else:
            dist.broadcast(out, ex.ranks[0], group=group)
        torch.cuda.current_stream().synchronize()
    return dict(gtop=float(out[0]), gbot=float(out[1]), err=float(out[2]), iter=int(out[3]),
                status=0)


def solve(ctx, rule=L.RULE_BOND, cur_rule=L.CUR_FORTRAN, Va=1.0, g0=1.0, leak=LEAK, itol=2,
          tol=1e-8, itmax=2500, full_x=False, group=None):
    """`conductance` with the loop inside libperc (perc_dslab_solve): the
    group's processes, one GPU each, bind their contexts to slab s of K on
    the first call (rank 0's RCCL unique id broadcast over the group), then
    every iteration's all-gathers and halos run on the context's stream
    with no host round trip.  Returns the perc_conductance fields on every
    process."""
    lib = L.lib()
    K, s = dist.get_world_size(group), dist.get_rank(group)
    # the communicator belongs to this group: keyed on its members and its
    # identity too, so another group of the same size and rank makes (and
    # perc_dslab_comm_init's release of the old one frees) a new one
    ranks = tuple(dist.get_process_group_ranks(group)) if group is not None else tuple(range(K))
    key = (K, s, ranks, id(group) if group is not None else None)
    if getattr(ctx, "_dslab_rank", None) != key:
        uid = C.create_string_buffer(L.DSLAB_ID_BYTES)
        if s == 0:
            L.check(lib.perc_dslab_unique_id(uid, L.DSLAB_ID_BYTES), "perc_dslab_unique_id")
        box = [uid.raw]
        dist.broadcast_object_list(box, src=dist.get_global_rank(group, 0) if group is not None else 0,
                                   group=group)
        uid = C.create_string_buffer(box[0], L.DSLAB_ID_BYTES)
        L.check(lib.perc_dslab_comm_init(ctx.h, K, s, uid, L.DSLAB_ID_BYTES), "perc_dslab_comm_init")
        ctx._dslab_rank = key
    res = L.CondResult()
    L.check(lib.perc_dslab_solve(ctx.h, rule, cur_rule, Va, g0, leak, itol, tol, itmax, int(full_x),
                                 C.byref(res)), "perc_dslab_solve")
    return {k: getattr(res, k) for k, _ in L.CondResult._fields_}
