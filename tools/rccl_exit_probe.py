#!/usr/bin/env python3
"""Which combination of torch.distributed "nccl" (torch's bundled RCCL) and
libperc (linked against /opt/rocm's RCCL) ends a process abnormally?  Each
case runs in a child process of its own (world size 1) and reports its exit
status; a case prints "done" before returning from main.  The probe stops
at the first case that does not exit cleanly and exits 3 (nothing more is
started on the GPU after an abnormal exit); the cases run from the plainest
(torch alone) to the most combined.

  python tools/rccl_exit_probe.py
"""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

CASES = {
    "torch_devid": dict(lib=False, devid=True, destroy=True, perc_rccl=False),
    "torch_lazy": dict(lib=False, devid=False, destroy=True, perc_rccl=False),
    "lib_devid": dict(lib=True, devid=True, destroy=True, perc_rccl=False),
    "lib_lazy": dict(lib=True, devid=False, destroy=True, perc_rccl=False),
    "lib_devid_nodestroy": dict(lib=True, devid=True, destroy=False, perc_rccl=False),
    "lib_rccl_then_torch": dict(lib=True, devid=True, destroy=True, perc_rccl=True),
    # a collective on the context's own stream (torch.cuda.ExternalStream), the context closed
    # before the group is destroyed; then the Python row-slab loop (dslab.conductance) the same way
    "extstream_allreduce": dict(lib=True, devid=True, destroy=True, perc_rccl=False, ext="allreduce"),
    "dslab_conductance": dict(lib=True, devid=True, destroy=True, perc_rccl=False, ext="dslab"),
}


def child(name):
    c = CASES[name]
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", str(29600 + list(CASES).index(name)))
    import torch
    import torch.distributed as dist
    if c["lib"]:
        from percolation_amd import _lib as PL
        from percolation_amd import api
        PL.lib()
        if c["perc_rccl"]:  # libperc's own communicator (group solve over RCCL, exchange forced)
            with api.Context(0, 128, 128, 0) as ctx:
                ctx.occupy_random(PL.BOND, 0, int(0.6 * api.nbonds(0, 128, 128, 0)), 7)
                ctx.label()
                api.dslab_solve_group([ctx], xport=PL.XPORT_RCCL | PL.XPORT_EXCHANGE, tol=1e-8, itmax=1000)
    kw = dict(device_id=torch.device("cuda", 0)) if c["devid"] else {}
    dist.init_process_group("nccl", rank=0, world_size=1, **kw)
    t = torch.ones(4, device="cuda")
    dist.all_reduce(t)
    torch.cuda.synchronize()
    if c.get("ext"):
        from percolation_amd import dslab
        ctx = api.Context(0, 256, 256, 0)
        ctx.occupy_random(PL.BOND, 0, int(0.6 * api.nbonds(0, 256, 256, 0)), 7)
        ctx.label()
        if c["ext"] == "allreduce":
            st = torch.cuda.ExternalStream(PL.lib().perc_stream(ctx.h), device=torch.device("cuda", 0))
            with torch.cuda.stream(st):
                dist.all_reduce(t)
            torch.cuda.synchronize()
        else:
            dslab.conductance(ctx, tol=1e-8, itmax=10000)
        ctx.close()
        print("context closed", flush=True)
    if c["destroy"]:
        dist.destroy_process_group()
    print("done", flush=True)


def main():
    if len(sys.argv) > 2 and sys.argv[1] == "--child":
        return child(sys.argv[2])
    out = {}
    for name in CASES:
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", name],
                           capture_output=True, text=True, timeout=180)
        out[name] = dict(rc=r.returncode, done="done" in r.stdout,
                         tail=(r.stderr.strip().splitlines() or [""])[-1][-160:])
        print(name, json.dumps(out[name]), flush=True)
        if r.returncode != 0:
            break
    print(json.dumps(out), flush=True)
    return 3 if any(v["rc"] != 0 for v in out.values()) else 0


if __name__ == "__main__":
    sys.exit(main())
