"""Setup time with the Galerkin products on the host vs on the GPU, and a
bit-for-bit comparison of the two hierarchies. One JSON line.

    python tools/setup_bench.py --kind poisson3d --grid 256 [--no-host]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kind", default="poisson3d")
    ap.add_argument("--grid", type=int, default=256)
    ap.add_argument("--no-host", action="store_true")
    args = ap.parse_args()
    import parallel_amg_amd as pa
    from parallel_amg_amd import hierarchy as HH
    from parallel_amg_amd.partitioned import Context

    ctx = Context(0)
    be = pa.SequentialBackend(1)
    t = time.time()
    A, offs, _ = pa.generate_problem(be, args.kind, args.grid)
    t_gen = time.time() - t
    phases = {}

    def timed(mod, name):
        f = getattr(mod, name)

        def g(*a, **k):
            t0 = time.time()
            r = f(*a, **k)
            key = name + ("_dev" if k.get("device") is not None else "")
            phases[key] = phases.get(key, 0.0) + time.time() - t0
            return r
        setattr(mod, name, g)
    for n in ("gershgorin", "aggregate", "tentative", "spgemm", "smooth", "transpose", "cholinv"):
        timed(HH.H, n)
    out = {"kind": args.kind, "grid": args.grid, "gen_s": round(t_gen, 2)}
    t = time.time()
    Hd = pa.build_hierarchy(be, A, offs, pa.SAParams(), device=ctx)
    out["gpu_setup_s"] = round(time.time() - t, 2)
    out["levels"] = Hd.nlevels
    if not args.no_host:
        t = time.time()
        Hh = pa.build_hierarchy(be, A, offs, pa.SAParams())
        out["host_setup_s"] = round(time.time() - t, 2)
        ok = True
        for l in range(Hd.nlevels):
            d, h = Hd.levels[l][0], Hh.levels[l][0]
            for w in ("A", "P", "R"):
                x, y = getattr(d, w), getattr(h, w)
                if x is None:
                    continue
                ok &= bool(np.array_equal(x.rowptr, y.rowptr) and np.array_equal(x.col, y.col)
                           and np.array_equal(x.val.view(np.int64), y.val.view(np.int64)))
        out["bit_identical"] = ok
    out["phases_s"] = {k: round(v, 2) for k, v in sorted(phases.items())}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
