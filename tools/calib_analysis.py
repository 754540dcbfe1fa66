#!/usr/bin/env python3
"""Counter calibration: turn the rocprofv3 passes of tools/gpu_steps.sh
``calib`` into per-access-width factors and physical traffic figures.

Input: OUT/cal1..cal4 (passes over tools/fetch_calib: known-byte kernels, one launch each, in
the order of OUT/cal*.jsonl) and OUT/kb1..kb4 (the same passes over tools/kbench.py's row
kernels). Passes: 1 FETCH_SIZE; 2 WRITE_SIZE; 3 TCC_EA0_RDREQ / _32B / _64B / _128B; 4
TCC_EA0_WRREQ / _64B, TCC_EA0_RDREQ_DRAM / _DRAM_32B.

For each known-byte kernel: every counter-derived byte figure over the bytes it must move
(useful bytes, or the 64-B / 128-B segments a strided read touches). For each row kernel: the
same figures, the candidate read formulas side by side, and the one the calibration supports
("read_bytes", see ``choose``) plus the writes. Prints one JSON document.

    python tools/calib_analysis.py gpurun_out/TAG > calib.json
"""
import collections
import csv
import glob
import json
import os
import re
import sys


def rows_of(d):
    out = []
    for f in sorted(glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)):
        out += list(csv.DictReader(open(f)))
    return out


def short(name):
    name = name.replace("pamg::(anonymous namespace)::", "").replace("void ", "")
    return re.sub(r"\(.*", "", name)


def per_dispatch(d):
    """{dispatch id: (kernel, blocks, {counter: value})} of one pass (values summed over the
    counter's instances, as rocprofv3 reports one row per counter and dispatch)."""
    disp = {}
    for r in rows_of(d):
        k = int(r["Dispatch_Id"])
        name = short(r["Kernel_Name"])
        blocks = int(r["Grid_Size"]) // max(1, int(r["Workgroup_Size"]))
        e = disp.setdefault(k, (name, blocks, {}))
        e[2][r["Counter_Name"]] = e[2].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return disp


def figures(c):
    """Byte figures from whatever counters a merged record holds."""
    f = {}
    if "FETCH_SIZE" in c:
        f["fetch_kib_x1024"] = c["FETCH_SIZE"] * 1024.0
        f["fetch_x2"] = 2.0 * c["FETCH_SIZE"] * 1024.0
    if "WRITE_SIZE" in c:
        f["write"] = c["WRITE_SIZE"] * 1024.0
    g = lambda k: c.get(k + "_sum", c.get(k))  # noqa: E731
    n, n32, n64, n128 = g("TCC_EA0_RDREQ"), g("TCC_EA0_RDREQ_32B"), g("TCC_EA0_RDREQ_64B"), g("TCC_EA0_RDREQ_128B")
    if None not in (n, n32, n64, n128):
        f["rdreq"] = n
        f["rdreq_x64"] = 64.0 * n
        f["rd_by_size"] = 32.0 * n32 + 64.0 * n64 + 128.0 * n128
        # if the size counters partition the requests (a request counted once, in its size)
        f["rd_sizes_cover"] = (n32 + n64 + n128) / n if n else None
        f["rd_32_64_128_frac"] = [round(v / n, 4) if n else None for v in (n32, n64, n128)]
    w, w64 = g("TCC_EA0_WRREQ"), g("TCC_EA0_WRREQ_64B")
    if None not in (w, w64):
        f["wr_by_size"] = 32.0 * (w - w64) + 64.0 * w64
    d, d32 = g("TCC_EA0_RDREQ_DRAM"), g("TCC_EA0_RDREQ_DRAM_32B")
    if None not in (d, d32):
        f["dram_rdreq"] = d
        f["dram_rd_x64"] = 64.0 * d
        f["dram_rd_by_size"] = 32.0 * d32 + 64.0 * (d - d32)
    return f


def known_kernels(out):
    """Merge the four passes over tools/fetch_calib, launch by launch (the flushes excluded)."""
    names = [json.loads(l) for l in open(os.path.join(out, "cal1.jsonl")) if l.startswith("{")]
    merged = [dict(n, counters={}) for n in names]
    for p in range(1, 5):
        d = os.path.join(out, f"cal{p}")
        if not os.path.isdir(d):
            continue
        disp = per_dispatch(d)
        # the measured kernels in launch order (not the flushes, nor the runtime's memset / copy kernels)
        launches = [disp[k] for k in sorted(disp) if disp[k][0].startswith("k_") and disp[k][0] != "k_flush"]
        for rec, (_nm, _b, c) in zip(merged, launches):
            rec["counters"].update(c)
    for rec in merged:
        f = figures(rec["counters"])
        rec["figures"] = f
        rec["ratio_to_bytes"] = {}
        want = rec["seg128_bytes"] if rec["kernel"].startswith("s8") else rec["useful_bytes"]
        for k, v in f.items():
            if isinstance(v, (int, float)) and k not in ("rdreq", "dram_rdreq", "rd_sizes_cover"):
                rec["ratio_to_bytes"][k] = round(v / want, 4) if want else None
    return merged


def choose(known):
    """The read formula whose ratio to the known bytes stays closest to 1 across the read
    kernels of every access width (coalesced 16/8/4/2/1 B and the scrambled 8-B gathers)."""
    reads = [r for r in known if r["kernel"] in ("r16", "r8", "r4", "r2", "r1", "g8")]
    best = None
    for k in ("fetch_x2", "fetch_kib_x1024", "rd_by_size", "rdreq_x64", "dram_rd_by_size", "dram_rd_x64"):
        rs = [r["ratio_to_bytes"].get(k) for r in reads]
        if not rs or None in rs:
            continue
        err = max(abs(x - 1.0) for x in rs)
        if best is None or err < best[1]:
            best = (k, err, rs)
    return {"formula": best[0], "max_abs_error": round(best[1], 4), "ratios": best[2]} if best else None


def row_kernels(out, formula):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for p in range(1, 5):
        d = os.path.join(out, f"kb{p}")
        if not os.path.isdir(d):
            continue
        for _k, (name, blocks, c) in per_dispatch(d).items():
            if not name.startswith("k_"):
                continue
            for cn, v in c.items():
                agg[(name, blocks)][cn].append(v)
    recs = []
    for (name, blocks), cs in sorted(agg.items()):
        c = {k: sum(v) / len(v) for k, v in cs.items()}
        f = figures(c)
        rec = {"kernel": name, "blocks": blocks, "figures": f}
        if formula and formula in f:
            rec["read_bytes"] = f[formula]
            wr = f.get("write", f.get("wr_by_size"))
            if wr is not None:
                rec["traffic_bytes"] = f[formula] + wr
        recs.append(rec)
    return recs


def main():
    out = sys.argv[1]
    known = known_kernels(out)
    ch = choose(known)
    print(json.dumps({"known_byte_kernels": known, "read_formula": ch,
                      "row_kernels": row_kernels(out, ch["formula"] if ch else None)}, indent=1))


if __name__ == "__main__":
    main()
