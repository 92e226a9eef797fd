#!/usr/bin/env python3
"""A/B sweep of classify launch variants in ONE process (interleaved rounds, median).

Every combination of the --tune lists (pg_set_tuning keys) classifies the same
device-resident workload; outputs are compared for equality against the first variant. To
compare builds (e.g. ``make -C vpp_amd/csrc variant V=pf2 DEFS=-DPG_PREFETCH=2``), run the
sweep once per build with VPP_AMD_LIB=vpp_amd/libpolicygpu_pf2.so; the "lib" field names it.

    python tools/sweep.py --config 3 --tune block_stage=256,512,1024 --tune blocks_per_cu=0,2
"""
import argparse
import ctypes as C
import itertools
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vpp_amd import _capi, device as D, workloads as W  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--tuples", type=int, default=0)
    ap.add_argument("--tune", action="append", default=[], help="key=v1,v2,...")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=60, help="untimed launches before the first round")
    ap.add_argument("--counters", action="store_true", help="classify with per-rule hit counters")
    ap.add_argument("--pre", action="append", default=[], help="key=v set before the tables are compiled")
    ap.add_argument("--ns", type=int, default=0, help="configs 3/5: namespaces (default 10)")
    ap.add_argument("--rules", type=int, default=0, help="config 2: rules of the gen-policy-shaped table")
    ap.add_argument("--mode", type=int, default=-1, help="cluster configs: classify in this mode (2 = CONN)")
    a = ap.parse_args()
    kw = {"n_tuples": a.tuples} if a.tuples else {}
    if a.rules:
        kw["n_rules"] = a.rules
    if a.ns:
        kw["n_ns"] = a.ns
    for t in a.pre:
        k, v = t.split("=")
        assert _capi.lib.pg_set_tuning(k.encode(), int(v)) == 0, t
    w = W.CONFIGS[a.config](0, **kw)
    e, n = w.engine, w.n_tuples
    if a.mode >= 0:
        w.mode = a.mode
    b = D.TupleBatch(n, with_sport=(w.mode == 2))
    D.gen_tuples(e, b, **w.gen)
    keys, vals = [], []
    for t in a.tune:
        k, v = t.split("=")
        keys.append(k)
        vals.append([int(x) for x in v.split(",")])
    combos = list(itertools.product(*vals)) if keys else [()]
    lib = _capi.lib
    outs = [torch.empty(n, dtype=torch.int32, device="cuda") for _ in combos]
    cnt = torch.zeros(e.num_counter_slots(), dtype=torch.int64, device="cuda") if a.counters else None
    cptr = cnt.data_ptr() if a.counters else None
    soa = b.soa()
    stream = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    times = {i: [] for i in range(len(combos))}
    # the first ~50 launches after the batch is generated run slower: warm up
    for _ in range(a.warmup):
        lib.pg_classify(e.h, w.mode, w.table_id, C.byref(soa), n, outs[0].data_ptr(), cptr, stream)
    torch.cuda.synchronize()
    for r in range(a.rounds):
        for i, combo in enumerate(combos):
            for k, v in zip(keys, combo):
                e.set_tuning(k, v)
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            lib.pg_classify(e.h, w.mode, w.table_id, C.byref(soa), n, outs[i].data_ptr(), cptr, stream)  # warm
            ev0.record()
            for _ in range(a.reps):
                assert lib.pg_classify(e.h, w.mode, w.table_id, C.byref(soa), n, outs[i].data_ptr(), cptr,
                                       stream) == 0
            ev1.record()
            torch.cuda.synchronize()
            times[i].append(ev0.elapsed_time(ev1) / a.reps)
    ref = outs[0]
    bpt = 17 if w.mode == 2 else 15
    name = os.path.basename(os.environ.get("VPP_AMD_LIB", "libpolicygpu.so"))
    for i, combo in enumerate(combos):
        ms = float(np.median(times[i]))
        extra = {"blob": e.table_stats(w.table_id)} if w.mode == 0 and i == 0 else {}
        print(json.dumps({"lib": name, "config": a.config if a.mode < 0 else "%dm%d" % (a.config, a.mode), "counters": a.counters, "pre": a.pre, "ns": a.ns, "rules": a.rules, **dict(zip(keys, combo)), "ms": round(ms, 4),
                          "gpps": round(n / ms / 1e6, 1), "GBps": round(n * bpt / ms / 1e6, 1),
                          "same_output": bool(torch.equal(outs[i], ref)),
                          "out_sha": __import__("hashlib").sha1(outs[i].cpu().numpy().tobytes()).hexdigest()[:12],
                          **extra}), flush=True)


if __name__ == "__main__":
    main()
