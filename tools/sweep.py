#!/usr/bin/env python3
"""A/B sweep of classify-kernel launch variants in ONE process (interleaved rounds, median).

Variants: grid size (blocks per CU), LDS staging on/off, and an alternate build of the
library (e.g. the non-temporal stream policy, ``make -C vpp_amd/csrc nt``) loaded side by
side. Every variant classifies the same device-resident workload; outputs are compared for
equality against the first variant.

    python tools/sweep.py --config 2 --bpc 2,4,8,16 --stage 0,1 [--alt vpp_amd/libpolicygpu_nt.so]
        [--root 8,12]
"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vpp_amd import _capi, device as D, renderer as R, workloads as W  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--tuples", type=int, default=0)
    ap.add_argument("--bpc", default="0,2,4,8", help="0 = occupancy-sized grid")
    ap.add_argument("--stage", default="1")
    ap.add_argument("--alt", default="")
    ap.add_argument("--root", default="", help="extra contexts with these trie root caps, e.g. 8,12")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    kw = {"n_tuples": a.tuples} if a.tuples else {}
    w = W.CONFIGS[a.config](0, **kw)
    e, n = w.engine, w.n_tuples
    b = D.TupleBatch(n, with_sport=(w.mode == 2))
    D.gen_tuples(e, b, **w.gen)
    names = e.ACLNames()
    keep = []
    ops = (_capi.pg_acl_op * len(names))()
    for i, nm in enumerate(names):
        acl = e.GetACLByName(nm)
        ops[i].key = ("config/vpp/acls/v2/acl/" + nm).encode()
        st = R._acl_struct(acl, keep)
        keep.append(st)
        ops[i].value = C.pointer(st)

    def clone(lib, root_bits):
        """Same ACLs in a fresh context of `lib`, tables compiled with the given root cap."""
        assert lib.pg_set_tuning(b"root_bits_max", root_bits) == 0
        h2 = lib.pg_create(0)
        assert lib.pg_apply_txn(h2, 1, ops, len(names)) == 0
        assert lib.pg_sync_tables(h2) == 0
        return h2, lib.pg_table_id(h2, names[w.table_id].encode())

    libs = [("main", _capi.lib, e.h, w.table_id)]
    if a.alt:
        alt = _capi.load(a.alt)
        libs.append(("alt", alt) + clone(alt, 16))
    for rb in [int(x) for x in a.root.split(",") if x]:
        for name, lib in list({(n_, l_) for n_, l_, _, _ in libs}):
            libs.append((f"{name}/root{rb}", lib) + clone(lib, rb))
    variants = []
    for name, lib, h, tid in libs:
        for bpc in [int(x) for x in a.bpc.split(",")]:
            for stage in [int(x) for x in a.stage.split(",")]:
                variants.append((name, lib, h, tid, bpc, stage))
    outs = [torch.empty(n, dtype=torch.int32, device="cuda") for _ in variants]
    soa = b.soa()
    stream = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    times = {i: [] for i in range(len(variants))}
    for r in range(a.rounds):
        for i, (name, lib, h, tid, bpc, stage) in enumerate(variants):
            lib.pg_set_tuning(b"blocks_per_cu", bpc)
            lib.pg_set_tuning(b"stage_max_words", 16384 if stage else 0)
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            lib.pg_classify(h, w.mode, tid, C.byref(soa), n, outs[i].data_ptr(), None, stream)  # warm
            ev0.record()
            for _ in range(a.reps):
                assert lib.pg_classify(h, w.mode, tid, C.byref(soa), n, outs[i].data_ptr(), None, stream) == 0
            ev1.record()
            torch.cuda.synchronize()
            times[i].append(ev0.elapsed_time(ev1) / a.reps)
    ref = outs[0]
    bpt = 17 if w.mode == 2 else 15
    res = []
    for i, v in enumerate(variants):
        ms = float(np.median(times[i]))
        res.append({"lib": v[0], "blocks_per_cu": v[4], "stage": v[5], "ms": round(ms, 4),
                    "gpps": round(n / ms / 1e6, 1), "GBps": round(n * bpt / ms / 1e6, 1),
                    "same_output": bool(torch.equal(outs[i], ref))})
    for r_ in res:
        print(json.dumps(r_))


if __name__ == "__main__":
    main()
