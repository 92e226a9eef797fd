#!/usr/bin/env python3
"""Per-launch durations of the classify kernel from a cold start (why the first launches of
a bench run are slower than the steady state).

Records one HIP-event pair per launch on the launch stream, in phases:
  cold     the bench's own sequence: workload built, batch generated, then N launches
  idle     the same after the process slept --idle seconds (GPU idle)
  busy     the same right after ~--busy-ms of other device work (a long memset loop on a
           scratch buffer, no classify launch), to separate clock ramp-up from anything the
           classify kernel itself warms (caches, TLB)
  regen    the batch regenerated (k_gen rewrites every tuple) and N launches again

    python tools/ramp_probe.py --config 2 --launches 120 > gpurun_out/ramp.json
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vpp_amd import _capi, device as D, workloads as W  # noqa: E402


def launches(lib, e, w, soa, n, out, k, stream):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(k + 1)]
    ev[0].record()
    for i in range(k):
        assert lib.pg_classify(e.h, w.mode, w.table_id, C.byref(soa), n, out.data_ptr(), None, stream) == 0
        ev[i + 1].record()
    torch.cuda.synchronize()
    return [round(ev[i].elapsed_time(ev[i + 1]) * 1e3, 1) for i in range(k)]  # us


def summary(us):
    q = lambda a, b: round(sum(us[a:b]) / max(1, len(us[a:b])), 1)  # noqa: E731
    return {"first5": q(0, 5), "6-25": q(5, 25), "26-50": q(25, 50), "51-100": q(50, 100), "last20": q(len(us) - 20,
                                                                                                        len(us))}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--launches", type=int, default=120)
    ap.add_argument("--idle", type=float, default=1.0)
    ap.add_argument("--busy-ms", type=float, default=200.0)
    a = ap.parse_args()
    lib = _capi.lib
    w = W.CONFIGS[a.config](0)
    e, n = w.engine, w.n_tuples
    b = D.TupleBatch(n, with_sport=(w.mode == 2))
    D.gen_tuples(e, b, **w.gen)
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    soa = b.soa()
    stream = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    res = {}
    res["cold"] = launches(lib, e, w, soa, n, out, a.launches, stream)
    time.sleep(a.idle)
    res["idle"] = launches(lib, e, w, soa, n, out, a.launches, stream)
    scratch = torch.empty(256 << 20, dtype=torch.uint8, device="cuda")
    t0 = time.perf_counter()
    while (time.perf_counter() - t0) * 1e3 < a.busy_ms:
        for _ in range(20):
            scratch.fill_(1)
        torch.cuda.synchronize()
    res["busy"] = launches(lib, e, w, soa, n, out, a.launches, stream)
    D.gen_tuples(e, b, **w.gen)
    res["regen"] = launches(lib, e, w, soa, n, out, a.launches, stream)
    for k, us in res.items():
        print(json.dumps({"phase": k, "config": a.config, "summary_us": summary(us), "us": us}), flush=True)


if __name__ == "__main__":
    main()
