#!/usr/bin/env python3
"""Measurement tool: per-launch time of back-to-back classify launches (config 2) -- plain
launches, and the same launches replayed from a captured graph -- to size the inter-kernel gap
(DESIGN.md §4 "Completion events": measured with a temporary build that skipped the per-launch
use-event record, 130.2 -> 127.1 us per config-2 launch, before the fence-free events)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vpp_amd import device as D, workloads as W  # noqa: E402


def timed(fn, reps=5):
    best = 1e30
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1))
    return best


def main():
    k = 40
    w = W.config2(0)
    e = w.engine
    b = D.TupleBatch(w.n_tuples, with_sport=False)
    D.gen_tuples(e, b, **w.gen)
    out = torch.empty(w.n_tuples, dtype=torch.int32, device="cuda")
    for _ in range(60):
        D.classify(e, w.mode, w.table_id, b, out)
    plain = timed(lambda: [D.classify(e, w.mode, w.table_id, b, out) for _ in range(k)])
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for _ in range(k):
                D.classify(e, w.mode, w.table_id, b, out)
    torch.cuda.current_stream().wait_stream(s)
    graph = timed(lambda: g.replay())
    print({"launches": k, "plain_us_per_launch": round(plain * 1e3 / k, 2), "graph_us_per_launch": round(graph * 1e3 / k, 2)})


if __name__ == "__main__":
    main()
