"""bench.py's CPU-baseline leg without a GPU: its samples must compare bit-exact with the
product's verdicts, so the baseline times the same calls the product answers. Here the
"GPU" verdicts are the oracle's own (World: the product's semantics, pinned elsewhere against
the reference's KATs), fed through bench.cpu_baseline with small sample budgets."""
import numpy as np
import torch

import bench
from oracle import gen as G
from oracle.world import World
from vpp_amd import workloads as W


class _Batch:
    """the slice of device.TupleBatch that cpu_baseline reads"""

    def __init__(self, tup):
        self.tup, self.n = tup, len(tup[0])

    def numpy(self, k):
        return tuple(x[:k] for x in self.tup)


def _run(w, n):
    tup = G.gen_tuples(n, **w.gen)[:5]
    wd = World(w.engine, w.local_ifs, w.node_if)
    if w.mode == 2:
        act, slot = wd.conn(*tup, threads=4)
    else:
        act, slot = wd.perpod(tup[0], tup[1], tup[3], tup[4], threads=4)
    verdicts = (act.astype(np.uint32) << 30) | slot.astype(np.uint32)
    out = torch.from_numpy(verdicts.view(np.int32).copy())
    return bench.cpu_baseline(w, _Batch(tup), out, n, faithful_s=0.2, budget_s=0.4)


def test_conn_baseline_uses_the_connection_endpoint_rules():
    """CONN (config 5's topology): remote pod <-> non-pod and non-pod <-> non-pod make no
    evaluation (aclengine_mock.go:343-347, 388-392) in the baseline too -- its sample and its
    reference-faithful sample equal the product's verdicts."""
    w = W.config5(0, n_tuples=1 << 14)
    r = _run(w, 1 << 14)
    assert r["sample_bit_exact_vs_gpu"] is True
    assert r["faithful_variant_bit_exact"] is True
    assert r["faithful_nthreads_bit_exact"] is True and r["faithful_nthreads_cores"] == bench.host_cores()


def test_perpod_baseline_bit_exact():
    """PERPOD (config 3): the pre-parsed and the reference-faithful samples, at one thread and at
    every core, equal the product's verdicts."""
    w = W.config3(0, n_tuples=1 << 14)
    r = _run(w, 1 << 14)
    assert r["sample_bit_exact_vs_gpu"] is True
    assert r["faithful_variant_bit_exact"] is True
    assert r["faithful_nthreads_bit_exact"] is True and r["faithful_nthreads_cores"] == bench.host_cores()
