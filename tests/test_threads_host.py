"""Host-side threading of the C ABI (CPU; the TSan build runs these, tools/tsan_tests.sh).

A cgo caller may drive several contexts from different OS threads at once, and set process
tuning defaults while another thread creates a context (include/policygpu.h: "distinct contexts
may be used concurrently from different threads"). ctypes releases the GIL during every
foreign call, so the threads below really run the library concurrently:
  * every acl_renderer_test.go scenario replayed by four threads, each on its own contexts
    (renderer txns, ApplyTxn, ACL dumps, counts, placement asserts);
  * four threads compiling their own cluster tables and classifying with the kernels' per-tuple
    code on the host (pg_debug_classify_host), checked against a single-threaded run;
  * pg_set_tuning of the process defaults racing pg_create.
"""
import threading

import numpy as np

import acl_fuzz as fz
import kat_driver as kd


def _run_threads(fn, n):
    errors = []

    def wrap(k):
        try:
            fn(k)
        except BaseException as ex:  # reported below
            errors.append((k, repr(ex)))

    th = [threading.Thread(target=wrap, args=(k,)) for k in range(n)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=600)
    assert not errors, errors


def test_renderer_scenarios_from_four_threads():
    scenarios = kd.load("acl_renderer_kats.json")

    def work(k):
        for sc in scenarios[k % len(scenarios):] + scenarios[:k % len(scenarios)]:
            bad = kd.run_scenario(kd.ProductBackend(gpu=False), sc)
            bad = [b for b in bad if not b[0]["kind"].startswith("Connection")]  # device-only checks
            assert not bad, (sc["name"], bad[:2])

    _run_threads(work, 4)


def test_host_classify_from_four_threads():
    from vpp_amd import workloads as W
    rng = np.random.default_rng(17)
    tup = fz.rand_tuples(rng, 30000, fz.ANCHORS + [W.ip_u32("10.10.1.1"), W.ip_u32("10.10.2.1")])
    w0 = W.config1(0, n_tuples=1 << 10)
    ref = w0.engine.debug_classify_host(w0.mode, w0.table_id, *tup, counters=True)
    res = [None] * 4

    def work(k):
        w = W.config1(0, n_tuples=1 << 10)  # its own contexts, compiled in this thread
        for _ in range(3):
            res[k] = w.engine.debug_classify_host(w.mode, w.table_id, *tup, counters=True)

    _run_threads(work, 4)
    for out, cnt in res:
        assert np.array_equal(out, ref[0]) and np.array_equal(cnt, ref[1])


def test_process_defaults_set_while_contexts_are_created():
    from vpp_amd import _capi
    from vpp_amd import renderer as R
    lib = _capi.lib
    seen = []

    def work(k):
        for i in range(200):
            if k == 0:
                assert lib.pg_set_tuning(b"hist_window", 1000 + (i % 7)) == 0
            else:
                e = R.Engine(0)
                seen.append(e.get_tuning("hist_window"))
                e.close()

    try:
        _run_threads(work, 3)
    finally:
        lib.pg_set_tuning(b"hist_window", 4096)
    assert set(seen) <= {4096} | {1000 + i for i in range(7)}
