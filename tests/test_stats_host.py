"""The statscollector value source (the sink is RegisterGaugeFunc,
plugins/statscollector/plugin_impl_statscollector.go:248-261) read through the C ABI without a
GPU: host snapshots of the counters, read by slot range and by stable rule identity (ACL name,
rule index) in the layout each snapshot was counted in. The snapshots are installed with
pg_debug_set_snapshot from the product's host classifier (pg_debug_classify_host), so nothing
here touches the device."""
import ctypes as C
import threading

import numpy as np
import pytest

from vpp_amd import _capi
from vpp_amd import renderer as R
from vpp_amd._capi import MODE_SINGLE, SNAP_CLUSTER, SNAP_GAUGE, SNAP_LOCAL, lib

import acl_fuzz as fz


def _engine(acls):
    e = R.Engine(0)
    e.SetVxlanBVIIfName("VXLAN-BVI")
    ops = [("config/vpp/acls/v2/acl/" + n, {"name": n, "rules": rules, "ingress": [], "egress": ["if-" + n]})
           for n, rules in acls.items()]
    e.ApplyTxn(True, ops)
    return e


def _set(e, which, cnt):
    a = np.ascontiguousarray(cnt, np.uint64)
    e._ck(lib.pg_debug_set_snapshot(e.h, which, a.ctypes.data_as(C.POINTER(C.c_uint64)), len(a)))


def _by_rule(e, which, name, idx):
    v, g = C.c_uint64(), C.c_uint64()
    rc = lib.pg_counter_of_rule(e.h, which, name.encode() if name is not None else None, idx, C.byref(v),
                                C.byref(g))
    return (None if rc == _capi.PG_ENOENT else (e._ck(rc), v.value, g.value)[1:])


def _range(e, which, first, n):
    buf = (C.c_uint64 * max(1, n))()
    g = C.c_uint64()
    k = e._ck(lib.pg_counters_snapshot_range(e.h, which, first, n, buf, C.byref(g)))
    return np.frombuffer(buf, np.uint64)[:k].copy(), g.value


def _classify_counts(e, name, seed):
    tid = e.table_id(name)
    tup = fz.rand_tuples(np.random.default_rng(seed), 20000, fz.ANCHORS)
    _, cnt = e.debug_classify_host(MODE_SINGLE, tid, *tup, counters=True)
    return cnt


def test_snapshot_reads_by_rule_identity_across_a_recompile():
    import random
    rnd = random.Random(3)
    acls = {"b": fz.rand_acl(rnd, 40, fz.ANCHORS, weird=False, tail="deny"),
            "d": fz.rand_acl(rnd, 25, fz.ANCHORS, weird=False, tail="permit")}
    e = _engine(acls)
    # nothing taken yet: no value, generation 0
    assert _by_rule(e, SNAP_GAUGE, "b", 0) is None
    v, g = _range(e, SNAP_LOCAL, 0, 8)
    assert len(v) == 0 and g == 0
    cnt = _classify_counts(e, "b", 1) + _classify_counts(e, "d", 2)
    assert cnt.sum() == 40000
    _set(e, SNAP_LOCAL, cnt)
    gen1 = lib.pg_counter_layout_gen(e.h)
    assert gen1 > 0
    # every rule of every ACL by identity == its slot (pg_table_info), one read each
    for name, rules in acls.items():
        base, n, dflt = e.table_info(e.table_id(name))
        assert n == len(rules)
        for i in range(n):
            assert _by_rule(e, SNAP_GAUGE, name, i) == (int(cnt[base + i]), gen1)
        assert _by_rule(e, SNAP_GAUGE, name, -1) == (int(cnt[dflt]), gen1)
        assert _by_rule(e, SNAP_GAUGE, name, n) is None  # past the ACL's rules
    ns = e.num_counter_slots()
    assert _by_rule(e, SNAP_GAUGE, None, -1) == (int(cnt[ns - 2]), gen1)
    assert _by_rule(e, SNAP_GAUGE, None, -2) == (int(cnt[ns - 1]), gen1)
    assert _by_rule(e, SNAP_GAUGE, "nope", 0) is None
    # ranges: any window, clipped at the end
    for first, n in ((0, ns), (5, 7), (ns - 3, 10), (ns, 4), (ns + 100, 1)):
        v, g = _range(e, SNAP_LOCAL, first, n)
        assert g == gen1 and np.array_equal(v, cnt[first:first + n])
    # the cluster snapshot is separate (never taken here) and the gauge is LOCAL without a
    # communicator
    assert _by_rule(e, SNAP_CLUSTER, "b", 0) is None
    # recompile with an ACL sorted ahead of both: every slot moves
    acls2 = dict(acls, a=fz.rand_acl(rnd, 30, fz.ANCHORS, weird=False, tail="deny"))
    e.ApplyTxn(True, [("config/vpp/acls/v2/acl/" + n, {"name": n, "rules": r, "ingress": [], "egress": ["if-" + n]})
                      for n, r in acls2.items()])
    cnt2 = _classify_counts(e, "a", 4)  # compiles the new layout
    gen2 = lib.pg_counter_layout_gen(e.h)
    assert gen2 > gen1
    base_b_new = e.table_info(e.table_id("b"))[0]
    base_b_old = 0
    assert base_b_new != base_b_old
    # the old snapshot still answers by identity in its own layout (and says which)
    assert _by_rule(e, SNAP_GAUGE, "b", 3) == (int(cnt[3]), gen1)
    assert _by_rule(e, SNAP_GAUGE, "a", 0) is None  # not in that layout
    _set(e, SNAP_LOCAL, cnt2)
    assert _by_rule(e, SNAP_GAUGE, "a", 0) == (int(cnt2[e.table_info(e.table_id("a"))[0]]), gen2)
    assert _by_rule(e, SNAP_GAUGE, "b", 3) == (int(cnt2[base_b_new + 3]), gen2)


def test_snapshot_readers_race_a_writer():
    """gauge reads on other threads while the snapshot is replaced (TSan build runs this too)"""
    import random
    rnd = random.Random(9)
    e = _engine({"x": fz.rand_acl(rnd, 50, fz.ANCHORS, weird=False, tail="deny")})
    cnt = _classify_counts(e, "x", 1)
    ns = len(cnt)
    _set(e, SNAP_LOCAL, cnt)
    stop = threading.Event()
    bad = []

    def reader():
        while not stop.is_set():
            r = _by_rule(e, SNAP_GAUGE, "x", 0)
            v, _ = _range(e, SNAP_LOCAL, 0, ns)
            # never torn: the whole range is one of the installed snapshots, cnt * m
            m = int(v.sum()) // int(cnt.sum()) if len(v) == ns else 0
            if r is None or m < 1 or not np.array_equal(v, cnt * np.uint64(m)):
                bad.append(r)

    th = [threading.Thread(target=reader) for _ in range(3)]
    for t in th:
        t.start()
    for k in range(300):
        _set(e, SNAP_LOCAL, cnt * (k + 1))
    stop.set()
    for t in th:
        t.join()
    assert not bad
    assert _by_rule(e, SNAP_GAUGE, "x", 0)[0] == int(cnt[0]) * 300


def test_snapshot_api_rejects_bad_arguments():
    e = _engine({"x": [{"action": 1, "src": "", "dst": ""}]})
    e.debug_classify_host(MODE_SINGLE, 0, *fz.rand_tuples(np.random.default_rng(0), 10, fz.ANCHORS))
    n = e.num_counter_slots()
    z = np.zeros(n + 1, np.uint64)
    p = z.ctypes.data_as(C.POINTER(C.c_uint64))
    assert lib.pg_debug_set_snapshot(e.h, SNAP_LOCAL, p, n + 1) == _capi.PG_EINVAL
    assert lib.pg_debug_set_snapshot(e.h, SNAP_GAUGE, p, n) == _capi.PG_EINVAL
    v = C.c_uint64()
    assert lib.pg_counter_of_rule(e.h, 7, b"x", 0, C.byref(v), None) == _capi.PG_EINVAL
    assert lib.pg_counter_of_rule(e.h, SNAP_LOCAL, None, 0, C.byref(v), None) in (_capi.PG_EINVAL, _capi.PG_ENOENT)
    assert lib.pg_counters_snapshot_range(e.h, 9, 0, 1, p, None) == _capi.PG_EINVAL
    with pytest.raises(Exception):
        _by_rule(e, SNAP_LOCAL, "x", -3)
