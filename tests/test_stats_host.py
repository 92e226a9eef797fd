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
    # the snapshot followed the recompile: unchanged ACLs answer with their counts in the new
    # layout (and say which), the new ACL with zero
    assert _by_rule(e, SNAP_GAUGE, "b", 3) == (int(cnt[3]), gen2)
    assert _by_rule(e, SNAP_GAUGE, "a", 0) == (0, gen2)
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


def _apply(e, acls):
    e.ApplyTxn(True, [("config/vpp/acls/v2/acl/" + n, {"name": n, "rules": r, "ingress": [], "egress": ["if-" + n]})
                      for n, r in acls.items()])


def test_counts_survive_a_commit_that_changes_another_acl():
    """A Commit that changes one ACL keeps every other ACL's counts (rules and default deny),
    and "no ACL" / "unresolved"; the changed ACL starts at zero, a removed one is gone
    (plugin_impl_statscollector.go:248-261: the gauge is a monotonic source)."""
    import random
    rnd = random.Random(11)
    acls = {"b": fz.rand_acl(rnd, 40, fz.ANCHORS, weird=False, tail="deny"),
            "d": fz.rand_acl(rnd, 25, fz.ANCHORS, weird=False, tail="permit"),
            "f": fz.rand_acl(rnd, 10, fz.ANCHORS, weird=False, tail="deny")}
    e = _engine(acls)
    cnt = _classify_counts(e, "b", 1) + _classify_counts(e, "d", 2) + _classify_counts(e, "f", 3)
    ns = len(cnt)
    cnt[ns - 2] += 7  # "no ACL"
    cnt[ns - 1] += 5  # "unresolved"
    _set(e, SNAP_LOCAL, cnt)
    _set(e, SNAP_CLUSTER, cnt * np.uint64(3))
    old = {n: e.table_info(e.table_id(n)) for n in acls}
    # d's rules change (one rule dropped), f is removed, a (sorted first) is added
    acls2 = {"a": fz.rand_acl(rnd, 30, fz.ANCHORS, weird=False, tail="deny"), "b": acls["b"], "d": acls["d"][1:]}
    _apply(e, acls2)
    e.num_counter_slots()  # compiles the new layout (no device)
    gen = lib.pg_counter_layout_gen(e.h)
    base, n, dflt = old["b"]
    for which, k in ((SNAP_LOCAL, 1), (SNAP_CLUSTER, 3)):
        for i in range(n):
            assert _by_rule(e, which, "b", i) == (int(cnt[base + i]) * k, gen)
        assert _by_rule(e, which, "b", -1) == (int(cnt[dflt]) * k, gen)
        for i in range(len(acls2["d"])):
            assert _by_rule(e, which, "d", i) == (0, gen)
        assert _by_rule(e, which, "d", -1) == (0, gen)
        assert _by_rule(e, which, "a", 0) == (0, gen)
        assert _by_rule(e, which, "f", 0) is None
        assert _by_rule(e, which, None, -1) == (int(cnt[ns - 2]) * k, gen)
        assert _by_rule(e, which, None, -2) == (int(cnt[ns - 1]) * k, gen)
    # the whole snapshot is in the new layout
    ns2 = e.num_counter_slots()
    v, g = _range(e, SNAP_LOCAL, 0, ns2)
    assert g == gen and len(v) == ns2
    nb, _, db = e.table_info(e.table_id("b"))
    assert np.array_equal(v[nb:nb + n], cnt[base:base + n]) and v[db] == cnt[dflt]
    assert int(v.sum()) == int(cnt[base:base + n].sum() + cnt[dflt] + cnt[ns - 2] + cnt[ns - 1])
    # a recompile that changes nothing (a compiler knob) keeps every count
    e.set_tuning("fd", 0)
    e.num_counter_slots()
    assert lib.pg_counter_layout_gen(e.h) > gen
    v2, _ = _range(e, SNAP_LOCAL, 0, ns2)
    assert np.array_equal(v2, v)
    # same name, same rule count, one rule's action flipped: a changed ACL
    b2 = [dict(r) for r in acls2["b"]]
    b2[0]["action"] = 1 - b2[0]["action"] if b2[0]["action"] in (0, 1) else 0
    _apply(e, dict(acls2, b=b2))
    e.num_counter_slots()
    assert _by_rule(e, SNAP_LOCAL, "b", 1)[0] == 0


def test_layout_generation_polled_during_recompiles():
    """pg_counter_layout_gen from other threads while the control thread recompiles (an atomic;
    the TSan build runs this too): it only ever increases"""
    import random
    rnd = random.Random(5)
    acls = {"x": fz.rand_acl(rnd, 30, fz.ANCHORS, weird=False, tail="deny")}
    e = _engine(acls)
    e.num_counter_slots()
    stop = threading.Event()
    bad = []

    def poll():
        last = 0
        while not stop.is_set():
            g = lib.pg_counter_layout_gen(e.h)
            if g < last:
                bad.append((last, g))
            last = g

    th = [threading.Thread(target=poll) for _ in range(2)]
    for t in th:
        t.start()
    for k in range(20):
        e.set_tuning("fd", k % 2)
        e.num_counter_slots()
    stop.set()
    for t in th:
        t.join()
    assert not bad


def test_stream_slot_bookkeeping():
    """CONN launches hand their deferred ANY-protocol packets to the k_conn_any after them on the
    same stream through a per-(table set, stream) mark word (device.hpp StreamSlots): one slot per
    stream, launch numbers strictly increasing and never 0 per slot, and numbers never repeated
    at a slot across a drain (clear) that reassigns slots to other streams."""
    rng = np.random.default_rng(1)
    streams = rng.integers(1, 80, size=3000).astype(np.uint64)  # 79 streams > 32 slots: drains
    streams[:40] = 0  # the null stream too
    n = len(streams)
    slot, seq = (C.c_uint32 * n)(), (C.c_uint32 * n)()
    assert lib.pg_debug_stream_slots(streams.ctypes.data_as(C.POINTER(C.c_uint64)), n, slot, seq) == 0
    slot, seq = np.frombuffer(slot, np.uint32), np.frombuffer(seq, np.uint32)
    assert slot.max() < 32 and seq.min() > 0
    # model: a stream keeps its slot until a drain; a drain happens only when a 33rd stream
    # arrives, and empties every slot
    live, last, drains = [], {}, 0
    for s, i, q in zip(streams.tolist(), slot.tolist(), seq.tolist()):
        if s not in live:
            if len(live) == 32:
                live, drains = [], drains + 1
            live.append(s)
        assert i == live.index(s)  # one slot per live stream, distinct across streams
        assert q > last.get(i, 0)  # per slot strictly increasing, across drains too
        last[i] = q
    assert drains > 10
    # the first 40 launches, all on the null stream: one slot, numbers 1..40
    assert set(slot[:40]) == {0} and np.array_equal(seq[:40], np.arange(1, 41))
    assert lib.pg_debug_stream_slots(None, 0, None, None) == 0
