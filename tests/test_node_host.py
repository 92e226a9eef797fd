"""The node classifier (fastpath.cpp build_node; PERPOD / CONN modes) checked on the host.

pg_debug_classify_host runs pg_classify's per-tuple code (vpp_amd/csrc/classify.hpp, the
templates the kernels instantiate) on the CPU. For every topology below the node path, the
per-table path (per-ACL blobs + IPv4 hash) and the C oracle's evalACL / testConnection
(oracle.world over the engine's exported ACLs) must agree bit-exactly on (action, counter
slot), and the node path's hit counters must equal the per-table path's.
"""
import random

import numpy as np
import pytest

import acl_fuzz as fz
from oracle import gen
from oracle.world import World
from vpp_amd import _capi
from vpp_amd import renderer as R
from vpp_amd import workloads as W
from vpp_amd._capi import MODE_CONN, MODE_PERPOD


def topology(rnd, n_pods=14, weird=False, big=False):
    """Local pods with random inbound/outbound ACLs on their TAPs (some reflective), two
    remote pods, one pod without an interface, and ACLs on the node-output interface."""
    e = R.Engine(0)
    e.SetMainInterfaceName("GbE")
    e.SetVxlanBVIIfName("VXLAN-BVI")
    e.SetHostInterconnectIfName("VPP-Host")
    local, ops, pod_ips, no_if = {}, [], [], []
    for k in range(n_pods):
        ip = 0x0A0A0000 | (k + 1)
        pod_ips.append(ip)
        another = k >= n_pods - 2
        ifn = "tap%d" % k if not another and k != 3 else None
        if ifn:
            e.SetPodIfName("ns/p%d" % k, ifn)
            local[ip] = ifn
        e.RegisterPod("ns/p%d" % k, W.ip_str(ip), another)
        if not ifn:
            if not another:
                no_if.append(ip)
            continue
        if rnd.random() < 0.6:
            inb = ([{"action": 2, "src": "", "dst": ""}] if rnd.random() < 0.4 else
                   fz.rand_acl(rnd, rnd.randint(0, 8), fz.ANCHORS + [ip], weird))
            ops.append(("config/vpp/acls/v2/acl/in-" + ifn, {"name": "in-" + ifn, "rules": inb, "ingress": [ifn],
                                                            "egress": []}))
        if rnd.random() < 0.8:
            outb = fz.rand_acl(rnd, rnd.randint(0, 40), fz.ANCHORS + pod_ips, weird, tail="deny")
            ops.append(("config/vpp/acls/v2/acl/out-" + ifn, {"name": "out-" + ifn, "rules": outb, "ingress": [],
                                                             "egress": [ifn]}))
    glob = fz.rand_acl(rnd, 30, fz.ANCHORS + pod_ips, weird, tail="permit")
    if big:  # one table past the cross-product limit (candidate mode): not covered by the node
        glob = [{"action": k % 2, "src": "10.%d.%d.0/24" % (k // 256, k % 256), "dst": "",
                 "udp": {"src": [0, 65535], "dst": [k % 1000, k % 1000 + 5]}} for k in range(17000)] + glob
    ops.append(("config/vpp/acls/v2/acl/g", {"name": "g", "rules": glob, "ingress": [], "egress": ["VXLAN-BVI"]}))
    e.ApplyTxn(True, ops)
    return e, (local, no_if), pod_ips


def tuples(seed, n, pod_ips, any_pct=0.02):
    rng = np.random.default_rng(seed)
    tup = list(fz.rand_tuples(rng, n, fz.ANCHORS + pod_ips, any_pct=any_pct))
    for k in (0, 1):  # most end points are pods
        m = rng.random(n) < 0.6
        tup[k][m] = np.array(pod_ips, np.uint32)[rng.integers(0, len(pod_ips), int(m.sum()))]
    return tuple(tup)


def check(e, local, tup, expect_node=True):
    src, dst, sport, dport, proto = tup
    assert (e.node_stats() is not None) == expect_node
    wd = World(e, local[0], "VXLAN-BVI", no_if_ips=local[1])
    act, slot = wd.perpod(src, dst, dport, proto, threads=4)
    pn, cpn = e.debug_classify_host(MODE_PERPOD, -1, *tup, counters=True, node=True)
    pt, cpt = e.debug_classify_host(MODE_PERPOD, -1, *tup, counters=True, node=False)
    for node in (True, False):  # the branching walks (HBM-resident images) too
        assert np.array_equal(e.debug_classify_host(MODE_PERPOD, -1, *tup, node=node, pred=False), pn)
        assert np.array_equal(e.debug_classify_host(MODE_CONN, -1, *tup, node=node, pred=False),
                              e.debug_classify_host(MODE_CONN, -1, *tup, node=node))
    # the node image without its common-row section (what the kernels run when it does not
    # fit their LDS budget): same verdicts and counters
    p0, c0 = e.debug_classify_host(MODE_PERPOD, -1, *tup, counters=True, node=True, common=False)
    assert np.array_equal(p0, pn) and np.array_equal(c0, cpn)
    q0, d0 = e.debug_classify_host(MODE_CONN, -1, *tup, counters=True, node=True, common=False)
    q1, d1 = e.debug_classify_host(MODE_CONN, -1, *tup, counters=True, node=True)
    assert np.array_equal(q0, q1) and np.array_equal(d0, d1)
    assert np.array_equal(pn, pt)
    assert np.array_equal(cpn, cpt)
    assert np.array_equal(pn >> 30, act.astype(np.uint32)), np.nonzero((pn >> 30) != act)[0][:8]
    assert np.array_equal(pn & 0x3FFFFFFF, slot)
    assert np.array_equal(cpn, np.bincount(pn & 0x3FFFFFFF, minlength=len(cpn)))
    conn, cslot = wd.conn(src, dst, sport, dport, proto, threads=4)
    cn, ccn = e.debug_classify_host(MODE_CONN, -1, *tup, counters=True, node=True)
    ct, cct = e.debug_classify_host(MODE_CONN, -1, *tup, counters=True, node=False)
    assert np.array_equal(cn, ct)
    assert np.array_equal(ccn, cct)
    assert np.array_equal(cn >> 30, conn.astype(np.uint32)), np.nonzero((cn >> 30) != conn)[0][:8]
    assert np.array_equal(cn & 0x3FFFFFFF, cslot)
    return pn, cn


@pytest.mark.parametrize("seed", range(6))
def test_random_topologies(seed):
    rnd = random.Random(2000 + seed)
    e, local, pod_ips = topology(rnd, weird=seed % 2 == 1)
    tup = tuples(seed, 20003 + seed, pod_ips)  # ragged: the kernels' one-tuple tail too
    pn, cn = check(e, local, tup)
    assert len(set((cn >> 30).tolist())) >= 2


def test_table_over_cross_limit_falls_back_per_table():
    rnd = random.Random(77)
    e, local, pod_ips = topology(rnd, big=True)
    assert e.table_stats(e.table_id("g"))["structure"] == "cand"
    check(e, local, tuples(77, 8000, pod_ips))


def test_node_disabled_and_rebuilt():
    rnd = random.Random(5)
    lib = _capi.lib
    try:
        assert lib.pg_set_tuning(b"node_build", 0) == 0
        e, local, pod_ips = topology(rnd)
        tup = tuples(5, 3000, pod_ips)
        assert e.node_stats() is None
        a = e.debug_classify_host(MODE_CONN, -1, *tup, node=True)  # falls back to per-table
        check(e, local, tup, expect_node=False)
    finally:
        assert lib.pg_set_tuning(b"node_build", 1) == 0
    e2, local2, _ = topology(random.Random(5))
    assert e2.node_stats() is not None
    assert np.array_equal(e2.debug_classify_host(MODE_CONN, -1, *tup, node=True), a)


@pytest.mark.parametrize("root_bits", [4, 8, 16])
def test_node_root_strides(root_bits):
    lib = _capi.lib
    try:
        assert lib.pg_set_tuning(b"node_root_bits", root_bits) == 0
        e, local, pod_ips = topology(random.Random(9))
        check(e, local, tuples(9, 6000, pod_ips))
    finally:
        assert lib.pg_set_tuning(b"node_root_bits", 12) == 0


def test_no_acls_and_unresolved_node_interface():
    e = R.Engine(0)
    e.SetMainInterfaceName("")  # no node-output interface: non-local addresses are unresolvable
    e.SetPodIfName("ns/a", "tapA")
    e.RegisterPod("ns/a", "10.0.0.1", False)
    e.ApplyTxn(True, [("config/vpp/acls/v2/acl/x", {"name": "x", "rules": [{"action": 2, "src": "", "dst": ""}],
                                                    "ingress": ["tapA"], "egress": []})])
    tup = tuples(3, 2000, [0x0A000001])
    pn = e.debug_classify_host(MODE_PERPOD, -1, *tup, node=True)
    pt = e.debug_classify_host(MODE_PERPOD, -1, *tup, node=False)
    assert np.array_equal(pn, pt)
    cn = e.debug_classify_host(MODE_CONN, -1, *tup, node=True)
    assert np.array_equal(cn, e.debug_classify_host(MODE_CONN, -1, *tup, node=False))
    assert 3 in set((cn >> 30).tolist())  # FAILURE for unresolvable end points


def test_config3_cluster_node_path():
    """Config 3's topology (1k pods, ~9.6k rules): node size and host parity on a sample."""
    w = W.config3(0, n_tuples=1 << 16)
    e = w.engine
    ns = e.node_stats()
    assert ns is not None and ns["image_bytes"] <= 64 << 10, ns  # staged in LDS by the kernel
    # most (table, source class) rows are the table's common row (no rule admits the source)
    assert ns["common_row_pairs"] >= 0.8 * ns["table_ipclass_pairs"], ns
    src, dst, sport, dport, proto = gen.gen_tuples(60001, **w.gen)
    wd = World(e, w.local_ifs, w.node_if)
    act, slot = wd.perpod(src, dst, dport, proto, threads=8)
    got = e.debug_classify_host(MODE_PERPOD, -1, src, dst, sport, dport, proto, node=True)
    assert np.array_equal(got >> 30, act.astype(np.uint32)) and np.array_equal(got & 0x3FFFFFFF, slot)
    conn, cslot = wd.conn(src, dst, sport, dport, proto, threads=8)
    got = e.debug_classify_host(MODE_CONN, -1, src, dst, sport, dport, proto, node=True)
    assert np.array_equal(got >> 30, conn.astype(np.uint32)) and np.array_equal(got & 0x3FFFFFFF, cslot)
    got0 = e.debug_classify_host(MODE_CONN, -1, src, dst, sport, dport, proto, node=True, common=False)
    assert np.array_equal(got0, got)
    # the global table's dst-specific rules: resolved by the list-verdict table (no records)
    assert ns["list_table_bytes"] > 0 and ns["list_record_bytes"] == 0, ns
    # every table covered, none in PAIR form: the uniform cross layout
    assert ns["uniform"], ns


def test_config8_more_than_64_tables_uniform_grouped_marks():
    """Config 8 (config 3's cluster with 20 apps per namespace: 202 per-pod tables, past the
    64 tables one 64-bit common-row mask per IP class marks one by one): still the uniform
    layout, its marks cover groups of tables (a clear group bit gathers the entry from the cross
    table), and PERPOD / CONN with counters equal the oracle and the layout without common rows."""
    w = W.config8(0, n_tuples=1 << 16)
    e = w.engine
    ns = e.node_stats()
    assert e.num_tables() > 64 and ns["uniform"] and ns["image_bytes"] <= 64 << 10, ns
    assert ns["common_row_pairs"] >= 0.5 * ns["table_ipclass_pairs"], ns
    src, dst, sport, dport, proto = gen.gen_tuples(40001, **w.gen)
    wd = World(e, w.local_ifs, w.node_if)
    act, slot = wd.perpod(src, dst, dport, proto, threads=8)
    got, cnt = e.debug_classify_host(MODE_PERPOD, -1, src, dst, sport, dport, proto, node=True, counters=True)
    assert np.array_equal(got >> 30, act.astype(np.uint32)) and np.array_equal(got & 0x3FFFFFFF, slot)
    assert np.array_equal(cnt, np.bincount(got & 0x3FFFFFFF, minlength=len(cnt)))
    conn, cslot, hist = wd.conn(src, dst, sport, dport, proto, threads=8, hist=True)
    got, cnt = e.debug_classify_host(MODE_CONN, -1, src, dst, sport, dport, proto, node=True, counters=True)
    assert np.array_equal(got >> 30, conn.astype(np.uint32)) and np.array_equal(got & 0x3FFFFFFF, cslot)
    assert np.array_equal(cnt, hist)
    got0 = e.debug_classify_host(MODE_CONN, -1, src, dst, sport, dport, proto, node=True, common=False)
    assert np.array_equal(got0, got)


def test_config9_more_than_254_tables_wide_records():
    """Config 9 (config 3's cluster with 50 apps per namespace: 502 per-pod tables, past the 254
    whose ids fit a byte of the class record): still the uniform layout, with wide class records
    (16-bit table ids beside 32-bit grouped common-row marks), and PERPOD / CONN with counters
    equal the oracle, the per-table path and the layout without common rows."""
    w = W.config9(0, n_tuples=1 << 16)
    e = w.engine
    ns = e.node_stats()
    assert e.num_tables() > 254 and ns["uniform"] and ns["wide_records"] and ns["image_bytes"] <= 64 << 10, ns
    assert ns["common_row_pairs"] >= 0.5 * ns["table_ipclass_pairs"], ns
    src, dst, sport, dport, proto = gen.gen_tuples(40001, **w.gen)
    wd = World(e, w.local_ifs, w.node_if)
    act, slot = wd.perpod(src, dst, dport, proto, threads=8)
    got, cnt = e.debug_classify_host(MODE_PERPOD, -1, src, dst, sport, dport, proto, node=True, counters=True)
    assert np.array_equal(got >> 30, act.astype(np.uint32)) and np.array_equal(got & 0x3FFFFFFF, slot)
    assert np.array_equal(cnt, np.bincount(got & 0x3FFFFFFF, minlength=len(cnt)))
    assert np.array_equal(e.debug_classify_host(MODE_PERPOD, -1, src, dst, sport, dport, proto, node=False), got)
    conn, cslot, hist = wd.conn(src, dst, sport, dport, proto, threads=8, hist=True)
    got, cnt = e.debug_classify_host(MODE_CONN, -1, src, dst, sport, dport, proto, node=True, counters=True)
    assert np.array_equal(got >> 30, conn.astype(np.uint32)) and np.array_equal(got & 0x3FFFFFFF, cslot)
    assert np.array_equal(cnt, hist)
    got0 = e.debug_classify_host(MODE_CONN, -1, src, dst, sport, dport, proto, node=True, common=False)
    assert np.array_equal(got0, got)
    assert len(set((got >> 30).tolist())) >= 3


def _many_tables(n_tables, seed):
    """n_tables - 1 local pods, each with its own small outbound ACL, and a global ACL on the
    node-output interface: n_tables tables, every one covered by the node."""
    rnd = random.Random(seed)
    e = R.Engine(0)
    e.SetMainInterfaceName("GbE")
    e.SetVxlanBVIIfName("VXLAN-BVI")
    e.SetHostInterconnectIfName("VPP-Host")
    local, ops, pod_ips = {}, [], []
    for k in range(n_tables - 1):
        ip = 0x0A0B0000 | (k + 1)
        pod_ips.append(ip)
        ifn = "tap%d" % k
        e.SetPodIfName("ns/p%d" % k, ifn)
        e.RegisterPod("ns/p%d" % k, W.ip_str(ip), False)
        local[ip] = ifn
        outb = []  # from a few pods, a few popular ports: a cross product the node keeps small
        for _ in range(rnd.randint(1, 3)):
            r = {"action": rnd.choice([0, 1, 1, 2]), "src": W.ip_str(rnd.choice(pod_ips)) + "/32", "dst": ""}
            if rnd.random() < 0.7:
                p = rnd.choice([80, 443, 8080])
                r[rnd.choice(["tcp", "udp"])] = {"src": [0, 65535], "dst": [p, p]}
            outb.append(r)
        outb.append({"action": 0, "src": "", "dst": ""})
        ops.append(("config/vpp/acls/v2/acl/out-" + ifn, {"name": "out-" + ifn, "rules": outb, "ingress": [],
                                                         "egress": [ifn]}))
    glob = [{"action": k % 2, "src": W.ip_str(pod_ips[k]) + "/32", "dst": ""} for k in range(12)]
    glob.append({"action": 1, "src": "", "dst": ""})
    ops.append(("config/vpp/acls/v2/acl/g", {"name": "g", "rules": glob, "ingress": [], "egress": ["VXLAN-BVI"]}))
    e.ApplyTxn(True, ops)
    return e, (local, []), pod_ips


@pytest.mark.parametrize("n_tables", [251, 252, 253, 255, 256])
def test_uniform_node_at_the_narrow_wide_record_boundary(n_tables):
    """Table counts either side of the class records' byte-wide table ids (fastpath.cpp
    build_node: narrow records while every id and the "no ACL" pseudo-table's id fit 0..254,
    wide 16-bit ids past that). Past 64 tables the common-row marks group 4 tables per bit, and
    the pseudo-table takes a group of its own, so its id is the table count rounded up to 4:
    252 tables -> 252 (narrow), 253 -> 256 (wide). The uniform layout either way, and PERPOD /
    CONN with counters equal to the oracle and the per-table path (check())."""
    e, local, pod_ips = _many_tables(n_tables, 900 + n_tables)
    assert e.num_tables() == n_tables
    ns = e.node_stats()
    assert ns["uniform"], ns
    assert ns["wide_records"] == (n_tables > 252), (n_tables, ns["wide_records"])
    pn, cn = check(e, local, tuples(n_tables, 6007, pod_ips))
    assert len(set((cn >> 30).tolist())) >= 2


def test_node_lists_table_or_records_in_image_or_cross():
    """A node cross entry with dst-specific rules ahead of its verdict resolves them the same
    three ways, all equal to the oracle: by the list-verdict table (default: one read at [list]
    [dst's node IP class]), by dst records copied into the image (node_list_table=0), and by
    records read from the cross array (node_list_table=0, node_list_words=0: no copy)."""
    w = W.config3(0, n_tuples=1 << 10, n_ns=4)
    src, dst, sport, dport, proto = gen.gen_tuples(30001, **w.gen)
    ns = w.engine.node_stats()
    assert ns["list_table_bytes"] > 0 and ns["list_record_bytes"] == 0 and not ns["list_records_in_image"], ns
    a = w.engine.debug_classify_host(MODE_PERPOD, -1, src, dst, sport, dport, proto, node=True)
    c = w.engine.debug_classify_host(MODE_CONN, -1, src, dst, sport, dport, proto, node=True)
    assert _capi.lib.pg_set_tuning(b"node_list_table", 0) == 0
    try:
        w1 = W.config3(0, n_tuples=1 << 10, n_ns=4)
        ns1 = w1.engine.node_stats()
        assert ns1["list_records_in_image"] and ns1["list_table_bytes"] == 0, ns1
        assert ns1["image_bytes"] >= ns1["list_record_bytes"] > 0, ns1
        assert np.array_equal(w1.engine.debug_classify_host(MODE_PERPOD, -1, src, dst, sport, dport, proto, node=True), a)
        assert np.array_equal(w1.engine.debug_classify_host(MODE_CONN, -1, src, dst, sport, dport, proto, node=True), c)
        assert _capi.lib.pg_set_tuning(b"node_list_words", 0) == 0
        w2 = W.config3(0, n_tuples=1 << 10, n_ns=4)
        ns2 = w2.engine.node_stats()
        assert not ns2["list_records_in_image"] and ns2["image_bytes"] == ns1["image_bytes"] - ns1["list_record_bytes"]
        assert np.array_equal(w2.engine.debug_classify_host(MODE_PERPOD, -1, src, dst, sport, dport, proto, node=True), a)
        assert np.array_equal(w2.engine.debug_classify_host(MODE_CONN, -1, src, dst, sport, dport, proto, node=True), c)
    finally:
        assert _capi.lib.pg_set_tuning(b"node_list_words", 4096) == 0
        assert _capi.lib.pg_set_tuning(b"node_list_table", 1) == 0
    wd = World(w.engine, w.local_ifs, w.node_if)
    act, slot = wd.perpod(src, dst, dport, proto, threads=8)
    assert np.array_equal(a >> 30, act.astype(np.uint32)) and np.array_equal(a & 0x3FFFFFFF, slot)
    conn, cslot = wd.conn(src, dst, sport, dport, proto, threads=8)
    assert np.array_equal(c >> 30, conn.astype(np.uint32)) and np.array_equal(c & 0x3FFFFFFF, cslot)


def test_list_table_at_dst_prefix_edges():
    """The list-verdict table answers a list by the node IP class of the rule's dst-side address,
    built from one address per class; that holds only if every address of a class lies in the
    same dst prefixes of every list table (the class key). Checked where it would break first:
    the first and last address of every dst prefix of every table, and their neighbours, as dst
    (PERPOD, CONN SYN) and as src (CONN SYN-ACK), against the record form (node_list_table=0)
    and the oracle."""
    import ipaddress
    w = W.config3(0, n_tuples=1 << 10, n_ns=4)
    e = w.engine
    assert e.node_stats()["list_table_bytes"] > 0
    edges = set()
    for name in e.ACLNames():
        for r in e.GetACLByName(name)["rules"]:
            if r.get("dst"):
                net = ipaddress.ip_network(r["dst"], strict=False)
                lo, hi = int(net.network_address), int(net.broadcast_address)
                edges.update(x & 0xFFFFFFFF for x in (lo - 1, lo, lo + 1, hi - 1, hi, hi + 1))
    edges = np.array(sorted(edges), np.uint32)
    rng = np.random.default_rng(5)
    pods = np.array(list(w.local_ifs), np.uint32)
    n = 20 * len(edges)
    dst = np.tile(edges, 20)
    src = pods[rng.integers(0, len(pods), n)]
    swap = rng.random(n) < 0.5  # the edge address as src too (CONN's reverse evaluations)
    src[swap], dst[swap] = dst[swap], src[swap]
    proto = rng.choice(np.array([0, 1], np.uint8), n)
    dport = np.array(W.CLUSTER_PORTS, np.uint16)[rng.integers(0, len(W.CLUSTER_PORTS), n)]
    sport = np.array(W.CLUSTER_PORTS, np.uint16)[rng.integers(0, len(W.CLUSTER_PORTS), n)]
    tup = (src, dst, sport, dport, proto)
    a = e.debug_classify_host(MODE_PERPOD, -1, *tup, node=True)
    c = e.debug_classify_host(MODE_CONN, -1, *tup, node=True)
    with e.tuning(node_list_table=0):
        assert e.node_stats()["list_table_bytes"] == 0
        assert np.array_equal(e.debug_classify_host(MODE_PERPOD, -1, *tup, node=True), a)
        assert np.array_equal(e.debug_classify_host(MODE_CONN, -1, *tup, node=True), c)
    wd = World(e, w.local_ifs, w.node_if)
    act, slot = wd.perpod(src, dst, dport, proto, threads=8)
    assert np.array_equal(a >> 30, act.astype(np.uint32)) and np.array_equal(a & 0x3FFFFFFF, slot)
    conn, cslot = wd.conn(*tup, threads=8)
    assert np.array_equal(c >> 30, conn.astype(np.uint32)) and np.array_equal(c & 0x3FFFFFFF, cslot)


def test_common_rows_disabled():
    """node_common=0: the image has no common-row section and classifies the same."""
    rnd = random.Random(77)
    e, local, pod_ips = topology(rnd)
    tup = tuples(78, 20000, pod_ips)
    on = e.debug_classify_host(MODE_CONN, -1, *tup, node=True)
    ns = e.node_stats()
    assert ns["common_row_pairs"] > 0 and ns["image_bytes"] > ns["base_image_bytes"]
    assert _capi.lib.pg_set_tuning(b"node_common", 0) == 0
    try:
        e2, local2, pod_ips2 = topology(random.Random(77))
        ns2 = e2.node_stats()
        recs = ns2["list_record_bytes"] if ns2["list_records_in_image"] else 0
        assert ns2["common_row_pairs"] == 0 and ns2["image_bytes"] == ns2["base_image_bytes"] + recs
        assert np.array_equal(e2.debug_classify_host(MODE_CONN, -1, *tup, node=True), on)
    finally:
        assert _capi.lib.pg_set_tuning(b"node_common", 1) == 0


def _pair_coverage(e):
    """(tables in PAIR form, of them covered by the node): tabinfo words are internal, so read
    the coverage through the node's behaviour: a covered PAIR table classifies through the node
    exactly like through its per-table blob, which check() asserts; here only the structures."""
    return [e.table_stats(t)["structure"] for t in range(e.num_tables())].count("pair")


@pytest.mark.parametrize("seed", range(4))
def test_pair_tables_in_the_node(seed):
    """Tables in the PAIR form (src class x dst class -> pair class x key class; forced with
    pair = 2 on dst-specific random ACLs) are covered by the node classifier: node == per-table
    == oracle, PERPOD and CONN, with counters, weird rules included."""
    e0 = R.Engine(0)
    try:
        assert _capi.lib.pg_set_tuning(b"pair", 2) == 0
        rnd = random.Random(3000 + seed)
        e, local, pod_ips = topology(rnd, weird=seed % 2 == 1)
    finally:
        assert _capi.lib.pg_set_tuning(b"pair", 1) == 0
    assert e0.get_tuning("pair") == 1 and e.get_tuning("pair") == 2
    assert _pair_coverage(e) >= 3
    check(e, local, tuples(seed, 30011, pod_ips))


def test_config6_pair_table_covered():
    """config 6's 36.5k-rule global table (PAIR) is in the node: its image grows by the table's
    class map and PERPOD equals the per-table path and the oracle on a sample."""
    w = W.config6(0, n_tuples=1 << 10)
    e = w.engine
    big = [t for t in range(e.num_tables()) if e.table_info(t)[1] > 30000]
    assert big and e.table_stats(big[0])["structure"] == "pair"
    ns = e.node_stats()
    assert ns is not None and ns["image_bytes"] <= 64 << 10, ns
    src, dst, sport, dport, proto = gen.gen_tuples(40000, **w.gen)
    wd = World(e, w.local_ifs, w.node_if)
    act, slot = wd.perpod(src, dst, dport, proto, threads=8)
    got = e.debug_classify_host(MODE_PERPOD, -1, src, dst, sport, dport, proto, node=True)
    assert np.array_equal(got >> 30, act.astype(np.uint32)) and np.array_equal(got & 0x3FFFFFFF, slot)


def test_uniform_records_with_mostly_range_classes():
    """Aligned node tries (uniform layout): a class with a leaf above the trie's last level
    needs a 32-byte aligned record, so such classes take every other record slot. With few
    pods and many source ranges most classes are ranges, the slots outnumber the classes
    (unused slots between them), and the node still equals the per-table path and the oracle."""
    rnd = random.Random(91)
    e = R.Engine(0)
    e.SetMainInterfaceName("GbE")
    e.SetVxlanBVIIfName("VXLAN-BVI")
    e.SetHostInterconnectIfName("VPP-Host")
    local, pod_ips, ops = {}, [], []
    for k in range(3):
        ip = 0x0A0A0000 | (k + 1)
        pod_ips.append(ip)
        e.SetPodIfName("ns/p%d" % k, "tap%d" % k)
        e.RegisterPod("ns/p%d" % k, W.ip_str(ip), False)
        local[ip] = "tap%d" % k
    ranges = [{"action": rnd.choice([0, 1, 2]), "src": "%d.%d.%d.0/%d" % (10 + k % 3, k, (7 * k) % 256, rnd.choice([20, 22, 24])),
               "dst": ""} for k in range(120)]
    for k in range(3):
        ops.append(("config/vpp/acls/v2/acl/out-tap%d" % k, {"name": "out-tap%d" % k, "rules": ranges[40 * k:40 * k + 40]
                                                              + [{"action": 0, "src": "", "dst": ""}],
                                                              "ingress": [], "egress": ["tap%d" % k]}))
    ops.append(("config/vpp/acls/v2/acl/g", {"name": "g", "rules": ranges[::2] + [{"action": 1, "src": "", "dst": ""}],
                                             "ingress": [], "egress": ["VXLAN-BVI"]}))
    e.ApplyTxn(True, ops)
    ns = e.node_stats()
    assert ns["uniform"], ns
    anchors = [int(np.uint32((10 + k % 3) << 24 | k << 16 | ((7 * k) % 256) << 8)) for k in range(120)]
    rng = np.random.default_rng(92)
    src, dst, sport, dport, proto = fz.rand_tuples(rng, 30000, anchors + pod_ips, any_pct=0.02)
    m = rng.random(len(src)) < 0.5
    dst[m] = np.array(pod_ips, np.uint32)[rng.integers(0, len(pod_ips), int(m.sum()))]
    check(e, (local, []), (src, dst, sport, dport, proto))


@pytest.mark.parametrize("config", [3, 5])
def test_uniform_cross_layout_equals_per_table_layout(config):
    """The node's uniform cross layout (rows over the node key classes, addresses computed) and
    the per-table layout (node_uniform=0: tabinfo / kmap reads) classify the same, counters
    included, with and without the common-row section."""
    w = W.CONFIGS[config](0, n_tuples=1 << 10, n_ns=4)
    e = w.engine
    assert e.node_stats()["uniform"]
    src, dst, sport, dport, proto = gen.gen_tuples(40003, **w.gen)
    ref = {cm: e.debug_classify_host(w.mode, -1, src, dst, sport, dport, proto, counters=True, node=True, common=cm)
           for cm in (True, False)}
    with e.tuning(node_uniform=0):
        assert not e.node_stats()["uniform"]
        for cm in (True, False):
            got, cnt = e.debug_classify_host(w.mode, -1, src, dst, sport, dport, proto, counters=True, node=True,
                                             common=cm)
            assert np.array_equal(got, ref[cm][0]) and np.array_equal(cnt, ref[cm][1])
    per_table = e.debug_classify_host(w.mode, -1, src, dst, sport, dport, proto, node=False)
    assert np.array_equal(per_table, ref[True][0])
