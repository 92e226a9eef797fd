"""The testConnection hit-counter oracle (CPU): every evalACL a connection makes, in the order
aclengine_mock.go:448-491 makes them, from the C oracle (oracle.c ora_conn with a trace) --
checked against the Python oracle's per-evaluation trace (oracle/aclengine.py
test_connection, pinned by the reference's KATs) on the 284 acl_renderer_test.go
connection checks and on random topologies with weird ACLs (every FAILURE branch), and the
histogram World.conn(hist=True) builds from it checked against a direct count.

The GPU side (tests/test_gpu_parity.py) asserts the device counters of config 5 and of random
CONN topologies equal this histogram."""
import random

import numpy as np
import pytest

import acl_fuzz as fz
import kat_driver as kd
from oracle import aclengine, fast, gonet, policy


def _acl_dicts(acl):
    out = []
    for r in acl.rules:
        d = {"action": r.action, "src": r.src_network, "dst": r.dst_network, "ip_rule": r.has_ip_rule,
             "ip": r.has_ip, "icmp": r.has_icmp, "macip": r.has_macip}
        for f in ("tcp", "udp"):
            s = getattr(r, f)
            if s is not None:
                d[f] = {"src": [s.src_range.lower, s.src_range.upper] if s.src_range is not None else None,
                        "dst": [s.dst_range.lower, s.dst_range.upper] if s.dst_range is not None else None}
        out.append(d)
    return out


def _c_world(eng, extra_ifs=()):
    """the Python oracle engine's installed ACLs and interface bindings, for the C oracle"""
    names = sorted(eng.cfg.by_name)
    acls = [fast.OraACL(_acl_dicts(eng.cfg.by_name[n])) for n in names]
    tid = {n: i for i, n in enumerate(names)}
    ifs = sorted(set(eng.cfg.by_if) | set(extra_ifs))
    ifx = {n: i for i, n in enumerate(ifs)}
    b = [eng.cfg.get_acls(n) for n in ifs]
    if_in = [tid[x[0].name] if x[0] is not None else -1 for x in b]
    if_out = [tid[x[1].name] if x[1] is not None else -1 for x in b]
    return acls, tid, ifx, if_in, if_out


def _py_trace(eng, tid, si, s, di, d, proto, sport, dport):
    tr = []
    conn = eng.test_connection(si, s, di, d, proto, sport, dport, trace=tr)
    return conn, [(tid[a.name] if a is not None else -1, i) for a, _, i in tr]


def _c_trace(acls, ifx, if_in, if_out, si, s, di, d, proto, sport, dport):
    conn, _, _, evt, evi = fast.test_connection(acls, if_in, if_out, [ifx[si]], [ifx[di]], [s], [d], [sport],
                                                [dport], [proto], threads=1, trace=True)
    return int(conn[0]), [(int(t), int(i)) for t, i in zip(evt[0], evi[0]) if t != -3]


def test_trace_matches_python_oracle_on_reference_kats():
    """acl_renderer_test.go's Connection* checks: verdict and the full evaluation sequence."""
    checked = 0
    for sc in kd.load("acl_renderer_kats.json"):
        ob = kd.OracleBackend()
        ob.setup(sc["setup"])
        node = sc["setup"]["vxlan_bvi"] or sc["setup"]["main_if"]
        for phase in sc["phases"]:
            for st in phase["steps"]:
                if st["op"] == "restart":
                    ob.restart()
                else:
                    ob.txn(st["resync"], st["renders"])
            eng = ob.engine
            ends = set(sc["setup"]["pod_ifs"].values()) | {node}
            acls, tid, ifx, if_in, if_out = _c_world(eng, ends)
            for c in phase["checks"]:
                if not c["kind"].startswith("Connection"):
                    continue
                a = c["args"]

                def ep(pod):
                    cfg = eng.pods[pod]
                    return (node if cfg.another_node else sc["setup"]["pod_ifs"][pod]), cfg.ip
                if c["kind"] == "ConnectionPodToPod":
                    (si, s), (di, d) = ep(a[0]), ep(a[1])
                elif c["kind"] == "ConnectionPodToInternet":
                    (si, s), di, d = ep(a[0]), node, gonet.parse_ip(a[1])
                else:
                    si, s, (di, d) = node, gonet.parse_ip(a[0]), ep(a[1])
                proto = kd.PROTO[a[2]]
                pc, pt = _py_trace(eng, tid, si, s, di, d, proto, a[3], a[4])
                cc, ct = _c_trace(acls, ifx, if_in, if_out, si, gonet.ipv4_u32(s), di, gonet.ipv4_u32(d), proto,
                                  a[3], a[4])
                assert pc == cc == kd.CONN[c["expect"]], (sc["name"], c)
                assert pt == ct, (sc["name"], c, pt, ct)
                checked += 1
    assert checked == 284


def _rand_engine(rnd, n_ifs=6, weird=True):
    ifs = policy.NodeIfaces()
    eng = aclengine.MockACLEngine(ifs)
    ops = {}
    names = ["if%d" % k for k in range(n_ifs)]
    for k, ifn in enumerate(names):
        for direction in ("in", "out"):
            if rnd.random() < 0.25:
                continue
            if direction == "in" and rnd.random() < 0.3:
                rules = [{"action": 2, "src": "", "dst": ""}]  # reflective ACL
            else:
                rules = fz.rand_acl(rnd, rnd.randint(0, 15), fz.ANCHORS, weird,
                                    tail=rnd.choice([None, "deny", "permit"]))
            acl = fz.to_oracle_acl("%s-%s" % (direction, ifn), rules)
            (acl.ingress if direction == "in" else acl.egress).append(ifn)
            ops[acl.name] = acl
    assert eng.apply_txn(True, ops) is None
    return eng, names


@pytest.mark.parametrize("seed", range(4))
def test_trace_matches_python_oracle_random_weird_topologies(seed):
    rnd = random.Random(4000 + seed)
    eng, names = _rand_engine(rnd, weird=True)
    acls, tid, ifx, if_in, if_out = _c_world(eng, names)
    rng = np.random.default_rng(seed)
    src, dst, sport, dport, proto = fz.rand_tuples(rng, 600, fz.ANCHORS, any_pct=0.03)
    for k in range(len(src)):
        si, di = rnd.choice(names), rnd.choice(names) if rnd.random() < 0.8 else None
        di = di or si  # same interface: the reflection shortcuts of :455-475
        s, d = gonet.u32_ipv4(int(src[k])), gonet.u32_ipv4(int(dst[k]))
        pc, pt = _py_trace(eng, tid, si, s, di, d, int(proto[k]), int(sport[k]), int(dport[k]))
        cc, ct = _c_trace(acls, ifx, if_in, if_out, si, int(src[k]), di, int(dst[k]), int(proto[k]), int(sport[k]),
                          int(dport[k]))
        assert pc == cc and pt == ct, (k, pt, ct)


def test_world_histogram_counts_every_evaluation():
    """World.conn(hist=True) == a direct count over the C trace, including unresolved
    interfaces (one count) and nil ACLs (the "no ACL" slot); its total is the number of
    evaluations, between one and four per connection."""
    from vpp_amd import workloads as W
    from oracle.world import World
    w = W.config1(0, n_tuples=1 << 14)
    wd = World(w.engine, w.local_ifs, w.node_if, no_if_ips=[W.ip_u32("10.10.9.9")])
    rng = np.random.default_rng(5)
    src, dst, sport, dport, proto = fz.rand_tuples(rng, 20000, fz.ANCHORS + list(wd.local_ips))
    m = rng.random(len(src)) < 0.6
    src[m] = wd.local_ips[rng.integers(0, len(wd.local_ips), int(m.sum()))]
    conn, slot, hist = wd.conn(src, dst, sport, dport, proto, threads=2, hist=True)
    sif, dif = wd.conn_ifs(src, dst)
    _, lt, li, evt, evi = fast.test_connection(wd.acls, wd.if_in, wd.if_out, sif, dif, src, dst, sport, dport, proto,
                                               2, trace=True)
    made = (evt != -3).sum(axis=1)
    assert made.min() >= 1 and made.max() <= 4 and int(hist.sum()) == int(made.sum())
    direct = np.zeros_like(hist)
    for t, i in zip(evt.ravel(), evi.ravel()):
        if t != -3:
            direct[wd.slots([t], [i])[0]] += 1
    assert np.array_equal(direct, hist)
    assert hist[wd.slot_unresolved] == int((conn == 3).sum() - ((lt >= -1) & (conn == 3)).sum())
    # the deciding evaluation is the last one made
    last = evt[np.arange(len(src)), made - 1]
    assert np.array_equal(last, lt)
