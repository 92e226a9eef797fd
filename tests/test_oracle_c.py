"""Pin the C oracle (oracle/oracle.c) to the Python oracle (itself pinned by the reference's
KATs) on randomised ACLs covering every evalACL branch, and on the KAT scenarios."""
import random

import numpy as np
import pytest

import acl_fuzz as fz
import kat_driver as kd
from oracle import fast


@pytest.mark.parametrize("seed", range(6))
def test_c_oracle_matches_python_oracle_random(seed):
    rnd = random.Random(seed)
    rules = fz.rand_acl(rnd, rnd.randint(1, 40), fz.ANCHORS, weird=True, tail=rnd.choice([None, "deny"]))
    src, dst, sport, dport, proto = fz.rand_tuples(np.random.default_rng(seed), 3000, fz.ANCHORS, any_pct=0.05)
    pa, pi = fz.py_eval(fz.to_oracle_acl("x", rules), src, dst, dport, proto)
    ca, ci = fast.eval_acl(fast.OraACL(rules), src, dst, dport, proto, threads=4)
    fa, fi = fast.eval_acl_faithful(rules, src, dst, dport, proto)
    assert (pa == ca).all() and (pi == ci).all()
    assert (pa == fa).all() and (pi == fi).all()


def test_c_oracle_nil_acl_permits():
    src = np.arange(10, dtype=np.uint32)
    a, i = fast.eval_acl(None, src, src, src.astype(np.uint16), np.zeros(10, np.uint8))
    assert (a == 1).all() and (i == -1).all()


def test_c_oracle_test_connection_matches_python_kats():
    """Replay acl_renderer_test.go phases: Connection* verdicts from the C testConnection
    over the oracle engine's installed ACLs equal the expected ones."""
    from oracle import gonet
    for sc in kd.load("acl_renderer_kats.json"):
        ob = kd.OracleBackend()
        ob.setup(sc["setup"])
        for phase in sc["phases"]:
            for st in phase["steps"]:
                if st["op"] == "restart":
                    ob.restart()
                else:
                    ob.txn(st["resync"], st["renders"])
            eng = ob.engine
            names = sorted(eng.cfg.by_name)
            acls = [fast.OraACL(_acl_dicts(eng.cfg.by_name[n])) for n in names]
            tid = {n: i for i, n in enumerate(names)}
            ifs = sorted(eng.cfg.by_if)
            ifx = {n: i for i, n in enumerate(ifs)}
            if_in = [tid[eng.cfg.by_if[n][0].name] if eng.cfg.by_if[n][0] else -1 for n in ifs] + [-1] * 16
            if_out = [tid[eng.cfg.by_if[n][1].name] if eng.cfg.by_if[n][1] else -1 for n in ifs] + [-1] * 16
            for c in phase["checks"]:
                if not c["kind"].startswith("Connection"):
                    continue
                # resolve endpoints like aclengine_mock.go:273-420
                a = c["args"]
                node = sc["setup"]["vxlan_bvi"] or sc["setup"]["main_if"]

                def ep(pod):
                    cfg = eng.pods[pod]
                    return (node if cfg.another_node else sc["setup"]["pod_ifs"][pod]), gonet.ipv4_u32(cfg.ip)
                if c["kind"] == "ConnectionPodToPod":
                    (si, s), (di, d) = ep(a[0]), ep(a[1])
                elif c["kind"] == "ConnectionPodToInternet":
                    (si, s), di, d = ep(a[0]), node, gonet.ipv4_u32(gonet.parse_ip(a[1]))
                else:
                    si, s, (di, d) = node, gonet.ipv4_u32(gonet.parse_ip(a[0])), ep(a[1])
                for n in (si, di):
                    if n not in ifx:
                        ifx[n] = len(ifx)
                conn, _, _ = fast.test_connection(acls, if_in, if_out, [ifx[si]], [ifx[di]], [s], [d], [a[3]],
                                                  [a[4]], [kd.PROTO[a[2]]])
                assert conn[0] == kd.CONN[c["expect"]], (sc["name"], c)


def _acl_dicts(acl):
    out = []
    for r in acl.rules:
        d = {"action": r.action, "src": r.src_network, "dst": r.dst_network}
        for f in ("tcp", "udp"):
            s = getattr(r, f)
            if s is not None:
                d[f] = {"src": [s.src_range.lower, s.src_range.upper], "dst": [s.dst_range.lower, s.dst_range.upper]}
        out.append(d)
    return out


@pytest.mark.parametrize("seed", range(4))
def test_faithful_conn_and_perpod_equal_the_preparsed_ones(seed):
    """The reference-faithful testConnection / per-pod evalACL (CIDR strings parsed per rule
    visit, aclengine_mock.go:535, 549; bench.py's reference-shaped CPU baseline of configs 3 and 5)
    give the pre-parsed oracle's verdicts, tables and indices on random topologies: weird rules,
    nil ACLs, unresolved interfaces, every protocol."""
    rnd = random.Random(100 + seed)
    rng = np.random.default_rng(seed)
    acls = [fast.OraACL(fz.rand_acl(rnd, rnd.randint(1, 30), fz.ANCHORS, weird=True,
                                    tail=rnd.choice([None, "deny", "permit"]))) for _ in range(5)]
    n_if = 7
    if_in = rng.integers(-1, len(acls), n_if).astype(np.int32)
    if_out = rng.integers(-1, len(acls), n_if).astype(np.int32)
    src, dst, sport, dport, proto = fz.rand_tuples(rng, 5000, fz.ANCHORS, any_pct=0.05)
    sif = rng.integers(-1, n_if, len(src)).astype(np.int32)
    dif = rng.integers(-1, n_if, len(src)).astype(np.int32)
    ref = fast.test_connection(acls, if_in, if_out, sif, dif, src, dst, sport, dport, proto, threads=2)
    got = fast.test_connection(acls, if_in, if_out, sif, dif, src, dst, sport, dport, proto, faithful=True)
    for r, g in zip(ref, got):
        assert np.array_equal(r, g)
    ref = fast.perpod(acls, if_out, dif, src, dst, dport, proto, threads=2)
    got = fast.perpod(acls, if_out, dif, src, dst, dport, proto, faithful=True)
    for r, g in zip(ref, got):
        assert np.array_equal(r, g)
