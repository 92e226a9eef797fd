"""§8 f4 on the device: VPP's session-rule lookup over the tables the VPPTCP renderer programs
(IngressOrientation ContivRule tables -> convertContivRule, session_rule.go:263-361),
installed with pg_session_table_install and classified by k_classify (SINGLE mode), against
oracle/vpptcp.py session_lookup (the most specific matching rule, found directly rather than
by the product's sort + first match).

VPP's own lookup is not in the reference: parity is unpinned beyond that restatement (DESIGN.md
§2). The tables come from the product renderer; that they equal the oracle renderer's tables
is pinned separately (tests/test_vpptcp.py: 97 vpptcp_renderer_test.go assertions, random
sequences, configurator chain).

The CPU tests run the kernels' per-tuple code on the host (pg_debug_classify_host); the GPU
test runs k_classify."""
import random

import numpy as np
import pytest

from oracle import configurator as OC
from oracle import policy as OP
from oracle import vpptcp as OV
from test_configurator import ora_policy, product_policy, rand_scenario
from test_vpptcp import Oracle, Product, rand_sequence
from vpp_amd import configurator as CF
from vpp_amd import renderer as R
from vpp_amd import vpptcp as V


def _cfg_world(seed):
    """configurator scenario -> product VPPTCP renderer; -> (MockSessionRules, ns indices)"""
    rnd = random.Random(700 + seed)
    sc = rand_scenario(rnd)
    pods = [p for p, ip in sc["pods"].items() if ip]
    idx = {p: 20 + i for i, p in enumerate(sorted(pods))}
    vpp, ipv4net = V.MockSessionRules(), V.MockIPv4Net()
    for p, i in idx.items():
        ipv4net.SetPodAppNsIndex(p, i)
    r = V.Renderer(V.Deps(IPv4Net=ipv4net, GoVPPChan=vpp.NewVPPChan()))
    r.Init()
    cfg = CF.PolicyConfigurator()
    for pod, ip in sc["pods"].items():
        if ip is not None:
            cfg.AddPodConfig(pod, ip)
    cfg.SetNatLoopbackIP(sc["nat"])
    assert cfg.RegisterRenderer(r) is None
    txn = cfg.NewTxn(sc["txn"]["resync"])
    for pod, plist in sc["txn"]["configure"]:
        txn.Configure(pod, [product_policy(sc["policies"][v]) for v in plist])
    assert txn.Commit() is None
    return vpp, sorted(idx.values()), (r, ipv4net)


def _seq_world(seed):
    """random renderer transactions (test_vpptcp.rand_sequence, source ports cleared: the
    renderer cache's rules never set one) -> (MockSessionRules, ns indices)"""
    rnd = random.Random(900 + seed)
    _, steps = rand_sequence(rnd)
    prod, ora = Product(), Oracle()
    for st in steps:
        if st[0] == "appns":
            prod.appns(st[1], st[2])
            ora.appns(st[1], st[2])
        elif st[0] == "renderer":
            prod.renderer(st[1])
            ora.renderer(st[1])
        else:
            for _, _, ing, eg, _ in st[2]:
                for x in ing + eg:
                    x[4] = 0
            try:
                ora.txn(st[1], st[2])
            except OP.ReferencePanic:
                break
            prod.txn(st[1], st[2])
    return prod.vpp, [10 + 5 * i for i in range(6)], prod


def _oracle_rules(vpp, scope, ns):
    """the product's table as oracle SessionRule records"""
    t = vpp.LocalTable(ns) if scope == V.ScopeLocal else vpp.GlobalTable()
    out = []
    for r in t.Rules():
        o = OV.SessionRule()
        o.transport_proto, o.is_ip4 = r.TransportProto, r.IsIP4
        o.lcl_ip, o.lcl_plen = bytearray(r.LclIP), r.LclPlen
        o.rmt_ip, o.rmt_plen = bytearray(r.RmtIP), r.RmtPlen
        o.lcl_port, o.rmt_port = r.LclPort, r.RmtPort
        o.action_index, o.appns_index, o.scope = r.ActionIndex, r.AppnsIndex, r.Scope
        o.set_tag(r.Tag)
        out.append(o)
    return out


def _inside(rng, ip, plen):
    if plen == 0:
        return int(rng.integers(0, 1 << 32))
    net = int.from_bytes(bytes(ip[:4]), "big")
    host = int(rng.integers(0, 1 << (32 - plen))) if plen < 32 else 0
    return ((net >> (32 - plen)) << (32 - plen) | host) & 0xFFFFFFFF


def _connections(rules, n, seed):
    """n connections (lcl ip, lcl port, rmt ip, rmt port, proto = renderer.Protocol): 70 %
    drawn inside a random rule's prefixes, on its port and protocol most of the time; the
    rest random"""
    rng = np.random.default_rng(seed)
    ports = [0, 22, 53, 80, 443, 1234, 8080]
    v4 = [r for r in rules if r.is_ip4 and r.lcl_plen <= 32 and r.rmt_plen <= 32]
    L = np.zeros((5, n), np.int64)
    for i in range(n):
        if v4 and rng.random() < 0.7:
            r = v4[int(rng.integers(0, len(v4)))]
            li, ri = _inside(rng, r.lcl_ip, r.lcl_plen), _inside(rng, r.rmt_ip, r.rmt_plen)
            lp = r.lcl_port if r.lcl_port and rng.random() < 0.8 else ports[int(rng.integers(0, len(ports)))]
            rp = r.rmt_port if r.rmt_port and rng.random() < 0.8 else ports[int(rng.integers(0, len(ports)))]
            pr = r.transport_proto if rng.random() < 0.9 else int(rng.choice([0, 1, 2]))
        else:
            li, ri = int(rng.integers(0, 1 << 32)), int(rng.integers(0, 1 << 32))
            lp, rp = ports[int(rng.integers(0, len(ports)))], int(rng.integers(0, 1 << 16))
            pr = int(rng.choice([0, 1, 2]))
        L[:, i] = (li, lp, ri, rp, pr)
    return L


def _acl_content(r, scope):
    """an oracle session rule as the ACL rule the product must have matched"""
    def net(ip, plen):
        return "" if plen == 0 else "%d.%d.%d.%d/%d" % (ip[0], ip[1], ip[2], ip[3], plen)
    lcl, rmt = net(r.lcl_ip, r.lcl_plen), net(r.rmt_ip, r.rmt_plen)
    glob = scope != V.ScopeLocal
    port = r.lcl_port if glob else r.rmt_port
    return (1 if r.action_index == OV.ACTION_ALLOW else 0, rmt if glob else lcl, lcl if glob else rmt,
            "udp" if r.transport_proto == 1 else "tcp", (port, port) if port else (0, 65535))


def _product_content(rule):
    sec = "udp" if rule["udp"] else "tcp"
    return (rule["action"], rule["src"], rule["dst"], sec, tuple(rule[sec]["dst"]))


def _check(e, tid, name, scope, rules, conns, got):
    acl = e.GetACLByName(name)
    assert len(acl["rules"]) == sum(1 for r in rules if r.is_ip4 and r.lcl_plen <= 32 and r.rmt_plen <= 32)
    base, dflt = e.slot_of_rule(tid, 0), e.slot_of_rule(tid, -1)
    act, slot = got >> 30, got & 0x3FFFFFFF
    bad = []
    for i in range(conns.shape[1]):
        li, lp, ri, rp, pr = (int(x) for x in conns[:, i])
        want = OV.session_lookup(rules, li, lp, ri, rp, pr)
        if want is None:
            ok = slot[i] == dflt and act[i] == 0
        else:
            k = int(slot[i]) - base
            ok = 0 <= k < len(acl["rules"]) and _product_content(acl["rules"][k]) == _acl_content(want, scope) \
                and act[i] == (1 if want.action_index == OV.ACTION_ALLOW else 0)
        if not ok:
            bad.append((i, li, lp, ri, rp, pr))
    assert not bad, bad[:5]


def _tables(vpp, ns_list):
    yield V.ScopeGlobal, 0
    for ns in ns_list:
        if vpp.LocalTable(ns).NumOfRules():
            yield V.ScopeLocal, ns


def _host_case(vpp, ns_list, seed, n=1500):
    e = R.Engine(0)
    checked = 0
    for scope, ns in _tables(vpp, ns_list):
        name = "session-%d-%d" % (scope, ns)
        tid = V.InstallSessionTable(e, vpp, scope, ns, name)
        rules = _oracle_rules(vpp, scope, ns)
        conns = _connections(rules, n, seed * 31 + ns)
        src, dst, dport = V.SessionTuples(scope, conns[0], conns[1], conns[2], conns[3])
        z = np.zeros(n, np.uint16)
        got = e.debug_classify_host(0, tid, src.astype(np.uint32), dst.astype(np.uint32), z,
                                    dport.astype(np.uint16), conns[4].astype(np.uint8))
        _check(e, tid, name, scope, rules, conns, got)
        checked += 1
    return checked


@pytest.mark.parametrize("seed", range(6))
def test_session_lookup_configurator_tables_host(seed):
    vpp, ns_list, _keep = _cfg_world(seed)
    assert _host_case(vpp, ns_list, seed) >= 1


@pytest.mark.parametrize("seed", range(10))
def test_session_lookup_random_renderer_tables_host(seed):
    vpp, ns_list, _keep = _seq_world(seed)
    assert _host_case(vpp, ns_list, 100 + seed) >= 1


def test_session_table_refusals():
    """a rule the first-match form cannot hold: a source port (LclPort of a local-table rule)
    -> PG_EINVAL, nothing installed"""
    p = Product()
    p.appns(("default", "pod1"), 10)
    p.renderer(0)
    assert p.txn(False, [[["default", "pod1"], "192.168.1.1", [[0, "", "10.0.0.0/8", 0, 1234, 22]], [], False]])
    e = R.Engine(0)
    with pytest.raises(R.PolicyError):
        V.InstallSessionTable(e, p.vpp, V.ScopeLocal, 10, "s")
    assert "s" not in e.ACLNames()


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(4))
def test_session_lookup_gpu(seed):
    """k_classify over every programmed table (configurator chain and random renderer
    transactions), 4096 connections each, against oracle session_lookup"""
    import torch
    from vpp_amd import device as D
    for vpp, ns_list, _keep in (_cfg_world(seed), _seq_world(seed)):
        e = R.Engine(0)
        for scope, ns in _tables(vpp, ns_list):
            name = "session-%d-%d" % (scope, ns)
            tid = V.InstallSessionTable(e, vpp, scope, ns, name)
            rules = _oracle_rules(vpp, scope, ns)
            n = 4096
            conns = _connections(rules, n, 5000 + seed * 31 + ns)
            src, dst, dport = V.SessionTuples(scope, conns[0], conns[1], conns[2], conns[3])
            b = D.TupleBatch.from_numpy(src.astype(np.uint32), dst.astype(np.uint32), np.zeros(n, np.uint16),
                                        dport.astype(np.uint16), conns[4].astype(np.uint8))
            out = torch.empty(n, dtype=torch.int32, device="cuda")
            D.classify(e, 0, tid, b, out)
            torch.cuda.synchronize()
            _check(e, tid, name, scope, rules, conns, out.cpu().numpy().view(np.uint32))
