"""VPPTCP renderer + VPP session-rule tables: the renderer cache's second
consumer (IngressOrientation), rendering ContivRule tables as VPP session rules.

* The 6 vpptcp_renderer_test.go scenarios (97 assertions: request / error counts, rule counts,
  HasRule; restated by tests/golden/make_vpptcp_golden.py) replayed against the product (C++
  behind the C ABI) and against the oracle restatement.
* Random transaction sequences (adds, updates, pod removals, ANY-protocol and deny-all rules,
  IPv6 networks, resyncs after renderer restarts, small channel bursts): after every commit
  the product's session-rule tables equal the oracle's rule for rule (all fields incl. tag),
  with the same request / error counts and commit outcome.
* ExportSessionRules on random rule lists, global and local: product == oracle.
* Configurator -> VPPTCP renderer: the programmed tables equal the oracle chain's.
No GPU: the reference classifies nothing on this path (the session-rule lookup is VPP's).
"""
import random

import pytest

import kat_driver as kd
from oracle import configurator as OC
from oracle import gonet
from oracle import policy as OP
from oracle import vpptcp as OV
from test_configurator import ora_policy, product_policy, rand_scenario
from vpp_amd import configurator as CF
from vpp_amd import renderer as R
from vpp_amd import vpptcp as V

FIX = kd.load("vpptcp_kats.json")


def pod_str(p):
    return "%s/%s" % tuple(p)


# --- backends -----------------------------------------------------------------------------
class Product:
    def __init__(self):
        self.vpp = V.MockSessionRules()
        self.ipv4net = V.MockIPv4Net()
        self.r = None

    def appns(self, pod, idx):
        self.ipv4net.SetPodAppNsIndex(pod, idx)

    def clear(self):
        self.vpp.Clear()

    def renderer(self, buf):
        self.r = V.Renderer(V.Deps(IPv4Net=self.ipv4net, GoVPPChan=self.vpp.NewVPPChan(), GoVPPChanBufSize=buf))
        self.r.Init()

    @staticmethod
    def rule(x):
        a, s, d, p, sp, dp = x
        return R.ContivRule(a, s or None, d or None, p, sp, dp)

    def txn(self, resync, renders):
        t = self.r.NewTxn(resync)
        for pod, ip, ing, eg, removed in renders:
            t.Render(pod, V.GetOneHostSubnet(ip) if ip else None, [self.rule(x) for x in ing],
                     [self.rule(x) for x in eg], removed)
        return t.Commit() is None

    def counts(self):
        return self.vpp.GetReqCount(), self.vpp.GetErrCount()

    def table(self, scope, ns):
        t = self.vpp.LocalTable(ns) if scope == "local" else self.vpp.GlobalTable()
        return t

    def num_rules(self, scope, ns):
        return self.table(scope, ns).NumOfRules()

    def has_rule(self, scope, ns, args):
        return self.table(scope, ns).HasRule(*args)

    def rules(self, scope, ns):
        return [(r.TransportProto, r.IsIP4, r.LclIP, r.LclPlen, r.RmtIP, r.RmtPlen, r.LclPort, r.RmtPort,
                 r.ActionIndex, r.AppnsIndex, r.Scope, r.Tag) for r in self.table(scope, ns).Rules()]


def ora_net(s):
    """The product's pg_ipnet -> net.IPNet conversion: address as written (4 bytes for IPv4)."""
    if not s:
        return gonet.IPNet()
    addr, _, plen = s.partition("/")
    ip = gonet.parse_ip(addr)
    v4 = gonet.to4(ip)
    if v4 is not None and ":" not in addr:
        return gonet.IPNet(v4, gonet.cidr_mask(int(plen), 32))
    return gonet.IPNet(gonet.to16(ip), gonet.cidr_mask(int(plen), 128))


class Oracle:
    def __init__(self):
        self.vpp = OV.SessionRuleTables()
        self.ipv4net = OV.IPv4Net()
        self.r = None

    def appns(self, pod, idx):
        self.ipv4net.set_pod_app_ns_index(pod_str(pod), idx)

    def clear(self):
        self.vpp.clear()

    def renderer(self, buf):
        self.r = OV.Renderer(self.ipv4net, self.vpp, buf)

    @staticmethod
    def rule(x):
        a, s, d, p, sp, dp = x
        return OP.ContivRule(a, ora_net(s), ora_net(d), p, sp, dp)

    def txn(self, resync, renders):
        t = self.r.new_txn(resync)
        for pod, ip, ing, eg, removed in renders:
            t.render(pod_str(pod), gonet.one_host_subnet(ip) if ip else None, [self.rule(x) for x in ing],
                     [self.rule(x) for x in eg], removed)
        return t.commit() is None

    def counts(self):
        return self.vpp.req_count, self.vpp.err_count

    def num_rules(self, scope, ns):
        t = self.vpp.table(OV.SCOPE_LOCAL if scope == "local" else OV.SCOPE_GLOBAL, ns)
        return 0 if t is None else len(t)

    def has_rule(self, scope, ns, args):
        return self.vpp.has_rule(OV.SCOPE_LOCAL if scope == "local" else OV.SCOPE_GLOBAL, ns, *args)

    def rules(self, scope, ns):
        t = self.vpp.table(OV.SCOPE_LOCAL if scope == "local" else OV.SCOPE_GLOBAL, ns) or []
        return [r.key() for r in t]


def run_kats(backend, sc):
    bad = []
    for st in sc["steps"]:
        op = st["op"]
        if op == "appns":
            backend.appns(st["pod"], st["index"])
        elif op == "clear":
            backend.clear()
        elif op == "renderer":
            backend.renderer(st["buf"])
        elif op == "txn":
            backend.txn(st["resync"], st["render"])
        else:
            w = st["what"]
            if w == "err_count":
                got = backend.counts()[1]
            elif w == "req_count":
                got = backend.counts()[0]
            elif w == "num_rules":
                got = backend.num_rules(st["scope"], st["ns"])
            else:
                got = backend.has_rule(st["scope"], st["ns"], st["args"])
            if got != st["value"]:
                bad.append((st["line"], w, got, st["value"]))
    return bad


SC = FIX["scenarios"]


def test_kat_count():
    assert FIX["n_checks"] == 97
    assert sum(1 for s in SC for st in s["steps"] if st["op"] == "expect") == 97


@pytest.mark.parametrize("sc", SC, ids=[s["name"] for s in SC])
def test_vpptcp_kats_product(sc):
    assert run_kats(Product(), sc) == []


@pytest.mark.parametrize("sc", SC, ids=[s["name"] for s in SC])
def test_vpptcp_kats_oracle(sc):
    assert run_kats(Oracle(), sc) == []


# --- random parity ----------------------------------------------------------------------------
NETS4 = ["10.0.0.0/8", "10.1.0.0/16", "10.1.2.0/24", "192.168.2.0/24", "192.168.1.1/32", "192.168.1.2/32",
         "10.1.2.3/8", "0.0.0.0/0", "128.0.0.0/1"]
NETS6 = ["fd00::/8", "fd00:1::/64", "::ffff:10.0.0.0/104", "2001:db8::1/128"]


def rand_rule(rnd, direction):
    nets = NETS4 + NETS6 if rnd.random() < 0.15 else NETS4
    net = rnd.choice(nets + [""] * 3)
    proto = rnd.choice([0, 0, 1, 1, 3, 3, 2])
    port = rnd.choice([0, 0, 22, 53, 80, 443]) if proto in (0, 1) else 0
    sport = rnd.choice([0, 0, 0, 1234]) if proto in (0, 1) else 0
    action = rnd.choice([0, 1])
    # ingress rules (vswitch point of view) carry the destination, egress rules the source
    return [action, "", net, proto, sport, port] if direction == 0 else [action, net, "", proto, sport, port]


def rand_sequence(rnd):
    pods = [("default", "pod%d" % i) for i in range(rnd.randint(1, 5))]
    ips = {p: "192.168.1.%d" % (i + 1) for i, p in enumerate(pods)}
    steps = [("appns", p, 10 + 5 * i) for i, p in enumerate(pods) if rnd.random() < 0.9]
    steps.append(("renderer", rnd.choice([0, 0, 1, 2, 5])))
    for _ in range(rnd.randint(2, 6)):
        if rnd.random() < 0.25:
            steps.append(("renderer", rnd.choice([0, 3])))  # restart; the next txn resyncs
            resync = True
        else:
            resync = rnd.random() < 0.15
        renders = []
        # a resync txn renders every pod: a pod left out (or removed) whose table the resync
        # imported from VPP has a nil PodIP and the reference panics (oracle ReferencePanic)
        for p in (pods if resync else rnd.sample(pods, rnd.randint(1, len(pods)))):
            removed = rnd.random() < 0.15 and not resync
            ing = [rand_rule(rnd, 0) for _ in range(rnd.randint(0, 4))] if not removed else []
            eg = [rand_rule(rnd, 1) for _ in range(rnd.randint(0, 4))] if not removed else []
            renders.append([list(p), ips[p] if not removed or rnd.random() < 0.5 else None, ing, eg, removed])
        steps.append(("txn", resync, renders))
    return pods, steps


def snapshot(b, ns_list):
    return {"counts": b.counts(), "global": sorted(b.rules("global", 0)),
            "local": {ns: sorted(b.rules("local", ns)) for ns in ns_list}}


@pytest.mark.parametrize("seed", range(40))
def test_random_sequences_product_equals_oracle(seed):
    rnd = random.Random(seed)
    _, steps = rand_sequence(rnd)
    prod, ora = Product(), Oracle()
    ns_list = [10 + 5 * i for i in range(6)]
    for st in steps:
        if st[0] == "appns":
            prod.appns(st[1], st[2])
            ora.appns(st[1], st[2])
        elif st[0] == "renderer":
            prod.renderer(st[1])
            ora.renderer(st[1])
        else:
            try:
                ok_o = ora.txn(st[1], st[2])
            except OP.ReferencePanic:
                # e.g. after a failed resync commit the cache keeps the imported pods' nil
                # PodIPs and the next commit panics in the reference: unpinned from here on
                break
            ok_p = prod.txn(st[1], st[2])
            assert ok_p == ok_o, st
            assert snapshot(prod, ns_list) == snapshot(ora, ns_list), st


def test_resync_removed_pod_reference_panics_product_defined():
    """A pod whose local table a resync imported from VPP and which the resync txn does not
    render: the reference dereferences its nil PodIP in Commit (Go panic). The oracle raises
    ReferencePanic; the product removes the pod's session rules (treating the IP as unset)."""
    prod, ora = Product(), Oracle()
    pod1, pod2 = ("default", "pod1"), ("default", "pod2")
    rule = [0, "", "10.0.0.0/8", 0, 0, 22]
    rule2 = [0, "", "10.0.0.0/8", 0, 0, 23]  # distinct tables: identical ones share one on import
    for b in (prod, ora):
        b.appns(pod1, 10)
        b.appns(pod2, 15)
        b.renderer(0)
        assert b.txn(False, [[list(pod1), "192.168.1.1", [rule], [], False],
                             [list(pod2), "192.168.1.2", [rule2], [], False]])
        b.renderer(0)
    with pytest.raises(OP.ReferencePanic):
        ora.txn(True, [[list(pod1), "192.168.1.1", [rule], [], False]])
    assert prod.txn(True, [[list(pod1), "192.168.1.1", [rule], [], False]])
    assert prod.num_rules("local", 15) == 0 and prod.num_rules("local", 10) == 1


@pytest.mark.parametrize("seed", range(20))
def test_export_session_rules_product_equals_oracle(seed):
    rnd = random.Random(1000 + seed)
    pv, ov = V.MockIPv4Net(), OV.IPv4Net()
    pv.SetPodAppNsIndex(("default", "pod1"), 7)
    ov.set_pod_app_ns_index("default/pod1", 7)
    for glob in (True, False):
        rules = [rand_rule(rnd, 1 if glob else 0) for _ in range(rnd.randint(0, 12))]
        if glob:  # global-table rules: destination = a pod
            for x in rules:
                x[2] = rnd.choice(["192.168.1.1/32", "192.168.1.2/32", "", "fd00::1/128"])
        pod = None if glob else ("default", rnd.choice(["pod1", "pod1", "ghost"]))
        got = V.ExportSessionRules([Product.rule(x) for x in rules], pod, V.GetOneHostSubnet("192.168.1.2"), pv)
        want = OV.export_session_rules([Oracle.rule(x) for x in rules], None if glob else pod_str(pod),
                                       gonet.one_host_subnet("192.168.1.2").ip, ov)
        assert [(r.TransportProto, r.IsIP4, r.LclIP, r.LclPlen, r.RmtIP, r.RmtPlen, r.LclPort, r.RmtPort,
                 r.ActionIndex, r.AppnsIndex, r.Scope, r.Tag) for r in got] == [r.key() for r in want]


def test_add_del_refusals_match_oracle():
    """session_rule_add_del replies: bad tag, duplicate add, unknown delete."""
    from vpp_amd import _capi
    import ctypes as C
    vpp, ora = V.MockSessionRules(), OV.SessionRuleTables()
    r = _capi.pg_session_rule()
    r.transport_proto, r.is_ip4, r.rmt_plen, r.action_index, r.scope = 0, 1, 8, OV.ACTION_DENY, OV.SCOPE_GLOBAL
    r.rmt_ip[0] = 10
    o = OV.SessionRule()
    o.transport_proto, o.is_ip4, o.rmt_plen, o.action_index, o.scope = 0, 1, 8, OV.ACTION_DENY, OV.SCOPE_GLOBAL
    o.rmt_ip[0] = 10
    seq = [("bad-tag", True), ("contiv/vpp-policy", True), ("contiv/vpp-policy-X", True),
           ("contiv/vpp-policy-X", False), ("contiv/vpp-policy", False), ("contiv/vpp-policy", False)]
    for tag, add in seq:
        # Go copies the tag into a zeroed [64]byte (a ctypes char-array store keeps old tail bytes)
        C.memset(C.addressof(r) + _capi.pg_session_rule.tag.offset, 0, 64)
        r.tag = tag.encode()
        o.set_tag(tag)
        assert _capi.lib.pg_session_rule_add_del(vpp.h, C.byref(r), int(add)) == ora.add_del(o, add), (tag, add)
        assert (vpp.GetReqCount(), vpp.GetErrCount()) == (ora.req_count, ora.err_count)


@pytest.mark.parametrize("seed", range(6))
def test_configurator_into_vpptcp_renderer(seed):
    """configurator -> VPPTCP renderer: the programmed session-rule tables equal the oracle
    chain's (oracle configurator -> oracle VPPTCP renderer)."""
    rnd = random.Random(300 + seed)
    sc = rand_scenario(rnd)
    pods = [p for p, ip in sc["pods"].items() if ip]
    idx = {p: 20 + i for i, p in enumerate(sorted(pods))}
    # product
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
    # oracle
    ovpp, oip = OV.SessionRuleTables(), OV.IPv4Net()
    for p, i in idx.items():
        oip.set_pod_app_ns_index(p, i)
    ocfg = OC.PolicyConfigurator({p: ip for p, ip in sc["pods"].items() if ip is not None}, sc["nat"])
    ocfg.renderers.append(OV.Renderer(oip, ovpp))
    otxn = ocfg.new_txn(sc["txn"]["resync"])
    for pod, plist in sc["txn"]["configure"]:
        otxn.configure(pod, [ora_policy(sc["policies"][v]) for v in plist])
    otxn.commit()

    def prod_rules(t):
        return sorted((x.TransportProto, x.IsIP4, x.LclIP, x.LclPlen, x.RmtIP, x.RmtPlen, x.LclPort, x.RmtPort,
                       x.ActionIndex, x.AppnsIndex, x.Scope, x.Tag) for x in t.Rules())

    assert (vpp.GetReqCount(), vpp.GetErrCount()) == (ovpp.req_count, ovpp.err_count)
    assert prod_rules(vpp.GlobalTable()) == sorted(x.key() for x in ovpp.glob)
    for p, i in idx.items():
        assert prod_rules(vpp.LocalTable(i)) == sorted(x.key() for x in (ovpp.local.get(i) or [])), p
