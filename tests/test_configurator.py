"""Policy configurator and mock renderer TestTraffic (§8 a13).

* The 10 configurator_test.go scenarios (174 TestTraffic + GetPodIP assertions, restated by
  tests/golden/make_configurator_golden.py) replayed against the product (C++ configurator +
  mock renderer behind the C ABI) and against the oracle restatement.
* Random policy sets (pods, IPBlocks with nested excepts, ports, nil vs. empty): the product's
  rendered lists equal the oracle's rule for rule, and TestTraffic agrees on random traffic.
* Configurator -> GPU ACL renderer: the ACLs the product installs equal those of the oracle
  configurator feeding the oracle ACL renderer.
"""
import random

import pytest

import kat_driver as kd
from oracle import configurator as OC
from oracle import gonet
from test_renderer_host import oracle_acls, product_acls
from vpp_amd import configurator as CF
from vpp_amd import renderer as R

FIX = kd.load("configurator_kats.json")["scenarios"]
ENUM = {"PolicyIngress": 0, "PolicyEgress": 1, "PolicyAll": 2, "MatchIngress": 0, "MatchEgress": 1, "TCP": 0, "UDP": 1}
TRAFFIC = {"IngressTraffic": 0, "EgressTraffic": 1}
EXPECT = {"DeniedTraffic": 0, "AllowedTraffic": 1, "UnmatchedTraffic": 2}


def ora_policy(p):
    return {"id": p["id"], "type": ENUM[p["type"]] if isinstance(p["type"], str) else p["type"],
            "matches": [{"type": ENUM[m["type"]] if isinstance(m["type"], str) else m["type"], "pods": m["pods"],
                         "blocks": m["blocks"],
                         "ports": [{"protocol": ENUM[x["protocol"]] if isinstance(x["protocol"], str)
                                    else x["protocol"], "number": x["number"]} for x in m["ports"]]}
                        for m in p["matches"]]}


def product_policy(p):
    p = ora_policy(p)
    return CF.ContivPolicy(p["id"], p["type"], [
        CF.Match(m["type"], Pods=m["pods"],
                 IPBlocks=None if m["blocks"] is None else [CF.IPBlock(b["network"], b["except"]) for b in m["blocks"]],
                 Ports=[CF.Port(x["protocol"], x["number"]) for x in m["ports"]]) for m in p["matches"]])


def run_product(sc):
    cfg = CF.PolicyConfigurator()
    for pod, ip in sc["pods"].items():
        if ip is not None:
            cfg.AddPodConfig(pod, ip)
    cfg.SetNatLoopbackIP(sc["nat"])
    mocks = {}
    for r in sc["renderers"]:
        mocks[r] = CF.MockRenderer(r)
        assert cfg.RegisterRenderer(mocks[r]) is None
    txn = cfg.NewTxn(sc["txn"]["resync"])
    for pod, plist in sc["txn"]["configure"]:
        txn.Configure(pod, [product_policy(sc["policies"][v]) for v in plist])
    assert txn.Commit() is None
    return cfg, mocks


def run_oracle(sc):
    cfg = OC.PolicyConfigurator({p: ip for p, ip in sc["pods"].items() if ip is not None}, sc["nat"])
    mocks = {}
    for r in sc["renderers"]:
        mocks[r] = OC.MockRenderer()
        cfg.renderers.append(mocks[r])
    txn = cfg.new_txn(sc["txn"]["resync"])
    for pod, plist in sc["txn"]["configure"]:
        txn.configure(pod, [ora_policy(sc["policies"][v]) for v in plist])
    txn.commit()
    return cfg, mocks


@pytest.mark.parametrize("sc", FIX, ids=[s["name"] for s in FIX])
def test_configurator_kats_product(sc):
    _, mocks = run_product(sc)
    for r, pod, ip, ml in sc["pod_ip"]:
        assert mocks[r].GetPodIP(pod) == (ip, ml)
    for t in sc["traffic"]:
        got = mocks[t["renderer"]].TestTraffic(t["pod"], TRAFFIC[t["direction"]], t["src"], t["dst"],
                                               kd.PROTO[t["proto"]], t["sport"], t["dport"])
        assert got == EXPECT[t["expect"]], "configurator_test.go:%d" % t["line"]


@pytest.mark.parametrize("sc", FIX, ids=[s["name"] for s in FIX])
def test_configurator_kats_oracle(sc):
    _, mocks = run_oracle(sc)
    for r, pod, ip, ml in sc["pod_ip"]:
        assert mocks[r].get_pod_ip(pod) == (ip, ml)
    for t in sc["traffic"]:
        got = mocks[t["renderer"]].test_traffic(t["pod"], TRAFFIC[t["direction"]], t["src"], t["dst"],
                                                kd.PROTO[t["proto"]], t["sport"], t["dport"])
        assert got == EXPECT[t["expect"]], "configurator_test.go:%d" % t["line"]


def test_kat_count():
    assert sum(len(s["traffic"]) for s in FIX) == 174


def rule_str(r):
    """ContivRule.String (api.go:81-101) of a product or oracle rule"""
    if isinstance(r, R.ContivRule):
        net = lambda n: "ANY" if not n.family else repr(n)  # noqa: E731
        return (r.Action, net(r.SrcNetwork), net(r.DestNetwork), r.Protocol, r.SrcPort, r.DestPort)
    net = lambda n: "ANY" if n.is_empty() else gonet.ipnet_string(n)  # noqa: E731
    return (r.action, net(r.src), net(r.dst), r.protocol, r.src_port, r.dst_port)


def rand_scenario(rnd):
    pods = {}
    for k in range(rnd.randint(2, 7)):
        x = rnd.random()  # mostly addressed pods; some known without an address, some unknown
        pods["ns%d/p%d" % (k % 2, k)] = "10.1.%d.%d" % (k // 4, k + 1) if x > 0.2 else ("" if x > 0.1 else None)
    pods["ns1/ghost"] = None  # referenced by policies, not in the cache
    names = list(pods)

    def block():
        base = rnd.choice(["10.0.0.0/8", "10.1.0.0/16", "192.168.0.0/16", "172.16.0.0/12"])
        n = gonet.parse_cidr(base)[1]
        ex = []
        for _ in range(rnd.randint(0, 3)):
            plen = rnd.randint(gonet.mask_size(n.mask)[0] + 1, 32)
            ip = gonet.ipv4_u32(n.ip) | rnd.getrandbits(32 - gonet.mask_size(n.mask)[0]) if plen < 33 else 0
            ip &= (0xFFFFFFFF << (32 - plen)) & 0xFFFFFFFF
            ex.append("%d.%d.%d.%d/%d" % (ip >> 24, ip >> 16 & 255, ip >> 8 & 255, ip & 255, plen))
        return {"network": base, "except": ex}

    policies = {}
    for i in range(rnd.randint(1, 5)):
        matches = []
        ptype = rnd.choice([0, 1, 2])
        for _ in range(rnd.randint(0, 3)):
            mtype = rnd.choice([0, 1])
            pods_v = rnd.choice([None, [], rnd.sample(names, rnd.randint(1, len(names)))])
            blocks = rnd.choice([None, [], [block() for _ in range(rnd.randint(1, 2))]])
            ports = [{"protocol": rnd.choice([0, 1]), "number": rnd.choice([0, 22, 53, 80, 443, 8080])}
                     for _ in range(rnd.choice([0, 0, 1, 2, 3]))]
            matches.append({"type": mtype, "pods": pods_v, "blocks": blocks, "ports": ports})
        policies["pol%d" % i] = {"id": "ns%d/policy%d" % (i % 2, i), "type": ptype, "matches": matches}
    configure = [[p, rnd.sample(list(policies), rnd.randint(0 if rnd.random() < 0.2 else 1, len(policies)))]
                 for p in rnd.sample(names, rnd.randint(1, len(names)))]
    return {"pods": pods, "nat": "10.1.255.254", "policies": policies, "renderers": ["m"],
            "txn": {"resync": rnd.random() < 0.5, "configure": configure}}


@pytest.mark.parametrize("seed", range(25))
def test_random_policies_product_equals_oracle(seed):
    rnd = random.Random(seed)
    sc = rand_scenario(rnd)
    _, pm = run_product(sc)
    _, om = run_oracle(sc)
    pm, om = pm["m"], om["m"]
    assert sorted(om.config) == sorted(p for p in sc["pods"] if pm.Rules(p, 0) is not None)
    for pod in om.config:
        for d in (0, 1):
            assert [rule_str(r) for r in pm.Rules(pod, d)] == [rule_str(r) for r in om.config[pod][1 + d]]
        assert pm.GetPodIP(pod) == om.get_pod_ip(pod)
    ips = ["10.1.0.1", "10.1.0.2", "10.1.1.5", "10.2.3.4", "192.168.7.1", "172.20.0.1", "8.8.8.8", "10.1.255.254"]
    for _ in range(300):
        pod = rnd.choice(list(sc["pods"]))
        q = (pod, rnd.choice([0, 1]), rnd.choice(ips), rnd.choice(ips), rnd.choice([0, 1, 2, 3]),
             rnd.choice([0, 22, 1000]), rnd.choice([0, 22, 53, 80, 443, 8080, 9999]))
        assert pm.TestTraffic(*q) == om.test_traffic(*q), q


@pytest.mark.parametrize("seed", range(6))
def test_configurator_into_gpu_renderer(seed):
    """configurator -> ACL renderer -> engine: the installed ACLs equal the oracle chain's."""
    rnd = random.Random(100 + seed)
    sc = rand_scenario(rnd)
    sc["txn"]["resync"] = True
    local = [p for p, ip in sc["pods"].items() if ip]
    setup = {"pod_ifs": {p: "tap-%d" % i for i, p in enumerate(local)}, "host_interconnect": "VPP-Host",
             "main_if": "GbE", "other_ifs": [], "vxlan_bvi": "VXLAN-BVI",
             "pods": [(p, ip, False) for p, ip in sc["pods"].items() if ip]}
    # product: configurator registered with the GPU renderer
    prod = kd.ProductBackend(gpu=False)
    prod.setup(setup)
    cfg = CF.PolicyConfigurator()
    for pod, ip in sc["pods"].items():
        if ip is not None:
            cfg.AddPodConfig(pod, ip)
    cfg.SetNatLoopbackIP(sc["nat"])
    assert cfg.RegisterRenderer(prod.renderer) is None
    txn = cfg.NewTxn(True)
    for pod, plist in sc["txn"]["configure"]:
        txn.Configure(pod, [product_policy(sc["policies"][v]) for v in plist])
    assert txn.Commit() is None
    # oracle: oracle configurator -> mock lists -> oracle ACL renderer
    ocfg, om = run_oracle(sc)
    ora = kd.OracleBackend()
    ora.setup(setup)

    def d(r):
        net = lambda n: "" if n.is_empty() else gonet.ipnet_string(n)  # noqa: E731
        return {"action": "PERMIT" if r.action else "DENY", "src": net(r.src), "dst": net(r.dst),
                "proto": {0: "TCP", 1: "UDP", 2: "OTHER", 3: "ANY"}[r.protocol], "sport": r.src_port,
                "dport": r.dst_port}
    renders = [{"pod": p, "ip": gonet.ip_string(c[0].ip), "ingress": [d(r) for r in c[1]],
                "egress": [d(r) for r in c[2]], "removed": False} for p, c in sorted(om["m"].config.items())]
    assert ora.txn(True, renders) is None
    o, p = oracle_acls(ora.engine), product_acls(prod.engine)
    assert sorted(o) == sorted(p)
    for name in o:
        assert o[name] == p[name], name
