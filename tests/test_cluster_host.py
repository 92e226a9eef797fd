"""Configs 3/5 topology (vpp_amd.workloads cluster: namespaces x apps, label-selector-shaped
rule lists, pods on this and another node) at a reduced size, on the host:

  * the product renderer's installed ACLs equal the oracle renderer's (names = FNV IDs,
    rules, interfaces) for the whole cluster;
  * the bench/test glue ``oracle.world.World`` (C oracle over the engine's exported ACLs,
    IP -> interface resolution) equals the pure-Python oracle's Connection* on pod-to-pod,
    pod-to-internet and internet-to-pod connections, and its per-pod mode equals evalACL on
    the outbound ACL of the destination interface.
"""
import random

import numpy as np
import pytest

import kat_driver as kd
from test_renderer_host import oracle_acls, product_acls
from oracle import fast
from oracle.world import World
from vpp_amd import renderer as R
from vpp_amd import workloads as W

N_NS, PODS, APPS = 4, 10, 2


def _d(rule):
    name = {0: "TCP", 1: "UDP", 2: "OTHER", 3: "ANY"}
    net = lambda n: repr(n) if n.family else ""
    return {"action": "PERMIT" if rule.Action else "DENY", "src": net(rule.SrcNetwork), "dst": net(rule.DestNetwork),
            "proto": name[rule.Protocol], "sport": rule.SrcPort, "dport": rule.DestPort}


@pytest.fixture(scope="module")
def cluster():
    pods = W.cluster_pods(N_NS, PODS, APPS)
    ingress, egress = W.cluster_rules(pods, N_NS, APPS)
    pod_ifs = {p["id"]: "tap-%s" % p["id"].replace("/", "-") for p in pods if not p["remote"]}
    setup = {"pod_ifs": pod_ifs, "host_interconnect": "VPP-Host", "main_if": "GbE", "other_ifs": [],
             "vxlan_bvi": "VXLAN-BVI", "pods": [(p["id"], W.ip_str(p["ip"]), p["remote"]) for p in pods]}
    renders = [{"pod": p["id"], "ip": W.ip_str(p["ip"]), "ingress": [_d(x) for x in ingress[(p["ns"], p["app"])]],
                "egress": [_d(x) for x in egress[(p["ns"], p["app"])]], "removed": False}
               for p in pods if not p["remote"]]
    ora, prod = kd.OracleBackend(), kd.ProductBackend(gpu=False)
    for b in (ora, prod):
        b.setup(setup)
        assert b.txn(True, renders) is None
    return pods, pod_ifs, ora, prod


def test_cluster_acls_equal_oracle(cluster):
    pods, pod_ifs, ora, prod = cluster
    o, p = oracle_acls(ora.engine), product_acls(prod.engine)
    assert sorted(o) == sorted(p)
    for name in o:
        assert o[name] == p[name], name
    assert len(o) > 3


def test_world_connections_equal_python_oracle(cluster):
    pods, pod_ifs, ora, prod = cluster
    e = prod.engine
    local = {p["ip"]: pod_ifs[p["id"]] for p in pods if not p["remote"]}
    wd = World(e, local, "VXLAN-BVI")
    rnd = random.Random(7)
    inet = ["8.8.8.8", "192.168.10.5", "192.168.99.1", "10.96.0.10"]
    q, exp = [], []
    ids = {p["id"]: p for p in pods}
    for _ in range(1500):
        proto = rnd.choice([R.TCP, R.UDP, R.OTHER])
        sp, dp = rnd.choice([1000, 40000, 22]), rnd.choice(W.CLUSTER_PORTS + [7])
        kind = rnd.random()
        a, b = rnd.choice(pods), rnd.choice(pods)
        if kind < 0.6:
            exp.append(ora.engine.connection_pod_to_pod(a["id"], b["id"], proto, sp, dp))
            q.append((a["ip"], b["ip"], sp, dp, proto))
        elif kind < 0.8 and not a["remote"]:
            ip = rnd.choice(inet)
            exp.append(ora.engine.connection_pod_to_internet(a["id"], ip, proto, sp, dp))
            q.append((a["ip"], W.ip_u32(ip), sp, dp, proto))
        elif not b["remote"]:
            ip = rnd.choice(inet)
            exp.append(ora.engine.connection_internet_to_pod(ip, b["id"], proto, sp, dp))
            q.append((W.ip_u32(ip), b["ip"], sp, dp, proto))
    src, dst, sport, dport, proto = (np.array(x) for x in zip(*q))
    conn, slot = wd.conn(src, dst, sport, dport, proto, threads=4)
    assert conn.tolist() == exp
    assert {0, 2} <= set(exp), sorted(set(exp))  # both denied and allowed connections occur
    assert ids  # topology non-empty
    assert slot.max() < e.num_counter_slots()

    # per-pod mode: evalACL(outbound ACL of dst's interface)
    act, slot = wd.perpod(src, dst, dport, proto, threads=4)
    dif = wd.resolve(dst)
    names = wd.names
    for i in range(0, len(q), 7):
        t = wd.if_out[dif[i]]
        acl = fast.OraACL(e.GetACLByName(names[t])["rules"]) if t >= 0 else None
        a1, i1 = fast.eval_acl(acl, src[i:i + 1], dst[i:i + 1], dport[i:i + 1], proto[i:i + 1], threads=1)
        assert act[i] == a1[0]
        exp_slot = (e.slot_of_rule(e.table_id(names[t]), int(i1[0])) if t >= 0 else e.num_counter_slots() - 2)
        assert slot[i] == exp_slot


def test_cluster_via_configurator_equals_oracle_chain():
    """Configs 3/5 are built by the policy configurator from K8s-shaped policies
    (workloads.cluster_engine): at a reduced size, the ACLs it installs equal those of the
    oracle configurator feeding the oracle ACL renderer."""
    from oracle import configurator as OC
    from oracle import gonet
    pods = W.cluster_pods(N_NS, PODS, APPS)
    pols = W.cluster_policies(pods, N_NS, APPS)
    # product chain: the workload builder itself, at this size
    e = R.Engine(0)
    e.SetMainInterfaceName("GbE")
    e.SetVxlanBVIIfName("VXLAN-BVI")
    e.SetHostInterconnectIfName("VPP-Host")
    import vpp_amd.workloads as WW
    orig = WW._new_engine
    WW._new_engine = lambda device: e
    try:
        e2, _, local, _ = W.cluster_engine(0, N_NS, PODS, APPS)
    finally:
        WW._new_engine = orig
    assert e2 is e
    # oracle chain
    as_dict = lambda p: {  # noqa: E731
        "id": "%s/%s" % p.ID, "type": p.Type,
        "matches": [{"type": m.Type, "pods": None if m.Pods is None else ["%s/%s" % R._pod(x) for x in m.Pods],
                     "blocks": None if m.IPBlocks is None else [
                         {"network": repr(b.Network), "except": [repr(x) for x in b.Except]} for b in m.IPBlocks],
                     "ports": [{"protocol": x.Protocol, "number": x.Number} for x in m.Ports]} for m in p.Matches]}
    ocfg = OC.PolicyConfigurator({p["id"]: W.ip_str(p["ip"]) for p in pods}, W.NAT_LOOPBACK_IP)
    mock = OC.MockRenderer()
    ocfg.renderers.append(mock)
    t = ocfg.new_txn(True)
    for p in pods:
        if not p["remote"]:
            t.configure(p["id"], [as_dict(x) for x in pols[(p["ns"], p["app"])]])
    t.commit()
    pod_ifs = {p["id"]: "tap-%s" % p["id"].replace("/", "-") for p in pods if not p["remote"]}
    setup = {"pod_ifs": pod_ifs, "host_interconnect": "VPP-Host", "main_if": "GbE", "other_ifs": [],
             "vxlan_bvi": "VXLAN-BVI", "pods": [(p["id"], W.ip_str(p["ip"]), p["remote"]) for p in pods]}
    ora = kd.OracleBackend()
    ora.setup(setup)

    def d(r):
        net = lambda n: "" if n.is_empty() else gonet.ipnet_string(n)  # noqa: E731
        return {"action": "PERMIT" if r.action else "DENY", "src": net(r.src), "dst": net(r.dst),
                "proto": {0: "TCP", 1: "UDP", 2: "OTHER", 3: "ANY"}[r.protocol], "sport": r.src_port,
                "dport": r.dst_port}
    renders = [{"pod": p, "ip": gonet.ip_string(c[0].ip), "ingress": [d(r) for r in c[1]],
                "egress": [d(r) for r in c[2]], "removed": False} for p, c in sorted(mock.config.items())]
    assert ora.txn(True, renders) is None
    o, p = oracle_acls(ora.engine), product_acls(e)
    assert sorted(o) == sorted(p) and len(o) > 3
    for name in o:
        assert o[name] == p[name], name


def test_k8s_object_cluster_equals_oracle_chain():
    """The cluster given as K8s objects (workloads.cluster_k8s: label / namespace selectors,
    named ports, IPBlocks) through policy cache -> processor -> configurator -> ACL renderer
    (workloads.cluster_engine_k8s) installs the same ACLs as the oracle chain (oracle cache ->
    oracle processor -> oracle configurator -> oracle ACL renderer). SURVEY.md §8 f3."""
    from oracle import configurator as OC
    from oracle import gonet
    from oracle import k8s_policy as OK
    n_ns, pods_per_ns, apps = 4, 20, 5
    e = R.Engine(0)
    e.SetMainInterfaceName("GbE")
    e.SetVxlanBVIIfName("VXLAN-BVI")
    e.SetHostInterconnectIfName("VPP-Host")
    import vpp_amd.workloads as WW
    orig = WW._new_engine
    WW._new_engine = lambda device: e
    try:
        e2, _, local, _, keep = W.cluster_engine_k8s(0, n_ns, pods_per_ns, apps)
    finally:
        WW._new_engine = orig
    assert e2 is e
    pods, nss, pols = W.cluster_k8s(n_ns, pods_per_ns, apps)
    ocache = OK.PolicyCache()
    ocfg = OC.PolicyConfigurator({}, W.NAT_LOOPBACK_IP)
    mock = OC.MockRenderer()
    ocfg.renderers.append(mock)
    OK.PolicyProcessor(ocache, ocfg, W.NODE_POD_SUBNET)
    ocache.resync(pods, nss, pols)
    ids = ["%s/%s" % (p["Namespace"], p["Name"]) for p in pods]
    remote = {i: p["IpAddress"].startswith("10.2.") for i, p in zip(ids, pods)}
    assert sorted(mock.config) == sorted(i for i in ids if not remote[i])
    setup = {"pod_ifs": {i: "tap-%s" % i.replace("/", "-") for i in ids if not remote[i]},
             "host_interconnect": "VPP-Host", "main_if": "GbE", "other_ifs": [], "vxlan_bvi": "VXLAN-BVI",
             "pods": [(i, p["IpAddress"], remote[i]) for i, p in zip(ids, pods)]}
    ora = kd.OracleBackend()
    ora.setup(setup)

    def d(r):
        net = lambda n: "" if n.is_empty() else gonet.ipnet_string(n)  # noqa: E731
        return {"action": "PERMIT" if r.action else "DENY", "src": net(r.src), "dst": net(r.dst),
                "proto": {0: "TCP", 1: "UDP", 2: "OTHER", 3: "ANY"}[r.protocol], "sport": r.src_port,
                "dport": r.dst_port}
    renders = [{"pod": p, "ip": gonet.ip_string(c[0].ip), "ingress": [d(r) for r in c[1]],
                "egress": [d(r) for r in c[2]], "removed": False} for p, c in sorted(mock.config.items())]
    assert ora.txn(True, renders) is None
    o, p = oracle_acls(ora.engine), product_acls(e)
    assert sorted(o) == sorted(p) and len(o) > 3
    for name in o:
        assert o[name] == p[name], name
    assert sum(len(a["rules"]) for a in p.values()) > 1000


@pytest.mark.parametrize("node", [True, False])
def test_k8s_object_cluster_host_classify_equals_world(node):
    """pg_classify's per-tuple code run on the host (PERPOD and CONN, node classifier and
    per-table path) over the K8s-object cluster equals the C oracle through oracle.world."""
    from vpp_amd._capi import MODE_CONN, MODE_PERPOD
    e, _, local, pool, keep = W.cluster_engine_k8s(0, 4, 30, 5)
    rng = np.random.default_rng(7)
    n = 60000
    src = pool[rng.integers(0, len(pool), n)]
    dst = pool[rng.integers(0, len(pool), n)]
    sport = rng.integers(0, 65536, n).astype(np.uint16)
    dport = np.array(W.CLUSTER_PORTS + [8000, 8001, 8002, 8003, 8004], np.uint16)[rng.integers(0, 12, n)]
    proto = np.array([6, 17, 1, 6, 17], np.uint8)[rng.integers(0, 5, n)]
    wd = World(e, local, "VXLAN-BVI")
    got = e.debug_classify_host(MODE_PERPOD, -1, src, dst, sport, dport, proto, node=node)
    act, slot = wd.perpod(src, dst, dport, proto, threads=4)
    assert ((got >> 30) == act.astype(np.uint32)).all() and ((got & 0x3FFFFFFF) == slot).all()
    got = e.debug_classify_host(MODE_CONN, -1, src, dst, sport, dport, proto, node=node)
    act, slot = wd.conn(src, dst, sport, dport, proto, threads=4)
    assert ((got >> 30) == act.astype(np.uint32)).all() and ((got & 0x3FFFFFFF) == slot).all()
    assert len(np.unique(act)) >= 2
