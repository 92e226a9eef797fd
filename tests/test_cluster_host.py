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
