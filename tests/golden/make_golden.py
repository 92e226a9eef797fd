#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ from the reference's own tests.

Run here (the reference is at /root/reference; it does not exist on the GPU box):

    python tests/golden/make_golden.py

Outputs (data only: inputs + expected outputs):
  * testdata.json          -- plugins/policy/renderer/testdata/testdata.go:29-290 values
                              and the constants of acl_renderer_test.go:41-50.
  * cache_tables.json      -- the 14 plugins/policy/renderer/cache/cache_test.go scenarios:
                              per transaction the pod updates, and the expected ordered rule
                              tables (local per pod, global), isolated pods and change counts.
                              Expected lists are transcribed from the test's literal
                              expectations (line numbers cited per scenario).
  * acl_renderer_kats.json -- the 7 plugins/policy/renderer/acl/acl_renderer_test.go
                              scenarios: the renderer transactions (transcribed) and every
                              assertion of the test (Connection* verdicts, ACL counts, ACL
                              change counts, reflective/global ACL placement, committed txn
                              counts), extracted by regex from the test source and assigned
                              to the transaction after which it is checked.
"""
import json
import os
import re
import sys

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))

# --- testdata.go:29-80 -------------------------------------------------------
PODS = ["default/pod1", "default/pod2", "default/pod3", "default/pod4", "default/pod5", "namespace2/pod6"]
POD_IPS = ["10.10.1.1", "10.10.1.2", "10.10.2.1", "10.10.2.2", "10.10.2.3", "10.10.10.1"]
POD_IFS = ["node1-tap1", "node1-tap2", "node1-tap3", "node1-tap4", "node1-tap5", "node2-tap1"]
P = dict(zip(["Pod%d" % i for i in range(1, 7)], PODS))
IP = dict(zip(["Pod%dIP" % i for i in range(1, 7)], POD_IPS))
IF = dict(zip(["Pod%dIfName" % i for i in range(1, 7)], POD_IFS))


def R(action, src, dst, proto, sport, dport):
    return {"action": action, "src": src, "dst": dst, "proto": proto, "sport": sport, "dport": dport}


def allow_all():
    return R("PERMIT", "", "", "ANY", 0, 0)


def deny_all():
    return R("DENY", "", "", "ANY", 0, 0)


# testdata.go:87-256
TS = {
    "Ts1": R("PERMIT", "192.168.0.0/16", "", "TCP", 0, 80),
    "Ts2": R("PERMIT", "", "192.168.0.0/16", "TCP", 0, 80),
    "Ts3.Rule1": R("PERMIT", "10.10.0.0/16", "", "ANY", 0, 0),
    "Ts4.Rule1": R("PERMIT", "", "10.10.0.0/16", "ANY", 0, 0),
    "Ts5.Rule1": R("PERMIT", "10.10.0.0/16", "", "TCP", 0, 0),
    "Ts6.Rule1": R("PERMIT", "", "10.10.0.0/16", "TCP", 0, 0),
}
TS7 = {
    "Pod1Ingress": [R("PERMIT", "", "10.10.0.0/16", "TCP", 0, 80), R("PERMIT", "", "", "UDP", 0, 161), deny_all()],
    "Pod1Egress": [R("PERMIT", "10.0.0.0/8", "", "UDP", 0, 53), R("PERMIT", "192.168.0.0/16", "", "UDP", 0, 514),
                   deny_all()],
    "Pod3Ingress": [R("PERMIT", "", "10.10.1.1/32", "UDP", 0, 0), R("PERMIT", "", "", "TCP", 0, 22), deny_all()],
    "Pod3Egress": [R("PERMIT", "10.0.0.0/8", "", "TCP", 0, 80), R("PERMIT", "10.0.0.0/8", "", "TCP", 0, 443),
                   R("PERMIT", "", "", "UDP", 0, 67), deny_all()],
}


def host(ip):
    return ip + "/32"


# cache_test.go:39-117 helpers
def modify_src(src_ip, *rules):
    return [dict(r, src=host(src_ip)) for r in rules]


def modify_dst(rule, *dst_ips):
    return [dict(rule, dst=host(d)) for d in dst_ips]


def allow_pod_egress(ip, port, proto):
    return R("PERMIT", host(ip), "", proto, 0, port)


def block_pod_egress(ip):
    return R("DENY", host(ip), "", "ANY", 0, 0)


def allow_pod_ingress(ip, port, proto):
    return R("PERMIT", "", host(ip), proto, 0, port)


def block_pod_ingress(ip):
    return R("DENY", "", host(ip), "ANY", 0, 0)


def cfg(pod_ip, ingress, egress, removed=False):
    return {"ip": pod_ip, "ingress": ingress, "egress": egress, "removed": removed}


# --- cache_test.go scenarios -------------------------------------------------
def cache_scenarios():
    sc = []
    p1, p3 = P["Pod1"], P["Pod3"]
    ip1, ip3 = IP["Pod1IP"], IP["Pod3IP"]

    # TestSingleEgressRuleOnePodEgressOrientation :183-259
    sc.append({"name": "TestSingleEgressRuleOnePodEgressOrientation", "src": "cache_test.go:183-259",
               "orientation": "egress",
               "txns": [{"updates": {p1: cfg(ip1, [], [TS["Ts1"]])}, "changes": 1,
                         "expect": {"local": {p1: [TS["Ts1"], allow_all()]}, "global": [], "isolated": [p1]}}]})
    # TestSingleEgressRuleOnePodIngressOrientation :261-341
    sc.append({"name": "TestSingleEgressRuleOnePodIngressOrientation", "src": "cache_test.go:261-341",
               "orientation": "ingress",
               "txns": [{"updates": {p1: cfg(ip1, [], [TS["Ts1"]])}, "changes": 1,
                         "expect": {"local": {p1: None}, "global": modify_dst(TS["Ts1"], ip1) + [allow_all()],
                                    "isolated": []}}]})
    # TestSingleIngressRuleOnePodEgressOrientation :343-422
    sc.append({"name": "TestSingleIngressRuleOnePodEgressOrientation", "src": "cache_test.go:343-422",
               "orientation": "egress",
               "txns": [{"updates": {p1: cfg(ip1, [TS["Ts2"]], [])}, "changes": 1,
                         "expect": {"local": {p1: None}, "global": modify_src(ip1, TS["Ts2"]) + [allow_all()],
                                    "isolated": []}}]})
    # TestSingleIngressRuleOnePodIngressOrientation :424-499
    sc.append({"name": "TestSingleIngressRuleOnePodIngressOrientation", "src": "cache_test.go:424-499",
               "orientation": "ingress",
               "txns": [{"updates": {p1: cfg(ip1, [TS["Ts2"]], [])}, "changes": 1,
                         "expect": {"local": {p1: [TS["Ts2"], allow_all()]}, "global": [], "isolated": [p1]}}]})

    # TestMultipleEgressRulesMultiplePodsEgressOrientation :501-601
    eg = [TS["Ts3.Rule1"], deny_all()]
    upd1 = {PODS[i]: cfg(POD_IPS[i], [], eg) for i in range(3)}
    upd2 = {PODS[i]: cfg(POD_IPS[i], [], eg) for i in range(6)}
    sc.append({"name": "TestMultipleEgressRulesMultiplePodsEgressOrientation", "src": "cache_test.go:501-601",
               "orientation": "egress",
               "txns": [{"updates": upd1, "changes": 1,
                         "expect": {"local": {p: eg for p in PODS[:3]}, "global": [], "isolated": PODS[:3]}},
                        {"updates": upd2, "changes": 1,
                         "expect": {"local": {p: eg for p in PODS}, "global": [], "isolated": PODS}}]})
    # TestMultipleEgressRulesMultiplePodsIngressOrientation :603-722
    sc.append({"name": "TestMultipleEgressRulesMultiplePodsIngressOrientation", "src": "cache_test.go:603-722",
               "orientation": "ingress",
               "txns": [{"updates": upd1, "changes": 1,
                         "expect": {"local": {p: None for p in PODS[:3]},
                                    "global": modify_dst(TS["Ts3.Rule1"], *POD_IPS[:3])
                                    + modify_dst(deny_all(), *POD_IPS[:3]) + [allow_all()], "isolated": []}},
                        {"updates": upd2, "changes": 1,
                         "expect": {"local": {p: None for p in PODS},
                                    "global": modify_dst(TS["Ts3.Rule1"], *POD_IPS)
                                    + modify_dst(deny_all(), *POD_IPS) + [allow_all()], "isolated": []}}]})
    # TestMultipleIngressRulesMultiplePodsEgressOrientation :724-838
    ing = [TS["Ts4.Rule1"], deny_all()]
    iupd1 = {PODS[i]: cfg(POD_IPS[i], ing, []) for i in range(3)}
    iupd2 = {PODS[i]: cfg(POD_IPS[i], ing, []) for i in range(6)}
    g1 = sum((modify_src(POD_IPS[i], *ing) for i in range(3)), []) + [allow_all()]
    g2 = sum((modify_src(POD_IPS[i], *ing) for i in range(6)), []) + [allow_all()]
    sc.append({"name": "TestMultipleIngressRulesMultiplePodsEgressOrientation", "src": "cache_test.go:724-838",
               "orientation": "egress",
               "txns": [{"updates": iupd1, "changes": 1,
                         "expect": {"local": {p: None for p in PODS[:3]}, "global": g1, "isolated": []}},
                        {"updates": iupd2, "changes": 1,
                         "expect": {"local": {p: None for p in PODS}, "global": g2, "isolated": []}}]})
    # TestMultipleIngressRulesMultiplePodsIngressOrientation :840-939
    sc.append({"name": "TestMultipleIngressRulesMultiplePodsIngressOrientation", "src": "cache_test.go:840-939",
               "orientation": "ingress",
               "txns": [{"updates": iupd1, "changes": 1,
                         "expect": {"local": {p: ing for p in PODS[:3]}, "global": [], "isolated": PODS[:3]}},
                        {"updates": iupd2, "changes": 1,
                         "expect": {"local": {p: ing for p in PODS}, "global": [], "isolated": PODS}}]})

    # TestCombinedRulesEgressOrientation :941-1104
    c1 = cfg(ip1, TS7["Pod1Ingress"][1:], TS7["Pod1Egress"][:2])
    c2 = cfg(ip1, TS7["Pod1Ingress"], TS7["Pod1Egress"])
    c3 = cfg(ip3, TS7["Pod3Ingress"], TS7["Pod3Egress"])
    e_p1 = [allow_pod_egress(ip1, 161, "UDP"), block_pod_egress(ip1),
            allow_pod_egress(ip3, 22, "TCP"), allow_pod_egress(ip3, 0, "UDP"), block_pod_egress(ip3),
            c1["egress"][1], c1["egress"][0], allow_all()]
    e_p3 = [block_pod_egress(ip1), block_pod_egress(ip3)] + TS7["Pod3Egress"]
    e_g = modify_src(ip1, *c1["ingress"][:2]) + modify_src(ip3, *c3["ingress"][:3]) + [allow_all()]
    e_p1_2 = [block_pod_egress(ip1), c2["egress"][1], c2["egress"][0], c2["egress"][2]]
    e_p3_2 = [allow_pod_egress(ip1, 80, "TCP"), block_pod_egress(ip1), block_pod_egress(ip3)] + TS7["Pod3Egress"]
    e_g_2 = modify_src(ip1, *c2["ingress"][:3]) + modify_src(ip3, *c3["ingress"][:3]) + [allow_all()]
    sc.append({"name": "TestCombinedRulesEgressOrientation", "src": "cache_test.go:941-1104",
               "orientation": "egress",
               "txns": [{"updates": {p1: c1, p3: c3}, "changes": 3,
                         "expect": {"local": {p1: e_p1, p3: e_p3}, "global": e_g, "isolated": [p1, p3]}},
                        {"updates": {p1: c2}, "changes": 5,
                         "expect": {"local": {p1: e_p1_2, p3: e_p3_2}, "global": e_g_2, "isolated": [p1, p3]}}]})
    # TestCombinedRulesIngressOrientation :1106-1278
    i_p1 = [block_pod_ingress(ip3), c1["ingress"][0], c1["ingress"][1]]
    i_p3 = [c3["ingress"][0], block_pod_ingress(ip3), c3["ingress"][1], c3["ingress"][2]]
    i_g = (modify_dst(c1["egress"][1], ip1) + modify_dst(c1["egress"][0], ip1)
           + sum((modify_dst(c3["egress"][k], ip3) for k in range(4)), []) + [allow_all()])
    i_p1_2 = [block_pod_ingress(ip1), allow_pod_ingress(ip3, 80, "TCP"), block_pod_ingress(ip3)] + c2["ingress"][:3]
    i_p3_2 = [allow_pod_ingress(ip1, 53, "UDP"), block_pod_ingress(ip1), block_pod_ingress(ip3),
              c3["ingress"][1], c3["ingress"][2]]
    i_g_2 = (modify_dst(c2["egress"][1], ip1) + modify_dst(c2["egress"][0], ip1)
             + modify_dst(c3["egress"][0], ip3) + modify_dst(c3["egress"][1], ip3)
             + modify_dst(c2["egress"][2], ip1) + modify_dst(c3["egress"][2], ip3)
             + modify_dst(c3["egress"][3], ip3) + [allow_all()])
    sc.append({"name": "TestCombinedRulesIngressOrientation", "src": "cache_test.go:1106-1278",
               "orientation": "ingress",
               "txns": [{"updates": {p1: c1, p3: c3}, "changes": 3,
                         "expect": {"local": {p1: i_p1, p3: i_p3}, "global": i_g, "isolated": [p1, p3]}},
                        {"updates": {p1: c2}, "changes": 5,
                         "expect": {"local": {p1: i_p1_2, p3: i_p3_2}, "global": i_g_2, "isolated": [p1, p3]}}]})

    # TestRemovedPodsEgressOrientation :1280-1391 (egress given out of order on purpose)
    eg_r = [deny_all(), TS["Ts3.Rule1"]]
    rupd1 = {PODS[i]: cfg(POD_IPS[i], [], eg_r) for i in range(3)}
    rupd2 = {PODS[i]: cfg(POD_IPS[i], [], eg_r) for i in range(2)}
    rupd2[p3] = cfg(ip3, [], [], True)
    sc.append({"name": "TestRemovedPodsEgressOrientation", "src": "cache_test.go:1280-1391",
               "orientation": "egress",
               "txns": [{"updates": rupd1, "changes": 1,
                         "expect": {"local": {p: eg for p in PODS[:3]}, "global": [], "isolated": PODS[:3]}},
                        {"updates": rupd2, "changes": 1,
                         "expect": {"local": {PODS[0]: eg, PODS[1]: eg, p3: None}, "global": [],
                                    "isolated": PODS[:2]}}],
               "flush_after": True})
    # TestRemovedPodsIngressOrientation :1393-1515
    rupd1i = {PODS[i]: cfg(POD_IPS[i], [], eg) for i in range(3)}
    rupd2i = {PODS[i]: cfg(POD_IPS[i], [], eg) for i in range(2)}
    rupd2i[p3] = cfg(ip3, [], [], True)
    sc.append({"name": "TestRemovedPodsIngressOrientation", "src": "cache_test.go:1393-1515",
               "orientation": "ingress",
               "txns": [{"updates": rupd1i, "changes": 1,
                         "expect": {"local": {p: None for p in PODS[:3]},
                                    "global": modify_dst(TS["Ts3.Rule1"], *POD_IPS[:3])
                                    + modify_dst(deny_all(), *POD_IPS[:3]) + [allow_all()], "isolated": []}},
                        {"updates": rupd2i, "changes": 1,
                         "expect": {"local": {p: None for p in PODS[:3]},
                                    "global": modify_dst(TS["Ts3.Rule1"], *POD_IPS[:2])
                                    + modify_dst(deny_all(), *POD_IPS[:2]) + [allow_all()], "isolated": []}}],
               "flush_after": True})
    # TestResyncEgressOrientation :1517-1665 (Resync with pre-built tables, then one txn)
    sc.append({"name": "TestResyncEgressOrientation", "src": "cache_test.go:1517-1665",
               "orientation": "egress",
               "resync": [{"type": "local", "pods": [p1], "rules": e_p1},
                          {"type": "local", "pods": [p3], "rules": e_p3},
                          {"type": "global", "pods": [], "rules": e_g}],
               "txns": [{"updates": {p1: c2, p3: c3}, "changes": 5,
                         "expect": {"local": {p1: e_p1_2, p3: e_p3_2}, "global": e_g_2, "isolated": [p1, p3]}}]})
    # TestResyncIngressOrientation :1667-1824
    sc.append({"name": "TestResyncIngressOrientation", "src": "cache_test.go:1667-1824",
               "orientation": "ingress",
               "resync": [{"type": "local", "pods": [p1], "rules": i_p1},
                          {"type": "local", "pods": [p3], "rules": i_p3},
                          {"type": "global", "pods": [], "rules": i_g}],
               "txns": [{"updates": {p1: c2, p3: c3}, "changes": 5,
                         "expect": {"local": {p1: i_p1_2, p3: i_p3_2}, "global": i_g_2, "isolated": [p1, p3]}}]})
    return sc


# --- acl_renderer_test.go scenarios -------------------------------------------
def acl_scenarios():
    p1, p2, p3, p6 = P["Pod1"], P["Pod2"], P["Pod3"], P["Pod6"]
    ip1, ip2, ip3, ip6 = IP["Pod1IP"], IP["Pod2IP"], IP["Pod3IP"], IP["Pod6IP"]

    def render(pod, ip, ingress, egress, removed=False):
        return {"pod": pod, "ip": ip, "ingress": ingress, "egress": egress, "removed": removed}

    base_setup = {"main_if": "GbE", "vxlan_bvi": "VXLAN-BVI", "host_interconnect": "VPP-Host", "other_ifs": []}
    c1 = (TS7["Pod1Ingress"][1:], TS7["Pod1Egress"][:2])
    c2 = (TS7["Pod1Ingress"], TS7["Pod1Egress"])
    c3 = (TS7["Pod3Ingress"], TS7["Pod3Egress"])
    ts5 = [TS["Ts5.Rule1"], deny_all()]
    ts6 = [TS["Ts6.Rule1"], deny_all()]
    sc = {}
    sc["TestEgressRulesOnePod"] = {
        "setup": dict(base_setup, pod_ifs={p1: IF["Pod1IfName"]}, pods=[[p1, ip1, False], [p6, ip6, True]]),
        "phases": [[{"op": "txn", "resync": True, "renders": [render(p1, ip1, [], ts5)]}],
                   [{"op": "txn", "resync": False, "renders": [render(p1, ip1, [], ts5)]}]]}
    sc["TestIngressRulesOnePod"] = {
        "setup": dict(base_setup, pod_ifs={p1: IF["Pod1IfName"]}, pods=[[p1, ip1, False], [p6, ip6, True]]),
        "phases": [[{"op": "txn", "resync": True, "renders": [render(p1, ip1, ts6, [])]}],
                   [{"op": "txn", "resync": False, "renders": [render(p1, ip1, ts6, [])]}]]}
    sc["TestEgressRulesTwoPods"] = {
        "setup": dict(base_setup, pod_ifs={p1: IF["Pod1IfName"], p2: IF["Pod2IfName"]},
                      pods=[[p1, ip1, False], [p2, ip2, False], [p6, ip6, True]]),
        "phases": [[{"op": "txn", "resync": True, "renders": [render(p1, ip1, [], ts5), render(p2, ip2, [], ts5)]}],
                   [{"op": "txn", "resync": False, "renders": [render(p2, ip2, [], [], True)]}]]}
    two = dict(base_setup, pod_ifs={p1: IF["Pod1IfName"], p3: IF["Pod3IfName"]},
               pods=[[p1, ip1, False], [p3, ip3, False], [p6, ip6, True]])
    sc["TestCombinedRules"] = {
        "setup": two,
        "phases": [[{"op": "txn", "resync": True, "renders": [render(p1, ip1, *c1), render(p3, ip3, *c3)]}],
                   [{"op": "txn", "resync": False, "renders": [render(p1, ip1, *c2)]}]]}
    sc["TestCombinedRulesWithResync"] = {
        "setup": two,
        "phases": [[{"op": "txn", "resync": True, "renders": [render(p1, ip1, *c1), render(p3, ip3, *c3)]}],
                   [{"op": "restart"},
                    {"op": "txn", "resync": True, "renders": [render(p1, ip1, *c2), render(p3, ip3, *c3)]}],
                   [{"op": "txn", "resync": True, "renders": [render(p1, ip1, *c1), render(p3, ip3, *c3)]}]]}
    sc["TestCombinedRulesWithResyncAndRemovedPod"] = {
        "setup": two,
        "phases": [[{"op": "txn", "resync": True, "renders": [render(p1, ip1, *c1), render(p3, ip3, *c3)]}],
                   [{"op": "restart"}, {"op": "txn", "resync": True, "renders": [render(p1, ip1, *c1)]}],
                   [{"op": "txn", "resync": True, "renders": [render(p1, ip1, *c1), render(p3, ip3, *c3)]}]]}
    sc["TestCombinedRulesWithRemovedPods"] = {
        "setup": two,
        "phases": [[{"op": "txn", "resync": True, "renders": [render(p1, ip1, *c1), render(p3, ip3, *c3)]}],
                   [{"op": "txn", "resync": False,
                     "renders": [render(p1, ip1, *c1), render(p3, ip3, [], [], True)]}],
                   [{"op": "txn", "resync": False, "renders": [render(p1, ip1, [], [], True)]}]]}
    return sc


CONST = {"googleDNS": "8.8.8.8", "somePort": 500, "somePort2": 600, "mainIfName": "GbE",
         "vxlanIfName": "VXLAN-BVI", "hostInterIfName": "VPP-Host"}


def _val(tok):
    tok = tok.strip()
    if tok in CONST:
        return CONST[tok]
    if tok in P:
        return P[tok]
    if tok in IF:
        return IF[tok]
    if tok.startswith('"'):
        return tok.strip('"')
    if tok.startswith("renderer."):
        return tok.split(".", 1)[1]
    if tok in ("true", "false"):
        return tok == "true"
    return int(tok)


def parse_acl_test_checks(names):
    """Extract every assertion of acl_renderer_test.go, grouped per commit phase."""
    path = os.path.join(REF, "plugins/policy/renderer/acl/acl_renderer_test.go")
    lines = open(path).read().split("\n")
    funcs = {}
    cur = None
    for no, line in enumerate(lines, 1):
        m = re.match(r"^func (Test\w+)\(", line)
        if m:
            cur = m.group(1)
            funcs[cur] = {"line": no, "phases": [], "commits": 0}
            continue
        if cur is None:
            continue
        f = funcs[cur]
        if re.search(r"\.Commit\(\)", line):
            f["commits"] += 1
            f["phases"].append([])
            continue
        if f["commits"] == 0:
            continue
        ph = f["phases"][-1]
        m = re.search(r"aclEngine\.(Connection\w+)\((.*?)\)\)\.To\(gomega\.Equal\((ConnAction\w+)\)\)", line)
        if m:
            args = [_val(a) for a in m.group(2).split(",")]
            ph.append({"kind": m.group(1), "args": args, "expect": m.group(3), "line": no})
            continue
        m = re.search(r"aclEngine\.GetNumOfACLs\(\)\)\.To\(gomega\.Equal\((\d+)\)\)", line)
        if m:
            ph.append({"kind": "NumACLs", "expect": int(m.group(1)), "line": no})
            continue
        m = re.search(r"aclEngine\.GetNumOfACLChanges\(\)\)\.To\(gomega\.Equal\((\d+)\)\)", line)
        if m:
            ph.append({"kind": "NumACLChanges", "expect": int(m.group(1)), "line": no})
            continue
        m = re.search(r"verifyReflectiveACL\(aclEngine, ipv4Net, contivConf, (.*?), (true|false), (true|false)\)", line)
        if m:
            ph.append({"kind": "ReflectiveACL", "if": _val(m.group(1)) if m.group(1) != '""' else "",
                       "on_output_ifs": m.group(2) == "true", "expect": m.group(3) == "true", "line": no})
            continue
        m = re.search(r"verifyGlobalTable\(aclEngine, ipv4Net, contivConf, (true|false)\)", line)
        if m:
            ph.append({"kind": "GlobalACL", "expect": m.group(1) == "true", "line": no})
            continue
        m = re.search(r"txnTracker\.CommittedTxns\)\.To\(gomega\.HaveLen\((\d+)\)\)", line)
        if m:
            ph.append({"kind": "CommittedTxns", "expect": int(m.group(1)), "line": no})
            continue
        m = re.search(r"txnTracker\.PendingTxns\)\.To\(gomega\.HaveLen\((\d+)\)\)", line)
        if m:
            ph.append({"kind": "PendingTxns", "expect": int(m.group(1)), "line": no})
            continue
    return {n: funcs[n] for n in names}


def main():
    if not os.path.isdir(REF):
        sys.exit("reference not present: fixtures are committed, nothing to do")
    td = {"pods": PODS, "pod_ips": POD_IPS, "pod_ifs": POD_IFS, "ts": TS, "ts7": TS7, "const": CONST,
          "src": "plugins/policy/renderer/testdata/testdata.go:29-290; acl_renderer_test.go:41-50"}
    json.dump(td, open(os.path.join(OUT, "testdata.json"), "w"), indent=1, sort_keys=True)
    json.dump(cache_scenarios(), open(os.path.join(OUT, "cache_tables.json"), "w"), indent=1)
    sc = acl_scenarios()
    checks = parse_acl_test_checks(list(sc))
    out = []
    n_conn = 0
    for name, s in sc.items():
        f = checks[name]
        assert len(f["phases"]) == len(s["phases"]), (name, len(f["phases"]), len(s["phases"]))
        for ph, chk in zip(s["phases"], f["phases"]):
            n_conn += sum(1 for c in chk if c["kind"].startswith("Connection"))
        out.append({"name": name, "src": "acl_renderer_test.go:%d" % f["line"], "setup": s["setup"],
                    "phases": [{"steps": st, "checks": ck} for st, ck in zip(s["phases"], f["phases"])]})
    json.dump(out, open(os.path.join(OUT, "acl_renderer_kats.json"), "w"), indent=1)
    print("acl_renderer KATs: %d Connection* verdicts in %d scenarios" % (n_conn, len(out)))


if __name__ == "__main__":
    main()
