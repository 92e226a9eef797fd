"""Synthetic workloads of BASELINE.json's configs, built through the
product's own renderer / ACL-ingestion path. Inputs are synthetic (no datasets exist for
this path); shapes follow the reference's own fixtures and perf generator:

  config 1  renderer unit-test scenario (acl_renderer_test.go TestCombinedRules, first txn),
            connection mode, 1M tuples
  config 2  1k-rule single table shaped like tests/policy/perf/gen-policy.py (/16-/24 CIDRs
            under (i+0x100)<<16 minus five /24-/32 excepts, x 20 TCP/UDP ports), first 999
            generated rules + deny-the-rest, 64M tuples (bench.py's default)
  config 3  1k pods / 10 namespaces / per-app K8s policies -> policy configurator -> ACL
            renderer: local tables + global table, per-pod (egress interface) mode
  config 4  100k-rule ACL ingested directly (vpp_acl key space), disjoint src prefixes,
            first-match depth Zipf(1.1), 5 % no-match
  config 5  config-3 topology in connection mode with per-rule hit counters
  config 7  the whole tests/policy/perf/gen-policy.py policy (1000 CIDRs x 5 excepts x 20 ports,
            ingress and egress) through the policy configurator: the pod's ~487k-rule table
  rule-count sweep: config 2's shape at any rule count (bench.py --rules N)
"""
import random

import numpy as np

from . import renderer as R
from ._capi import MODE_CONN, MODE_PERPOD, MODE_SINGLE

SEEDS = {1: 0xC0DE0001, 2: 0xC0DE0002, 3: 0xC0DE0003, 4: 0xC0DE0004, 5: 0xC0DE0005, 6: 0xC0DE0006, 7: 0xC0DE0007,
         8: 0xC0DE0008, 9: 0xC0DE0009}
POPULAR_PORTS = [22, 53, 67, 80, 81, 161, 162, 443, 514, 8080]


def ip_str(v):
    return "%d.%d.%d.%d" % (v >> 24 & 255, v >> 16 & 255, v >> 8 & 255, v & 255)


def ip_u32(s):
    a, b, c, d = (int(x) for x in s.split("."))
    return (a << 24) | (b << 16) | (c << 8) | d


def mask_ip(ip, plen):
    return ip & ((0xFFFFFFFF << (32 - plen)) & 0xFFFFFFFF) if plen else 0


def subtract_subnet(n1, n2):
    """IPv4 form of the configurator's subtractSubnet (configurator_impl.go:562-594)."""
    (ip1, l1), (ip2, l2) = n1, n2
    if l1 > l2:
        return [n1] if mask_ip(ip1, l2) != mask_ip(ip2, l2) else []
    if l1 == l2:
        return [n1] if ip1 != ip2 else []
    if mask_ip(ip2, l1) != mask_ip(ip1, l1):
        return [n1]
    out = []
    for bit in range(l1, l2):
        sub = mask_ip(ip2, bit + 1) ^ (1 << (31 - bit))
        out.append((sub, bit + 1))
    return out


class Workload:
    """local_ifs {IPv4 u32: TAP} and node_if describe the node's interfaces (PERPOD/CONN)."""

    def __init__(self, config, engine, mode, table_id, gen, n_tuples, desc, renderer=None, local_ifs=None,
                 node_if="VXLAN-BVI", counters=False):
        self.config, self.engine, self.mode, self.table_id = config, engine, mode, table_id
        self.gen, self.n_tuples, self.desc, self.renderer = gen, n_tuples, desc, renderer
        self.local_ifs, self.node_if, self.counters = local_ifs or {}, node_if, counters

    def stats(self):
        e = self.engine
        nt = e.num_tables()
        return {"tables": nt, "rules": e.num_counter_slots() - nt - 2}


def _new_engine(device):
    e = R.Engine(device)
    e.SetMainInterfaceName("GbE")
    e.SetVxlanBVIIfName("VXLAN-BVI")
    e.SetHostInterconnectIfName("VPP-Host")
    return e


# ---- config 1 ------------------------------------------------------------------------
TESTDATA_PODS = ["default/pod1", "default/pod2", "default/pod3", "default/pod4", "default/pod5", "namespace2/pod6"]
TESTDATA_IPS = ["10.10.1.1", "10.10.1.2", "10.10.2.1", "10.10.2.2", "10.10.2.3", "10.10.10.1"]


def _rule(a, s, d, p, dp):
    return R.ContivRule(a, R.IPNet(s), R.IPNet(d), p, 0, dp)


def config1(device=0, n_tuples=1 << 20):
    """TestCombinedRules (acl_renderer_test.go:447-553) tables, testdata.go:172-256 rules."""
    P, D = R.ActionPermit, R.ActionDeny
    deny = _rule(D, "", "", R.ANY, 0)
    pod1_in = [_rule(P, "", "", R.UDP, 161), deny]                                  # Ts7.Pod1Ingress[1:]
    pod1_eg = [_rule(P, "10.0.0.0/8", "", R.UDP, 53), _rule(P, "192.168.0.0/16", "", R.UDP, 514)]
    pod3_in = [_rule(P, "", "10.10.1.1/32", R.UDP, 0), _rule(P, "", "", R.TCP, 22), deny]
    pod3_eg = [_rule(P, "10.0.0.0/8", "", R.TCP, 80), _rule(P, "10.0.0.0/8", "", R.TCP, 443),
               _rule(P, "", "", R.UDP, 67), deny]
    e = _new_engine(device)
    e.SetPodIfName("default/pod1", "node1-tap1")
    e.SetPodIfName("default/pod3", "node1-tap3")
    e.RegisterPod("default/pod1", "10.10.1.1", False)
    e.RegisterPod("default/pod3", "10.10.2.1", False)
    e.RegisterPod("namespace2/pod6", "10.10.10.1", True)
    r = R.Renderer(e)
    t = r.NewTxn(True)
    t.Render("default/pod1", R.IPNet.host("10.10.1.1"), pod1_in, pod1_eg, False)
    t.Render("default/pod3", R.IPNet.host("10.10.2.1"), pod3_in, pod3_eg, False)
    err = t.Commit()
    assert err is None, err
    pool = [ip_u32(x) for x in TESTDATA_IPS] * 4 + [ip_u32(x) for x in ("8.8.8.8", "10.10.50.1", "192.168.1.1")] * 6
    gen = dict(seed=SEEDS[1], ip_pool=np.array(pool, np.uint32), pool_pct=70, dst_pool_pct=70,
               port_pool=np.array(POPULAR_PORTS, np.uint16), port_pool_pct=50, tcp_pct=45, udp_pct=45)
    return Workload(1, e, MODE_CONN, -1, gen, n_tuples, "TestCombinedRules tables, testConnection by IP", r,
                    local_ifs={ip_u32("10.10.1.1"): "node1-tap1", ip_u32("10.10.2.1"): "node1-tap3"})


# ---- config 2 ------------------------------------------------------------------------
def gen_policy_rules(seed, max_rules=999, num_excepts=5, num_ports=20):
    """tests/policy/perf/gen-policy.py:35-60 ipBlocks x ports, turned into ContivRules the way
    the configurator does for an ingress policy (SrcNetwork = subtracted block piece)."""
    rnd = random.Random(seed)
    ports = [(R.TCP if rnd.randint(0, 1) == 0 else R.UDP, rnd.randint(0, 65535)) for _ in range(num_ports)]
    rules = []
    i = 0
    while len(rules) < max_rules:
        prefix = (i + 0x100) << 16
        cidr = rnd.randint(prefix, prefix | 0xFFFF)
        ml = rnd.randint(16, 24)
        cidr = mask_ip(cidr, ml)
        excepts = []
        for _ in range(num_excepts):
            ex = rnd.randint(cidr, cidr | ((1 << (32 - ml)) - 1))
            el = rnd.randint(24, 32)
            excepts.append((mask_ip(ex, el), el))
        pieces = [(cidr, ml)]
        for ex in excepts:
            pieces = [q for p in pieces for q in subtract_subnet(p, ex)]
        for ip, pl in pieces:
            for proto, port in ports:
                rules.append(R.ContivRule(R.ActionPermit, R.IPNet("%s/%d" % (ip_str(ip), pl)), R.IPNet(), proto, 0,
                                          port))
        i += 1
    return rules[:max_rules]


def config2(device=0, n_tuples=64 << 20, n_rules=1000):
    """n_rules: the table's rules (n_rules - 1 generated + deny-the-rest); 1000 = BASELINE's config 2"""
    e = _new_engine(device)
    pod = "default/db-0"
    e.SetPodIfName(pod, "node1-tap-db0")
    e.RegisterPod(pod, "10.1.0.10", False)
    r = R.Renderer(e)
    rules = gen_policy_rules(SEEDS[2], max_rules=n_rules - 1) + [R.ContivRule(R.ActionDeny, R.IPNet(), R.IPNet(), R.ANY,
                                                                              0, 0)]
    t = r.NewTxn(True)
    t.Render(pod, R.IPNet.host("10.1.0.10"), [], rules, False)
    err = t.Commit()
    assert err is None, err
    acl = e.GetOutboundACL("node1-tap-db0")
    tid = e.table_id(acl["name"])
    gen = dict(seed=SEEDS[2], table_id=tid, inside_pct=50, tcp_pct=45, udp_pct=45)
    return Workload(2, e, MODE_SINGLE, tid, gen, n_tuples, "gen-policy 1k-rule table (%d rules)" % len(acl["rules"]),
                    r)


def gen_policy_blocks(rnd, num_cidrs=1000, num_excepts=5):
    """tests/policy/perf/gen-policy.py:39-51 genIpBlocks: CIDR i under (i + 0x100) << 16, mask
    /16-/24, five /24-/32 excepts inside it"""
    from . import configurator as CF
    blocks = []
    for i in range(num_cidrs):
        prefix = (i + 0x100) << 16
        cidr = rnd.randint(prefix, prefix | 0xFFFF)
        ml = rnd.randint(16, 24)
        cidr = mask_ip(cidr, ml)
        ex = []
        for _ in range(num_excepts):
            e = rnd.randint(cidr, cidr | ((1 << (32 - ml)) - 1))
            el = rnd.randint(24, 32)
            ex.append("%s/%d" % (ip_str(mask_ip(e, el)), el))
        blocks.append(CF.IPBlock("%s/%d" % (ip_str(cidr), ml), ex))
    return blocks


def gen_policy_ports(rnd, num_ports=20):
    """gen-policy.py:53-62 genPorts"""
    from . import configurator as CF
    return [CF.Port(CF.TCP if rnd.randint(0, 1) == 0 else CF.UDP, rnd.randint(0, 65535)) for _ in range(num_ports)]


def config7(device=0, n_tuples=64 << 20):
    """The whole gen-policy.py NetworkPolicy (1000 ingress + 1000 egress ipBlocks with 5 excepts
    each, 20 ports each) for pod role=db, through the policy configurator (IPBlock minus excepts
    by subtractSubnet, x ports, NAT-loopback permit, deny-the-rest) into the GPU renderer; SINGLE
    mode on the pod's table (the ingress part, ~487k rules; the egress part lands in the
    global table)."""
    from . import configurator as CF
    e = _new_engine(device)
    pod, ip = "default/db-0", "10.1.0.10"
    e.SetPodIfName(pod, "node1-tap-db0")
    e.RegisterPod(pod, ip, False)
    r = R.Renderer(e)
    rnd = random.Random(SEEDS[7])
    ing = CF.Match(CF.MatchIngress, IPBlocks=gen_policy_blocks(rnd), Ports=gen_policy_ports(rnd))
    eg = CF.Match(CF.MatchEgress, IPBlocks=gen_policy_blocks(rnd), Ports=gen_policy_ports(rnd))
    cfg = CF.PolicyConfigurator()
    cfg.AddPodConfig(pod, ip)
    cfg.SetNatLoopbackIP(NAT_LOOPBACK_IP)
    assert cfg.RegisterRenderer(r) is None
    t = cfg.NewTxn(True)
    t.Configure(pod, [CF.ContivPolicy("default/test-network-policy", CF.PolicyAll, [ing, eg])])
    err = t.Commit()
    assert err is None, err
    acl = e.GetOutboundACL("node1-tap-db0")
    tid = e.table_id(acl["name"])
    gen = dict(seed=SEEDS[7], table_id=tid, inside_pct=50, tcp_pct=45, udp_pct=45)
    w = Workload(7, e, MODE_SINGLE, tid, gen, n_tuples,
                 "gen-policy.py policy through the configurator (%d-rule pod table)" % len(acl["rules"]), r)
    w.control = cfg
    return w


# ---- config 4 ------------------------------------------------------------------------
def zipf_cdf(n, s=1.1):
    w = 1.0 / np.power(np.arange(1, n + 1, dtype=np.float64), s)
    c = np.cumsum(w)
    c /= c[-1]
    u = np.minimum(np.floor(c * 4294967296.0), 4294967295.0).astype(np.uint64)
    u[-1] = 4294967295
    return u.astype(np.uint32)


def big_acl_rules(n_rules, seed):
    """Disjoint src prefixes (/26../32) packed in 10.0.0.0/8, random L4 section and action."""
    rnd = random.Random(seed)
    rules = []
    addr = 10 << 24
    for _ in range(n_rules):
        pl = rnd.randint(26, 32)
        size = 1 << (32 - pl)
        addr = (addr + size - 1) & ~(size - 1)
        src = "%s/%d" % (ip_str(addr), pl)
        addr += size
        kind = rnd.random()
        rule = {"action": rnd.choice([0, 1]), "src": src, "dst": ""}
        if kind < 0.4:
            lo = rnd.randint(1, 65000)
            rule["tcp"] = {"src": [0, 65535], "dst": [lo, lo + rnd.choice([0, 0, 10, 500])]}
        elif kind < 0.8:
            lo = rnd.randint(1, 65000)
            rule["udp"] = {"src": [0, 65535], "dst": [lo, lo + rnd.choice([0, 0, 10, 500])]}
        rules.append(rule)
    assert addr <= (11 << 24)
    return rules


def config4(device=0, n_tuples=64 << 20, n_rules=100000):
    e = _new_engine(device)
    acl = {"name": "contiv-policy-bigtable", "ingress": [], "egress": ["node1-tap-big"],
           "rules": big_acl_rules(n_rules, SEEDS[4])}
    e.ApplyTxn(True, [("config/vpp/acls/v2/acl/" + acl["name"], acl)])
    tid = e.table_id(acl["name"])
    gen = dict(seed=SEEDS[4], table_id=tid, inside_pct=95, nomatch_pct=5, zipf_cdf=zipf_cdf(n_rules),
               tcp_pct=45, udp_pct=45)
    return Workload(4, e, MODE_SINGLE, tid, gen, n_tuples, "100k-rule ACL, Zipf(1.1) first-match depth")


# ---- configs 3 and 5 -------------------------------------------------------------------
INTERNET_HOSTS = ["8.8.8.8", "1.1.1.1", "192.168.10.5", "192.168.20.7", "10.96.0.10"]
CLUSTER_PORTS = [80, 8080, 443, 53, 5353, 22, 9090]


def cluster_pods(n_ns=10, pods_per_ns=100, apps=5, remote_pct=10):
    """Pods ns<k>/app<a>-<j> with IP 10.1.k.(j+1); the last remote_pct % of every namespace
    run on another node."""
    pods = []
    for k in range(n_ns):
        for j in range(pods_per_ns):
            remote = j >= pods_per_ns * (100 - remote_pct) // 100
            pods.append({"id": "ns%d/app%d-%d" % (k, j % apps, j), "ns": k, "app": j % apps,
                         "ip": (10 << 24) | (1 << 16) | (k << 8) | (j + 1), "remote": remote})
    return pods


def cluster_rules(pods, n_ns, apps):
    """Per-pod ContivRule lists as the configurator would emit them for label-selector
    policies (one ContivRule per selected peer /32 x port, IPBlock minus excepts via
    subtractSubnet, deny-the-rest), keyed by (namespace, app).

    egress (traffic to the pod, src = peer):
      app (a+1) of the same namespace -> TCP 80, 8080
      app a of namespace k+1          -> TCP 443
      app (a+2) of namespaces k+3, k+5, k+7 -> UDP 53, 5353
      192.168.0.0/16 except 192.168.10.0/24 -> TCP 22
      deny the rest
    ingress (traffic from the pod, dst = peer), app-0 pods only:
      TCP 443 anywhere, UDP 53 to 10.96.0.10, TCP 80 to its namespace's /24, deny the rest
    """
    P, D = R.ActionPermit, R.ActionDeny
    by = {}
    for p in pods:
        by.setdefault((p["ns"], p["app"]), []).append(p)
    deny = R.ContivRule(D, R.IPNet(), R.IPNet(), R.ANY, 0, 0)
    host = lambda ip: R.IPNet("%s/32" % ip_str(ip))
    egress, ingress = {}, {}
    block = subtract_subnet((ip_u32("192.168.0.0"), 16), (ip_u32("192.168.10.0"), 24))
    for k in range(n_ns):
        for a in range(apps):
            rl = []
            for q in by[(k, (a + 1) % apps)]:
                rl += [R.ContivRule(P, host(q["ip"]), R.IPNet(), R.TCP, 0, port) for port in (80, 8080)]
            for q in by[((k + 1) % n_ns, a)]:
                rl.append(R.ContivRule(P, host(q["ip"]), R.IPNet(), R.TCP, 0, 443))
            for kk in ((k + 3) % n_ns, (k + 5) % n_ns, (k + 7) % n_ns):
                for q in by[(kk, (a + 2) % apps)]:
                    rl += [R.ContivRule(P, host(q["ip"]), R.IPNet(), R.UDP, 0, port) for port in (53, 5353)]
            for ip, pl in block:
                rl.append(R.ContivRule(P, R.IPNet("%s/%d" % (ip_str(ip), pl)), R.IPNet(), R.TCP, 0, 22))
            rl.append(deny)
            egress[(k, a)] = rl
            ingress[(k, a)] = [] if a else [
                R.ContivRule(P, R.IPNet(), R.IPNet(), R.TCP, 0, 443),
                R.ContivRule(P, R.IPNet(), R.IPNet("10.96.0.10/32"), R.UDP, 0, 53),
                R.ContivRule(P, R.IPNet(), R.IPNet("10.1.%d.0/24" % k), R.TCP, 0, 80),
                deny]
    return ingress, egress


def cluster_policies(pods, n_ns, apps):
    """The K8s policies behind cluster_rules, as configurator.ContivPolicy objects: one per
    (namespace, app), selecting the peer pods by label (expanded to pod IDs, as the policy
    processor does), IPBlocks with excepts, ports. The configurator turns them into the
    ContivRule lists (adding the NAT-loopback permit and the deny-the-rest rules)."""
    from . import configurator as CF
    by = {}
    for p in pods:
        by.setdefault((p["ns"], p["app"]), []).append(p["id"])
    out = {}
    for k in range(n_ns):
        for a in range(apps):
            ingress = [  # traffic to the pod (the vswitch's egress direction)
                CF.Match(CF.MatchIngress, Pods=by[(k, (a + 1) % apps)],
                         Ports=[CF.Port(CF.TCP, 80), CF.Port(CF.TCP, 8080)]),
                CF.Match(CF.MatchIngress, Pods=by[((k + 1) % n_ns, a)], Ports=[CF.Port(CF.TCP, 443)]),
                CF.Match(CF.MatchIngress, Pods=[q for kk in ((k + 3) % n_ns, (k + 5) % n_ns, (k + 7) % n_ns)
                                                for q in by[(kk, (a + 2) % apps)]],
                         Ports=[CF.Port(CF.UDP, 53), CF.Port(CF.UDP, 5353)]),
                CF.Match(CF.MatchIngress, IPBlocks=[CF.IPBlock("192.168.0.0/16", ["192.168.10.0/24"])],
                         Ports=[CF.Port(CF.TCP, 22)]),
            ]
            pols = [CF.ContivPolicy("ns%d/app%d-ingress" % (k, a), CF.PolicyIngress, ingress)]
            if a == 0:  # app-0 pods also restrict what they send
                pols.append(CF.ContivPolicy("ns%d/app%d-egress" % (k, a), CF.PolicyEgress, [
                    CF.Match(CF.MatchEgress, Ports=[CF.Port(CF.TCP, 443)]),
                    CF.Match(CF.MatchEgress, IPBlocks=[CF.IPBlock("10.96.0.10/32")], Ports=[CF.Port(CF.UDP, 53)]),
                    CF.Match(CF.MatchEgress, IPBlocks=[CF.IPBlock("10.1.%d.0/24" % k)],
                             Ports=[CF.Port(CF.TCP, 80)]),
                ]))
            out[(k, a)] = pols
    return out


NAT_LOOPBACK_IP = "10.1.255.254"


def cluster_engine(device=0, n_ns=10, pods_per_ns=100, apps=5):
    """Configs 3/5: the cluster's policies -> policy configurator (every pod in its cache, the
    pods of this node configured) -> GPU ACL renderer -> engine."""
    from . import configurator as CF
    e = _new_engine(device)
    pods = cluster_pods(n_ns, pods_per_ns, apps)
    local = {}
    for p in pods:
        if not p["remote"]:
            ifn = "tap-%s" % p["id"].replace("/", "-")
            e.SetPodIfName(p["id"], ifn)
            local[p["ip"]] = ifn
        e.RegisterPod(p["id"], ip_str(p["ip"]), p["remote"])
    policies = cluster_policies(pods, n_ns, apps)
    r = R.Renderer(e)
    cfg = CF.PolicyConfigurator()
    for p in pods:
        cfg.AddPodConfig(p["id"], ip_str(p["ip"]))
    cfg.SetNatLoopbackIP(NAT_LOOPBACK_IP)
    assert cfg.RegisterRenderer(r) is None
    t = cfg.NewTxn(True)
    for p in pods:
        if not p["remote"]:  # the configurator of this node is told about its own pods
            t.Configure(p["id"], policies[(p["ns"], p["app"])])
    err = t.Commit()
    assert err is None, err
    pool = [p["ip"] for p in pods] + [ip_u32(x) for x in INTERNET_HOSTS] * 10
    return e, r, local, np.array(pool, np.uint32)


NODE_POD_SUBNET = "10.1.0.0/16"  # IPAM.PodSubnetThisNode() of the K8s-object cluster


def cluster_k8s(n_ns=10, pods_per_ns=100, apps=5, remote_pct=10):
    """The cluster as K8s objects (KSR model dicts, see vpp_amd/k8s.py) for the policy cache
    and processor: label / namespace selectors, IPBlocks with excepts,
    numbered and named ports. Pods ns<k>/app<a>-<j> on this node get 10.1.k.(j+1), the last
    remote_pct % of every namespace run elsewhere (10.2.k.(j+1)).

    Per (namespace k, app a), policy "app<a>-ingress" (PolicyType INGRESS) for pods app=app<a>:
      from pods app=app<a+1> (same namespace)          TCP 80 and the named port "http"
      from namespaces name=ns<k+1>                     TCP 443
      from namespaces group In [g<(k+1)%3>] + pods with app NotIn [app0]   UDP 53
      from 192.168.0.0/16 except 192.168.10.0/24       TCP 22
    and for app0 pods "app0-egress" (EGRESS): TCP 443 anywhere, UDP 53 to 10.96.0.10/32,
    the named port "http" of namespace ns<k>'s pods."""
    lbl = lambda k, v: {"Key": k, "Value": v}  # noqa: E731
    namespaces = [{"Name": "ns%d" % k, "Label": [lbl("name", "ns%d" % k), lbl("group", "g%d" % (k % 3))]}
                  for k in range(n_ns)]
    pods = []
    for k in range(n_ns):
        for j in range(pods_per_ns):
            remote = j >= pods_per_ns * (100 - remote_pct) // 100
            pods.append({"Name": "app%d-%d" % (j % apps, j), "Namespace": "ns%d" % k,
                         "Label": [lbl("app", "app%d" % (j % apps)), lbl("tier", "t%d" % (j % 2))],
                         "IpAddress": "10.%d.%d.%d" % (2 if remote else 1, k, j + 1),
                         "Container": [{"Name": "main", "Port": [{"Name": "http", "ContainerPort": 8000 + j % apps}]}]})
    tcp = lambda n: {"Protocol": 0, "Port": {"Type": 0, "Number": n}}  # noqa: E731
    udp = lambda n: {"Protocol": 1, "Port": {"Type": 0, "Number": n}}  # noqa: E731
    named = {"Protocol": 0, "Port": {"Type": 1, "Name": "http"}}
    policies = []
    for k in range(n_ns):
        for a in range(apps):
            policies.append({
                "Name": "app%d-ingress" % a, "Namespace": "ns%d" % k, "PolicyType": 1,
                "Pods": {"MatchLabel": [lbl("app", "app%d" % a)]},
                "IngressRule": [
                    {"Port": [tcp(80), named], "From": [{"Pods": {"MatchLabel": [lbl("app", "app%d" % ((a + 1) % apps))]}}]},
                    {"Port": [tcp(443)], "From": [{"Namespaces": {"MatchLabel": [lbl("name", "ns%d" % ((k + 1) % n_ns))]}}]},
                    {"Port": [udp(53)], "From": [{
                        "Namespaces": {"MatchExpression": [{"Key": "group", "Operator": 0, "Value": ["g%d" % ((k + 1) % 3)]}]},
                        "Pods": {"MatchExpression": [{"Key": "app", "Operator": 1, "Value": ["app0"]}]}}]},
                    {"Port": [tcp(22)], "From": [{"IpBlock": {"Cidr": "192.168.0.0/16", "Except": ["192.168.10.0/24"]}}]},
                ]})
        policies.append({
            "Name": "app0-egress", "Namespace": "ns%d" % k, "PolicyType": 2,
            "Pods": {"MatchLabel": [lbl("app", "app0")]},
            "EgressRule": [
                {"Port": [tcp(443)], "To": []},
                {"Port": [udp(53)], "To": [{"IpBlock": {"Cidr": "10.96.0.10/32"}}]},
                {"Port": [named], "To": [{"Namespaces": {"MatchLabel": [lbl("name", "ns%d" % k)]}}]},
            ]})
    return pods, namespaces, policies


def cluster_engine_k8s(device=0, n_ns=10, pods_per_ns=100, apps=5):
    """The K8s-object cluster through the whole control path of the reference: policy cache
    (Resync) -> policy processor (selector expansion, named ports, this node's pods) ->
    policy configurator -> GPU ACL renderer -> engine. Returns (engine, renderer, local
    interfaces {IPv4: TAP}, tuple IP pool, (cache, processor, configurator))."""
    from . import configurator as CF
    from . import k8s as K
    e = _new_engine(device)
    pods, namespaces, policies = cluster_k8s(n_ns, pods_per_ns, apps)
    local = {}
    for p in pods:
        pid = "%s/%s" % (p["Namespace"], p["Name"])
        remote = p["IpAddress"].startswith("10.2.")
        if not remote:
            ifn = "tap-%s" % pid.replace("/", "-")
            e.SetPodIfName(pid, ifn)
            local[ip_u32(p["IpAddress"])] = ifn
        e.RegisterPod(pid, p["IpAddress"], remote)
    r = R.Renderer(e)
    cfg = CF.PolicyConfigurator()
    cfg.SetNatLoopbackIP(NAT_LOOPBACK_IP)
    assert cfg.RegisterRenderer(r) is None
    cache = K.PolicyCache()
    proc = K.PolicyProcessor(cache, cfg, NODE_POD_SUBNET)
    err = cache.Resync(pods, namespaces, policies)
    assert err is None, err
    pool = [ip_u32(p["IpAddress"]) for p in pods] + [ip_u32(x) for x in INTERNET_HOSTS] * 10
    return e, r, local, np.array(pool, np.uint32), (cache, proc, cfg)


def config3(device=0, n_tuples=125 << 20, n_ns=10):
    e, r, local, pool = cluster_engine(device, n_ns=n_ns)
    gen = dict(seed=SEEDS[3], ip_pool=pool, pool_pct=85, dst_pool_pct=88,
               port_pool=np.array(CLUSTER_PORTS, np.uint16), port_pool_pct=80, tcp_pct=60, udp_pct=30)
    return Workload(3, e, MODE_PERPOD, -1, gen, n_tuples,
                    "1k pods / 10 namespaces, per-pod tables + global, evalACL on the dst interface", r,
                    local_ifs=local)


def config5(device=0, n_tuples=125 << 20, n_ns=10):
    e, r, local, pool = cluster_engine(device, n_ns=n_ns)
    gen = dict(seed=SEEDS[5], ip_pool=pool, pool_pct=85, dst_pool_pct=88,
               port_pool=np.array(CLUSTER_PORTS, np.uint16), port_pool_pct=80, tcp_pct=60, udp_pct=30)
    return Workload(5, e, MODE_CONN, -1, gen, n_tuples,
                    "config-3 topology, testConnection both directions, per-rule hit counters", r,
                    local_ifs=local, counters=True)


def config8(device=0, n_tuples=125 << 20, n_ns=10, apps=20):
    """Config 3's cluster with 20 apps per namespace instead of 5: ~210 distinct per-pod tables
    (per-pod tables are unbounded in the reference, cache_impl.go:409-466) -- past the 64 tables
    one 64-bit common-row mask per IP class covers (the uniform layout's grouped marks)."""
    e, r, local, pool = cluster_engine(device, n_ns=n_ns, apps=apps)
    gen = dict(seed=SEEDS[8], ip_pool=pool, pool_pct=85, dst_pool_pct=88,
               port_pool=np.array(CLUSTER_PORTS, np.uint16), port_pool_pct=80, tcp_pct=60, udp_pct=30)
    return Workload(8, e, MODE_PERPOD, -1, gen, n_tuples,
                    "1k pods / 10 namespaces x 20 apps (~210 tables), evalACL on the dst interface", r,
                    local_ifs=local)


def config9(device=0, n_tuples=125 << 20, n_ns=10, apps=50):
    """Config 3's cluster with 50 apps per namespace: ~500 distinct per-pod tables (per-pod tables
    are unbounded in the reference, cache_impl.go:409-466) -- past the 254 tables whose ids fit a
    byte of the uniform layout's class record (its wide records: 16-bit table ids)."""
    e, r, local, pool = cluster_engine(device, n_ns=n_ns, apps=apps)
    gen = dict(seed=SEEDS[9], ip_pool=pool, pool_pct=85, dst_pool_pct=88,
               port_pool=np.array(CLUSTER_PORTS, np.uint16), port_pool_pct=80, tcp_pct=60, udp_pct=30)
    return Workload(9, e, MODE_PERPOD, -1, gen, n_tuples,
                    "1k pods / 10 namespaces x 50 apps (~500 tables), evalACL on the dst interface", r,
                    local_ifs=local)


def config6(device=0, n_tuples=125 << 20, n_ns=10):
    """Config 3's shape given as K8s objects: namespace-wide selectors make
    the rule lists ~6.7x longer (64.6k rules in 52 tables)."""
    e, r, local, pool, keep = cluster_engine_k8s(device, n_ns=n_ns)
    gen = dict(seed=SEEDS[6], ip_pool=pool, pool_pct=85, dst_pool_pct=88,
               port_pool=np.array(CLUSTER_PORTS + [8000, 8001, 8002, 8003, 8004], np.uint16), port_pool_pct=80,
               tcp_pct=60, udp_pct=30)
    w = Workload(6, e, MODE_PERPOD, -1, gen, n_tuples,
                 "K8s objects (10 ns x 100 pods, label/namespace selectors) -> policy cache / processor / "
                 "configurator -> per-pod tables, evalACL on the dst interface", r, local_ifs=local)
    w.control = keep  # the cache / processor / configurator stay alive with the engine
    return w


def table_histogram(e):
    """rules per table -> number of tables (config 3's table-size histogram)."""
    h = {}
    for t in range(e.num_tables()):
        n = e.table_info(t)[1]
        h[n] = h.get(n, 0) + 1
    return dict(sorted(h.items()))


CONFIGS = {1: config1, 2: config2, 3: config3, 4: config4, 5: config5, 6: config6, 7: config7, 8: config8,
           9: config9}
