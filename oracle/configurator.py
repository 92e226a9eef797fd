"""Policy configurator and mock renderer (TEST INFRASTRUCTURE ONLY; see oracle/__init__.py).

CPU restatement of:
  * plugins/policy/configurator/configurator_impl.go:113-254   NewTxn / Configure / Commit
  * configurator_impl.go:263-472                                generateRules
  * configurator_impl.go:474-550                                ContivPolicies sort/Equals,
                                                                ContivRules.Insert/CopySlice
  * configurator_impl.go:562-594                                subtractSubnet
  * mock/renderer/renderer_mock.go:39-185                       MockRenderer (GetPodIP,
                                                                TestTraffic, Render, Commit)
Pinned by the 174 TestTraffic assertions of configurator_test.go
(tests/golden/configurator_kats.json). Go map iteration order does not affect results here
(every pod is rendered independently); pods are iterated in sorted order.

Policies are plain dicts as in the fixture: {"id": "ns/name", "type": 0|1|2, "matches":
[{"type": 0|1, "pods": [...] | None, "blocks": [{"network", "except"}] | None,
"ports": [{"protocol": 0|1, "number"}]}]} with CIDR strings.
"""
from __future__ import annotations

from . import gonet
from .gonet import IPNet
from .policy import ACTION_DENY, ACTION_PERMIT, ANY, TCP, UDP, ContivRule

POLICY_INGRESS, POLICY_EGRESS, POLICY_ALL = 0, 1, 2
MATCH_INGRESS, MATCH_EGRESS = 0, 1
PORT_TCP, PORT_UDP = 0, 1
INGRESS_TRAFFIC, EGRESS_TRAFFIC = 0, 1
DENIED, ALLOWED, UNMATCHED = 0, 1, 2


class ContivRules:
    """configurator_impl.go:517-550"""

    def __init__(self):
        self.ordered, self.rules = [], []

    def insert(self, rule: ContivRule) -> bool:
        lo, hi = 0, len(self.ordered)
        while lo < hi:  # sort.Search: first i with rule.Compare(ordered[i]) <= 0
            mid = (lo + hi) // 2
            if rule.compare(self.ordered[mid]) <= 0:
                hi = mid
            else:
                lo = mid + 1
        if lo < len(self.ordered) and rule.compare(self.ordered[lo]) == 0:
            return False
        self.ordered.insert(lo, rule)
        self.rules.append(rule)
        return True

    def copy_slice(self):
        return [r.copy() for r in self.rules]


def subtract_subnet(net1: IPNet, net2: IPNet):
    """configurator_impl.go:562-594"""
    ones1, _ = gonet.mask_size(net1.mask)
    ones2, _ = gonet.mask_size(net2.mask)
    if ones1 > ones2:
        return [] if gonet.contains(net2, net1.ip) else [net1]
    if ones1 == ones2:
        return [] if gonet.ip_equal(net1.ip, net2.ip) else [net1]
    if not gonet.contains(net1, net2.ip):
        return [net1]
    out = []
    for bit in range(ones1, ones2):
        mask = gonet.cidr_mask(bit + 1, len(net2.mask) * 8)
        ip = bytearray(gonet.ip_mask(net2.ip, mask))
        ip[bit // 8] ^= 1 << (7 - bit % 8)
        out.append(IPNet(bytes(ip), mask))
    return out


def _cidr(s):
    return gonet.parse_cidr(s)[1]


class PolicyConfigurator:
    def __init__(self, pod_ips, nat_loopback):
        """pod_ips: {"ns/name": IP string or "" (no address)} = the policy cache (LookupPod);
        pods missing from it are unknown. nat_loopback: IPAM.NatLoopbackIP() string."""
        self.pod_ips = dict(pod_ips)
        self.nat = gonet.parse_ip(nat_loopback) if nat_loopback else None
        self.renderers = []
        self.pod_ip_addresses = {}

    def new_txn(self, resync):
        return ConfiguratorTxn(self, resync)


class ConfiguratorTxn:
    def __init__(self, cfg, resync):
        self.cfg, self.resync, self.config = cfg, resync, {}
        self.pod_ip_addresses = {} if resync else dict(cfg.pod_ip_addresses)

    def configure(self, pod, policies):
        self.config[pod] = list(policies)

    def generate_rules(self, direction, policies) -> ContivRules:
        rules = ContivRules()
        has_policy = all_allowed = False

        def permit(proto=ANY, dport=0, src=None, dst=None):
            return ContivRule(ACTION_PERMIT, src or IPNet(), dst or IPNet(), proto, 0, dport)

        for policy in policies:
            if (policy["type"] == POLICY_INGRESS and direction == MATCH_EGRESS) or \
                    (policy["type"] == POLICY_EGRESS and direction == MATCH_INGRESS):
                continue
            has_policy = True
            for match in policy["matches"]:
                if match["type"] != direction:
                    continue
                peers = []
                for peer in match["pods"] or []:
                    ip = self.cfg.pod_ips.get(peer)
                    if not ip:
                        continue
                    n = gonet.one_host_subnet(ip)
                    if n is not None:
                        peers.append(n)
                subnets_all = []
                for block in match["blocks"] or []:
                    subnets = [_cidr(block["network"])]
                    for ex in block["except"]:
                        subnets = [s for sub in subnets for s in subtract_subnet(sub, _cidr(ex))]
                    subnets_all += subnets
                ports = match["ports"]
                proto = lambda p: TCP if p["protocol"] == PORT_TCP else UDP  # noqa: E731

                def with_peer(n, pr=ANY, dport=0):
                    return permit(pr, dport, src=n) if direction == MATCH_INGRESS else permit(pr, dport, dst=n)

                if match["pods"] is None and match["blocks"] is None:
                    if not ports:
                        rules.insert(permit())
                        all_allowed = True
                    else:
                        for p in ports:
                            rules.insert(permit(proto(p), p["number"]))
                for n in peers + subnets_all:
                    if not ports:
                        rules.insert(with_peer(n))
                    else:
                        for p in ports:
                            rules.insert(with_peer(n, proto(p), p["number"]))
        if has_policy and not all_allowed:
            if direction == MATCH_INGRESS:
                nat = gonet.one_host_subnet_from_ip(self.cfg.nat) if self.cfg.nat else IPNet(b"", gonet.cidr_mask(128, 128))
                rules.insert(permit(src=nat))
            rules.insert(ContivRule(ACTION_DENY, IPNet(), IPNet(), ANY, 0, 0))
        return rules

    def commit(self):
        processed = []
        txns = []
        for pod in sorted(self.config):
            ingress, egress = ContivRules(), ContivRules()
            had = pod in self.pod_ip_addresses
            pod_ip = self.pod_ip_addresses.get(pod)
            ip = self.cfg.pod_ips.get(pod)
            delete = False
            if not ip:
                if not had:
                    continue
                delete = True
                del self.pod_ip_addresses[pod]
            if not delete:
                pod_ip = gonet.one_host_subnet(ip)
                if pod_ip is None:
                    continue
                self.pod_ip_addresses[pod] = pod_ip
                policies = sorted(self.config[pod], key=lambda p: tuple(p["id"].split("/", 1)))
                ids = [p["id"] for p in policies]
                hit = [x for x in processed if x[0] == ids]
                if hit:
                    ingress, egress = hit[-1][1], hit[-1][2]
                else:
                    egress = self.generate_rules(MATCH_INGRESS, policies)
                    ingress = self.generate_rules(MATCH_EGRESS, policies)
                    processed.append((ids, ingress, egress))
            if not txns:
                txns = [r.new_txn(self.resync) for r in self.cfg.renderers]
            for t in txns:
                t.render(pod, pod_ip, ingress.copy_slice(), egress.copy_slice(), delete)
        for t in txns:
            t.commit()
        self.cfg.pod_ip_addresses = dict(self.pod_ip_addresses)


class MockRenderer:
    """mock/renderer/renderer_mock.go"""

    def __init__(self):
        self.config = {}

    def new_txn(self, resync):
        return _MockTxn(self, resync)

    def get_pod_ip(self, pod):
        c = self.config.get(pod)
        if c is None or c[0] is None:
            return "", 0
        return gonet.ip_string(c[0].ip), gonet.mask_size(c[0].mask)[0]

    def test_traffic(self, pod, direction, src_ip: str, dst_ip: str, protocol, sport, dport):
        c = self.config.get(pod)
        if c is None:
            return UNMATCHED
        src, dst = gonet.parse_ip(src_ip), gonet.parse_ip(dst_ip)
        for r in (c[1] if direction == INGRESS_TRAFFIC else c[2]):
            if not r.src.is_empty() and not gonet.contains(r.src, src):
                continue
            if not r.dst.is_empty() and not gonet.contains(r.dst, dst):
                continue
            if r.protocol != ANY:
                if r.protocol != protocol:
                    continue
                if r.src_port != 0 and r.src_port != sport:
                    continue
                if r.dst_port != 0 and r.dst_port != dport:
                    continue
            return ALLOWED if r.action == ACTION_PERMIT else DENIED
        return UNMATCHED


class _MockTxn:
    def __init__(self, r, resync):
        self.r, self.resync, self.config = r, resync, {}

    def render(self, pod, pod_ip, ingress, egress, removed):
        if removed:
            self.config.pop(pod, None)
        else:
            self.config[pod] = (pod_ip, ingress, egress)

    def commit(self):
        if self.resync:
            self.r.config = self.config
        else:
            self.r.config.update(self.config)
