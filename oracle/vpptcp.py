"""VPPTCP renderer and VPP session-rule tables (TEST INFRASTRUCTURE ONLY).

CPU restatement of:
  * plugins/policy/renderer/vpptcp/rule/session_rule.go   SessionRule (:73-86), Compare
    (:168-209), ExportSessionRules (:213-260), convertContivRule (:263-361),
    ImportSessionRules (:365-476)
  * plugins/policy/renderer/vpptcp/vpptcp_renderer.go     Renderer.Init (:59-69), Render
    (:88-98), Commit (:102-188), dumpRules (:191-234), updateRules (:264-316)
  * plugins/policy/renderer/cache/cache_api.go:321-334    ContivRuleTable.DiffRules
  * plugins/policy/utils/utils.go:261-267                 CompareIPNetsBytes
  * mock/sessionrules/sessionrules_mock.go                the session-rule tables: hasRule
    (:137-228), session_rule_add_del / session_rules_dump handling (:231-341), addDelRule
    (:344-364)
Only tests/ import this module. Pinned by the 97 assertions of vpptcp_renderer_test.go
(tests/golden/vpptcp_kats.json).

Where the reference iterates a Go map (pods of a transaction, the mock's local tables on a
dump, GetPodByAppNsIndex) this restatement iterates in sorted order; the results the tests
observe (table contents, counts) do not depend on that order. Where the reference would dereference
a nil PodIP (a pod whose configuration was rebuilt by a cache resync and is then removed, or
one rendered without an IP) this restatement raises policy.ReferencePanic; the product instead
treats the missing IP as matching no rule network.
"""
from __future__ import annotations

from . import gonet
from .gonet import IPNet
from . import policy as P

TAG_PREFIX = "contiv/vpp-policy"
ANY_PROTOCOL_TAG = "-ANY"
SPLIT_TAG = "-SPLIT"
SCOPE_GLOBAL, SCOPE_LOCAL, SCOPE_BOTH = 1, 2, 3
ACTION_DO_NOTHING = 0xFFFFFFFF
ACTION_DENY = 0xFFFFFFFF - 1
ACTION_ALLOW = 0xFFFFFFFF - 2
PROTO_TCP, PROTO_UDP = 0, 1


class SessionRule:
    __slots__ = ("transport_proto", "is_ip4", "lcl_ip", "lcl_plen", "rmt_ip", "rmt_plen", "lcl_port", "rmt_port",
                 "action_index", "appns_index", "scope", "tag")

    def __init__(self):
        self.transport_proto = 0
        self.is_ip4 = 0
        self.lcl_ip = bytearray(16)
        self.lcl_plen = 0
        self.rmt_ip = bytearray(16)
        self.rmt_plen = 0
        self.lcl_port = 0
        self.rmt_port = 0
        self.action_index = 0
        self.appns_index = 0
        self.scope = 0
        self.tag = bytearray(64)

    def copy(self) -> "SessionRule":
        c = SessionRule()
        for k in self.__slots__:
            v = getattr(self, k)
            setattr(c, k, bytearray(v) if isinstance(v, bytearray) else v)
        return c

    def set_tag(self, s: str):
        b = s.encode()[:64]
        self.tag = bytearray(b) + bytearray(64 - len(b))

    def tag_str(self) -> str:
        return bytes(self.tag).split(b"\0", 1)[0].decode()

    def key(self):
        """All fields as plain values (for comparing tables in tests)."""
        return (self.transport_proto, self.is_ip4, bytes(self.lcl_ip), self.lcl_plen, bytes(self.rmt_ip),
                self.rmt_plen, self.lcl_port, self.rmt_port, self.action_index, self.appns_index, self.scope,
                self.tag_str())

    def compare(self, o: "SessionRule", compare_tag: bool) -> int:
        """session_rule.go:168-209."""
        for a, b in ((self.appns_index, o.appns_index), (self.scope, o.scope),
                     (self.action_index, o.action_index), (self.is_ip4, o.is_ip4)):
            c = P.compare_ints(a, b)
            if c:
                return c
        c = compare_ipnets_bytes(self.lcl_plen, self.lcl_ip, o.lcl_plen, o.lcl_ip)
        if c:
            return c
        c = compare_ipnets_bytes(self.rmt_plen, self.rmt_ip, o.rmt_plen, o.rmt_ip)
        if c:
            return c
        for a, b in ((self.transport_proto, o.transport_proto), (self.lcl_port, o.lcl_port),
                     (self.rmt_port, o.rmt_port)):
            c = P.compare_ints(a, b)
            if c:
                return c
        if compare_tag:
            return P._bytes_compare(bytes(self.tag), bytes(o.tag))
        return 0


def compare_ipnets_bytes(ap, a, bp, b) -> int:
    """utils.go:261-267."""
    c = P.compare_ints(ap, bp)
    if c:
        return c
    return P._bytes_compare(bytes(a), bytes(b))


def _in_prefix(addr: int, ip: bytes, plen: int) -> bool:
    if plen == 0:
        return True
    if plen > 32:  # an IPv4 rule with an IPv6-length prefix (mixed-family ContivRule)
        return False
    net = int.from_bytes(bytes(ip[:4]), "big")
    m = (0xFFFFFFFF << (32 - plen)) & 0xFFFFFFFF
    return (addr & m) == (net & m)


def session_lookup(table, lcl_ip: int, lcl_port: int, rmt_ip: int, rmt_port: int, proto: int):
    """VPP's session-rule lookup over one table (the product: pg_session_table_install): the
    most specific IPv4 rule matching the connection -- specificity lcl_plen + rmt_plen + one
    per set port, ties to the rule first in SessionRule.Compare order (with tag) -- or None.
    A rule matches when its transport protocol is the packet's (proto: renderer.Protocol,
    TCP 0 / UDP 1, as the ACL engine's packets carry it), both
    addresses are inside its prefixes and each set port equals the packet's. VPP's own lookup
    is not in the reference: parity unpinned beyond this restatement, which follows the
    containment order renderer/api.go:111-112 gives the ContivRules the rules come from."""
    want = {0: 0, 1: 1}.get(proto)  # renderer.Protocol TCP / UDP -> TransportProto
    best = None
    for r in table:
        if not r.is_ip4 or want is None or r.transport_proto != want:
            continue
        if not (_in_prefix(lcl_ip, r.lcl_ip, r.lcl_plen) and _in_prefix(rmt_ip, r.rmt_ip, r.rmt_plen)):
            continue
        if (r.lcl_port and r.lcl_port != lcl_port) or (r.rmt_port and r.rmt_port != rmt_port):
            continue
        w = r.lcl_plen + r.rmt_plen + (r.lcl_port != 0) + (r.rmt_port != 0)
        if best is None or w > best[0] or (w == best[0] and r.compare(best[1], True) < 0):
            best = (w, r)
    return None if best is None else best[1]


class IPv4Net:
    """The renderer's IPv4Net dependency (session_rule.go:88-95), as the test's mock."""

    def __init__(self):
        self.pod_to_ns = {}

    def set_pod_app_ns_index(self, pod, idx):
        self.pod_to_ns[pod] = idx

    def get_ns_index(self, pod):
        return self.pod_to_ns.get(pod)

    def get_pod_by_app_ns_index(self, idx):
        for pod in sorted(self.pod_to_ns):
            if self.pod_to_ns[pod] == idx:
                return pod
        return None


def _copy(dst: bytearray, ip):
    """copy(dst[:], ip)."""
    if ip:
        dst[:len(ip)] = ip


def _plen(mask) -> int:
    return gonet.mask_size(mask)[0]


def _convert(rule: P.ContivRule, glob: bool, ns_index: int, tag_prefix: str):
    """convertContivRule (session_rule.go:263-361)."""
    sr = SessionRule()
    sr.transport_proto = PROTO_TCP if rule.protocol == P.TCP else PROTO_UDP
    if glob and (len(rule.src.ip) == 0 or gonet.to4(rule.src.ip) is not None):
        sr.is_ip4 = 1
    if not glob and (len(rule.dst.ip) == 0 or gonet.to4(rule.dst.ip) is not None):
        sr.is_ip4 = 1
    if glob:
        _copy(sr.lcl_ip, gonet.to4(rule.dst.ip) if sr.is_ip4 else gonet.to16(rule.dst.ip))
        sr.lcl_plen = _plen(rule.dst.mask)
    sr.lcl_port = rule.dst_port if glob else rule.src_port
    rmt = rule.src if glob else rule.dst
    if len(rmt.ip) > 0:
        _copy(sr.rmt_ip, gonet.to4(rmt.ip) if sr.is_ip4 else gonet.to16(rmt.ip))
        sr.rmt_plen = _plen(rmt.mask)
    sr.rmt_port = rule.src_port if glob else rule.dst_port
    sr.action_index = ACTION_ALLOW if rule.action == P.ACTION_PERMIT else ACTION_DENY
    sr.appns_index = ns_index
    sr.scope = SCOPE_GLOBAL if glob else SCOPE_LOCAL
    if (glob and len(rule.src.ip) == 0) or (not glob and len(rule.dst.ip) == 0):
        sr.rmt_plen = 1
        sr2 = sr.copy()
        sr.set_tag(tag_prefix + SPLIT_TAG)
        sr2.rmt_ip[0] = 1 << 7
        sr2.set_tag(tag_prefix + SPLIT_TAG)
        return [sr, sr2]
    sr.set_tag(tag_prefix)
    return [sr]


def export_session_rules(rules, pod, pod_ip: bytes, ipv4net: IPv4Net):
    """session_rule.go:213-260 (pod None: global table)."""
    glob = pod is None
    out = []
    ns_index = 0
    if not glob:
        ns_index = ipv4net.get_ns_index(pod)
        if ns_index is None:
            return out
    for rule in rules:
        if rule.dst_port == 0 and rule.action == P.ACTION_PERMIT and (
                (glob and len(rule.src.ip) == 0) or (not glob and len(rule.dst.ip) == 0)):
            continue
        if not glob and len(rule.dst.ip) > 0:
            ones, bits = gonet.mask_size(rule.dst.mask)
            if ones == bits and gonet.ip_equal(rule.dst.ip, pod_ip or b""):
                continue
        if rule.protocol == P.ANY:
            tcp, udp = rule.copy(), rule.copy()
            tcp.protocol, udp.protocol = P.TCP, P.UDP
            out += _convert(tcp, glob, ns_index, TAG_PREFIX + ANY_PROTOCOL_TAG)
            out += _convert(udp, glob, ns_index, TAG_PREFIX + ANY_PROTOCOL_TAG)
        else:
            out += _convert(rule, glob, ns_index, TAG_PREFIX)
    return out


def import_session_rules(rules, ipv4net: IPv4Net):
    """session_rule.go:365-476."""
    glob = P.ContivRuleTable(P.GLOBAL)
    local = {}
    for rule in rules:
        rule = rule.copy()
        cr = P.ContivRule()
        tag = rule.tag_str()
        if tag.endswith(SPLIT_TAG):
            if rule.rmt_ip[0] != 0:
                continue
            rule.rmt_plen = 0
            tag = tag[:-len(SPLIT_TAG)]
        if tag.endswith(ANY_PROTOCOL_TAG):
            if rule.transport_proto == PROTO_UDP:
                continue
            cr.protocol = P.ANY
        else:
            cr.protocol = P.UDP if rule.transport_proto == PROTO_UDP else P.TCP
        g = rule.scope == SCOPE_GLOBAL
        sip, splen = (rule.rmt_ip, rule.rmt_plen) if g else (rule.lcl_ip, rule.lcl_plen)
        dip, dplen = (rule.lcl_ip, rule.lcl_plen) if g else (rule.rmt_ip, rule.rmt_plen)
        iplen = 4 if rule.is_ip4 > 0 else 16
        cr.src = IPNet(bytes(sip[:iplen]), gonet.cidr_mask(splen, iplen * 8)) if splen > 0 else IPNet()
        cr.dst = IPNet(bytes(dip[:iplen]), gonet.cidr_mask(dplen, iplen * 8)) if dplen > 0 else IPNet()
        cr.src_port, cr.dst_port = (rule.rmt_port, rule.lcl_port) if g else (rule.lcl_port, rule.rmt_port)
        cr.action = P.ACTION_PERMIT if rule.action_index == ACTION_ALLOW else P.ACTION_DENY
        if g:
            glob.insert_rule(cr)
            continue
        pod = ipv4net.get_pod_by_app_ns_index(rule.appns_index)
        if pod is None:
            continue
        if pod not in local:
            t = P.ContivRuleTable(P.LOCAL)
            t.pods.add(pod)
            local[pod] = t
        local[pod].insert_rule(cr)
    return [glob] + [local[p] for p in sorted(local)]


def diff_rules(a: P.ContivRuleTable, b: P.ContivRuleTable):
    """cache_api.go:321-334 -> (not in b, not in a)."""
    return [r for r in a.rules if not b.has_rule(r)], [r for r in b.rules if not a.has_rule(r)]


class SessionRuleTables:
    """mock/sessionrules: VPP's session-rule tables behind the binary API."""

    def __init__(self, tag_prefix=TAG_PREFIX):
        self.tag_prefix = tag_prefix
        self.clear()

    def clear(self):
        self.local = {}
        self.glob = []
        self.err_count = 0
        self.req_count = 0

    @staticmethod
    def _add_del(table, rule, is_add):
        for i, r2 in enumerate(table):
            if rule.compare(r2, not is_add) == 0:
                if is_add:
                    return False
                del table[i]
                return True
        if is_add:
            table.append(rule)
            return True
        return False

    def add_del(self, rule: SessionRule, is_add: bool) -> int:
        self.req_count += 1
        if not rule.tag_str().startswith(self.tag_prefix):
            self.err_count += 1
            return 1
        rule = rule.copy()
        table = self.local.setdefault(rule.appns_index, []) if rule.scope == SCOPE_LOCAL else self.glob
        if not self._add_del(table, rule, is_add):
            self.err_count += 1
            return 1
        return 0

    def dump(self):
        self.req_count += 2  # session_rules_dump + control_ping
        out = []
        for ns in sorted(self.local):
            out += [r.copy() for r in self.local[ns]]
        return out + [r.copy() for r in self.glob]

    def table(self, scope, ns):
        return self.local.get(ns) if scope == SCOPE_LOCAL else self.glob

    def has_rule(self, scope, ns, lcl_ip, lcl_port, rmt_ip, rmt_port, proto, action) -> bool:
        """sessionrules_mock.go:137-228."""
        table = self.table(scope, ns)
        if table is None:
            return False
        r = SessionRule()
        r.lcl_port, r.rmt_port = lcl_port, rmt_port
        r.appns_index = ns if scope == SCOPE_LOCAL else 0
        r.scope = scope
        r.transport_proto = {"TCP": PROTO_TCP, "UDP": PROTO_UDP}.get(proto, 0)
        r.action_index = {"ALLOW": ACTION_ALLOW, "DENY": ACTION_DENY}.get(action, 0)
        is4 = 0
        for s, dst, attr in ((lcl_ip, r.lcl_ip, "lcl_plen"), (rmt_ip, r.rmt_ip, "rmt_plen")):
            if not s:
                continue
            if "/" not in s:
                ip = gonet.parse_ip(s)
                if ip is None:
                    return False
                n = gonet.one_host_subnet_from_ip(ip)
            else:
                p = gonet.parse_cidr(s)
                if p is None:
                    return False
                n = p[1]
            v4 = gonet.to4(n.ip)
            if v4 is not None:
                is4 = 1
                _copy(dst, v4)
            else:
                _copy(dst, gonet.to16(n.ip))
            setattr(r, attr, _plen(n.mask))
        if not lcl_ip and not rmt_ip:
            is4 = 1
        r.is_ip4 = is4
        return any(r.compare(x, False) == 0 for x in table)


class Renderer:
    """vpptcp.Renderer over SessionRuleTables (the govpp channel peer)."""

    def __init__(self, ipv4net: IPv4Net, vpp: SessionRuleTables, chan_buf_size=0):
        self.ipv4net, self.vpp, self.chan_buf_size = ipv4net, vpp, chan_buf_size
        self.cache = P.RendererCache(P.INGRESS_ORIENTATION)

    def new_txn(self, resync):
        return RendererTxn(self, resync)

    def update_rules(self, add, remove):
        """vpptcp_renderer.go:264-316."""
        reqs = [(r, False) for r in remove] + [(r, True) for r in add]
        burst = self.chan_buf_size or 100
        i = 0
        while i < len(reqs):
            chunk = reqs[i:i + burst]
            i += len(chunk)
            rvs = [self.vpp.add_del(r, a) for r, a in chunk]
            if any(rvs):
                return "failed to update VPPTCP session rule"
        return None


class RendererTxn:
    def __init__(self, r: Renderer, resync: bool):
        self.r, self.resync = r, resync
        self.cache_txn = r.cache.new_txn()

    def render(self, pod, pod_ip, ingress, egress, removed):
        self.cache_txn.update(pod, P.PodConfig(pod_ip, list(ingress), list(egress), removed))
        return self

    def commit(self):
        """vpptcp_renderer.go:102-188 -> None or an error string."""
        r = self.r
        added, removed = [], []
        if self.resync:
            dumped = [x for x in r.vpp.dump() if x.tag_str().startswith(TAG_PREFIX)]
            err = r.cache.resync(import_session_rules(dumped, r.ipv4net))
            if err:
                return err
            txn_pods = self.cache_txn.get_updated_pods()
            for pod in sorted(r.cache.get_all_pods()):
                if pod not in txn_pods:
                    self.cache_txn.update(pod, P.PodConfig(removed=True))
        for pod in sorted(self.cache_txn.get_updated_pods()):
            cfg = self.cache_txn.get_pod_config(pod)
            if cfg.removed:
                cfg = r.cache.get_pod_config(pod)
                if cfg is None:
                    continue
            new, gone = [], []
            orig = r.cache.get_local_table_by_pod(pod)
            nxt = self.cache_txn.get_local_table_by_pod(pod)
            if orig is None and nxt is not None:
                new = list(nxt.rules)
            if orig is not None and nxt is None:
                gone = list(orig.rules)
            if orig is not None and nxt is not None and orig.get_id() != nxt.get_id():
                gone, new = diff_rules(orig, nxt)
            if cfg.pod_ip is None:  # podCfg.PodIP.IP on a nil *net.IPNet
                raise P.ReferencePanic("nil PodIP in vpptcp Commit (pod %s)" % (pod,))
            ip = cfg.pod_ip.ip
            added += export_session_rules(new, pod, ip, r.ipv4net)
            removed += export_session_rules(gone, pod, ip, r.ipv4net)
        gone, new = diff_rules(r.cache.get_global_table(), self.cache_txn.get_global_table())
        added += export_session_rules(new, None, None, r.ipv4net)
        removed += export_session_rules(gone, None, None, r.ipv4net)
        if added or removed:
            err = r.update_rules(added, removed)
            if err:
                return err
        self.cache_txn.commit()
        return None
