"""ContivRule ordering, rule tables, renderer cache and ACL renderer (TEST INFRASTRUCTURE ONLY).

CPU restatement of:
  * plugins/policy/renderer/api.go:65-191         ContivRule, Compare, String, enums
  * plugins/policy/utils/utils.go:175-291          CompareInts/IPNets/Ports, GetOneHostSubnet
  * plugins/policy/renderer/cache/cache_api.go     ContivRuleTable (InsertRule :268, getRuleIndex
                                                   :338, RemoveByPredicate :301, GetID :249)
  * plugins/policy/renderer/cache/local_tables.go  LocalTables, compareRuleLists :242
  * plugins/policy/renderer/cache/ports.go         Ports, getAllowed{Ingress,Egress}Ports
  * plugins/policy/renderer/cache/cache_impl.go    RendererCache/Txn (refreshTables :409,
                                                   buildLocalTable :470, installLocalRules :519,
                                                   installAllowedPorts :590, rebuildGlobalTable :622)
  * plugins/policy/renderer/acl/acl_renderer.go    Renderer/Txn Render/Commit/commitResync,
                                                   reflectiveACL, renderACL, renderInterfaces
Go map iteration order is randomised by the runtime; every place where the reference
iterates a map, the result is order-independent (sorted inserts, set semantics) and this
restatement iterates in a fixed order.
"""
from __future__ import annotations

import bisect
from dataclasses import dataclass, field

from . import gonet
from .gonet import IPNet

# --- enums (api.go:140-176) -------------------------------------------------
ACTION_DENY, ACTION_PERMIT = 0, 1
TCP, UDP, OTHER, ANY = 0, 1, 2, 3
ANY_PORT = 0


def action_string(a: int) -> str:
    return {ACTION_DENY: "DENY", ACTION_PERMIT: "PERMIT"}.get(a, "INVALID")


def proto_string(p: int) -> str:
    return {TCP: "TCP", UDP: "UDP", OTHER: "OTHER", ANY: "ANY"}.get(p, "INVALID")


@dataclass
class ContivRule:
    """renderer.ContivRule (api.go:65-77)."""
    action: int = ACTION_PERMIT
    src: IPNet = field(default_factory=IPNet)
    dst: IPNet = field(default_factory=IPNet)
    protocol: int = ANY
    src_port: int = 0
    dst_port: int = 0

    def copy(self) -> "ContivRule":
        return ContivRule(self.action, self.src, self.dst, self.protocol, self.src_port, self.dst_port)

    def string(self) -> str:
        """api.go:81-101."""
        src = "ANY" if self.src.is_empty() else gonet.ipnet_string(self.src)
        dst = "ANY" if self.dst.is_empty() else gonet.ipnet_string(self.dst)
        sp = "ANY" if self.src_port == 0 else str(self.src_port)
        dp = "ANY" if self.dst_port == 0 else str(self.dst_port)
        pr = proto_string(self.protocol)
        return "Rule <%s %s[%s:%s] -> %s[%s:%s]>" % (action_string(self.action), src, pr, sp, dst, pr, dp)

    def compare(self, o: "ContivRule") -> int:
        """api.go:113-137."""
        c = compare_ipnets(self.src, o.src)
        if c:
            return c
        c = compare_ipnets(self.dst, o.dst)
        if c:
            return c
        c = compare_ints(self.protocol, o.protocol)
        if c:
            return c
        if self.protocol != ANY:
            c = compare_ports(self.src_port, o.src_port)
            if c:
                return c
            c = compare_ports(self.dst_port, o.dst_port)
            if c:
                return c
        return compare_ints(self.action, o.action)


def compare_ints(a: int, b: int) -> int:
    """utils.go:175-183."""
    return -1 if a < b else (1 if a > b else 0)


def _bytes_compare(a: bytes, b: bytes) -> int:
    return -1 if a < b else (1 if a > b else 0)


def compare_ipnets(a: IPNet, b: IPNet) -> int:
    """utils.go:187-239."""
    if len(a.ip) == 0:
        return 0 if len(b.ip) == 0 else 1
    if len(b.ip) == 0:
        return -1
    a4, b4 = gonet.to4(a.ip), gonet.to4(b.ip)
    if a4 is not None:
        if b4 is None:
            return -1
        an = IPNet(a4, a.mask)
    else:
        an = IPNet(gonet.to16(a.ip), a.mask)
    if b4 is not None:
        if a4 is None:
            return 1
        bn = IPNet(b4, b.mask)
    else:
        bn = IPNet(gonet.to16(b.ip), b.mask)
    a_ones, bits = gonet.mask_size(an.mask)
    b_ones, _ = gonet.mask_size(bn.mask)
    common = min(a_ones, b_ones)
    cm = gonet.cidr_mask(common, bits)
    am, bm = gonet.ip_mask(an.ip, cm), gonet.ip_mask(bn.ip, cm)
    if am is not None and bm is not None and gonet.ip_equal(am, bm) or (am is None and bm is None):
        return compare_ints(b_ones, a_ones)
    c = _bytes_compare(bn.mask, an.mask)
    if c:
        return c
    return _bytes_compare(an.ip, bn.ip)


def compare_ports(a: int, b: int) -> int:
    """utils.go:243-257."""
    if a == b:
        return 0
    if a == 0:
        return 1
    if b == 0:
        return -1
    return -1 if a < b else 1


def allow_all() -> ContivRule:
    return ContivRule(ACTION_PERMIT, IPNet(), IPNet(), ANY, 0, 0)


def deny_all() -> ContivRule:
    return ContivRule(ACTION_DENY, IPNet(), IPNet(), ANY, 0, 0)


def fnv64a(data: bytes) -> int:
    h = 0xCBF29CE484222325
    for c in data:
        h ^= c
        h = (h * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
    return h


# --- ContivRuleTable (cache_api.go:208-347) ---------------------------------
LOCAL, GLOBAL = 0, 1
GLOBAL_TABLE_ID = "NODE-GLOBAL"


class ContivRuleTable:
    def __init__(self, ttype: int = LOCAL):
        self.type = ttype
        self.pods: set = set()
        self.rules: list = []          # == Rules[:NumOfRules]
        self.slice_len = 0             # == len(Rules): nil-padded high-water mark
        self.private = None
        self._id = ""

    @property
    def num_rules(self) -> int:
        return len(self.rules)

    def get_id(self) -> str:
        if self._id:
            return self._id
        if self.type == GLOBAL:
            self._id = GLOBAL_TABLE_ID
        else:
            s = "[" + " ".join(r.string() for r in self.rules) + "]"
            self._id = "%x" % fnv64a(s.encode())
        return self._id

    def _index(self, rule):
        lo, hi = 0, len(self.rules)
        while lo < hi:                      # sort.Search(n, rule.Compare(Rules[i]) <= 0)
            mid = (lo + hi) // 2
            if rule.compare(self.rules[mid]) <= 0:
                hi = mid
            else:
                lo = mid + 1
        return lo, (lo < len(self.rules) and rule.compare(self.rules[lo]) == 0)

    def insert_rule(self, rule) -> bool:
        idx, present = self._index(rule)
        if present:
            return False
        if len(self.rules) == self.slice_len:
            self.slice_len += 1
        self.rules.insert(idx, rule)
        return True

    def has_rule(self, rule) -> bool:
        return self._index(rule)[1]

    def remove_by_predicate(self, pred) -> int:
        n0 = len(self.rules)
        self.rules = [r for r in self.rules if not pred(r)]
        return n0 - len(self.rules)


def compare_rule_lists(a, b) -> int:
    """local_tables.go:242-263."""
    if a is None and b is None:
        return 0
    if a is None:
        return -1
    if b is None:
        return 1
    c = compare_ints(len(a), len(b))
    if c:
        return c
    for x, y in zip(a, b):
        c = x.compare(y)
        if c:
            return c
    return 0


class ReferencePanic(RuntimeError):
    """The reference would dereference a nil pointer here (Go panic): a nil *ContivRule, or
    the nil PodIP of a pod configuration rebuilt by a cache resync."""


def compare_rules_to_padded(a, table) -> int:
    """compareRuleLists(rules, table.Rules) with the *untrimmed* slice, as used by
    lookupIdxByRules (local_tables.go:233-238)."""
    c = compare_ints(len(a), table.slice_len)
    if c:
        return c
    for i, x in enumerate(a):
        if i >= table.num_rules:
            raise ReferencePanic("nil rule in compareRuleLists")
        c = x.compare(table.rules[i])
        if c:
            return c
    return 0


class LocalTables:
    """local_tables.go:43-263."""

    def __init__(self):
        self.tables: list = []
        self.by_id: dict = {}
        self.by_pod: dict = {}

    def _idx_by_rules(self, rules):
        lo, hi = 0, len(self.tables)
        while lo < hi:
            mid = (lo + hi) // 2
            if compare_rules_to_padded(rules, self.tables[mid]) <= 0:
                hi = mid
            else:
                lo = mid + 1
        return lo

    def insert(self, table) -> bool:
        if table.get_id() in self.by_id:
            return False
        idx = self._idx_by_rules(table.rules)
        self.tables.insert(idx, table)
        self.by_id[table.get_id()] = table
        for pod in sorted(table.pods):
            self.unassign_pod(None, pod)
            self.by_pod[pod] = table
        return True

    def remove(self, table) -> bool:
        for i, t in enumerate(self.tables):
            if t is table:
                del self.tables[i]
                self.by_id.pop(table.get_id(), None)
                for pod in list(table.pods):
                    self.by_pod.pop(pod, None)
                return True
        return False

    def assign_pod(self, table, pod):
        self.unassign_pod(None, pod)
        table.pods.add(pod)
        self.by_pod[pod] = table

    def unassign_pod(self, table, pod):
        if table is not None:
            table.pods.discard(pod)
        t2 = self.by_pod.get(pod)
        if t2 is not None and (table is None or table is t2):
            t2.pods.discard(pod)
            del self.by_pod[pod]

    def lookup_by_id(self, tid):
        return self.by_id.get(tid)

    def lookup_by_rules(self, rules):
        idx = self._idx_by_rules(rules)
        if idx < len(self.tables) and compare_rule_lists(rules, self.tables[idx].rules) == 0:
            return self.tables[idx]
        return None

    def lookup_by_pod(self, pod):
        return self.by_pod.get(pod)

    def isolated_pods(self) -> set:
        return {p for p, t in self.by_pod.items() if t.num_rules > 0}


# --- Ports (ports.go) -------------------------------------------------------
class Ports(set):
    def has(self, port):
        return 0 in self or port in self

    def is_subset_of(self, p2) -> bool:
        if p2.has(ANY_PORT):
            return True
        if self.has(ANY_PORT):
            return False
        return all(p2.has(p) for p in self)

    def intersection(self, p2):
        if self.has(ANY_PORT):
            return p2
        if p2.has(ANY_PORT):
            return self
        return Ports(p for p in self if p2.has(p))


def allowed_egress_ports(src_ip: IPNet, egress):
    """ports.go:107-137."""
    tcp, udp, anyp, has_deny = Ports(), Ports(), False, False
    for r in egress:
        if r.action == ACTION_DENY:
            has_deny = True
            continue
        if not r.src.is_empty():
            if src_ip is None:
                raise ReferencePanic("nil pod IP in getAllowedEgressPorts")
            if not gonet.contains(r.src, src_ip.ip):
                continue
        if r.protocol == TCP:
            tcp.add(r.dst_port)
        elif r.protocol == UDP:
            udp.add(r.dst_port)
        elif r.protocol == ANY:
            tcp.add(0)
            udp.add(0)
            anyp = True
    if not has_deny:
        return Ports([0]), Ports([0]), True
    return tcp, udp, anyp


def allowed_ingress_ports(dst_ip: IPNet, ingress):
    """ports.go:141-171."""
    tcp, udp, anyp, has_deny = Ports(), Ports(), False, False
    for r in ingress:
        if r.action == ACTION_DENY:
            has_deny = True
            continue
        if not r.dst.is_empty():
            if dst_ip is None:
                raise ReferencePanic("nil pod IP in getAllowedIngressPorts")
            if not gonet.contains(r.dst, dst_ip.ip):
                continue
        if r.protocol == TCP:
            tcp.add(r.dst_port)
        elif r.protocol == UDP:
            udp.add(r.dst_port)
        elif r.protocol == ANY:
            tcp.add(0)
            udp.add(0)
            anyp = True
    if not has_deny:
        return Ports([0]), Ports([0]), True
    return tcp, udp, anyp


# --- Renderer cache (cache_impl.go) -----------------------------------------
INGRESS_ORIENTATION, EGRESS_ORIENTATION = 0, 1


@dataclass
class PodConfig:
    pod_ip: IPNet = None
    ingress: list = field(default_factory=list)
    egress: list = field(default_factory=list)
    removed: bool = False


@dataclass
class TxnChange:
    table: ContivRuleTable
    previous_pods: set


class RendererCache:
    def __init__(self, orientation=EGRESS_ORIENTATION):
        self.orientation = orientation
        self.flush()

    def flush(self):
        self.local_tables = LocalTables()
        self.global_table = ContivRuleTable(GLOBAL)
        self.global_table.get_id()
        self.config: dict = {}

    def new_txn(self):
        return RendererCacheTxn(self)

    def resync(self, tables):
        """cache_impl.go:100-138."""
        config, local, glob = {}, LocalTables(), ContivRuleTable(GLOBAL)
        for t in tables:
            if t is None:
                continue
            if t.type == GLOBAL:
                glob = t
                continue
            if len(t.pods) == 0:
                continue
            local.insert(t)
            for pod in t.pods:
                if pod in config:
                    return "pod assigned to multiple local tables: %s" % pod
                config[pod] = PodConfig()
        self.local_tables, self.global_table, self.config = local, glob, config
        return None

    def get_pod_config(self, pod):
        return self.config.get(pod)

    def get_all_pods(self) -> set:
        return set(self.config)

    def get_isolated_pods(self) -> set:
        return self.local_tables.isolated_pods()

    def get_local_table_by_pod(self, pod):
        t = self.local_tables.lookup_by_pod(pod)
        if t is not None and t.num_rules == 0:
            return None
        return t

    def get_global_table(self):
        return self.global_table


def _shallow_table(src: ContivRuleTable, pods) -> ContivRuleTable:
    t = ContivRuleTable(src.type)
    t.rules = src.rules          # shallow copy of rules, as in cache_impl.go:419-425
    t.slice_len = src.slice_len
    t.pods = set(pods)
    t.private = src.private
    return t


class RendererCacheTxn:
    def __init__(self, cache: RendererCache):
        self.cache = cache
        self.local_tables = LocalTables()
        self.global_table = None
        self.up_to_date = False
        self.config: dict = {}

    # --- View
    def update(self, pod, cfg: PodConfig):
        self.config[pod] = cfg
        self.up_to_date = False

    def get_updated_pods(self) -> set:
        return set(self.config)

    def get_removed_pods(self) -> set:
        return {p for p, c in self.config.items() if c.removed}

    def get_pod_config(self, pod):
        if pod in self.config:
            return self.config[pod]
        return self.cache.get_pod_config(pod)

    def get_all_pods(self) -> set:
        pods = self.cache.get_all_pods()
        for p, c in self.config.items():
            if not c.removed:
                pods.add(p)
            else:
                pods.discard(p)
        return pods

    def get_isolated_pods(self) -> set:
        if not self.up_to_date:
            self.refresh_tables()
        iso = self.local_tables.isolated_pods()
        for pod in self.cache.get_isolated_pods():
            if self.local_tables.lookup_by_pod(pod) is None:
                iso.add(pod)
        return iso

    def get_local_table_by_pod(self, pod):
        if not self.up_to_date:
            self.refresh_tables()
        t = self.local_tables.lookup_by_pod(pod)
        if t is not None and t.num_rules == 0:
            return None
        if t is not None:
            return t
        return self.cache.get_local_table_by_pod(pod)

    def get_global_table(self):
        if not self.up_to_date:
            self.refresh_tables()
        if self.global_table is not None:
            return self.global_table
        return self.cache.global_table

    # --- changes / commit
    def get_changes(self):
        if not self.up_to_date:
            self.refresh_tables()
        changes = []
        for t in self.local_tables.tables:
            orig = self.cache.local_tables.lookup_by_id(t.get_id())
            if t.num_rules == 0:
                continue
            if len(t.pods) == 0 and orig is None:
                continue
            if orig is not None and t.pods == orig.pods:
                continue
            changes.append(TxnChange(t, set(orig.pods) if orig is not None else set()))
        if self.global_table is not None and compare_rule_lists(
                self.global_table.rules, self.cache.global_table.rules) != 0:
            changes.append(TxnChange(self.global_table, set()))
        return changes

    def commit(self):
        if not self.up_to_date:
            self.refresh_tables()
        c = self.cache
        for t in self.local_tables.tables:
            orig = c.local_tables.lookup_by_id(t.get_id())
            if orig is not None:
                if len(t.pods) == 0:
                    c.local_tables.remove(t)
                elif t.pods != orig.pods:
                    for pod in sorted(orig.pods):
                        if pod not in t.pods:
                            c.local_tables.unassign_pod(orig, pod)
                    for pod in sorted(t.pods):
                        if pod not in orig.pods:
                            c.local_tables.assign_pod(orig, pod)
                    orig.private = t.private
            elif len(t.pods) != 0:
                c.local_tables.insert(t)
        if self.global_table is not None and compare_rule_lists(
                self.global_table.rules, c.global_table.rules) != 0:
            c.global_table = self.global_table
        for pod, cfg in sorted(self.config.items()):
            if cfg.removed:
                c.config.pop(pod, None)
                c.local_tables.unassign_pod(None, pod)
            else:
                c.config[pod] = cfg

    # --- table derivation
    def refresh_tables(self):
        for pod in sorted(self.get_all_pods() | self.get_removed_pods()):
            cfg = self.get_pod_config(pod)
            new_table = self.build_local_table(pod, cfg)
            orig = self.cache.local_tables.lookup_by_pod(pod)
            if orig is not None and self.local_tables.lookup_by_id(orig.get_id()) is None:
                self.local_tables.insert(_shallow_table(orig, orig.pods))
            txn_table = self.local_tables.lookup_by_rules(new_table.rules)
            if txn_table is not None:
                self.local_tables.assign_pod(txn_table, pod)
                continue
            cache_table = self.cache.local_tables.lookup_by_rules(new_table.rules)
            if cache_table is not None:
                t = _shallow_table(cache_table, cache_table.pods)
                t.pods.add(pod)
                self.local_tables.insert(t)
                continue
            self.local_tables.insert(new_table)
        self.rebuild_global_table()
        self.up_to_date = True

    def build_local_table(self, dst_pod, dst_cfg: PodConfig) -> ContivRuleTable:
        table = ContivRuleTable(LOCAL)
        table.pods.add(dst_pod)
        if dst_cfg.removed:
            return table
        rules = dst_cfg.egress if self.cache.orientation == EGRESS_ORIENTATION else dst_cfg.ingress
        for r in rules:
            table.insert_rule(r.copy())
        for src_pod in sorted(self.get_all_pods()):
            self.install_local_rules(table, dst_cfg, self.get_pod_config(src_pod))
        # cache_impl.go:496 tests len(table.Rules) (the slice, nil-padded after removals); the
        # slice only grows and installLocalRules always re-inserts after removing, so this
        # equals "NumOfRules > 0" here.
        if table.slice_len > 0:
            all_matched = any(r.protocol == ANY and r.dst_port == 0 and r.src.is_empty() and r.dst.is_empty()
                              for r in table.rules)
            if not all_matched:
                table.insert_rule(allow_all())
        return table

    def install_local_rules(self, dst_table, dst_cfg: PodConfig, src_cfg: PodConfig):
        egress_or = self.cache.orientation == EGRESS_ORIENTATION
        if egress_or:
            src_tcp, src_udp, src_any = allowed_ingress_ports(dst_cfg.pod_ip, src_cfg.ingress)
            dst_tcp, dst_udp, dst_any = allowed_egress_ports(src_cfg.pod_ip, dst_cfg.egress)
        else:
            src_tcp, src_udp, src_any = allowed_egress_ports(dst_cfg.pod_ip, src_cfg.egress)
            dst_tcp, dst_udp, dst_any = allowed_ingress_ports(src_cfg.pod_ip, dst_cfg.ingress)
        if src_any:
            return
        if dst_any or not dst_tcp.is_subset_of(src_tcp) or not dst_udp.is_subset_of(src_udp):
            def pred(rule):
                addr = rule.src if egress_or else rule.dst
                if addr.is_empty():
                    return False
                ones, bits = gonet.mask_size(addr.mask)
                if ones != bits or not gonet.ip_equal(addr.ip, src_cfg.pod_ip.ip):
                    return False
                return True
            dst_table.remove_by_predicate(pred)
            self.install_allowed_ports(dst_table, src_cfg.pod_ip, dst_tcp.intersection(src_tcp), TCP)
            self.install_allowed_ports(dst_table, src_cfg.pod_ip, dst_udp.intersection(src_udp), UDP)
            r = ContivRule(ACTION_DENY, IPNet(), IPNet(), ANY, 0, 0)
            if egress_or:
                r.src = src_cfg.pod_ip
            else:
                r.dst = src_cfg.pod_ip
            dst_table.insert_rule(r)

    def install_allowed_ports(self, dst_table, src_pod_ip, ports: Ports, proto):
        tmpl = ContivRule(ACTION_PERMIT, IPNet(), IPNet(), proto, 0, 0)
        if self.cache.orientation == EGRESS_ORIENTATION:
            tmpl.src = src_pod_ip
        else:
            tmpl.dst = src_pod_ip
        if 0 in ports:
            dst_table.insert_rule(tmpl)
            return
        for port in sorted(ports):
            r = tmpl.copy()
            r.dst_port = port
            dst_table.insert_rule(r)

    def rebuild_global_table(self):
        self.global_table = ContivRuleTable(GLOBAL)
        for pod in sorted(self.get_all_pods()):
            cfg = self.get_pod_config(pod)
            rules = cfg.ingress if self.cache.orientation == EGRESS_ORIENTATION else cfg.egress
            for r in rules:
                rc = r.copy()
                if self.cache.orientation == EGRESS_ORIENTATION:
                    rc.src = cfg.pod_ip
                else:
                    rc.dst = cfg.pod_ip
                self.global_table.insert_rule(rc)
        if self.global_table.num_rules > 0:
            self.global_table.insert_rule(allow_all())


# --- vpp_acl model (vendor/.../api/models/vpp/acl/acl.proto:24-113) ---------
ACL_DENY, ACL_PERMIT, ACL_REFLECT = 0, 1, 2
MAX_PORT = 0xFFFF


@dataclass
class PortRange:
    lower: int = 0
    upper: int = 0


@dataclass
class L4Section:                 # ACL_Rule_IpRule_Tcp / _Udp (flags omitted)
    src_range: PortRange = None
    dst_range: PortRange = None


@dataclass
class AclRule:
    action: int = ACL_DENY
    has_ip_rule: bool = True
    has_ip: bool = True
    has_icmp: bool = False
    has_macip: bool = False
    src_network: str = ""
    dst_network: str = ""
    tcp: L4Section = None
    udp: L4Section = None


@dataclass
class ACL:
    name: str
    rules: list = field(default_factory=list)
    ingress: list = field(default_factory=list)      # Interfaces.Ingress
    egress: list = field(default_factory=list)       # Interfaces.Egress

    def clone(self) -> "ACL":
        return ACL(self.name, list(self.rules), list(self.ingress), list(self.egress))


ACL_NAME_PREFIX = "contiv-policy-"
REFLECTIVE_ACL_NAME = "REFLECTION"


@dataclass
class NodeIfaces:
    """The ipv4net / contivconf getters the renderer and engine depend on
    (mock/ipv4net/ipv4net_mock.go:70-110, acl_renderer_test.go:58-83)."""
    pod_if: dict = field(default_factory=dict)       # podID -> ifName
    host_interconnect: str = ""
    main_if: str = ""
    other_ifs: list = field(default_factory=list)
    vxlan_bvi: str = ""

    def get_if_name(self, pod):
        n = self.pod_if.get(pod)
        return (n, True) if n is not None else ("", False)


def render_acl(table: ContivRuleTable, reflective: bool, ifaces: NodeIfaces, pod_if_cache: dict) -> ACL:
    """acl_renderer.go:295-362."""
    name = ACL_NAME_PREFIX + (REFLECTIVE_ACL_NAME if reflective else table.get_id())
    acl = ACL(name)
    ing, eg = render_interfaces(table.pods, reflective, ifaces, pod_if_cache)
    acl.ingress, acl.egress = ing, eg
    for r in table.rules:
        ar = AclRule()
        if r.action == ACTION_DENY:
            ar.action = ACL_DENY
        elif reflective:
            ar.action = ACL_REFLECT
        else:
            ar.action = ACL_PERMIT
        if not r.src.is_empty():
            ar.src_network = gonet.ipnet_string(r.src)
        if not r.dst.is_empty():
            ar.dst_network = gonet.ipnet_string(r.dst)
        if r.protocol in (TCP, UDP):
            sec = L4Section(PortRange(r.src_port, MAX_PORT if r.src_port == 0 else r.src_port),
                            PortRange(r.dst_port, MAX_PORT if r.dst_port == 0 else r.dst_port))
            if r.protocol == TCP:
                ar.tcp = sec
            else:
                ar.udp = sec
        acl.rules.append(ar)
    table.private = acl
    return acl


def render_interfaces(pods, ingress: bool, ifaces: NodeIfaces, pod_if_cache: dict):
    """acl_renderer.go:366-390."""
    ing, eg = [], []
    for pod in sorted(pods):
        name = pod_if_cache.get(pod)
        if name is None:
            name, found = ifaces.get_if_name(pod)
            if not found:
                continue
        pod_if_cache[pod] = name
        (ing if ingress else eg).append(name)
    return ing, eg


def node_output_interfaces(ifaces: NodeIfaces):
    """acl_renderer.go:277-292."""
    out = [ifaces.host_interconnect]
    if ifaces.main_if:
        out.append(ifaces.main_if)
    out.extend(ifaces.other_ifs)
    if ifaces.vxlan_bvi:
        out.append(ifaces.vxlan_bvi)
    return out


class AclRenderer:
    """acl_renderer.go:51-250 (EgressOrientation cache). ``apply`` receives
    (resync: bool, ops: dict key->ACL|None) exactly once per committed controller txn."""

    def __init__(self, ifaces: NodeIfaces, apply):
        self.ifaces = ifaces
        self.apply = apply
        self.cache = RendererCache(EGRESS_ORIENTATION)
        self.pod_ifs: dict = {}

    def new_txn(self, resync: bool):
        return AclRendererTxn(self, resync)


class AclRendererTxn:
    def __init__(self, r: AclRenderer, resync: bool):
        self.r = r
        self.cache_txn = r.cache.new_txn()
        self.resync = resync

    def render(self, pod, pod_ip, ingress, egress, removed):
        self.cache_txn.update(pod, PodConfig(pod_ip, list(ingress), list(egress), removed))
        return self

    def _reflective(self) -> ACL:
        t = ContivRuleTable(LOCAL)
        t.rules = [allow_all()]
        t.slice_len = 1
        t.pods = self.cache_txn.get_isolated_pods()
        acl = render_acl(t, True, self.r.ifaces, self.r.pod_ifs)
        if self.cache_txn.get_global_table().num_rules > 0:
            acl.ingress = acl.ingress + node_output_interfaces(self.r.ifaces)
        return acl

    def commit(self):
        if self.resync:
            return self._commit_resync()
        r = self.r
        has_reflective = r.cache.get_global_table().num_rules != 0 or len(r.cache.get_isolated_pods()) > 0
        changes = self.cache_txn.get_changes()
        if not changes:
            self.cache_txn.commit()
            return None
        ops = {}
        global_table = None
        for ch in changes:
            if ch.table.type == GLOBAL:
                global_table = ch.table
                continue
            if len(ch.previous_pods) == 0:
                acl = render_acl(ch.table, False, r.ifaces, r.pod_ifs)
                ops[acl.name] = acl
            elif len(ch.table.pods) != 0:
                acl = ch.table.private.clone()
                acl.ingress, acl.egress = render_interfaces(ch.table.pods, False, r.ifaces, r.pod_ifs)
                ops[acl.name] = acl
            else:
                ops[ch.table.private.name] = None
        gt_added_or_deleted = False
        if global_table is not None:
            gacl = render_acl(global_table, False, r.ifaces, r.pod_ifs)
            if global_table.num_rules == 0:
                ops[gacl.name] = None
                gt_added_or_deleted = True
            else:
                gacl.egress = node_output_interfaces(r.ifaces)
                ops[gacl.name] = gacl
                if r.cache.get_global_table().num_rules == 0:
                    gt_added_or_deleted = True
        if gt_added_or_deleted or self.cache_txn.get_isolated_pods() != r.cache.get_isolated_pods():
            racl = self._reflective()
            if len(racl.ingress) == 0:
                if has_reflective:
                    ops[racl.name] = None
            else:
                ops[racl.name] = racl
        err = r.apply(False, ops)
        self.cache_txn.commit()
        return err

    def _commit_resync(self):
        r = self.r
        r.cache.flush()
        r.pod_ifs = {}
        ops = {}
        for ch in self.cache_txn.get_changes():
            acl = render_acl(ch.table, False, r.ifaces, r.pod_ifs)
            if ch.table.type == GLOBAL:
                acl.egress = node_output_interfaces(r.ifaces)
            ops[acl.name] = acl
        racl = self._reflective()
        if len(racl.ingress) != 0:
            ops[racl.name] = racl
        err = r.apply(True, ops)
        self.cache_txn.commit()
        return err
