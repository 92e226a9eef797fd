"""Python mirror of the K8s policy cache (plugins/policy/cache) and the policy processor
(plugins/policy/processor), keeping the reference's names so the parity tests read like
cache_test.go. Everything delegates to the C ABI (vpp_amd/csrc/k8s.cpp, processor.cpp).

KSR objects are plain dicts with the Go field names of plugins/ksr/model (pod.Pod,
namespace.Namespace, policy.Policy), e.g.

    {"Name": "pod1", "Namespace": "ns1", "Label": [{"Key": "role", "Value": "db"}],
     "IpAddress": "10.1.1.3", "Container": [{"Name": "c", "Port": [{"Name": "http", "ContainerPort": 80}]}]}

and cross the boundary in their protobuf wire form (``encode_pod`` / ``encode_namespace`` /
``encode_policy``: proto3, field numbers of the .proto files), as a Go caller would pass
``proto.Marshal(obj)``.

    cache = PolicyCache()
    proc = PolicyProcessor(cache, configurator, "10.1.1.0/24")   # IPAM.PodSubnetThisNode()
    cache.Resync(pods=[...], namespaces=[...], policies=[...])     # -> processor -> configurator
    cache.Update(POD, old_pod, new_pod)                            # data_change.go event
"""
import ctypes as C

from . import _capi
from . import renderer as R
from ._capi import lib

POD, NAMESPACE, POLICY = 0, 1, 2
# policy.Policy_LabelSelector_LabelExpression_Operator
IN, NOT_IN, EXISTS, DOES_NOT_EXIST = 0, 1, 2, 3
# policy.Policy_PolicyType
DEFAULT, INGRESS, EGRESS, INGRESS_AND_EGRESS = 0, 1, 2, 3

Q_PODS_BY_LABEL_SELECTOR_INSIDE_NS, Q_PODS_BY_NS_LABEL_SELECTOR, Q_PODS_BY_NAMESPACE, Q_ALL_PODS = 0, 1, 2, 3
Q_POLICIES_BY_POD, Q_ALL_POLICIES, Q_ALL_NAMESPACES = 4, 5, 6
Q_MATCH_LABEL_PODS_INSIDE_NS, Q_PODS_BY_NS_LABELS, Q_MATCH_EXPRESSION_PODS_INSIDE_NS, Q_PODS_BY_NS_EXPRESSIONS = 7, 8, 9, 10
Q_IDX_POD_LABEL, Q_IDX_POD_KEY, Q_IDX_POD_NS_LABEL, Q_IDX_POD_NS_KEY = 11, 12, 13, 14
Q_IDX_NS_LABEL, Q_IDX_NS_KEY, Q_IDX_POLICY_LABEL, Q_IDX_POLICY_NS_LABEL = 15, 16, 17, 18


# ---- protobuf (proto3) encoding ---------------------------------------------------------------
def _varint(n):
    n &= (1 << 64) - 1
    out = bytearray()
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _tag(f, wt):
    return _varint(f << 3 | wt)


def _s(f, v):  # singular string: omitted when empty
    return _rs(f, v) if v else b""


def _rs(f, v):  # repeated string element: always written
    b = v.encode()
    return _tag(f, 2) + _varint(len(b)) + b


def _i(f, v):  # singular int / enum: omitted when zero
    return _tag(f, 0) + _varint(int(v)) if v else b""


def _m(f, b):  # embedded message (present, possibly empty)
    return _tag(f, 2) + _varint(len(b)) + b


def _labels(f, labels):
    return b"".join(_m(f, _s(1, l.get("Key", "")) + _s(2, l.get("Value", ""))) for l in labels or [])


def encode_selector(sel):
    """policy.Policy_LabelSelector"""
    out = _labels(1, sel.get("MatchLabel"))
    for x in sel.get("MatchExpression") or []:
        out += _m(2, _s(1, x.get("Key", "")) + _i(2, x.get("Operator", 0)) +
                  b"".join(_rs(3, v) for v in x.get("Value") or []))
    return out


def encode_pod(p):
    """pod.Pod"""
    out = _s(1, p.get("Name", "")) + _s(2, p.get("Namespace", "")) + _labels(3, p.get("Label"))
    out += _s(4, p.get("IpAddress", "")) + _s(5, p.get("HostIpAddress", ""))
    for c in p.get("Container") or []:
        ports = b"".join(_m(2, _s(1, q.get("Name", "")) + _i(2, q.get("HostPort", 0)) + _i(3, q.get("ContainerPort", 0))
                            + _i(4, q.get("Protocol", 0)) + _s(5, q.get("HostIpAddress", "")))
                         for q in c.get("Port") or [])
        out += _m(6, _s(1, c.get("Name", "")) + ports)
    return out


def encode_namespace(n):
    """namespace.Namespace"""
    return _s(1, n.get("Name", "")) + _labels(3, n.get("Label"))


def _encode_rule(r, peers_key):
    out = b""
    for p in r.get("Port") or []:
        pn = p.get("Port")
        body = b""
        if pn is not None:
            body += _m(1, _i(1, pn.get("Type", 0)) + _i(2, pn.get("Number", 0)) + _s(3, pn.get("Name", "")))
        out += _m(1, body + _i(3, p.get("Protocol", 0)))
    for peer in r.get(peers_key) or []:
        body = b""
        if peer.get("Pods") is not None:
            body += _m(1, encode_selector(peer["Pods"]))
        if peer.get("Namespaces") is not None:
            body += _m(2, encode_selector(peer["Namespaces"]))
        if peer.get("IpBlock") is not None:
            ib = peer["IpBlock"]
            body += _m(3, _s(1, ib.get("Cidr", "")) + b"".join(_rs(2, e) for e in ib.get("Except") or []))
        out += _m(2, body)
    return out


def encode_policy(p):
    """policy.Policy"""
    out = _s(1, p.get("Name", "")) + _s(2, p.get("Namespace", "")) + _labels(3, p.get("Label"))
    if p.get("Pods") is not None:
        out += _m(4, encode_selector(p["Pods"]))
    out += _i(5, p.get("PolicyType", 0))
    out += b"".join(_m(6, _encode_rule(r, "From")) for r in p.get("IngressRule") or [])
    out += b"".join(_m(7, _encode_rule(r, "To")) for r in p.get("EgressRule") or [])
    return out


ENCODE = {POD: encode_pod, NAMESPACE: encode_namespace, POLICY: encode_policy}


def _b(s):
    return s.encode() if isinstance(s, str) else s


def _names(fn):
    need = C.c_size_t()
    n = fn(None, 0, C.byref(need))
    if n < 0:
        raise R.PolicyError(n, "policy cache query")
    if n == 0:
        return []
    buf = C.create_string_buffer(need.value + 1)
    fn(buf, need.value + 1, C.byref(need))
    return buf.raw[:need.value].decode().split("\n")


class PolicyCache:
    """cache.PolicyCache (PolicyCacheAPI). Lookups of objects return (found, wire bytes | None);
    name lists come back sorted ("ns/name" IDs; namespace IDs are names)."""

    def __init__(self):
        self.h = lib.pg_policy_cache_new()

    # ConfigIndex.Register* / Unregister* (index only)
    def Register(self, kind, id_, obj):
        pb = None if obj is None else ENCODE[kind](obj)
        rc = lib.pg_policy_cache_register(self.h, kind, _b(id_), pb, len(pb or b""))
        if rc:
            raise R.PolicyError(rc, "Register")

    def Unregister(self, kind, id_):
        return lib.pg_policy_cache_unregister(self.h, kind, _b(id_)) == 1

    # data_change.go / data_resync.go
    def Update(self, kind, prev, new):
        a = None if prev is None else ENCODE[kind](prev)
        b = None if new is None else ENCODE[kind](new)
        rc = lib.pg_policy_cache_update(self.h, kind, a, len(a or b""), b, len(b or b""))
        return None if rc == 0 else R.PolicyError(rc, lib.pg_policy_cache_last_error(self.h).decode())

    def Resync(self, pods=(), namespaces=(), policies=()):
        objs = [(POD, encode_pod(p)) for p in pods] + [(NAMESPACE, encode_namespace(n)) for n in namespaces] + \
               [(POLICY, encode_policy(p)) for p in policies]
        n = len(objs)
        kinds = (C.c_int * max(1, n))(*[k for k, _ in objs])
        bufs = (C.c_char_p * max(1, n))(*[b for _, b in objs])
        lens = (C.c_size_t * max(1, n))(*[len(b) for _, b in objs])
        rc = lib.pg_policy_cache_resync(self.h, kinds, bufs, lens, n)
        return None if rc == 0 else R.PolicyError(rc, lib.pg_policy_cache_last_error(self.h).decode())

    def _lookup(self, kind, id_):
        need = C.c_size_t()
        f = lib.pg_policy_cache_lookup(self.h, kind, _b(id_), None, 0, C.byref(need))
        if f != 1:
            return False, None
        if need.value == C.c_size_t(-1).value:
            return True, None
        buf = C.create_string_buffer(max(1, need.value))
        lib.pg_policy_cache_lookup(self.h, kind, _b(id_), buf, need.value, C.byref(need))
        return True, buf.raw[:need.value]

    def LookupPod(self, pod):
        return self._lookup(POD, pod)

    def LookupPolicy(self, policy):
        return self._lookup(POLICY, policy)

    def LookupNamespace(self, ns):
        return self._lookup(NAMESPACE, ns)

    def query(self, q, arg=None, selector=None):
        sel = None if selector is None else encode_selector(selector)
        return _names(lambda out, cap, need: lib.pg_policy_cache_query(
            self.h, q, _b(arg) if arg is not None else None, sel, len(sel or b""), out, cap, need))

    def LookupPodsByLabelSelectorInsideNs(self, ns, sel):
        return self.query(Q_PODS_BY_LABEL_SELECTOR_INSIDE_NS, ns, sel)

    def LookupPodsByNsLabelSelector(self, sel):
        return self.query(Q_PODS_BY_NS_LABEL_SELECTOR, None, sel)

    def LookupPodsByNamespace(self, ns):
        return self.query(Q_PODS_BY_NAMESPACE, ns)

    def ListAllPods(self):
        return self.query(Q_ALL_PODS)

    def LookupPoliciesByPod(self, pod):
        return self.query(Q_POLICIES_BY_POD, pod)

    def ListAllPolicies(self):
        return self.query(Q_ALL_POLICIES)

    def ListAllNamespaces(self):
        return self.query(Q_ALL_NAMESPACES)

    # match_label.go / match_expression.go building blocks
    def getMatchLabelPodsInsideNs(self, ns, labels):
        return self.query(Q_MATCH_LABEL_PODS_INSIDE_NS, ns, {"MatchLabel": labels})

    def getPodsByNsLabelSelector(self, labels):
        return self.query(Q_PODS_BY_NS_LABELS, None, {"MatchLabel": labels})

    def getMatchExpressionPodsInsideNs(self, ns, exprs):
        return self.query(Q_MATCH_EXPRESSION_PODS_INSIDE_NS, ns, {"MatchExpression": exprs})

    def getPodsByNsMatchExpression(self, exprs):
        return self.query(Q_PODS_BY_NS_EXPRESSIONS, None, {"MatchExpression": exprs})

    def __del__(self):
        if getattr(self, "h", None) and lib is not None:
            lib.pg_policy_cache_free(self.h)
            self.h = None


class PolicyProcessor:
    """processor.PolicyProcessor watching `cache` and configuring `configurator`
    (configurator.PolicyConfigurator, which then looks pods up in the cache)."""

    def __init__(self, cache, configurator, pod_subnet_this_node):
        self.cache, self.configurator = cache, configurator  # keep both alive
        net = R.IPNet(pod_subnet_this_node).c()
        self.h = lib.pg_policy_processor_new(cache.h, configurator.h, C.byref(net))
        if not self.h:
            raise R.PolicyError(_capi.PG_EINVAL, "pg_policy_processor_new")

    def Process(self, resync, pods):
        arr = (C.c_char_p * max(1, len(pods)))(*[_b(p) for p in pods])
        rc = lib.pg_policy_processor_process(self.h, int(resync), arr, len(pods))
        return None if rc == 0 else R.PolicyError(rc, lib.pg_policy_processor_last_error(self.h).decode())

    def __del__(self):
        if getattr(self, "h", None) and lib is not None:
            lib.pg_policy_processor_free(self.h)
            self.h = None
