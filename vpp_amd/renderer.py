"""Python face of the engine, mirroring the reference's interfaces for this path.

Names follow the reference so parity tests read like its own tests:

* ``ContivRule``, ``ActionType``, ``ProtocolType``     renderer/api.go:65-176
* ``Renderer.NewTxn`` / ``Txn.Render`` / ``Txn.Commit``  renderer/api.go:33-61 (PolicyRendererAPI)
* ``Engine.RegisterPod`` / ``Connection*`` / ``GetNumOfACLs`` / ``GetInboundACL`` ...
                                                       mock/aclengine/aclengine_mock.go
* ``Engine.SetPodIfName`` / ``SetVxlanBVIIfName`` / ...  mock/ipv4net/ipv4net_mock.go:40-66

Everything below delegates to the C ABI (``_capi``); evalACL / testConnection run on the GPU.
"""
import ctypes as C
import ipaddress
import json

from . import _capi
from ._capi import lib

# renderer.ActionType / ProtocolType (api.go:140-176)
ActionDeny, ActionPermit = 0, 1
TCP, UDP, OTHER, ANY = 0, 1, 2, 3
# aclengine ConnectionAction / ACLAction (aclengine_mock.go:39-71)
ConnActionDenySyn, ConnActionDenySynAck, ConnActionAllow, ConnActionFailure = 0, 1, 2, 3
ACLActionDeny, ACLActionPermit, ACLActionReflect, ACLActionFailure = 0, 1, 2, 3
# cache.Orientation
IngressOrientation, EgressOrientation = 0, 1


class PolicyError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("%s (code %d)" % (msg, code))
        self.code = code


def _b(s):
    return s.encode() if isinstance(s, str) else s


class IPNet:
    """net.IPNet: ``IPNet()`` is the empty network (match all); ``IPNet("10.0.0.0/8")`` parses a
    CIDR (keeping the address as written, like a Go IPNet built by hand would)."""

    __slots__ = ("family", "prefix_len", "addr")

    def __init__(self, cidr=None):
        if not cidr:
            self.family, self.prefix_len, self.addr = 0, 0, b""
            return
        ip, _, plen = cidr.partition("/")
        a = ipaddress.ip_address(ip)
        self.family = a.version
        self.addr = a.packed
        self.prefix_len = int(plen) if plen else (32 if a.version == 4 else 128)

    @classmethod
    def host(cls, ip):
        """utils.GetOneHostSubnet (utils.go:271-291)."""
        n = cls(ip)
        n.prefix_len = 32 if n.family == 4 else 128
        return n

    def c(self):
        v = _capi.pg_ipnet()
        v.family = self.family
        v.prefix_len = self.prefix_len
        for i, x in enumerate(self.addr):
            v.addr[i] = x
        return v

    def __repr__(self):
        if not self.family:
            return "ANY"
        return "%s/%d" % (ipaddress.ip_address(self.addr), self.prefix_len)


class ContivRule:
    """renderer.ContivRule (api.go:65-77)."""

    __slots__ = ("Action", "SrcNetwork", "DestNetwork", "Protocol", "SrcPort", "DestPort")

    def __init__(self, Action=ActionPermit, SrcNetwork=None, DestNetwork=None, Protocol=ANY, SrcPort=0, DestPort=0):
        self.Action = Action
        self.SrcNetwork = SrcNetwork if isinstance(SrcNetwork, IPNet) else IPNet(SrcNetwork)
        self.DestNetwork = DestNetwork if isinstance(DestNetwork, IPNet) else IPNet(DestNetwork)
        self.Protocol = Protocol
        self.SrcPort = SrcPort
        self.DestPort = DestPort

    def c(self):
        r = _capi.pg_contiv_rule()
        r.action, r.protocol, r.src_port, r.dst_port = self.Action, self.Protocol, self.SrcPort, self.DestPort
        r.src = self.SrcNetwork.c()
        r.dst = self.DestNetwork.c()
        return r

    def __repr__(self):
        return "Rule <%s %s[%d:%d] -> %s[%d:%d]>" % (
            "PERMIT" if self.Action else "DENY", self.SrcNetwork, self.Protocol, self.SrcPort, self.DestNetwork,
            self.Protocol, self.DestPort)


def _rules_array(rules):
    arr = (_capi.pg_contiv_rule * max(1, len(rules)))()
    for i, r in enumerate(rules):
        arr[i] = r.c()
    return arr, len(rules)


def _pod(pod):
    """podmodel.ID as "namespace/name" or (namespace, name)."""
    if isinstance(pod, str):
        ns, _, name = pod.partition("/")
        return ns, name
    return pod


class Engine:
    """The device ACL engine (one GPU): MockACLEngine's API + ipv4net/contivconf setters."""

    def __init__(self, device=0):
        self.h = lib.pg_create(device)
        if not self.h:
            raise PolicyError(_capi.PG_ENOMEM, "pg_create failed")
        self._keep = []
        self.registered_pods = {}  # "ns/name" -> (IP, anotherNode) as given to RegisterPod

    def close(self):
        if self.h:
            lib.pg_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _ck(self, rc):
        if rc < 0:
            raise PolicyError(rc, lib.pg_last_error(self.h).decode())
        return rc

    # tuning knobs of this context (pg_ctx_set_tuning; include/policygpu.h lists the keys)
    def set_tuning(self, key, value):
        self._ck(lib.pg_ctx_set_tuning(self.h, _b(key), int(value)))

    def get_tuning(self, key):
        v = C.c_int()
        self._ck(lib.pg_ctx_get_tuning(self.h, _b(key), C.byref(v)))
        return v.value

    def tuning(self, **kw):
        """context manager: the given knobs set for the block, restored afterwards"""
        import contextlib

        @contextlib.contextmanager
        def cm():
            old = {k: self.get_tuning(k) for k in kw}
            try:
                for k, v in kw.items():
                    self.set_tuning(k, v)
                yield self
            finally:
                for k, v in old.items():
                    self.set_tuning(k, v)
        return cm()

    @property
    def device(self):
        return self._ck(lib.pg_ctx_device(self.h))

    # ipv4net / contivconf setters
    def SetPodIfName(self, pod, if_name):
        ns, name = _pod(pod)
        self._ck(lib.pg_set_pod_if_name(self.h, _b(ns), _b(name), _b(if_name)))

    def SetHostInterconnectIfName(self, n):
        self._ck(lib.pg_set_host_interconnect_if_name(self.h, _b(n)))

    def SetMainInterfaceName(self, n):
        self._ck(lib.pg_set_main_interface_name(self.h, _b(n)))

    def SetOtherVPPInterfaces(self, names):
        arr = (C.c_char_p * max(1, len(names)))(*[_b(x) for x in names])
        self._ck(lib.pg_set_other_vpp_interfaces(self.h, arr, len(names)))

    def SetVxlanBVIIfName(self, n):
        self._ck(lib.pg_set_vxlan_bvi_if_name(self.h, _b(n)))

    def RegisterPod(self, pod, ip, another_node):
        ns, name = _pod(pod)
        self._ck(lib.pg_register_pod(self.h, _b(ns), _b(name), _b(ip), int(another_node)))
        self.registered_pods["%s/%s" % (ns, name)] = (ip, bool(another_node))

    # ACL install / introspection
    def ApplyTxn(self, resync, ops):
        """ops: list of (key, acl dict or None); acl dicts as returned by GetACLByName."""
        keep = []
        arr = (_capi.pg_acl_op * max(1, len(ops)))()
        for i, (key, acl) in enumerate(ops):
            arr[i].key = _b(key)
            if acl is not None:
                a = _acl_struct(acl, keep)
                keep.append(a)
                arr[i].value = C.pointer(a)
        return self._ck(lib.pg_apply_txn(self.h, int(resync), arr, len(ops)))

    def GetNumOfACLs(self):
        return self._ck(lib.pg_num_acls(self.h))

    def GetNumOfACLChanges(self):
        return self._ck(lib.pg_num_acl_changes(self.h))

    def NumCommittedTxns(self):
        return self._ck(lib.pg_num_committed_txns(self.h))

    def GetACLByName(self, name):
        n = lib.pg_acl_json(self.h, _b(name), None, 0)
        if n == _capi.PG_ENOENT:
            return None
        self._ck(n)
        buf = C.create_string_buffer(n)
        self._ck(lib.pg_acl_json(self.h, _b(name), buf, n))
        return json.loads(buf.value.decode())

    def ACLNames(self):
        n = self._ck(lib.pg_acl_names_json(self.h, None, 0))
        buf = C.create_string_buffer(n)
        self._ck(lib.pg_acl_names_json(self.h, buf, n))
        return json.loads(buf.value.decode())

    def _if_acls(self, if_name):
        a, b = C.create_string_buffer(512), C.create_string_buffer(512)
        self._ck(lib.pg_interface_acls(self.h, _b(if_name), a, 512, b, 512))
        return a.value.decode(), b.value.decode()

    def GetInboundACL(self, if_name):
        n = self._if_acls(if_name)[0]
        return self.GetACLByName(n) if n else None

    def GetOutboundACL(self, if_name):
        n = self._if_acls(if_name)[1]
        return self.GetACLByName(n) if n else None

    # device tables
    def sync(self):
        self._ck(lib.pg_sync_tables(self.h))

    def table_id(self, acl_name):
        return self._ck(lib.pg_table_id(self.h, _b(acl_name)))

    def num_tables(self):
        return self._ck(lib.pg_num_tables(self.h))

    def num_counter_slots(self):
        return self._ck(lib.pg_num_counter_slots(self.h))

    def slot_info(self, slot):
        t, r = C.c_int32(), C.c_int32()
        self._ck(lib.pg_slot_info(self.h, slot, C.byref(t), C.byref(r)))
        return t.value, r.value

    def table_info(self, tid):
        b, n, d = C.c_uint32(), C.c_uint32(), C.c_uint32()
        self._ck(lib.pg_table_info(self.h, tid, C.byref(b), C.byref(n), C.byref(d)))
        return b.value, n.value, d.value

    def table_stats(self, tid):
        v = [C.c_uint32() for _ in range(4)]
        self._ck(lib.pg_table_stats(self.h, tid, *[C.byref(x) for x in v]))
        f, nbytes, nsc, nkc = (x.value for x in v)
        mode = "linear" if f & 8 else ("fd" if f & 32 else ("pair" if f & 16 else ("candi" if f & 128 else (
            "cand" if f & 4 else ("cross+lists" if f & 2 else "cross")))))
        return {"structure": mode, "blob_bytes": nbytes, "src_classes": nsc, "key_classes": nkc,
                "dst_free": bool(f & 64)}

    def debug_walk(self, acl_name, src, dst, dport, proto):
        """TESTS ONLY: host walk of the ACL's compiled blob (see pg_debug_walk_blob)."""
        import numpy as np
        n = len(src)
        a = [np.ascontiguousarray(x, dt) for x, dt in ((src, np.uint32), (dst, np.uint32), (dport, np.uint16),
                                                       (proto, np.uint8))]
        out = np.empty(n, np.uint32)
        p = lambda x: x.ctypes.data_as(C.c_void_p)
        self._ck(lib.pg_debug_walk_blob(self.h, _b(acl_name), p(a[0]), p(a[1]), p(a[2]), p(a[3]), n, p(out)))
        return out

    def debug_classify_host(self, mode, table_id, src, dst, sport, dport, proto, counters=False, node=True,
                            pred=True, common=True):
        """TESTS ONLY: pg_classify's per-tuple code run on the host (pg_debug_classify_host).
        ``common``: the node image's common-row section (when it was built).
        -> verdict words (u32), and the u64 hit counters when ``counters``."""
        import numpy as np
        n = len(src)
        a = [np.ascontiguousarray(x, dt) for x, dt in ((src, np.uint32), (dst, np.uint32), (sport, np.uint16),
                                                       (dport, np.uint16), (proto, np.uint8))]
        p = lambda x: x.ctypes.data_as(C.c_void_p)
        t = _capi.pg_tuple_soa(p(a[0]), p(a[1]), p(a[2]), p(a[3]), p(a[4]))
        out = np.empty(n, np.uint32)
        cnt = np.zeros(self.num_counter_slots(), np.uint64) if counters else None
        self._ck(lib.pg_debug_classify_host(self.h, mode, table_id, C.byref(t), n, p(out),
                                            p(cnt) if counters else None,
                                            int(node) | (2 if pred else 0) | (4 if common else 0)))
        return (out, cnt) if counters else out

    def debug_walk_stats(self, table_id, src, dst, dport, proto):
        """MEASUREMENT: per tuple, the loads a SINGLE launch on table_id makes of the table's
        structure (pg_debug_walk_stats) -> (lds_reads u32[n], mem_reads u32[n], launch STAGE)"""
        import numpy as np
        n = len(src)
        a = [np.ascontiguousarray(x, dt) for x, dt in ((src, np.uint32), (dst, np.uint32), (dport, np.uint16),
                                                       (proto, np.uint8))]
        p = lambda x: x.ctypes.data_as(C.c_void_p)
        t = _capi.pg_tuple_soa(p(a[0]), p(a[1]), None, p(a[2]), p(a[3]))
        nl, nm, st = np.zeros(n, np.uint32), np.zeros(n, np.uint32), C.c_int()
        self._ck(lib.pg_debug_walk_stats(self.h, table_id, C.byref(t), n, nl.ctypes.data_as(C.POINTER(C.c_uint32)),
                                         nm.ctypes.data_as(C.POINTER(C.c_uint32)), C.byref(st)))
        return nl, nm, st.value

    def node_stats(self):
        """node classifier size {ip_classes, key_classes, image_bytes, cross_bytes}, or None."""
        a, b = C.c_uint32(), C.c_uint32()
        c, d = C.c_uint64(), C.c_uint64()
        rc = lib.pg_node_stats(self.h, C.byref(a), C.byref(b), C.byref(c), C.byref(d))
        if rc == -2:  # PG_ENOENT
            return None
        self._ck(rc)
        st = {"ip_classes": a.value, "key_classes": b.value, "image_bytes": c.value, "cross_bytes": d.value}
        base, common, pairs = C.c_uint64(), C.c_uint64(), C.c_uint64()
        self._ck(lib.pg_node_common_stats(self.h, C.byref(base), C.byref(common), C.byref(pairs)))
        st.update(base_image_bytes=base.value, common_row_pairs=common.value, table_ipclass_pairs=pairs.value)
        rb, inimg = C.c_uint64(), C.c_int()
        self._ck(lib.pg_node_list_stats(self.h, C.byref(rb), C.byref(inimg)))
        st.update(list_record_bytes=rb.value, list_records_in_image=bool(inimg.value))
        lt = C.c_uint64()
        self._ck(lib.pg_node_list_table_stats(self.h, C.byref(lt)))
        st.update(list_table_bytes=lt.value)
        u = self._ck(lib.pg_node_uniform(self.h))
        st.update(uniform=bool(u), wide_records=u == 2)
        return st

    def slot_of_rule(self, tid, idx):
        """counter slot of rule ``idx`` of table ``tid`` (idx -1: the table's default deny)."""
        base, n, dflt = self.table_info(tid)
        return base + idx if idx >= 0 else dflt

    # Connection* (aclengine_mock.go:273-420), testConnection evaluated on the GPU
    def connections(self, queries):
        """queries: list of (kind, a, b, proto, sport, dport) with kind in
        {"PodToPod", "PodToInternet", "InternetToPod"}; returns (ConnActions, slots)."""
        n = len(queries)
        arr = (_capi.pg_conn_query * max(1, n))()
        for i, (kind, a, b, proto, sport, dport) in enumerate(queries):
            q = arr[i]
            q.kind = {"PodToPod": 0, "PodToInternet": 1, "InternetToPod": 2}[kind]
            if q.kind == 0:
                (q.src_namespace, q.src_name), (q.dst_namespace, q.dst_name) = map(
                    lambda p: tuple(map(_b, _pod(p))), (a, b))
            elif q.kind == 1:
                q.src_namespace, q.src_name = map(_b, _pod(a))
                q.dst_ip = _b(b)
            else:
                q.src_ip = _b(a)
                q.dst_namespace, q.dst_name = map(_b, _pod(b))
            q.protocol, q.src_port, q.dst_port = proto, sport, dport
        out = (C.c_int32 * max(1, n))()
        slots = (C.c_uint32 * max(1, n))()
        self._ck(lib.pg_connections(self.h, arr, n, out, slots))
        return list(out[:n]), list(slots[:n])

    def ConnectionPodToPod(self, src_pod, dst_pod, protocol, src_port, dst_port):
        return self.connections([("PodToPod", src_pod, dst_pod, protocol, src_port, dst_port)])[0][0]

    def ConnectionPodToInternet(self, src_pod, dst_ip, protocol, src_port, dst_port):
        return self.connections([("PodToInternet", src_pod, dst_ip, protocol, src_port, dst_port)])[0][0]

    def ConnectionInternetToPod(self, src_ip, dst_pod, protocol, src_port, dst_port):
        return self.connections([("InternetToPod", src_ip, dst_pod, protocol, src_port, dst_port)])[0][0]


def _acl_struct(acl, keep):
    rules = (_capi.pg_acl_rule * max(1, len(acl["rules"])))()
    for i, r in enumerate(acl["rules"]):
        x = rules[i]
        x.action = r["action"]
        x.has_macip_rule = int(r.get("macip", False))
        x.has_ip_rule = int(r.get("ip_rule", True))
        x.has_ip = int(r.get("ip", True))
        x.has_icmp = int(r.get("icmp", False))
        x.src_network = _b(r.get("src", ""))
        x.dst_network = _b(r.get("dst", ""))
        for name in ("tcp", "udp"):
            sec = r.get(name)
            if sec:
                l4 = getattr(x, name)
                l4.present = 1
                if sec.get("src") is not None:
                    l4.has_src_range = 1
                    l4.src_range.lower_port, l4.src_range.upper_port = sec["src"]
                if sec.get("dst") is not None:
                    l4.has_dst_range = 1
                    l4.dst_range.lower_port, l4.dst_range.upper_port = sec["dst"]
    ing = (C.c_char_p * max(1, len(acl["ingress"])))(*[_b(s) for s in acl["ingress"]])
    eg = (C.c_char_p * max(1, len(acl["egress"])))(*[_b(s) for s in acl["egress"]])
    keep += [rules, ing, eg]
    a = _capi.pg_acl()
    a.name = _b(acl["name"])
    a.rules = C.cast(rules, C.POINTER(_capi.pg_acl_rule))
    a.n_rules = len(acl["rules"])
    a.ingress = C.cast(ing, C.POINTER(C.c_char_p))
    a.n_ingress = len(acl["ingress"])
    a.egress = C.cast(eg, C.POINTER(C.c_char_p))
    a.n_egress = len(acl["egress"])
    return a


class Txn:
    """renderer.Txn (api.go:44-61)."""

    def __init__(self, engine, h):
        self.engine = engine
        self.h = h

    def Render(self, pod, podIP, ingress, egress, removed):
        ns, name = _pod(pod)
        ip = podIP.c() if podIP is not None else None
        ia, ni = _rules_array(ingress)
        ea, ne = _rules_array(egress)
        self.engine._ck(lib.pg_txn_render(self.h, _b(ns), _b(name), C.byref(ip) if ip is not None else None,
                                          ia, ni, ea, ne, int(removed)))
        return self

    def Commit(self):
        h, self.h = self.h, None
        rc = lib.pg_txn_commit(h)
        if rc < 0:
            return PolicyError(rc, lib.pg_last_error(self.engine.h).decode())
        return None

    def __del__(self):
        if getattr(self, "h", None) and lib is not None:
            lib.pg_txn_free(self.h)


class Renderer:
    """The GPU policy renderer (PolicyRendererAPI), EgressOrientation like the ACL renderer."""

    def __init__(self, engine, orientation=EgressOrientation):
        self.engine = engine
        self.h = lib.pg_renderer_new(engine.h, orientation)

    def NewTxn(self, resync):
        return Txn(self.engine, lib.pg_renderer_new_txn(self.h, int(resync)))

    def __del__(self):
        # at interpreter shutdown module globals may already be gone: skip, the process exits
        if getattr(self, "h", None) and lib is not None:
            lib.pg_renderer_free(self.h)
            self.h = None
