"""Mock ACL engine restated on the CPU (TEST INFRASTRUCTURE ONLY).

Follows /root/reference/mock/aclengine/aclengine_mock.go:
  * ConnectionAction / ACLAction enums            :39-71
  * ApplyTxn                                      :151-228
  * GetNumOfACLs / Get{In,Out}boundACL / GetACLByName / GetNumOfACLChanges :238-269
  * ConnectionPodToPod / PodToInternet / InternetToPod :273-420
  * testConnection                                :424-501
  * evalACL (hot loop, with the matched rule index surfaced) :503-652
  * ACLConfig GetACLs / DelACL / PutACL           :655-712
"""
from __future__ import annotations

from dataclasses import dataclass

from . import gonet
from .policy import (ACL, ACL_DENY, ACL_PERMIT, ACL_REFLECT, NodeIfaces, TCP, UDP, OTHER)

CONN_DENY_SYN, CONN_DENY_SYN_ACK, CONN_ALLOW, CONN_FAILURE = 0, 1, 2, 3
ACT_DENY, ACT_PERMIT, ACT_REFLECT, ACT_FAILURE = 0, 1, 2, 3
MAX_PORT_NUM = 0xFFFF
NO_RULE = -1          # evalACL returned without matching a rule (nil ACL / default deny)

CONN_NAMES = {CONN_DENY_SYN: "ConnActionDenySyn", CONN_DENY_SYN_ACK: "ConnActionDenySynAck",
              CONN_ALLOW: "ConnActionAllow", CONN_FAILURE: "ConnActionFailure"}


class ACLConfig:
    def __init__(self):
        self.by_name: dict = {}
        self.by_if: dict = {}       # ifName -> [inbound, outbound]
        self.changes = 0

    def get_acls(self, if_name):
        return self.by_if.get(if_name, [None, None])

    def del_acl(self, name):
        if name not in self.by_name:
            return "cannot find ACL: %s" % name
        del self.by_name[name]
        for cfg in self.by_if.values():
            if cfg[0] is not None and cfg[0].name == name:
                cfg[0] = None
            if cfg[1] is not None and cfg[1].name == name:
                cfg[1] = None
        self.changes += 1
        return None

    def put_acl(self, acl: ACL):
        if acl is None:
            return "ACL is nil"
        if len(acl.ingress) == 0 and len(acl.egress) == 0:
            return "ACL with empty interfaces"
        if acl.name in self.by_name:
            self.del_acl(acl.name)
            self.changes -= 1
        self.by_name[acl.name] = acl
        for ifn in acl.ingress:
            self.by_if.setdefault(ifn, [None, None])[0] = acl
        for ifn in acl.egress:
            self.by_if.setdefault(ifn, [None, None])[1] = acl
        self.changes += 1
        return None


@dataclass
class PodCfg:
    ip: bytes
    another_node: bool


def eval_acl(acl, src_ip: bytes, dst_ip: bytes, protocol: int, dst_port: int):
    """aclengine_mock.go:503-652 -> (ACLAction, matched rule index or NO_RULE)."""
    if acl is None:
        return ACT_PERMIT, NO_RULE
    for idx, rule in enumerate(acl.rules):
        if rule.has_macip:
            return ACT_FAILURE, idx
        if not rule.has_ip_rule:
            return ACT_FAILURE, idx
        if rule.has_icmp or not rule.has_ip:
            return ACT_FAILURE, idx
        if rule.udp is not None and rule.tcp is not None:
            return ACT_FAILURE, idx
        if rule.src_network != "":
            r = gonet.parse_cidr(rule.src_network)
            if r is None:
                return ACT_FAILURE, idx
            if not gonet.contains(r[1], src_ip):
                continue
        if rule.dst_network != "":
            r = gonet.parse_cidr(rule.dst_network)
            if r is None:
                return ACT_FAILURE, idx
            if not gonet.contains(r[1], dst_ip):
                continue
        if protocol in (TCP, UDP):
            mine, other = (rule.tcp, rule.udp) if protocol == TCP else (rule.udp, rule.tcp)
            if other is not None:
                continue
            if mine is not None:
                sr = mine.src_range
                if sr is None:
                    return ACT_FAILURE, idx
                if sr.lower != 0 or sr.upper != MAX_PORT_NUM:
                    return ACT_FAILURE, idx
                dr = mine.dst_range
                if dr is None:
                    return ACT_FAILURE, idx
                if dst_port < (dr.lower & 0xFFFF) or dst_port > (dr.upper & 0xFFFF):
                    continue
        elif protocol == OTHER:
            if rule.tcp is not None or rule.udp is not None:
                continue
        if rule.action == ACL_DENY:
            return ACT_DENY, idx
        if rule.action == ACL_PERMIT:
            return ACT_PERMIT, idx
        if rule.action == ACL_REFLECT:
            return ACT_REFLECT, idx
        return ACT_FAILURE, idx
    return ACT_DENY, NO_RULE


class MockACLEngine:
    def __init__(self, ifaces: NodeIfaces):
        self.ifaces = ifaces
        self.pods: dict = {}
        self.cfg = ACLConfig()
        self.committed_txns = 0

    # --- install
    def register_pod(self, pod, ip: str, another_node: bool):
        self.pods[pod] = PodCfg(gonet.parse_ip(ip), another_node)

    def clear_acls(self):
        ch = self.cfg.changes
        self.cfg = ACLConfig()
        self.cfg.changes = ch

    def apply_txn(self, resync: bool, ops: dict):
        """ApplyTxn for one controller txn (aclengine_mock.go:151-228). Map iteration order is
        random in Go; keys are applied in sorted order here."""
        self.committed_txns += 1
        if resync:
            self.clear_acls()
            for _, acl in sorted(ops.items()):
                err = self.cfg.put_acl(acl)
                if err:
                    return err
            return None
        for name, acl in sorted(ops.items()):
            err = self.cfg.put_acl(acl) if acl is not None else self.cfg.del_acl(name)
            if err:
                return err
        return None

    def num_acls(self):
        return len(self.cfg.by_name)

    def num_acl_changes(self):
        return self.cfg.changes

    def inbound_acl(self, if_name):
        return self.cfg.get_acls(if_name)[0]

    def outbound_acl(self, if_name):
        return self.cfg.get_acls(if_name)[1]

    def acl_by_name(self, name):
        return self.cfg.by_name.get(name)

    # --- connection simulation
    def _node_if(self):
        n = self.ifaces.vxlan_bvi
        if n == "":
            n = self.ifaces.main_if
        return n

    def connection_pod_to_pod(self, src_pod, dst_pod, proto, sport, dport):
        s, d = self.pods.get(src_pod), self.pods.get(dst_pod)
        if s is None or d is None:
            return CONN_FAILURE
        if s.another_node:
            sif = self._node_if()
            if sif == "":
                return CONN_FAILURE
        else:
            sif, ok = self.ifaces.get_if_name(src_pod)
            if not ok:
                return CONN_FAILURE
        if d.another_node:
            dif = self._node_if()
            if dif == "":
                return CONN_FAILURE
        else:
            dif, ok = self.ifaces.get_if_name(dst_pod)
            if not ok:
                return CONN_FAILURE
        return self.test_connection(sif, s.ip, dif, d.ip, proto, sport, dport)

    def connection_pod_to_internet(self, src_pod, dst_ip: str, proto, sport, dport):
        s = self.pods.get(src_pod)
        if s is None or s.another_node:
            return CONN_FAILURE
        sif, ok = self.ifaces.get_if_name(src_pod)
        if not ok:
            return CONN_FAILURE
        dif = self._node_if()
        if dif == "":
            return CONN_FAILURE
        ip = gonet.parse_ip(dst_ip)
        if ip is None:
            return CONN_FAILURE
        return self.test_connection(sif, s.ip, dif, ip, proto, sport, dport)

    def connection_internet_to_pod(self, src_ip: str, dst_pod, proto, sport, dport):
        d = self.pods.get(dst_pod)
        if d is None or d.another_node:
            return CONN_FAILURE
        sif = self._node_if()
        if sif == "":
            return CONN_FAILURE
        ip = gonet.parse_ip(src_ip)
        if ip is None:
            return CONN_FAILURE
        dif, ok = self.ifaces.get_if_name(dst_pod)
        if not ok:
            return CONN_FAILURE
        return self.test_connection(sif, ip, dif, d.ip, proto, sport, dport)

    def test_connection(self, src_if, src_ip, dst_if, dst_ip, proto, sport, dport, trace=None):
        """aclengine_mock.go:424-501. ``trace`` (list) receives (acl, action, idx) per evaluation."""
        src_refl = dst_refl = False
        s_in, s_out = self.cfg.get_acls(src_if)
        d_in, d_out = self.cfg.get_acls(dst_if)

        def ev(acl, a, b, port):
            act, idx = eval_acl(acl, a, b, proto, port)
            if trace is not None:
                trace.append((acl, act, idx))
            return act

        a = ev(s_in, src_ip, dst_ip, dport)
        if a == ACT_FAILURE:
            return CONN_FAILURE
        if a == ACT_DENY:
            return CONN_DENY_SYN
        if a == ACT_REFLECT:
            src_refl = True
            if src_if == dst_if:
                dst_refl = True
        if not dst_refl:
            a = ev(d_out, src_ip, dst_ip, dport)
            if a == ACT_FAILURE:
                return CONN_FAILURE
            if a == ACT_DENY:
                return CONN_DENY_SYN
            if a == ACT_REFLECT:
                dst_refl = True
                if src_if == dst_if:
                    src_refl = True
        if not dst_refl:
            a = ev(d_in, dst_ip, src_ip, sport)
            if a == ACT_FAILURE:
                return CONN_FAILURE
            if a == ACT_DENY:
                return CONN_DENY_SYN_ACK
        if not src_refl:
            a = ev(s_out, dst_ip, src_ip, sport)
            if a == ACT_FAILURE:
                return CONN_FAILURE
            if a == ACT_DENY:
                return CONN_DENY_SYN_ACK
        return CONN_ALLOW
