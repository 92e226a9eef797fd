"""VPPTCP renderer (Python face over the C ABI), mirroring the reference's names.

* ``Renderer(Deps(IPv4Net=..., GoVPPChan=..., GoVPPChanBufSize=...))``, ``Init``, ``NewTxn``,
  ``Txn.Render`` / ``Txn.Commit``      plugins/policy/renderer/vpptcp/vpptcp_renderer.go:33-188
* ``SessionRule`` + ``ExportSessionRules``   plugins/policy/renderer/vpptcp/rule/session_rule.go
* ``MockIPv4Net.SetPodAppNsIndex``     the test's IPv4Net (vpptcp_renderer_test.go:36-62)
* ``MockSessionRules`` (``Clear``, ``NewVPPChan``, ``GetErrCount``, ``GetReqCount``,
  ``LocalTable(ns)`` / ``GlobalTable()`` . ``NumOfRules`` / ``HasRule``)
                                       mock/sessionrules/sessionrules_mock.go:25-228

Example (the shape of vpptcp_renderer_test.go)::

    vpp = MockSessionRules(); ipv4net = MockIPv4Net(); ipv4net.SetPodAppNsIndex(pod1, 10)
    r = Renderer(Deps(IPv4Net=ipv4net, GoVPPChan=vpp.NewVPPChan())); r.Init()
    r.NewTxn(False).Render(pod1, GetOneHostSubnet("192.168.1.1"), ingress, egress, False).Commit()
    vpp.LocalTable(10).HasRule("", 0, "10.0.0.0/8", 22, "TCP", "DENY")
"""
import ctypes as C

from . import _capi
from . import renderer as R
from ._capi import lib

SessionRuleTagPrefix = "contiv/vpp-policy"
ScopeGlobal, ScopeLocal, ScopeBoth = 1, 2, 3
ActionDoNothing, ActionDeny, ActionAllow = 0xFFFFFFFF, 0xFFFFFFFE, 0xFFFFFFFD
ProtoTCP, ProtoUDP = 0, 1


def _b(s):
    return s.encode() if isinstance(s, str) else s


def GetOneHostSubnet(ip):
    return R.IPNet.host(ip)


class SessionRule:
    """rule.SessionRule (session_rule.go:73-86) as a plain record."""

    __slots__ = ("TransportProto", "IsIP4", "LclIP", "LclPlen", "RmtIP", "RmtPlen", "LclPort", "RmtPort",
                 "ActionIndex", "AppnsIndex", "Scope", "Tag")

    @classmethod
    def from_c(cls, c):
        s = cls()
        s.TransportProto, s.IsIP4 = c.transport_proto, c.is_ip4
        s.LclIP, s.LclPlen = bytes(c.lcl_ip), c.lcl_plen
        s.RmtIP, s.RmtPlen = bytes(c.rmt_ip), c.rmt_plen
        s.LclPort, s.RmtPort = c.lcl_port, c.rmt_port
        s.ActionIndex, s.AppnsIndex, s.Scope = c.action_index, c.appns_index, c.scope
        s.Tag = c.tag.rstrip(b"\0").decode(errors="replace") if isinstance(c.tag, bytes) else c.tag
        return s

    def key(self):
        return (self.TransportProto, self.IsIP4, self.LclIP, self.LclPlen, self.RmtIP, self.RmtPlen, self.LclPort,
                self.RmtPort, self.ActionIndex, self.AppnsIndex, self.Scope, self.Tag)

    def __eq__(self, o):
        return self.key() == o.key()

    def __repr__(self):
        return "SessionRule%r" % (self.key(),)


def _read_rules(fn, *args):
    n = fn(*args, None, 0)
    if n < 0:
        raise R.PolicyError(n, "session rules")
    arr = (_capi.pg_session_rule * max(1, n))()
    fn(*args, arr, n)
    return [SessionRule.from_c(arr[i]) for i in range(n)]


class MockIPv4Net:
    """The IPv4Net dependency: pod -> VPP application namespace index."""

    def __init__(self):
        self.h = lib.pg_appns_new()

    def SetPodAppNsIndex(self, pod, idx):
        ns, name = R._pod(pod)
        lib.pg_appns_set(self.h, _b(ns), _b(name), idx)

    def __del__(self):
        if getattr(self, "h", None) and lib is not None:
            lib.pg_appns_free(self.h)
            self.h = None


class _TableCheck:
    def __init__(self, vpp, scope, ns):
        self.vpp, self.scope, self.ns = vpp, scope, ns

    def NumOfRules(self):
        return lib.pg_session_rules_table(self.vpp.h, self.scope, self.ns, None, 0)

    def Rules(self):
        return _read_rules(lib.pg_session_rules_table, self.vpp.h, self.scope, self.ns)

    def HasRule(self, lclIP, lclPort, rmtIP, rmtPort, proto, action):
        return lib.pg_session_rules_has_rule(self.vpp.h, self.scope, self.ns, _b(lclIP), lclPort, _b(rmtIP),
                                             rmtPort, _b(proto), _b(action)) == 1


class MockSessionRules:
    """VPP's session-rule tables behind the binary API (mock/sessionrules)."""

    def __init__(self, tagPrefix=SessionRuleTagPrefix):
        self.h = lib.pg_session_rules_new(_b(tagPrefix))

    def Clear(self):
        lib.pg_session_rules_clear(self.h)

    def NewVPPChan(self):
        return self

    def _counts(self):
        req, err = C.c_int(), C.c_int()
        lib.pg_session_rules_counts(self.h, C.byref(req), C.byref(err))
        return req.value, err.value

    def GetReqCount(self):
        return self._counts()[0]

    def GetErrCount(self):
        return self._counts()[1]

    def LocalTable(self, nsIndex):
        return _TableCheck(self, ScopeLocal, nsIndex)

    def GlobalTable(self):
        return _TableCheck(self, ScopeGlobal, 0)

    def __del__(self):
        if getattr(self, "h", None) and lib is not None:
            lib.pg_session_rules_free(self.h)
            self.h = None


class Deps:
    def __init__(self, IPv4Net=None, GoVPPChan=None, GoVPPChanBufSize=0, Log=None):
        self.IPv4Net, self.GoVPPChan, self.GoVPPChanBufSize = IPv4Net, GoVPPChan, GoVPPChanBufSize


def ExportSessionRules(rules, podID, podIP, ipv4net):
    """session_rule.go:213-260 (podID None: the global table)."""
    arr, n = R._rules_array(rules)
    ns, name = R._pod(podID) if podID is not None else (None, None)
    ip = podIP.c() if podIP is not None else None
    return _read_rules(lib.pg_export_session_rules, ipv4net.h, arr, n, _b(ns), _b(name),
                       C.byref(ip) if ip is not None else None)


class Renderer:
    def __init__(self, deps):
        self.Deps = deps
        self.h = None

    def Init(self):
        d = self.Deps
        self.h = lib.pg_vpptcp_renderer_new(d.GoVPPChan.h, d.IPv4Net.h, d.GoVPPChanBufSize)
        if not self.h:
            raise R.PolicyError(_capi.PG_ENOMEM, "pg_vpptcp_renderer_new failed")
        return None

    def NewTxn(self, resync):
        return Txn(self, lib.pg_vpptcp_new_txn(self.h, int(resync)))

    def __del__(self):
        if getattr(self, "h", None) and lib is not None:
            lib.pg_vpptcp_renderer_free(self.h)
            self.h = None


class Txn:
    def __init__(self, r, h):
        self.r, self.h = r, h

    def Render(self, pod, podIP, ingress, egress, removed):
        ns, name = R._pod(pod)
        ia, ni = R._rules_array(ingress)
        ea, ne = R._rules_array(egress)
        ip = podIP.c() if podIP is not None else None
        rc = lib.pg_vpptcp_txn_render(self.h, _b(ns), _b(name), C.byref(ip) if ip is not None else None, ia, ni,
                                      ea, ne, int(removed))
        if rc != 0:
            raise R.PolicyError(rc, "Render")
        return self

    def Commit(self):
        h, self.h = self.h, None
        rc = lib.pg_vpptcp_txn_commit(h)
        if rc != 0:
            return R.PolicyError(rc, lib.pg_vpptcp_last_error(self.r.h).decode())
        return None

    def __del__(self):
        if getattr(self, "h", None) and lib is not None:
            lib.pg_vpptcp_txn_free(self.h)
            self.h = None


# --- session-rule lookup on the device (pg_session_table_install) --------------------------------
def InstallSessionTable(engine, vpp, scope, nsIndex, aclName):
    """VPP's session-rule table (ScopeLocal + nsIndex, or ScopeGlobal) of ``vpp`` installed in
    ``engine`` as the ACL ``aclName``; returns its table id for SINGLE-mode classification.
    Tuple fields per scope: ``SessionTuples``."""
    engine._ck(lib.pg_session_table_install(engine.h, vpp.h, scope, nsIndex, _b(aclName)))
    return engine.table_id(aclName)


def SessionTuples(scope, lcl_ip, lcl_port, rmt_ip, rmt_port):
    """(src_ip, dst_ip, dst_port) of connections looked up in a table of ``scope``: a local
    table keys on (local address, remote address, remote port), the global table on (remote
    address, local address, local port)."""
    if scope == ScopeLocal:
        return lcl_ip, rmt_ip, rmt_port
    return rmt_ip, lcl_ip, lcl_port
