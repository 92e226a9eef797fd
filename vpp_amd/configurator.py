"""Python mirror of the policy configurator (plugins/policy/configurator) and the mock
renderer (mock/renderer), keeping the reference's names so the parity tests read like
configurator_test.go. Everything delegates to the C ABI (vpp_amd/csrc/configurator.cpp).

    cfg = PolicyConfigurator()
    cfg.AddPodConfig(("default", "pod1"), "192.168.1.1")   # the policy cache's LookupPod data
    cfg.SetNatLoopbackIP("10.1.255.254")                   # IPAM.NatLoopbackIP()
    mock = MockRenderer(); cfg.RegisterRenderer(mock)      # or a renderer.Renderer (GPU ACL)
    txn = cfg.NewTxn(False); txn.Configure(pod1, [policy1]); txn.Commit()
    mock.TestTraffic(pod1, EgressTraffic, "192.168.1.2", "192.168.1.1", TCP, 123, 80)
"""
import ctypes as C
import ipaddress

from . import _capi
from . import renderer as R
from ._capi import lib

# configurator.PolicyType / MatchType / ProtocolType (configurator_api.go:168-236)
PolicyIngress, PolicyEgress, PolicyAll = 0, 1, 2
MatchIngress, MatchEgress = 0, 1
TCP, UDP = 0, 1
# mock/renderer TrafficDirection / TrafficAction (renderer_mock.go:13-37)
IngressTraffic, EgressTraffic = 0, 1
DeniedTraffic, AllowedTraffic, UnmatchedTraffic = 0, 1, 2


def ParseCIDR(s):
    """net.ParseCIDR's network: the address masked to the prefix (configurator_test.go
    parseIPNet)."""
    n = ipaddress.ip_network(s, strict=False)
    return R.IPNet("%s/%d" % (n.network_address, n.prefixlen))


class Port:
    def __init__(self, Protocol=TCP, Number=0):
        self.Protocol, self.Number = Protocol, Number


class IPBlock:
    def __init__(self, Network, Except=()):
        self.Network = Network if isinstance(Network, R.IPNet) else ParseCIDR(Network)
        self.Except = [e if isinstance(e, R.IPNet) else ParseCIDR(e) for e in Except]


class Match:
    """Pods / IPBlocks None = Go nil (both nil: match anything on L3)."""

    def __init__(self, Type=MatchIngress, Pods=None, IPBlocks=None, Ports=None):
        self.Type, self.Pods, self.IPBlocks, self.Ports = Type, Pods, IPBlocks, Ports or []


class ContivPolicy:
    def __init__(self, ID, Type=PolicyIngress, Matches=()):
        self.ID, self.Type, self.Matches = R._pod(ID), Type, list(Matches)


def _b(s):
    return s.encode() if isinstance(s, str) else s


def _policies_array(policies, keep):
    arr = (_capi.pg_policy * max(1, len(policies)))()
    for i, p in enumerate(policies):
        x = arr[i]
        ns, name = _b(p.ID[0]), _b(p.ID[1])
        keep += [ns, name]
        x.id.ns, x.id.name = ns, name
        x.type = p.Type
        ms = (_capi.pg_match * max(1, len(p.Matches)))()
        keep.append(ms)
        for k, m in enumerate(p.Matches):
            y = ms[k]
            y.type = m.Type
            y.pods_nil = int(m.Pods is None)
            pods = list(m.Pods or [])
            pa = (_capi.pg_pod_id * max(1, len(pods)))()
            for j, pod in enumerate(pods):
                pns, pn = (_b(v) for v in R._pod(pod))
                keep += [pns, pn]
                pa[j].ns, pa[j].name = pns, pn
            y.pods, y.n_pods = pa, len(pods)
            y.blocks_nil = int(m.IPBlocks is None)
            blocks = list(m.IPBlocks or [])
            ba = (_capi.pg_ipblock * max(1, len(blocks)))()
            for j, bl in enumerate(blocks):
                ba[j].network = bl.Network.c()
                ex = (_capi.pg_ipnet * max(1, len(bl.Except)))()
                for q, e in enumerate(bl.Except):
                    ex[q] = e.c()
                keep.append(ex)
                ba[j].except_, ba[j].n_except = ex, len(bl.Except)
            y.blocks, y.n_blocks = ba, len(blocks)
            po = (_capi.pg_cfg_port * max(1, len(m.Ports)))()
            for j, prt in enumerate(m.Ports):
                po[j].protocol, po[j].number = prt.Protocol, prt.Number
            y.ports, y.n_ports = po, len(m.Ports)
            keep += [pa, ba, po]
        x.matches, x.n_matches = ms, len(p.Matches)
    return arr


class MockRenderer:
    """mock/renderer.MockRenderer: stores the rendered lists; TestTraffic evaluates them."""

    def __init__(self, name="mock"):
        self.name = name
        self.h = lib.pg_mock_renderer_new()

    def GetPodIP(self, pod):
        ns, name = (_b(v) for v in R._pod(pod))
        buf = C.create_string_buffer(64)
        ml = C.c_int()
        lib.pg_mock_renderer_pod_ip(self.h, ns, name, buf, 64, C.byref(ml))
        return buf.value.decode(), ml.value

    def Rules(self, pod, direction):
        """the pod's ingress (IngressTraffic) / egress list as rendered, or None"""
        ns, name = (_b(v) for v in R._pod(pod))
        n = lib.pg_mock_renderer_rules(self.h, ns, name, direction, None, 0)
        if n < 0:
            return None
        arr = (_capi.pg_contiv_rule * max(1, n))()
        lib.pg_mock_renderer_rules(self.h, ns, name, direction, arr, n)
        out = []
        for r in arr[:n]:
            def net(v):
                if not v.family:
                    return R.IPNet()
                a = ipaddress.ip_address(bytes(v.addr[:4] if v.family == 4 else v.addr[:16]))
                return R.IPNet("%s/%d" % (a, v.prefix_len))
            out.append(R.ContivRule(r.action, net(r.src), net(r.dst), r.protocol, r.src_port, r.dst_port))
        return out

    def TestTraffic(self, pod, direction, srcIP, destIP, protocol, srcPort, destPort):
        ns, name = (_b(v) for v in R._pod(pod))
        rc = lib.pg_mock_renderer_test_traffic(self.h, ns, name, direction, _b(srcIP), _b(destIP), protocol, srcPort,
                                               destPort)
        if rc < 0:
            raise R.PolicyError(rc, "TestTraffic")
        return rc

    def InstallTraffic(self, engine, pod, direction, aclName):
        """TestTraffic on the device: the pod's ingress / egress list installed in ``engine`` as
        the ACL ``aclName``; returns its table id (None: the pod was not rendered, every packet
        UnmatchedTraffic). Verdicts of pg_classify SINGLE on it: ``TrafficOf``."""
        ns, name = (_b(v) for v in R._pod(pod))
        rc = lib.pg_mock_renderer_install(engine.h, self.h, ns, name, direction, _b(aclName))
        if rc == _capi.PG_ENOENT:
            return None
        engine._ck(rc)
        return engine.table_id(aclName)

    @staticmethod
    def TrafficOf(engine, table_id, verdicts):
        """verdict words of a TestTraffic table -> TrafficAction (Denied 0, Allowed 1,
        Unmatched 2)"""
        import numpy as np
        v = np.asarray(verdicts, np.uint32)
        act = np.where((v >> 30) == 1, 1, 0)
        return np.where((v & 0x3FFFFFFF) == engine.slot_of_rule(table_id, -1), 2, act)

    def __del__(self):
        if getattr(self, "h", None) and lib is not None:
            lib.pg_mock_renderer_free(self.h)
            self.h = None


class PolicyConfigurator:
    """configurator.PolicyConfigurator with its Deps reduced to data: the policy cache's pod
    addresses (AddPodConfig / DelPodConfig) and the NAT-loopback address."""

    def __init__(self):
        self.h = lib.pg_configurator_new()
        self._renderers = []  # keep registered renderers alive

    def AddPodConfig(self, pod, ip):
        ns, name = (_b(v) for v in R._pod(pod))
        assert lib.pg_configurator_set_pod(self.h, ns, name, _b(ip or "")) == 0

    def DelPodConfig(self, pod):
        ns, name = (_b(v) for v in R._pod(pod))
        assert lib.pg_configurator_set_pod(self.h, ns, name, None) == 0

    def SetNatLoopbackIP(self, ip):
        assert lib.pg_configurator_set_nat_loopback(self.h, _b(ip) if ip else None) == 0

    def RegisterRenderer(self, r):
        from . import vpptcp
        if isinstance(r, MockRenderer):
            rc = lib.pg_configurator_register_mock(self.h, r.h)
        elif isinstance(r, vpptcp.Renderer):  # the VPPTCP session-rule renderer
            rc = lib.pg_configurator_register_vpptcp(self.h, r.h)
        else:  # renderer.Renderer: the GPU ACL renderer
            rc = lib.pg_configurator_register_renderer(self.h, r.h)
        self._renderers.append(r)
        return None if rc == 0 else R.PolicyError(rc, "RegisterRenderer")

    def NewTxn(self, resync):
        return ConfiguratorTxn(self, lib.pg_configurator_new_txn(self.h, int(resync)))

    def __del__(self):
        if getattr(self, "h", None) and lib is not None:
            lib.pg_configurator_free(self.h)
            self.h = None


class ConfiguratorTxn:
    def __init__(self, cfg, h):
        self.cfg, self.h = cfg, h

    def Configure(self, pod, policies):
        ns, name = (_b(v) for v in R._pod(pod))
        keep = []
        arr = _policies_array(list(policies), keep)
        rc = lib.pg_cfg_txn_configure(self.h, ns, name, arr, len(policies))
        if rc:
            raise R.PolicyError(rc, lib.pg_configurator_last_error(self.cfg.h).decode())
        return self

    def Commit(self):
        h, self.h = self.h, None
        rc = lib.pg_cfg_txn_commit(h)
        return None if rc == 0 else R.PolicyError(rc, lib.pg_configurator_last_error(self.cfg.h).decode())

    def __del__(self):
        if getattr(self, "h", None) and lib is not None:
            lib.pg_cfg_txn_free(self.h)
