"""Random vpp_acl ACLs and tuples covering every evalACL branch (test helper).

Rules include the renderer's normal shapes (CIDR src/dst, TCP/UDP sections with exact or
any ports, no L4 section) plus every failure/edge branch of evalACL
(aclengine_mock.go:510-649): MAC-IP rules, missing IpRule/Ip, ICMP, TCP+UDP, unparsable
CIDRs, IPv6 and IPv4-mapped-IPv6 CIDRs, non-canonical host bits, bad/missing port ranges,
port values above 65535 (uint16 truncation) and REFLECT / out-of-range actions.
"""
import random

import numpy as np

from oracle import aclengine, policy


def rand_cidr(rnd, anchors):
    k = rnd.random()
    if k < 0.55:
        base = rnd.choice(anchors)
        plen = rnd.choice([8, 12, 16, 20, 24, 24, 28, 30, 32, 32])
        ip = base & ((0xFFFFFFFF << (32 - plen)) & 0xFFFFFFFF) if plen else 0
        if rnd.random() < 0.1:           # host bits set (masked by ParseCIDR)
            ip |= rnd.getrandbits(32 - plen) if plen < 32 else 0
        return "%d.%d.%d.%d/%d" % (ip >> 24, ip >> 16 & 255, ip >> 8 & 255, ip & 255, plen)
    if k < 0.62:
        return "0.0.0.0/0"
    if k < 0.70:
        b = rnd.choice(anchors)
        p = rnd.choice([96, 104, 112, 120, 128, 88, 64])
        return "::ffff:%d.%d.%d.%d/%d" % (b >> 24, b >> 16 & 255, b >> 8 & 255, b & 255, p)
    if k < 0.75:
        return rnd.choice(["::/0", "2001:db8::/32", "fe80::1/64", "::/96"])
    if k < 0.80:
        return rnd.choice(["10.0.0.0", "10.0.0.0/33", "300.1.1.1/8", "10.0.0/8", "abc", "10.0.0.0/", "/8",
                           "010.001.0.0/16", "1.2.3.4/08", "::ffff:10.0.0.0/129", "1:2:3:4:5:6:7:8:9/64"])
    return ""


def rand_l4(rnd):
    k = rnd.random()
    if k < 0.75:
        lo = rnd.choice([0, 22, 53, 80, 443, rnd.randint(1, 65535)])
        hi = lo if rnd.random() < 0.6 else min(65535, lo + rnd.randint(0, 2000))
        if rnd.random() < 0.1:
            lo, hi = 0, 65535
        return {"src": [0, 65535], "dst": [lo, hi]}
    if k < 0.80:
        return {"src": None, "dst": [0, 65535]}
    if k < 0.85:
        return {"src": [0, 65534], "dst": [0, 65535]}
    if k < 0.90:
        return {"src": [0, 65535], "dst": None}
    if k < 0.95:
        return {"src": [0, 65535], "dst": [65536 + rnd.randint(0, 100), 65536 + rnd.randint(100, 70000)]}
    return {"src": [0, 65535], "dst": [rnd.randint(1000, 2000), rnd.randint(0, 999)]}


def rand_rule(rnd, anchors, weird=True):
    r = {"action": rnd.choice([0, 1, 1, 2]), "src": rand_cidr(rnd, anchors), "dst": rand_cidr(rnd, anchors)}
    if not weird:
        for f in ("src", "dst"):
            if r[f] and (":" in r[f] or not r[f].count(".") == 3 or "/" not in r[f]):
                r[f] = ""
            elif r[f]:
                try:
                    a, p = r[f].split("/")
                    if int(p) > 32 or any(int(x) > 255 for x in a.split(".")) or a.startswith("0") and a != "0.0.0.0":
                        r[f] = ""
                except ValueError:
                    r[f] = ""
    k = rnd.random()
    if k < 0.35:
        r["tcp"] = rand_l4(rnd) if weird else {"src": [0, 65535], "dst": sorted([rnd.randint(0, 65535)] * 2)}
    elif k < 0.70:
        r["udp"] = rand_l4(rnd) if weird else {"src": [0, 65535], "dst": sorted([rnd.randint(0, 65535)] * 2)}
    if weird:
        z = rnd.random()
        if z < 0.015:
            r["macip"] = True
        elif z < 0.03:
            r["ip_rule"] = False
        elif z < 0.045:
            r["icmp"] = True
        elif z < 0.06:
            r["ip"] = False
        elif z < 0.075:
            r["tcp"] = rand_l4(rnd)
            r["udp"] = rand_l4(rnd)
        elif z < 0.09:
            r["action"] = rnd.choice([3, 7, -1])
    return r


def rand_acl(rnd, n, anchors, weird=True, tail=None):
    rules = [rand_rule(rnd, anchors, weird) for _ in range(n)]
    if tail == "deny":
        rules.append({"action": 0, "src": "", "dst": ""})
    elif tail == "permit":
        rules.append({"action": 1, "src": "", "dst": ""})
    return rules


def rand_tuples(rnd_np, n, anchors, any_pct=0.0):
    """src/dst: 50 % near an anchor (inside many prefixes), 50 % uniform; proto TCP/UDP/OTHER
    (+ ANY/invalid codes when any_pct > 0); ports biased to the popular ones."""
    anchors = np.array(anchors, np.uint32)

    def ips():
        near = anchors[rnd_np.integers(0, len(anchors), n)] ^ (rnd_np.integers(0, 1 << 12, n).astype(np.uint32))
        uni = rnd_np.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
        return np.where(rnd_np.random(n) < 0.5, near, uni).astype(np.uint32)

    src, dst = ips(), ips()
    proto = rnd_np.choice(np.array([0, 1, 2], np.uint8), n, p=[0.45, 0.45, 0.10])
    if any_pct:
        m = rnd_np.random(n) < any_pct
        proto[m] = rnd_np.choice(np.array([3, 7, 255], np.uint8), int(m.sum()))
    pop = np.array([0, 22, 53, 80, 443, 1000, 1500, 65535], np.uint16)
    dport = np.where(rnd_np.random(n) < 0.5, pop[rnd_np.integers(0, len(pop), n)],
                     rnd_np.integers(0, 65536, n)).astype(np.uint16)
    sport = rnd_np.integers(0, 65536, n).astype(np.uint16)
    return src, dst, sport, dport, proto


def to_oracle_acl(name, rules):
    """dict rules -> oracle.policy.ACL (for the pure-Python evalACL)."""
    acl = policy.ACL(name)
    for r in rules:
        ar = policy.AclRule(action=r["action"], has_ip_rule=r.get("ip_rule", True), has_ip=r.get("ip", True),
                            has_icmp=r.get("icmp", False), has_macip=r.get("macip", False),
                            src_network=r.get("src") or "", dst_network=r.get("dst") or "")
        for f in ("tcp", "udp"):
            s = r.get(f)
            if s:
                sec = policy.L4Section(policy.PortRange(*s["src"]) if s.get("src") is not None else None,
                                       policy.PortRange(*s["dst"]) if s.get("dst") is not None else None)
                setattr(ar, f, sec)
        acl.rules.append(ar)
    return acl


def py_eval(acl, src, dst, dport, proto):
    from oracle import gonet
    out_a, out_i = [], []
    for s, d, p, pr in zip(src, dst, dport, proto):
        a, i = aclengine.eval_acl(acl, gonet.u32_ipv4(int(s)), gonet.u32_ipv4(int(d)), int(pr), int(p))
        out_a.append(a)
        out_i.append(i)
    return np.array(out_a), np.array(out_i)


ANCHORS = [0x0A0A0101, 0x0A0A0201, 0x0A0A0A01, 0x0A000000, 0xC0A80101, 0x08080808, 0xAC100001, 0x01020304]
