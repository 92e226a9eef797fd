"""numpy restatement of the device tuple generator (vpp_amd/csrc/device.hip k_gen): pool /
uniform modes, and "inside a rule" sampling (uniform or Zipf rule choice) given the table's
ACL rules. TEST INFRASTRUCTURE ONLY: lets the CPU regenerate any shard
[index_base, index_base + n) of a device-generated workload, so a multi-rank run can be
checked without moving tuples (tests/test_multirank.py, tests/test_gpu_parity.py).
"""
import ipaddress

import numpy as np

M = np.uint64(0xFFFFFFFFFFFFFFFF)


def _mix64(z):
    with np.errstate(over="ignore"):
        z = z + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def _rnd(seed, i, f):
    with np.errstate(over="ignore"):
        return _mix64(np.uint64(seed) ^ _mix64(i * np.uint64(16) + np.uint64(f)))


KEY_UDP, KEY_OTHER, KEY_MAX = 0x10000, 0x20000, 0x2FFFF


def _net(cidr):
    """CIDR string -> (net, mask) of an IPv4 network as Go's ParseCIDR masks it; "" = any"""
    if not cidr:
        return 0, 0
    n = ipaddress.ip_network(cidr, strict=False)
    if n.version != 4:
        raise NotImplementedError("inside sampling of an IPv6 rule")
    return int(n.network_address), int(n.netmask)


def compile_rule(r):
    """(snet, smask, dnet, dmask, klo, khi) of a well-formed vpp_acl rule dict -- the fields of
    engine.cpp compile_acl_rule the generator reads (FAILURE-encoded rules are not sampled)."""
    if r.get("macip") or r.get("icmp") or not r.get("ip_rule", True) or not r.get("ip", True) or \
            (r.get("tcp") and r.get("udp")):
        raise NotImplementedError("inside sampling of a FAILURE-encoded rule")
    snet, smask = _net(r.get("src", ""))
    dnet, dmask = _net(r.get("dst", ""))
    sec, base = (r["tcp"], 0) if r.get("tcp") else ((r["udp"], KEY_UDP) if r.get("udp") else (None, 0))
    if sec is None:
        return snet, smask, dnet, dmask, 0, KEY_MAX
    if sec.get("src") != [0, 65535] or sec.get("dst") is None:
        return snet, smask, dnet, dmask, base, base + 0xFFFF
    lo, hi = sec["dst"][0] & 0xFFFF, sec["dst"][1] & 0xFFFF
    return (snet, smask, dnet, dmask, 1, 0) if lo > hi else (snet, smask, dnet, dmask, base + lo, base + hi)


def gen_tuples(n, seed, index_base=0, ip_pool=None, pool_pct=0, dst_pool_pct=0, port_pool=None, port_pool_pct=0,
               tcp_pct=45, udp_pct=45, nomatch_pct=0, table_id=-1, inside_pct=0, zipf_cdf=None, rules=None, **_):
    """rules: the ACL rule dicts of table_id (needed for inside_pct > 0)"""
    inside = table_id >= 0 and inside_pct > 0
    if inside and rules is None:
        raise NotImplementedError("inside-a-rule sampling needs the table's rules")
    i = np.arange(index_base, index_base + n, dtype=np.uint64)
    lo = lambda x: (x & np.uint64(0xFFFFFFFF)).astype(np.uint64)
    hi = lambda x: (x >> np.uint64(32)).astype(np.uint64)
    r0, r1, r2, r3, r4, r5 = (_rnd(seed, i, f) for f in range(6))
    pct = lo(r0) % np.uint64(100)
    pp = lo(r3) % np.uint64(100)
    proto = np.where(pp < tcp_pct, 0, np.where(pp < tcp_pct + udp_pct, 1, 2)).astype(np.uint8)
    dp = (r4 & np.uint64(0xFFFF)).astype(np.uint32)
    if port_pool is not None and len(port_pool):
        pool = np.asarray(port_pool, np.uint32)
        use = hi(r4) % np.uint64(100) < port_pool_pct
        dp = np.where(use, pool[(lo(r4) % np.uint64(len(pool))).astype(np.int64)], dp)
    src = lo(r1).astype(np.uint32)
    dst = lo(r2).astype(np.uint32)
    if ip_pool is not None and len(ip_pool):
        pool = np.asarray(ip_pool, np.uint32)
        k = np.uint64(len(pool))
        src = np.where(hi(r1) % np.uint64(100) < pool_pct, pool[(lo(r1) % k).astype(np.int64)], src)
        dst = np.where(hi(r2) % np.uint64(100) < dst_pool_pct, pool[(lo(r2) % k).astype(np.int64)], dst)
    if inside:
        cr = np.array([compile_rule(r) for r in rules], np.uint64).reshape(-1, 6)
        r6 = _rnd(seed, i, 6)
        if zipf_cdf is not None:
            k = np.searchsorted(np.asarray(zipf_cdf, np.uint64), hi(r6), side="right")
        else:
            k = r6 % np.uint64(len(rules))
        k = k.astype(np.int64)
        snet, smask, dnet, dmask, klo, khi = (cr[k, j] for j in range(6))
        m = pct < inside_pct
        full = np.uint64(0xFFFFFFFF)
        src = np.where(m, (snet | (lo(r1) & (~smask & full))).astype(np.uint32), src)
        dst = np.where(m, (dnet | (lo(r2) & (~dmask & full))).astype(np.uint32), dst)
        ok = m & (klo <= khi)
        span = np.where(ok, khi - klo + np.uint64(1), np.uint64(1))
        key = klo + (r4 >> np.uint64(16)) % span
        proto = np.where(ok, np.where(key < KEY_UDP, 0, np.where(key < KEY_OTHER, 1, 2)), proto).astype(np.uint8)
        dp = np.where(ok & (key < KEY_OTHER), (key & np.uint64(0xFFFF)).astype(np.uint32), dp)
    if nomatch_pct:
        src = np.where(pct >= 100 - nomatch_pct, np.uint32(0xF0000000) | (lo(r1).astype(np.uint32) & np.uint32(0x0FFFFFFF)),
                       src)
    sport = (r5 & np.uint64(0xFFFF)).astype(np.uint16)
    return src.astype(np.uint32), dst.astype(np.uint32), sport, dp.astype(np.uint16), proto
