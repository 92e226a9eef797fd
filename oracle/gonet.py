"""Go 1.11 ``net`` semantics used on the policy path (TEST INFRASTRUCTURE ONLY).

The reference (Go, CI on Go 1.11.x per /root/reference/.travis.yml:11-12) relies on the
standard library for: ``net.ParseCIDR`` (mock/aclengine/aclengine_mock.go:535,549),
``IPNet.Contains`` (aclengine_mock.go:541,555; renderer/cache/ports.go:118,152),
``IPNet.String`` (renderer/acl/acl_renderer.go:318,321; renderer/api.go:86-89) and
``IP.To4``/``IPMask.Size`` (plugins/policy/utils/utils.go:187-239).
The stdlib is not part of /root/reference; this module restates its published
algorithm (src/net/ip.go, Go 1.11) and is pinned through the reference's own KATs.

Representation: an IP is ``bytes`` of length 4 or 16 (Go's ``net.IP``), a mask is
``bytes`` of length 4 or 16 (Go's ``net.IPMask``). ``IPNet`` = (ip, mask); the empty
IPNet (``&net.IPNet{}``) is ``IPNet(b"", b"")``.
"""
from __future__ import annotations

from dataclasses import dataclass

IPV4LEN = 4
IPV6LEN = 16
_V4_IN_V6 = bytes([0] * 10 + [0xFF, 0xFF])
_BIG = 0xFFFFFF


@dataclass(frozen=True)
class IPNet:
    ip: bytes = b""
    mask: bytes = b""

    def is_empty(self) -> bool:
        return len(self.ip) == 0


def ipv4(a: int, b: int, c: int, d: int) -> bytes:
    """net.IPv4 -- returns the 16-byte form."""
    return _V4_IN_V6 + bytes([a, b, c, d])


def to4(ip: bytes):
    """net.IP.To4."""
    if len(ip) == IPV4LEN:
        return ip
    if len(ip) == IPV6LEN and ip[:12] == _V4_IN_V6:
        return ip[12:]
    return None


def to16(ip: bytes):
    if len(ip) == IPV4LEN:
        return _V4_IN_V6 + ip
    if len(ip) == IPV6LEN:
        return ip
    return None


def cidr_mask(ones: int, bits: int) -> bytes:
    """net.CIDRMask."""
    if bits not in (8 * IPV4LEN, 8 * IPV6LEN) or ones < 0 or ones > bits:
        return b""
    out = bytearray(bits // 8)
    n = ones
    for i in range(len(out)):
        if n >= 8:
            out[i] = 0xFF
            n -= 8
            continue
        out[i] = (~(0xFF >> n)) & 0xFF
        n = 0
    return bytes(out)


def mask_size(m: bytes):
    """net.IPMask.Size -> (ones, bits); (0, 0) for a non-canonical mask."""
    ones = simple_mask_length(m)
    if ones == -1:
        return 0, 0
    return ones, len(m) * 8


def simple_mask_length(m: bytes) -> int:
    n = 0
    for i, v in enumerate(m):
        if v == 0xFF:
            n += 8
            continue
        while v & 0x80:
            n += 1
            v = (v << 1) & 0xFF
        if v != 0:
            return -1
        for w in m[i + 1:]:
            if w != 0:
                return -1
        break
    return n


def ip_mask(ip: bytes, mask: bytes):
    """net.IP.Mask."""
    if len(mask) == IPV6LEN and len(ip) == IPV4LEN and mask[:12] == b"\xff" * 12:
        mask = mask[12:]
    if len(mask) == IPV4LEN and len(ip) == IPV6LEN and ip[:12] == _V4_IN_V6:
        ip = ip[12:]
    if len(mask) != len(ip):
        return None
    return bytes(a & b for a, b in zip(ip, mask))


def _dtoi(s: str):
    n = 0
    i = 0
    while i < len(s) and "0" <= s[i] <= "9":
        n = n * 10 + (ord(s[i]) - 48)
        if n >= _BIG:
            return _BIG, i, False
        i += 1
    if i == 0:
        return 0, 0, False
    return n, i, True


def _xtoi(s: str):
    n = 0
    i = 0
    while i < len(s):
        c = s[i]
        if "0" <= c <= "9":
            n = n * 16 + (ord(c) - 48)
        elif "a" <= c <= "f":
            n = n * 16 + (ord(c) - 97 + 10)
        elif "A" <= c <= "F":
            n = n * 16 + (ord(c) - 65 + 10)
        else:
            break
        if n >= _BIG:
            return 0, i, False
        i += 1
    if i == 0:
        return 0, i, False
    return n, i, True


def parse_ipv4(s: str):
    p = [0, 0, 0, 0]
    for i in range(IPV4LEN):
        if len(s) == 0:
            return None
        if i > 0:
            if s[0] != ".":
                return None
            s = s[1:]
        n, c, ok = _dtoi(s)
        if not ok or n > 0xFF:
            return None
        s = s[c:]
        p[i] = n
    if len(s) != 0:
        return None
    return ipv4(*p)


def parse_ipv6(s: str):
    ip = bytearray(IPV6LEN)
    ellipsis = -1
    if len(s) >= 2 and s[0] == ":" and s[1] == ":":
        ellipsis = 0
        s = s[2:]
        if len(s) == 0:
            return bytes(ip)
    i = 0
    while i < IPV6LEN:
        n, c, ok = _xtoi(s)
        if not ok or n > 0xFFFF:
            return None
        if c < len(s) and s[c] == ".":
            if ellipsis < 0 and i != IPV6LEN - IPV4LEN:
                return None
            if i + IPV4LEN > IPV6LEN:
                return None
            ip4 = parse_ipv4(s)
            if ip4 is None:
                return None
            ip[i:i + 4] = ip4[12:16]
            s = ""
            i += IPV4LEN
            break
        ip[i] = n >> 8
        ip[i + 1] = n & 0xFF
        i += 2
        s = s[c:]
        if len(s) == 0:
            break
        if s[0] != ":" or len(s) == 1:
            return None
        s = s[1:]
        if s[0] == ":":
            if ellipsis >= 0:
                return None
            ellipsis = i
            s = s[1:]
            if len(s) == 0:
                break
    if len(s) != 0:
        return None
    if i < IPV6LEN:
        if ellipsis < 0:
            return None
        n = IPV6LEN - i
        for j in range(i - 1, ellipsis - 1, -1):
            ip[j + n] = ip[j]
        for j in range(ellipsis + n - 1, ellipsis - 1, -1):
            ip[j] = 0
    elif ellipsis >= 0:
        return None
    return bytes(ip)


def parse_ip(s: str):
    """net.ParseIP (no zone)."""
    for ch in s:
        if ch == ".":
            return parse_ipv4(s)
        if ch == ":":
            return parse_ipv6(s)
    return None


def parse_cidr(s: str):
    """net.ParseCIDR -> (ip, IPNet) or None on error."""
    i = s.find("/")
    if i < 0:
        return None
    addr, mask = s[:i], s[i + 1:]
    iplen = IPV4LEN
    ip = parse_ipv4(addr)
    if ip is None:
        iplen = IPV6LEN
        ip = parse_ipv6(addr)
    n, j, ok = _dtoi(mask)
    if ip is None or not ok or j != len(mask) or n < 0 or n > 8 * iplen:
        return None
    m = cidr_mask(n, 8 * iplen)
    return ip, IPNet(ip_mask(ip, m), m)


def network_number_and_mask(n: IPNet):
    ip = to4(n.ip)
    if ip is None:
        ip = n.ip
        if len(ip) != IPV6LEN:
            return None, None
    m = n.mask
    if len(m) == IPV4LEN:
        if len(ip) != IPV4LEN:
            return None, None
    elif len(m) == IPV6LEN:
        if len(ip) == IPV4LEN:
            m = m[12:]
    else:
        return None, None
    return ip, m


def contains(n: IPNet, ip: bytes) -> bool:
    """net.IPNet.Contains."""
    nn, m = network_number_and_mask(n)
    x = to4(ip)
    if x is not None:
        ip = x
    if nn is None or len(ip) != len(nn):
        return False
    for a, b, c in zip(nn, m, ip):
        if a & b != c & b:
            return False
    return True


def ip_equal(a: bytes, b: bytes) -> bool:
    """net.IP.Equal."""
    if len(a) == len(b):
        return a == b
    if len(a) == IPV4LEN and len(b) == IPV6LEN:
        return b[:12] == _V4_IN_V6 and a == b[12:]
    if len(a) == IPV6LEN and len(b) == IPV4LEN:
        return a[:12] == _V4_IN_V6 and a[12:] == b
    return False


def ip_string(ip: bytes) -> str:
    """net.IP.String."""
    if len(ip) == 0:
        return "<nil>"
    p4 = to4(ip)
    if p4 is not None:
        return "%d.%d.%d.%d" % tuple(p4)
    if len(ip) != IPV6LEN:
        return "?" + ip.hex()
    e0, e1 = -1, -1
    i = 0
    while i < IPV6LEN:
        j = i
        while j < IPV6LEN and ip[j] == 0 and ip[j + 1] == 0:
            j += 2
        if j > i and j - i > e1 - e0:
            e0, e1 = i, j
            i = j
        i += 2
    if e1 - e0 <= 2:
        e0, e1 = -1, -1
    out = []
    i = 0
    while i < IPV6LEN:
        if i == e0:
            out.append("::")
            i = e1
            if i >= IPV6LEN:
                break
        elif i > 0:
            out.append(":")
        out.append("%x" % ((ip[i] << 8) | ip[i + 1]))
        i += 2
    return "".join(out)


def ipnet_string(n: IPNet) -> str:
    """net.IPNet.String."""
    nn, m = network_number_and_mask(n)
    if nn is None or m is None:
        return "<nil>"
    ones = simple_mask_length(m)
    if ones == -1:
        return ip_string(nn) + "/" + m.hex()
    return ip_string(nn) + "/" + str(ones)


def one_host_subnet(addr: str):
    """plugins/policy/utils/utils.go:271-291 GetOneHostSubnet."""
    ip = parse_ip(addr)
    if ip is None:
        return None
    return one_host_subnet_from_ip(ip)


def one_host_subnet_from_ip(ip: bytes) -> IPNet:
    if to4(ip) is not None:
        return IPNet(ip, cidr_mask(32, 32))
    return IPNet(ip, cidr_mask(128, 128))


def ip_network(addr: str) -> IPNet:
    """renderer/testdata/testdata.go:260-266 IpNetwork: ParseCIDR network or empty."""
    if addr == "":
        return IPNet()
    r = parse_cidr(addr)
    return r[1]


def ipv4_u32(ip: bytes) -> int:
    x = to4(ip)
    assert x is not None
    return int.from_bytes(x, "big")


def u32_ipv4(v: int) -> bytes:
    return ipv4(*(v >> 24 & 255, v >> 16 & 255, v >> 8 & 255, v & 255))
