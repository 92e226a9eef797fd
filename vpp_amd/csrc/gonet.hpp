// Go 1.11 `net` semantics used on the policy path.
//
// The reference relies on the Go standard library for net.ParseCIDR (evalACL,
// mock/aclengine/aclengine_mock.go:535,549), IPNet.Contains (:541,555; renderer/cache/
// ports.go:118,152), IPNet.String (renderer/acl/acl_renderer.go:318,321), IP.To4/IPMask.Size
// (plugins/policy/utils/utils.go:187-239). These are restated here on fixed-size byte
// arrays so that rule ordering, ACL rendering and CIDR parsing behave exactly like Go,
// including the IPv4-mapped-IPv6 and non-canonical corner cases.
#pragma once
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>

namespace pg {

struct Bytes {  // net.IP / net.IPMask: length 0, 4 or 16
    uint8_t len = 0;
    uint8_t b[16] = {};
    bool operator==(const Bytes& o) const { return len == o.len && std::memcmp(b, o.b, len) == 0; }
};

static const uint8_t kV4InV6[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0xff, 0xff};

inline Bytes mk(const uint8_t* p, int n) {
    Bytes r;
    r.len = (uint8_t)n;
    std::memcpy(r.b, p, n);
    return r;
}
inline Bytes ipv4(uint8_t a, uint8_t b, uint8_t c, uint8_t d) {  // net.IPv4: 16-byte form
    Bytes r;
    r.len = 16;
    std::memcpy(r.b, kV4InV6, 12);
    r.b[12] = a, r.b[13] = b, r.b[14] = c, r.b[15] = d;
    return r;
}
inline bool to4(const Bytes& ip, Bytes* out) {  // net.IP.To4
    if (ip.len == 4) { *out = ip; return true; }
    if (ip.len == 16 && std::memcmp(ip.b, kV4InV6, 12) == 0) { *out = mk(ip.b + 12, 4); return true; }
    return false;
}
inline Bytes to16(const Bytes& ip) {
    if (ip.len == 4) {
        Bytes r;
        r.len = 16;
        std::memcpy(r.b, kV4InV6, 12);
        std::memcpy(r.b + 12, ip.b, 4);
        return r;
    }
    return ip;
}
inline Bytes cidr_mask(int ones, int bits) {  // net.CIDRMask
    Bytes r;
    if ((bits != 32 && bits != 128) || ones < 0 || ones > bits) return r;
    r.len = (uint8_t)(bits / 8);
    int n = ones;
    for (int i = 0; i < r.len; i++) {
        if (n >= 8) { r.b[i] = 0xff; n -= 8; continue; }
        r.b[i] = (uint8_t)(~(0xffu >> n));
        n = 0;
    }
    return r;
}
inline int simple_mask_length(const Bytes& m) {
    int n = 0;
    for (int i = 0; i < m.len; i++) {
        uint8_t v = m.b[i];
        if (v == 0xff) { n += 8; continue; }
        while (v & 0x80) { n++; v = (uint8_t)(v << 1); }
        if (v != 0) return -1;
        for (int j = i + 1; j < m.len; j++)
            if (m.b[j] != 0) return -1;
        break;
    }
    return n;
}
inline void mask_size(const Bytes& m, int* ones, int* bits) {  // net.IPMask.Size
    int o = simple_mask_length(m);
    if (o == -1) { *ones = 0; *bits = 0; return; }
    *ones = o;
    *bits = m.len * 8;
}
inline bool ip_mask(Bytes ip, Bytes mask, Bytes* out) {  // net.IP.Mask; false = nil
    if (mask.len == 16 && ip.len == 4) {
        bool ff = true;
        for (int i = 0; i < 12; i++) ff &= mask.b[i] == 0xff;
        if (ff) mask = mk(mask.b + 12, 4);
    }
    if (mask.len == 4 && ip.len == 16 && std::memcmp(ip.b, kV4InV6, 12) == 0) ip = mk(ip.b + 12, 4);
    if (mask.len != ip.len) return false;
    Bytes r;
    r.len = ip.len;
    for (int i = 0; i < ip.len; i++) r.b[i] = ip.b[i] & mask.b[i];
    *out = r;
    return true;
}
inline bool ip_equal(const Bytes& a, const Bytes& b) {  // net.IP.Equal
    if (a.len == b.len) return std::memcmp(a.b, b.b, a.len) == 0;
    if (a.len == 4 && b.len == 16) return std::memcmp(b.b, kV4InV6, 12) == 0 && std::memcmp(a.b, b.b + 12, 4) == 0;
    if (a.len == 16 && b.len == 4) return std::memcmp(a.b, kV4InV6, 12) == 0 && std::memcmp(a.b + 12, b.b, 4) == 0;
    return false;
}

struct IPNet {
    Bytes ip, mask;
    bool empty() const { return ip.len == 0; }
};

inline bool network_number_and_mask(const IPNet& n, Bytes* ip, Bytes* m) {
    if (!to4(n.ip, ip)) {
        *ip = n.ip;
        if (ip->len != 16) return false;
    }
    *m = n.mask;
    if (m->len == 4) {
        if (ip->len != 4) return false;
    } else if (m->len == 16) {
        if (ip->len == 4) *m = mk(m->b + 12, 4);
    } else {
        return false;
    }
    return true;
}
inline bool contains(const IPNet& n, Bytes ip) {  // net.IPNet.Contains
    Bytes nn, m, x;
    if (!network_number_and_mask(n, &nn, &m)) return false;
    if (to4(ip, &x)) ip = x;
    if (ip.len != nn.len) return false;
    for (int i = 0; i < ip.len; i++)
        if ((nn.b[i] & m.b[i]) != (ip.b[i] & m.b[i])) return false;
    return true;
}

constexpr int kBig = 0xFFFFFF;
inline bool dtoi(const char* s, size_t len, int* n, size_t* used) {
    int v = 0;
    size_t i = 0;
    for (; i < len && s[i] >= '0' && s[i] <= '9'; i++) {
        v = v * 10 + (s[i] - '0');
        if (v >= kBig) { *n = kBig; *used = i; return false; }
    }
    if (i == 0) { *n = 0; *used = 0; return false; }
    *n = v;
    *used = i;
    return true;
}
inline bool xtoi(const char* s, size_t len, int* n, size_t* used) {
    int v = 0;
    size_t i = 0;
    for (; i < len; i++) {
        char c = s[i];
        if (c >= '0' && c <= '9') v = v * 16 + (c - '0');
        else if (c >= 'a' && c <= 'f') v = v * 16 + (c - 'a' + 10);
        else if (c >= 'A' && c <= 'F') v = v * 16 + (c - 'A' + 10);
        else break;
        if (v >= kBig) { *n = 0; *used = i; return false; }
    }
    if (i == 0) { *n = 0; *used = 0; return false; }
    *n = v;
    *used = i;
    return true;
}
inline bool parse_ipv4(const char* s, size_t len, Bytes* out) {
    uint8_t p[4];
    for (int i = 0; i < 4; i++) {
        if (len == 0) return false;
        if (i > 0) {
            if (s[0] != '.') return false;
            s++, len--;
        }
        int n;
        size_t c;
        if (!dtoi(s, len, &n, &c) || n > 0xff) return false;
        s += c, len -= c;
        p[i] = (uint8_t)n;
    }
    if (len != 0) return false;
    *out = ipv4(p[0], p[1], p[2], p[3]);
    return true;
}
inline bool parse_ipv6(const char* s, size_t len, Bytes* out) {
    Bytes ip;
    ip.len = 16;
    int ellipsis = -1;
    if (len >= 2 && s[0] == ':' && s[1] == ':') {
        ellipsis = 0;
        s += 2, len -= 2;
        if (len == 0) { *out = ip; return true; }
    }
    int i = 0;
    while (i < 16) {
        int n;
        size_t c;
        if (!xtoi(s, len, &n, &c) || n > 0xffff) return false;
        if (c < len && s[c] == '.') {
            if (ellipsis < 0 && i != 12) return false;
            if (i + 4 > 16) return false;
            Bytes ip4;
            if (!parse_ipv4(s, len, &ip4)) return false;
            std::memcpy(ip.b + i, ip4.b + 12, 4);
            len = 0;
            i += 4;
            break;
        }
        ip.b[i] = (uint8_t)(n >> 8);
        ip.b[i + 1] = (uint8_t)n;
        i += 2;
        s += c, len -= c;
        if (len == 0) break;
        if (s[0] != ':' || len == 1) return false;
        s++, len--;
        if (s[0] == ':') {
            if (ellipsis >= 0) return false;
            ellipsis = i;
            s++, len--;
            if (len == 0) break;
        }
    }
    if (len != 0) return false;
    if (i < 16) {
        if (ellipsis < 0) return false;
        int n = 16 - i;
        for (int j = i - 1; j >= ellipsis; j--) ip.b[j + n] = ip.b[j];
        for (int j = ellipsis + n - 1; j >= ellipsis; j--) ip.b[j] = 0;
    } else if (ellipsis >= 0) {
        return false;
    }
    *out = ip;
    return true;
}
inline bool parse_ip(const std::string& s, Bytes* out) {  // net.ParseIP (no zone)
    for (char ch : s) {
        if (ch == '.') return parse_ipv4(s.data(), s.size(), out);
        if (ch == ':') return parse_ipv6(s.data(), s.size(), out);
    }
    return false;
}
// net.ParseCIDR -> network (false = parse error)
inline bool parse_cidr(const std::string& s, IPNet* net) {
    size_t slash = s.find('/');
    if (slash == std::string::npos) return false;
    const char* addr = s.data();
    size_t alen = slash;
    const char* mask = s.data() + slash + 1;
    size_t mlen = s.size() - slash - 1;
    int iplen = 4;
    Bytes ip;
    bool ok = parse_ipv4(addr, alen, &ip);
    if (!ok) {
        iplen = 16;
        ok = parse_ipv6(addr, alen, &ip);
    }
    int n;
    size_t used;
    bool okm = dtoi(mask, mlen, &n, &used);
    if (!ok || !okm || used != mlen || n < 0 || n > 8 * iplen) return false;
    Bytes m = cidr_mask(n, 8 * iplen);
    Bytes masked;
    ip_mask(ip, m, &masked);
    net->ip = masked;
    net->mask = m;
    return true;
}

inline std::string ip_string(const Bytes& ip) {  // net.IP.String
    if (ip.len == 0) return "<nil>";
    Bytes p4;
    char buf[64];
    if (to4(ip, &p4)) {
        std::snprintf(buf, sizeof buf, "%u.%u.%u.%u", p4.b[0], p4.b[1], p4.b[2], p4.b[3]);
        return buf;
    }
    if (ip.len != 16) {
        std::string r = "?";
        for (int i = 0; i < ip.len; i++) {
            std::snprintf(buf, sizeof buf, "%02x", ip.b[i]);
            r += buf;
        }
        return r;
    }
    int e0 = -1, e1 = -1;
    for (int i = 0; i < 16; i += 2) {
        int j = i;
        while (j < 16 && ip.b[j] == 0 && ip.b[j + 1] == 0) j += 2;
        if (j > i && j - i > e1 - e0) { e0 = i; e1 = j; i = j; }
    }
    if (e1 - e0 <= 2) e0 = e1 = -1;
    std::string r;
    for (int i = 0; i < 16; i += 2) {
        if (i == e0) {
            r += "::";
            i = e1;
            if (i >= 16) break;
        } else if (i > 0) {
            r += ":";
        }
        std::snprintf(buf, sizeof buf, "%x", (unsigned)((ip.b[i] << 8) | ip.b[i + 1]));
        r += buf;
    }
    return r;
}
inline std::string ipnet_string(const IPNet& n) {  // net.IPNet.String
    Bytes nn, m;
    if (!network_number_and_mask(n, &nn, &m)) return "<nil>";
    int l = simple_mask_length(m);
    if (l == -1) {
        std::string r = ip_string(nn) + "/";
        char buf[4];
        for (int i = 0; i < m.len; i++) {
            std::snprintf(buf, sizeof buf, "%02x", m.b[i]);
            r += buf;
        }
        return r;
    }
    return ip_string(nn) + "/" + std::to_string(l);
}

// Compiled IPv4 match of a parsed network against IPv4 packets: (addr & mask) == net.
// Returns false when the network can never contain an IPv4 address.
inline bool ipv4_match_form(const IPNet& n, uint32_t* net, uint32_t* msk) {
    Bytes nn, m;
    if (!network_number_and_mask(n, &nn, &m)) return false;
    if (nn.len != 4) return false;
    uint32_t a = ((uint32_t)nn.b[0] << 24) | ((uint32_t)nn.b[1] << 16) | ((uint32_t)nn.b[2] << 8) | nn.b[3];
    uint32_t k = ((uint32_t)m.b[0] << 24) | ((uint32_t)m.b[1] << 16) | ((uint32_t)m.b[2] << 8) | m.b[3];
    *msk = k;
    *net = a & k;
    return true;
}
inline uint32_t ipv4_u32(const Bytes& ip) {
    Bytes x;
    if (!to4(ip, &x)) return 0;
    return ((uint32_t)x.b[0] << 24) | ((uint32_t)x.b[1] << 16) | ((uint32_t)x.b[2] << 8) | x.b[3];
}

}  // namespace pg
