// Device ACL engine: ACL install semantics + the table compiler.
#include "engine.hpp"

#include <algorithm>
#include <set>

#include "../../include/policygpu.h"

namespace pg {

// ---- compile one vpp_acl rule (aclengine_mock.go:510-649) --------------------------------
// Every outcome of evalACL for a rule is expressed as (src predicate, dst predicate,
// key range, action-on-key-match, action-for-ANY-packets):
//   * structural errors (MAC-IP, no IpRule, ICMP, no Ip, TCP+UDP) and an unparsable src
//     CIDR return FAILURE for every packet before any match test (:511-539);
//   * a src/dst network that cannot contain an IPv4 address never matches (:541,555);
//   * an unparsable dst CIDR returns FAILURE once src matched (:551-553);
//   * a TCP section with a bad/missing src range or missing dst range returns FAILURE for
//     TCP packets whose src/dst matched (:570-588), and never matches UDP/OTHER packets;
//   * ANY (or any unknown) packet protocol skips the L4 test entirely (:562 switch).
DevRule compile_acl_rule(const AclRule& r) {
    DevRule d{};
    auto never = [&]() {
        d.klo = 1;
        d.khi = 0;
        d.act = (kActNever << 4) | kActDeny;
        return d;
    };
    auto all_fail = [&]() {
        d.klo = 0;
        d.khi = kKeyMax;
        d.act = (kActFailure << 4) | kActFailure;
        return d;
    };
    if (r.has_macip || !r.has_ip_rule || r.has_icmp || !r.has_ip || (r.tcp.present && r.udp.present)) {
        d.snet = d.smask = d.dnet = d.dmask = 0;
        return all_fail();
    }
    if (!r.src_network.empty()) {
        IPNet n;
        if (!parse_cidr(r.src_network, &n)) return all_fail();
        if (!ipv4_match_form(n, &d.snet, &d.smask)) return never();
    }
    if (!r.dst_network.empty()) {
        IPNet n;
        if (!parse_cidr(r.dst_network, &n)) {
            d.dnet = d.dmask = 0;
            return all_fail();  // src predicate kept
        }
        if (!ipv4_match_form(n, &d.dnet, &d.dmask)) return never();
    }
    uint32_t a = (r.action == kAclDeny || r.action == kAclPermit || r.action == kAclReflect) ? (uint32_t)r.action
                                                                                             : kActFailure;
    const L4Section* s = r.tcp.present ? &r.tcp : (r.udp.present ? &r.udp : nullptr);
    uint32_t base = r.tcp.present ? 0u : kKeyUDP;
    if (!s) {
        d.klo = 0;
        d.khi = kKeyMax;
        d.act = (a << 4) | a;
        return d;
    }
    if (!s->has_src || s->src.lower != 0 || s->src.upper != 0xFFFF || !s->has_dst) {
        d.klo = base;
        d.khi = base + 0xFFFF;
        d.act = (a << 4) | kActFailure;
        return d;
    }
    uint32_t lo = s->dst.lower & 0xFFFF, hi = s->dst.upper & 0xFFFF;  // uint16 truncation (:589)
    if (lo > hi) {
        d.klo = 1;
        d.khi = 0;
    } else {
        d.klo = base + lo;
        d.khi = base + hi;
    }
    d.act = (a << 4) | a;
    return d;
}

static bool unconditional(const DevRule& r) {  // matches every packet that reaches it
    return r.dmask == 0 && r.klo == 0 && r.khi == kKeyMax;
}

// ---- src-interval index ---------------------------------------------------------------
// The IPv4 src space is cut at every rule's src-prefix boundary; inside one interval the
// set of rules whose src matches is constant. Each interval keeps that set (ascending rule
// index, truncated after the first rule that matches unconditionally), so the device only
// tests dst + L4 of the candidates and the first hit is the first match of the ACL.
bool build_table_index(const DevRule* rules, uint32_t n, HostTableSet& h, DevTable& hdr, uint64_t cand_budget) {
    std::vector<uint32_t> bnd{0};
    for (uint32_t i = 0; i < n; i++) {
        const DevRule& r = rules[i];
        if (r.smask == 0 || (r.klo > r.khi && (r.act >> 4) == kActNever)) continue;
        bnd.push_back(r.snet);
        uint64_t end = (uint64_t)r.snet + (uint64_t)(~r.smask) + 1ull;
        if (end < (1ull << 32)) bnd.push_back((uint32_t)end);
    }
    std::sort(bnd.begin(), bnd.end());
    bnd.erase(std::unique(bnd.begin(), bnd.end()), bnd.end());
    uint32_t nb = (uint32_t)bnd.size();

    // sweep: events per boundary (rules starting / ending there)
    std::vector<std::pair<uint32_t, uint32_t>> starts, ends;  // (addr, rule)
    std::set<uint32_t> active;                                // rule indices whose src covers the sweep point
    for (uint32_t i = 0; i < n; i++) {
        const DevRule& r = rules[i];
        if (r.klo > r.khi && (r.act >> 4) == kActNever) continue;  // never matches
        if (r.smask == 0) {
            active.insert(i);
            continue;
        }
        starts.push_back({r.snet, i});
        uint64_t end = (uint64_t)r.snet + (uint64_t)(~r.smask) + 1ull;
        if (end < (1ull << 32)) ends.push_back({(uint32_t)end, i});
    }
    std::sort(starts.begin(), starts.end());
    std::sort(ends.begin(), ends.end());
    size_t si = 0, ei = 0;
    uint64_t total = 0;
    hdr.bnd_base = (uint32_t)h.bnd.size();
    hdr.nb = nb;
    for (uint32_t k = 0; k < nb; k++) {
        uint32_t a = bnd[k];
        while (ei < ends.size() && ends[ei].first <= a) active.erase(ends[ei++].second);
        while (si < starts.size() && starts[si].first <= a) active.insert(starts[si++].second);
        h.bnd.push_back(a);
        uint32_t first = (uint32_t)(h.cand_rule.size());
        uint32_t cnt = 0;
        for (uint32_t ri : active) {
            const DevRule& r = rules[ri];
            if (r.klo <= r.khi || (r.act >> 4) != kActNever) {
                h.cand.push_back(r.dnet);
                h.cand.push_back(r.dmask);
                h.cand.push_back(r.klo | ((r.act & 0xFF) << 24));
                h.cand.push_back(r.khi);
                h.cand_rule.push_back(ri);
                cnt++;
            }
            if (unconditional(r)) break;
        }
        h.ivl.push_back(first);
        h.ivl.push_back(cnt);
        total += cnt;
        if (total > cand_budget) return false;
    }
    // radix over the top bits: interval containing (x << shift)
    uint32_t bits = 0;
    while ((1u << bits) < nb && bits < 16) bits++;
    if (nb > 8 && bits < 16) bits++;
    if (nb <= 8) bits = 0;
    hdr.radix_base = (uint32_t)h.radix.size();
    hdr.radix_shift = 32 - bits;
    uint32_t nbuckets = 1u << bits;
    uint32_t k = 0;
    for (uint32_t x = 0; x < nbuckets; x++) {
        uint64_t addr = bits ? ((uint64_t)x << (32 - bits)) : 0;
        while (k + 1 < nb && bnd[k + 1] <= addr) k++;
        h.radix.push_back(k);
    }
    h.radix.push_back(nb - 1);
    return true;
}

// ---- Engine ------------------------------------------------------------------------------
Engine::~Engine() {
    if (cur) dev_free(cur);
    if (counters) dev_release(counters);
}

std::string Engine::del_acl(const std::string& name) {  // aclengine_mock.go:664-680
    auto it = by_name.find(name);
    if (it == by_name.end()) return "cannot find ACL: " + name;
    by_name.erase(it);
    for (auto& kv : by_if) {
        if (kv.second.first && kv.second.first->name == name) kv.second.first = nullptr;
        if (kv.second.second && kv.second.second->name == name) kv.second.second = nullptr;
    }
    changes++;
    dirty = true;
    return "";
}

std::string Engine::put_acl(const ACLPtr& acl) {  // aclengine_mock.go:683-712
    if (!acl) return "ACL is nil";
    if (acl->ingress.empty() && acl->egress.empty()) return "ACL with empty interfaces";
    if (by_name.count(acl->name)) {
        del_acl(acl->name);
        changes--;
    }
    by_name[acl->name] = acl;
    for (auto& i : acl->ingress) by_if[i].first = acl;
    for (auto& i : acl->egress) by_if[i].second = acl;
    changes++;
    dirty = true;
    return "";
}

std::string Engine::apply_txn(bool resync, const AclOps& ops) {  // aclengine_mock.go:151-228
    committed++;
    dirty = true;
    if (resync) {
        by_name.clear();
        by_if.clear();
        for (auto& kv : ops) {
            std::string e = put_acl(kv.second);
            if (!e.empty()) return e;
        }
        return "";
    }
    for (auto& kv : ops) {
        std::string e = kv.second ? put_acl(kv.second) : del_acl(kv.first);
        if (!e.empty()) return e;
    }
    return "";
}

std::string engine_apply_cb(void* engine, bool resync, const AclOps& ops) {
    return static_cast<Engine*>(engine)->apply_txn(resync, ops);
}

std::string Engine::node_if_name() const {
    return !ifaces.vxlan_bvi.empty() ? ifaces.vxlan_bvi : ifaces.main_if;
}

int Engine::iface_of(const std::string& name) const {
    auto it = iface_index.find(name);
    return it == iface_index.end() ? -1 : it->second;
}

const DevTableSet* Engine::view() const { return cur ? &dev_view(cur) : nullptr; }

static uint32_t hash_ip(uint32_t ip) {
    ip ^= ip >> 16;
    ip *= 0x7feb352du;
    ip ^= ip >> 15;
    ip *= 0x846ca68bu;
    ip ^= ip >> 16;
    return ip;
}

int Engine::sync() {
    if (!dirty && cur) return PG_OK;
    HostTableSet h;
    table_of_acl.clear();
    table_names.clear();
    slot_table.clear();
    slot_rule.clear();
    for (auto& kv : by_name) {
        int t = (int)table_names.size();
        table_of_acl[kv.first] = t;
        table_names.push_back(kv.first);
        DevTable hdr{};
        hdr.rule_base = (uint32_t)h.rules.size();
        hdr.n_rules = (uint32_t)kv.second->rules.size();
        for (size_t i = 0; i < kv.second->rules.size(); i++) {
            h.rules.push_back(compile_acl_rule(kv.second->rules[i]));
            slot_table.push_back(t);
            slot_rule.push_back((int32_t)i);
        }
        h.tabs.push_back(hdr);
    }
    const uint64_t budget = 1ull << 27;  // candidate entries (2 GiB at 16+4 B) before linear fallback
    for (size_t t = 0; t < h.tabs.size(); t++) {
        DevTable& hdr = h.tabs[t];
        size_t b0 = h.bnd.size(), i0 = h.ivl.size(), r0 = h.radix.size(), c0 = h.cand.size(), cr0 = h.cand_rule.size();
        if (!build_table_index(h.rules.data() + hdr.rule_base, hdr.n_rules, h, hdr, budget)) {
            h.bnd.resize(b0), h.ivl.resize(i0), h.radix.resize(r0), h.cand.resize(c0), h.cand_rule.resize(cr0);
            hdr.flags = 1;  // linear scan
            hdr.nb = 0;
        }
    }
    uint32_t T = (uint32_t)h.tabs.size();
    for (uint32_t t = 0; t < T; t++) slot_table.push_back((int32_t)t), slot_rule.push_back(-1);
    slot_table.push_back(-1), slot_rule.push_back(-1);  // no ACL
    slot_table.push_back(-1), slot_rule.push_back(-2);  // unresolved interface

    // interfaces
    iface_index.clear();
    auto add_if = [&](const std::string& n) {
        if (!iface_index.count(n)) iface_index[n] = (int)iface_index.size();
    };
    for (auto& kv : by_if) add_if(kv.first);
    for (auto& kv : ifaces.pod_if) add_if(kv.second);
    for (auto& n : ifaces.node_output_ifs()) add_if(n);
    h.ifaces.assign(iface_index.size() * 2, -1);
    for (auto& kv : by_if) {
        int i = iface_index[kv.first];
        if (kv.second.first) h.ifaces[2 * i] = table_of_acl[kv.second.first->name];
        if (kv.second.second) h.ifaces[2 * i + 1] = table_of_acl[kv.second.second->name];
    }
    std::string nif = node_if_name();
    h.node_if = nif.empty() ? -1 : iface_index[nif];
    // local pod IP -> TAP interface
    std::vector<std::pair<uint32_t, int32_t>> ipmap;
    for (auto& kv : pods) {
        Bytes v4;
        if (kv.second.another_node || !to4(kv.second.ip, &v4)) continue;
        std::string ifn;
        int32_t idx = ifaces.if_name(kv.first, &ifn) ? iface_index[ifn] : -2;
        ipmap.push_back({ipv4_u32(v4), idx});
    }
    uint32_t cap = 16;
    while (cap < 2 * ipmap.size() + 16) cap <<= 1;
    h.iphash.assign(2 * cap, 0xFFFFFFFFu);
    h.iphash_mask = cap - 1;
    for (auto& e : ipmap) {
        uint32_t s = hash_ip(e.first) & h.iphash_mask;
        while (h.iphash[2 * s + 1] != 0xFFFFFFFFu && h.iphash[2 * s] != e.first) s = (s + 1) & h.iphash_mask;
        h.iphash[2 * s] = e.first;
        h.iphash[2 * s + 1] = (uint32_t)e.second;
    }

    std::string err;
    DeviceBuffers* nb = dev_upload(h, &err);
    if (!nb) {
        last_error = "upload: " + err;
        return PG_EIO;
    }
    if (cur) dev_free(cur);  // dev_upload synchronises before returning: old set is idle
    cur = nb;
    size_t slots = dev_view(cur).n_slots;
    if (slots != counter_slots) {
        if (counters) dev_release(counters);
        counters = (unsigned long long*)dev_alloc(slots * sizeof(unsigned long long), &err);
        if (!counters) {
            last_error = err;
            counter_slots = 0;
            return PG_ENOMEM;
        }
        counter_slots = slots;
    }
    // slot meanings change with the tables: counters restart from zero
    if (dev_memset(counters, 0, slots * 8, nullptr, &err) != 0 || dev_sync(&err) != 0) {
        last_error = err;
        return PG_EIO;
    }
    dirty = false;
    return PG_OK;
}

}  // namespace pg
