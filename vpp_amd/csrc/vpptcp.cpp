// VPPTCP renderer + VPP session-rule tables (see vpptcp.hpp for the reference map).
#include "vpptcp.hpp"

#include <algorithm>
#include <cstring>

namespace pg {

const char* kSessionRuleTagPrefix = "contiv/vpp-policy";
static const char* kAnyProtocolTag = "-ANY";
static const char* kSplitTag = "-SPLIT";

static bool has_suffix(const std::string& s, const std::string& suf) {
    return s.size() >= suf.size() && s.compare(s.size() - suf.size(), suf.size(), suf) == 0;
}

// utils.CompareIPNetsBytes (utils.go:261-267): prefix length, then the 16 raw bytes
static int compare_ipnets_bytes(uint8_t ap, const uint8_t* a, uint8_t bp, const uint8_t* b) {
    int o = compare_ints(ap, bp);
    if (o != 0) return o;
    int c = std::memcmp(a, b, 16);
    return c < 0 ? -1 : (c > 0 ? 1 : 0);
}

// utils.CompareInts over Go's 64-bit int: u32 fields stay non-negative
static int cmp64(int64_t a, int64_t b) { return a < b ? -1 : (a > b ? 1 : 0); }

int SessionRule::compare(const SessionRule& o, bool compare_tag) const {
    int c;
    if ((c = cmp64(appns_index, o.appns_index))) return c;
    if ((c = compare_ints(scope, o.scope))) return c;
    if ((c = cmp64(action_index, o.action_index))) return c;
    if ((c = compare_ints(is_ip4, o.is_ip4))) return c;
    if ((c = compare_ipnets_bytes(lcl_plen, lcl_ip, o.lcl_plen, o.lcl_ip))) return c;
    if ((c = compare_ipnets_bytes(rmt_plen, rmt_ip, o.rmt_plen, o.rmt_ip))) return c;
    if ((c = compare_ints(transport_proto, o.transport_proto))) return c;
    if ((c = compare_ints(lcl_port, o.lcl_port))) return c;
    if ((c = compare_ints(rmt_port, o.rmt_port))) return c;
    if (compare_tag) {
        int t = std::memcmp(tag, o.tag, sizeof(tag));
        return t < 0 ? -1 : (t > 0 ? 1 : 0);
    }
    return 0;
}

std::string SessionRule::tag_str() const {
    size_t n = 0;
    while (n < sizeof(tag) && tag[n]) n++;
    return std::string(tag, n);
}

void SessionRule::set_tag(const std::string& t) {
    std::memset(tag, 0, sizeof(tag));
    std::memcpy(tag, t.data(), std::min(t.size(), sizeof(tag)));
}

bool AppNsIndex::ns_index(const PodID& pod, uint32_t* out) const {
    auto it = by_pod.find(pod);
    if (it == by_pod.end()) return false;
    *out = it->second;
    return true;
}

bool AppNsIndex::pod_by_ns_index(uint32_t idx, PodID* out) const {
    for (auto& kv : by_pod)
        if (kv.second == idx) {
            *out = kv.first;
            return true;
        }
    return false;
}

// copy(dst[:], ip) of a net.IP holding 0, 4 or 16 bytes
static void copy_ip(uint8_t* dst, const Bytes& ip) { std::memcpy(dst, ip.b, ip.len); }

static int plen_of(const Bytes& mask) {  // ones, _ := Mask.Size()
    int ones = 0, bits = 0;
    mask_size(mask, &ones, &bits);
    return ones < 0 ? 0 : ones;
}

// convertContivRule (session_rule.go:263-361): rule protocol is TCP or UDP here
static void convert_contiv_rule(const ContivRule& rule, bool global, uint32_t ns_index, const std::string& tag_prefix,
                                std::vector<SessionRule>* out) {
    SessionRule sr;
    sr.transport_proto = rule.protocol == kTCP ? kSrProtoTCP : kSrProtoUDP;
    Bytes v4;
    if (global && (rule.src.ip.len == 0 || to4(rule.src.ip, &v4))) sr.is_ip4 = 1;
    if (!global && (rule.dst.ip.len == 0 || to4(rule.dst.ip, &v4))) sr.is_ip4 = 1;
    if (global) {  // local tables: lcl 0/0
        if (sr.is_ip4) {
            if (to4(rule.dst.ip, &v4)) copy_ip(sr.lcl_ip, v4);
        } else if (rule.dst.ip.len) {
            copy_ip(sr.lcl_ip, to16(rule.dst.ip));
        }
        sr.lcl_plen = (uint8_t)plen_of(rule.dst.mask);
    }
    sr.lcl_port = global ? rule.dst_port : rule.src_port;
    const IPNet& rmt = global ? rule.src : rule.dst;
    if (rmt.ip.len > 0) {
        if (sr.is_ip4) {
            if (to4(rmt.ip, &v4)) copy_ip(sr.rmt_ip, v4);
        } else {
            copy_ip(sr.rmt_ip, to16(rmt.ip));
        }
        sr.rmt_plen = (uint8_t)plen_of(rmt.mask);
    }
    sr.rmt_port = global ? rule.src_port : rule.dst_port;
    sr.action_index = rule.action == kPermit ? kSrActionAllow : kSrActionDeny;
    sr.appns_index = ns_index;
    sr.scope = global ? kScopeGlobal : kScopeLocal;
    if ((global && rule.src.ip.len == 0) || (!global && rule.dst.ip.len == 0)) {
        // deny-all split into two halves of the address space (avoids VPP proxy rules)
        sr.rmt_plen = 1;
        SessionRule sr2 = sr;
        sr.set_tag(tag_prefix + kSplitTag);
        out->push_back(sr);
        sr2.rmt_ip[0] = 1 << 7;
        sr2.set_tag(tag_prefix + kSplitTag);
        out->push_back(sr2);
    } else {
        sr.set_tag(tag_prefix);
        out->push_back(sr);
    }
}

std::vector<SessionRule> export_session_rules(const std::vector<ContivRule>& rules, const PodID* pod,
                                              const Bytes& pod_ip, const AppNsIndex& ns) {
    const bool global = pod == nullptr;
    std::vector<SessionRule> out;
    uint32_t ns_index = 0;
    if (!global && !ns.ns_index(*pod, &ns_index)) return out;  // "Unable to get the namespace index"
    const std::string prefix = kSessionRuleTagPrefix;
    for (auto& rule : rules) {
        // allow-all destination rules are the stack's default behaviour
        if (rule.dst_port == 0 && rule.action == kPermit &&
            ((global && rule.src.ip.len == 0) || (!global && rule.dst.ip.len == 0)))
            continue;
        if (!global && rule.dst.ip.len > 0) {  // same source as destination
            int ones = 0, bits = 0;
            mask_size(rule.dst.mask, &ones, &bits);
            if (ones == bits && ip_equal(rule.dst.ip, pod_ip)) continue;
        }
        if (rule.protocol == kANY) {  // the stack carries TCP and UDP only: one rule each
            ContivRule tcp = rule, udp = rule;
            tcp.protocol = kTCP;
            udp.protocol = kUDP;
            convert_contiv_rule(tcp, global, ns_index, prefix + kAnyProtocolTag, &out);
            convert_contiv_rule(udp, global, ns_index, prefix + kAnyProtocolTag, &out);
        } else {
            convert_contiv_rule(rule, global, ns_index, prefix, &out);
        }
    }
    return out;
}

std::vector<TablePtr> import_session_rules(const std::vector<SessionRule>& rules, const AppNsIndex& ns) {
    auto global = std::make_shared<ContivRuleTable>();
    global->type = kGlobal;
    std::map<PodID, TablePtr> locals;
    for (SessionRule rule : rules) {
        ContivRule cr;
        std::string tag = rule.tag_str();
        if (has_suffix(tag, kSplitTag)) {  // merge the two halves of a split rule
            if (rule.rmt_ip[0] != 0) continue;
            rule.rmt_plen = 0;
            tag.resize(tag.size() - std::strlen(kSplitTag));
        }
        if (has_suffix(tag, kAnyProtocolTag)) {  // merge the TCP and UDP copies of an ANY rule
            if (rule.transport_proto == kSrProtoUDP) continue;
            cr.protocol = kANY;
        } else {
            cr.protocol = rule.transport_proto == kSrProtoUDP ? kUDP : kTCP;
        }
        const bool gscope = rule.scope == kScopeGlobal;
        const uint8_t* sip = gscope ? rule.rmt_ip : rule.lcl_ip;
        const uint8_t* dip = gscope ? rule.lcl_ip : rule.rmt_ip;
        const uint8_t splen = gscope ? rule.rmt_plen : rule.lcl_plen;
        const uint8_t dplen = gscope ? rule.lcl_plen : rule.rmt_plen;
        const int iplen = rule.is_ip4 ? 4 : 16;
        if (splen > 0) {
            cr.src.ip = mk(sip, iplen);
            cr.src.mask = cidr_mask(splen, iplen * 8);
        }
        if (dplen > 0) {
            cr.dst.ip = mk(dip, iplen);
            cr.dst.mask = cidr_mask(dplen, iplen * 8);
        }
        cr.src_port = gscope ? rule.rmt_port : rule.lcl_port;
        cr.dst_port = gscope ? rule.lcl_port : rule.rmt_port;
        cr.action = rule.action_index == kSrActionAllow ? kPermit : kDeny;
        if (gscope) {
            global->insert_rule(cr);
            continue;
        }
        PodID pod;
        if (!ns.pod_by_ns_index(rule.appns_index, &pod)) continue;  // "Failed to get pod ..."
        auto& t = locals[pod];
        if (!t) {
            t = std::make_shared<ContivRuleTable>();
            t->type = kLocal;
            t->pods.insert(pod);
        }
        t->insert_rule(cr);
    }
    std::vector<TablePtr> tables{global};
    for (auto& kv : locals) tables.push_back(kv.second);
    return tables;
}

void diff_rules(const ContivRuleTable& a, const ContivRuleTable& b, std::vector<ContivRule>* not_in_b,
                std::vector<ContivRule>* not_in_a) {
    for (auto& r : a.rules)
        if (!b.has_rule(r)) not_in_b->push_back(r);
    for (auto& r : b.rules)
        if (!a.has_rule(r)) not_in_a->push_back(r);
}

// --- session-rule lookup as a first-match ACL ----------------------------------------------------
static std::string v4_cidr(const uint8_t* ip, uint8_t plen) {
    if (plen == 0) return std::string();  // 0/0: any address
    return std::to_string(ip[0]) + "." + std::to_string(ip[1]) + "." + std::to_string(ip[2]) + "." +
           std::to_string(ip[3]) + "/" + std::to_string(plen);
}

ACLPtr session_table_acl(const std::vector<SessionRule>& table, int scope, const std::string& name, std::string* err) {
    std::vector<const SessionRule*> v;
    for (const SessionRule& r : table)
        // the engine classifies IPv4 packets; an IPv4 rule with a prefix longer than 32 bits (a
        // global rule whose ContivRule mixes families, session_rule.go:280-297) matches none
        if (r.is_ip4 && r.lcl_plen <= 32 && r.rmt_plen <= 32) v.push_back(&r);
    auto weight = [](const SessionRule* r) {
        return (int)r->lcl_plen + (int)r->rmt_plen + (r->lcl_port != 0) + (r->rmt_port != 0);
    };
    std::stable_sort(v.begin(), v.end(), [&](const SessionRule* a, const SessionRule* b) {
        const int wa = weight(a), wb = weight(b);
        if (wa != wb) return wa > wb;
        return a->compare(*b, true) < 0;
    });
    const bool global = scope != kScopeLocal;
    auto acl = std::make_shared<ACL>();
    acl->name = name;
    acl->ingress = {name};  // the ACL engine takes ACLs applied to an interface (its own name)
    for (const SessionRule* r : v) {
        // the key port: the remote one of a local table, the local one of the global table
        if ((global && r->rmt_port) || (!global && r->lcl_port)) {
            *err = "session rule port on the side the table does not key on";
            return nullptr;
        }
        if (r->action_index != kSrActionAllow && r->action_index != kSrActionDeny) {
            *err = "session rule action other than ALLOW / DENY";
            return nullptr;
        }
        AclRule a;
        a.action = r->action_index == kSrActionAllow ? kAclPermit : kAclDeny;
        const std::string lcl = v4_cidr(r->lcl_ip, r->lcl_plen), rmt = v4_cidr(r->rmt_ip, r->rmt_plen);
        a.src_network = global ? rmt : lcl;
        a.dst_network = global ? lcl : rmt;
        const uint16_t port = global ? r->lcl_port : r->rmt_port;
        L4Section& s = r->transport_proto == kSrProtoUDP ? a.udp : a.tcp;
        s.present = s.has_src = s.has_dst = true;
        s.src = PortRange{0, 0xFFFF};
        s.dst = port ? PortRange{port, port} : PortRange{0, 0xFFFF};
        acl->rules.push_back(a);
    }
    return acl;
}

// --- VPP session-rule tables ----------------------------------------------------------------

void SessionRuleTables::clear() {
    local.clear();
    global.clear();
    req_count = err_count = 0;
}

// addDelRule (sessionrules_mock.go:344-364): add rejects a rule equal up to the tag, delete
// needs an exact match including the tag
static bool add_del_rule(std::vector<SessionRule>& table, const SessionRule& rule, bool is_add) {
    for (size_t i = 0; i < table.size(); i++) {
        if (rule.compare(table[i], !is_add) == 0) {
            if (is_add) return false;
            table.erase(table.begin() + (long)i);
            return true;
        }
    }
    if (is_add) {
        table.push_back(rule);
        return true;
    }
    return false;
}

int SessionRuleTables::add_del(const SessionRule& rule, bool is_add) {
    req_count++;
    const std::string tag = rule.tag_str();
    if (tag.rfind(tag_prefix, 0) != 0) {
        err_count++;  // "Invalid tag"
        return 1;
    }
    bool ok = rule.scope == kScopeLocal ? add_del_rule(local[rule.appns_index], rule, is_add)
                                        : add_del_rule(global, rule, is_add);
    if (!ok) {
        err_count++;
        return 1;
    }
    return 0;
}

std::vector<SessionRule> SessionRuleTables::dump() {
    req_count += 2;  // session_rules_dump + the control_ping closing the multi-request
    std::vector<SessionRule> out;
    for (auto& kv : local) out.insert(out.end(), kv.second.begin(), kv.second.end());
    out.insert(out.end(), global.begin(), global.end());
    return out;
}

const std::vector<SessionRule>* SessionRuleTables::table(int scope, uint32_t ns_index) const {
    if (scope != kScopeLocal) return &global;
    auto it = local.find(ns_index);
    return it == local.end() ? nullptr : &it->second;
}

// net.ParseCIDR for "a/b", getOneHostSubnet (net.ParseIP + full mask) for a bare address
static bool test_net(const std::string& s, IPNet* n) {
    if (s.find('/') == std::string::npos) {
        Bytes ip;
        if (!parse_ip(s, &ip)) return false;  // the mock would dereference nil here
        Bytes v4;
        n->ip = ip;
        n->mask = to4(ip, &v4) ? cidr_mask(32, 32) : cidr_mask(128, 128);
        return true;
    }
    return parse_cidr(s, n);
}

bool SessionRuleTables::has_rule(int scope, uint32_t ns_index, const std::string& lcl_ip, uint16_t lcl_port,
                                 const std::string& rmt_ip, uint16_t rmt_port, const std::string& proto,
                                 const std::string& action) const {
    const std::vector<SessionRule>* t = table(scope, ns_index);
    if (!t) return false;
    SessionRule r;
    r.lcl_port = lcl_port;
    r.rmt_port = rmt_port;
    r.appns_index = scope == kScopeLocal ? ns_index : 0;
    r.scope = (uint8_t)(scope == kScopeLocal ? kScopeLocal : kScopeGlobal);
    r.transport_proto = proto == "UDP" ? kSrProtoUDP : kSrProtoTCP;  // unknown -> 0
    r.action_index = action == "ALLOW" ? kSrActionAllow : (action == "DENY" ? kSrActionDeny : 0);
    uint8_t is4 = 0;
    for (int side = 0; side < 2; side++) {
        const std::string& s = side ? rmt_ip : lcl_ip;
        if (s.empty()) continue;
        IPNet n;
        if (!test_net(s, &n)) return false;
        uint8_t* dst = side ? r.rmt_ip : r.lcl_ip;
        Bytes v4;
        if (to4(n.ip, &v4)) {
            is4 = 1;
            copy_ip(dst, v4);
        } else {
            copy_ip(dst, to16(n.ip));
        }
        (side ? r.rmt_plen : r.lcl_plen) = (uint8_t)plen_of(n.mask);
    }
    if (lcl_ip.empty() && rmt_ip.empty()) is4 = 1;
    r.is_ip4 = is4;
    for (auto& x : *t)
        if (r.compare(x, false) == 0) return true;
    return false;
}

// --- renderer ------------------------------------------------------------------------------

std::unique_ptr<CfgRendererTxn> VppTcpRenderer::new_txn(bool resync) {
    return std::make_unique<VppTcpRendererTxn>(this, resync);
}

// updateRules (vpptcp_renderer.go:264-316): deletes first, then adds, sent in bursts of the
// channel's buffer size; a burst is sent whole before its replies are read, and the first
// failed reply ends the update.
std::string VppTcpRenderer::update_rules(const std::vector<SessionRule>& add, const std::vector<SessionRule>& remove) {
    std::vector<std::pair<const SessionRule*, bool>> reqs;
    for (auto& r : remove) reqs.push_back({&r, false});
    for (auto& r : add) reqs.push_back({&r, true});
    const size_t burst = chan_buf_size > 0 ? (size_t)chan_buf_size : 100;
    for (size_t i = 0; i < reqs.size();) {
        size_t j = std::min(burst, reqs.size() - i);
        std::vector<int> retvals;
        for (size_t k = 0; k < j; k++) retvals.push_back(vpp->add_del(*reqs[i + k].first, reqs[i + k].second));
        i += j;
        for (int rv : retvals)
            if (rv != 0) return "failed to update VPPTCP session rule";
    }
    return "";
}

void VppTcpRendererTxn::render(const PodID& pod, const IPNet* pod_ip, const std::vector<ContivRule>& ingress,
                               const std::vector<ContivRule>& egress, bool removed) {
    auto cfg = std::make_shared<PodConfig>();
    if (pod_ip) {
        cfg->has_ip = true;
        cfg->pod_ip = *pod_ip;
    }
    cfg->ingress = ingress;
    cfg->egress = egress;
    cfg->removed = removed;
    cache_txn.update(pod, cfg);
}

std::string VppTcpRendererTxn::commit() {
    std::vector<SessionRule> added, removed;
    auto append = [](std::vector<SessionRule>* dst, const std::vector<SessionRule>& src) {
        dst->insert(dst->end(), src.begin(), src.end());
    };
    if (resync) {  // re-synchronise with VPP first
        std::vector<SessionRule> dumped;  // dumpRules: only rules installed by this renderer
        for (auto& x : r->vpp->dump())
            if (x.tag_str().rfind(kSessionRuleTagPrefix, 0) == 0) dumped.push_back(x);
        auto tables = import_session_rules(dumped, *r->ipv4net);
        std::string err = r->cache.resync(tables);
        if (!err.empty()) return err;
        const PodSet txn_pods = cache_txn.updated_pods();
        for (auto& pod : r->cache.all_pods()) {
            if (txn_pods.count(pod)) continue;
            auto cfg = std::make_shared<PodConfig>();
            cfg->removed = true;
            cache_txn.update(pod, cfg);
        }
    }
    for (auto& pod : cache_txn.updated_pods()) {
        PodConfigPtr cfg = cache_txn.pod_config(pod);
        if (cfg->removed) {
            auto it = r->cache.config.find(pod);
            if (it == r->cache.config.end() || !it->second) continue;  // removed pod which does not exist
            cfg = it->second;
        }
        std::vector<ContivRule> new_rules, removed_rules;
        TablePtr orig = r->cache.local_table_by_pod(pod);
        TablePtr next = cache_txn.local_table_by_pod(pod);
        if (!orig && next) new_rules = next->rules;
        if (orig && !next) removed_rules = orig->rules;
        if (orig && next && orig->get_id() != next->get_id()) diff_rules(*orig, *next, &removed_rules, &new_rules);
        // podCfg.PodIP.IP: a config without an IP (e.g. one rebuilt by a resync) has a nil
        // IPNet in the reference; here it compares equal to no rule's network.
        const Bytes pod_ip = cfg->has_ip ? cfg->pod_ip.ip : Bytes();
        append(&added, export_session_rules(new_rules, &pod, pod_ip, *r->ipv4net));
        append(&removed, export_session_rules(removed_rules, &pod, pod_ip, *r->ipv4net));
    }
    TablePtr og = r->cache.global, ng = cache_txn.global_table();
    std::vector<ContivRule> removed_rules, new_rules;
    diff_rules(*og, *ng, &removed_rules, &new_rules);
    append(&added, export_session_rules(new_rules, nullptr, Bytes(), *r->ipv4net));
    append(&removed, export_session_rules(removed_rules, nullptr, Bytes(), *r->ipv4net));
    if (!added.empty() || !removed.empty()) {
        std::string err = r->update_rules(added, removed);
        if (!err.empty()) return err;
    }
    cache_txn.commit();
    return "";
}

}  // namespace pg
