// Host-side policy path: ordering, rule tables, renderer cache, ACL renderer.
// See policy.hpp for the reference file:line map.
#include "policy.hpp"

#include <algorithm>
#include <stdexcept>

namespace pg {

const char* kGlobalTableID = "NODE-GLOBAL";

// ---- ordering (api.go:113-137, utils.go:175-257) --------------------------------
int compare_ints(int a, int b) { return a < b ? -1 : (a > b ? 1 : 0); }

static int bytes_compare(const Bytes& a, const Bytes& b) {  // bytes.Compare
    size_t n = std::min(a.len, b.len);
    int c = std::memcmp(a.b, b.b, n);
    if (c) return c < 0 ? -1 : 1;
    return compare_ints(a.len, b.len);
}

int compare_ipnets(const IPNet& a, const IPNet& b) {
    if (a.ip.len == 0) return b.ip.len == 0 ? 0 : 1;
    if (b.ip.len == 0) return -1;
    Bytes a4, b4;
    bool av4 = to4(a.ip, &a4), bv4 = to4(b.ip, &b4);
    IPNet an, bn;
    if (av4) {
        if (!bv4) return -1;
        an = {a4, a.mask};
    } else {
        an = {to16(a.ip), a.mask};
    }
    if (bv4) {
        if (!av4) return 1;
        bn = {b4, b.mask};
    } else {
        bn = {to16(b.ip), b.mask};
    }
    int a_ones, bits, b_ones, bbits;
    mask_size(an.mask, &a_ones, &bits);
    mask_size(bn.mask, &b_ones, &bbits);
    int common = std::min(a_ones, b_ones);
    Bytes cm = cidr_mask(common, bits);
    Bytes am, bm;
    bool aok = ip_mask(an.ip, cm, &am), bok = ip_mask(bn.ip, cm, &bm);
    Bytes nil;
    if (ip_equal(aok ? am : nil, bok ? bm : nil)) return compare_ints(b_ones, a_ones);
    int c = bytes_compare(bn.mask, an.mask);
    if (c) return c;
    return bytes_compare(an.ip, bn.ip);
}

int compare_ports(uint16_t a, uint16_t b) {
    if (a == b) return 0;
    if (a == 0) return 1;
    if (b == 0) return -1;
    return a < b ? -1 : 1;
}

int ContivRule::compare(const ContivRule& o) const {
    int c = compare_ipnets(src, o.src);
    if (c) return c;
    c = compare_ipnets(dst, o.dst);
    if (c) return c;
    c = compare_ints(protocol, o.protocol);
    if (c) return c;
    if (protocol != kANY) {
        c = compare_ports(src_port, o.src_port);
        if (c) return c;
        c = compare_ports(dst_port, o.dst_port);
        if (c) return c;
    }
    return compare_ints(action, o.action);
}

static const char* action_str(int a) { return a == kDeny ? "DENY" : (a == kPermit ? "PERMIT" : "INVALID"); }
static const char* proto_str(int p) {
    switch (p) {
        case kTCP: return "TCP";
        case kUDP: return "UDP";
        case kOTHER: return "OTHER";
        case kANY: return "ANY";
    }
    return "INVALID";
}

std::string ContivRule::str() const {  // api.go:81-101
    std::string s = src.empty() ? "ANY" : ipnet_string(src);
    std::string d = dst.empty() ? "ANY" : ipnet_string(dst);
    std::string sp = src_port ? std::to_string(src_port) : "ANY";
    std::string dp = dst_port ? std::to_string(dst_port) : "ANY";
    std::string p = proto_str(protocol);
    return std::string("Rule <") + action_str(action) + " " + s + "[" + p + ":" + sp + "] -> " + d + "[" + p + ":" +
           dp + "]>";
}

ContivRule allow_all_rule() {
    ContivRule r;
    r.action = kPermit;
    r.protocol = kANY;
    return r;
}

// ---- ContivRuleTable (cache_api.go:208-347) --------------------------------------
const std::string& ContivRuleTable::get_id() const {
    if (!id.empty()) return id;
    if (type == kGlobal) {
        id = kGlobalTableID;
        return id;
    }
    std::string s = "[";  // fmt.Sprintf("%v", Rules[:NumOfRules])
    for (size_t i = 0; i < rules.size(); i++) {
        if (i) s += " ";
        s += rules[i].str();
    }
    s += "]";
    uint64_t h = 0xcbf29ce484222325ull;  // fnv.New64a
    for (unsigned char c : s) {
        h ^= c;
        h *= 0x100000001b3ull;
    }
    char buf[32];
    std::snprintf(buf, sizeof buf, "%llx", (unsigned long long)h);
    id = buf;
    return id;
}

size_t ContivRuleTable::index_of(const ContivRule& r, bool* present) const {
    size_t lo = 0, hi = rules.size();
    while (lo < hi) {  // sort.Search(n, rule.Compare(Rules[i]) <= 0)
        size_t mid = (lo + hi) / 2;
        if (r.compare(rules[mid]) <= 0) hi = mid;
        else lo = mid + 1;
    }
    *present = lo < rules.size() && r.compare(rules[lo]) == 0;
    return lo;
}

bool ContivRuleTable::insert_rule(const ContivRule& r) {
    bool present;
    size_t idx = index_of(r, &present);
    if (present) return false;
    if (rules.size() == slice_len) slice_len++;
    rules.insert(rules.begin() + idx, r);
    return true;
}

void ContivRuleTable::insert_rules(const std::vector<ContivRule>& rs) {
    if (rs.size() < 64) {
        for (const ContivRule& r : rs) insert_rule(r);
        return;
    }
    // sorted, first of each equal run kept (a later equal rule is "already in"), then merged
    // with the table, skipping rules already there
    std::vector<ContivRule> add(rs);
    std::stable_sort(add.begin(), add.end(), [](const ContivRule& a, const ContivRule& b) { return a.compare(b) < 0; });
    add.erase(std::unique(add.begin(), add.end(), [](const ContivRule& a, const ContivRule& b) { return a.compare(b) == 0; }),
              add.end());
    std::vector<ContivRule> out;
    out.reserve(rules.size() + add.size());
    size_t i = 0, j = 0;
    while (i < rules.size() || j < add.size()) {
        if (j == add.size()) {
            out.push_back(rules[i++]);
            continue;
        }
        if (i == rules.size()) {
            out.push_back(add[j++]);
            continue;
        }
        const int c = rules[i].compare(add[j]);
        if (c < 0) out.push_back(rules[i++]);
        else if (c > 0) out.push_back(add[j++]);
        else out.push_back(rules[i++]), j++;  // already in the table
    }
    rules.swap(out);
    slice_len = std::max(slice_len, rules.size());  // append(nil) once NumOfRules reached len(Rules)
}

bool ContivRuleTable::has_rule(const ContivRule& r) const {
    bool present;
    index_of(r, &present);
    return present;
}

int compare_rule_lists(const std::vector<ContivRule>& a, const std::vector<ContivRule>& b) {
    int c = compare_ints((int)a.size(), (int)b.size());
    if (c) return c;
    for (size_t i = 0; i < a.size(); i++) {
        c = a[i].compare(b[i]);
        if (c) return c;
    }
    return 0;
}

// compareRuleLists(rules, table.Rules) against the untrimmed (nil-padded) slice, as
// lookupIdxByRules does (local_tables.go:233-238). Reaching a nil entry panics in Go.
static int compare_to_padded(const std::vector<ContivRule>& a, const ContivRuleTable& t) {
    int c = compare_ints((int)a.size(), (int)t.slice_len);
    if (c) return c;
    for (size_t i = 0; i < a.size(); i++) {
        if (i >= t.rules.size()) throw std::runtime_error("reference panic: nil rule in compareRuleLists");
        c = a[i].compare(t.rules[i]);
        if (c) return c;
    }
    return 0;
}

// ---- LocalTables (local_tables.go) ----------------------------------------------
size_t LocalTables::idx_by_rules(const std::vector<ContivRule>& rules) const {
    size_t lo = 0, hi = tables.size();
    while (lo < hi) {
        size_t mid = (lo + hi) / 2;
        if (compare_to_padded(rules, *tables[mid]) <= 0) hi = mid;
        else lo = mid + 1;
    }
    return lo;
}

bool LocalTables::insert(const TablePtr& t) {
    if (by_id.count(t->get_id())) return false;
    size_t idx = idx_by_rules(t->rules);
    tables.insert(tables.begin() + idx, t);
    by_id[t->get_id()] = t;
    PodSet pods = t->pods;
    for (auto& pod : pods) {
        unassign_pod(nullptr, pod);
        by_pod[pod] = t;
    }
    return true;
}

bool LocalTables::remove(const TablePtr& t) {
    for (size_t i = 0; i < tables.size(); i++) {
        if (tables[i] == t) {
            tables.erase(tables.begin() + i);
            by_id.erase(t->get_id());
            for (auto& pod : t->pods) by_pod.erase(pod);
            return true;
        }
    }
    return false;
}

void LocalTables::assign_pod(const TablePtr& t, const PodID& pod) {
    unassign_pod(nullptr, pod);
    t->pods.insert(pod);
    by_pod[pod] = t;
}

void LocalTables::unassign_pod(const TablePtr& t, const PodID& pod) {
    if (t) t->pods.erase(pod);
    auto it = by_pod.find(pod);
    if (it != by_pod.end()) {
        if (!t || t == it->second) {
            it->second->pods.erase(pod);
            by_pod.erase(it);
        }
    }
}

TablePtr LocalTables::lookup_by_id(const std::string& id) const {
    auto it = by_id.find(id);
    return it == by_id.end() ? nullptr : it->second;
}

TablePtr LocalTables::lookup_by_rules(const std::vector<ContivRule>& rules) const {
    size_t idx = idx_by_rules(rules);
    if (idx < tables.size() && compare_rule_lists(rules, tables[idx]->rules) == 0) return tables[idx];
    return nullptr;
}

TablePtr LocalTables::lookup_by_pod(const PodID& pod) const {
    auto it = by_pod.find(pod);
    return it == by_pod.end() ? nullptr : it->second;
}

PodSet LocalTables::isolated_pods() const {
    PodSet s;
    for (auto& kv : by_pod)
        if (kv.second->num_rules() > 0) s.insert(kv.first);
    return s;
}

// ---- Ports (ports.go) ---------------------------------------------------------------
namespace {
using Ports = std::set<uint16_t>;
bool ports_has(const Ports& p, uint16_t port) { return p.count(0) || p.count(port); }
bool ports_subset(const Ports& p, const Ports& p2) {
    if (ports_has(p2, 0)) return true;
    if (ports_has(p, 0)) return false;
    for (auto x : p)
        if (!ports_has(p2, x)) return false;
    return true;
}
Ports ports_intersection(const Ports& p, const Ports& p2) {
    if (ports_has(p, 0)) return p2;
    if (ports_has(p2, 0)) return p;
    Ports r;
    for (auto x : p)
        if (ports_has(p2, x)) r.insert(x);
    return r;
}
// getAllowedEgressPorts (egress=true, checks rule.SrcNetwork) / getAllowedIngressPorts
void allowed_ports(const IPNet& ip, const std::vector<ContivRule>& rules, bool egress, Ports* tcp, Ports* udp,
                   bool* any) {
    tcp->clear();
    udp->clear();
    *any = false;
    bool has_deny = false;
    for (auto& r : rules) {
        if (r.action == kDeny) {
            has_deny = true;
            continue;
        }
        const IPNet& n = egress ? r.src : r.dst;
        if (!n.empty() && !contains(n, ip.ip)) continue;
        switch (r.protocol) {
            case kTCP: tcp->insert(r.dst_port); break;
            case kUDP: udp->insert(r.dst_port); break;
            case kANY:
                tcp->insert(0);
                udp->insert(0);
                *any = true;
                break;
        }
    }
    if (!has_deny) {
        *tcp = Ports{0};
        *udp = Ports{0};
        *any = true;
    }
}
}  // namespace

// ---- RendererCache (cache_impl.go) -------------------------------------------------
void RendererCache::flush() {
    local = LocalTables();
    global = std::make_shared<ContivRuleTable>();
    global->type = kGlobal;
    global->get_id();
    config.clear();
}

std::string RendererCache::resync(const std::vector<TablePtr>& tables) {
    std::map<PodID, PodConfigPtr> cfg;
    LocalTables lt;
    auto gt = std::make_shared<ContivRuleTable>();
    gt->type = kGlobal;
    for (auto& t : tables) {
        if (!t) continue;
        if (t->type == kGlobal) {
            gt = t;
            continue;
        }
        if (t->pods.empty()) continue;
        lt.insert(t);
        for (auto& pod : t->pods) {
            if (cfg.count(pod)) return "pod assigned to multiple local tables: " + pod.str();
            cfg[pod] = std::make_shared<PodConfig>();
        }
    }
    local = lt;
    global = gt;
    config = cfg;
    return "";
}

PodSet RendererCache::all_pods() const {
    PodSet s;
    for (auto& kv : config) s.insert(kv.first);
    return s;
}

TablePtr RendererCache::local_table_by_pod(const PodID& pod) const {
    auto t = local.lookup_by_pod(pod);
    if (t && t->num_rules() == 0) return nullptr;
    return t;
}

void RendererCacheTxn::update(const PodID& pod, PodConfigPtr cfg) {
    config[pod] = std::move(cfg);
    up_to_date = false;
}

PodSet RendererCacheTxn::updated_pods() const {
    PodSet s;
    for (auto& kv : config) s.insert(kv.first);
    return s;
}

PodSet RendererCacheTxn::removed_pods() const {
    PodSet s;
    for (auto& kv : config)
        if (kv.second->removed) s.insert(kv.first);
    return s;
}

PodConfigPtr RendererCacheTxn::pod_config(const PodID& pod) const {
    auto it = config.find(pod);
    if (it != config.end()) return it->second;
    auto jt = cache->config.find(pod);
    return jt == cache->config.end() ? nullptr : jt->second;
}

PodSet RendererCacheTxn::all_pods() const {
    PodSet pods = cache->all_pods();
    for (auto& kv : config) {
        if (!kv.second->removed) pods.insert(kv.first);
        else pods.erase(kv.first);
    }
    return pods;
}

PodSet RendererCacheTxn::isolated_pods() {
    if (!up_to_date) refresh();
    PodSet iso = local.isolated_pods();
    for (auto& pod : cache->isolated_pods())
        if (!local.lookup_by_pod(pod)) iso.insert(pod);
    return iso;
}

TablePtr RendererCacheTxn::local_table_by_pod(const PodID& pod) {
    if (!up_to_date) refresh();
    auto t = local.lookup_by_pod(pod);
    if (t && t->num_rules() == 0) return nullptr;
    if (t) return t;
    return cache->local_table_by_pod(pod);
}

TablePtr RendererCacheTxn::global_table() {
    if (!up_to_date) refresh();
    return global ? global : cache->global;
}

std::vector<TxnChange> RendererCacheTxn::changes() {
    if (!up_to_date) refresh();
    std::vector<TxnChange> out;
    for (auto& t : local.tables) {
        auto orig = cache->local.lookup_by_id(t->get_id());
        if (t->num_rules() == 0) continue;
        if (t->pods.empty() && !orig) continue;
        if (orig && t->pods == orig->pods) continue;
        out.push_back({t, orig ? orig->pods : PodSet{}});
    }
    if (global && compare_rule_lists(global->rules, cache->global->rules) != 0) out.push_back({global, PodSet{}});
    return out;
}

void RendererCacheTxn::commit() {
    if (!up_to_date) refresh();
    for (auto& t : local.tables) {
        auto orig = cache->local.lookup_by_id(t->get_id());
        if (orig) {
            if (t->pods.empty()) {
                cache->local.remove(t);
            } else if (t->pods != orig->pods) {
                PodSet op = orig->pods;
                for (auto& pod : op)
                    if (!t->pods.count(pod)) cache->local.unassign_pod(orig, pod);
                for (auto& pod : t->pods)
                    if (!orig->pods.count(pod)) cache->local.assign_pod(orig, pod);
                orig->priv = t->priv;
            }
        } else if (!t->pods.empty()) {
            cache->local.insert(t);
        }
    }
    if (global && compare_rule_lists(global->rules, cache->global->rules) != 0) cache->global = global;
    for (auto& kv : config) {
        if (kv.second->removed) {
            cache->config.erase(kv.first);
            cache->local.unassign_pod(nullptr, kv.first);
        } else {
            cache->config[kv.first] = kv.second;
        }
    }
}

static TablePtr shallow_copy(const ContivRuleTable& src) {
    auto t = std::make_shared<ContivRuleTable>();
    t->type = src.type;
    t->rules = src.rules;
    t->slice_len = src.slice_len;
    t->pods = src.pods;
    t->priv = src.priv;
    return t;
}

void RendererCacheTxn::refresh() {
    PodSet pods = all_pods();
    for (auto& p : removed_pods()) pods.insert(p);
    for (auto& pod : pods) {
        auto cfg = pod_config(pod);
        auto nt = build_local_table(pod, *cfg);
        auto orig = cache->local.lookup_by_pod(pod);
        if (orig && !local.lookup_by_id(orig->get_id())) local.insert(shallow_copy(*orig));
        auto tt = local.lookup_by_rules(nt->rules);
        if (tt) {
            local.assign_pod(tt, pod);
            continue;
        }
        auto ct = cache->local.lookup_by_rules(nt->rules);
        if (ct) {
            auto t = shallow_copy(*ct);
            t->pods.insert(pod);
            local.insert(t);
            continue;
        }
        local.insert(nt);
    }
    rebuild_global();
    up_to_date = true;
}

TablePtr RendererCacheTxn::build_local_table(const PodID& pod, const PodConfig& cfg) {
    auto t = std::make_shared<ContivRuleTable>();
    t->type = kLocal;
    t->pods.insert(pod);
    if (cfg.removed) return t;
    const auto& rules = cache->orientation == kEgressOrientation ? cfg.egress : cfg.ingress;
    t->insert_rules(rules);
    for (auto& sp : all_pods()) install_local_rules(*t, cfg, *pod_config(sp));
    if (t->slice_len > 0) {  // len(table.Rules) > 0 (cache_impl.go:496)
        bool all_matched = false;
        for (auto& r : t->rules)
            if (r.protocol == kANY && r.dst_port == 0 && r.src.empty() && r.dst.empty()) {
                all_matched = true;
                break;
            }
        if (!all_matched) t->insert_rule(allow_all_rule());
    }
    return t;
}

void RendererCacheTxn::install_local_rules(ContivRuleTable& dst, const PodConfig& dcfg, const PodConfig& scfg) {
    bool eg = cache->orientation == kEgressOrientation;
    Ports stcp, sudp, dtcp, dudp;
    bool sany, dany;
    if (eg) {
        allowed_ports(dcfg.pod_ip, scfg.ingress, false, &stcp, &sudp, &sany);
        allowed_ports(scfg.pod_ip, dcfg.egress, true, &dtcp, &dudp, &dany);
    } else {
        allowed_ports(dcfg.pod_ip, scfg.egress, true, &stcp, &sudp, &sany);
        allowed_ports(scfg.pod_ip, dcfg.ingress, false, &dtcp, &dudp, &dany);
    }
    if (sany) return;
    if (dany || !ports_subset(dtcp, stcp) || !ports_subset(dudp, sudp)) {
        const IPNet& sip = scfg.pod_ip;
        dst.remove_by_predicate([&](const ContivRule& r) {
            const IPNet& a = eg ? r.src : r.dst;
            if (a.empty()) return false;
            int ones, bits;
            mask_size(a.mask, &ones, &bits);
            if (ones != bits || !ip_equal(a.ip, sip.ip)) return false;
            return true;
        });
        install_allowed_ports(dst, sip, ports_intersection(dtcp, stcp), kTCP);
        install_allowed_ports(dst, sip, ports_intersection(dudp, sudp), kUDP);
        ContivRule r;
        r.action = kDeny;
        r.protocol = kANY;
        if (eg) r.src = sip;
        else r.dst = sip;
        dst.insert_rule(r);
    }
}

void RendererCacheTxn::install_allowed_ports(ContivRuleTable& dst, const IPNet& src_ip, const std::set<uint16_t>& ports,
                                             int proto) {
    ContivRule t;
    t.action = kPermit;
    t.protocol = proto;
    if (cache->orientation == kEgressOrientation) t.src = src_ip;
    else t.dst = src_ip;
    if (ports.count(0)) {
        dst.insert_rule(t);
        return;
    }
    for (auto p : ports) {
        ContivRule r = t;
        r.dst_port = p;
        dst.insert_rule(r);
    }
}

void RendererCacheTxn::rebuild_global() {
    global = std::make_shared<ContivRuleTable>();
    global->type = kGlobal;
    bool eg = cache->orientation == kEgressOrientation;
    for (auto& pod : all_pods()) {
        auto cfg = pod_config(pod);
        std::vector<ContivRule> rs = eg ? cfg->ingress : cfg->egress;
        for (auto& r : rs) {
            if (eg) r.src = cfg->pod_ip;
            else r.dst = cfg->pod_ip;
        }
        global->insert_rules(rs);
    }
    if (global->num_rules() > 0) global->insert_rule(allow_all_rule());
}

// ---- ACL renderer (acl_renderer.go) ---------------------------------------------------
std::vector<std::string> NodeIfaces::node_output_ifs() const {
    std::vector<std::string> out{host_interconnect};
    if (!main_if.empty()) out.push_back(main_if);
    for (auto& o : other_ifs) out.push_back(o);
    if (!vxlan_bvi.empty()) out.push_back(vxlan_bvi);
    return out;
}

void RendererTxn::render(const PodID& pod, const IPNet* pod_ip, std::vector<ContivRule> ingress,
                         std::vector<ContivRule> egress, bool removed) {
    auto cfg = std::make_shared<PodConfig>();
    if (pod_ip) {
        cfg->has_ip = true;
        cfg->pod_ip = *pod_ip;
    }
    cfg->ingress = std::move(ingress);
    cfg->egress = std::move(egress);
    cfg->removed = removed;
    cache_txn.update(pod, cfg);
}

void RendererTxn::render_interfaces(const PodSet& pods, bool ingress, std::vector<std::string>* in,
                                    std::vector<std::string>* eg) {
    for (auto& pod : pods) {
        std::string name;
        auto it = r->pod_ifs.find(pod);
        if (it != r->pod_ifs.end()) {
            name = it->second;
        } else if (!r->ifaces->if_name(pod, &name)) {
            continue;  // pod removed meanwhile (acl_renderer.go:372-380)
        }
        r->pod_ifs[pod] = name;
        (ingress ? in : eg)->push_back(name);
    }
}

ACLPtr RendererTxn::render_acl(ContivRuleTable& t, bool reflective) {  // acl_renderer.go:295-362
    auto acl = std::make_shared<ACL>();
    acl->name = std::string("contiv-policy-") + (reflective ? "REFLECTION" : t.get_id());
    render_interfaces(t.pods, reflective, &acl->ingress, &acl->egress);
    for (auto& rule : t.rules) {
        AclRule ar;
        if (rule.action == kDeny) ar.action = kAclDeny;
        else if (reflective) ar.action = kAclReflect;
        else ar.action = kAclPermit;
        if (!rule.src.empty()) ar.src_network = ipnet_string(rule.src);
        if (!rule.dst.empty()) ar.dst_network = ipnet_string(rule.dst);
        if (rule.protocol == kTCP || rule.protocol == kUDP) {
            L4Section s;
            s.present = s.has_src = s.has_dst = true;
            s.src.lower = rule.src_port;
            s.src.upper = rule.src_port == 0 ? 0xFFFF : rule.src_port;
            s.dst.lower = rule.dst_port;
            s.dst.upper = rule.dst_port == 0 ? 0xFFFF : rule.dst_port;
            (rule.protocol == kTCP ? ar.tcp : ar.udp) = s;
        }
        acl->rules.push_back(ar);
    }
    t.priv = acl;
    return acl;
}

ACLPtr RendererTxn::reflective_acl() {  // acl_renderer.go:253-273
    ContivRuleTable t;
    t.rules = {allow_all_rule()};
    t.slice_len = 1;
    t.pods = cache_txn.isolated_pods();
    auto acl = render_acl(t, true);
    if (cache_txn.global_table()->num_rules() > 0)
        for (auto& i : r->ifaces->node_output_ifs()) acl->ingress.push_back(i);
    return acl;
}

std::string RendererTxn::commit() {  // acl_renderer.go:138-217
    if (resync) return commit_resync();
    bool has_reflective = r->cache.global->num_rules() != 0 || !r->cache.isolated_pods().empty();
    auto chs = cache_txn.changes();
    if (chs.empty()) {
        cache_txn.commit();
        return "";
    }
    AclOps ops;
    TablePtr gt;
    for (auto& ch : chs) {
        if (ch.table->type == kGlobal) {
            gt = ch.table;
            continue;
        }
        if (ch.previous_pods.empty()) {
            auto acl = render_acl(*ch.table, false);
            ops[acl->name] = acl;
        } else if (!ch.table->pods.empty()) {
            auto acl = std::make_shared<ACL>(*ch.table->priv);  // proto.Clone
            acl->ingress.clear();
            acl->egress.clear();
            render_interfaces(ch.table->pods, false, &acl->ingress, &acl->egress);
            ops[acl->name] = acl;
        } else {
            ops[ch.table->priv->name] = nullptr;
        }
    }
    bool gt_added_or_deleted = false;
    if (gt) {
        auto gacl = render_acl(*gt, false);
        if (gt->num_rules() == 0) {
            ops[gacl->name] = nullptr;
            gt_added_or_deleted = true;
        } else {
            gacl->egress = r->ifaces->node_output_ifs();
            ops[gacl->name] = gacl;
            if (r->cache.global->num_rules() == 0) gt_added_or_deleted = true;
        }
    }
    if (gt_added_or_deleted || cache_txn.isolated_pods() != r->cache.isolated_pods()) {
        auto racl = reflective_acl();
        if (racl->ingress.empty()) {
            if (has_reflective) ops[racl->name] = nullptr;
        } else {
            ops[racl->name] = racl;
        }
    }
    std::string err = r->apply(r->engine, false, ops);
    cache_txn.commit();
    return err;
}

std::string RendererTxn::commit_resync() {  // acl_renderer.go:220-250
    r->cache.flush();
    r->pod_ifs.clear();
    AclOps ops;
    for (auto& ch : cache_txn.changes()) {
        auto acl = render_acl(*ch.table, false);
        if (ch.table->type == kGlobal) acl->egress = r->ifaces->node_output_ifs();
        ops[acl->name] = acl;
    }
    auto racl = reflective_acl();
    if (!racl->ingress.empty()) ops[racl->name] = racl;
    std::string err = r->apply(r->engine, true, ops);
    cache_txn.commit();
    return err;
}

}  // namespace pg
