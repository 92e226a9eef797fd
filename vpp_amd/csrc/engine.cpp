// Device ACL engine: ACL install semantics + the table compiler.
#include "engine.hpp"

#include "classify.hpp"

#include <algorithm>
#include <mutex>
#include <set>

#include "../../include/policygpu.h"

namespace pg {

// ---- tuning --------------------------------------------------------------------------------
namespace {
std::mutex& defaults_mu() {
    static std::mutex mu;
    return mu;
}
Tuning& defaults() {
    static Tuning t;
    return t;
}
}  // namespace

Tuning default_tuning() {
    std::lock_guard<std::mutex> lk(defaults_mu());
    return defaults();
}

int default_tuning_set(const std::string& key, int value) {
    std::lock_guard<std::mutex> lk(defaults_mu());
    return tuning_set(defaults(), key, value);
}

namespace {
struct Knob {
    const char* key;
    uint32_t Tuning::*field;
    int lo, hi;
    bool compiler;
    bool allowed(int v) const;
};
const Knob kKnobs[] = {
    {"root_bits_max", &Tuning::root_bits_max, 4, 16, true},
    {"lc_lds", &Tuning::lc_lds, 0, 1 << 30, true},
    {"lc_dense12", &Tuning::lc_dense12, 1, 1 << 30, true},
    {"lc_max_stride", &Tuning::lc_max_stride, 12, 18, true},
    {"lc_root_bits", &Tuning::lc_root_bits, 4, 14, true},
    {"pair", &Tuning::pair, 0, 2, true},
    {"node_build", &Tuning::node_build, 0, 1, true},
    {"node_root_bits", &Tuning::node_root_bits, 4, 16, true},
    {"node_key_root_bits", &Tuning::node_key_root_bits, 2, 10, true},
    {"node_common", &Tuning::node_common, 0, 1, true},
    {"fd", &Tuning::fd, 0, 1, true},
    {"candi", &Tuning::candi, 0, 1, true},
    {"candi_window_bits", &Tuning::candi_window_bits, 0, 13, true},
    {"candi_window_root_bits", &Tuning::candi_window_root_bits, 4, 14, true},
    {"cross_max_rules", &Tuning::cross_max_rules, 0, 1 << 24, true},
    {"node_hist_cells", &Tuning::node_hist_cells, 0, 8192, false},
    {"node_list_words", &Tuning::node_list_words, 0, 16384, true},
    {"node_uniform", &Tuning::node_uniform, 0, 1, true},
    {"node_list_table", &Tuning::node_list_table, 0, 1, true},
    {"blocks_per_cu", &Tuning::blocks_per_cu, 0, 64, false},
    {"stage_max_words", &Tuning::stage_max_words, 0, 36864, false},
    {"node_stage_max_words", &Tuning::node_stage_max_words, 0, 36864, false},
    {"stage_root_max_words", &Tuning::stage_root_max_words, 0, 36864, false},
    {"node_path", &Tuning::node_path, 0, 1, false},
    {"node_common_lds_max", &Tuning::node_common_lds_max, 0, 160 << 10, false},
    {"block_stage", &Tuning::block_stage, 0, 1024, false},
    {"hist_window", &Tuning::hist_window, 1, 16382, false},
    {"launch_max_tuples", &Tuning::launch_max_tuples, 0, (1 << 30) - 64, false},
};
bool Knob::allowed(int v) const {
    if (field == &Tuning::lc_max_stride) return v == 12 || v == 16 || v == 18;
    if (field == &Tuning::block_stage) return v == 0 || v == 256 || v == 512 || v == 1024;
    if (field == &Tuning::launch_max_tuples) return v % 64 == 0;  // (pieces stay vector-aligned)
    return true;
}
}  // namespace

int tuning_set(Tuning& t, const std::string& key, int value, bool* compiler) {
    for (const Knob& k : kKnobs) {
        if (key != k.key) continue;
        if (value < k.lo || value > k.hi || !k.allowed(value)) return -1;
        t.*(k.field) = (uint32_t)value;
        if (compiler) *compiler = k.compiler;
        return 0;
    }
    return -1;
}

int tuning_get(const Tuning& t, const std::string& key, int* value) {
    for (const Knob& k : kKnobs) {
        if (key != k.key) continue;
        if (value) *value = (int)(t.*(k.field));
        return 0;
    }
    return -1;
}

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

// ---- counters across recompiles -----------------------------------------------------------
uint64_t acl_rules_hash(const ACL& acl) {
    uint64_t h = 1469598103934665603ull;
    auto mix = [&](const void* p, size_t n) {
        for (size_t i = 0; i < n; i++) h = (h ^ ((const uint8_t*)p)[i]) * 1099511628211ull;
    };
    auto u32 = [&](uint32_t v) { mix(&v, 4); };
    auto str = [&](const std::string& s) { u32((uint32_t)s.size()), mix(s.data(), s.size()); };
    auto l4 = [&](const L4Section& s) {
        u32(s.present | s.has_src << 1 | s.has_dst << 2);
        u32(s.src.lower), u32(s.src.upper), u32(s.dst.lower), u32(s.dst.upper);
    };
    u32((uint32_t)acl.rules.size());
    for (const AclRule& r : acl.rules) {
        u32((uint32_t)r.action);
        u32(r.has_macip | r.has_ip_rule << 1 | r.has_ip << 2 | r.has_icmp << 3);
        str(r.src_network), str(r.dst_network);
        l4(r.tcp), l4(r.udp);
    }
    return h;
}

std::vector<uint32_t> slot_remap(const SlotLayout& from, const SlotLayout& to, bool* identity) {
    std::vector<uint32_t> m(to.slots, kNoSlot);
    for (const auto& kv : to.tabs) {
        const auto it = from.tabs.find(kv.first);
        if (it == from.tabs.end()) continue;
        const SlotLayout::Tab &a = it->second, &b = kv.second;
        if (a.n != b.n || a.rules_hash != b.rules_hash) continue;  // changed: starts at zero
        for (uint32_t r = 0; r < b.n; r++) m[b.base + r] = a.base + r;
        m[b.dflt] = a.dflt;
    }
    m[to.noacl] = from.noacl;
    m[to.unresolved] = from.unresolved;
    if (identity) {
        bool id = from.slots == to.slots;
        for (uint32_t s = 0; id && s < to.slots; s++) id = m[s] == s;
        *identity = id;
    }
    return m;
}

// a snapshot's counts carried into layout L (the slots of changed / new ACLs read zero)
static void remap_snapshot(CounterSnapshot& s, const std::shared_ptr<const SlotLayout>& L) {
    if (!s.layout || s.layout == L) return;
    const std::vector<uint32_t> m = slot_remap(*s.layout, *L);
    std::vector<uint64_t> v(L->slots, 0);
    for (uint32_t i = 0; i < L->slots; i++)
        if (m[i] != kNoSlot && m[i] < s.v.size()) v[i] = s.v[m[i]];
    s.v.swap(v);
    s.layout = L;
}

// ---- Engine ------------------------------------------------------------------------------
Engine::~Engine() {
    if (comm) dev_comm_destroy(comm);
    if (comm_check) dev_release(comm_check);
    if (reduced) dev_release(reduced);
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
    touch();
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
    touch();
    return "";
}

std::string Engine::apply_txn(bool resync, const AclOps& ops) {  // aclengine_mock.go:151-228
    committed++;
    touch();
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

int Engine::sync() {
    if (!dirty && cur) return PG_OK;
    if (!compiled) compile();
    HostTableSet& h = host;
    std::string err;
    DeviceBuffers* nb = dev_upload(h, &err);
    if (!nb) {
        last_error = "upload: " + err;
        return PG_EIO;
    }
    // waits for the launches that read the old set -- among them every launch that counted into
    // `counters` (pg_classify, pg_reset_counters record their use of it), so they are final
    if (cur) dev_free(cur);
    cur = nb;
    const size_t slots = dev_view(cur).n_slots;
    // the counts of unchanged ACLs carry over to their new slots (slot_remap); changed and new
    // ones start at zero. The device counters keep their address while the slot count holds.
    const bool carry = counters && counted_layout;  // (else: nothing counted yet)
    bool identity = false;
    std::vector<uint32_t> map;
    if (carry) map = slot_remap(*counted_layout, *layout, &identity);
    // A failed step leaves the counters in the layout they were counted in (counted_layout and
    // the buffer unchanged: the next sync carries them over again) -- except a remap in place
    // that failed part-way, after which the counts restart
    if (!(carry && identity)) {
        unsigned long long* from = nullptr;  // the counts to carry: the old buffer or a copy of it
        unsigned long long* into = counters;  // where the new layout's counts go
        if (carry && slots == counter_slots) {  // remap through a copy, into the same buffer
            from = (unsigned long long*)dev_alloc(counter_slots * 8, &err);
            if (!from || dev_copy_d2d_async(from, counters, counter_slots * 8, nullptr, &err) != 0 ||
                dev_stream_sync(nullptr, &err) != 0) {
                dev_release(from);
                last_error = err;
                return PG_ENOMEM;
            }
        } else if (slots != counter_slots || !counters) {
            into = (unsigned long long*)dev_alloc(slots * sizeof(unsigned long long), &err);
            if (!into) {
                last_error = err;
                return PG_ENOMEM;
            }
            if (carry) from = counters;
        }
        int rc = from ? dev_counters_remap(into, from, map.data(), slots, &err)
                      : dev_memset(into, 0, slots * 8, nullptr, &err);
        if (rc == 0) rc = dev_stream_sync(nullptr, &err);
        if (rc != 0) {
            if (into != counters) {
                dev_release(into);  // the old buffer, in its old layout, stays
            } else {
                dev_release(from);
                counted_layout = nullptr;  // in place, part-way: the counts restart
            }
            last_error = err;
            return PG_EIO;
        }
        if (into != counters) {  // the new buffer replaces the old one
            dev_release(counters);
            counters = into;
            counter_slots = slots;
        } else {
            dev_release(from);
        }
    }
    counted_layout = layout;
    dirty = false;
    return PG_OK;
}

// ACLs -> host image of the device table set (rules, blobs, interface maps); no GPU needed.
void Engine::compile() {
    host = HostTableSet();
    HostTableSet& h = host;
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
    const uint32_t NR = (uint32_t)h.rules.size();
    h.blob_words.assign(h.tabs.size(), 0);
    h.blob_prefix.assign(h.tabs.size(), 0);
    std::vector<TableAnalysis*> an(h.tabs.size(), nullptr);
    for (size_t t = 0; t < h.tabs.size(); t++) {
        DevTable& hdr = h.tabs[t];
        std::vector<uint32_t> blob;
        hdr.dflt = (kActDeny << 30) | (NR + (uint32_t)t);
        bool ok = build_fast_table(h.rules.data() + hdr.rule_base, hdr.n_rules, hdr.rule_base, NR + (uint32_t)t, blob,
                                   1ull << 22, tune, &an[t]);
        // fewer dependent loads in dense subtrees
        if (ok && (blob.size() > kStageBlobWords || (tune.lc_lds && blob.size() >= tune.lc_lds))) {
            std::vector<uint32_t> lc;
            if (build_fast_table(h.rules.data() + hdr.rule_base, hdr.n_rules, hdr.rule_base, NR + (uint32_t)t, lc,
                                 1ull << 22, tune, nullptr, true) &&
                (blob.size() > kStageBlobWords || lc.size() <= kStageBlobWords))
                blob.swap(lc);
        }
        // dst-independent CROSS tables: the fixed-depth form (no dst stream, no per-lane
        // branches in the walk); staged whole in LDS when it fits, else its prefix
        bool dst_free = true;  // no rule tests dst (ANY-protocol packets included)
        for (uint32_t r = 0; r < hdr.n_rules; r++) dst_free &= h.rules[hdr.rule_base + r].dmask == 0;
        if (ok && tune.fd && an[t] && dst_free) {
            std::vector<uint32_t> fd;
            if (build_fd_blob(*an[t], (kActDeny << 30) | (NR + (uint32_t)t), tune, fd, 1u << 22, tune.stage_max_words)) {
                blob.swap(fd);
                h.blob_prefix[t] = blob[9];
            }
        }
        ok = ok && (uint64_t)blob.size() * 4u < kMaxLoaderBytes;  // (the loaders' 32-bit byte offsets)
        if (ok) {
            while (blob.size() % 4) blob.push_back(0);
            hdr.blob_off = (uint32_t)h.blobs.size();
            hdr.fsk = blob[0] | (blob[3] << 8) | (blob[5] << 16) | (dst_free ? kFlagDstFree : 0u);
            hdr.kroot = blob[4];
            hdr.xoff = blob[6];
            hdr.nkc = blob[7];
            h.blob_words[t] = (uint32_t)blob.size();
            h.blobs.insert(h.blobs.end(), blob.begin(), blob.end());
        } else {
            hdr.fsk = kFlagLinear;  // linear scan fallback
        }
    }
    uint32_t T = (uint32_t)h.tabs.size();
    for (uint32_t t = 0; t < T; t++) slot_table.push_back((int32_t)t), slot_rule.push_back(-1);
    slot_table.push_back(-1), slot_rule.push_back(-1);  // no ACL
    slot_table.push_back(-1), slot_rule.push_back(-2);  // unresolved interface
    layout_hash = 1469598103934665603ull;
    auto fnv = [&](const void* p, size_t n) {
        for (size_t i = 0; i < n; i++) layout_hash = (layout_hash ^ ((const uint8_t*)p)[i]) * 1099511628211ull;
    };
    for (uint32_t t = 0; t < T; t++) {
        fnv(table_names[t].data(), table_names[t].size() + 1);
        fnv(&h.tabs[t].n_rules, 4);
    }
    {
        auto L = std::make_shared<SlotLayout>();
        L->gen = ++layout_gen;
        for (uint32_t t = 0; t < T; t++)
            L->tabs[table_names[t]] = SlotLayout::Tab{h.tabs[t].rule_base, h.tabs[t].n_rules, NR + t,
                                                      acl_rules_hash(*by_name.at(table_names[t]))};
        L->noacl = NR + T;
        L->unresolved = NR + T + 1;
        L->slots = NR + T + 2;
        layout = std::move(L);
        // the host snapshots follow (the device counters follow at the upload, sync()): a gauge
        // keyed by (ACL name, rule index) reads the same count before and after a recompile that
        // left its ACL unchanged
        std::lock_guard<std::mutex> lk(snap_mu);
        remap_snapshot(snap_local, layout);
        remap_snapshot(snap_cluster, layout);
    }
    layout_gen_pub.store(layout_gen, std::memory_order_release);

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
    const int32_t node_ifc = nif.empty() ? -1 : iface_index[nif];
    if (node_ifc >= 0) h.node_in = h.ifaces[2 * node_ifc], h.node_out = h.ifaces[2 * node_ifc + 1];
    // end point of every other address: the node-output interface, kind "not a pod"
    h.node_if = node_ifc >= 0 ? node_ifc | kEndInet : -1;
    // the last rule of the inbound ACL the most interfaces share (at least two; the renderer's
    // reflective ACL): CONN kernels count it in a register (device.hpp slot_hot_in)
    {
        std::vector<uint32_t> uses(h.tabs.size(), 0);
        for (size_t i = 0; i + 1 < h.ifaces.size(); i += 2)
            if (h.ifaces[i] >= 0 && (size_t)h.ifaces[i] < uses.size()) uses[h.ifaces[i]]++;
        h.slot_hot_in = 0xFFFFFFFFu;
        uint32_t best = 1;
        for (size_t t = 0; t < uses.size(); t++)
            if (uses[t] > best && h.tabs[t].n_rules)
                best = uses[t], h.slot_hot_in = h.tabs[t].rule_base + h.tabs[t].n_rules - 1u;
    }
    // registered pod IP -> {interface, its inbound / outbound tables}: a local pod's TAP (-2 =
    // no known interface: unresolvable, FAILURE), a pod on another node the node-output
    // interface marked kEndRemote (aclengine_mock.go:291-299, 343-347, 388-392)
    struct Ent {
        uint32_t ip;
        int32_t ifc, tin, tout;
    };
    std::vector<Ent> ipmap;
    for (auto& kv : pods) {
        Bytes v4;
        if (!to4(kv.second.ip, &v4)) continue;
        if (kv.second.another_node) {  // (no node-output interface: unresolvable like any other address)
            if (node_ifc >= 0) ipmap.push_back(Ent{ipv4_u32(v4), node_ifc | kEndRemote, h.node_in, h.node_out});
            continue;
        }
        std::string ifn;
        Ent e{ipv4_u32(v4), -2, -1, -1};
        if (ifaces.if_name(kv.first, &ifn)) {
            e.ifc = iface_index[ifn];
            e.tin = h.ifaces[2 * e.ifc];
            e.tout = h.ifaces[2 * e.ifc + 1];
        }
        ipmap.push_back(e);
    }
    uint32_t cap = 16;
    while (cap < 2 * ipmap.size() + 16) cap <<= 1;
    h.iphash.assign(4 * cap, 0xFFFFFFFFu);
    h.iphash_mask = cap - 1;
    for (auto& e : ipmap) {
        uint32_t s = hash_ip(e.ip) & h.iphash_mask;
        while (h.iphash[4 * s + 1] != 0xFFFFFFFFu && h.iphash[4 * s] != e.ip) s = (s + 1) & h.iphash_mask;
        h.iphash[4 * s] = e.ip;
        h.iphash[4 * s + 1] = (uint32_t)e.ifc;
        h.iphash[4 * s + 2] = (uint32_t)e.tin;
        h.iphash[4 * s + 3] = (uint32_t)e.tout;
    }
    // node classifier for the PERPOD / CONN modes (same end points as the iphash)
    std::vector<NodePod> np;
    for (auto& e : ipmap) np.push_back(NodePod{e.ip, e.ifc, e.tin, e.tout});
    build_node(h, an, np, NodePod{0, h.node_if, h.node_in, h.node_out}, tune);
    for (TableAnalysis* a : an) free_analysis(a);
    compiled = true;
}

}  // namespace pg
