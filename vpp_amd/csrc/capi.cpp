// extern "C" boundary (include/policygpu.h). Converts the flat C structs into the host
// model, forwards to the renderer / engine and maps failures to PG_* codes + last_error.
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <stdexcept>

#include "capi_internal.hpp"
#include "classify.hpp"

using namespace pg;

IPNet pg::to_ipnet(const pg_ipnet& n) {
    IPNet r;
    if (n.family == 4) {
        r.ip = mk(n.addr, 4);
        r.mask = cidr_mask(n.prefix_len, 32);
    } else if (n.family == 6) {
        r.ip = mk(n.addr, 16);
        r.mask = cidr_mask(n.prefix_len, 128);
    }
    return r;
}

pg_ipnet pg::to_pg_ipnet(const IPNet& n) {
    pg_ipnet v{};
    if (n.ip.len == 0) return v;
    int ones = 0, bits = 0;
    mask_size(n.mask, &ones, &bits);
    Bytes v4;
    if (to4(n.ip, &v4) && bits == 32) {
        v.family = 4;
        std::memcpy(v.addr, v4.b, 4);
    } else {
        v.family = 6;
        const Bytes b16 = to16(n.ip);
        std::memcpy(v.addr, b16.b, 16);
    }
    v.prefix_len = (uint8_t)(ones < 0 ? 0 : ones);
    return v;
}

namespace {

ContivRule to_rule(const pg_contiv_rule& c) {
    ContivRule r;
    r.action = c.action;
    r.protocol = c.protocol;
    r.src_port = c.src_port;
    r.dst_port = c.dst_port;
    r.src = to_ipnet(c.src);
    r.dst = to_ipnet(c.dst);
    return r;
}

std::string sv(const char* s) { return s ? std::string(s) : std::string(); }

L4Section to_l4(const pg_l4& l) {
    L4Section s;
    s.present = l.present;
    s.has_src = l.has_src_range;
    s.has_dst = l.has_dst_range;
    s.src = {l.src_range.lower_port, l.src_range.upper_port};
    s.dst = {l.dst_range.lower_port, l.dst_range.upper_port};
    return s;
}

ACLPtr to_acl(const pg_acl& a) {
    auto acl = std::make_shared<ACL>();
    acl->name = sv(a.name);
    for (size_t i = 0; i < a.n_rules; i++) {
        const pg_acl_rule& x = a.rules[i];
        AclRule r;
        r.action = x.action;
        r.has_macip = x.has_macip_rule;
        r.has_ip_rule = x.has_ip_rule;
        r.has_ip = x.has_ip;
        r.has_icmp = x.has_icmp;
        r.src_network = sv(x.src_network);
        r.dst_network = sv(x.dst_network);
        r.tcp = to_l4(x.tcp);
        r.udp = to_l4(x.udp);
        acl->rules.push_back(r);
    }
    for (size_t i = 0; i < a.n_ingress; i++) acl->ingress.push_back(sv(a.ingress[i]));
    for (size_t i = 0; i < a.n_egress; i++) acl->egress.push_back(sv(a.egress[i]));
    return acl;
}

int fail(pg_ctx* c, int code, const std::string& msg) {
    if (c) c->eng.last_error = msg;
    return code;
}

// Every entry point that touches the device makes the context's GPU current for the call and
// restores the caller's afterwards: contexts on different GPUs can share a process, and a cgo
// caller's goroutine may move between OS threads between two calls.
struct DeviceGuard {
    int prev = -1, dev = 0;
    bool ok = true;
    std::string err;
    explicit DeviceGuard(const pg_ctx* c) : dev(c->eng.device) {
        if (dev_get_device(&prev) != 0) prev = -1;
        if (prev != dev) ok = dev_set_device(dev, &err) == 0;
    }
    ~DeviceGuard() {
        if (prev >= 0 && prev != dev) (void)dev_set_device(prev, nullptr);
    }
};
#define DEVICE_GUARD(ctx)                                             \
    DeviceGuard guard_(ctx);                                          \
    if (!guard_.ok) return fail(ctx, PG_EIO, "set device: " + guard_.err)

std::string json_escape(const std::string& s) {
    std::string o;
    for (char ch : s) {
        if (ch == '"' || ch == '\\') o += '\\';
        o += ch;
    }
    return o;
}

uint32_t pkt_key_host(int proto, uint16_t port) {
    switch (proto) {
        case kTCP: return port;
        case kUDP: return kKeyUDP | port;
        case kOTHER: return kKeyOTHER;
    }
    return kKeyANY;
}

}  // namespace

#define GUARD_BEGIN try {
#define GUARD_END(ctx)                                         \
    }                                                          \
    catch (const std::exception& e) {                          \
        return fail(ctx, PG_EFAULT, e.what());                 \
    }                                                          \
    catch (...) {                                              \
        return fail(ctx, PG_EFAULT, "unknown C++ exception");  \
    }

extern "C" {

const char* pg_version(void) { return "policygpu 0.1 (gfx950)"; }

pg_ctx* pg_create(int hip_device) {
    if (hip_device < 0) return nullptr;
    auto* c = new (std::nothrow) pg_ctx();
    if (!c) return nullptr;
    c->eng.device = hip_device;  // made current by every device-touching call (DeviceGuard)
    return c;
}

void pg_destroy(pg_ctx* ctx) {
    if (!ctx) return;
    const Engine& E = ctx->eng;
    if (E.cur || E.counters || E.comm || E.comm_check) {  // device resources: free them on their GPU
        DeviceGuard g(ctx);
        delete ctx;
        return;
    }
    delete ctx;
}

// process defaults: contexts created afterwards start from them
int pg_set_tuning(const char* key, int value) {
    if (!key) return PG_EINVAL;
    return default_tuning_set(key, value) == 0 ? PG_OK : PG_EINVAL;
}

int pg_ctx_set_tuning(pg_ctx* ctx, const char* key, int value) {
    if (!ctx || !key) return PG_EINVAL;
    bool compiler = false;
    if (tuning_set(ctx->eng.tune, key, value, &compiler) != 0)
        return fail(ctx, PG_EINVAL, std::string("bad tuning key or value: ") + key);
    if (compiler) ctx->eng.touch();  // recompiled (and re-uploaded) on the next use
    return PG_OK;
}

int pg_ctx_get_tuning(const pg_ctx* ctx, const char* key, int* value) {
    if (!key || !value) return PG_EINVAL;
    return tuning_get(ctx ? ctx->eng.tune : default_tuning(), key, value) == 0 ? PG_OK : PG_EINVAL;
}

int pg_ctx_device(const pg_ctx* ctx) { return ctx ? ctx->eng.device : PG_EINVAL; }

const char* pg_last_error(const pg_ctx* ctx) { return ctx ? ctx->eng.last_error.c_str() : "null context"; }

int pg_set_pod_if_name(pg_ctx* ctx, const char* ns, const char* name, const char* if_name) {
    if (!ctx || !ns || !name || !if_name) return PG_EINVAL;
    ctx->eng.ifaces.pod_if[PodID{ns, name}] = if_name;
    ctx->eng.touch();
    return PG_OK;
}
int pg_set_host_interconnect_if_name(pg_ctx* ctx, const char* n) {
    if (!ctx) return PG_EINVAL;
    ctx->eng.ifaces.host_interconnect = sv(n);
    ctx->eng.touch();
    return PG_OK;
}
int pg_set_main_interface_name(pg_ctx* ctx, const char* n) {
    if (!ctx) return PG_EINVAL;
    ctx->eng.ifaces.main_if = sv(n);
    ctx->eng.touch();
    return PG_OK;
}
int pg_set_other_vpp_interfaces(pg_ctx* ctx, const char* const* names, size_t n) {
    if (!ctx) return PG_EINVAL;
    ctx->eng.ifaces.other_ifs.clear();
    for (size_t i = 0; i < n; i++) ctx->eng.ifaces.other_ifs.push_back(sv(names[i]));
    ctx->eng.touch();
    return PG_OK;
}
int pg_set_vxlan_bvi_if_name(pg_ctx* ctx, const char* n) {
    if (!ctx) return PG_EINVAL;
    ctx->eng.ifaces.vxlan_bvi = sv(n);
    ctx->eng.touch();
    return PG_OK;
}
int pg_register_pod(pg_ctx* ctx, const char* ns, const char* name, const char* ip, int another_node) {
    if (!ctx || !ns || !name || !ip) return PG_EINVAL;
    PodReg reg;
    parse_ip(ip, &reg.ip);  // net.ParseIP; nil on failure like the reference
    reg.another_node = another_node != 0;
    ctx->eng.pods[PodID{ns, name}] = reg;
    ctx->eng.touch();
    return PG_OK;
}

pg_renderer* pg_renderer_new(pg_ctx* ctx, int orientation) {
    if (!ctx) return nullptr;
    auto* r = new (std::nothrow) pg_renderer();
    if (!r) return nullptr;
    r->ctx = ctx;
    r->r.reset(new Renderer(&ctx->eng.ifaces, &ctx->eng, engine_apply_cb,
                            orientation == PG_ORIENT_INGRESS ? kIngressOrientation : kEgressOrientation));
    return r;
}
void pg_renderer_free(pg_renderer* r) { delete r; }

pg_txn* pg_renderer_new_txn(pg_renderer* r, int resync) {
    if (!r) return nullptr;
    auto* t = new (std::nothrow) pg_txn();
    if (!t) return nullptr;
    t->ctx = r->ctx;
    t->t.reset(new RendererTxn(r->r.get(), resync != 0));
    return t;
}

int pg_txn_render(pg_txn* txn, const char* ns, const char* name, const pg_ipnet* pod_ip,
                  const pg_contiv_rule* ingress, size_t n_in, const pg_contiv_rule* egress, size_t n_eg, int removed) {
    if (!txn || !ns || !name) return PG_EINVAL;
    GUARD_BEGIN
    std::vector<ContivRule> in, eg;
    for (size_t i = 0; i < n_in; i++) in.push_back(to_rule(ingress[i]));
    for (size_t i = 0; i < n_eg; i++) eg.push_back(to_rule(egress[i]));
    IPNet ip;
    const IPNet* pip = nullptr;
    if (pod_ip && pod_ip->family != 0) {
        ip = to_ipnet(*pod_ip);
        pip = &ip;
    }
    txn->t->render(PodID{ns, name}, pip, std::move(in), std::move(eg), removed != 0);
    return PG_OK;
    GUARD_END(txn->ctx)
}

int pg_txn_commit(pg_txn* txn) {
    if (!txn) return PG_EINVAL;
    pg_ctx* ctx = txn->ctx;
    int rc = PG_OK;
    try {
        std::string e = txn->t->commit();
        if (!e.empty()) rc = fail(ctx, PG_EFAULT, e);
    } catch (const std::exception& ex) {
        rc = fail(ctx, PG_EFAULT, ex.what());
    }
    delete txn;
    return rc;
}
void pg_txn_free(pg_txn* txn) { delete txn; }

int pg_apply_txn(pg_ctx* ctx, int resync, const pg_acl_op* ops, size_t n) {
    if (!ctx) return PG_EINVAL;
    GUARD_BEGIN
    static const std::string prefix = "config/vpp/acls/v2/acl/";
    AclOps m;
    for (size_t i = 0; i < n; i++) {
        std::string key = sv(ops[i].key);
        if (key.compare(0, prefix.size(), prefix) != 0) return fail(ctx, PG_EFAULT, "non-ACL changed in txn");
        std::string name = key.substr(prefix.size());
        if (ops[i].value) {
            m[name] = to_acl(*ops[i].value);
        } else {
            if (resync) return fail(ctx, PG_EFAULT, "failed to cast ACL value");
            m[name] = nullptr;
        }
    }
    std::string e = ctx->eng.apply_txn(resync != 0, m);
    if (!e.empty()) return fail(ctx, PG_EFAULT, e);
    return PG_OK;
    GUARD_END(ctx)
}

int pg_num_acls(pg_ctx* ctx) { return ctx ? (int)ctx->eng.by_name.size() : PG_EINVAL; }
int pg_num_acl_changes(pg_ctx* ctx) { return ctx ? ctx->eng.changes : PG_EINVAL; }
int pg_num_committed_txns(pg_ctx* ctx) { return ctx ? ctx->eng.committed : PG_EINVAL; }

int pg_acl_json(pg_ctx* ctx, const char* acl_name, char* buf, size_t cap) {
    if (!ctx || !acl_name) return PG_EINVAL;
    auto it = ctx->eng.by_name.find(acl_name);
    if (it == ctx->eng.by_name.end()) return PG_ENOENT;
    const ACL& a = *it->second;
    std::string s = "{\"name\":\"" + json_escape(a.name) + "\",\"ingress\":[";
    for (size_t i = 0; i < a.ingress.size(); i++) s += (i ? ",\"" : "\"") + json_escape(a.ingress[i]) + "\"";
    s += "],\"egress\":[";
    for (size_t i = 0; i < a.egress.size(); i++) s += (i ? ",\"" : "\"") + json_escape(a.egress[i]) + "\"";
    s += "],\"rules\":[";
    auto l4 = [](const L4Section& x) {
        if (!x.present) return std::string("null");
        auto rng = [](bool has, const PortRange& p) {
            return has ? "[" + std::to_string(p.lower) + "," + std::to_string(p.upper) + "]" : std::string("null");
        };
        return "{\"src\":" + rng(x.has_src, x.src) + ",\"dst\":" + rng(x.has_dst, x.dst) + "}";
    };
    for (size_t i = 0; i < a.rules.size(); i++) {
        const AclRule& r = a.rules[i];
        if (i) s += ",";
        s += "{\"action\":" + std::to_string(r.action) + ",\"src\":\"" + json_escape(r.src_network) +
             "\",\"dst\":\"" + json_escape(r.dst_network) + "\",\"tcp\":" + l4(r.tcp) + ",\"udp\":" + l4(r.udp) +
             ",\"icmp\":" + (r.has_icmp ? "true" : "false") + ",\"macip\":" + (r.has_macip ? "true" : "false") +
             ",\"ip_rule\":" + (r.has_ip_rule ? "true" : "false") + ",\"ip\":" + (r.has_ip ? "true" : "false") + "}";
    }
    s += "]}";
    if (buf && cap > 0) {
        size_t k = std::min(cap - 1, s.size());
        std::memcpy(buf, s.data(), k);
        buf[k] = 0;
    }
    return (int)s.size() + 1;
}

int pg_acl_names_json(pg_ctx* ctx, char* buf, size_t cap) {
    if (!ctx) return PG_EINVAL;
    std::string s = "[";
    bool first = true;
    for (auto& kv : ctx->eng.by_name) {
        s += (first ? "\"" : ",\"") + json_escape(kv.first) + "\"";
        first = false;
    }
    s += "]";
    if (buf && cap > 0) {
        size_t k = std::min(cap - 1, s.size());
        std::memcpy(buf, s.data(), k);
        buf[k] = 0;
    }
    return (int)s.size() + 1;
}

int pg_interface_acls(pg_ctx* ctx, const char* if_name, char* inbound, size_t in_cap, char* outbound,
                      size_t out_cap) {
    if (!ctx || !if_name) return PG_EINVAL;
    std::string in, out;
    auto it = ctx->eng.by_if.find(if_name);
    if (it != ctx->eng.by_if.end()) {
        if (it->second.first) in = it->second.first->name;
        if (it->second.second) out = it->second.second->name;
    }
    auto cp = [](char* b, size_t cap, const std::string& s) {
        if (b && cap) {
            size_t k = std::min(cap - 1, s.size());
            std::memcpy(b, s.data(), k);
            b[k] = 0;
        }
    };
    cp(inbound, in_cap, in);
    cp(outbound, out_cap, out);
    return PG_OK;
}

int pg_sync_tables(pg_ctx* ctx) {
    if (!ctx) return PG_EINVAL;
    DEVICE_GUARD(ctx);
    GUARD_BEGIN
    return ctx->eng.sync();
    GUARD_END(ctx)
}

// Table / slot metadata comes from the host image of the table set: compile, no upload
// (usable without a GPU).
static int ensure_compiled(pg_ctx* ctx) {
    GUARD_BEGIN
    if (!ctx->eng.compiled) ctx->eng.compile();
    return PG_OK;
    GUARD_END(ctx)
}

int pg_table_id(pg_ctx* ctx, const char* acl_name) {
    if (!ctx || !acl_name) return PG_EINVAL;
    int rc = ensure_compiled(ctx);
    if (rc) return rc;
    auto it = ctx->eng.table_of_acl.find(acl_name);
    return it == ctx->eng.table_of_acl.end() ? PG_ENOENT : it->second;
}

int pg_num_tables(pg_ctx* ctx) {
    if (!ctx) return PG_EINVAL;
    int rc = ensure_compiled(ctx);
    return rc ? rc : (int)ctx->eng.table_names.size();
}

int pg_num_counter_slots(pg_ctx* ctx) {
    if (!ctx) return PG_EINVAL;
    int rc = ensure_compiled(ctx);
    return rc ? rc : (int)ctx->eng.slot_table.size();
}

int pg_slot_info(pg_ctx* ctx, uint32_t slot, int32_t* table_id, int32_t* rule_index) {
    if (!ctx) return PG_EINVAL;
    int rc = ensure_compiled(ctx);
    if (rc) return rc;
    if (slot >= ctx->eng.slot_table.size()) return PG_EINVAL;
    if (table_id) *table_id = ctx->eng.slot_table[slot];
    if (rule_index) *rule_index = ctx->eng.slot_rule[slot];
    return PG_OK;
}

int pg_table_info(pg_ctx* ctx, int table_id, uint32_t* rule_base, uint32_t* n_rules, uint32_t* default_slot) {
    if (!ctx) return PG_EINVAL;
    int rc = ensure_compiled(ctx);
    if (rc) return rc;
    const HostTableSet& H = ctx->eng.host;
    if (table_id < 0 || (size_t)table_id >= H.tabs.size()) return fail(ctx, PG_EINVAL, "table id out of range");
    if (rule_base) *rule_base = H.tabs[table_id].rule_base;
    if (n_rules) *n_rules = H.tabs[table_id].n_rules;
    if (default_slot) *default_slot = (uint32_t)H.rules.size() + (uint32_t)table_id;
    return PG_OK;
}

int pg_table_stats(pg_ctx* ctx, int table_id, uint32_t* flags, uint32_t* blob_bytes, uint32_t* n_src_classes,
                   uint32_t* n_key_classes) {
    if (!ctx) return PG_EINVAL;
    GUARD_BEGIN
    Engine& E = ctx->eng;
    if (!E.compiled) E.compile();
    if (table_id < 0 || (size_t)table_id >= E.host.tabs.size()) return fail(ctx, PG_EINVAL, "table id out of range");
    const DevTable& hd = E.host.tabs[table_id];
    const uint32_t words = E.host.blob_words[table_id];
    const uint32_t* b = E.host.blobs.data() + hd.blob_off;
    if (flags) *flags = hd.fsk & 0xFFu;
    if (blob_bytes) *blob_bytes = words * 4;
    if (n_src_classes) *n_src_classes = words ? b[10] : 0;
    if (n_key_classes)
        *n_key_classes = !words ? 0 : (hd.fsk & kFlagFD) ? b[8] : (hd.fsk & (kFlagCross | kFlagPair)) ? b[7] : 0;
    return PG_OK;
    GUARD_END(ctx)
}

int pg_debug_walk_blob(pg_ctx* ctx, const char* acl_name, const uint32_t* src, const uint32_t* dst,
                       const uint16_t* dst_port, const uint8_t* proto, uint64_t n, uint32_t* out) {
    if (!ctx || !acl_name || (n && (!src || !dst || !dst_port || !proto || !out))) return PG_EINVAL;
    GUARD_BEGIN
    Engine& E = ctx->eng;
    if (!E.compiled) E.compile();
    auto it = E.table_of_acl.find(acl_name);
    if (it == E.table_of_acl.end()) return fail(ctx, PG_ENOENT, "no such ACL");
    const DevTable& hd = E.host.tabs[it->second];
    const bool linear = (hd.fsk & kFlagLinear) != 0;
    if (hd.fsk & kFlagFD) {  // the FD walk (one tuple at a time; ANY keys: linear, dst unused)
        DevTableSet T{};
        T.rules = E.host.rules.data();
        for (uint64_t i = 0; i < n; i++) {
            const uint32_t s1[1] = {src[i]}, dp1[1] = {dst_port[i]}, pr1[1] = {proto[i]};
            uint32_t w1[1];
            const uint32_t* b = E.host.blobs.data() + hd.blob_off;
            classify_fd_q<false, 1>(T, DevLoader{b}, DevLoader{b}, hd, s1, dp1, pr1, Hist{nullptr, nullptr}, w1);
            out[i] = w1[0];
        }
        return PG_OK;
    }
    // the kernels' lockstep walk, 4 tuples at a time
    constexpr int Q = 4;
    HostLoader ld[Q];
    BlobTab tb[Q];
    for (int j = 0; j < Q; j++) {
        ld[j] = HostLoader{E.host.blobs.data() + hd.blob_off};
        tb[j] = BlobTab{hd.fsk, hd.dflt, hd.kroot, hd.xoff, hd.nkc, hd.rule_base};
    }
    for (uint64_t i0 = 0; i0 < n; i0 += Q) {
        bool on[Q];
        uint32_t s4[Q], d4[Q], k4[Q], w4[Q];
        for (int j = 0; j < Q; j++) {
            const uint64_t i = i0 + j;
            const bool in = i < n;
            s4[j] = in ? src[i] : 0;
            d4[j] = in ? dst[i] : 0;
            k4[j] = in ? (proto[i] > 2 ? kKeyANY : pkt_key_host(proto[i], dst_port[i])) : 0;
            on[j] = in && !linear && k4[j] < kWalkKeyLimit;
            w4[j] = 0;
        }
        blob_walk(ld, tb, on, s4, d4, k4, w4);
        for (int j = 0; j < Q && i0 + j < n; j++) {
            if (on[j]) {
                out[i0 + j] = w4[j];
                continue;
            }
            uint32_t w = hd.dflt;  // mirror of eval_linear_lane
            for (uint32_t r = 0; r < hd.n_rules; r++) {
                const DevRule& R = E.host.rules[hd.rule_base + r];
                if ((s4[j] & R.smask) != R.snet || (d4[j] & R.dmask) != R.dnet) continue;
                if (k4[j] >= kKeyANY) {
                    if ((R.act >> 4) == kActNever) continue;
                    w = (((R.act >> 4) & 3u) << 30) | (hd.rule_base + r);
                    break;
                }
                if (k4[j] >= R.klo && k4[j] <= R.khi) {
                    w = ((R.act & 3u) << 30) | (hd.rule_base + r);
                    break;
                }
            }
            out[i0 + j] = w;
        }
    }
    return PG_OK;
    GUARD_END(ctx)
}

}  // extern "C"

namespace {
// A host loader that counts the reads of a walk by where the launch would find the word: in
// the LDS-staged part of the blob, or in HBM / L2 (a gather). u2 / u4 reads count once (one
// load instruction per lane on the device).
struct CountingLoader {
    const uint32_t* b;
    bool lds;
    uint32_t* n_lds;
    uint32_t* n_mem;
    void hit() const { ++*(lds ? n_lds : n_mem); }
    uint32_t u32(uint32_t i) const { return hit(), b[i]; }
    uint32_t at_byte(uint32_t off) const { return hit(), b[off >> 2]; }
    W2 u2(uint32_t i) const { return hit(), W2{b[i], b[i + 1]}; }
    W4 u4(uint32_t i) const { return hit(), W4{b[i], b[i + 1], b[i + 2], b[i + 3]}; }
};
}  // namespace

extern "C" {
int pg_debug_walk_stats(pg_ctx* ctx, int table_id, const pg_tuple_soa* t, uint64_t n, uint32_t* lds_reads,
                        uint32_t* mem_reads, int* stage) {
    if (!ctx || !t || (n && (!t->src_ip || !t->dst_ip || !t->dst_port || !t->proto || !lds_reads || !mem_reads)))
        return PG_EINVAL;
    GUARD_BEGIN
    Engine& E = ctx->eng;
    if (!E.compiled) E.compile();
    if (table_id < 0 || (uint32_t)table_id >= E.host.tabs.size()) return fail(ctx, PG_EINVAL, "table id out of range");
    const DevTable& hd = E.host.tabs[table_id];
    const Tuning& tu = E.tune;
    const uint32_t words = E.host.blob_words[table_id], prefix = E.host.blob_prefix[table_id];
    const uint32_t root_words = blob_root_words(hd.fsk, hd.nkc);
    const bool linear = (hd.fsk & kFlagLinear) != 0;
    // the launch device.hip launch_classify picks for this table (SINGLE mode)
    int st = 0;
    if (hd.fsk & kFlagFD) st = words <= tu.stage_max_words ? 4 : (prefix <= tu.stage_root_max_words ? 5 : 0);
    else if (!linear && words && words <= tu.stage_max_words) st = 1;
    else if (!linear && words && root_words <= tu.stage_root_max_words) st = 2;
    if (stage) *stage = st;
    const uint32_t* blob = E.host.blobs.data() + hd.blob_off;
    for (uint64_t i = 0; i < n; i++) {
        uint32_t nl = 0, nm = 0;
        const uint32_t s = t->src_ip[i], d = t->dst_ip[i];
        const uint32_t key = t->proto[i] > 2 ? kKeyANY : pkt_key_host(t->proto[i], t->dst_port[i]);
        bool scan = linear || key >= kWalkKeyLimit;
        if (!linear && !scan) {
            const CountingLoader whole{blob, st == 1 || st == 4, &nl, &nm};
            if (hd.fsk & kFlagFD) {
                const CountingLoader lp{blob, true, &nl, &nm};
                const uint32_t s1[1] = {s}, k1[1] = {key};
                uint32_t w1[1];
                if (st == 5) fd_walk<true>(lp, CountingLoader{blob, false, &nl, &nm}, hd.fsk, hd.kroot, hd.xoff, hd.nkc, s1, k1, w1);
                else fd_walk(whole, whole, hd.fsk, hd.kroot, hd.xoff, hd.nkc, s1, k1, w1);
            } else {
                const CountingLoader ld[1] = {whole};
                const CountingLoader ld0[1] = {CountingLoader{blob, st != 0, &nl, &nm}};
                const BlobTab tb[1] = {BlobTab{hd.fsk, hd.dflt, hd.kroot, hd.xoff, hd.nkc, hd.rule_base}};
                const bool on[1] = {true};
                const uint32_t s1[1] = {s}, d1[1] = {d}, k1[1] = {key};
                uint32_t w1[1];
                blob_walk(ld, ld0, tb, on, s1, d1, k1, w1);
            }
        }
        if (scan) {  // the linear scan: one rule read per rule visited
            for (uint32_t r = 0; r < hd.n_rules; r++) {
                nm++;
                const DevRule& R = E.host.rules[hd.rule_base + r];
                if ((s & R.smask) != R.snet || (d & R.dmask) != R.dnet) continue;
                if (key >= kKeyANY ? (R.act >> 4) != kActNever : (key >= R.klo && key <= R.khi)) break;
            }
        }
        lds_reads[i] = nl;
        mem_reads[i] = nm;
    }
    return PG_OK;
    GUARD_END(ctx)
}
}  // extern "C"

namespace {
// host view of the compiled table set (pointers into the host image)
DevTableSet host_view(const HostTableSet& h) {
    DevTableSet v{};
    v.rules = h.rules.data();
    v.tabs = h.tabs.data();
    v.blobs = h.blobs.data();
    v.ifaces = h.ifaces.data();
    v.iphash = h.iphash.data();
    v.iphash_mask = h.iphash_mask;
    v.node_if = h.node_if;
    v.node_in = h.node_in;
    v.node_out = h.node_out;
    v.n_rules = (uint32_t)h.rules.size();
    v.n_tables = (uint32_t)h.tabs.size();
    v.n_ifaces = (uint32_t)(h.ifaces.size() / 2);
    v.slot_noacl = v.n_rules + v.n_tables;
    v.slot_unresolved = v.slot_noacl + 1;
    v.n_slots = v.slot_unresolved + 1;
    v.slot_hot_in = h.slot_hot_in;
    v.node = h.node;
    v.node.img = h.node_img.empty() ? nullptr : h.node_img.data();
    v.node.cross = h.node_img.empty() ? nullptr : h.node_cross.data();
    v.host_tabs = h.tabs.data();
    v.host_blob_words = h.blob_words.data();
    v.host_blob_prefix = h.blob_prefix.data();
    return v;
}

template <int MODE, int Q, bool PRED, bool CM, bool UNI, bool WIDE>
void host_q(const DevTableSet& T, bool node, int table_id, const pg_tuple_soa* t, uint64_t i, uint32_t* out,
            const Hist& h) {
    uint32_t s[Q], d[Q], sp[Q], dp[Q], pr[Q], o[Q] = {};
    for (int j = 0; j < Q; j++) {
        s[j] = t->src_ip[i + j], d[j] = t->dst_ip[i + j], dp[j] = t->dst_port[i + j], pr[j] = t->proto[i + j];
        sp[j] = MODE == 2 ? t->src_port[i + j] : 0u;
    }
    if constexpr (MODE == 0) {
        const DevTable tab = load_tab(T.tabs, table_id);
        if ((tab.fsk & kFlagCandI) && (tab.fsk & kFlagDstFree)) {  // the kernels' STAGE 6 walk
            const DevLoader b{T.blobs + tab.blob_off};
            classify_candi_q<true, Q>(T, b, b, tab, s, dp, pr, h, o);
        } else {
            classify_q<0, true, Q, PRED>(T, T.blobs, tab, s, d, sp, dp, pr, h, o);
        }
    } else {
        if (node && MODE == 2 && UNI) {
            // as the device runs CONN over a uniform node: ANY-protocol packets deferred by the
            // classify kernel to k_node_any (device.hip PG_CONN_DEFER_ANY), then classified
            classify_node_q<MODE, true, Q, PRED, CM, false, UNI, true, WIDE>(T, T.node, DevLoader{T.node.img}, s, d, sp, dp,
                                                                         pr, h, o);
            for (int j = 0; j < Q; j++)
                if (pr[j] > 2u) o[j] = conn_any_1<true>(T, s[j], d[j], h);
        } else if (node) {
            classify_node_q<MODE, true, Q, PRED, CM, false, UNI, false, WIDE>(T, T.node, DevLoader{T.node.img}, s, d, sp, dp,
                                                                          pr, h, o);
        }
        else classify_q<MODE, true, Q, PRED>(T, T.blobs, DevTable{}, s, d, sp, dp, pr, h, o);
    }
    for (int j = 0; j < Q; j++) out[i + j] = o[j];
}

template <int MODE, bool PRED, bool CM, bool UNI, bool WIDE>
void host_classify(const DevTableSet& T, bool node, int table_id, const pg_tuple_soa* t, uint64_t n, uint32_t* out,
                   const Hist& h) {
    const uint64_t nq = n & ~(uint64_t)3;  // the kernels' quads, then one tuple at a time
    for (uint64_t i = 0; i < nq; i += 4) host_q<MODE, 4, PRED, CM, UNI, WIDE>(T, node, table_id, t, i, out, h);
    for (uint64_t i = nq; i < n; i++) host_q<MODE, 1, PRED, CM, UNI, WIDE>(T, node, table_id, t, i, out, h);
}
template <int MODE, bool UNI, bool WIDE = false>
void host_classify(const DevTableSet& T, bool node, bool pred, bool cm, int table_id, const pg_tuple_soa* t,
                   uint64_t n, uint32_t* out, const Hist& h) {
    if (pred && cm) host_classify<MODE, true, true, UNI, WIDE>(T, node, table_id, t, n, out, h);
    else if (pred) host_classify<MODE, true, false, UNI, WIDE>(T, node, table_id, t, n, out, h);
    else if (cm) host_classify<MODE, false, true, UNI, WIDE>(T, node, table_id, t, n, out, h);
    else host_classify<MODE, false, false, UNI, WIDE>(T, node, table_id, t, n, out, h);
}
}  // namespace

extern "C" {

int pg_debug_classify_host(pg_ctx* ctx, int mode, int table_id, const pg_tuple_soa* t, uint64_t n, uint32_t* out,
                           uint64_t* counters, int node) {
    if (!ctx || !t || mode < 0 || mode > 2) return PG_EINVAL;
    GUARD_BEGIN
    Engine& E = ctx->eng;
    if (!E.compiled) E.compile();
    const DevTableSet T = host_view(E.host);
    if (mode == PG_MODE_SINGLE && (table_id < 0 || (uint32_t)table_id >= T.n_tables))
        return fail(ctx, PG_EINVAL, "table id out of range");
    if (n == 0) return PG_OK;
    if (!out || !t->src_ip || !t->dst_ip || !t->dst_port || !t->proto || (mode == PG_MODE_CONN && !t->src_port))
        return fail(ctx, PG_EINVAL, "missing tuple field");
    const bool use_node = (node & 1) && T.node.img != nullptr, pred = (node & 2) != 0;
    const bool cm = use_node && (node & 4) && T.node.cmap != 0;
    const Hist h{nullptr, (unsigned long long*)counters};
    const bool uni = use_node && T.node.uniform;  // the layout the node was built with
    const bool wide = uni && T.node.wide;          // ... and its class records
    if (mode == 0) host_classify<0, false>(T, false, pred, false, table_id, t, n, out, h);
    else if (mode == 1 && wide) host_classify<1, true, true>(T, use_node, pred, cm, table_id, t, n, out, h);
    else if (mode == 1 && uni) host_classify<1, true>(T, use_node, pred, cm, table_id, t, n, out, h);
    else if (mode == 1) host_classify<1, false>(T, use_node, pred, cm, table_id, t, n, out, h);
    else if (wide) host_classify<2, true, true>(T, use_node, pred, cm, table_id, t, n, out, h);
    else if (uni) host_classify<2, true>(T, use_node, pred, cm, table_id, t, n, out, h);
    else host_classify<2, false>(T, use_node, pred, cm, table_id, t, n, out, h);
    return PG_OK;
    GUARD_END(ctx)
}

int pg_debug_set_snapshot(pg_ctx* ctx, int which, const uint64_t* counters, size_t n) {
    if (!ctx || (!counters && n) || (which != PG_SNAP_LOCAL && which != PG_SNAP_CLUSTER)) return PG_EINVAL;
    GUARD_BEGIN
    Engine& E = ctx->eng;
    if (!E.compiled) E.compile();
    if (n != E.layout->slots) return fail(ctx, PG_EINVAL, "counter count differs from the compiled slots");
    std::lock_guard<std::mutex> lk(E.snap_mu);
    CounterSnapshot& s = which == PG_SNAP_LOCAL ? E.snap_local : E.snap_cluster;
    s.v.assign(counters, counters + n);
    s.layout = E.layout;
    return PG_OK;
    GUARD_END(ctx)
}

int pg_debug_stream_slots(const uint64_t* streams, size_t n, uint32_t* slot_out, uint32_t* seq_out) {
    if ((!streams || !slot_out || !seq_out) && n) return PG_EINVAL;
    StreamSlots S;  // what dev_any_mark does per launch, without the events and the device words
    for (size_t k = 0; k < n; k++) {
        const void* s = (const void*)(uintptr_t)streams[k];
        size_t i = 0;
        bool added = false;
        if (!S.slot(s, &i, &added)) {  // (device.hip use_slot: drains the recorded launches first)
            S.clear();
            S.slot(s, &i, &added);
        }
        slot_out[k] = (uint32_t)i;
        seq_out[k] = S.draw(i);
    }
    return PG_OK;
}

int pg_node_stats(pg_ctx* ctx, uint32_t* ip_classes, uint32_t* key_classes, uint64_t* image_bytes,
                  uint64_t* cross_bytes) {
    if (!ctx) return PG_EINVAL;
    GUARD_BEGIN
    Engine& E = ctx->eng;
    if (!E.compiled) E.compile();
    const HostTableSet& h = E.host;
    if (h.node_img.empty()) return fail(ctx, PG_ENOENT, "no node classifier (disabled or over budget)");
    if (ip_classes) *ip_classes = h.node.n_ipc;
    if (key_classes) *key_classes = h.node.gk;
    if (image_bytes) *image_bytes = h.node_img.size() * 4;
    if (cross_bytes) *cross_bytes = h.node_cross.size() * 4;
    return PG_OK;
    GUARD_END(ctx)
}

int pg_node_common_stats(pg_ctx* ctx, uint64_t* base_image_bytes, uint64_t* common_pairs, uint64_t* pairs) {
    if (!ctx) return PG_EINVAL;
    GUARD_BEGIN
    Engine& E = ctx->eng;
    if (!E.compiled) E.compile();
    const HostTableSet& h = E.host;
    if (h.node_img.empty()) return fail(ctx, PG_ENOENT, "no node classifier (disabled or over budget)");
    uint64_t covered = 0, common = 0;
    for (size_t t = 0; t < h.tabs.size(); t++)
        if ((h.node.uniform ? h.node_aux : h.node_img)[h.node.tabinfo + 4 * t + 1] >> 31) covered++;
    if (h.node.cmap && h.node.uniform)  // one 64-bit (wide records: 32-bit) mask per IP class, in the class records
        for (size_t g = 0; g < h.node.n_ipc; g++)
            for (size_t t = 0; t < h.tabs.size(); t++) {
                const size_t b = t >> h.node.gshift;
                common += (h.node_img[h.node.cmap + (g << h.node.cmap_shift) + (b >> 5)] >> (b & 31)) & 1u;
            }
    else if (h.node.cmap)
        for (size_t i = h.node.cmap; i < (h.node.lrec ? h.node.lrec : h.node.img_words); i++) common += (uint64_t)__builtin_popcount(h.node_img[i]);
    if (base_image_bytes) *base_image_bytes = (uint64_t)h.node.img_words_base * 4;
    if (common_pairs) *common_pairs = common;
    if (pairs) *pairs = covered * h.node.n_ipc;
    return PG_OK;
    GUARD_END(ctx)
}

int pg_node_list_stats(pg_ctx* ctx, uint64_t* record_bytes, int* in_image) {
    if (!ctx) return PG_EINVAL;
    GUARD_BEGIN
    Engine& E = ctx->eng;
    if (!E.compiled) E.compile();
    const HostTableSet& h = E.host;
    if (h.node_img.empty()) return fail(ctx, PG_ENOENT, "no node classifier (disabled or over budget)");
    if (record_bytes) *record_bytes = (uint64_t)h.node_rec_words * 4;
    if (in_image) *in_image = h.node.lrec != 0;
    return PG_OK;
    GUARD_END(ctx)
}

int pg_node_list_table_stats(pg_ctx* ctx, uint64_t* table_bytes) {
    if (!ctx) return PG_EINVAL;
    GUARD_BEGIN
    Engine& E = ctx->eng;
    if (!E.compiled) E.compile();
    const HostTableSet& h = E.host;
    if (h.node_img.empty()) return fail(ctx, PG_ENOENT, "no node classifier (disabled or over budget)");
    if (table_bytes) *table_bytes = (uint64_t)h.node_list_tab_words * 4;
    return PG_OK;
    GUARD_END(ctx)
}

int pg_node_uniform(pg_ctx* ctx) {
    if (!ctx) return PG_EINVAL;
    GUARD_BEGIN
    Engine& E = ctx->eng;
    if (!E.compiled) E.compile();
    if (E.host.node_img.empty()) return fail(ctx, PG_ENOENT, "no node classifier (disabled or over budget)");
    return E.host.node.uniform ? (E.host.node.wide ? 2 : 1) : 0;
    GUARD_END(ctx)
}

int pg_classify(pg_ctx* ctx, int mode, int table_id, const pg_tuple_soa* t, uint64_t n, uint32_t* out,
                uint64_t* counters, void* stream) {
    if (!ctx || !t || mode < 0 || mode > 2) return PG_EINVAL;
    DEVICE_GUARD(ctx);
    GUARD_BEGIN
    int rc = ctx->eng.sync();
    if (rc) return rc;
    const DevTableSet& T = *ctx->eng.view();
    if (mode == PG_MODE_SINGLE && (table_id < 0 || (uint32_t)table_id >= T.n_tables))
        return fail(ctx, PG_EINVAL, "table id out of range");
    if (n == 0) return PG_OK;
    if (!out) return fail(ctx, PG_EINVAL, "null output");
    if (!t->src_ip || !t->dst_ip || !t->dst_port || !t->proto || (mode == PG_MODE_CONN && !t->src_port))
        return fail(ctx, PG_EINVAL, "missing tuple field");
    std::string err;
    DevTableSet TL = T;
    // PERPOD / CONN: the launch stream's mark word and this launch's number (device.hpp StreamSlots)
    if (mode != PG_MODE_SINGLE && !(TL.any_mark = dev_any_mark(ctx->eng.cur, stream, &TL.any_seq, &err)))
        return fail(ctx, PG_EIO, err);
    if (dev_classify(TL, ctx->eng.tune, mode, table_id, t->src_ip, t->dst_ip, t->src_port, t->dst_port, t->proto, n,
                     out, (unsigned long long*)counters, stream, &err) != 0 ||
        dev_mark_use(ctx->eng.cur, stream, counters != nullptr, &err) != 0)
        return fail(ctx, PG_EIO, err);
    return PG_OK;
    GUARD_END(ctx)
}

int pg_classify_linear(pg_ctx* ctx, int table_id, const pg_tuple_soa* t, uint64_t n, uint32_t* out, void* stream) {
    if (!ctx || !t || !out) return PG_EINVAL;
    DEVICE_GUARD(ctx);
    GUARD_BEGIN
    int rc = ctx->eng.sync();
    if (rc) return rc;
    const DevTableSet& T = *ctx->eng.view();
    if (table_id < 0 || (uint32_t)table_id >= T.n_tables) return fail(ctx, PG_EINVAL, "table id out of range");
    std::string err;
    if (dev_classify_linear(T, table_id, t->src_ip, t->dst_ip, t->dst_port, t->proto, n, out, stream, &err) != 0 ||
        dev_mark_use(ctx->eng.cur, stream, false, &err) != 0)
        return fail(ctx, PG_EIO, err);
    return PG_OK;
    GUARD_END(ctx)
}

int pg_stream_probe(pg_ctx* ctx, int fields, const pg_tuple_soa* t, uint64_t n, uint32_t* out, void* stream) {
    if (!ctx || !t || fields < 0 || fields > 3) return PG_EINVAL;
    DEVICE_GUARD(ctx);
    GUARD_BEGIN
    if (n == 0) return PG_OK;
    if (!out || !t->src_ip || !t->dst_port || !t->proto || ((fields & 1) && !t->dst_ip) ||
        ((fields & 2) && !t->src_port))
        return fail(ctx, PG_EINVAL, "missing tuple field");
    std::string err;
    if (dev_stream_probe(ctx->eng.tune, fields, t->src_ip, t->dst_ip, t->src_port, t->dst_port, t->proto, n, out,
                         stream, &err) != 0)
        return fail(ctx, PG_EIO, err);
    return PG_OK;
    GUARD_END(ctx)
}

uint64_t* pg_counters_device(pg_ctx* ctx) {
    if (!ctx) return nullptr;
    DeviceGuard g(ctx);
    if (!g.ok || ctx->eng.sync() != PG_OK) return nullptr;
    return (uint64_t*)ctx->eng.counters;
}

int pg_reset_counters(pg_ctx* ctx, void* stream) {
    if (!ctx) return PG_EINVAL;
    DEVICE_GUARD(ctx);
    int rc = ctx->eng.sync();
    if (rc) return rc;
    std::string err;
    // the reset is a counter write on `stream`: pg_read_counters waits for it like for a launch
    if (dev_memset(ctx->eng.counters, 0, ctx->eng.counter_slots * 8, stream, &err) != 0 ||
        dev_mark_use(ctx->eng.cur, stream, true, &err) != 0)
        return fail(ctx, PG_EIO, err);
    return PG_OK;
}

int pg_read_counters(pg_ctx* ctx, uint64_t* host_out, size_t n) {
    if (!ctx || !host_out) return PG_EINVAL;
    DEVICE_GUARD(ctx);
    Engine& E = ctx->eng;
    int rc = E.sync();
    if (rc) return rc;
    std::string err;
    std::vector<uint64_t> v(E.counter_slots);
    // the launches of this context that count have completed (their streams' events), then copy
    if (dev_wait_uses(E.cur, &err) != 0 || dev_copy_d2h(v.data(), E.counters, E.counter_slots * 8, &err) != 0)
        return fail(ctx, PG_EIO, err);
    size_t k = std::min(n, E.counter_slots);
    std::memcpy(host_out, v.data(), k * 8);
    std::lock_guard<std::mutex> lk(E.snap_mu);
    E.snap_local.v.swap(v);
    E.snap_local.layout = E.layout;
    return (int)k;
}

// the snapshot a `which` names (PG_SNAP_*); the gauge's: the cluster sum once a communicator exists
static const CounterSnapshot* pick_snapshot(const Engine& E, int which) {
    if (which == PG_SNAP_GAUGE) which = E.comm ? PG_SNAP_CLUSTER : PG_SNAP_LOCAL;
    if (which == PG_SNAP_LOCAL) return &E.snap_local;
    if (which == PG_SNAP_CLUSTER) return &E.snap_cluster;
    return nullptr;
}

int pg_counters_snapshot(const pg_ctx* ctx, uint64_t* host_out, size_t n) {
    if (!ctx || (!host_out && n)) return PG_EINVAL;
    const Engine& E = ctx->eng;
    std::lock_guard<std::mutex> lk(E.snap_mu);
    const CounterSnapshot* s = pick_snapshot(E, PG_SNAP_GAUGE);
    const size_t k = std::min(n, s->v.size());
    if (k) std::memcpy(host_out, s->v.data(), k * 8);
    return (int)s->v.size();
}

int pg_counters_snapshot_range(const pg_ctx* ctx, int which, uint32_t first, uint32_t n, uint64_t* host_out,
                               uint64_t* layout_gen) {
    if (!ctx || (!host_out && n)) return PG_EINVAL;
    const Engine& E = ctx->eng;
    std::lock_guard<std::mutex> lk(E.snap_mu);
    const CounterSnapshot* s = pick_snapshot(E, which);
    if (!s) return PG_EINVAL;
    if (layout_gen) *layout_gen = s->layout ? s->layout->gen : 0;
    const size_t sz = s->v.size();
    const size_t k = first >= sz ? 0 : std::min<size_t>(n, sz - first);
    if (k) std::memcpy(host_out, s->v.data() + first, k * 8);
    return (int)k;
}

int pg_counter_of_rule(const pg_ctx* ctx, int which, const char* acl_name, int rule_index, uint64_t* value,
                       uint64_t* layout_gen) {
    if (!ctx || !value || rule_index < -2) return PG_EINVAL;
    const Engine& E = ctx->eng;
    std::lock_guard<std::mutex> lk(E.snap_mu);
    const CounterSnapshot* s = pick_snapshot(E, which);
    if (!s) return PG_EINVAL;
    if (!s->layout) return PG_ENOENT;  // no snapshot taken yet
    const SlotLayout& L = *s->layout;
    if (layout_gen) *layout_gen = L.gen;
    uint32_t slot;
    if (!acl_name) {
        if (rule_index == -1) slot = L.noacl;
        else if (rule_index == -2) slot = L.unresolved;
        else return PG_EINVAL;
    } else {
        auto it = L.tabs.find(acl_name);
        if (it == L.tabs.end() || rule_index < -1 || (rule_index >= 0 && (uint32_t)rule_index >= it->second.n))
            return PG_ENOENT;
        slot = rule_index < 0 ? it->second.dflt : it->second.base + (uint32_t)rule_index;
    }
    if (slot >= s->v.size()) return PG_ENOENT;
    *value = s->v[slot];
    return PG_OK;
}

uint64_t pg_counter_layout_gen(const pg_ctx* ctx) {
    if (!ctx) return 0;
    // (any thread: compile() publishes the generation after the layout and snapshots are in place)
    return ctx->eng.layout_gen_pub.load(std::memory_order_acquire);
}

// ---- RCCL: per-rule hit counters summed over GPUs --------------------------
int pg_comm_unique_id(uint8_t* id) {
    if (!id) return PG_EINVAL;
    std::string err;
    return dev_comm_unique_id(id, &err) == 0 ? PG_OK : PG_EIO;
}

static int comm_attach(pg_ctx* ctx, void* comm, int rank, int nranks) {
    Engine& E = ctx->eng;
    std::string err;
    if (!E.comm_check && !(E.comm_check = (unsigned long long*)dev_alloc(4 * 8, &err)))
        return fail(ctx, PG_ENOMEM, err);
    void* old = E.comm;
    {
        std::lock_guard<std::mutex> lk(E.snap_mu);  // pick_snapshot reads E.comm under it
        E.comm = comm;
    }
    if (old) dev_comm_destroy(old);
    E.comm_rank = rank;
    E.comm_nranks = nranks;
    return PG_OK;
}

int pg_comm_init_rank(pg_ctx* ctx, int nranks, const uint8_t* id, int rank) {
    if (!ctx || !id || nranks < 1 || rank < 0 || rank >= nranks) return PG_EINVAL;
    DEVICE_GUARD(ctx);
    std::string err;
    void* c = dev_comm_init_rank(nranks, id, rank, &err);
    if (!c) return fail(ctx, PG_EIO, err);
    return comm_attach(ctx, c, rank, nranks);
}

int pg_comm_init_all(pg_ctx* const* ctxs, int n) {
    if (!ctxs || n < 1) return PG_EINVAL;
    std::vector<int> devs(n);
    for (int i = 0; i < n; i++) {
        if (!ctxs[i]) return PG_EINVAL;
        devs[i] = ctxs[i]->eng.device;
    }
    DeviceGuard g(ctxs[0]);
    std::vector<void*> comms(n, nullptr);
    std::string err;
    if (dev_comm_init_all(comms.data(), devs.data(), n, &err) != 0) return fail(ctxs[0], PG_EIO, err);
    for (int i = 0; i < n; i++) {
        DeviceGuard gi(ctxs[i]);
        int rc = gi.ok ? comm_attach(ctxs[i], comms[i], i, n) : fail(ctxs[i], PG_EIO, gi.err);
        if (rc) {
            for (int j = i + 1; j < n; j++) dev_comm_destroy(comms[j]);
            return rc;
        }
    }
    return PG_OK;
}

int pg_comm_destroy(pg_ctx* ctx) {
    if (!ctx) return PG_EINVAL;
    DEVICE_GUARD(ctx);
    void* old = ctx->eng.comm;
    {
        std::lock_guard<std::mutex> lk(ctx->eng.snap_mu);  // pick_snapshot reads E.comm under it
        ctx->eng.comm = nullptr;
    }
    if (old) dev_comm_destroy(old);
    ctx->eng.comm_rank = -1;
    ctx->eng.comm_nranks = 0;
    return PG_OK;
}

int pg_comm_rank(const pg_ctx* ctx, int* rank, int* nranks) {
    if (!ctx) return PG_EINVAL;
    if (rank) *rank = ctx->eng.comm_rank;
    if (nranks) *nranks = ctx->eng.comm_nranks;
    return ctx->eng.comm ? PG_OK : PG_ENOENT;
}

// Restores the device that was current when it was made, whatever the calls in between set
// (the all-reduce below visits every context's GPU).
struct RestoreDevice {
    int prev = -1;
    RestoreDevice() {
        if (dev_get_device(&prev) != 0) prev = -1;
    }
    ~RestoreDevice() {
        int now = -1;
        if (prev >= 0 && (dev_get_device(&now) != 0 || now != prev)) (void)dev_set_device(prev, nullptr);
    }
};

// The contexts' counters summed over their communicator (k = 1: this process's rank of a
// multi-process communicator; k > 1: every context of one pg_comm_init_all group, in one RCCL
// group call). First a max all-reduce of {slots, layout hash, ~slots, ~hash} proves that every
// rank compiled the same counter layout (a mismatched all-reduce would hang or mix slots);
// then ncclAllReduce(u64, sum) of a device copy of the counters: the counters themselves stay
// this rank's own, so a periodic gauge may reduce again without compounding earlier sums.
// Synchronous; the host snapshots hold the sums afterwards.
static int allreduce_counters(pg_ctx* const* ctxs, int k, void* const* streams) {
    RestoreDevice restore;
    std::vector<void*> comms(k), sts(k);
    std::vector<unsigned long long*> chk(k), bufs(k);
    std::vector<int> devs(k);
    std::string err;
    for (int i = 0; i < k; i++) {
        pg_ctx* c = ctxs[i];
        if (!c) return PG_EINVAL;
        Engine& E = c->eng;
        if (!E.comm) return fail(c, PG_EINVAL, "no communicator (pg_comm_init_rank / pg_comm_init_all)");
        if (k > 1 && E.comm_nranks != k) return fail(c, PG_EINVAL, "contexts are not one pg_comm_init_all group");
        if (dev_set_device(E.device, &err) != 0) return fail(c, PG_EIO, err);
        int rc = E.sync();
        if (rc) return rc;
        if (E.reduced_slots != E.counter_slots) {
            if (E.reduced) dev_release(E.reduced);
            E.reduced_slots = 0;
            if (!(E.reduced = (unsigned long long*)dev_alloc(E.counter_slots * 8, &err)))
                return fail(c, PG_ENOMEM, err);
            E.reduced_slots = E.counter_slots;
        }
        const uint64_t n = E.counter_slots, h = E.layout_hash;
        const uint64_t v[4] = {n, h, ~n, ~h};
        sts[i] = streams ? streams[i] : nullptr;
        if (dev_wait_uses(E.cur, &err) != 0 || dev_copy_h2d(E.comm_check, v, sizeof v, &err) != 0 ||
            dev_copy_d2d_async(E.reduced, E.counters, E.counter_slots * 8, sts[i], &err) != 0)
            return fail(c, PG_EIO, err);
        comms[i] = E.comm, chk[i] = E.comm_check;
        bufs[i] = E.reduced, devs[i] = E.device;
    }
    if (dev_comm_allreduce_u64(comms.data(), chk.data(), devs.data(), sts.data(), k, 4, true, &err) != 0)
        return fail(ctxs[0], PG_EIO, err);
    for (int i = 0; i < k; i++) {
        Engine& E = ctxs[i]->eng;
        uint64_t v[4];
        if (dev_set_device(E.device, &err) != 0 || dev_stream_sync(sts[i], &err) != 0 ||
            dev_copy_d2h(v, E.comm_check, sizeof v, &err) != 0)
            return fail(ctxs[i], PG_EIO, err);
        const uint64_t n = E.counter_slots, h = E.layout_hash;
        if (v[0] != n || v[1] != h || v[2] != ~n || v[3] != ~h)
            return fail(ctxs[i], PG_EFAULT, "ranks hold different counter layouts (tables differ): not reduced");
    }
    if (dev_comm_allreduce_u64(comms.data(), bufs.data(), devs.data(), sts.data(), k, ctxs[0]->eng.counter_slots,
                               false, &err) != 0)
        return fail(ctxs[0], PG_EIO, err);
    for (int i = 0; i < k; i++) {
        Engine& E = ctxs[i]->eng;
        std::vector<uint64_t> v(E.counter_slots);
        if (dev_set_device(E.device, &err) != 0 || dev_stream_sync(sts[i], &err) != 0 ||
            dev_copy_d2h(v.data(), E.reduced, E.counter_slots * 8, &err) != 0)
            return fail(ctxs[i], PG_EIO, err);
        std::lock_guard<std::mutex> lk(E.snap_mu);
        E.snap_cluster.v.swap(v);
        E.snap_cluster.layout = E.layout;
    }
    return PG_OK;
}

int pg_allreduce_counters(pg_ctx* ctx, void* stream) {
    if (!ctx) return PG_EINVAL;
    GUARD_BEGIN
    pg_ctx* c[1] = {ctx};
    void* s[1] = {stream};
    return allreduce_counters(c, 1, s);
    GUARD_END(ctx)
}

int pg_allreduce_counters_all(pg_ctx* const* ctxs, int n) {
    if (!ctxs || n < 1 || !ctxs[0]) return PG_EINVAL;
    GUARD_BEGIN
    return allreduce_counters(ctxs, n, nullptr);
    GUARD_END(ctxs[0])
}

int pg_gen_tuples(pg_ctx* ctx, const pg_gen_spec* spec, uint64_t n, uint32_t* src, uint32_t* dst, uint16_t* sport,
                  uint16_t* dport, uint8_t* proto, void* stream) {
    if (!ctx || !spec || !src || !dst || !dport || !proto) return PG_EINVAL;
    DEVICE_GUARD(ctx);
    GUARD_BEGIN
    int rc = ctx->eng.sync();
    if (rc) return rc;
    const DevTableSet& T = *ctx->eng.view();
    if (spec->table_id >= 0 && (uint32_t)spec->table_id >= T.n_tables) return fail(ctx, PG_EINVAL, "table id");
    if (spec->table_id >= 0 && spec->inside_pct > 0) {
        std::vector<DevTable> tabs(1);
        // n_rules of the table must be > 0 for inside sampling
        auto it = ctx->eng.by_name.find(ctx->eng.table_names[spec->table_id]);
        if (it->second->rules.empty()) return fail(ctx, PG_EINVAL, "inside sampling on an empty table");
    }
    std::string err;
    GenParams g{};
    g.seed = spec->seed;
    g.index_base = spec->index_base;
    g.table_id = spec->table_id;
    g.inside_pct = spec->inside_pct;
    g.pool_pct = spec->pool_pct;
    g.port_pool_pct = spec->port_pool_pct;
    g.tcp_pct = spec->tcp_pct;
    g.udp_pct = spec->udp_pct;
    g.nomatch_pct = spec->nomatch_pct;
    g.dst_pool_pct = spec->dst_pool_pct;
    g.n_ip_pool = spec->ip_pool ? spec->n_ip_pool : 0;
    g.n_port_pool = spec->port_pool ? spec->n_port_pool : 0;
    void *ipp = nullptr, *pp = nullptr, *zc = nullptr;
    auto cleanup = [&]() {
        dev_stream_sync(stream, nullptr);  // k_gen has read the pools
        dev_release(ipp);
        dev_release(pp);
        dev_release(zc);
    };
    if (g.n_ip_pool) {
        ipp = dev_alloc(g.n_ip_pool * 4, &err);
        if (!ipp || dev_copy_h2d(ipp, spec->ip_pool, g.n_ip_pool * 4, &err)) return cleanup(), fail(ctx, PG_EIO, err);
        g.ip_pool = (const uint32_t*)ipp;
    }
    if (g.n_port_pool) {
        pp = dev_alloc(g.n_port_pool * 2, &err);
        if (!pp || dev_copy_h2d(pp, spec->port_pool, g.n_port_pool * 2, &err)) return cleanup(), fail(ctx, PG_EIO, err);
        g.port_pool = (const uint16_t*)pp;
    }
    if (spec->zipf_cdf && spec->table_id >= 0) {
        size_t nr = ctx->eng.by_name[ctx->eng.table_names[spec->table_id]]->rules.size();
        zc = dev_alloc(nr * 4, &err);
        if (!zc || dev_copy_h2d(zc, spec->zipf_cdf, nr * 4, &err)) return cleanup(), fail(ctx, PG_EIO, err);
        g.zipf_cdf = (const uint32_t*)zc;
    }
    int r2 = dev_gen(T, g, n, src, dst, sport, dport, proto, stream, &err);
    cleanup();
    if (r2 != 0) return fail(ctx, PG_EIO, err);
    return PG_OK;
    GUARD_END(ctx)
}

// Connection* preamble (aclengine_mock.go:273-420) on the host, testConnection on the device.
int pg_connections(pg_ctx* ctx, const pg_conn_query* q, size_t n, int32_t* out, uint32_t* out_slot) {
    if (!ctx || (!q && n) || (!out && n)) return PG_EINVAL;
    DEVICE_GUARD(ctx);
    GUARD_BEGIN
    Engine& E = ctx->eng;
    int rc = E.sync();
    if (rc) return rc;
    const DevTableSet& T = *E.view();
    std::vector<ConnQueryDev> dq;
    std::vector<int64_t> where(n, -1);
    std::string node_if = E.node_if_name();
    for (size_t i = 0; i < n; i++) {
        const pg_conn_query& c = q[i];
        std::string sif, dif;
        Bytes sip, dip;
        bool ok = true;
        auto pod_if = [&](const char* ns, const char* nm, bool allow_remote, std::string* ifn, Bytes* ip) {
            auto it = E.pods.find(PodID{sv(ns), sv(nm)});
            if (it == E.pods.end()) return false;
            *ip = it->second.ip;
            if (it->second.another_node) {
                if (!allow_remote || node_if.empty()) return false;
                *ifn = node_if;
                return true;
            }
            return E.ifaces.if_name(PodID{sv(ns), sv(nm)}, ifn);
        };
        if (c.kind == 0) {
            ok = pod_if(c.src_namespace, c.src_name, true, &sif, &sip) &&
                 pod_if(c.dst_namespace, c.dst_name, true, &dif, &dip);
        } else if (c.kind == 1) {
            ok = pod_if(c.src_namespace, c.src_name, false, &sif, &sip) && !node_if.empty() &&
                 parse_ip(sv(c.dst_ip), &dip);
            dif = node_if;
        } else if (c.kind == 2) {
            ok = !node_if.empty() && parse_ip(sv(c.src_ip), &sip) &&
                 pod_if(c.dst_namespace, c.dst_name, false, &dif, &dip);
            sif = node_if;
        } else {
            return fail(ctx, PG_EINVAL, "bad query kind");
        }
        if (!ok) {
            out[i] = PG_CONN_FAILURE;
            if (out_slot) out_slot[i] = T.slot_unresolved;
            continue;
        }
        Bytes s4, d4;
        if (!to4(sip, &s4) || !to4(dip, &d4)) return fail(ctx, PG_EINVAL, "IPv6 endpoints are not classified");
        ConnQueryDev d{};
        d.src_ip = ipv4_u32(s4);
        d.dst_ip = ipv4_u32(d4);
        d.src_if = E.iface_of(sif);
        d.dst_if = E.iface_of(dif);
        if (d.src_if < 0 || d.dst_if < 0) return fail(ctx, PG_EFAULT, "interface not compiled");
        d.key_syn = pkt_key_host(c.protocol, c.dst_port);
        d.key_synack = pkt_key_host(c.protocol, c.src_port);
        where[i] = (int64_t)dq.size();
        dq.push_back(d);
    }
    std::vector<uint32_t> res(dq.size());
    std::string err;
    if (dev_conn_queries(T, dq.data(), dq.size(), res.data(), &err) != 0) return fail(ctx, PG_EIO, err);
    for (size_t i = 0; i < n; i++) {
        if (where[i] < 0) continue;
        uint32_t w = res[where[i]];
        out[i] = (int32_t)(w >> 30);
        if (out_slot) out_slot[i] = w & 0x3FFFFFFFu;
    }
    return PG_OK;
    GUARD_END(ctx)
}

}  // extern "C"
