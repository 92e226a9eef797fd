// The VPPTCP renderer: the second consumer of the renderer cache (IngressOrientation), which
// turns ContivRule tables into VPP session rules for the VPP TCP host stack, and the VPP
// session-rule tables it programs over the binary API (session_rule_add_del /
// session_rules_dump), as the reference's mock holds them.
//
// Reference (itaimlx/vpp):
//   vpptcp.Renderer / RendererTxn (Init, NewTxn, Render, Commit, dumpRules, updateRules)
//                                           plugins/policy/renderer/vpptcp/vpptcp_renderer.go:33-316
//   rule.SessionRule, Compare, ExportSessionRules, convertContivRule, ImportSessionRules
//                                           plugins/policy/renderer/vpptcp/rule/session_rule.go:31-476
//   ContivRuleTable.DiffRules               plugins/policy/renderer/cache/cache_api.go:321-334
//   utils.CompareIPNetsBytes                plugins/policy/utils/utils.go:261-267
//   MockSessionRules (tables, add/del, dump, HasRule, request/error counts)
//                                           mock/sessionrules/sessionrules_mock.go:25-416
//
// No packet classification happens on this path in the reference (VPP's session-rule lookup
// is VPP code, absent from the reference): this is control plane, rendered on the host.
#pragma once
#include <cstdint>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "configurator.hpp"
#include "policy.hpp"

namespace pg {

enum SessionScope { kScopeGlobal = 1, kScopeLocal = 2, kScopeBoth = 3 };
constexpr uint32_t kSrActionDoNothing = ~0u;
constexpr uint32_t kSrActionDeny = ~0u - 1;
constexpr uint32_t kSrActionAllow = ~0u - 2;
enum { kSrProtoTCP = 0, kSrProtoUDP = 1 };
extern const char* kSessionRuleTagPrefix;  // "contiv/vpp-policy"

struct SessionRule {
    uint8_t transport_proto = 0;
    uint8_t is_ip4 = 0;
    uint8_t lcl_ip[16] = {};
    uint8_t lcl_plen = 0;
    uint8_t rmt_ip[16] = {};
    uint8_t rmt_plen = 0;
    uint16_t lcl_port = 0, rmt_port = 0;
    uint32_t action_index = 0;
    uint32_t appns_index = 0;
    uint8_t scope = 0;
    char tag[64] = {};
    int compare(const SessionRule& o, bool compare_tag) const;  // session_rule.go:168-209
    std::string tag_str() const;                                // up to the first NUL
    void set_tag(const std::string& t);                         // copy(Tag[:], t)
};

// The two IPv4Net getters the renderer needs (session_rule.go:88-95): pod <-> VPP application
// namespace index.
struct AppNsIndex {
    std::map<PodID, uint32_t> by_pod;
    bool ns_index(const PodID& pod, uint32_t* out) const;
    bool pod_by_ns_index(uint32_t idx, PodID* out) const;  // first pod in PodID order
};

// session_rule.go:213-260 (pod == nullptr: global table)
std::vector<SessionRule> export_session_rules(const std::vector<ContivRule>& rules, const PodID* pod,
                                              const Bytes& pod_ip, const AppNsIndex& ns);
// session_rule.go:365-476: the global table first, then one local table per pod
std::vector<TablePtr> import_session_rules(const std::vector<SessionRule>& rules, const AppNsIndex& ns);
// cache_api.go:321-334
void diff_rules(const ContivRuleTable& a, const ContivRuleTable& b, std::vector<ContivRule>* not_in_b,
                std::vector<ContivRule>* not_in_a);

// VPP's session-rule tables as the binary API sees them (mock/sessionrules): local tables keyed
// by application namespace index, one global table, request and error counters.
struct SessionRuleTables {
    std::string tag_prefix;
    std::map<uint32_t, std::vector<SessionRule>> local;
    std::vector<SessionRule> global;
    int req_count = 0, err_count = 0;
    explicit SessionRuleTables(std::string prefix) : tag_prefix(std::move(prefix)) {}
    void clear();
    int add_del(const SessionRule& r, bool is_add);  // session_rule_add_del: retval (0 ok)
    std::vector<SessionRule> dump();                 // session_rules_dump + control_ping
    const std::vector<SessionRule>* table(int scope, uint32_t ns_index) const;
    // MockSessionRules.hasRule (sessionrules_mock.go:137-228): address strings as the tests
    // write them ("" = unset, a bare address = one-host subnet, else a CIDR)
    bool has_rule(int scope, uint32_t ns_index, const std::string& lcl_ip, uint16_t lcl_port,
                  const std::string& rmt_ip, uint16_t rmt_port, const std::string& proto,
                  const std::string& action) const;
};

// VPP's session-rule lookup over one table, as a first-match ACL the classification engine
// compiles (pg_session_table_install): the table's IPv4 rules ordered most specific first --
// specificity = lcl_plen + rmt_plen + one per specific port, ties in SessionRule::compare
// order -- so a rule strictly inside another always precedes it (the containment order
// renderer/api.go:111-112 gives ContivRules). Packet fields: a LOCAL table keys on (src = the
// local address, dst = the remote address, dport = the remote port), the GLOBAL table on
// (src = remote, dst = local, dport = local port), the other port is 0 (any) in every rule
// convertContivRule emits (session_rule.go:263-361). No match = the ACL's default slot (VPP:
// no session rule applies). nullptr + *err for a rule the form cannot hold (a port on the other
// side, an action other than ALLOW / DENY).
ACLPtr session_table_acl(const std::vector<SessionRule>& table, int scope, const std::string& name, std::string* err);

struct VppTcpRenderer : CfgRenderer {
    const AppNsIndex* ipv4net;
    SessionRuleTables* vpp;
    int chan_buf_size;  // GoVPPChanBufSize (0 = 100)
    RendererCache cache;
    VppTcpRenderer(const AppNsIndex* ns, SessionRuleTables* v, int buf)
        : ipv4net(ns), vpp(v), chan_buf_size(buf), cache(kIngressOrientation) {}
    std::unique_ptr<CfgRendererTxn> new_txn(bool resync) override;
    std::string update_rules(const std::vector<SessionRule>& add, const std::vector<SessionRule>& remove);
};

struct VppTcpRendererTxn : CfgRendererTxn {
    VppTcpRenderer* r;
    RendererCacheTxn cache_txn;
    bool resync;
    VppTcpRendererTxn(VppTcpRenderer* rr, bool rs) : r(rr), cache_txn(&rr->cache), resync(rs) {}
    void render(const PodID& pod, const IPNet* pod_ip, const std::vector<ContivRule>& ingress,
                const std::vector<ContivRule>& egress, bool removed) override;
    std::string commit() override;  // "" = ok
};

}  // namespace pg
