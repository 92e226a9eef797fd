// Host side of the policy path above the device: ContivRule ordering, rule tables, the
// renderer cache (both orientations), the vpp_acl model and the GPU renderer that renders
// tables into ACLs exactly like the reference's ACL renderer.
//
// Reference (itaimlx/vpp):
//   renderer.ContivRule / Compare / String          plugins/policy/renderer/api.go:65-191
//   utils.Compare{Ints,IPNets,Ports}                plugins/policy/utils/utils.go:175-257
//   cache.ContivRuleTable / LocalTables / Ports     plugins/policy/renderer/cache/{cache_api,local_tables,ports}.go
//   cache.RendererCache / RendererCacheTxn          plugins/policy/renderer/cache/cache_impl.go:29-667
//   vpp_acl.ACL                                     vendor/.../api/models/vpp/acl/acl.proto:24-113
//   acl.Renderer / RendererTxn                      plugins/policy/renderer/acl/acl_renderer.go:51-390
#pragma once
#include <map>
#include <memory>
#include <set>
#include <string>
#include <vector>

#include "gonet.hpp"

namespace pg {

enum Action { kDeny = 0, kPermit = 1 };
enum Proto { kTCP = 0, kUDP = 1, kOTHER = 2, kANY = 3 };

struct PodID {
    std::string ns, name;
    bool operator<(const PodID& o) const { return ns < o.ns || (ns == o.ns && name < o.name); }
    bool operator==(const PodID& o) const { return ns == o.ns && name == o.name; }
    std::string str() const { return ns + "/" + name; }
};
using PodSet = std::set<PodID>;

struct ContivRule {
    int action = kPermit;
    IPNet src, dst;
    int protocol = kANY;
    uint16_t src_port = 0, dst_port = 0;
    int compare(const ContivRule& o) const;
    std::string str() const;
};

int compare_ints(int a, int b);
int compare_ipnets(const IPNet& a, const IPNet& b);
int compare_ports(uint16_t a, uint16_t b);
ContivRule allow_all_rule();

// --- vpp_acl model -----------------------------------------------------------
struct PortRange {
    uint32_t lower = 0, upper = 0;
};
struct L4Section {
    bool present = false, has_src = false, has_dst = false;
    PortRange src, dst;
};
enum AclAction { kAclDeny = 0, kAclPermit = 1, kAclReflect = 2 };
struct AclRule {
    int action = kAclDeny;
    bool has_macip = false, has_ip_rule = true, has_ip = true, has_icmp = false;
    std::string src_network, dst_network;
    L4Section tcp, udp;
};
struct ACL {
    std::string name;
    std::vector<AclRule> rules;
    std::vector<std::string> ingress, egress;
};
using ACLPtr = std::shared_ptr<ACL>;

// --- rule tables --------------------------------------------------------------
enum TableType { kLocal = 0, kGlobal = 1 };
extern const char* kGlobalTableID;

struct ContivRuleTable {
    int type = kLocal;
    PodSet pods;
    std::vector<ContivRule> rules;  // Rules[:NumOfRules]
    size_t slice_len = 0;           // len(Rules): nil-padded high-water mark
    ACLPtr priv;                    // Private (rendered ACL)
    mutable std::string id;
    size_t num_rules() const { return rules.size(); }
    const std::string& get_id() const;
    bool insert_rule(const ContivRule& r);
    // InsertRule of every rule of rs in order, in O((n + k) log k): the same table and
    // NumOfRules / len(Rules) as k single inserts
    void insert_rules(const std::vector<ContivRule>& rs);
    bool has_rule(const ContivRule& r) const;
    size_t index_of(const ContivRule& r, bool* present) const;
    template <class P>
    int remove_by_predicate(P pred) {
        size_t n0 = rules.size();
        std::vector<ContivRule> keep;
        keep.reserve(n0);
        for (auto& r : rules)
            if (!pred(r)) keep.push_back(r);
        rules.swap(keep);
        return (int)(n0 - rules.size());
    }
};
using TablePtr = std::shared_ptr<ContivRuleTable>;

int compare_rule_lists(const std::vector<ContivRule>& a, const std::vector<ContivRule>& b);

struct LocalTables {
    std::vector<TablePtr> tables;  // ordered by rules
    std::map<std::string, TablePtr> by_id;
    std::map<PodID, TablePtr> by_pod;
    bool insert(const TablePtr& t);
    bool remove(const TablePtr& t);
    void assign_pod(const TablePtr& t, const PodID& pod);
    void unassign_pod(const TablePtr& t, const PodID& pod);  // t may be null
    TablePtr lookup_by_id(const std::string& id) const;
    TablePtr lookup_by_rules(const std::vector<ContivRule>& rules) const;
    TablePtr lookup_by_pod(const PodID& pod) const;
    PodSet isolated_pods() const;
    size_t idx_by_rules(const std::vector<ContivRule>& rules) const;
};

// --- renderer cache -----------------------------------------------------------
enum Orientation { kIngressOrientation = 0, kEgressOrientation = 1 };

struct PodConfig {
    bool has_ip = false;
    IPNet pod_ip;
    std::vector<ContivRule> ingress, egress;
    bool removed = false;
};
using PodConfigPtr = std::shared_ptr<PodConfig>;

struct TxnChange {
    TablePtr table;
    PodSet previous_pods;
};

struct RendererCache;
struct RendererCacheTxn {
    RendererCache* cache;
    LocalTables local;
    TablePtr global;  // null = no change computed
    bool up_to_date = false;
    std::map<PodID, PodConfigPtr> config;

    explicit RendererCacheTxn(RendererCache* c) : cache(c) {}
    void update(const PodID& pod, PodConfigPtr cfg);
    PodSet updated_pods() const;
    PodSet removed_pods() const;
    PodConfigPtr pod_config(const PodID& pod) const;
    PodSet all_pods() const;
    PodSet isolated_pods();
    TablePtr local_table_by_pod(const PodID& pod);
    TablePtr global_table();
    std::vector<TxnChange> changes();
    void commit();

   private:
    void refresh();
    TablePtr build_local_table(const PodID& pod, const PodConfig& cfg);
    void install_local_rules(ContivRuleTable& dst, const PodConfig& dcfg, const PodConfig& scfg);
    void install_allowed_ports(ContivRuleTable& dst, const IPNet& src_ip, const std::set<uint16_t>& ports, int proto);
    void rebuild_global();
};

struct RendererCache {
    int orientation = kEgressOrientation;
    LocalTables local;
    TablePtr global;
    std::map<PodID, PodConfigPtr> config;
    explicit RendererCache(int orient) : orientation(orient) { flush(); }
    void flush();
    std::string resync(const std::vector<TablePtr>& tables);
    PodSet all_pods() const;
    PodSet isolated_pods() const { return local.isolated_pods(); }
    TablePtr local_table_by_pod(const PodID& pod) const;
};

// --- interface naming (ipv4net / contivconf getters) ---------------------------
struct NodeIfaces {
    std::map<PodID, std::string> pod_if;
    std::string host_interconnect, main_if, vxlan_bvi;
    std::vector<std::string> other_ifs;
    bool if_name(const PodID& pod, std::string* out) const {
        auto it = pod_if.find(pod);
        if (it == pod_if.end()) return false;
        *out = it->second;
        return true;
    }
    std::vector<std::string> node_output_ifs() const;  // acl_renderer.go:277-292
};

// One controller transaction worth of ACL changes: key = ACL name, value null = delete.
using AclOps = std::map<std::string, ACLPtr>;
using ApplyFn = std::string (*)(void* engine, bool resync, const AclOps& ops);

// --- the GPU renderer (acl_renderer.go semantics, EgressOrientation by default) ----
struct Renderer {
    const NodeIfaces* ifaces;
    void* engine;
    ApplyFn apply;
    RendererCache cache;
    std::map<PodID, std::string> pod_ifs;  // podInterfaces
    Renderer(const NodeIfaces* i, void* e, ApplyFn a, int orient) : ifaces(i), engine(e), apply(a), cache(orient) {}
};

struct RendererTxn {
    Renderer* r;
    RendererCacheTxn cache_txn;
    bool resync;
    RendererTxn(Renderer* rr, bool rs) : r(rr), cache_txn(&rr->cache), resync(rs) {}
    void render(const PodID& pod, const IPNet* pod_ip, std::vector<ContivRule> ingress,
                std::vector<ContivRule> egress, bool removed);
    std::string commit();  // "" = ok

   private:
    std::string commit_resync();
    ACLPtr render_acl(ContivRuleTable& t, bool reflective);
    void render_interfaces(const PodSet& pods, bool ingress, std::vector<std::string>* in,
                           std::vector<std::string>* eg);
    ACLPtr reflective_acl();
};

}  // namespace pg
