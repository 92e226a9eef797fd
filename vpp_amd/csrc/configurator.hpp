// The policy configurator: K8s-shaped policies of a pod -> the ordered ContivRule lists its
// renderers receive, plus the mock renderer that stores those lists and
// evaluates traffic against them (§8 a13, the reference's test oracle for the configurator).
//
// Reference (itaimlx/vpp):
//   configurator.ContivPolicy / Match / IPBlock / Port      plugins/policy/configurator/configurator_api.go:41-271
//   PolicyConfigurator.NewTxn / Txn.Configure / Commit      plugins/policy/configurator/configurator_impl.go:104-254
//   generateRules                                           configurator_impl.go:263-472
//   ContivPolicies sort / Equals, ContivRules.Insert/Copy   configurator_impl.go:474-550
//   subtractSubnet                                          configurator_impl.go:562-594
//   utils.GetOneHostSubnet(FromIP)                          plugins/policy/utils/utils.go:270-291
//   MockRenderer (NewTxn / Render / Commit / TestTraffic)   mock/renderer/renderer_mock.go:39-185
#pragma once
#include <set>
#include <functional>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "policy.hpp"

namespace pg {

enum PolicyType { kPolicyIngress = 0, kPolicyEgress = 1, kPolicyAll = 2 };
enum MatchType { kMatchIngress = 0, kMatchEgress = 1 };
enum PortProto { kPortTCP = 0, kPortUDP = 1 };

struct CfgPort {
    int protocol = kPortTCP;
    uint16_t number = 0;
};
struct CfgIPBlock {
    IPNet network;
    std::vector<IPNet> except;
};
struct CfgMatch {
    int type = kMatchIngress;
    bool pods_nil = true;    // Go nil slice (vs. empty): "match anything" needs both nil
    std::vector<PodID> pods;
    bool blocks_nil = true;
    std::vector<CfgIPBlock> blocks;
    std::vector<CfgPort> ports;
};
struct CfgPolicy {
    PodID id;  // policymodel.ID {Namespace, Name}
    int type = kPolicyIngress;
    std::vector<CfgMatch> matches;
};
using CfgPolicies = std::vector<std::shared_ptr<const CfgPolicy>>;

// ContivRules: insertion order (what renderers receive) + ordered set (deduplication)
// The reference keeps a sorted slice for dedup (binary search + O(n) shift per insert); a set
// under the same total order gives the same answers in O(log n), which matters for policies
// with ~500k rules (tests/policy/perf/gen-policy.py's shape).
struct RuleLess {
    bool operator()(const ContivRule& a, const ContivRule& b) const { return a.compare(b) < 0; }
};
struct ContivRules {
    std::set<ContivRule, RuleLess> ordered;
    std::vector<ContivRule> rules;  // in insertion order (CopySlice)
    bool insert(const ContivRule& r);
};

// IPs of net1 not in net2, as subnets (configurator_impl.go:562-594)
std::vector<IPNet> subtract_subnet(const IPNet& net1, const IPNet& net2);
// utils.GetOneHostSubnetFromIP: /32 (IPv4) or /128 around the address
IPNet one_host_subnet(const Bytes& ip);

// A renderer as the configurator sees it (renderer.PolicyRendererAPI).
struct CfgRendererTxn {
    virtual ~CfgRendererTxn() = default;
    virtual void render(const PodID& pod, const IPNet* pod_ip, const std::vector<ContivRule>& ingress,
                        const std::vector<ContivRule>& egress, bool removed) = 0;
    virtual std::string commit() = 0;  // "" = ok
};
struct CfgRenderer {
    virtual ~CfgRenderer() = default;
    virtual std::unique_ptr<CfgRendererTxn> new_txn(bool resync) = 0;
};

// mock/renderer: stores what it is given; TestTraffic evaluates it
enum TrafficDirection { kIngressTraffic = 0, kEgressTraffic = 1 };
enum TrafficAction { kDeniedTraffic = 0, kAllowedTraffic = 1, kUnmatchedTraffic = 2 };
struct MockRenderer : CfgRenderer {
    struct Cfg {
        bool has_ip = false;
        IPNet ip;
        std::vector<ContivRule> ingress, egress;
    };
    std::map<PodID, Cfg> config;
    std::unique_ptr<CfgRendererTxn> new_txn(bool resync) override;
    int test_traffic(const PodID& pod, int direction, const Bytes& src, const Bytes& dst, int protocol,
                     uint16_t src_port, uint16_t dst_port) const;
    // TestTraffic on the device (pg_mock_renderer_install): the pod's ingress / egress list as a
    // first-match ACL named `name` (applied to an interface of that name, as the ACL engine
    // wants). A TCP / UDP rule matches its protocol and destination port (0 = any), an ANY rule
    // every packet, its ports ignored -- TestTraffic's semantics; the ACL's default slot =
    // UnmatchedTraffic. nullptr + *err: pod not rendered (*missing), or a rule this form cannot
    // hold (a source port, protocol OTHER; the configurator emits neither).
    ACLPtr traffic_acl(const PodID& pod, int direction, const std::string& name, std::string* err,
                       bool* missing) const;
};

struct PolicyConfigurator {
    // policy cache (LookupPod): pods known to the cache and their IP address ("" = none) ...
    std::map<PodID, std::string> pod_data;
    // ... or, when set, the K8s policy cache itself (k8s.hpp PolicyCache, wired by the processor)
    std::function<bool(const PodID&, std::string*)> lookup_pod;
    // IP address of a pod known to the cache; false = unknown pod
    bool pod_ip(const PodID& pod, std::string* ip) const {
        if (lookup_pod) return lookup_pod(pod, ip);
        auto it = pod_data.find(pod);
        if (it == pod_data.end()) return false;
        *ip = it->second;
        return true;
    }
    // IPAM.NatLoopbackIP(); empty Bytes = nil
    Bytes nat_loopback;
    std::vector<CfgRenderer*> renderers;
    std::map<PodID, IPNet> pod_ip_addresses;  // as rendered by the last Commit
};

struct PolicyConfiguratorTxn {
    PolicyConfigurator* cfg;
    bool resync;
    std::map<PodID, CfgPolicies> config;
    std::map<PodID, IPNet> pod_ip_addresses;
    PolicyConfiguratorTxn(PolicyConfigurator* c, bool rs);
    void configure(const PodID& pod, CfgPolicies policies) { config[pod] = std::move(policies); }
    std::string commit();
    ContivRules generate_rules(int direction, const CfgPolicies& policies) const;
};

}  // namespace pg
