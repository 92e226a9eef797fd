// The policy processor: turns K8s network policies into the per-pod
// ContivPolicy lists the configurator renders, re-processing the pods an event affects.
//
// Reference (itaimlx/vpp):
//   PolicyProcessor.Process                       plugins/policy/processor/processor.go:73-149
//   Resync / Add|Del|UpdatePod / ...Policy / ...Namespace   processor.go:151-316
//   filterHostPods                                processor.go:343-367
//   getPodsAssignedToPolicy / getPoliciesReferencingPod / ...Namespace   processor.go:369-527
//   calculateMatches / portNameToNumber           plugins/policy/processor/matches_calculator.go:14-221
//   is*LabelSelectorMatch / isMatchLabel / isMatchExpression
//                                                 plugins/policy/processor/match_label_selector.go:33-323
//
// Deterministic where the reference iterates Go maps: pods are processed in sorted order, so a
// policy whose ingress port is given by name resolves it against the first pod (in that order)
// that selects it, as the reference does against whichever pod its map yields first.
// Inputs the reference would dereference as nil (a policy without pod selector, a pod in a
// namespace the cache does not hold, a named port of a pod no longer cached) are read as empty.
#pragma once
#include <map>
#include <string>

#include "configurator.hpp"
#include "k8s.hpp"

namespace pg {

struct PolicyProcessor : PolicyCacheWatcher {
    PolicyCache* cache;
    PolicyConfigurator* configurator;
    IPNet pod_subnet_this_node;                 // IPAM.PodSubnetThisNode()
    std::map<std::string, Bytes> pod_ip_address_map;  // podIPAddressMap

    PolicyProcessor(PolicyCache* c, PolicyConfigurator* cfg, const IPNet& subnet);
    ~PolicyProcessor() override;

    std::string process(bool resync, std::vector<std::string> pods);

    std::string resync(const ResyncData& data) override;
    std::string add_pod(const std::string& id, const K8sPod& pod) override;
    std::string del_pod(const std::string& id, const K8sPod& pod) override;
    std::string update_pod(const std::string& id, const K8sPod& old_pod, const K8sPod& new_pod) override;
    std::string add_policy(const K8sPolicy& p) override;
    std::string del_policy(const K8sPolicy& p) override;
    std::string update_policy(const K8sPolicy& old_p, const K8sPolicy& new_p) override;
    std::string add_namespace(const K8sNamespace&) override { return ""; }
    std::string del_namespace(const K8sNamespace&) override { return ""; }
    std::string update_namespace(const K8sNamespace& old_ns, const K8sNamespace& new_ns) override;

    // building blocks, exposed for the parity tests
    std::vector<std::string> filter_host_pods(const std::vector<std::string>& pods) const;
    std::vector<CfgMatch> calculate_matches(const K8sPolicy& policy, const std::string& pod_id,
                                            std::string* err) const;
    std::vector<std::string> pods_assigned_to_policy(const K8sPolicy& policy) const;
    // sorted by policy ID
    std::vector<const K8sPolicy*> policies_referencing_pod(const K8sPod& pod) const;
    std::vector<const K8sPolicy*> policies_referencing_namespace(const K8sNamespace& ns) const;
};

}  // namespace pg
