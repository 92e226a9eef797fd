"""ctypes binding of include/policygpu.h (the same C ABI a cgo stub would bind).

The shared library is built in-tree (``vpp_amd/libpolicygpu.so``, see
``__graft_entry__.build()``). There is no fallback: if the library is missing the import
fails loudly, so nothing can silently run on the CPU.
"""
import ctypes as C
import os

try:
    # torch wheels bundle their own HIP runtime under the same SONAME (libamdhip64.so.7) as
    # /opt/rocm's; whichever is loaded first serves the whole process. Load torch's first so
    # torch-allocated HBM, torch streams and these kernels share one runtime.
    import torch  # noqa: F401
except ImportError:  # C-ABI users without torch (e.g. a cgo host) use the system runtime
    pass

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libpolicygpu.so")

PG_OK, PG_ENOENT, PG_EIO, PG_ENOMEM, PG_EINVAL, PG_EFAULT = 0, -2, -5, -12, -22, -14
MODE_SINGLE, MODE_PERPOD, MODE_CONN = 0, 1, 2
ORIENT_INGRESS, ORIENT_EGRESS = 0, 1


class pg_ipnet(C.Structure):
    _fields_ = [("family", C.c_uint8), ("prefix_len", C.c_uint8), ("_pad", C.c_uint8 * 2), ("addr", C.c_uint8 * 16)]


class pg_contiv_rule(C.Structure):
    _fields_ = [("action", C.c_int32), ("protocol", C.c_int32), ("src_port", C.c_uint16), ("dst_port", C.c_uint16),
                ("src", pg_ipnet), ("dst", pg_ipnet)]


class pg_port_range(C.Structure):
    _fields_ = [("lower_port", C.c_uint32), ("upper_port", C.c_uint32)]


class pg_l4(C.Structure):
    _fields_ = [("present", C.c_uint8), ("has_src_range", C.c_uint8), ("has_dst_range", C.c_uint8),
                ("_pad", C.c_uint8), ("src_range", pg_port_range), ("dst_range", pg_port_range)]


class pg_acl_rule(C.Structure):
    _fields_ = [("action", C.c_int32), ("has_macip_rule", C.c_uint8), ("has_ip_rule", C.c_uint8),
                ("has_ip", C.c_uint8), ("has_icmp", C.c_uint8), ("src_network", C.c_char_p),
                ("dst_network", C.c_char_p), ("tcp", pg_l4), ("udp", pg_l4)]


class pg_acl(C.Structure):
    _fields_ = [("name", C.c_char_p), ("rules", C.POINTER(pg_acl_rule)), ("n_rules", C.c_size_t),
                ("ingress", C.POINTER(C.c_char_p)), ("n_ingress", C.c_size_t),
                ("egress", C.POINTER(C.c_char_p)), ("n_egress", C.c_size_t)]


class pg_acl_op(C.Structure):
    _fields_ = [("key", C.c_char_p), ("value", C.POINTER(pg_acl))]


class pg_tuple_soa(C.Structure):
    _fields_ = [("src_ip", C.c_void_p), ("dst_ip", C.c_void_p), ("src_port", C.c_void_p),
                ("dst_port", C.c_void_p), ("proto", C.c_void_p)]


class pg_gen_spec(C.Structure):
    _fields_ = [("seed", C.c_uint64), ("index_base", C.c_uint64), ("table_id", C.c_int32),
                ("inside_pct", C.c_uint32), ("ip_pool", C.POINTER(C.c_uint32)), ("n_ip_pool", C.c_uint32),
                ("pool_pct", C.c_uint32), ("port_pool", C.POINTER(C.c_uint16)), ("n_port_pool", C.c_uint32),
                ("port_pool_pct", C.c_uint32), ("tcp_pct", C.c_uint32), ("udp_pct", C.c_uint32),
                ("zipf_cdf", C.POINTER(C.c_uint32)), ("nomatch_pct", C.c_uint32), ("dst_pool_pct", C.c_uint32)]


class pg_conn_query(C.Structure):
    _fields_ = [("kind", C.c_int32), ("src_namespace", C.c_char_p), ("src_name", C.c_char_p),
                ("dst_namespace", C.c_char_p), ("dst_name", C.c_char_p), ("src_ip", C.c_char_p),
                ("dst_ip", C.c_char_p), ("protocol", C.c_int32), ("src_port", C.c_uint16), ("dst_port", C.c_uint16)]


class pg_pod_id(C.Structure):
    _fields_ = [("ns", C.c_char_p), ("name", C.c_char_p)]


class pg_cfg_port(C.Structure):
    _fields_ = [("protocol", C.c_int32), ("number", C.c_uint16), ("_pad", C.c_uint16)]


class pg_ipblock(C.Structure):
    _fields_ = [("network", pg_ipnet), ("except_", C.POINTER(pg_ipnet)), ("n_except", C.c_size_t)]


class pg_match(C.Structure):
    _fields_ = [("type", C.c_int32), ("pods_nil", C.c_int32), ("pods", C.POINTER(pg_pod_id)), ("n_pods", C.c_size_t),
                ("blocks_nil", C.c_int32), ("_pad", C.c_int32), ("blocks", C.POINTER(pg_ipblock)),
                ("n_blocks", C.c_size_t), ("ports", C.POINTER(pg_cfg_port)), ("n_ports", C.c_size_t)]


class pg_policy(C.Structure):
    _fields_ = [("id", pg_pod_id), ("type", C.c_int32), ("_pad", C.c_int32), ("matches", C.POINTER(pg_match)),
                ("n_matches", C.c_size_t)]


class pg_session_rule(C.Structure):
    _fields_ = [("transport_proto", C.c_uint8), ("is_ip4", C.c_uint8), ("lcl_ip", C.c_uint8 * 16),
                ("lcl_plen", C.c_uint8), ("rmt_ip", C.c_uint8 * 16), ("rmt_plen", C.c_uint8),
                ("lcl_port", C.c_uint16), ("rmt_port", C.c_uint16), ("action_index", C.c_uint32),
                ("appns_index", C.c_uint32), ("scope", C.c_uint8), ("tag", C.c_char * 64)]


SNAP_GAUGE, SNAP_LOCAL, SNAP_CLUSTER = 0, 1, 2  # pg_counters_snapshot_range / pg_counter_of_rule

_P = C.c_void_p
_SIGS = {
    "pg_version": (C.c_char_p, []),
    "pg_create": (_P, [C.c_int]),
    "pg_destroy": (None, [_P]),
    "pg_set_tuning": (C.c_int, [C.c_char_p, C.c_int]),
    "pg_ctx_set_tuning": (C.c_int, [_P, C.c_char_p, C.c_int]),
    "pg_ctx_get_tuning": (C.c_int, [_P, C.c_char_p, C.POINTER(C.c_int)]),
    "pg_ctx_device": (C.c_int, [_P]),
    "pg_counters_snapshot": (C.c_int, [_P, C.POINTER(C.c_uint64), C.c_size_t]),
    "pg_counters_snapshot_range": (C.c_int, [_P, C.c_int, C.c_uint32, C.c_uint32, C.POINTER(C.c_uint64),
                                             C.POINTER(C.c_uint64)]),
    "pg_counter_of_rule": (C.c_int, [_P, C.c_int, C.c_char_p, C.c_int, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    "pg_counter_layout_gen": (C.c_uint64, [_P]),
    "pg_debug_set_snapshot": (C.c_int, [_P, C.c_int, C.POINTER(C.c_uint64), C.c_size_t]),
    "pg_debug_stream_slots": (C.c_int, [C.POINTER(C.c_uint64), C.c_size_t, C.POINTER(C.c_uint32),
                                        C.POINTER(C.c_uint32)]),
    "pg_comm_unique_id": (C.c_int, [C.c_char_p]),
    "pg_comm_init_rank": (C.c_int, [_P, C.c_int, C.c_char_p, C.c_int]),
    "pg_comm_init_all": (C.c_int, [C.POINTER(_P), C.c_int]),
    "pg_comm_destroy": (C.c_int, [_P]),
    "pg_comm_rank": (C.c_int, [_P, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    "pg_allreduce_counters": (C.c_int, [_P, _P]),
    "pg_allreduce_counters_all": (C.c_int, [C.POINTER(_P), C.c_int]),
    "pg_last_error": (C.c_char_p, [_P]),
    "pg_set_pod_if_name": (C.c_int, [_P, C.c_char_p, C.c_char_p, C.c_char_p]),
    "pg_set_host_interconnect_if_name": (C.c_int, [_P, C.c_char_p]),
    "pg_set_main_interface_name": (C.c_int, [_P, C.c_char_p]),
    "pg_set_other_vpp_interfaces": (C.c_int, [_P, C.POINTER(C.c_char_p), C.c_size_t]),
    "pg_set_vxlan_bvi_if_name": (C.c_int, [_P, C.c_char_p]),
    "pg_register_pod": (C.c_int, [_P, C.c_char_p, C.c_char_p, C.c_char_p, C.c_int]),
    "pg_renderer_new": (_P, [_P, C.c_int]),
    "pg_renderer_free": (None, [_P]),
    "pg_renderer_new_txn": (_P, [_P, C.c_int]),
    "pg_txn_render": (C.c_int, [_P, C.c_char_p, C.c_char_p, C.POINTER(pg_ipnet), C.POINTER(pg_contiv_rule),
                                C.c_size_t, C.POINTER(pg_contiv_rule), C.c_size_t, C.c_int]),
    "pg_txn_commit": (C.c_int, [_P]),
    "pg_txn_free": (None, [_P]),
    "pg_apply_txn": (C.c_int, [_P, C.c_int, C.POINTER(pg_acl_op), C.c_size_t]),
    "pg_num_acls": (C.c_int, [_P]),
    "pg_num_acl_changes": (C.c_int, [_P]),
    "pg_num_committed_txns": (C.c_int, [_P]),
    "pg_acl_json": (C.c_int, [_P, C.c_char_p, C.c_char_p, C.c_size_t]),
    "pg_acl_names_json": (C.c_int, [_P, C.c_char_p, C.c_size_t]),
    "pg_interface_acls": (C.c_int, [_P, C.c_char_p, C.c_char_p, C.c_size_t, C.c_char_p, C.c_size_t]),
    "pg_sync_tables": (C.c_int, [_P]),
    "pg_table_id": (C.c_int, [_P, C.c_char_p]),
    "pg_num_tables": (C.c_int, [_P]),
    "pg_num_counter_slots": (C.c_int, [_P]),
    "pg_slot_info": (C.c_int, [_P, C.c_uint32, C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
    "pg_table_info": (C.c_int, [_P, C.c_int, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]),
    "pg_classify":(C.c_int, [_P, C.c_int, C.c_int, C.POINTER(pg_tuple_soa), C.c_uint64, _P, _P, _P]),
    "pg_table_stats": (C.c_int, [_P, C.c_int, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), C.POINTER(C.c_uint32),
                                 C.POINTER(C.c_uint32)]),
    "pg_debug_walk_blob": (C.c_int, [_P, C.c_char_p, _P, _P, _P, _P, C.c_uint64, _P]),
    "pg_debug_classify_host": (C.c_int, [_P, C.c_int, C.c_int, C.POINTER(pg_tuple_soa), C.c_uint64, _P, _P,
                                         C.c_int]),
    "pg_node_stats": (C.c_int, [_P, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), C.POINTER(C.c_uint64),
                                C.POINTER(C.c_uint64)]),
    "pg_node_common_stats": (C.c_int, [_P, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    "pg_node_list_stats": (C.c_int, [_P, C.POINTER(C.c_uint64), C.POINTER(C.c_int)]),
    "pg_node_list_table_stats": (C.c_int, [_P, C.POINTER(C.c_uint64)]),
    "pg_node_uniform": (C.c_int, [_P]),
    "pg_configurator_new": (_P, []),
    "pg_configurator_free": (None, [_P]),
    "pg_configurator_last_error": (C.c_char_p, [_P]),
    "pg_configurator_register_renderer": (C.c_int, [_P, _P]),
    "pg_configurator_register_mock": (C.c_int, [_P, _P]),
    "pg_configurator_set_pod": (C.c_int, [_P, C.c_char_p, C.c_char_p, C.c_char_p]),
    "pg_configurator_set_nat_loopback": (C.c_int, [_P, C.c_char_p]),
    "pg_configurator_new_txn": (_P, [_P, C.c_int]),
    "pg_cfg_txn_configure": (C.c_int, [_P, C.c_char_p, C.c_char_p, C.POINTER(pg_policy), C.c_size_t]),
    "pg_cfg_txn_commit": (C.c_int, [_P]),
    "pg_cfg_txn_free": (None, [_P]),
    "pg_mock_renderer_new": (_P, []),
    "pg_mock_renderer_free": (None, [_P]),
    "pg_mock_renderer_pod_ip": (C.c_int, [_P, C.c_char_p, C.c_char_p, C.c_char_p, C.c_size_t, C.POINTER(C.c_int)]),
    "pg_mock_renderer_rules": (C.c_int, [_P, C.c_char_p, C.c_char_p, C.c_int, C.POINTER(pg_contiv_rule),
                                         C.c_size_t]),
    "pg_mock_renderer_test_traffic": (C.c_int, [_P, C.c_char_p, C.c_char_p, C.c_int, C.c_char_p, C.c_char_p, C.c_int,
                                                C.c_uint16, C.c_uint16]),
    "pg_policy_cache_new": (_P, []),
    "pg_policy_cache_free": (None, [_P]),
    "pg_policy_cache_last_error": (C.c_char_p, [_P]),
    "pg_policy_cache_register": (C.c_int, [_P, C.c_int, C.c_char_p, C.c_char_p, C.c_size_t]),
    "pg_policy_cache_unregister": (C.c_int, [_P, C.c_int, C.c_char_p]),
    "pg_policy_cache_update": (C.c_int, [_P, C.c_int, C.c_char_p, C.c_size_t, C.c_char_p, C.c_size_t]),
    "pg_policy_cache_resync": (C.c_int, [_P, C.POINTER(C.c_int), C.POINTER(C.c_char_p), C.POINTER(C.c_size_t),
                                         C.c_size_t]),
    "pg_policy_cache_lookup": (C.c_int, [_P, C.c_int, C.c_char_p, C.c_char_p, C.c_size_t, C.POINTER(C.c_size_t)]),
    "pg_policy_cache_query": (C.c_int, [_P, C.c_int, C.c_char_p, C.c_char_p, C.c_size_t, C.c_char_p, C.c_size_t,
                                        C.POINTER(C.c_size_t)]),
    "pg_policy_processor_new": (_P, [_P, _P, C.POINTER(pg_ipnet)]),
    "pg_policy_processor_free": (None, [_P]),
    "pg_policy_processor_process": (C.c_int, [_P, C.c_int, C.POINTER(C.c_char_p), C.c_size_t]),
    "pg_policy_processor_last_error": (C.c_char_p, [_P]),
    "pg_classify_linear": (C.c_int, [_P, C.c_int, C.POINTER(pg_tuple_soa), C.c_uint64, _P, _P]),
    "pg_debug_walk_stats": (C.c_int, [_P, C.c_int, C.POINTER(pg_tuple_soa), C.c_uint64, C.POINTER(C.c_uint32),
                                      C.POINTER(C.c_uint32), C.POINTER(C.c_int)]),
    "pg_stream_probe": (C.c_int, [_P, C.c_int, C.POINTER(pg_tuple_soa), C.c_uint64, _P, _P]),
    "pg_counters_device": (_P, [_P]),
    "pg_reset_counters": (C.c_int, [_P, _P]),
    "pg_read_counters": (C.c_int, [_P, C.POINTER(C.c_uint64), C.c_size_t]),
    "pg_gen_tuples": (C.c_int, [_P, C.POINTER(pg_gen_spec), C.c_uint64, _P, _P, _P, _P, _P, _P]),
    "pg_connections": (C.c_int, [_P, C.POINTER(pg_conn_query), C.c_size_t, C.POINTER(C.c_int32),
                                 C.POINTER(C.c_uint32)]),
    "pg_session_rules_new": (_P, [C.c_char_p]),
    "pg_session_rules_free": (None, [_P]),
    "pg_session_rules_clear": (C.c_int, [_P]),
    "pg_session_rules_counts": (C.c_int, [_P, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    "pg_session_rule_add_del": (C.c_int, [_P, C.POINTER(pg_session_rule), C.c_int]),
    "pg_session_rules_table": (C.c_int, [_P, C.c_int, C.c_uint32, C.POINTER(pg_session_rule), C.c_size_t]),
    "pg_session_rules_has_rule": (C.c_int, [_P, C.c_int, C.c_uint32, C.c_char_p, C.c_uint16, C.c_char_p,
                                            C.c_uint16, C.c_char_p, C.c_char_p]),
    "pg_appns_new": (_P, []),
    "pg_appns_free": (None, [_P]),
    "pg_appns_set": (C.c_int, [_P, C.c_char_p, C.c_char_p, C.c_uint32]),
    "pg_export_session_rules": (C.c_int, [_P, C.POINTER(pg_contiv_rule), C.c_size_t, C.c_char_p, C.c_char_p,
                                          C.POINTER(pg_ipnet), C.POINTER(pg_session_rule), C.c_size_t]),
    "pg_vpptcp_renderer_new": (_P, [_P, _P, C.c_int]),
    "pg_vpptcp_renderer_free": (None, [_P]),
    "pg_vpptcp_last_error": (C.c_char_p, [_P]),
    "pg_vpptcp_new_txn": (_P, [_P, C.c_int]),
    "pg_vpptcp_txn_render": (C.c_int, [_P, C.c_char_p, C.c_char_p, C.POINTER(pg_ipnet), C.POINTER(pg_contiv_rule),
                                       C.c_size_t, C.POINTER(pg_contiv_rule), C.c_size_t, C.c_int]),
    "pg_vpptcp_txn_commit": (C.c_int, [_P]),
    "pg_vpptcp_txn_free": (None, [_P]),
    "pg_configurator_register_vpptcp": (C.c_int, [_P, _P]),
    "pg_session_table_install": (C.c_int, [_P, _P, C.c_int, C.c_uint32, C.c_char_p]),
    "pg_mock_renderer_install": (C.c_int, [_P, _P, C.c_char_p, C.c_char_p, C.c_int, C.c_char_p]),
}
EXPORTED = sorted(_SIGS)


def load(path=LIB_PATH, partial=False):
    """partial: an A/B build of an earlier revision (tools/sweep.py) may lack entry points added
    since; they are left unbound instead of failing the load"""
    if not os.path.exists(path):
        raise ImportError("libpolicygpu.so not built (%s): run __graft_entry__.build()" % path)
    lib = C.CDLL(path)
    for name, (res, args) in _SIGS.items():
        if partial and not hasattr(lib, name):
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


# VPP_AMD_LIB: load an A/B build of the same library (tools/sweep.py); default the in-tree build
lib = load(os.environ.get("VPP_AMD_LIB", LIB_PATH), partial="VPP_AMD_LIB" in os.environ)
