/*
 * policygpu -- MI355X-native network-policy classification engine for Contiv-VPP.
 *
 * C ABI (the cgo boundary). Every entry point takes plain pointers and sizes; nothing here
 * retains a caller pointer after it returns (cgo pointer-passing rules). All calls are
 * synchronous from the caller's point of view unless a hip stream is passed, and a context
 * is not re-entrant (the reference drives the renderer from one event-loop goroutine,
 * plugins/controller/plugin_controller.go:428).
 *
 * Reference interfaces replaced (file:line under itaimlx/vpp):
 *   renderer.PolicyRendererAPI.NewTxn        plugins/policy/renderer/api.go:33-41
 *   renderer.Txn.Render / Txn.Commit         plugins/policy/renderer/api.go:44-61
 *   renderer.ContivRule                      plugins/policy/renderer/api.go:65-77
 *   acl.Renderer (Init/NewTxn/Commit)        plugins/policy/renderer/acl/acl_renderer.go:93-250
 *   MockACLEngine.ApplyTxn/PutACL/DelACL     mock/aclengine/aclengine_mock.go:151-228, 664-712
 *   MockACLEngine.RegisterPod                mock/aclengine/aclengine_mock.go:144-148
 *   MockACLEngine.Connection*                mock/aclengine/aclengine_mock.go:273-420
 *   MockACLEngine.evalACL / testConnection   mock/aclengine/aclengine_mock.go:424-652 (device)
 *   ipv4net.API getters used by the path     mock/ipv4net/ipv4net_mock.go:70-110
 *   contivconf main/other interfaces         plugins/policy/renderer/acl/acl_renderer.go:70-79
 *   statscollector.RegisterGaugeFunc sink    plugins/statscollector/plugin_impl_statscollector.go:248-261
 *                                            (pg_read_counters is the pull-style value source)
 */
#ifndef POLICYGPU_H
#define POLICYGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes (negative errno style) ---------------------------------------- */
#define PG_OK 0
#define PG_ENOENT (-2)    /* unknown pod / ACL / interface                               */
#define PG_EIO (-5)       /* HIP runtime error                                           */
#define PG_ENOMEM (-12)   /* host or device allocation failed                            */
#define PG_EINVAL (-22)   /* invalid argument                                            */
#define PG_EFAULT (-14)   /* the operation failed the way the reference's would (Commit / ApplyTxn error) */

/* ---- enums: values identical to the reference ------------------------------------ */
enum { PG_ACTION_DENY = 0, PG_ACTION_PERMIT = 1 };                 /* renderer.ActionType    */
enum { PG_PROTO_TCP = 0, PG_PROTO_UDP = 1, PG_PROTO_OTHER = 2, PG_PROTO_ANY = 3 }; /* ProtocolType */
enum { PG_ACL_DENY = 0, PG_ACL_PERMIT = 1, PG_ACL_REFLECT = 2, PG_ACL_FAILURE = 3 }; /* ACLAction */
enum { PG_CONN_DENY_SYN = 0, PG_CONN_DENY_SYN_ACK = 1, PG_CONN_ALLOW = 2, PG_CONN_FAILURE = 3 };
enum { PG_ORIENT_INGRESS = 0, PG_ORIENT_EGRESS = 1 };             /* cache.Orientation      */

/* net.IPNet: family 0 = empty network (&net.IPNet{}, "match all"), 4 or 6.
 * addr is the *unmasked* address as the caller holds it (IPv4 in addr[0..3]);
 * prefix_len is the mask's ones (net.CIDRMask(prefix_len, 32|128)).                    */
typedef struct pg_ipnet {
    uint8_t family;
    uint8_t prefix_len;
    uint8_t _pad[2];
    uint8_t addr[16];
} pg_ipnet;

/* renderer.ContivRule */
typedef struct pg_contiv_rule {
    int32_t action;    /* PG_ACTION_*  */
    int32_t protocol;  /* PG_PROTO_*   */
    uint16_t src_port; /* 0 = any      */
    uint16_t dst_port; /* 0 = any      */
    pg_ipnet src;
    pg_ipnet dst;
} pg_contiv_rule;

/* ---- vpp_acl.ACL wire model (vendor/github.com/ligato/vpp-agent/api/models/vpp/acl/acl.proto:24-113)
 * Strings are CIDRs as rendered by the reference ("" = field unset).                   */
typedef struct pg_port_range {
    uint32_t lower_port;
    uint32_t upper_port;
} pg_port_range;

typedef struct pg_l4 {
    uint8_t present;       /* section exists (ipRule.Tcp / ipRule.Udp != nil) */
    uint8_t has_src_range; /* SourcePortRange != nil                          */
    uint8_t has_dst_range; /* DestinationPortRange != nil                     */
    uint8_t _pad;
    pg_port_range src_range;
    pg_port_range dst_range;
} pg_l4;

typedef struct pg_acl_rule {
    int32_t action; /* vpp_acl.ACL_Rule_Action: 0 DENY, 1 PERMIT, 2 REFLECT */
    uint8_t has_macip_rule;
    uint8_t has_ip_rule;
    uint8_t has_ip;
    uint8_t has_icmp;
    const char* src_network;
    const char* dst_network;
    pg_l4 tcp;
    pg_l4 udp;
} pg_acl_rule;

typedef struct pg_acl {
    const char* name;
    const pg_acl_rule* rules;
    size_t n_rules;
    const char* const* ingress; /* Interfaces.Ingress */
    size_t n_ingress;
    const char* const* egress;  /* Interfaces.Egress  */
    size_t n_egress;
} pg_acl;

typedef struct pg_acl_op {
    const char* key;     /* "config/vpp/acls/v2/acl/<name>" (vpp_acl.Key) */
    const pg_acl* value; /* NULL = delete                                  */
} pg_acl_op;

/* ---- tuples (device pointers, SoA) ------------------------------------------------- */
typedef struct pg_tuple_soa {
    const uint32_t* src_ip;   /* host-order IPv4                      */
    const uint32_t* dst_ip;
    const uint16_t* src_port; /* only read by PG_MODE_CONN            */
    const uint16_t* dst_port;
    const uint8_t* proto;     /* PG_PROTO_*                           */
} pg_tuple_soa;

/* Classification modes.
 *  SINGLE: evalACL(table, src, dst, proto, dport) for one table         (configs 1,2,4)
 *  PERPOD: evalACL(outbound ACL of the interface the packet leaves by --
 *          dst pod's TAP or the node-output interface)                  (config 3)
 *  CONN:   testConnection over the src/dst interfaces resolved by IP    (config 5)
 * Output word: bits 31-30 = ACLAction (SINGLE/PERPOD) or ConnAction (CONN),
 *              bits 29-0  = counter slot of the deciding rule (see pg_num_counter_slots). */
enum { PG_MODE_SINGLE = 0, PG_MODE_PERPOD = 1, PG_MODE_CONN = 2 };
#define PG_VERDICT_ACTION(w) ((uint32_t)(w) >> 30)
#define PG_VERDICT_SLOT(w) ((uint32_t)(w)&0x3FFFFFFFu)

/* ---- engine context (one GPU) ------------------------------------------------------ */
typedef struct pg_ctx pg_ctx;
typedef struct pg_renderer pg_renderer;
typedef struct pg_txn pg_txn;

/* One context per GPU. Every call that touches the device makes hip_device current for its
 * duration and restores the caller's current device afterwards, so contexts on different GPUs
 * can be driven from one process, and a cgo caller may call from any OS thread. A context is
 * not re-entrant; distinct contexts may be used concurrently from different threads. */
pg_ctx* pg_create(int hip_device);
int pg_ctx_device(const pg_ctx* ctx);
/* Tuning knobs (key, value):
 * launches -- "blocks_per_cu" (cap on resident workgroups per CU of the classify grid;
 * default 0 = as many as registers/LDS allow), "stage_max_words" (largest table blob staged
 * in LDS, default 16384 = 64 KiB), "stage_root_max_words" (larger blobs: header + src-trie
 * root staged, default 16400), "node_path" (1/0: classify PERPOD / CONN through the node
 * classifier when it exists, default 1; 0 = per-table blobs and the IP hash),
 * "node_stage_max_words" (largest node image staged in LDS, default 16384),
 * "node_common_lds_max" (LDS bytes up to which the node image's common-row section is staged,
 * default 80 KiB), "block_stage" (workgroup size of LDS-staged classify launches: 256, 512 or
 * 1024; default 0 = per mode), "hist_window" (hit counters of a table set with more than 16382
 * slots: LDS cells kept for the classified table's first rules -- its default-deny slot and last
 * rule always get one -- the rest counted with global atomics; default 4096), "node_hist_cells"
 * (PERPOD / CONN launches over a table set with more than 16382 slots: cells of the LDS cache the
 * hit counters go through -- the hottest slots of each workgroup's stream claim them, the rest
 * take global atomics -- rounded down to a power of two, up to 8192; default 256, < 16 = none);
 * table compiler (the context recompiles and re-uploads on its next use; hit counters carry over)
 * -- "root_bits_max" (cap of the src/key trie root stride, 4..16, default 16), "node_build"
 * (1/0: build the node classifier for PERPOD / CONN, default 1), "node_root_bits" (its IPv4 /
 * key trie root stride cap, default 12), "node_key_root_bits" (cap of the uniform layout's
 * key trie root stride, 2..10; the strides tried are 2, 6 and 10 (18 - root a multiple of 4),
 * so the cap is rounded down to one of them -- 10 saves a level for ~4 KiB of image; default
 * 6), "lc_lds" (table blobs of at least this many words are
 * rebuilt with level-compressed 12/16-bit trie strides and keep them when the result still
 * fits in LDS; default 4096, 0 = off; blobs too large for LDS are always level-compressed),
 * "lc_dense12" (boundaries a subtree needs for a 12-bit stride, default 16), "lc_max_stride"
 * (widest level-compressed stride: 12, 16 or 18, default 16), "lc_root_bits" (src-trie root
 * stride cap of blobs read from HBM, whose root alone a launch stages in LDS: 4..14, default
 * 13), "candi" (1/0: candidates inline in the 8-B trie entries of HBM-resident candidate tables
 * no live rule of which tests dst, default 1), "candi_window_bits" (such a table's LDS window:
 * the terminal entries of the 2^bits addresses of the aligned window where its earliest rules
 * sit, staged with the root, so a lookup there makes no trie gather; 0..13, 0 = none, default
 * 11; left out when it would not stage with the root), "candi_window_root_bits" (root stride cap
 * of a table with a window, default 12: root + window in 32 KiB), "fd" (1/0: fixed-depth form of dst-independent
 * cross-product tables, default 1), "node_common" (1/0: common-row section of node
 * images, default 1), "node_uniform" (1/0: the node's uniform cross layout where every table
 * is covered and none is in PAIR form, default 1), "node_list_table" (1/0: in the uniform layout
 * a node cross entry whose table still has dst-specific rules ahead of its verdict resolves them
 * by one read of a list-verdict table indexed by the dst's node IP class -- the IPv4 classes then
 * also separate those rules' dst prefixes -- instead of walking dst records; 0 = records, which
 * rules the uniform layout out for a set with such rules; default 1), "node_list_words"
 * (record form: node dst records up to this many words go into the node image, so a launch that
 * stages the image walks them in LDS; default 4096, 0 = never), "pair" (1/0: the PAIR structure -- src x dst classes, then x key classes
 * -- for tables the cross product cannot take, default 1; 0 = candidate lists; 2 = wherever it
 * fits, for tests), "launch_max_tuples" (a pg_classify batch larger than this takes several
 * kernel launches of at most this many tuples, in order on the stream; a multiple of 64, 0 =
 * the largest a launch's 32-bit stream offsets allow, 2^30 - 64; default 0).
 * pg_ctx_set_tuning sets one context's knob; pg_set_tuning sets the process default that
 * contexts created afterwards start from. PG_EINVAL for an unknown key or a value out of range. */
int pg_ctx_set_tuning(pg_ctx* ctx, const char* key, int value);
int pg_ctx_get_tuning(const pg_ctx* ctx, const char* key, int* value); /* ctx NULL: process default */
int pg_set_tuning(const char* key, int value);
void pg_destroy(pg_ctx* ctx);
const char* pg_last_error(const pg_ctx* ctx);
const char* pg_version(void);

/* ipv4net / contivconf roles the renderer and the engine depend on */
int pg_set_pod_if_name(pg_ctx* ctx, const char* pod_namespace, const char* pod_name, const char* if_name);
int pg_set_host_interconnect_if_name(pg_ctx* ctx, const char* if_name);
int pg_set_main_interface_name(pg_ctx* ctx, const char* if_name);
int pg_set_other_vpp_interfaces(pg_ctx* ctx, const char* const* if_names, size_t n);
int pg_set_vxlan_bvi_if_name(pg_ctx* ctx, const char* if_name);
/* MockACLEngine.RegisterPod */
int pg_register_pod(pg_ctx* ctx, const char* pod_namespace, const char* pod_name, const char* ip, int another_node);

/* ---- renderer (PolicyRendererAPI) -------------------------------------------------- */
pg_renderer* pg_renderer_new(pg_ctx* ctx, int orientation);
void pg_renderer_free(pg_renderer* r);
pg_txn* pg_renderer_new_txn(pg_renderer* r, int resync);
int pg_txn_render(pg_txn* txn, const char* pod_namespace, const char* pod_name, const pg_ipnet* pod_ip,
                  const pg_contiv_rule* ingress, size_t n_ingress, const pg_contiv_rule* egress, size_t n_egress,
                  int removed);
int pg_txn_commit(pg_txn* txn); /* renders, applies to the engine, frees txn */
void pg_txn_free(pg_txn* txn);  /* abandon without commit                    */

/* ---- ACL ingestion (vpp-agent key space) and introspection -------------------------- */
int pg_apply_txn(pg_ctx* ctx, int resync, const pg_acl_op* ops, size_t n_ops);
int pg_num_acls(pg_ctx* ctx);
int pg_num_acl_changes(pg_ctx* ctx);
int pg_num_committed_txns(pg_ctx* ctx);
/* JSON of one ACL ({"name","ingress","egress","rules":[...]}) -> bytes needed (incl. NUL). */
int pg_acl_json(pg_ctx* ctx, const char* acl_name, char* buf, size_t cap);
/* JSON array of all installed ACL names (sorted) -> bytes needed (incl. NUL) */
int pg_acl_names_json(pg_ctx* ctx, char* buf, size_t cap);
/* names of the ACLs bound to an interface ("" when none) */
int pg_interface_acls(pg_ctx* ctx, const char* if_name, char* inbound, size_t in_cap, char* outbound,
                      size_t out_cap);

/* ---- device tables and classification ---------------------------------------------- */
int pg_sync_tables(pg_ctx* ctx); /* compile + upload (double-buffered swap); implicit in classify */
int pg_table_id(pg_ctx* ctx, const char* acl_name);
int pg_num_tables(pg_ctx* ctx);
int pg_num_counter_slots(pg_ctx* ctx);
/* global rule slot -> (table id, rule index in its ACL); rule index -1 for a table's
 * default-deny slot; table id -1 for the "no ACL" (permit) slot */
int pg_slot_info(pg_ctx* ctx, uint32_t slot, int32_t* table_id, int32_t* rule_index);
/* table -> (first rule slot, rules, default-deny slot) */
int pg_table_info(pg_ctx* ctx, int table_id, uint32_t* rule_base, uint32_t* n_rules, uint32_t* default_slot);

/* classification structure of a table: flags (1 cross, 2 dst lists, 4 candidate mode,
 * 8 linear fallback), blob bytes, src / key equivalence classes */
int pg_table_stats(pg_ctx* ctx, int table_id, uint32_t* flags, uint32_t* blob_bytes, uint32_t* n_src_classes,
                   uint32_t* n_key_classes);

int pg_classify(pg_ctx* ctx, int mode, int table_id, const pg_tuple_soa* tuples, uint64_t n, uint32_t* out,
                uint64_t* counters, void* hip_stream);

/* TESTS ONLY -- never on the classify path: walk one ACL's compiled classification blob on
 * the host (the same walk code the kernels instantiate) for n host tuples, so the table
 * compiler can be checked against the oracle without a GPU. Does not touch the device. */
int pg_debug_walk_blob(pg_ctx* ctx, const char* acl_name, const uint32_t* src, const uint32_t* dst,
                       const uint16_t* dst_port, const uint8_t* proto, uint64_t n, uint32_t* out);
/* TESTS ONLY -- never on the classify path: pg_classify's per-tuple code (classify.hpp, the
 * same templates the kernels instantiate) run on the host over host tuples, any mode, with
 * optional host u64 counters. flags: bit 0 = node classifier when it exists (else the
 * per-table path), bit 1 = the predicated trie walks the kernels use on LDS-staged images
 * (else the branching ones they use on HBM-resident ones), bit 2 = the node image's
 * common-row section when it was built (the kernels use it when it fits their LDS budget).
 * Does not touch the device. */
int pg_debug_classify_host(pg_ctx* ctx, int mode, int table_id, const pg_tuple_soa* tuples, uint64_t n,
                           uint32_t* out, uint64_t* counters, int flags);
/* TESTS ONLY -- never on the classify path: install n host counters (e.g. from
 * pg_debug_classify_host) as the LOCAL or CLUSTER snapshot in the currently compiled slot layout,
 * so the snapshot readers below can be tested without a GPU. n must equal the slot count. */
int pg_debug_set_snapshot(pg_ctx* ctx, int which, const uint64_t* counters, size_t n);
/* TESTS ONLY -- never on the classify path: the per-stream launch-mark bookkeeping of PERPOD / CONN launches
 * (device.hpp StreamSlots, which pg_classify uses to hand a launch's deferred ANY-protocol packets
 * to the k_node_any launched after it on the same stream) replayed for n launches on the given
 * stream handles: slot_out[k] = the mark word launch k writes, seq_out[k] = its launch number. No
 * device work. */
int pg_debug_stream_slots(const uint64_t* streams, size_t n, uint32_t* slot_out, uint32_t* seq_out);
/* TESTS / MEASUREMENT ONLY -- never on the classify path: per tuple, the loads a SINGLE-mode
 * launch on table_id makes of the table's classification structure, split by where the launch
 * finds the word: lds_reads (the LDS-staged part) and mem_reads (HBM / L2 gathers; rule reads of
 * the linear scan for ANY-protocol packets). *stage = the staging the launch uses (device.hip
 * k_classify STAGE: 0 none, 1 blob, 2 src root, 4 FD blob, 5 FD prefix). Runs the kernels' walk
 * code on the host with counting loaders; does not touch the device. */
int pg_debug_walk_stats(pg_ctx* ctx, int table_id, const pg_tuple_soa* tuples, uint64_t n, uint32_t* lds_reads,
                        uint32_t* mem_reads, int* stage);
/* node classifier (PERPOD / CONN) size: IPv4 classes, L4-key classes, LDS image bytes,
 * cross-table bytes; PG_ENOENT when it was not built */
int pg_node_stats(pg_ctx* ctx, uint32_t* ip_classes, uint32_t* key_classes, uint64_t* image_bytes,
                  uint64_t* cross_bytes);
/* node image layout: bytes of the base image (without the common-row section), and how many of
 * the covered (table, IPv4 class) pairs read the table's common row from the image instead of
 * the cross table (0 when the section was not built); PG_ENOENT when there is no node */
int pg_node_common_stats(pg_ctx* ctx, uint64_t* base_image_bytes, uint64_t* common_pairs, uint64_t* pairs);
/* the node classifier's dst records (the dst-specific rules its cross entries still test, record
 * form): their bytes, and whether a copy ends the node image (tuning "node_list_words"); 0 bytes in
 * the list-table form (pg_node_list_table_stats); PG_ENOENT: no node */
int pg_node_list_stats(pg_ctx* ctx, uint64_t* record_bytes, int* in_image);
/* the node classifier's list-verdict table (tuning "node_list_table"): its bytes in the cross
 * array (0 = the record form, or no lists); PG_ENOENT: no node */
int pg_node_list_table_stats(pg_ctx* ctx, uint64_t* table_bytes);
/* 1 when the node classifier uses the uniform cross layout (every table covered, none in PAIR
 * form, tuning "node_uniform": entry addresses computed, no per-table info reads), 2 when it does
 * with wide class records (255 tables or more: 16-bit table ids, 32-bit common-row marks), else
 * 0; PG_ENOENT: no node */
int pg_node_uniform(pg_ctx* ctx);
/* reference-shaped linear-scan kernel (K1) on one table, for validation and comparison */
int pg_classify_linear(pg_ctx* ctx, int table_id, const pg_tuple_soa* tuples, uint64_t n, uint32_t* out,
                       void* hip_stream);
/* MEASUREMENT -- not part of the reference's interface: the stream ceiling of a pg_classify
 * launch. Issues exactly the loads a launch makes of the tuple fields (src, dst_port, proto;
 * dst_ip when fields & 1, src_port when fields & 2) and its 4-B store per tuple, with the same
 * vector widths and grid, but no classification (out[i] = xor of the fields). bench.py times
 * it beside the classify kernel: classify rate / probe rate = how close the classification
 * comes to what moving its own bytes costs on this GPU. Fields and out must be vector-aligned
 * (16-B src / dst / out); PG_EIO otherwise. */
int pg_stream_probe(pg_ctx* ctx, int fields, const pg_tuple_soa* tuples, uint64_t n, uint32_t* out,
                    void* hip_stream);
/* device-resident per-rule hit counters (u64, pg_num_counter_slots entries) */
uint64_t* pg_counters_device(pg_ctx* ctx);
int pg_reset_counters(pg_ctx* ctx, void* hip_stream);
/* waits for this context's classify launches, copies min(n, slots) counters -> slots copied
 * (also refreshes the LOCAL host snapshot) */
int pg_read_counters(pg_ctx* ctx, uint64_t* host_out, size_t n);
/* ---- host snapshots: the statscollector value source -----------------------------------
 * (RegisterGaugeFunc, plugin_impl_statscollector.go:248-261: a pull-style gauge whose value
 * function runs at scrape time, on its own goroutine.) The library keeps two host copies of the
 * counters, each with the slot layout it was counted in; reading them never touches the GPU and
 * is safe from any thread while the context classifies:
 *   PG_SNAP_LOCAL    this GPU's counts, as of the last pg_read_counters
 *   PG_SNAP_CLUSTER  the sum over the communicator, as of the last pg_allreduce_counters*
 *   PG_SNAP_GAUGE    CLUSTER once the context has a communicator, else LOCAL: a monotonic
 *                    source either way (neither call writes the other's copy)
 * Slots are renumbered whenever the tables are recompiled, so a gauge should be keyed by a
 * stable rule identity -- (ACL name, rule index) -- and read with pg_counter_of_rule, which
 * resolves it in the snapshot's own layout. Counts survive a recompile: every ACL present before
 * and after it under the same name with the same rules keeps its counts (its rules and its
 * default deny), as do "no ACL" and "unresolved" -- in the device counters (carried to the new
 * slots when the new tables are uploaded) and in both host snapshots (when they are compiled);
 * the slots of new or changed ACLs start at zero. */
enum { PG_SNAP_GAUGE = 0, PG_SNAP_LOCAL = 1, PG_SNAP_CLUSTER = 2 };
/* PG_SNAP_GAUGE snapshot: copies min(n, slots) -> number of slots in it (0 before the first read) */
int pg_counters_snapshot(const pg_ctx* ctx, uint64_t* host_out, size_t n);
/* slots [first, first + n) of a snapshot (clipped to its size) -> number copied; *layout_gen
 * (optional) = the layout generation of that snapshot (0: none taken yet) */
int pg_counters_snapshot_range(const pg_ctx* ctx, int which, uint32_t first, uint32_t n, uint64_t* host_out,
                               uint64_t* layout_gen);
/* one rule's count in a snapshot by its stable identity: ACL name and rule index (-1: the ACL's
 * default deny); acl_name NULL with rule_index -1 = the "no ACL" slot, -2 = the unresolved-
 * interface slot. O(log ACLs), no allocation. PG_ENOENT: no snapshot yet, or the ACL / index
 * does not exist in the snapshot's layout. *layout_gen (optional) as above. */
int pg_counter_of_rule(const pg_ctx* ctx, int which, const char* acl_name, int rule_index, uint64_t* value,
                       uint64_t* layout_gen);
/* generation of the compiled slot layout (increments on every recompile; 0 = never compiled):
 * an agent re-registers gauges for new (ACL, rule) identities when it changes. Any thread. */
uint64_t pg_counter_layout_gen(const pg_ctx* ctx);

/* ---- RCCL over xGMI: per-rule hit counters summed over the GPUs of a node -------------
 * (the statscollector path). The classify path itself has no exchange.
 * Multi-process (one process per GPU): rank 0 calls pg_comm_unique_id and hands the bytes to
 * the other ranks (any side channel), every rank calls pg_comm_init_rank on its context.
 * One process driving several GPUs: pg_comm_init_all over one context per GPU.
 * pg_allreduce_counters / pg_allreduce_counters_all first check that every rank compiled the
 * same counter layout (slots, ACL names, rules per ACL; PG_EFAULT if not, nothing reduced), then
 * sum a device copy of the counters (ncclAllReduce u64 sum) into the host snapshots. The
 * device counters keep this rank's own counts (pg_read_counters still returns them), so a
 * periodic gauge may all-reduce again without a reset in between. The caller's current device
 * is restored on every return path.
 * Synchronous. RCCL (librccl.so.1) is loaded on first use. */
#define PG_COMM_ID_BYTES 128
int pg_comm_unique_id(uint8_t id[PG_COMM_ID_BYTES]);
int pg_comm_init_rank(pg_ctx* ctx, int nranks, const uint8_t id[PG_COMM_ID_BYTES], int rank);
int pg_comm_init_all(pg_ctx* const* ctxs, int n);
int pg_comm_destroy(pg_ctx* ctx);
int pg_comm_rank(const pg_ctx* ctx, int* rank, int* nranks); /* PG_ENOENT: no communicator */
int pg_allreduce_counters(pg_ctx* ctx, void* hip_stream);
int pg_allreduce_counters_all(pg_ctx* const* ctxs, int n);

/* ---- synthetic input generation on device (bench / parity workloads) ----------------- */
typedef struct pg_gen_spec {
    uint64_t seed;
    uint64_t index_base;      /* global index of tuple 0 (multi-GPU shards)               */
    int32_t table_id;         /* >= 0: "inside a rule" sampling from this table           */
    uint32_t inside_pct;      /* % of tuples sampled inside a rule's predicate            */
    const uint32_t* ip_pool;  /* host array: pool of "known" IPs (pods / internet hosts)  */
    uint32_t n_ip_pool;
    uint32_t pool_pct;        /* % of src/dst drawn from ip_pool (else uniform u32)       */
    const uint16_t* port_pool;/* host array of popular dst ports                          */
    uint32_t n_port_pool;
    uint32_t port_pool_pct;   /* % of dst ports drawn from port_pool                      */
    uint32_t tcp_pct, udp_pct;/* protocol mix (rest OTHER)                                */
    const uint32_t* zipf_cdf; /* host array, n_rules+1 entries scaled to 2^32: rule index  *
                               * follows it (config 4); NULL = uniform rule choice        */
    uint32_t nomatch_pct;     /* % forced outside every rule's src (config 4)             */
    uint32_t dst_pool_pct;    /* % of dst drawn from ip_pool (config 3/5: local pods)     */
} pg_gen_spec;

int pg_gen_tuples(pg_ctx* ctx, const pg_gen_spec* spec, uint64_t n, uint32_t* src_ip, uint32_t* dst_ip,
                  uint16_t* src_port, uint16_t* dst_port, uint8_t* proto, void* hip_stream);

/* ---- Connection* (MockACLEngine) evaluated on the device ------------------------------ */
typedef struct pg_conn_query {
    int32_t kind;              /* 0 PodToPod, 1 PodToInternet, 2 InternetToPod */
    const char* src_namespace; /* pod endpoints                                  */
    const char* src_name;
    const char* dst_namespace;
    const char* dst_name;
    const char* src_ip;        /* internet endpoints (string, net.ParseIP)       */
    const char* dst_ip;
    int32_t protocol;
    uint16_t src_port;
    uint16_t dst_port;
} pg_conn_query;
/* out[i] = ConnAction; out_slot (optional) = deciding slot per query */
int pg_connections(pg_ctx* ctx, const pg_conn_query* q, size_t n, int32_t* out, uint32_t* out_slot);

/* ---- policy configurator ------------------------------------------
 * configurator.PolicyConfiguratorAPI / Txn (plugins/policy/configurator/configurator_api.go:28-54,
 * configurator_impl.go:104-472): K8s-shaped policies per pod -> ordered ContivRule lists
 * rendered into every registered renderer (the GPU ACL renderer and/or mock renderers).
 * The policy cache's pod data (LookupPod) and the IPAM NAT-loopback address are set
 * explicitly. Go nil-vs-empty matters for Match.Pods / IPBlocks: *_nil = 1 means nil. */
enum { PG_POLICY_INGRESS = 0, PG_POLICY_EGRESS = 1, PG_POLICY_ALL = 2 }; /* configurator.PolicyType */
enum { PG_MATCH_INGRESS = 0, PG_MATCH_EGRESS = 1 };                       /* configurator.MatchType  */
enum { PG_PORT_TCP = 0, PG_PORT_UDP = 1 };                                /* configurator.ProtocolType */
typedef struct pg_pod_id {
    const char* ns;
    const char* name;
} pg_pod_id;
typedef struct pg_cfg_port { /* configurator.Port */
    int32_t protocol;
    uint16_t number;
    uint16_t _pad;
} pg_cfg_port;
typedef struct pg_ipblock { /* configurator.IPBlock */
    pg_ipnet network;
    const pg_ipnet* except;
    size_t n_except;
} pg_ipblock;
typedef struct pg_match { /* configurator.Match */
    int32_t type;
    int32_t pods_nil;
    const pg_pod_id* pods;
    size_t n_pods;
    int32_t blocks_nil;
    int32_t _pad;
    const pg_ipblock* blocks;
    size_t n_blocks;
    const pg_cfg_port* ports;
    size_t n_ports;
} pg_match;
typedef struct pg_policy { /* configurator.ContivPolicy */
    pg_pod_id id;
    int32_t type;
    int32_t _pad;
    const pg_match* matches;
    size_t n_matches;
} pg_policy;

typedef struct pg_configurator pg_configurator;
typedef struct pg_cfg_txn pg_cfg_txn;
typedef struct pg_mock_renderer pg_mock_renderer;

pg_configurator* pg_configurator_new(void);
void pg_configurator_free(pg_configurator* c);
const char* pg_configurator_last_error(const pg_configurator* c);
/* PolicyConfigurator.RegisterRenderer (configurator_impl.go:104-107); the renderer must
 * outlive the configurator's transactions */
int pg_configurator_register_renderer(pg_configurator* c, pg_renderer* r);
int pg_configurator_register_mock(pg_configurator* c, pg_mock_renderer* r);
/* policy cache LookupPod data: ip = NULL removes the pod, "" = known without an address */
int pg_configurator_set_pod(pg_configurator* c, const char* ns, const char* name, const char* ip);
/* IPAM.NatLoopbackIP() (net.ParseIP form; NULL or unparsable = nil) */
int pg_configurator_set_nat_loopback(pg_configurator* c, const char* ip);
pg_cfg_txn* pg_configurator_new_txn(pg_configurator* c, int resync);
/* Txn.Configure: replaces the pod's set of policies (copied) */
int pg_cfg_txn_configure(pg_cfg_txn* t, const char* ns, const char* name, const pg_policy* policies, size_t n);
/* Txn.Commit: renders every configured pod into every renderer and commits them; frees t.
 * PG_EFAULT (message in pg_configurator_last_error) when a renderer's Commit failed. */
int pg_cfg_txn_commit(pg_cfg_txn* t);
void pg_cfg_txn_free(pg_cfg_txn* t);

/* mock/renderer.MockRenderer (mock/renderer/renderer_mock.go:39-185): stores the rendered
 * lists; TestTraffic evaluates them. direction: 0 = INGRESS (from the pod
 * to the vswitch), 1 = EGRESS; result: 0 DENIED, 1 ALLOWED, 2 UNMATCHED. */
pg_mock_renderer* pg_mock_renderer_new(void);
void pg_mock_renderer_free(pg_mock_renderer* r);
/* GetPodIP: writes the address ("" when unknown) and the mask length */
int pg_mock_renderer_pod_ip(pg_mock_renderer* r, const char* ns, const char* name, char* ip, size_t cap,
                            int* masklen);
/* the pod's ingress/egress list in rendered order -> number of rules (PG_ENOENT: no pod) */
int pg_mock_renderer_rules(pg_mock_renderer* r, const char* ns, const char* name, int direction,
                           pg_contiv_rule* out, size_t cap);
int pg_mock_renderer_test_traffic(pg_mock_renderer* r, const char* ns, const char* name, int direction,
                                  const char* src_ip, const char* dst_ip, int protocol, uint16_t src_port,
                                  uint16_t dst_port);
/* TestTraffic on the device: the pod's ingress (direction 0) / egress (1) list of r installed
 * in ctx as the ACL acl_name (a put, as by pg_apply_txn; again after a new Commit), so that
 * pg_classify(ctx, PG_MODE_SINGLE, pg_table_id(ctx, acl_name), ...) answers TestTraffic for
 * a batch: PERMIT = AllowedTraffic, DENY = DeniedTraffic (with the rule's slot), the ACL's
 * default slot = UnmatchedTraffic. Tuples carry the ContivRule protocol (TCP 0 / UDP 1 /
 * OTHER 2) and the destination port; TestTraffic's source-port test needs no field because
 * the configurator never sets a rule's source port -- a list that has one (or a protocol-OTHER
 * rule) is refused with PG_EINVAL. PG_ENOENT: the pod was not rendered (TestTraffic:
 * UnmatchedTraffic for every packet). */
int pg_mock_renderer_install(pg_ctx* ctx, const pg_mock_renderer* r, const char* ns, const char* name, int direction,
                             const char* acl_name);

/* ---- K8s policy cache and processor ------------------------------
 * The KSR objects cross the boundary in their protobuf wire form (proto.Marshal of
 * plugins/ksr/model/{pod,namespace,policy}.Pod / Namespace / Policy), so the Go side
 * passes what it holds. policy.Policy_LabelSelector travels the same way for queries.
 * cache.PolicyCacheAPI (plugins/policy/cache/cache_api.go:30-116, cache_impl.go),
 * processor.PolicyProcessor (plugins/policy/processor/processor.go:34-527). Name lists come
 * back sorted and '\n'-joined (the reference returns them in Go map order). */
typedef struct pg_policy_cache pg_policy_cache;
typedef struct pg_policy_processor pg_policy_processor;
enum { PG_K8S_POD = 0, PG_K8S_NAMESPACE = 1, PG_K8S_POLICY = 2 };
enum {
    PG_Q_PODS_BY_LABEL_SELECTOR_INSIDE_NS = 0, /* arg = namespace, selector        */
    PG_Q_PODS_BY_NS_LABEL_SELECTOR = 1,        /* selector                         */
    PG_Q_PODS_BY_NAMESPACE = 2,                /* arg = namespace                  */
    PG_Q_ALL_PODS = 3,
    PG_Q_POLICIES_BY_POD = 4,                  /* arg = "ns/name"                  */
    PG_Q_ALL_POLICIES = 5,
    PG_Q_ALL_NAMESPACES = 6,
    PG_Q_MATCH_LABEL_PODS_INSIDE_NS = 7,       /* arg = namespace, selector labels (match_label.go) */
    PG_Q_PODS_BY_NS_LABELS = 8,                /* selector labels                  */
    PG_Q_MATCH_EXPRESSION_PODS_INSIDE_NS = 9,  /* arg = namespace, selector expressions (match_expression.go) */
    PG_Q_PODS_BY_NS_EXPRESSIONS = 10,          /* selector expressions             */
    /* secondary indexes (podmap.go / namespacemap.go / policymap.go), arg = index value */
    PG_Q_IDX_POD_LABEL = 11, PG_Q_IDX_POD_KEY = 12, PG_Q_IDX_POD_NS_LABEL = 13, PG_Q_IDX_POD_NS_KEY = 14,
    PG_Q_IDX_NS_LABEL = 15, PG_Q_IDX_NS_KEY = 16, PG_Q_IDX_POLICY_LABEL = 17, PG_Q_IDX_POLICY_NS_LABEL = 18
};
pg_policy_cache* pg_policy_cache_new(void);
void pg_policy_cache_free(pg_policy_cache* c);
const char* pg_policy_cache_last_error(const pg_policy_cache* c);
/* ConfigIndex.Register* / Unregister* (index only, no events); pb NULL = a nil object.
 * unregister -> 1 found, 0 not */
int pg_policy_cache_register(pg_policy_cache* c, int kind, const char* id, const uint8_t* pb, size_t len);
int pg_policy_cache_unregister(pg_policy_cache* c, int kind, const char* id);
/* Update (data_change.go): prev NULL = add, next NULL = delete, both = update; the
 * watchers (processor) run inside. PG_EFAULT + last_error when a watcher fails. */
int pg_policy_cache_update(pg_policy_cache* c, int kind, const uint8_t* prev, size_t prev_len, const uint8_t* next,
                           size_t next_len);
/* Resync (data_resync.go): the whole K8s state, n objects of the given kinds */
int pg_policy_cache_resync(pg_policy_cache* c, const int* kinds, const uint8_t* const* objs, const size_t* lens,
                           size_t n);
/* Lookup{Pod,Namespace,Policy}: 1 found (wire bytes as registered -> out, *out_len; a nil
 * object has *out_len = (size_t)-1), 0 not found */
int pg_policy_cache_lookup(const pg_policy_cache* c, int kind, const char* id, uint8_t* out, size_t cap,
                           size_t* out_len);
/* name-list queries -> number of names; '\n'-joined into out when *out_len (bytes, no NUL)
 * fits cap */
int pg_policy_cache_query(const pg_policy_cache* c, int query, const char* arg, const uint8_t* selector,
                          size_t selector_len, char* out, size_t cap, size_t* out_len);
/* PolicyProcessor watching the cache and configuring cfg (which then looks pods up in the
 * cache); pod_subnet = IPAM.PodSubnetThisNode() */
pg_policy_processor* pg_policy_processor_new(pg_policy_cache* c, pg_configurator* cfg, const pg_ipnet* pod_subnet);
void pg_policy_processor_free(pg_policy_processor* p);
/* Process(resync, pods) with pods as "ns/name" */
int pg_policy_processor_process(pg_policy_processor* p, int resync, const char* const* pods, size_t n);
const char* pg_policy_processor_last_error(const pg_policy_processor* p);

/* ---- VPPTCP renderer and VPP session-rule tables -------------------
 * The renderer cache's second consumer: IngressOrientation tables rendered as VPP session
 * rules for the VPP TCP host stack.
 *   vpptcp.Renderer Init/NewTxn/Render/Commit  plugins/policy/renderer/vpptcp/vpptcp_renderer.go:58-188
 *   dumpRules / updateRules                    vpptcp_renderer.go:191-316
 *   rule.SessionRule, Export/ImportSessionRules plugins/policy/renderer/vpptcp/rule/session_rule.go:72-476
 *   rule.IPv4Net (GetNsIndex/GetPodByAppNsIndex) session_rule.go:88-95      -> pg_appns
 *   session_rule_add_del / session_rules_dump  binary API as mock/sessionrules/sessionrules_mock.go
 *                                              holds it                    -> pg_session_rules
 * Host-side control plane: the reference classifies nothing on this path (the session-rule
 * lookup is VPP's). */
enum { PG_SCOPE_GLOBAL = 1, PG_SCOPE_LOCAL = 2, PG_SCOPE_BOTH = 3 };
#define PG_SR_ACTION_DO_NOTHING 0xFFFFFFFFu
#define PG_SR_ACTION_DENY 0xFFFFFFFEu
#define PG_SR_ACTION_ALLOW 0xFFFFFFFDu
typedef struct pg_session_rule { /* rule.SessionRule (session_rule.go:73-86) */
    uint8_t transport_proto;     /* 0 TCP, 1 UDP */
    uint8_t is_ip4;
    uint8_t lcl_ip[16];
    uint8_t lcl_plen;
    uint8_t rmt_ip[16];
    uint8_t rmt_plen;
    uint16_t lcl_port;
    uint16_t rmt_port;
    uint32_t action_index;
    uint32_t appns_index;
    uint8_t scope;
    char tag[64];
} pg_session_rule;
typedef struct pg_session_rules pg_session_rules;
typedef struct pg_appns pg_appns;
typedef struct pg_vpptcp_renderer pg_vpptcp_renderer;
typedef struct pg_vpptcp_txn pg_vpptcp_txn;

/* VPP's session-rule tables; tag_prefix NULL = "contiv/vpp-policy" (rules with another tag
 * are refused). Every add/del counts one request, a dump two (dump + control_ping). */
pg_session_rules* pg_session_rules_new(const char* tag_prefix);
void pg_session_rules_free(pg_session_rules* s);
int pg_session_rules_clear(pg_session_rules* s);
int pg_session_rules_counts(const pg_session_rules* s, int* req_count, int* err_count);
/* session_rule_add_del: the reply's retval (0 ok, 1 refused: bad tag, duplicate add, unknown delete) */
int pg_session_rule_add_del(pg_session_rules* s, const pg_session_rule* rule, int is_add);
/* rules of the global table (scope GLOBAL) or of ns_index's local table (scope LOCAL), in
 * installation order -> count (copies min(count, cap)) */
int pg_session_rules_table(const pg_session_rules* s, int scope, uint32_t ns_index, pg_session_rule* out, size_t cap);
/* MockSessionRules.{Local,Global}Table().HasRule: "" = unset address, a bare address = its
 * one-host subnet; proto "TCP"/"UDP"; action "ALLOW"/"DENY" -> 1 / 0 */
int pg_session_rules_has_rule(const pg_session_rules* s, int scope, uint32_t ns_index, const char* lcl_ip,
                              uint16_t lcl_port, const char* rmt_ip, uint16_t rmt_port, const char* proto,
                              const char* action);
/* pod -> VPP application namespace index (IPv4Net.GetNsIndex / GetPodByAppNsIndex) */
pg_appns* pg_appns_new(void);
void pg_appns_free(pg_appns* a);
int pg_appns_set(pg_appns* a, const char* pod_namespace, const char* pod_name, uint32_t ns_index);
/* ExportSessionRules: pod_name NULL = global table -> count (copies min(count, cap)) */
int pg_export_session_rules(const pg_appns* a, const pg_contiv_rule* rules, size_t n, const char* pod_namespace,
                            const char* pod_name, const pg_ipnet* pod_ip, pg_session_rule* out, size_t cap);
/* the renderer keeps pointers to vpp and ipv4net (both must outlive it); chan_buf_size =
 * GoVPPChanBufSize (0 = 100: requests are sent in bursts of that size) */
pg_vpptcp_renderer* pg_vpptcp_renderer_new(pg_session_rules* vpp, const pg_appns* ipv4net, int chan_buf_size);
void pg_vpptcp_renderer_free(pg_vpptcp_renderer* r);
const char* pg_vpptcp_last_error(const pg_vpptcp_renderer* r);
pg_vpptcp_txn* pg_vpptcp_new_txn(pg_vpptcp_renderer* r, int resync);
int pg_vpptcp_txn_render(pg_vpptcp_txn* t, const char* pod_namespace, const char* pod_name, const pg_ipnet* pod_ip,
                         const pg_contiv_rule* ingress, size_t n_ingress, const pg_contiv_rule* egress,
                         size_t n_egress, int removed);
/* renders and programs the session rules, frees t; PG_EFAULT + pg_vpptcp_last_error when a
 * request failed (the cache then keeps its previous state, as the reference's does) */
int pg_vpptcp_txn_commit(pg_vpptcp_txn* t);
void pg_vpptcp_txn_free(pg_vpptcp_txn* t);
/* PolicyConfigurator.RegisterRenderer for the VPPTCP renderer */
int pg_configurator_register_vpptcp(pg_configurator* c, pg_vpptcp_renderer* r);

/* VPP's session-rule lookup on the device. Installs the session-rule table (scope PG's
 * kScopeLocal = 2 with its application-namespace index, or kScopeGlobal = 1) of s into ctx as
 * the ACL acl_name (a put, as by pg_apply_txn; call again after the table changed), so that
 * pg_classify(ctx, PG_MODE_SINGLE, pg_table_id(ctx, acl_name), ...) classifies connections by
 * it: the table's IPv4 rules (prefixes up to 32 bits) ordered most specific first (lcl_plen + rmt_plen + one per set
 * port, ties in SessionRule.Compare order, session_rule.go:168-209) and first match, which is
 * the containment order renderer/api.go:111-112 defines for the ContivRules they come from
 * (convertContivRule, session_rule.go:263-361). Tuple fields: a local table keys on
 * (src_ip = local address, dst_ip = remote address, dst_port = remote port), the global table
 * on (src_ip = remote, dst_ip = local, dst_port = local port); proto TCP / UDP. Verdict PERMIT =
 * ALLOW, DENY = DENY with the rule's slot, the ACL's default slot = no session rule applies.
 * The reference has no session-rule lookup (VPP's own code): parity unpinned beyond the
 * restatement in oracle/vpptcp.py. PG_EINVAL (+ pg_last_error) for a rule this form cannot
 * hold: a port on the side the table does not key on, an action other than ALLOW / DENY. */
int pg_session_table_install(pg_ctx* ctx, const pg_session_rules* s, int scope, uint32_t ns_index,
                             const char* acl_name);

#ifdef __cplusplus
}
#endif
#endif /* POLICYGPU_H */
