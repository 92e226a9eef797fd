// Per-tuple semantics of the classify path, written once for both sides: the gfx950 kernels
// (device.hip) instantiate it with LDS / global loaders, and pg_debug_classify_host (tests
// only, never on the classify path) instantiates it on the host, so every compiled structure
// -- per-table blobs, the node classifier, interface resolution, the testConnection fusion --
// is checked against the oracle on CPU with the code the GPU runs.
//
// One evaluation == evalACL (mock/aclengine/aclengine_mock.go:503-652) over the ACL a table
// was compiled from (engine.cpp compile_acl_rule); the output word packs the ACLAction (or
// ConnAction) in bits 31-30 and the deciding counter slot in bits 29-0.
//
// Every function works on Q tuples of one lane "in lockstep": each dependent step issues the
// loads of all Q tuples before consuming any, so a lane has up to Q independent chains in
// flight (Q = 4 in the kernels' main loop, 1 in the remainder loop).
#pragma once
#include <cstdint>
#include <type_traits>

#include "blobwalk.hpp"
#include "device.hpp"

namespace pg {

#if defined(__HIP_DEVICE_COMPILE__)
#define PG_NOINLINE __device__ __noinline__
#else
#define PG_NOINLINE inline
#endif
#ifndef PG_AGG_ROUNDS  // wave-aggregation rounds of hit-counter increments (Hist::inc)
#define PG_AGG_ROUNDS 0
#endif
#ifndef PG_FD_SKIP  // FD walks over a blob in HBM: no re-read of a finished lane's self word
#define PG_FD_SKIP 1
#endif
#ifndef PG_MUL24  // node cross-entry index products as 24-bit multiplies
#define PG_MUL24 1
#endif
#ifndef PG_NODE_FB_Q1  // node kernels: per-table fallback one tuple at a time
#define PG_NODE_FB_Q1 1
#endif
#ifndef PG_NODE_FB_CALL  // node kernels: that fallback is an out-of-line call (keeps it out of
#define PG_NODE_FB_CALL 1  // the hot loop's code and register allocation)
#endif

// TCP -> port, UDP -> 0x10000 | port, OTHER -> 0x20000, anything else -> 0x30000 (branch-free)
PG_HD uint32_t pkt_key(uint32_t proto, uint32_t port) {
    const uint32_t p = proto < 3u ? proto : 3u;
    return (p << 16) | (p < 2u ? port : 0u);
}
PG_HD uint32_t verdict(uint32_t act, uint32_t slot) { return (act << 30) | slot; }
// a * b for operands below 2^16 (class indices x row widths): one full-rate 24-bit multiply on
// the device, where the compiler otherwise emits a 64-bit multiply-add for the u32 product
PG_HD uint32_t mul24(uint32_t a, uint32_t b) {
#if defined(__HIP_DEVICE_COMPILE__) && PG_MUL24
    return __umul24(a, b);
#else
    return a * b;
#endif
}
// a * b + c for a, b below 2^24 (v_mad_u32_u24 on the device)
PG_HD uint32_t mad24(uint32_t a, uint32_t b, uint32_t c) {
#if defined(__HIP_DEVICE_COMPILE__) && PG_MUL24
    return __umul24(a, b) + c;
#else
    return a * b + c;
#endif
}
// bit i & 31 of w (one v_bfe_u32: its offset operand reads the low 5 bits)
PG_HD uint32_t bit_of(uint32_t w, uint32_t i) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_ubfe(w, i, 1u);
#else
    return (w >> (i & 31u)) & 1u;
#endif
}
constexpr uint32_t kSlotMask = 0x3FFFFFFFu;

PG_HD uint32_t hash_ip(uint32_t ip) {
    ip ^= ip >> 16;
    ip *= 0x7feb352du;
    ip ^= ip >> 15;
    ip *= 0x846ca68bu;
    ip ^= ip >> 16;
    return ip;
}

// Linear first-match over a table's compiled rules: LINEAR tables and ANY-protocol packets
// (rare). Scalar arguments only, so the call needs no stack frame.
PG_NOINLINE uint32_t eval_linear(const DevRule* rules, uint32_t base, uint32_t nr, uint32_t dflt, uint32_t src,
                                 uint32_t dst, uint32_t key) {
    const bool any = key >= kKeyANY;
    for (uint32_t i = 0; i < nr; i++) {
        const DevRule r = rules[base + i];
        if ((src & r.smask) != r.snet || (dst & r.dmask) != r.dnet) continue;
        if (any) {
            if ((r.act >> 4) != kActNever) return verdict((r.act >> 4) & 3u, base + i);
        } else if (key >= r.klo && key <= r.khi) {
            return verdict(r.act & 3u, base + i);
        }
    }
    return dflt;
}

// 16/8/4-byte loads from LDS or global memory (the device infers the address space).
// Loads from a table array in global memory by 32-bit BYTE offsets (every array a loader reads
// is below kMaxLoaderBytes, checked where the arrays are built): the device load is then the
// array's SGPR base plus a 32-bit VGPR offset, with no 64-bit address arithmetic per gather.
struct DevLoader {
    const uint32_t* b;
    template <class V>
    PG_HD const V& ref(uint32_t off) const {
        return *reinterpret_cast<const V*>(reinterpret_cast<const char*>(b) + off);
    }
    PG_HD uint32_t u32(uint32_t i) const { return ref<uint32_t>(i * 4u); }
    PG_HD uint32_t at_byte(uint32_t off) const { return ref<uint32_t>(off); }
    PG_HD uint32_t u16(uint32_t i) const { return ref<uint16_t>(i * 2u); }  // halfword i
    PG_HD W2 u2(uint32_t i) const {
#if defined(__HIP_DEVICE_COMPILE__)
        const uint2 v = ref<uint2>(i * 4u);
        return W2{v.x, v.y};
#else
        return W2{b[i], b[i + 1]};
#endif
    }
    PG_HD W4 u4(uint32_t i) const {
#if defined(__HIP_DEVICE_COMPILE__)
        const uint4 v = ref<uint4>(i * 4u);
        return W4{v.x, v.y, v.z, v.w};
#else
        return W4{b[i], b[i + 1], b[i + 2], b[i + 3]};
#endif
    }
    // at byte addresses (8- / 16-byte aligned): node class records
    PG_HD W2 u2_at_byte(uint32_t off) const { return u2(off / 4u); }
    PG_HD W4 u4_at_byte(uint32_t off) const { return u4(off / 4u); }
};

// Loads from the kernel's LDS image, which starts at LDS address 0 (k_classify's dynamic shared
// memory; the kernel declares no static LDS): addresses are the offsets themselves, so a trie
// step is a shift and a shifted add, not also an add of the (link-time zero) base.
struct LdsLoader {
#if defined(__HIP_DEVICE_COMPILE__)
    template <class T>
    static __device__ __forceinline__ T at(uint32_t byte) {
        return *reinterpret_cast<const __attribute__((address_space(3))) T*>((uintptr_t)byte);
    }
    PG_HD uint32_t u32(uint32_t i) const { return at<uint32_t>(i * 4u); }
    PG_HD uint32_t at_byte(uint32_t off) const { return at<uint32_t>(off); }
    PG_HD uint32_t u16(uint32_t i) const { return at<uint16_t>(i * 2u); }
    PG_HD W2 u2(uint32_t i) const {
        const uint2 v = at<uint2>(i * 4u);
        return W2{v.x, v.y};
    }
    PG_HD W4 u4(uint32_t i) const {
        const uint4 v = at<uint4>(i * 4u);
        return W4{v.x, v.y, v.z, v.w};
    }
    PG_HD W2 u2_at_byte(uint32_t off) const {
        const uint2 v = at<uint2>(off);
        return W2{v.x, v.y};
    }
    PG_HD W4 u4_at_byte(uint32_t off) const {
        const uint4 v = at<uint4>(off);
        return W4{v.x, v.y, v.z, v.w};
    }
#else  // host builds never instantiate it (kernels only)
    uint32_t u32(uint32_t) const { return 0; }
    uint32_t at_byte(uint32_t) const { return 0; }
    uint32_t u16(uint32_t) const { return 0; }
    W2 u2(uint32_t) const { return W2{0, 0}; }
    W4 u4(uint32_t) const { return W4{0, 0, 0, 0}; }
    W2 u2_at_byte(uint32_t) const { return W2{0, 0}; }
    W4 u4_at_byte(uint32_t) const { return W4{0, 0, 0, 0}; }
#endif
};

PG_HD DevTable load_tab(const DevTable* tabs, int32_t t) {
    const DevLoader l{reinterpret_cast<const uint32_t*>(tabs + t)};
    const W4 a = l.u4(0), c = l.u4(4);
    return DevTable{a.x, a.y, a.z, a.w, c.x, c.y, c.z, c.w};
}

// evalACL of Q tuples against their tables' per-table blobs, in lockstep.
// act[j]: evaluate tuple j against tab[j]; blobs: base the tables' blob_off is relative to
// (the global blob array, or the LDS copy of a staged table).
// rootb (SINGLE mode, a blob whose src-trie root alone is staged): the LDS copy of the
// table blob's first words, read for the root load only.
template <bool PRED = false, int Q>
PG_HD void eval_q(const DevTableSet& T, const uint32_t* blobs, const DevTable (&tab)[Q], const bool (&act)[Q],
                  const uint32_t (&src)[Q], const uint32_t (&dst)[Q], const uint32_t (&key)[Q], uint32_t (&w)[Q],
                  const uint32_t* rootb = nullptr) {
    DevLoader ld[Q], ld0[Q];
    BlobTab tb[Q];
    bool on[Q], fd[Q], anyfd = false;
    // on[j] depends on the table only (uniform when every lane has the same table, as in
    // SINGLE mode); ANY-protocol keys (< 2^18, a valid trie address) are walked too and their
    // result replaced by the linear scan below
    PG_UNROLL
    for (int j = 0; j < Q; j++) {
        ld[j] = DevLoader{blobs + tab[j].blob_off};
        ld0[j] = rootb ? DevLoader{rootb} : ld[j];
        tb[j] = BlobTab{tab[j].fsk, tab[j].dflt, tab[j].kroot, tab[j].xoff, tab[j].nkc, tab[j].rule_base};
        fd[j] = act[j] && (tab[j].fsk & kFlagFD);
        on[j] = act[j] && !fd[j] && !(tab[j].fsk & kFlagLinear);
        anyfd |= fd[j];
    }
    blob_walk<PRED>(ld, ld0, tb, on, src, dst, key, w);
    if (anyfd) {  // FD tables, one lane at a time (their walk has no per-lane state to share)
        PG_UNROLL
        for (int j = 0; j < Q; j++) {
            if (!fd[j]) continue;
            const uint32_t s1[1] = {src[j]}, k1[1] = {key[j]};
            uint32_t w1[1];
            fd_walk(ld[j], ld[j], tab[j].fsk, tab[j].kroot, tab[j].xoff, tab[j].nkc, s1, k1, w1);
            w[j] = w1[0];
        }
    }
    PG_UNROLL
    for (int j = 0; j < Q; j++)
        if (act[j] && ((!on[j] && !fd[j]) || key[j] >= kWalkKeyLimit))
            w[j] = eval_linear(T.rules, tab[j].rule_base, tab[j].n_rules, tab[j].dflt, src[j], dst[j], key[j]);
}

// evalACL of one tuple against one table by its per-table blob (and the linear scan for LINEAR
// tables and ANY-protocol keys): the node kernels' rare fallback, out of line on the device.
// Scalar arguments only, so the call needs no stack frame for them.
PG_NOINLINE uint32_t eval_one(const DevRule* rules, const uint32_t* blobs, const DevTable* tabs, int32_t t,
                              uint32_t src, uint32_t dst, uint32_t key) {
    const DevTable tab = load_tab(tabs, t);
    if (tab.fsk & kFlagFD) {
        const uint32_t s1[1] = {src}, k1[1] = {key};
        uint32_t w1[1];
        const DevLoader ld{blobs + tab.blob_off};
        fd_walk(ld, ld, tab.fsk, tab.kroot, tab.xoff, tab.nkc, s1, k1, w1);
        if (key < kWalkKeyLimit) return w1[0];
    } else if (!(tab.fsk & kFlagLinear) && key < kWalkKeyLimit) {
        const DevLoader ld[1] = {DevLoader{blobs + tab.blob_off}};
        const BlobTab tb[1] = {BlobTab{tab.fsk, tab.dflt, tab.kroot, tab.xoff, tab.nkc, tab.rule_base}};
        const bool on[1] = {true};
        const uint32_t s1[1] = {src}, d1[1] = {dst}, k1[1] = {key};
        uint32_t w1[1];
        blob_walk(ld, tb, on, s1, d1, k1, w1);
        return w1[0];
    }
    return eval_linear(rules, tab.rule_base, tab.n_rules, tab.dflt, src, dst, key);
}

// tables of a connection end point: interface (-1/-2 unresolvable) and its ACLs
struct End {
    int32_t ifc, tin, tout;
};

// IPv4 -> end point by the iphash (per-table path): a local pod's TAP, else the node-output
// interface (VXLAN BVI or main; aclengine_mock.go:273-420), marked as a remote pod's or a
// non-pod address's (device.hpp kEndRemote / kEndInet). One 16-B load per probe step.
template <int Q>
PG_HD void probe_q(const DevTableSet& T, const uint32_t (&ip)[Q], End (&e)[Q]) {
    const DevLoader H{T.iphash};
    uint32_t s[Q];
    W4 v[Q];
    bool pend[Q];
    PG_UNROLL
    for (int j = 0; j < Q; j++) {
        s[j] = hash_ip(ip[j]) & T.iphash_mask;
        v[j] = H.u4(4u * s[j]);
        pend[j] = true;
    }
    for (;;) {
        bool more = false;
        PG_UNROLL
        for (int j = 0; j < Q; j++) {
            if (!pend[j]) continue;
            if (v[j].y == 0xFFFFFFFFu) {
                e[j] = End{T.node_if, T.node_in, T.node_out};
                pend[j] = false;
            } else if (v[j].x == ip[j]) {
                e[j] = End{(int32_t)v[j].y, (int32_t)v[j].z, (int32_t)v[j].w};
                pend[j] = false;
            } else {
                s[j] = (s[j] + 1u) & T.iphash_mask;
                v[j] = H.u4(4u * s[j]);
                more = true;
            }
        }
        if (!more) break;
    }
}

// per-rule hit counters: LDS histogram (u32) or global u64 slots on the device, plain u64
// slots on the host
// kFullLds: lds (when set) holds every slot (node kernels); kAggGlobal: with lds unset, global
// increments are aggregated per distinct slot over the wave (PERPOD node kernels)
// kCache: node kernels, which may count through an LDS slot cache (ckey)
// kFullOnly: node kernels whose LDS histogram holds every slot (device.hip STAGE + 16): an
// increment is one LDS atomic, with none of the window / hot-slot / global tests in the code
constexpr uint32_t kCacheEmpty = 0xFFFFFFFFu;  // slot-cache key of a free cell (slots are < 2^30)
#ifndef PG_CACHE_PROBES  // slot cache: cells tried (linear probing) before a global atomic
#define PG_CACHE_PROBES 4
#endif
// kHotRegs (kFullOnly builds): slots hot and hot2 are counted in registers
// kHalf (kFullOnly builds, device.hip STAGE + 256): 16-bit cells, two slots per LDS word (slot s
// in the half s & 1 of word s >> 1), for node sets whose 32-bit histogram would leave LDS for
// one workgroup per CU. The increment that takes a cell to 0x8000 moves 0x8000 to the slot's
// global counter (the cell cannot reach 0x10000 before that lane's subtraction lands: that
// would take 0x8000 more increments of one slot by one workgroup in between)
template <bool kFullLds = false, bool kAggGlobal = false, bool kCache = false, bool kFullOnly = false,
          bool kHotRegs = false, bool kHalf = false>
struct HistT {
    uint32_t* lds;
    unsigned long long* glob;
    // device, lds set: cells [0, wn) count slots [wbase, wbase + wn), cells wn and wn + 1 count
    // slots xslot and xslot1, other slots go to glob (device.hip k_classify)
    uint32_t wbase = 0, wn = 0xFFFFFFFFu, xslot = 0xFFFFFFFFu, xslot1 = 0xFFFFFFFFu;
    bool full = true;  // the window holds every slot (wave-uniform: the common case costs no test)
    // SINGLE kernels: slot `hot` (the table's last rule: a catch-all takes every unmatched
    // packet) counted per lane in a register and added once at the end (flush_hot) -- many
    // lanes of a wave on one LDS address serialise their atomics
    uint32_t hot = 0xFFFFFFFFu, hot2 = 0xFFFFFFFFu;  // (hot2: kFullOnly builds only)
    mutable uint32_t nhot = 0, nhot2 = 0;
    // node kernels over a table set with more slots than the full histogram: an LDS cache of
    // 2^k cells, keys ckey[0, cmask] and counts after them (ckey[cmask + 2 + c]); cell cmask + 1
    // holds `hot`. A slot takes the first cell, from hash(slot) on, that holds it or that it
    // claims while free (LDS compare-and-swap); after PG_CACHE_PROBES occupied cells it goes to
    // a global atomic. Hot slots come first in a workgroup's stream, so they hold cells: config
    // 6 counts 95 % of its increments in its 256 most frequent slots, 99 % in 4096 (the per-table
    // rule windows this replaces covered 93 % with 4096 cells, and the increments they left to
    // global atomics halved its rate). 256 cells (2 KiB) keep three workgroups per CU beside the
    // image: config 6 with counters 99 -> 144 Gpps (A/B on MI355X; 1024 cells 129, 4096 128).
    uint32_t* ckey = nullptr;
    uint32_t cmask = 0, cshift = 32;
#if defined(__HIP_DEVICE_COMPILE__)
    // one increment of slot in the 16-bit-cell histogram (kHalf)
    __device__ void half_add(uint32_t slot) const {
        const uint32_t sh = (slot & 1u) << 4;
        const uint32_t old = atomicAdd(&lds[slot >> 1], 1u << sh);
        if (((old >> sh) & 0xFFFFu) == 0x7FFFu) {
            atomicSub(&lds[slot >> 1], 0x8000u << sh);
            atomicAdd(&glob[slot], 0x8000ull);
        }
    }
#endif
    // one increment of a slot that is never `hot` / `hot2` (the unresolved-interface slot): the
    // full-histogram builds skip the register tests (their loop-invariant results were hoisted
    // out of the CONN loop and spilled, each reload a vmcnt(0) wait)
    PG_HD void inc_cold(uint32_t slot) const {
#if defined(__HIP_DEVICE_COMPILE__) && !defined(PG_PROBE_NOINC)
        if constexpr (kFullOnly && kHalf) {
            half_add(slot);
            return;
        } else if constexpr (kFullOnly) {
            atomicAdd(&lds[slot], 1u);
            return;
        }
#endif
        inc_t(slot, -1);
    }
    // one increment of an evaluation of table t (t < 0: no table; its slot is past the rules)
    PG_HD void inc_t(uint32_t slot, int32_t t) const {
#if defined(__HIP_DEVICE_COMPILE__) && !defined(PG_PROBE_NOINC)
        if (kCache && ckey) {
            if (slot == hot) {
                nhot++;
                return;
            }
            uint32_t* cnt = ckey + cmask + 2u;
            uint32_t c = (slot * 0x9E3779B1u) >> cshift;
#pragma unroll
            for (int p = 0; p < PG_CACHE_PROBES; p++) {
                const uint32_t k = __atomic_load_n(&ckey[c], __ATOMIC_RELAXED);
                if (k == slot) {
                    atomicAdd(&cnt[c], 1u);
                    return;
                }
                if (k == kCacheEmpty) {
                    const uint32_t old = atomicCAS(&ckey[c], kCacheEmpty, slot);
                    if (old == kCacheEmpty || old == slot) {
                        atomicAdd(&cnt[c], 1u);
                        return;
                    }
                }
                c = (c + 1u) & cmask;
            }
#if defined(PG_PROBE_NOGLOBINC)  // measurement build only: increments past the cache dropped
            return;
#endif
            // the cache is full along this slot's probe sequence: one global atomic per distinct
            // slot over the wave's lanes
            for (;;) {
                const uint32_t lead = __builtin_amdgcn_readfirstlane(slot);
                const unsigned long long m = __ballot(slot == lead);
                if (slot == lead) {
                    if (__lane_id() == (unsigned)(__ffsll((long long)m) - 1))
                        atomicAdd(&glob[lead], (unsigned long long)__popcll(m));
                    break;
                }
            }
            return;
        }
#endif
        inc(slot);
    }
    // one increment of the slot of verdict word w (bits 29-0). The CONN full-histogram build
    // compares w << 2 -- the slot's byte offset, the action bits shifted out -- with the two
    // register-counted slots' offsets and adds at that offset: no mask of the action bits
    PG_HD void inc_w(uint32_t w) const {
#if defined(__HIP_DEVICE_COMPILE__) && !defined(PG_PROBE_NOINC)
        if constexpr (kFullOnly && kHotRegs && kHalf) {
            const uint32_t sl = w & 0x3FFFFFFFu;
            nhot += sl == hot;
            nhot2 += sl == hot2;
            if (sl != hot && sl != hot2) half_add(sl);
            return;
        } else if constexpr (kFullOnly && kHotRegs) {
            const uint32_t b = w << 2;
            nhot += b == hot << 2;
            nhot2 += b == hot2 << 2;
            if (b != hot << 2 && b != hot2 << 2)
                atomicAdd(reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(lds) + b), 1u);
            return;
        }
#endif
        inc_t(w & 0x3FFFFFFFu, 0);
    }
    PG_HD void inc(uint32_t slot) const {
#if defined(__HIP_DEVICE_COMPILE__) && defined(PG_PROBE_NOINC)  // measurement build only
        if (slot == 0xFFFFFFFFu) lds[0] = 0;
#elif defined(__HIP_DEVICE_COMPILE__)
        if constexpr (kFullOnly && kHotRegs) {  // CONN's two hottest slots in registers
            nhot += slot == hot;
            nhot2 += slot == hot2;
            if (slot != hot && slot != hot2) {
                if constexpr (kHalf) half_add(slot);
                else atomicAdd(&lds[slot], 1u);
            }
            return;
        } else if constexpr (kFullOnly && kHalf) {
            half_add(slot);
            return;
        } else if constexpr (kFullOnly) {
            atomicAdd(&lds[slot], 1u);
            return;
        }
        if (slot == hot) {
            nhot++;
            return;
        }
        // One LDS (or global) atomic per lane. PG_AGG_ROUNDS > 0 first lets the lanes that
        // share the first active lane's slot (a reflective ACL's rule, "no ACL", a default
        // deny) add their count with one atomic, per round; A/B on MI355X with warmed-up
        // launches (tools/sweep.py): 0 rounds beats 1 / 2 / 3 by 3-14 % on configs 2, 3, 5.
        bool done = false;
#pragma unroll
        for (int r = 0; r < PG_AGG_ROUNDS; r++) {
            if (!done) {
                const uint32_t lead = __builtin_amdgcn_readfirstlane(slot);
                const unsigned long long m = __ballot(slot == lead);
                if (slot == lead) {
                    if (__lane_id() == (unsigned)(__ffsll((long long)m) - 1)) {
                        const uint32_t c = lead - wbase;
                        if (lds && c < wn) atomicAdd(&lds[c], (uint32_t)__popcll(m));
                        else if (lds && lead == xslot) atomicAdd(&lds[wn], (uint32_t)__popcll(m));
                        else if (lds && lead == xslot1) atomicAdd(&lds[wn + 1], (uint32_t)__popcll(m));
                        else if (glob) atomicAdd(&glob[lead], (unsigned long long)__popcll(m));
                    }
                    done = true;
                }
            }
        }
        if (!done) {
            const uint32_t c = slot - wbase;
            bool g = false;
#if defined(PG_PROBE_PLAINST)  // measurement build only: a plain LDS store in place of the atomic
            if (lds && (kFullLds || full)) lds[slot] = 1u;
#else
            if (lds && (kFullLds || full)) atomicAdd(&lds[slot], 1u);
#endif
            else if (lds && c < wn) atomicAdd(&lds[c], 1u);
            else if (lds && slot == xslot) atomicAdd(&lds[wn], 1u);
            else if (lds && slot == xslot1) atomicAdd(&lds[wn + 1], 1u);
            else g = glob != nullptr;
            if (g && !(kAggGlobal && !lds)) {
                atomicAdd(&glob[slot], 1ull);
            } else if (g) {
                // PERPOD node kernels over a table set larger than the LDS histogram (every
                // increment a global atomic): aggregated per distinct slot over the wave's lanes,
                // one atomic per slot instead of one per lane -- the per-table catch-alls
                // serialise at the L2 otherwise (config 6 with counters 5.6 -> 8.3 Gpps; on
                // SINGLE's windowed histogram, whose global slots are mostly distinct, the loop
                // cost 3-11 %; in the register-capped CONN kernel its code cost 2.5 %)
                for (;;) {
                    const uint32_t lead = __builtin_amdgcn_readfirstlane(slot);
                    const unsigned long long m = __ballot(slot == lead);
                    if (slot == lead) {
                        if (__lane_id() == (unsigned)(__ffsll((long long)m) - 1))
                            atomicAdd(&glob[lead], (unsigned long long)__popcll(m));
                        break;
                    }
                }
            }
        }
#else
        if (glob) glob[slot]++;
#endif
    }
    PG_HD void flush_hot() const {  // device: the register count of `hot` into the histogram
#if defined(__HIP_DEVICE_COMPILE__)
        if constexpr (kHalf) {  // (16-bit cells) the wave's register counts straight to the global counters
            uint32_t a = nhot, b = nhot2;
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) a += __shfl_xor(a, o), b += __shfl_xor(b, o);
            if (__lane_id() == 0) {
                if (a) atomicAdd(&glob[hot], (unsigned long long)a);
                if (kHotRegs && b) atomicAdd(&glob[hot2], (unsigned long long)b);
            }
            nhot = nhot2 = 0;
            return;
        }
        if (kHotRegs && nhot2) {
            atomicAdd(&lds[hot2], nhot2);
            nhot2 = 0;
        }
        if (nhot) {
            const uint32_t h0 = hot;
            const uint32_t n = nhot;
            nhot = 0;
            const uint32_t c = h0 - wbase;
            if (kCache && ckey) atomicAdd(&ckey[2u * cmask + 3u], n);  // the hot cell's count (cnt[cmask + 1])
            else if (lds && (kFullLds || full)) atomicAdd(&lds[h0], n);
            else if (lds && c < wn) atomicAdd(&lds[c], n);
            else if (lds && h0 == xslot) atomicAdd(&lds[wn], n);
            else if (lds && h0 == xslot1) atomicAdd(&lds[wn + 1], n);
            else if (glob) atomicAdd(&glob[h0], (unsigned long long)n);
        }
#endif
    }
};
using Hist = HistT<false>;

// SINGLE mode over an FD table (uniform: tab0): Q tuples per lane, fixed-depth walks in
// lockstep; ANY-protocol packets take the linear scan. prefix: the blob's prefix (its LDS copy
// in the kernels), blob: the whole blob (the same LDS copy when it is staged whole, else HBM).
// The dst address is not an input: no rule of an FD table tests it (engine.cpp compile).
template <bool COUNT, int Q, class LP, class LB>
PG_HD void classify_fd_q(const DevTableSet& T, const LP& prefix, const LB& blob, const DevTable& tab0,
                         const uint32_t (&s)[Q], const uint32_t (&dp)[Q], const uint32_t (&pr)[Q], const Hist& h,
                         uint32_t (&out)[Q]) {
    uint32_t key[Q];
    bool any = false;
    PG_UNROLL
    for (int j = 0; j < Q; j++) key[j] = pkt_key(pr[j], dp[j]), any |= key[j] >= kWalkKeyLimit;
    fd_walk<PG_FD_SKIP && !std::is_same<LB, LdsLoader>::value>(prefix, blob, tab0.fsk, tab0.kroot, tab0.xoff, tab0.nkc,
                                                               s, key, out);
    if (any) {
        PG_UNROLL
        for (int j = 0; j < Q; j++)  // no rule of an FD table tests dst (engine.cpp): any dst will do
            if (key[j] >= kWalkKeyLimit)
                out[j] = eval_linear(T.rules, tab0.rule_base, tab0.n_rules, tab0.dflt, s[j], 0u, key[j]);
    }
    if (COUNT) {
        PG_UNROLL
        for (int j = 0; j < Q; j++) h.inc(out[j] & kSlotMask);
    }
}

// SINGLE mode over a CANDI table whose root alone is staged (uniform: tab0; device.hip STAGE 6):
// the root from `root`, the 8-B entries and records from `blob`, with none of the generic blob
// walk's per-lane structure tests; ANY-protocol packets take the linear scan. No rule of a CANDI
// table tests dst (fastpath.cpp), so dst is not an input.
template <bool COUNT, int Q, class L0, class L>
PG_HD void classify_candi_q(const DevTableSet& T, const L0& root, const L& blob, const DevTable& tab0,
                            const uint32_t (&s)[Q], const uint32_t (&dp)[Q], const uint32_t (&pr)[Q], const Hist& h,
                            uint32_t (&out)[Q]) {
    uint32_t key[Q], zero[Q], pos[Q];
    bool on[Q], pend[Q], any = false;
    L ld[Q];
    L0 ld0[Q];
    BlobTab tb[Q];
    PG_UNROLL
    for (int j = 0; j < Q; j++) {
        key[j] = pkt_key(pr[j], dp[j]);
        any |= key[j] >= kWalkKeyLimit;
        zero[j] = 0;
        pos[j] = 0;
        on[j] = true;
        pend[j] = false;
        ld[j] = blob;
        ld0[j] = root;
        tb[j] = BlobTab{tab0.fsk, tab0.dflt, tab0.kroot, tab0.xoff, tab0.nkc, tab0.rule_base};
    }
    candi_walk(ld, ld0, tb, on, s, key, out, pend, pos);
    rec_walk(ld, tb, zero, key, pend, pos, out);
    if (any) {
        PG_UNROLL
        for (int j = 0; j < Q; j++)
            if (key[j] >= kWalkKeyLimit)
                out[j] = eval_linear(T.rules, tab0.rule_base, tab0.n_rules, tab0.dflt, s[j], 0u, key[j]);
    }
    if (COUNT) {
        PG_UNROLL
        for (int j = 0; j < Q; j++) h.inc(out[j] & kSlotMask);
    }
}

// ---- evaluators: evalACL of Q tuples on tables t[j], forward (src -> dst, SYN key) or
// reverse (dst -> src, SYN-ACK key; testConnection's second half) ----------------------------

// per-table blobs (global memory)
template <int Q>
struct TabEval {
    const DevTableSet& T;
    const uint32_t (&src)[Q];
    const uint32_t (&dst)[Q];
    const uint32_t (&ksyn)[Q];
    const uint32_t (&kack)[Q];
    PG_HD void operator()(const int32_t (&t)[Q], const bool (&act)[Q], bool rev, uint32_t (&w)[Q]) const {
        DevTable tab[Q];
        PG_UNROLL
        for (int j = 0; j < Q; j++) tab[j] = act[j] ? load_tab(T.tabs, t[j]) : DevTable{};
        eval_q(T, T.blobs, tab, act, rev ? dst : src, rev ? src : dst, rev ? kack : ksyn, w);
    }
};

// Node classifier (fastpath.cpp build_node): IPv4 -> node IP class and L4 key -> node key
// class by tries in the node image (LDS when staged), then one entry of the node cross
// table per evaluation, cross[tabinfo[t].base + ipclass * nkc_t + kmap[t][keyclass]]: a
// verdict, or (kNodeList) the first of the dst records to test. Tables the node does not
// cover, LINEAR tables and ANY-protocol packets take the per-table path.
// Fixed-depth trie lookups (DevNode: a leaf points at its class record; a record that a leaf
// above the last level points at holds that leaf's value in its first word), in lockstep and
// without per-lane branches: the root read (stride s1 over a W-bit address), then depth - 1
// steps of one bit-field extract and one shifted add each (blobwalk.hpp node_child_byte, the
// aligned encoding for the uniform layout, A) at a per-level bit offset. r: the record byte
// addresses; the class is (r >> record shift) - self. PRED is unused (kept for the callers).
template <bool PRED, bool A, class L, int Q>
PG_HD void node_trie_q(const L& ld, uint32_t root, uint32_t s1, uint32_t W, uint32_t depth, const uint32_t (&a)[Q],
                       uint32_t (&r)[Q]) {
    uint32_t rem = W - s1;
    PG_UNROLL
    for (int j = 0; j < Q; j++) r[j] = ld.u32(root + (a[j] >> (W - s1)));
    for (uint32_t l = 1; l < depth; l++) {
        rem = node_next_shift(rem);
        PG_UNROLL
        for (int j = 0; j < Q; j++) r[j] = ld.at_byte(node_child_byte<A>(r[j], a[j], rem));
    }
    PG_UNROLL
    for (int j = 0; j < Q; j++) r[j] = A ? r[j] : r[j] >> 5;
}

// The IPv4 trie (addresses a) and the L4-key trie (keys b) in one lockstep loop: independent
// walks, so their dependent LDS reads overlap. rr: the IPv4 class records' byte addresses; cb:
// the key classes. IS1 / ID / KS1 / KD: the tries' root strides and depths when known at compile
// time (node_walks: the common shapes), so every level's shift is a constant and the walks
// unroll into straight-line code; 0 = read from N at run time.
template <bool PRED, bool A, uint32_t IS1 = 0, uint32_t ID = 0, uint32_t KS1 = 0, uint32_t KD = 0, class L, int QA,
          int QB>
PG_HD void node_trie2_q(const L& ld, const DevNode& N, const uint32_t (&a)[QA], uint32_t (&rr)[QA],
                        const uint32_t (&b)[QB], uint32_t (&cb)[QB]) {
    const uint32_t is1 = IS1 ? IS1 : N.ip_s1, ks1 = KS1 ? KS1 : N.key_k1;
    const uint32_t idp = ID ? ID : N.ip_depth, kdp = KD ? KD : N.key_depth;
    uint32_t ea[QA], eb[QB], ra = 32u - is1, rb = 18u - ks1;
    PG_UNROLL
    for (int j = 0; j < QA; j++) ea[j] = ld.u32(a[j] >> (32u - is1));
    PG_UNROLL
    for (int j = 0; j < QB; j++) eb[j] = ld.u32(N.key_root + (b[j] >> (18u - ks1)));
    const uint32_t dmin = idp < kdp ? idp : kdp;
    auto step_a = [&]() {
        ra = node_next_shift(ra);
        PG_UNROLL
        for (int j = 0; j < QA; j++) ea[j] = ld.at_byte(node_child_byte<A>(ea[j], a[j], ra));
    };
    auto step_b = [&]() {
        rb = node_next_shift(rb);
        PG_UNROLL
        for (int j = 0; j < QB; j++) eb[j] = ld.at_byte(node_child_byte<A>(eb[j], b[j], rb));
    };
    if constexpr (ID != 0 && KD != 0) {  // straight-line code, constant shifts
        constexpr uint32_t DM = ID < KD ? ID : KD;
        PG_UNROLL
        for (uint32_t l = 1; l < DM; l++) step_a(), step_b();
        PG_UNROLL
        for (uint32_t l = DM; l < ID; l++) step_a();
        PG_UNROLL
        for (uint32_t l = DM; l < KD; l++) step_b();
    } else {
        for (uint32_t l = 1; l < dmin; l++) step_a(), step_b();
        for (uint32_t l = dmin; l < idp; l++) step_a();
        for (uint32_t l = dmin; l < kdp; l++) step_b();
    }
    PG_UNROLL
    for (int j = 0; j < QA; j++) rr[j] = A ? ea[j] : ea[j] >> 5;
    PG_UNROLL
    for (int j = 0; j < QB; j++) cb[j] = (eb[j] >> (A ? node_key_rec_shift<A>() : node_key_rec_shift<A>() + 5)) - N.kself;
}

#ifndef PG_NODE_WALK2  // node kernels: IPv4 and key tries in one lockstep walk
#define PG_NODE_WALK2 1
#endif
#ifndef PG_NODE_SHAPES  // uniform-layout walks: the common trie shapes compiled with constant shifts
#define PG_NODE_SHAPES 1
#endif

// node_trie2_q, with the tries' shape as compile-time constants when it is one of the common ones
// of the uniform layout (aligned tries: IPv4 root 8 bits + three 8-bit levels; key root 6 bits +
// 8 + 4, 2 bits + 8 + 8, or 10 bits + 8 -- fastpath.cpp build_node picks the fewest levels, then
// the smallest image), else read at run time. The shape test is uniform (a scalar branch).
template <bool PRED, bool A, class L, int QA, int QB>
PG_HD void node_walks(const L& ld, const DevNode& N, const uint32_t (&a)[QA], uint32_t (&rr)[QA],
                      const uint32_t (&b)[QB], uint32_t (&cb)[QB]) {
    if constexpr (A && PG_NODE_SHAPES) {
        const uint32_t shape = N.ip_s1 | N.ip_depth << 8 | N.key_k1 << 16 | N.key_depth << 24;
        if (shape == (8u | 4u << 8 | 6u << 16 | 3u << 24))
            return node_trie2_q<PRED, A, 8, 4, 6, 3>(ld, N, a, rr, b, cb);
        if (shape == (8u | 4u << 8 | 2u << 16 | 3u << 24))
            return node_trie2_q<PRED, A, 8, 4, 2, 3>(ld, N, a, rr, b, cb);
        if (shape == (8u | 4u << 8 | 10u << 16 | 2u << 24))
            return node_trie2_q<PRED, A, 8, 4, 10, 2>(ld, N, a, rr, b, cb);
    }
    node_trie2_q<PRED, A>(ld, N, a, rr, b, cb);
}

// end point of a node IP class outside the uniform layout (ipinfo: {interface, tin | tout << 16},
// 0xFFFF = no ACL); the uniform layout's class records pack it (node_end_packed)
template <class L>
PG_HD End node_end(const L& img, const DevNode& N, uint32_t ipc) {
    const W2 v = img.u2(N.ipinfo + 2u * ipc);
    const uint32_t tin = v.y & 0xFFFFu, tout = v.y >> 16;
    return End{(int32_t)v.x, tin == 0xFFFFu ? -1 : (int32_t)tin, tout == 0xFFFFu ? -1 : (int32_t)tout};
}
// packed end point (uniform layout, narrow records): interface index (14 bits) | end-point kind
// << 14 (0xFFFF: unresolved) | tin << 16 | tout << 24 (tnil = no ACL, DevNode tnil)
PG_HD End node_end_packed(uint32_t p, uint32_t tnil) {
    const uint32_t f = p & 0xFFFFu, tin = (p >> 16) & 0xFFu, tout = p >> 24;
    return End{f == 0xFFFFu ? -1 : (int32_t)((f & 0x3FFFu) | ((f >> 14) << kEndKindShift)), tin == tnil ? -1 : (int32_t)tin,
               tout == tnil ? -1 : (int32_t)tout};
}

// wide class records (DevNode wide: 255 tables or more): interface index | kind << 14 (0xFFFF:
// unresolved) in p, tin | tout << 16 in q (0xFFFF = no ACL)
PG_HD End node_end_wide(uint32_t p, uint32_t q) {
    const uint32_t f = p & 0xFFFFu, tin = q & 0xFFFFu, tout = q >> 16;
    return End{f == 0xFFFFu ? -1 : (int32_t)((f & 0x3FFFu) | ((f >> 14) << kEndKindShift)),
               tin == 0xFFFFu ? -1 : (int32_t)tin, tout == 0xFFFFu ? -1 : (int32_t)tout};
}

struct NoHook {
    PG_HD void operator()() const {}
};

// H: called once per lane, right after the first evaluation's cross-entry loads are issued
// (the kernels issue the next quad's stream loads there; see device.hip PG_PREFETCH)
// CM: the node image's common-row section is in use (device.hpp DevNode): evaluations whose
// (table, IP class) row is the table's common row read it from the image, not the cross table.
// NP: the node set has no PAIR tables (the launcher's build for it: no PAIR code at all)
// UNI: the node's uniform cross layout (DevNode uniform; implies NP): entry addresses computed
// NOFB: no lane ever needs the per-table path (the caller deferred every ANY-protocol packet
// and the node covers every table): its code is left out
template <class L, int Q, class H = NoHook, bool CM = false, bool NP = false, bool UNI = false, bool NOFB = false>
struct NodeEval {
    const DevTableSet& T;
    const DevNode& N;
    const L& img;
    const uint32_t (&src)[Q];
    const uint32_t (&dst)[Q];
    const uint32_t (&ksyn)[Q];
    const uint32_t (&kack)[Q];
    const uint32_t (&cs)[Q];  // node IP class of src
    const uint32_t (&cd)[Q];  // node IP class of dst
    const uint32_t (&gsyn)[Q];  // node key class of the SYN key
    const uint32_t (&gack)[Q];
    const H& hook;
    bool* hooked;
    // UNI with common rows: the common-row masks of the src and dst IP classes (DevNode uniform)
    const W2 (*msk_s)[Q] = nullptr;
    const W2 (*msk_d)[Q] = nullptr;
    PG_HD void operator()(const int32_t (&t)[Q], const bool (&act)[Q], bool rev, uint32_t (&w)[Q]) const {
        bool on[Q], fb[Q];
        first(t, act, rev, on, fb, w);
        rest(t, rev, on, fb, w);
    }
    // The first word of each evaluation (cross entry or common-row word) for the lanes the node
    // covers (on), and which lanes need the per-table path (fb). It depends only on (t, rev):
    // issuing testConnection's four evaluations this way up front was tried (A/B on MI355X,
    // config 5: no gain at two tuples per chunk with counters, -4 % at one without).
    PG_HD void first(const int32_t (&t)[Q], const bool (&act)[Q], bool rev, bool (&on)[Q], bool (&fb)[Q],
                     uint32_t (&w)[Q]) const {
        const DevLoader X{N.cross};
        const uint32_t(&k)[Q] = rev ? kack : ksyn;
        const uint32_t(&ca)[Q] = rev ? cd : cs;  // the IP class on the rule's src side
        const uint32_t(&cb)[Q] = rev ? cs : cd;  // ... and on its dst side (PAIR tables)
        const uint32_t(&gk)[Q] = rev ? gack : gsyn;
        bool cm[Q], pr[Q];
        uint32_t pos[Q], pv[Q] = {}, pk[Q] = {};
        if constexpr (UNI) {  // every table covered, none in PAIR form: no tabinfo / kmap reads
            PG_UNROLL
            for (int j = 0; j < Q; j++) {
                const uint32_t tt = act[j] ? (uint32_t)t[j] : 0u;
                uint32_t cw = 0;
                if (CM) {  // bit t (past 64 tables: t's group) of the rule-src-side class's mask
                    const W2 m = rev ? (*msk_d)[j] : (*msk_s)[j];
                    const uint32_t tb = tt >> N.gshift;
                    cw = bit_of(tb < 32u ? m.x : m.y, tb);
                }
                on[j] = act[j] && k[j] < kWalkKeyLimit;
                cm[j] = CM && cw != 0u;
                // both addresses, then a select (no branch): the common row's entry in the image,
                // or the cross entry (t * G + class) * GK + key class = t * tstride + class * GK + k
                const uint32_t pc = mad24(tt, N.gk, N.crow0 + gk[j]);
                const uint32_t px = mad24(tt, N.tstride, mad24(ca[j], N.gk, gk[j]));
                pos[j] = cm[j] ? pc : px;
                fb[j] = act[j] && !on[j];
                pr[j] = false;
            }
        } else {
        // branch-free: every lane reads its (or table 0's) image words, the flags select
        PG_UNROLL
        for (int j = 0; j < Q; j++) {
            const uint32_t tt = act[j] ? (uint32_t)t[j] : 0u;
            const W4 ti = img.u4(N.tabinfo + 4u * tt);  // {cross base, nkc | covered << 31, common row, 0}
            const uint32_t lk = img.u16(2u * N.kmap + (tt << N.gk_shift) + gk[j]);
            uint32_t cw = 0;
            if (CM) cw = img.u32(N.cmap + (tt << N.cmap_shift) + (ca[j] >> 5u)) >> (ca[j] & 31u);
            on[j] = act[j] && k[j] < kWalkKeyLimit && (ti.y >> 31);
            cm[j] = CM && (cw & 1u);
            pos[j] = cm[j] ? ti.z + lk : ti.x + mul24(ca[j], ti.y & 0xFFFFu) + lk;
            fb[j] = act[j] && !on[j];
            // PAIR table (kNodePairFlag): the pair map entry first, its verdict row after (a
            // uniform test first: node sets without PAIR tables skip this code)
            pr[j] = !NP && N.n_pair && on[j] && (ti.y & kNodePairFlag);
            if (pr[j]) {
                const uint32_t mo = ti.w & 0xFFFFu;
                const uint32_t sc = img.u32(mo + ca[j]) & 0xFFFFu, dc = img.u32(mo + cb[j]) >> 16;
                pos[j] = ti.x + mul24(sc, ti.w >> 16) + dc;
                pv[j] = ti.z + lk;
                pk[j] = ti.y & 0xFFFFu;
            }
        }
        }
        PG_UNROLL
        for (int j = 0; j < Q; j++) {
            if (!on[j]) continue;
#if defined(PG_PROBE_NOGATHER)  // measurement build only: no cross-entry load
            w[j] = pos[j] & 0x3FFFu;
#else
            if (!cm[j]) w[j] = X.u32(pos[j]);
#endif
        }
        if (!NP && N.n_pair) {
            PG_UNROLL
            for (int j = 0; j < Q; j++)
                if (pr[j]) w[j] = X.u32(pv[j] + w[j] * pk[j]);
        }
        if (CM) {
            PG_UNROLL
            for (int j = 0; j < Q; j++)
                if (on[j] && cm[j]) w[j] = img.u32(pos[j]);
        }
        if (!*hooked) {
            *hooked = true;
#if defined(__HIP_DEVICE_COMPILE__)
            __builtin_amdgcn_sched_barrier(0);
#endif
            hook();
#if defined(__HIP_DEVICE_COMPILE__)
            __builtin_amdgcn_sched_barrier(0);
#endif
        }
    }
    // the rest of the evaluations first() started: dst records of kNodeList words, the
    // per-table path for fb lanes
    PG_HD void rest(const int32_t (&t)[Q], bool rev, const bool (&on)[Q], const bool (&fb)[Q], uint32_t (&w)[Q]) const {
        const DevLoader X{N.cross};
        const uint32_t(&a)[Q] = rev ? dst : src;
        const uint32_t(&b)[Q] = rev ? src : dst;
        const uint32_t(&k)[Q] = rev ? kack : ksyn;
        bool pend[Q];
        uint32_t pos[Q];
        PG_UNROLL
        for (int j = 0; j < Q; j++) {
            pend[j] = false;
            pos[j] = 0;
            if (!on[j]) continue;
#if defined(PG_PROBE_NOLIST)  // measurement build only: dst records not walked
            w[j] &= ~kNodeList;
#endif
            pend[j] = (w[j] & kNodeList) != 0u;
            pos[j] = (w[j] & kNodeRecMask) << 2;
        }
        // list-verdict table (N.lv0): one read at [list][node IP class of the rule's dst-side
        // address] (fastpath.cpp build_node: the uniform layout's list form; the other layouts
        // keep the records, so their kernels carry one list path only)
        if constexpr (UNI) {
            const uint32_t(&cb)[Q] = rev ? cs : cd;
            PG_UNROLL
            for (int j = 0; j < Q; j++)
                if (pend[j]) w[j] = X.u32(N.lv0 + (w[j] & kNodeRecMask) * N.n_ipc + cb[j]);
            PG_UNROLL
            for (int j = 0; j < Q; j++) pend[j] = false;
        }
        // record form: dst records until the first match (every list ends with a match-all
        // record), from the image (N.lrec, uniform) or the cross array
        auto walk = [&](const auto& R, uint32_t delta) {
            for (;;) {
                bool more = false;
                PG_UNROLL
                for (int j = 0; j < Q; j++) more |= pend[j];
                if (!more) break;
                PG_UNROLL
                for (int j = 0; j < Q; j++) {
                    if (!pend[j]) continue;
                    const W4 r = R.u4(pos[j] + delta);
                    if (rec_match(r, b[j], k[j])) {
                        w[j] = r.w;
                        pend[j] = false;
                    } else {
                        pos[j] += 4u;
                    }
                }
            }
        };
        if constexpr (!UNI) {
            if (N.lrec) walk(img, N.lrec - N.rec0);
            else walk(X, 0u);
        }
        bool anyfb = false;
        PG_UNROLL
        for (int j = 0; j < Q; j++) anyfb |= fb[j];
#if defined(PG_PROBE_NOFB)  // measurement build only: the per-table fallback compiled out
        anyfb = false;
#endif
        if (NOFB) anyfb = false;
        if (anyfb) {
#if PG_NODE_FB_CALL
            for (int j = 0; j < Q; j++)
                if (fb[j]) w[j] = eval_one(T.rules, T.blobs, T.tabs, t[j], a[j], b[j], k[j]);
#elif PG_NODE_FB_Q1
            // the per-table path one tuple at a time: it is rare here (tables the node does
            // not cover, ANY-protocol packets), and a lockstep walk of Q tuples would size the
            // whole kernel's register allocation
            for (int j = 0; j < Q; j++) {
                if (!fb[j]) continue;
                const DevTable tab1[1] = {load_tab(T.tabs, t[j])};
                const bool on1[1] = {true};
                const uint32_t a1[1] = {a[j]}, b1[1] = {b[j]}, k1[1] = {k[j]};
                uint32_t w1[1];
                eval_q(T, T.blobs, tab1, on1, a1, b1, k1, w1);
                w[j] = w1[0];
            }
#else
            DevTable tab[Q];
            PG_UNROLL
            for (int j = 0; j < Q; j++) tab[j] = fb[j] ? load_tab(T.tabs, t[j]) : DevTable{};
            uint32_t wf[Q];
            eval_q(T, T.blobs, tab, fb, a, b, k, wf);
            PG_UNROLL
            for (int j = 0; j < Q; j++)
                if (fb[j]) w[j] = wf[j];
#endif
        }
    }
};

// one evalACL step of testConnection / per-pod mode: tables t[j] (-1 = no ACL: PERMIT)
template <int Q, bool COUNT, class EV, class HS>
PG_HD void eval_step(const DevTableSet& T, const EV& ev, const int32_t (&t)[Q], const bool (&run)[Q], bool rev,
                     const HS& h, uint32_t (&w)[Q]) {
    bool act[Q];
    PG_UNROLL
    for (int j = 0; j < Q; j++) {
        act[j] = run[j] && t[j] >= 0;
        if (run[j] && t[j] < 0) w[j] = verdict(kActPermit, T.slot_noacl);  // nil ACL (:506-508)
    }
    ev(t, act, rev, w);
    if (COUNT) {
        PG_UNROLL
        for (int j = 0; j < Q; j++)
            if (run[j]) h.inc_t(w[j] & kSlotMask, t[j]);
    }
}

// testConnection (aclengine_mock.go:424-501) of Q connections on resolved end points, each
// of its up-to-4 evalACL steps in lockstep over the Q connections.
// dfr (optional): connections deferred by the caller -- no evaluation and no count here (the
// device's CONN node build classifies ANY-protocol packets after its main loop, device.hip)
template <int Q, bool COUNT, class EV, class HS>
PG_HD void conn_q(const DevTableSet& T, const EV& ev, const End (&es)[Q], const End (&ed)[Q], const HS& h,
                  uint32_t (&out)[Q], const bool* dfr = nullptr) {
    bool live[Q], srefl[Q], drefl[Q], same[Q], run[Q];
    uint32_t w[Q];
    int32_t t[Q];
    PG_UNROLL
    for (int j = 0; j < Q; j++) {
        const bool df = dfr && dfr[j];
        // both interfaces resolved, and a pair the reference has a Connection* call for: the
        // end-point kinds (device.hpp kEndRemote / kEndInet) add to less than 3 -- remote pod <->
        // non-pod and non-pod <-> non-pod fail before any evaluation (aclengine_mock.go:343-347,
        // 388-392). Interfaces keep their kind bits, so "same interface" (srcIfName == dstIfName)
        // holds for remote <-> remote, both through the node-output interface.
        live[j] = !df && es[j].ifc >= 0 && ed[j].ifc >= 0 &&
                  ((uint32_t)es[j].ifc >> kEndKindShift) + ((uint32_t)ed[j].ifc >> kEndKindShift) < 3u;
        srefl[j] = drefl[j] = false;
        same[j] = es[j].ifc == ed[j].ifc;
        w[j] = 0;
        if (!live[j]) {
            out[j] = verdict(3u, T.slot_unresolved);
            if (COUNT && !df) h.inc_cold(T.slot_unresolved);
        }
    }
    // SYN: src interface inbound
    PG_UNROLL
    for (int j = 0; j < Q; j++) t[j] = es[j].tin, run[j] = live[j];
    eval_step<Q, COUNT>(T, ev, t, run, false, h, w);
    PG_UNROLL
    for (int j = 0; j < Q; j++) {
        if (!run[j]) continue;
        const uint32_t a = w[j] >> 30;
        if (a == kActFailure || a == kActDeny) {
            out[j] = verdict(a == kActFailure ? 3u : 0u, w[j] & kSlotMask);
            live[j] = false;
        } else if (a == kActReflect) {
            srefl[j] = true;
            drefl[j] = same[j];
        }
    }
    // SYN: dst interface outbound
    PG_UNROLL
    for (int j = 0; j < Q; j++) t[j] = ed[j].tout, run[j] = live[j] && !drefl[j];
    eval_step<Q, COUNT>(T, ev, t, run, false, h, w);
    PG_UNROLL
    for (int j = 0; j < Q; j++) {
        if (!run[j]) continue;
        const uint32_t a = w[j] >> 30;
        if (a == kActFailure || a == kActDeny) {
            out[j] = verdict(a == kActFailure ? 3u : 0u, w[j] & kSlotMask);
            live[j] = false;
        } else if (a == kActReflect) {
            drefl[j] = true;
            if (same[j]) srefl[j] = true;
        }
    }
    // SYN-ACK: dst interface inbound
    PG_UNROLL
    for (int j = 0; j < Q; j++) t[j] = ed[j].tin, run[j] = live[j] && !drefl[j];
    eval_step<Q, COUNT>(T, ev, t, run, true, h, w);
    PG_UNROLL
    for (int j = 0; j < Q; j++) {
        if (!run[j]) continue;
        const uint32_t a = w[j] >> 30;
        if (a == kActFailure || a == kActDeny) {
            out[j] = verdict(a == kActFailure ? 3u : 1u, w[j] & kSlotMask);
            live[j] = false;
        }
    }
    // SYN-ACK: src interface outbound
    PG_UNROLL
    for (int j = 0; j < Q; j++) t[j] = es[j].tout, run[j] = live[j] && !srefl[j];
    eval_step<Q, COUNT>(T, ev, t, run, true, h, w);
    PG_UNROLL
    for (int j = 0; j < Q; j++) {
        if (!live[j]) continue;
        const uint32_t a = w[j] >> 30;
        if (run[j] && (a == kActFailure || a == kActDeny)) out[j] = verdict(a == kActFailure ? 3u : 1u, w[j] & kSlotMask);
        else out[j] = verdict(2u, w[j] & kSlotMask);  // allowed; slot of the last evaluation
    }
}

#ifndef PG_CONN_UNI  // CONN over a uniform node: conn_uni_q (the packed end points as they are)
#define PG_CONN_UNI 1
#endif
#ifndef PG_POD_UNI  // PERPOD over a uniform node: the same evaluation (uni_eval) on the dst record
#define PG_POD_UNI 1
#endif

// One evalACL of tables t (NIL = no ACL: PERMIT, aclengine_mock.go:506-508) over the lanes `run`
// of a uniform node (DevNode uniform): the cross-entry address from (table, IP class ca on the
// rule's src side, key class g), read from the image when ca's common-row mark m for the table
// is set, else from the cross array; a list resolves through the list-verdict table at the
// rule-dst-side class cb. Counted (run lanes) into h. Key classes of valid keys only (the
// callers leave ANY-protocol packets out of `run`).
// "No ACL" (DevNode tnil): with the common-row section staged (CM) a narrow record's pseudo-table
// reads its row of PERMIT words like any common row, so only wide records and launches without the
// section test the id.
template <int Q, bool COUNT, bool CM, bool WIDE, class L, class HS>
PG_HD void uni_eval(const DevTableSet& T, const DevNode& N, const L& img, const uint32_t (&t)[Q], const bool (&run)[Q],
                    const uint32_t (&ca)[Q], const uint32_t (&cb)[Q], const uint32_t (&g)[Q], const W2 (&m)[Q],
                    const HS& h, uint32_t (&w)[Q]) {
    constexpr bool NILROW = CM && !WIDE;
    const DevLoader X{N.cross};
    bool on[Q], cm[Q];
    uint32_t pos[Q];
    PG_UNROLL
    for (int j = 0; j < Q; j++) {
        on[j] = run[j] && (NILROW || t[j] != N.tnil);
        uint32_t cw = 0;
        if (CM) {  // bit t >> gshift of the class's marks (wide records: one 32-bit word)
            const uint32_t tb = t[j] >> N.gshift;
            cw = WIDE ? bit_of(m[j].x, tb) : (uint32_t)((((uint64_t)m[j].y << 32) | m[j].x) >> (tb & 63u)) & 1u;
        }
        cm[j] = CM && cw != 0u;
        // the common row's entry in the image, or the cross entry t * tstride + class * GK + k
        const uint32_t pc = mad24(t[j], N.gk, N.crow0 + g[j]);
        const uint32_t px = mad24(t[j], N.tstride, mad24(ca[j], N.gk, g[j]));
        pos[j] = cm[j] ? pc : px;
        if (!NILROW && run[j] && !on[j]) w[j] = verdict(kActPermit, T.slot_noacl);  // nil ACL
    }
    PG_UNROLL
    for (int j = 0; j < Q; j++)
        if (on[j] && !cm[j]) w[j] = X.u32(pos[j]);
    if (CM) {
        PG_UNROLL
        for (int j = 0; j < Q; j++)
            if (on[j] && cm[j]) w[j] = img.u32(pos[j]);
    }
    PG_UNROLL
    for (int j = 0; j < Q; j++)  // a list: its verdict for the rule-dst-side address's class
        if (on[j] && (w[j] & kNodeList)) w[j] = X.u32(N.lv0 + (w[j] & kNodeRecMask) * N.n_ipc + cb[j]);
    if (COUNT) {
        PG_UNROLL
        for (int j = 0; j < Q; j++)
            if (run[j]) h.inc_w(w[j]);
    }
}
// an evaluation's ACLAction stops testConnection: DENY (0) or FAILURE (3) -- w + 2^30 then has
// bit 31 clear (PERMIT and REFLECT set it)
PG_HD bool conn_stop(uint32_t w) { return (w + 0x40000000u) < 0x80000000u; }

// testConnection (aclengine_mock.go:424-501) of Q connections over a uniform node's class
// records, ANY-protocol packets deferred (device.hip PG_CONN_DEFER_ANY): conn_q's steps, run on
// the records' packed end points as they are instead of decoded End structs -- the kinds of the
// two interfaces add to 3 or more exactly when the pair has no Connection* call or an interface
// is unresolved (0xFFFF has kind 3), "same interface" is equality of the 16-bit interface
// fields, and a table id equal to DevNode tnil is "no ACL". Every
// evaluation computes its cross-entry address from (table, IP class, key class) and reads it
// from the image when the class's common-row mark is set, else from the cross array; lists
// resolve through the list-verdict table. (Two schedules that ran the SYN-ACK half elsewhere --
// numbered wave-wide and run on other lanes, or the last evaluation in a per-lane loop after all
// of a lane's connections -- measured slower on MI355X, DESIGN.md Appendix A.) Same verdicts, slots and counts as conn_q over NodeEval (tests/test_node_host.py: node ==
// per-table path == oracle).
// rs / rd: the src / dst class records {self, packed end point, marks lo, marks hi} (wide:
// {self, interface, marks, tin | tout << 16}); cs / cd: their classes; gs / ga: the key classes
// of the SYN key (dport) and the SYN-ACK key (sport); dfr: deferred (no evaluation, no count).
template <int Q, bool COUNT, bool CM, bool WIDE, class L, class HS>
PG_HD void conn_uni_q(const DevTableSet& T, const DevNode& N, const L& img, const W4 (&rs)[Q], const W4 (&rd)[Q],
                      const uint32_t (&cs)[Q], const uint32_t (&cd)[Q], const uint32_t (&gs)[Q],
                      const uint32_t (&ga)[Q], const bool (&dfr)[Q], const HS& h, uint32_t (&out)[Q]) {
    bool live[Q], same[Q], srefl[Q], drefl[Q], run[Q];
    uint32_t tsi[Q], tso[Q], tdi[Q], tdo[Q], t[Q], w[Q];
    PG_UNROLL
    for (int j = 0; j < Q; j++) {
        const uint32_t ps = rs[j].y, pd = rd[j].y;
        live[j] = !dfr[j] && ((ps >> 14) & 3u) + ((pd >> 14) & 3u) < 3u;
        same[j] = ((ps ^ pd) & 0xFFFFu) == 0u;
        if (WIDE) {
            tsi[j] = rs[j].w & 0xFFFFu, tso[j] = rs[j].w >> 16, tdi[j] = rd[j].w & 0xFFFFu, tdo[j] = rd[j].w >> 16;
        } else {
            tsi[j] = (ps >> 16) & 0xFFu, tso[j] = ps >> 24, tdi[j] = (pd >> 16) & 0xFFu, tdo[j] = pd >> 24;
        }
        srefl[j] = drefl[j] = false;
        w[j] = 0;
        if (!live[j]) {
            out[j] = verdict(3u, T.slot_unresolved);
            if (COUNT && !dfr[j]) h.inc_cold(T.slot_unresolved);
        }
    }
    W2 ms[Q], md[Q];  // the two classes' common-row marks
    PG_UNROLL
    for (int j = 0; j < Q; j++) ms[j] = W2{rs[j].z, rs[j].w}, md[j] = W2{rd[j].z, rd[j].w};
    // SYN: src interface inbound (the rule's src side is the src class, the SYN key's class). A
    // SYN evaluation that stops the connection gives its ConnAction in the ACLAction bits as they
    // are (DENY 0 -> DenySyn 0, FAILURE 3 -> Failure 3); a SYN-ACK one ORs in 1 (-> DenySynAck 1,
    // Failure 3)
    PG_UNROLL
    for (int j = 0; j < Q; j++) t[j] = tsi[j], run[j] = live[j];
    uni_eval<Q, COUNT, CM, WIDE>(T, N, img, t, run, cs, cd, gs, ms, h, w);
    PG_UNROLL
    for (int j = 0; j < Q; j++) {
        const bool stop = run[j] && conn_stop(w[j]), refl = run[j] && (w[j] >> 30) == kActReflect;
        if (stop) out[j] = w[j];
        live[j] = live[j] && !stop;
        srefl[j] = refl;
        drefl[j] = refl && same[j];
    }
    // SYN: dst interface outbound
    PG_UNROLL
    for (int j = 0; j < Q; j++) t[j] = tdo[j], run[j] = live[j] && !drefl[j];
    uni_eval<Q, COUNT, CM, WIDE>(T, N, img, t, run, cs, cd, gs, ms, h, w);
    PG_UNROLL
    for (int j = 0; j < Q; j++) {
        const bool stop = run[j] && conn_stop(w[j]), refl = run[j] && (w[j] >> 30) == kActReflect;
        if (stop) out[j] = w[j];
        live[j] = live[j] && !stop;
        drefl[j] = drefl[j] || refl;
        srefl[j] = srefl[j] || (refl && same[j]);
    }
    // SYN-ACK: dst interface inbound (reversed packet: the rule's src side is the dst class, the
    // SYN-ACK key's class)
    PG_UNROLL
    for (int j = 0; j < Q; j++) t[j] = tdi[j], run[j] = live[j] && !drefl[j];
    uni_eval<Q, COUNT, CM, WIDE>(T, N, img, t, run, cd, cs, ga, md, h, w);
    PG_UNROLL
    for (int j = 0; j < Q; j++) {
        const bool stop = run[j] && conn_stop(w[j]);
        if (stop) out[j] = w[j] | 1u << 30;
        live[j] = live[j] && !stop;
    }
    // SYN-ACK: src interface outbound
    PG_UNROLL
    for (int j = 0; j < Q; j++) t[j] = tso[j], run[j] = live[j] && !srefl[j];
    uni_eval<Q, COUNT, CM, WIDE>(T, N, img, t, run, cd, cs, ga, md, h, w);
    PG_UNROLL
    for (int j = 0; j < Q; j++)  // allowed: the slot of the last evaluation
        if (live[j]) out[j] = run[j] && conn_stop(w[j]) ? w[j] | 1u << 30 : (w[j] & kSlotMask) | 2u << 30;
}

// evalACL of ANY-protocol packets (the L4 test skipped, aclengine_mock.go:562): the first rule
// whose src and dst match, with its ANY action (engine.cpp compile_acl_rule) -- eval_linear's
// ANY branch, inline: the CONN node build's deferred pass calls nothing (a call anywhere in a
// kernel costs its whole SGPR allocation)
template <int Q>
struct AnyEval {
    const DevTableSet& T;
    const uint32_t (&src)[Q];
    const uint32_t (&dst)[Q];
    PG_HD void operator()(const int32_t (&t)[Q], const bool (&act)[Q], bool rev, uint32_t (&w)[Q]) const {
        for (int j = 0; j < Q; j++) {
            if (!act[j]) continue;
            const DevTable tab = load_tab(T.tabs, t[j]);
            const uint32_t a = rev ? dst[j] : src[j], b = rev ? src[j] : dst[j];
            uint32_t v = tab.dflt;
            for (uint32_t i = 0; i < tab.n_rules; i++) {
                const DevRule r = T.rules[tab.rule_base + i];
                if ((a & r.smask) == r.snet && (b & r.dmask) == r.dnet && (r.act >> 4) != kActNever) {
                    v = verdict((r.act >> 4) & 3u, tab.rule_base + i);
                    break;
                }
            }
            w[j] = v;
        }
    }
};

// testConnection of one ANY-protocol connection through the iphash and AnyEval (the CONN node
// build's deferred pass, device.hip PG_CONN_DEFER_ANY)
template <bool COUNT, class HS>
PG_HD uint32_t conn_any_1(const DevTableSet& T, uint32_t s, uint32_t d, const HS& h) {
    const uint32_t ips[2] = {s, d};
    End e[2];
    probe_q(T, ips, e);
    const End es[1] = {e[0]}, ed[1] = {e[1]};
    const uint32_t s1[1] = {s}, d1[1] = {d};
    const AnyEval<1> ev{T, s1, d1};
    uint32_t o[1];
    conn_q<1, COUNT>(T, ev, es, ed, h, o);
    return o[0];
}

// the per-pod evaluation (the outbound ACL of dst's interface) of one ANY-protocol packet through
// the iphash and AnyEval (the PERPOD node build's deferred pass, device.hip PG_POD_DEFER_ANY)
template <bool COUNT, class HS>
PG_HD uint32_t pod_any_1(const DevTableSet& T, uint32_t s, uint32_t d, const HS& h) {
    const uint32_t d1[1] = {d}, s1[1] = {s};
    End e[1];
    probe_q(T, d1, e);
    const bool run[1] = {e[0].ifc >= 0};
    const int32_t t[1] = {e[0].tout};
    uint32_t o[1] = {verdict(kActFailure, T.slot_unresolved)};
    if (COUNT && !run[0]) h.inc_cold(T.slot_unresolved);
    const AnyEval<1> ev{T, s1, d1};
    eval_step<1, COUNT>(T, ev, t, run, false, h, o);
    return o[0];
}

// Q tuples of one lane, any mode, per-table path. SINGLE: tab0 is the (uniform) table, its
// blob at `blobs`.
template <int MODE, bool COUNT, int Q, bool PRED = false, class HS = Hist>
PG_HD void classify_q(const DevTableSet& T, const uint32_t* blobs, const DevTable& tab0, const uint32_t (&s)[Q],
                      const uint32_t (&d)[Q], const uint32_t (&sp)[Q], const uint32_t (&dp)[Q],
                      const uint32_t (&pr)[Q], const HS& h, uint32_t (&out)[Q], const uint32_t* rootb = nullptr) {
    uint32_t key[Q], kack[Q];
    PG_UNROLL
    for (int j = 0; j < Q; j++) key[j] = pkt_key(pr[j], dp[j]), kack[j] = pkt_key(pr[j], sp[j]);
    if (MODE == 0) {  // SINGLE
        DevTable tab[Q];
        bool act[Q];
        PG_UNROLL
        for (int j = 0; j < Q; j++) tab[j] = tab0, act[j] = true;
        eval_q<PRED>(T, blobs, tab, act, s, d, key, out, rootb);
        if (COUNT) {
            PG_UNROLL
            for (int j = 0; j < Q; j++) h.inc(out[j] & kSlotMask);
        }
        return;
    }
    const TabEval<Q> ev{T, s, d, key, kack};
    if (MODE == 1) {  // PERPOD: outbound ACL of the interface dst is reached by
        End e[Q];
        probe_q(T, d, e);
        int32_t t[Q];
        bool run[Q];
        PG_UNROLL
        for (int j = 0; j < Q; j++) {
            run[j] = e[j].ifc >= 0;
            t[j] = e[j].tout;
            if (!run[j]) {
                out[j] = verdict(kActFailure, T.slot_unresolved);
                if (COUNT) h.inc_cold(T.slot_unresolved);
            }
        }
        eval_step<Q, COUNT>(T, ev, t, run, false, h, out);
    } else {  // CONN
        uint32_t ips[2 * Q];
        End e[2 * Q];
        PG_UNROLL
        for (int j = 0; j < Q; j++) ips[j] = s[j], ips[Q + j] = d[j];
        probe_q(T, ips, e);
        End es[Q], ed[Q];
        PG_UNROLL
        for (int j = 0; j < Q; j++) es[j] = e[j], ed[j] = e[Q + j];
        conn_q<Q, COUNT>(T, ev, es, ed, h, out);
    }
}

// Q tuples of one lane, PERPOD / CONN, node path. `img` reads the node image (LDS copy or
// global memory).
// DEFER (PERPOD / CONN over a uniform node, every table covered): ANY-protocol packets (the
// only ones the node cannot classify) are left to the caller -- no evaluation, no count, a
// placeholder verdict -- so the evaluation carries no per-table fallback (device.hip
// PG_CONN_DEFER_ANY, PG_POD_DEFER_ANY)
// WIDE (UNI): the node's wide class records (DevNode wide: 16-bit table ids in record word 3, the
// common-row marks one 32-bit word)
template <int MODE, bool COUNT, int Q, bool PRED = false, bool CM = false, bool NP = false, bool UNI = false,
          bool DEFER = false, bool WIDE = false, class L, class HS, class H = NoHook>
PG_HD void classify_node_q(const DevTableSet& T, const DevNode& N, const L& img, const uint32_t (&s)[Q],
                           const uint32_t (&d)[Q], const uint32_t (&sp)[Q], const uint32_t (&dp)[Q],
                           const uint32_t (&pr)[Q], const HS& h, uint32_t (&out)[Q], const H& hook = H()) {
    uint32_t key[Q], kack[Q];
    PG_UNROLL
    for (int j = 0; j < Q; j++) key[j] = pkt_key(pr[j], dp[j]), kack[j] = MODE == 2 ? pkt_key(pr[j], sp[j]) : key[j];
    // CONN over a uniform node, ANY-protocol packets deferred: the keys of the other protocols
    // as pkt_key gives them, and for a deferred packet any key below 2^18 (its walks' results are
    // not used) -- so the keys need no clamp before the walks
    constexpr bool KEYS18 = MODE == 2 && UNI && DEFER && PG_CONN_UNI;
    if constexpr (KEYS18) {
        PG_UNROLL
        for (int j = 0; j < Q; j++) {
            const uint32_t prm = (pr[j] & 3u) << 16, pm = pr[j] < 2u ? 0xFFFFu : 0u;
            key[j] = prm | (dp[j] & pm);
            kack[j] = prm | (sp[j] & pm);
        }
    }
    // node IP class records of src and dst, node key classes of both keys: 2Q + 2Q trie walks
    uint32_t ips[2 * Q], rec[2 * Q];
    PG_UNROLL
    for (int j = 0; j < Q; j++) ips[j] = s[j], ips[Q + j] = d[j];
    uint32_t cs[Q], cd[Q], gs[Q], ga[Q];
#if PG_NODE_WALK2 && !defined(PG_PROBE_NOWALK)
    if (MODE == 2) {
        uint32_t keys[2 * Q], kc[2 * Q];
        PG_UNROLL
        for (int j = 0; j < Q; j++) {
            keys[j] = KEYS18 || key[j] < kWalkKeyLimit ? key[j] : 0u;
            keys[Q + j] = KEYS18 || kack[j] < kWalkKeyLimit ? kack[j] : 0u;
        }
        node_walks<PRED, UNI>(img, N, ips, rec, keys, kc);
        PG_UNROLL
        for (int j = 0; j < Q; j++) gs[j] = kc[j], ga[j] = kc[Q + j];
    } else {
        uint32_t keys[Q];
        PG_UNROLL
        for (int j = 0; j < Q; j++) keys[j] = key[j] < kWalkKeyLimit ? key[j] : 0u;
#if defined(PG_PROBE_NODSTWALK)  // measurement build only: PERPOD walks src only (dst class = src's)
        {
            uint32_t sa[Q], sr[Q];
            PG_UNROLL
            for (int j = 0; j < Q; j++) sa[j] = ips[j];
            node_walks<PRED, UNI>(img, N, sa, sr, keys, gs);
            PG_UNROLL
            for (int j = 0; j < Q; j++) rec[j] = sr[j], rec[Q + j] = sr[j];
        }
#else
        node_walks<PRED, UNI>(img, N, ips, rec, keys, gs);
#endif
        PG_UNROLL
        for (int j = 0; j < Q; j++) ga[j] = gs[j];
    }
#else
#if defined(PG_PROBE_NOWALK)  // measurement build only: IP classes without the trie walk
    PG_UNROLL
    for (int j = 0; j < 2 * Q; j++) rec[j] = (ips[j] % N.n_ipc + N.ipself) << node_ip_rec_shift<UNI>();
#else
    node_trie_q<PRED, UNI>(img, 0u, N.ip_s1, 32u, N.ip_depth, ips, rec);
#endif
    {
        const uint32_t nk = MODE == 2 ? 2 * Q : Q;
        uint32_t keys[2 * Q], kr[2 * Q];
        PG_UNROLL
        for (int j = 0; j < Q; j++) {
            keys[j] = key[j] < kWalkKeyLimit ? key[j] : 0u;
            keys[Q + j] = kack[j] < kWalkKeyLimit ? kack[j] : 0u;
        }
        node_trie_q<PRED, UNI>(img, N.key_root, N.key_k1, 18u, N.key_depth, keys, kr);
        PG_UNROLL
        for (int j = 0; j < Q; j++) {
            gs[j] = (kr[j] >> node_key_rec_shift<UNI>()) - N.kself;
            ga[j] = nk > (uint32_t)Q ? (kr[Q + j] >> node_key_rec_shift<UNI>()) - N.kself : gs[j];
        }
    }
#endif
    // the class numbers (cross-array rows): records from record ipself on
    constexpr uint32_t RS = node_ip_rec_shift<UNI>();
    PG_UNROLL
    for (int j = 0; j < Q; j++) cs[j] = (rec[j] >> RS) - N.ipself, cd[j] = (rec[Q + j] >> RS) - N.ipself;
    bool hooked = false;
    if constexpr (MODE == 2 && UNI && DEFER && PG_CONN_UNI) {  // CONN over the class records as they are
        W4 rs[Q], rd[Q];
        bool dfr[Q];
        PG_UNROLL
        for (int j = 0; j < Q; j++) {
            rs[j] = img.u4_at_byte(rec[j]), rd[j] = img.u4_at_byte(rec[Q + j]);
            dfr[j] = pr[j] > 2u;  // (ANY protocol: both keys >= kWalkKeyLimit in pkt_key)
        }
        conn_uni_q<Q, COUNT, CM, WIDE>(T, N, img, rs, rd, cs, cd, gs, ga, dfr, h, out);
        hook();
        return;
    }
    if constexpr (MODE == 1 && UNI && PG_POD_UNI) {  // PERPOD: the dst record's outbound table as it is
        uint32_t t[Q];
        bool run[Q], fbk[Q];
        W2 ms[Q];
        PG_UNROLL
        for (int j = 0; j < Q; j++) {
            const uint32_t pd = img.at_byte(rec[Q + j] + 4u);  // interface | kind << 14 (0xFFFF: unresolved)
            t[j] = WIDE ? img.at_byte(rec[Q + j] + 12u) >> 16 : pd >> 24;
            ms[j] = !CM ? W2{0u, 0u} : (WIDE ? W2{img.at_byte(rec[j] + 8u), 0u} : img.u2_at_byte(rec[j] + 8u));
            const bool df = DEFER && key[j] >= kWalkKeyLimit;  // (deferred: left to the caller)
            run[j] = !df && (pd & 0xFFFFu) != 0xFFFFu;
            if (!run[j]) {
                out[j] = verdict(kActFailure, T.slot_unresolved);
                if (COUNT && !df) h.inc_cold(T.slot_unresolved);
            }
            // ANY-protocol packets (no key class) on a table: the per-table path below
            fbk[j] = run[j] && key[j] >= kWalkKeyLimit && t[j] != N.tnil;
            run[j] = run[j] && !fbk[j];
        }
        uni_eval<Q, COUNT, CM, WIDE>(T, N, img, t, run, cs, cd, gs, ms, h, out);
        bool anyfb = false;
        PG_UNROLL
        for (int j = 0; j < Q; j++) anyfb |= fbk[j];
        if (!DEFER && anyfb) {
            for (int j = 0; j < Q; j++) {
                if (!fbk[j]) continue;
                out[j] = eval_one(T.rules, T.blobs, T.tabs, (int32_t)t[j], s[j], d[j], key[j]);
                if (COUNT) h.inc_t(out[j] & kSlotMask, (int32_t)t[j]);
            }
        }
        hook();
        return;
    }
    W2 mks[Q], mkd[Q];  // UNI: the common-row masks of the two classes, read once per tuple
    End es[Q], ed[Q];   // CONN: both end points; PERPOD: ed
    PG_UNROLL
    for (int j = 0; j < Q; j++) {
        if constexpr (UNI && WIDE) {  // record {self, interface, marks, tin | tout << 16}
            if (MODE == 2) {
                const W4 rs = img.u4_at_byte(rec[j]), rd = img.u4_at_byte(rec[Q + j]);
                es[j] = node_end_wide(rs.y, rs.w), ed[j] = node_end_wide(rd.y, rd.w);
                mks[j] = W2{rs.z, 0u}, mkd[j] = W2{rd.z, 0u};  // (T <= 32 << gshift: the low word only)
            } else {
                const W2 rd = img.u2_at_byte(rec[Q + j] + 8u);  // {marks, tables} of dst's record
                ed[j] = node_end_wide(img.at_byte(rec[Q + j] + 4u), rd.y);
                mks[j] = W2{CM ? img.at_byte(rec[j] + 8u) : 0u, 0u};
                mkd[j] = mks[j];
            }
        } else if constexpr (UNI) {  // record {self, packed end point, mask lo, mask hi}
            if (MODE == 2) {
                const W4 rs = img.u4_at_byte(rec[j]), rd = img.u4_at_byte(rec[Q + j]);
                es[j] = node_end_packed(rs.y, N.tnil), ed[j] = node_end_packed(rd.y, N.tnil);
                mks[j] = W2{rs.z, rs.w}, mkd[j] = W2{rd.z, rd.w};
            } else {
                ed[j] = node_end_packed(img.at_byte(rec[Q + j] + 4u), N.tnil);
                mks[j] = CM ? img.u2_at_byte(rec[j] + 8u) : W2{0u, 0u};
                mkd[j] = mks[j];
            }
        } else {  // self words; ipinfo {interface, tin | tout << 16} per class
            if (MODE == 2) es[j] = node_end(img, N, cs[j]);
            ed[j] = node_end(img, N, cd[j]);
        }
    }
    constexpr bool DF = DEFER && UNI;
    const NodeEval<L, Q, H, CM, NP || UNI, UNI, DF> ev{T, N, img, s, d, key, kack, cs, cd, gs, ga, hook, &hooked, &mks, &mkd};
    if (MODE == 1) {
        int32_t t[Q];
        bool run[Q];
        PG_UNROLL
        for (int j = 0; j < Q; j++) {
            // (DF) an ANY-protocol packet: left to the caller (placeholder verdict, no count)
            const bool df = DF && key[j] >= kWalkKeyLimit;
            run[j] = !df && ed[j].ifc >= 0;
            t[j] = ed[j].tout;
            if (!run[j]) {
                out[j] = verdict(kActFailure, T.slot_unresolved);
                if (COUNT && !df) h.inc_cold(T.slot_unresolved);
            }
        }
        eval_step<Q, COUNT>(T, ev, t, run, false, h, out);
    } else {
        if (DF) {
            bool dfr[Q];
            PG_UNROLL
            for (int j = 0; j < Q; j++) dfr[j] = key[j] >= kWalkKeyLimit || kack[j] >= kWalkKeyLimit;
            conn_q<Q, COUNT>(T, ev, es, ed, h, out, dfr);
        } else {
            conn_q<Q, COUNT>(T, ev, es, ed, h, out);
        }
    }
    if (!hooked) hook();  // no evaluation ran in this lane
}

}  // namespace pg
