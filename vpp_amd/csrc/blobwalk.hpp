// The walk of a classification blob (layout: fastpath.cpp), written once for both sides:
// the HIP kernels instantiate it with a loader that issues 16/8/4-byte LDS or global loads,
// and pg_debug_walk_blob (tests only, never on the classify path) instantiates it with a
// host loader, so the table compiler is checked against the oracle without a GPU.
//
// The walk is "lockstep" over Q tuples (Q = 4 per lane in the kernels): every dependent
// step (trie level, cross entry, record) issues the loads of all Q tuples before consuming
// any of them, so a lane keeps up to 2Q independent loads in flight instead of one chain.
#pragma once
#include <cstdint>

#if defined(__HIPCC__)
#define PG_HD __host__ __device__ __forceinline__
#define PG_UNROLL _Pragma("unroll")
#else
#define PG_HD inline
#define PG_UNROLL _Pragma("GCC unroll 4")
#endif

namespace pg {

constexpr uint32_t kFlagCross = 1u, kFlagLists = 2u, kFlagCand = 4u, kFlagLinear = 8u, kFlagPair = 16u;
// FD ("fixed depth", fastpath.cpp build_fd_blob): a CROSS table whose verdict does not
// depend on the dst address, laid out so that every lookup is exactly D dependent reads per
// field and one verdict read, with no per-lane branches (fd_walk below).
constexpr uint32_t kFlagFD = 32u;
// no rule of the table tests dst (set by engine.cpp in DevTable::fsk, not in the blob): SINGLE
// launches do not read the dst stream
constexpr uint32_t kFlagDstFree = 64u;
// CANDI ("candidates inline", fastpath.cpp build_candi): a CAND table no live rule of which
// tests dst, read from HBM. Below the (LDS-staged, 4-B) src root, trie entries are 8 B and a
// leaf carries its src class's single candidate (or the table's default) itself, so most
// lookups end with the trie read instead of a further record gather (blobwalk candi_walk).
constexpr uint32_t kFlagCandI = 128u;
// 8-B CANDI entry {w0, w1}: w1 bit 31 clear = an inline candidate: key range klo = w0 & 0x3FFFF,
// khi = w0 >> 18 | (w1 & 15) << 14, action (w1 >> 4) & 3, rule w1 >> 6 (relative to the table's
// first rule; kCandiDefault = the table's default verdict); w1 bit 31 set = kCandiInternal:
// child block at word w0, stride w1 & 31; else the class's record list at record w0.
constexpr uint32_t kCandiNode = 1u << 31, kCandiInternal = 1u << 30, kCandiDefault = 0x1FFFFFFu;

constexpr uint32_t kPairHdr = 12u;  // PAIR blob header words: dst root, d1, pair table, n_dst_classes
constexpr uint32_t kLeaf = 0x80000000u;
// non-leaf trie entry: child block offset (words) | child stride << kTrieStrideShift
constexpr uint32_t kTrieStrideShift = 26u, kTrieChildMask = (1u << kTrieStrideShift) - 1u;
PG_HD uint32_t trie_child(uint32_t e) { return e & kTrieChildMask; }
PG_HD uint32_t trie_stride(uint32_t e) { return (e >> kTrieStrideShift) & 31u; }
// Node-image tries (LDS-staged). The node tries take uniform strides below the root (min(8,
// bits left)), so the bit offset of a level's index is the same for every entry -- a per-level
// constant the walk keeps in a scalar register (node_next_shift). A leaf points at its
// class's record (DevNode) with stride 0: a record a leaf above the last level points at holds
// that leaf's value in its first word, so a finished lookup re-reads it and every lookup takes
// exactly the trie's depth in reads. Two encodings:
//  * aligned (the uniform node layout; fastpath.cpp build_trie kEncNodeA): an entry is a byte
//    address. The builder places every child table at an address congruent to its stride mod
//    32 (strides below the root are then 8 or 4: the root stride is a multiple of 4), so the
//    entry's low 5 bits are the stride, and a leaf above the last level points at a record on a
//    32-byte boundary. The child entry of address a is at byte
//      e + 4 * ((a >> shift) & ((1 << (e & 31)) - 1))
//    -- on the device one v_bfe_u32 (its width operand is e itself: the hardware reads only the
//    low 5 bits) and one v_lshl_add_u32.
//  * shifted (kEncNode): entry = byte address << 5 | stride, any strides: one shift of e more.
constexpr uint32_t kNodeChildMaxWords = 1u << 25;  // 128 MiB of image (shifted byte addresses in 32 bits)
constexpr uint32_t kNodeStride = 8;  // stride of the levels below the root
PG_HD constexpr uint32_t node_entry(uint32_t child_words, uint32_t stride, bool aligned) {
    return aligned ? child_words * 4u : (child_words * 4u) << 5 | stride;
}
// bits below the next level, given the bits below the current one (uniform per level)
PG_HD uint32_t node_next_shift(uint32_t rem) { return rem - (rem < kNodeStride ? rem : kNodeStride); }
template <bool ALIGNED>
PG_HD uint32_t node_child_byte(uint32_t e, uint32_t a, uint32_t shift) {
#if defined(__HIP_DEVICE_COMPILE__)
    const uint32_t idx = __builtin_amdgcn_ubfe(a, shift, e);
#else
    const uint32_t w = e & 31u;
    const uint32_t idx = shift >= 32u ? 0u : (a >> shift) & (w >= 32u ? 0xFFFFFFFFu : ((1u << w) - 1u));
#endif
    return (ALIGNED ? e : e >> 5) + (idx << 2);
}
// node class records (DevNode), log2 bytes: the uniform layout (aligned tries, A) IPv4 16 B
// and key 32 B; otherwise 4-B self words
template <bool A>
PG_HD constexpr uint32_t node_ip_rec_shift() { return A ? 4u : 2u; }
template <bool A>
PG_HD constexpr uint32_t node_key_rec_shift() { return A ? 5u : 2u; }
constexpr uint32_t kSrcRoot = 16u;       // the src trie root follows the 16-word blob header
// CANDI window (fastpath.cpp, the CANDI builder): blob words [candi_window_off, + 2 * size) after
// the src root hold the terminal 8-B entry of every address of [base, base + size) (DevTable /
// BlobTab kroot = base, nkc = size; size 0 = no window), staged in LDS with the root
PG_HD constexpr uint32_t candi_window_off(uint32_t s1) { return kSrcRoot + (1u << s1); }
// words of a blob's prefix a launch stages when the src root alone is staged: header, root and
// (CANDI) the window, rounded to 16 B
PG_HD constexpr uint32_t blob_root_words(uint32_t fsk, uint32_t nkc) {
    return (((fsk & kFlagCandI) && nkc ? candi_window_off((fsk >> 8) & 0xFFu) + 2u * nkc
                                       : kSrcRoot + (1u << ((fsk >> 8) & 0xFFu))) + 3u) & ~3u;
}
// the largest table array (a table's blob, the node image, the node cross array) a DevLoader
// reads: its byte offsets are 32-bit (classify.hpp)
constexpr uint64_t kMaxLoaderBytes = 1ull << 32;
constexpr uint32_t kWalkKeyLimit = 0x30000u;  // keys >= this (ANY protocol) take the linear path
// key bound of records that match every key: covers the whole 18-bit walk range, ANY keys
// included, so every list terminates for any key the walk is given
constexpr uint32_t kRecKeyAll = 0x3FFFFu;

struct W2 {
    uint32_t x, y;
};
struct W4 {
    uint32_t x, y, z, w;
};

// What a walk needs of a table (the device keeps it in DevTable, 32 B).
struct BlobTab {
    uint32_t fsk;    // flags | s1 << 8 | k1 << 16
    uint32_t dflt;   // default verdict (DENY << 30 | default slot)
    uint32_t kroot;  // key trie root (words)
    uint32_t xoff;   // cross table (CROSS) or first record (CAND), words
    uint32_t nkc;    // key classes
    uint32_t rbase;  // first rule's counter slot (CANDI inline candidates)
};

// Record (16 B): {dnet, klo | dlen << 18 | last << 24, khi, verdict}: matches when the dst
// prefix of length dlen equals dnet and klo <= key <= khi. Dst lists (LISTS, node lists) end
// with a record that matches every packet and carries the fall-through verdict; candidate
// lists (CAND) instead flag their last record (kRecLast): no match there -> the table's
// default deny (an empty candidate list is one match-all record carrying it).
constexpr uint32_t kRecLast = 1u << 24;
PG_HD uint32_t rec_mask(uint32_t dlen) { return dlen ? (0xFFFFFFFFu << (32u - dlen)) : 0u; }
PG_HD bool rec_match(const W4& r, uint32_t dst, uint32_t key) {
    return (dst & rec_mask((r.y >> 18) & 63u)) == r.x && key >= (r.y & 0x3FFFFu) && key <= r.z;
}

// on[j]: tuple j is walked (table present, not LINEAR). w[j] is only written for those. Keys
// must be < 2^18; the result for keys >= kWalkKeyLimit (ANY protocol) is meaningless and the
// caller replaces it.
// PRED: the trie descent issues a load for every tuple at every level (a finished tuple
// re-reads word 0) instead of branching per tuple: cheaper when the blob is in LDS, where a
// wasted read costs little and per-lane branches cost exec-mask juggling.
// ld0: loaders for the src trie root (a blob whose root alone is staged in LDS: ld0 reads the
// LDS copy, ld the blob in HBM; otherwise the same loaders).
// CANDI lanes (ci) of a walk: the 4-B root (ld0), then 8-B entries until an inline candidate
// (w set) or a pointer to the class's record list (pend, pos: the caller walks the records,
// rec_walk). A lane that finished issues no further load. An address in the table's window
// reads its terminal entry from ld0 instead (no root read, no gather).
template <class L, class L0, int Q>
PG_HD void candi_walk(const L (&ld)[Q], const L0 (&ld0)[Q], const BlobTab (&tb)[Q], const bool (&ci)[Q],
                      const uint32_t (&src)[Q], const uint32_t (&key)[Q], uint32_t (&w)[Q], bool (&pend)[Q],
                      uint32_t (&pos)[Q]) {
    uint32_t cw[Q], cst[Q], ss[Q];
    bool cwalk[Q];
    // a window entry (terminal): a record-list pointer or an inline candidate
    auto entry = [&](int j, const W2& v) {
        if (v.y & kCandiNode) {
            pos[j] = tb[j].xoff + 4u * v.x;
            pend[j] = true;
            return;
        }
        const uint32_t klo = v.x & 0x3FFFFu, khi = (v.x >> 18) | ((v.y & 15u) << 14);
        const uint32_t rel = (v.y >> 6) & kCandiDefault;
        const bool hit = key[j] >= klo && key[j] <= khi && rel != kCandiDefault;
        w[j] = hit ? (((v.y >> 4) & 3u) << 30) | (tb[j].rbase + rel) : tb[j].dflt;
    };
    PG_UNROLL
    for (int j = 0; j < Q; j++) {
        cwalk[j] = false;
        cw[j] = cst[j] = ss[j] = 0;
        if (!ci[j]) continue;
        const uint32_t s1 = (tb[j].fsk >> 8) & 0xFFu;
        ss[j] = 32u - s1;
        const uint32_t wd = src[j] - tb[j].kroot;
        if (wd < tb[j].nkc) {  // the window: the address's terminal entry (never internal)
            entry(j, ld0[j].u2(candi_window_off(s1) + 2u * wd));
            continue;
        }
        const uint32_t e = ld0[j].u32(kSrcRoot + (src[j] >> ss[j]));
        if (e & kLeaf) {
            pos[j] = tb[j].xoff + 4u * (e & ~kLeaf);
            pend[j] = true;
        } else {
            cw[j] = trie_child(e);
            cst[j] = trie_stride(e);
            cwalk[j] = true;
        }
    }
    for (;;) {
        bool more = false;
        PG_UNROLL
        for (int j = 0; j < Q; j++) more |= cwalk[j];
        if (!more) break;
        PG_UNROLL
        for (int j = 0; j < Q; j++) {
            if (!cwalk[j]) continue;
            ss[j] -= cst[j];
            // (the entry decoded in place, not through entry(): A/B on MI355X, config 4 with
            // counters 108.8 vs 113.4 Gpps)
            const W2 v = ld[j].u2(cw[j] + 2u * ((src[j] >> ss[j]) & ((1u << cst[j]) - 1u)));
            if (v.y & kCandiNode) {
                if (v.y & kCandiInternal) {
                    cw[j] = v.x;
                    cst[j] = v.y & 31u;
                } else {
                    pos[j] = tb[j].xoff + 4u * v.x;
                    pend[j] = true;
                    cwalk[j] = false;
                }
            } else {
                const uint32_t klo = v.x & 0x3FFFFu, khi = (v.x >> 18) | ((v.y & 15u) << 14);
                const uint32_t rel = (v.y >> 6) & kCandiDefault;
                const bool hit = key[j] >= klo && key[j] <= khi && rel != kCandiDefault;
                w[j] = hit ? (((v.y >> 4) & 3u) << 30) | (tb[j].rbase + rel) : tb[j].dflt;
                cwalk[j] = false;
            }
        }
    }
}

// records of the pend lanes until the first match (every list ends with a match-all record or
// flags its last one: no match there -> the table's default)
template <class L, int Q>
PG_HD void rec_walk(const L (&ld)[Q], const BlobTab (&tb)[Q], const uint32_t (&dst)[Q], const uint32_t (&key)[Q],
                    bool (&pend)[Q], uint32_t (&pos)[Q], uint32_t (&w)[Q]) {
    for (;;) {
        bool more = false;
        PG_UNROLL
        for (int j = 0; j < Q; j++) more |= pend[j];
        if (!more) break;
        PG_UNROLL
        for (int j = 0; j < Q; j++) {
            if (!pend[j]) continue;
            const W4 r = ld[j].u4(pos[j]);
            if (rec_match(r, dst[j], key[j])) {
                w[j] = r.w;
                pend[j] = false;
            } else if (r.y & kRecLast) {
                w[j] = tb[j].dflt;
                pend[j] = false;
            } else {
                pos[j] += 4u;
            }
        }
    }
}

template <bool PRED = false, class L, class L0, int Q>
PG_HD void blob_walk(const L (&ld)[Q], const L0 (&ld0)[Q], const BlobTab (&tb)[Q], const bool (&on)[Q],
                     const uint32_t (&src)[Q], const uint32_t (&dst)[Q], const uint32_t (&key)[Q], uint32_t (&w)[Q]) {
    uint32_t es[Q], ek[Q], ss[Q], sk[Q], ed[Q], sd[Q];
    // CANDI lanes (kFlagCandI): 8-B entries below the root, inline candidates (candi_walk)
    uint32_t pos[Q];
    bool ci[Q], pend[Q], anyci = false;
    PG_UNROLL
    for (int j = 0; j < Q; j++) {
        ci[j] = on[j] && (tb[j].fsk & kFlagCandI);
        anyci |= ci[j];
        pend[j] = false;
        pos[j] = 0;
    }
    if (anyci) candi_walk(ld, ld0, tb, ci, src, key, w, pend, pos);
    PG_UNROLL
    for (int j = 0; j < Q; j++) {
        es[j] = ek[j] = ed[j] = kLeaf;
        ss[j] = sk[j] = sd[j] = 0;
        if (on[j] && !ci[j]) {
            ss[j] = 32u - ((tb[j].fsk >> 8) & 0xFFu);
            es[j] = ld0[j].u32(kSrcRoot + (src[j] >> ss[j]));
            if (tb[j].fsk & (kFlagCross | kFlagPair)) {
                sk[j] = 18u - ((tb[j].fsk >> 16) & 0xFFu);
                ek[j] = ld[j].u32(tb[j].kroot + (key[j] >> sk[j]));
            }
        }
    }
    // PAIR tables: the dst trie too (its root and stride are in the blob header)
    PG_UNROLL
    for (int j = 0; j < Q; j++) {
        if (on[j] && !ci[j] && (tb[j].fsk & kFlagPair)) {
            const W2 h = ld[j].u2(kPairHdr);
            sd[j] = 32u - h.y;
            ed[j] = ld[j].u32(h.x + (dst[j] >> sd[j]));
        }
    }
    // descend the multibit tries (root stride, then each node's stride) of all Q tuples together
    for (;;) {
        bool more = false;
        PG_UNROLL
        for (int j = 0; j < Q; j++) more |= !(es[j] & ek[j] & ed[j] & kLeaf);
        if (!more) break;
        PG_UNROLL
        for (int j = 0; j < Q; j++) {
            if (!(ed[j] & kLeaf)) {
                const uint32_t st = trie_stride(ed[j]);
                sd[j] -= st;
                ed[j] = ld[j].u32(trie_child(ed[j]) + ((dst[j] >> sd[j]) & ((1u << st) - 1u)));
            }
            if (PRED) {
                const bool ds = !(es[j] & kLeaf), dk = !(ek[j] & kLeaf);
                const uint32_t ts = ds ? trie_stride(es[j]) : 0u, tk = dk ? trie_stride(ek[j]) : 0u;
                const uint32_t ns = ss[j] - ts, nk = sk[j] - tk;
                const uint32_t is = ds ? trie_child(es[j]) + ((src[j] >> ns) & ((1u << ts) - 1u)) : 0u;
                const uint32_t ik = dk ? trie_child(ek[j]) + ((key[j] >> nk) & ((1u << tk) - 1u)) : 0u;
                const uint32_t vs = ld[j].u32(is), vk = ld[j].u32(ik);
                es[j] = ds ? vs : es[j];
                ek[j] = dk ? vk : ek[j];
                ss[j] = ds ? ns : ss[j];
                sk[j] = dk ? nk : sk[j];
                continue;
            }
            if (!(es[j] & kLeaf)) {
                const uint32_t st = trie_stride(es[j]);
                ss[j] -= st;
                es[j] = ld[j].u32(trie_child(es[j]) + ((src[j] >> ss[j]) & ((1u << st) - 1u)));
            }
            if (!(ek[j] & kLeaf)) {
                const uint32_t st = trie_stride(ek[j]);
                sk[j] -= st;
                ek[j] = ld[j].u32(trie_child(ek[j]) + ((key[j] >> sk[j]) & ((1u << st) - 1u)));
            }
        }
    }
    // cross entry, or the first record of the src class's candidate list (CANDI lanes: set above)
    PG_UNROLL
    for (int j = 0; j < Q; j++) {
        if (!on[j] || ci[j]) continue;
        const uint32_t sc = es[j] & ~kLeaf;
        if (tb[j].fsk & kFlagPair) {  // (src, dst) -> pair class -> x key class -> verdict
            const W2 h = ld[j].u2(kPairHdr + 2u);
            const uint32_t pc = ld[j].u32(h.x + sc * h.y + (ed[j] & ~kLeaf));
            w[j] = ld[j].u32(tb[j].xoff + pc * tb[j].nkc + (ek[j] & ~kLeaf));
        } else if (tb[j].fsk & kFlagCross) {
            const uint32_t idx = sc * tb[j].nkc + (ek[j] & ~kLeaf);
            if (!(tb[j].fsk & kFlagLists)) {
                w[j] = ld[j].u32(tb[j].xoff + idx);
            } else {
                const W2 e = ld[j].u2(tb[j].xoff + 2u * idx);
                w[j] = e.x;
                pos[j] = e.y;  // 0: no dst-specific rule ahead of the verdict
                pend[j] = e.y != 0u;
            }
        } else {
            pos[j] = tb[j].xoff + 4u * sc;
            pend[j] = true;
        }
    }
    // records until the first match (every list ends with a match-all record)
    rec_walk(ld, tb, dst, key, pend, pos, w);
}

template <bool PRED = false, class L, int Q>
PG_HD void blob_walk(const L (&ld)[Q], const BlobTab (&tb)[Q], const bool (&on)[Q], const uint32_t (&src)[Q],
                     const uint32_t (&dst)[Q], const uint32_t (&key)[Q], uint32_t (&w)[Q]) {
    blob_walk<PRED>(ld, ld, tb, on, src, dst, key, w);
}

// FD blob walk (layout: fastpath.cpp build_fd_blob). Tries in the kEncWords encoding
// (non-leaf entry = child WORD offset << 10 | stride << 5 | shift of the child level); a leaf is
// a pointer to a word that points to itself (stride 0), so a finished lookup re-reads that
// word and every lookup takes the same D reads: src -> the self word heading its src class's
// verdict row, key -> the self word of its key class. Verdict = the word at (src self) +
// (key self) + bias, i.e. row[1 + key class]. fsk: s1 << 8 | k1 << 16; kroot: key trie root;
// depth: reads of the src walk | reads of the key walk << 8 (each walk takes its own trie's
// depth: a shallow key trie does not re-read its self words for the src trie's extra levels);
// bias: 1 - (first key self word).
// lp reads the blob's prefix (header, src root, key trie and self words: the LDS copy when a
// launch stages only that), lb everything else (the src levels below the root and the rows).
PG_HD uint32_t fd_child(uint32_t e, uint32_t a) {
#if defined(__HIP_DEVICE_COMPILE__)
    return (e >> 10) + __builtin_amdgcn_ubfe(a, e, e >> 5);
#else
    const uint32_t w = (e >> 5) & 31u;
    return (e >> 10) + ((a >> (e & 31u)) & ((1u << w) - 1u));
#endif
}
// SKIP (the src levels in HBM / L2): a lane whose src entry is already a self word (stride 0)
// does not re-read it -- an exec-masked gather costs the texture path nothing for that lane, and
// large FD tables are bound by that path (profiles/r03_v2_config7_util.json: TA busy 0.93)
#ifndef PG_FD_SPLIT  // each FD walk takes its own trie's depth
#define PG_FD_SPLIT 1
#endif
template <bool SKIP = false, class LP, class LB, int Q>
PG_HD void fd_walk(const LP& lp, const LB& lb, uint32_t fsk, uint32_t kroot, uint32_t depth, uint32_t bias,
                   const uint32_t (&src)[Q], const uint32_t (&key)[Q], uint32_t (&w)[Q]) {
    const uint32_t ss = 32u - ((fsk >> 8) & 0xFFu), sk = 18u - ((fsk >> 16) & 0xFFu);
    uint32_t es[Q], ek[Q];
    PG_UNROLL
    for (int j = 0; j < Q; j++) {
        es[j] = lp.u32(kSrcRoot + (src[j] >> ss));
        ek[j] = lp.u32(kroot + (key[j] >> sk));
    }
#if PG_FD_SPLIT
    const uint32_t ds = depth & 0xFFu, dk = depth >> 8, dmin = ds < dk ? ds : dk;
#else  // A/B build: both walks take the deeper trie's depth
    const uint32_t ds = (depth & 0xFFu) > (depth >> 8) ? depth & 0xFFu : depth >> 8, dk = ds, dmin = ds;
#endif
    for (uint32_t l = 1; l < dmin; l++) {  // both walks in lockstep (independent reads overlap)
        PG_UNROLL
        for (int j = 0; j < Q; j++) {
            if (!SKIP || (es[j] & 0x3E0u)) es[j] = lb.u32(fd_child(es[j], src[j]));
            ek[j] = lp.u32(fd_child(ek[j], key[j]));
        }
    }
    if (ds == dk) {  // (uniform) equal depths, the compiler's default: no further loop control
        PG_UNROLL
        for (int j = 0; j < Q; j++) w[j] = lb.u32((es[j] >> 10) + (ek[j] >> 10) + bias);
        return;
    }
    for (uint32_t l = dmin; l < ds; l++) {
        PG_UNROLL
        for (int j = 0; j < Q; j++)
            if (!SKIP || (es[j] & 0x3E0u)) es[j] = lb.u32(fd_child(es[j], src[j]));
    }
    for (uint32_t l = dmin; l < dk; l++) {
        PG_UNROLL
        for (int j = 0; j < Q; j++) ek[j] = lp.u32(fd_child(ek[j], key[j]));
    }
    PG_UNROLL
    for (int j = 0; j < Q; j++) w[j] = lb.u32((es[j] >> 10) + (ek[j] >> 10) + bias);
}

struct HostLoader {
    const uint32_t* b;
    uint32_t u32(uint32_t i) const { return b[i]; }
    uint32_t at_byte(uint32_t off) const { return b[off >> 2]; }
    W2 u2(uint32_t i) const { return W2{b[i], b[i + 1]}; }
    W4 u4(uint32_t i) const { return W4{b[i], b[i + 1], b[i + 2], b[i + 3]}; }
};

}  // namespace pg
