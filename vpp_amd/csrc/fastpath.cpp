// Builder of the per-table classification blob (the structure the K2 kernel walks).
//
// A table is the compiled first-match rule list of one ACL. The blob answers
// evalACL(table, src, dst, key) for every TCP/UDP/OTHER packet with a bounded number of
// dependent loads, independent of rule depth:
//
//   src  --multibit trie (root stride s1, then 8-bit strides; leaf-pushed)-->  src class
//   key  --multibit trie over the 18-bit L4 key (root stride k1, then 8)----->  key class
//   CROSS mode:  cross[src class][key class] -> verdict of the first rule whose src and L4
//                match and whose dst is ANY, plus (LISTS) the short ordered list of
//                dst-specific rules in front of it, tested on dst only.
//   CAND mode:   (tables too large for a cross product) the src trie's leaf is the first
//                record of the class's ordered candidate list (rules whose src matches),
//                tested on dst + L4 key.
//
// src classes = equivalence classes of the elementary src intervals (cut at every rule's
// prefix boundary) by the ordered list of rules whose src covers them, truncated after the
// first rule that matches every packet reaching it. key classes = equivalence classes of
// the elementary key segments by the set of rules whose key range covers them. The first
// match of the ACL is the first rule of (src list) whose key range covers the key and whose
// dst matches, which is exactly what the cross product precomputes (RFC, Gupta & McKeown,
// SIGCOMM'99, specialised to first-match with a dst residue).
//
// Blob words (u32), all offsets relative to the blob start so it can be read from HBM or
// copied verbatim into LDS:
//   [0]  flags: 1 = CROSS, 2 = LISTS, 4 = CAND, 16 = PAIR, 32 = FD (build_fd_blob), 128 = CANDI
//        (candidates inline in 8-B trie entries below the root; build_fast_table CANDI section)
//   [1]  default verdict (DENY << 30 | table's default slot)
//   [2]  src trie root (always 16)   [3] s1     [4] key trie root   [5] k1
//   [6]  CROSS: cross table (u32 verdicts, or LISTS: u2 {verdict, first record | 0});
//        CAND: first record
//   [7]  n_key_classes   [10] n_src_classes   [8, 9, 11] reserved
//   PAIR (flag 16): [6] pair x key verdicts, [12] dst trie root, [13] d1, [14] (src class x
//        dst class) -> pair class table, [15] n_dst_classes
//   records (16 B, blobwalk.hpp): {dnet, klo | dst prefix length << 18 | last << 24, khi,
//   verdict}; a dst list (LISTS, node lists) ends with a match-all record carrying the
//   fall-through verdict, a candidate list (CAND, CANDI) flags its last record instead (no
//   match there: the table's default deny; an empty list is one match-all record carrying it).
#include <algorithm>
#include <map>
#include <set>
#include <unordered_map>

#include "blobwalk.hpp"
#include "engine.hpp"

namespace pg {

namespace {

struct VecHash {
    size_t operator()(const std::vector<uint32_t>& v) const {
        uint64_t h = 1469598103934665603ull;
        for (uint32_t x : v) {
            h ^= x;
            h *= 1099511628211ull;
        }
        return (size_t)h;
    }
};

// Multibit trie over [0, 2^W): intervals given by sorted starts `bnd` (bnd[0] == 0) and a
// class per interval. Appends blocks to `blob`; returns the root offset, or kTrieFail when
// the blob outgrows the 2^26-word child pointers. A non-leaf entry holds its child's offset
// and stride (blobwalk.hpp trie_child/trie_stride); children take 8-bit strides, or with
// `lc` (level compression, for tries read from HBM) 18 / 16 / 12 bits when their span holds
// at least 8192 / 2048 / 256 interval boundaries: about the memory of the 8-bit levels they
// replace, one or two dependent loads fewer. 18-bit strides only when Tuning::lc_max_stride allows
// (off by default: a 1 MiB child per 2^18 span made config 4's blob 13.8 MB, over the 4 MB
// L2 of an XCD; at 16 it is 6.2 MB and 4 % faster).
constexpr uint32_t kTrieFail = 0xFFFFFFFFu;
// Tuning::lc_dense12: boundaries in a child's span that earn it a 12-bit stride;
// Tuning::lc_max_stride: widest stride level compression may pick (A/B on MI355X, config 4:
// 16 = +4 % over 18, 12 = -3 %)
// HBM-resident blobs: the root alone is staged in LDS, its stride capped by Tuning::lc_root_bits
// (default 12: 16 KiB per workgroup; A/B on MI355X, config 4: 163 Gpps at 12 vs 131 at 14 --
// the 64 KiB root of 14 bits held the launch to half the resident waves)
// enc: kEncBlob (blobwalk.hpp trie_child / trie_stride); kEncNode / kEncNodeA, the node
// image's shifted / aligned encodings (blobwalk.hpp node_child_byte): a non-leaf entry is the
// child's BYTE address << 5 | stride, or (aligned) the BYTE address itself with the child
// placed at an address = its stride mod 32 (strides 8 or 4); the levels below the root take
// uniform strides (the bit offset of a level is a per-level constant), so a step is one
// bit-field extract and one shifted add; kEncWords, the FD blobs' (blobwalk.hpp fd_walk): the
// child's WORD offset << 10 | stride << 5 | shift, children below 16 MiB.
enum TrieEnc { kEncBlob = 0, kEncNode = 1, kEncWords = 2, kEncNodeA = 3 };
constexpr uint32_t kWordsChildMax = 1u << 22;
// cstride: the stride of the levels below the root without level compression (8; FD blobs
// that must fit LDS try 6 and 4: more, smaller levels)
uint32_t build_trie(std::vector<uint32_t>& blob, const std::vector<uint64_t>& bnd, const std::vector<uint32_t>& cls,
                    uint32_t W, uint32_t s1, const Tuning& tu, bool lc = false, int enc = kEncBlob,
                    uint32_t cstride = 8) {
    // interval index containing address a
    auto find = [&](uint64_t a) { return (size_t)(std::upper_bound(bnd.begin(), bnd.end(), a) - bnd.begin()) - 1; };
    struct Job {
        uint32_t block;  // offset of the block in blob
        uint64_t base;   // first address covered by the block
        uint32_t shift;  // address bits below this level
        uint32_t stride;
    };
    std::vector<Job> stack;
    uint32_t root = (uint32_t)blob.size();
    blob.resize(blob.size() + (1u << s1), 0);
    stack.push_back({root, 0, W - s1, s1});
    while (!stack.empty()) {
        Job j = stack.back();
        stack.pop_back();
        uint64_t span = 1ull << j.shift;
        for (uint32_t e = 0; e < (1u << j.stride); e++) {
            uint64_t a = j.base + (uint64_t)e * span;
            if (a >= (1ull << W)) {  // beyond the key space: unreachable, point at class 0
                blob[j.block + e] = kLeaf | cls[0];
                continue;
            }
            size_t k = find(a);
            bool split = k + 1 < bnd.size() && bnd[k + 1] < a + span;
            if (!split || j.shift == 0) {
                blob[j.block + e] = kLeaf | cls[k];
                continue;
            }
            uint32_t st = std::min<uint32_t>(cstride, j.shift);
            if (lc && j.shift >= 12) {
                const size_t inside = (size_t)(std::lower_bound(bnd.begin(), bnd.end(), a + span) - bnd.begin()) - k - 1;
                if (tu.lc_max_stride >= 18 && j.shift >= 18 && inside >= 8192) st = 18;
                else if (tu.lc_max_stride >= 16 && j.shift >= 16 && inside >= 2048) st = 16;
                else if (inside >= tu.lc_dense12) st = 12;
            }
            if (enc == kEncNodeA) {  // the child at a byte address = its stride mod 32 (blobwalk.hpp)
                if (st % 4u) return kTrieFail;
                while ((blob.size() * 4u) % 32u != st % 32u) blob.push_back(0);
            }
            uint32_t child = (uint32_t)blob.size();
            const bool node = enc == kEncNode || enc == kEncNodeA;
            const uint64_t lim = node ? kNodeChildMaxWords : (enc == kEncWords ? kWordsChildMax : kTrieChildMask);
            if ((uint64_t)child + (1ull << st) > lim) return kTrieFail;
            blob.resize(blob.size() + (1u << st), 0);
            blob[j.block + e] = node               ? node_entry(child, st, enc == kEncNodeA)
                                : enc == kEncWords ? (child << 10 | st << 5 | (j.shift - st))
                                                   : child | (st << kTrieStrideShift);
            stack.push_back({child, a, j.shift - st, st});
        }
    }
    return root;
}

// root stride: enough root entries (~4 per interval boundary) that most lookups end at the
// root or one level below, capped by Tuning::root_bits_max (a 2^16-entry root is 256 KiB)
uint32_t pick_stride(size_t nb, uint32_t W, const Tuning& tu) {
    uint32_t s = 4;
    while (s < tu.root_bits_max && s < W && (1ull << s) < 4 * (uint64_t)nb) s += 4;
    return std::min(s, W);
}

bool unconditional(const DevRule& r) { return r.dmask == 0 && r.klo == 0 && r.khi == kKeyMax; }
bool live(const DevRule& r) { return r.klo <= r.khi; }  // can match a TCP/UDP/OTHER packet

constexpr uint32_t kPairMaxRules = 1u << 16;
constexpr uint64_t kPairBudget = 1ull << 22;  // entries of each PAIR phase table (16 MiB)
constexpr size_t kPairListMin = 16;  // CROSS dst lists longer than this: PAIR instead
constexpr uint64_t kNodeCrossBudget = 1ull << 25;  // node cross entries (128 MiB)
constexpr uint64_t kNodeListTabBudget = 1ull << 24;  // node list-verdict entries (64 MiB)

}  // namespace

// The classes of one table, kept for the node classifier (cross-product tables only).
struct TableAnalysis {
    const DevRule* rules = nullptr;
    uint32_t rule_base = 0;
    std::vector<uint64_t> sb;          // src elementary interval starts
    std::vector<uint32_t> sint_cls;    // their src classes
    uint32_t nsc = 0;
    std::vector<uint64_t> kb;          // key segment starts
    std::vector<uint32_t> kseg_cls;    // their key classes
    uint32_t nkc = 0;
    std::vector<uint32_t> cverd;       // [src class][key class] verdict
    std::vector<std::vector<uint32_t>> clist;  // dst-specific rules in front of it
    // PAIR tables (cverd / clist empty): dst intervals and classes, the (src class, dst
    // class) -> pair class map and the pair class x key class verdicts
    bool pair = false;
    std::vector<uint64_t> db;
    std::vector<uint32_t> dint_cls;
    uint32_t ndc = 0, npc = 0;
    std::vector<uint32_t> pmap, xv;
};

void free_analysis(TableAnalysis* an) { delete an; }

bool build_fast_table(const DevRule* rules, uint32_t n, uint32_t rule_base, uint32_t default_slot,
                      std::vector<uint32_t>& blob, uint64_t cross_budget, const Tuning& tu, TableAnalysis** an,
                      bool lc) {
    if (an) *an = nullptr;
    blob.assign(16, 0);
    const uint32_t dflt = (kActDeny << 30) | default_slot;
    blob[1] = dflt;
    auto verdict = [&](uint32_t i) { return ((rules[i].act & 3u) << 30) | (rule_base + i); };
    // records test the dst as a prefix length: every compiled dst mask is a CIDR mask
    auto dlen = [](uint32_t m, uint32_t* len) {
        uint32_t l = (uint32_t)__builtin_popcount(m);
        if (rec_mask(l) != m) return false;
        *len = l;
        return true;
    };
    for (uint32_t i = 0; i < n; i++) {
        uint32_t l = 0;
        if (live(rules[i]) && !dlen(rules[i].dmask, &l)) return false;
    }
    auto put_rec = [&](uint32_t dnet, uint32_t dl, uint32_t klo, uint32_t khi, uint32_t v) {
        blob.push_back(dnet);
        blob.push_back(klo | (dl << 18));
        blob.push_back(khi);
        blob.push_back(v);
    };

    // ---- src: elementary intervals and their candidate lists ------------------------------
    std::vector<uint64_t> sb{0};
    for (uint32_t i = 0; i < n; i++) {
        const DevRule& r = rules[i];
        if (r.smask == 0 || !live(r)) continue;
        sb.push_back(r.snet);
        uint64_t end = (uint64_t)r.snet + (uint64_t)(~r.smask) + 1ull;
        if (end < (1ull << 32)) sb.push_back(end);
    }
    std::sort(sb.begin(), sb.end());
    sb.erase(std::unique(sb.begin(), sb.end()), sb.end());
    std::vector<std::pair<uint64_t, uint32_t>> starts, ends;
    std::set<uint32_t> active;
    for (uint32_t i = 0; i < n; i++) {
        const DevRule& r = rules[i];
        if (!live(r)) continue;
        if (r.smask == 0) {
            active.insert(i);
            continue;
        }
        starts.push_back({r.snet, i});
        uint64_t end = (uint64_t)r.snet + (uint64_t)(~r.smask) + 1ull;
        if (end < (1ull << 32)) ends.push_back({end, i});
    }
    std::sort(starts.begin(), starts.end());
    std::sort(ends.begin(), ends.end());
    std::unordered_map<std::vector<uint32_t>, uint32_t, VecHash> src_cls_of;
    std::vector<std::vector<uint32_t>> src_lists;
    std::vector<uint32_t> sint_cls(sb.size());
    size_t si = 0, ei = 0;
    uint64_t total_cand = 0;
    for (size_t k = 0; k < sb.size(); k++) {
        while (ei < ends.size() && ends[ei].first <= sb[k]) active.erase(ends[ei++].second);
        while (si < starts.size() && starts[si].first <= sb[k]) active.insert(starts[si++].second);
        std::vector<uint32_t> lst;
        for (uint32_t ri : active) {
            lst.push_back(ri);
            if (unconditional(rules[ri])) break;
        }
        auto it = src_cls_of.find(lst);
        if (it == src_cls_of.end()) {
            it = src_cls_of.emplace(lst, (uint32_t)src_lists.size()).first;
            total_cand += lst.size() + 1;
            src_lists.push_back(lst);
            if (total_cand > (1ull << 26)) return false;
        }
        sint_cls[k] = it->second;
    }
    const uint32_t nsc = (uint32_t)src_lists.size();
    blob[10] = nsc;

    // ---- key classes and the cross product, if it fits ---------------------------------------
    bool cross = n <= tu.cross_max_rules && tu.pair != 2;  // pair = 2: PAIR wherever it fits (tests)
    std::vector<uint64_t> kb{0};
    std::vector<uint32_t> kseg_cls;
    std::vector<std::vector<uint32_t>> key_sets;  // sorted rule indices covering the segment
    std::vector<uint32_t> cverd;
    std::vector<std::vector<uint32_t>> clist;
    bool lists = false;
    size_t max_list = 0;
    // key classes: segments x rules covering them; false when that exceeds the work budget
    // (e.g. thousands of all-key rules over many segments), then no cross product / PAIR
    auto compute_keys = [&]() -> bool {
        for (uint32_t i = 0; i < n; i++) {
            if (!live(rules[i])) continue;
            kb.push_back(rules[i].klo);
            if ((uint64_t)rules[i].khi + 1 <= kKeyMax) kb.push_back((uint64_t)rules[i].khi + 1);
        }
        std::sort(kb.begin(), kb.end());
        kb.erase(std::unique(kb.begin(), kb.end()), kb.end());
        std::vector<std::pair<uint64_t, uint32_t>> ks, ke;
        for (uint32_t i = 0; i < n; i++) {
            if (!live(rules[i])) continue;
            ks.push_back({rules[i].klo, i});
            if ((uint64_t)rules[i].khi + 1 <= kKeyMax) ke.push_back({(uint64_t)rules[i].khi + 1, i});
        }
        std::sort(ks.begin(), ks.end());
        std::sort(ke.begin(), ke.end());
        std::set<uint32_t> kact;
        std::unordered_map<std::vector<uint32_t>, uint32_t, VecHash> key_cls_of;
        size_t a = 0, b = 0;
        uint64_t work = 0;
        kseg_cls.resize(kb.size());
        for (size_t k = 0; k < kb.size(); k++) {
            while (b < ke.size() && ke[b].first <= kb[k]) kact.erase(ke[b++].second);
            while (a < ks.size() && ks[a].first <= kb[k]) kact.insert(ks[a++].second);
            if ((work += kact.size()) > (1ull << 28)) {
                key_sets.clear();
                return false;
            }
            std::vector<uint32_t> v(kact.begin(), kact.end());
            auto it = key_cls_of.find(v);
            if (it == key_cls_of.end()) {
                it = key_cls_of.emplace(v, (uint32_t)key_sets.size()).first;
                key_sets.push_back(std::move(v));
            }
            kseg_cls[k] = it->second;
        }
        return true;
    };
    bool keys_ok = true;
    if (cross) {
        keys_ok = compute_keys();
        if (!keys_ok) cross = false;
        if ((uint64_t)nsc * key_sets.size() > cross_budget) cross = false;
    }
    if (cross) {
        // first rule of (src class list) covering the key class; dst-specific rules in front
        // of it form the class pair's dst list
        const uint32_t nkc = (uint32_t)key_sets.size();
        const size_t words = (n + 63) / 64;
        std::vector<uint64_t> kbits((size_t)nkc * words, 0);
        for (uint32_t c = 0; c < nkc; c++)
            for (uint32_t r : key_sets[c]) kbits[(size_t)c * words + r / 64] |= 1ull << (r % 64);
        cverd.assign((size_t)nsc * nkc, dflt);
        clist.assign((size_t)nsc * nkc, {});
        for (uint32_t s = 0; s < nsc && cross; s++) {
            for (uint32_t c = 0; c < nkc; c++) {
                const uint64_t* bits = kbits.data() + (size_t)c * words;
                std::vector<uint32_t>& L = clist[(size_t)s * nkc + c];
                for (uint32_t r : src_lists[s]) {
                    if (!((bits[r / 64] >> (r % 64)) & 1)) continue;
                    if (rules[r].dmask == 0) {
                        cverd[(size_t)s * nkc + c] = verdict(r);
                        break;
                    }
                    L.push_back(r);
                }
                if (L.size() > 255) {  // long dst lists: the candidate form is as good
                    cross = false;
                    break;
                }
                if (!L.empty()) lists = true;
                max_list = std::max<size_t>(max_list, L.size());
            }
        }
    }

    // a failed PAIR attempt may have appended to the blob: back to the bare header
    auto blob_header_only = [&]() {
        blob.resize(16);
        blob[0] = 0;
    };
    // ---- PAIR mode: src class x dst class -> pair class, pair class x key class -> verdict ----
    // For tables whose dst-specific rules are too many for CROSS dst lists (or that exceed
    // its rule bound): the third field gets its own trie and the cross product is taken in
    // two phases (RFC's phase-2 combination): each (src class, dst class) maps to the class
    // of its ordered rule list (the src list filtered by dst, truncated at the first rule
    // matching every key), and that class times the key class to the first rule covering it.
    auto try_pair = [&]() -> bool {
        if (!keys_ok || (key_sets.empty() && !(keys_ok = compute_keys()))) return false;
        const uint32_t nkc = (uint32_t)key_sets.size();
        // dst elementary intervals, classed by the set of dst-specific rules covering them
        std::vector<uint64_t> db{0};
        std::vector<std::pair<uint64_t, uint32_t>> dst_s, dst_e;
        for (uint32_t i = 0; i < n; i++) {
            const DevRule& r = rules[i];
            if (r.dmask == 0 || !live(r)) continue;
            db.push_back(r.dnet);
            dst_s.push_back({r.dnet, i});
            const uint64_t end = (uint64_t)r.dnet + (uint64_t)(~r.dmask) + 1ull;
            if (end < (1ull << 32)) {
                db.push_back(end);
                dst_e.push_back({end, i});
            }
        }
        std::sort(db.begin(), db.end());
        db.erase(std::unique(db.begin(), db.end()), db.end());
        std::sort(dst_s.begin(), dst_s.end());
        std::sort(dst_e.begin(), dst_e.end());
        std::set<uint32_t> dact;
        std::unordered_map<std::vector<uint32_t>, uint32_t, VecHash> dst_cls_of;
        std::vector<std::vector<uint32_t>> dst_sets;
        std::vector<uint32_t> dint_cls(db.size());
        size_t a = 0, b = 0;
        for (size_t k = 0; k < db.size(); k++) {
            while (b < dst_e.size() && dst_e[b].first <= db[k]) dact.erase(dst_e[b++].second);
            while (a < dst_s.size() && dst_s[a].first <= db[k]) dact.insert(dst_s[a++].second);
            std::vector<uint32_t> v(dact.begin(), dact.end());
            auto it = dst_cls_of.find(v);
            if (it == dst_cls_of.end()) {
                it = dst_cls_of.emplace(v, (uint32_t)dst_sets.size()).first;
                dst_sets.push_back(std::move(v));
            }
            dint_cls[k] = it->second;
        }
        const uint32_t ndc = (uint32_t)dst_sets.size();
        const size_t words = (n + 63) / 64;
        uint64_t work = 0;
        for (uint32_t sc = 0; sc < nsc; sc++) work += (uint64_t)src_lists[sc].size() * ndc;
        if ((uint64_t)nsc * ndc <= kPairBudget && (uint64_t)ndc * words <= (1ull << 26) && work <= (1ull << 30)) {
            std::vector<uint64_t> dbits((size_t)ndc * words, 0);
            for (uint32_t d = 0; d < ndc; d++)
                for (uint32_t r : dst_sets[d]) dbits[(size_t)d * words + r / 64] |= 1ull << (r % 64);
            std::vector<uint32_t> pmap((size_t)nsc * ndc);
            std::unordered_map<std::vector<uint32_t>, uint32_t, VecHash> pc_of;
            std::vector<std::vector<uint32_t>> pc_lists;
            std::vector<uint32_t> L;
            for (uint32_t sc = 0; sc < nsc; sc++)
                for (uint32_t d = 0; d < ndc; d++) {
                    const uint64_t* bits = dbits.data() + (size_t)d * words;
                    L.clear();
                    for (uint32_t r : src_lists[sc]) {
                        if (rules[r].dmask != 0 && !((bits[r / 64] >> (r % 64)) & 1)) continue;
                        L.push_back(r);
                        if (rules[r].klo == 0 && rules[r].khi == kKeyMax) break;  // every key matches
                    }
                    auto it = pc_of.find(L);
                    if (it == pc_of.end()) {
                        it = pc_of.emplace(L, (uint32_t)pc_lists.size()).first;
                        pc_lists.push_back(L);
                    }
                    pmap[(size_t)sc * ndc + d] = it->second;
                }
            const uint32_t npc = (uint32_t)pc_lists.size();
            if ((uint64_t)npc * nkc <= kPairBudget) {
                std::vector<uint64_t> kbits((size_t)nkc * words, 0);
                for (uint32_t c = 0; c < nkc; c++)
                    for (uint32_t r : key_sets[c]) kbits[(size_t)c * words + r / 64] |= 1ull << (r % 64);
                std::vector<uint32_t> xv((size_t)npc * nkc, dflt);
                for (uint32_t p = 0; p < npc; p++)
                    for (uint32_t c = 0; c < nkc; c++) {
                        const uint64_t* bits = kbits.data() + (size_t)c * words;
                        for (uint32_t r : pc_lists[p])
                            if ((bits[r / 64] >> (r % 64)) & 1) {
                                xv[(size_t)p * nkc + c] = verdict(r);
                                break;
                            }
                    }
                const uint32_t s1 = std::min<uint32_t>(pick_stride(sb.size(), 32, tu), lc ? tu.lc_root_bits : 32u);
                if (build_trie(blob, sb, sint_cls, 32, s1, tu, lc) != kSrcRoot) return false;
                const uint32_t k1 = pick_stride(kb.size(), 18, tu);
                const uint32_t kroot = build_trie(blob, kb, kseg_cls, 18, k1, tu, lc);
                const uint32_t d1 = pick_stride(db.size(), 32, tu);
                const uint32_t droot = kroot == kTrieFail ? kTrieFail : build_trie(blob, db, dint_cls, 32, d1, tu, lc);
                if (droot == kTrieFail) return false;
                while (blob.size() % 4) blob.push_back(0);
                const size_t poff = blob.size();
                blob.insert(blob.end(), pmap.begin(), pmap.end());
                while (blob.size() % 4) blob.push_back(0);
                const size_t xoff = blob.size();
                blob.insert(blob.end(), xv.begin(), xv.end());
                if (blob.size() >= 0x7FFFFFF0u) return false;
                blob[0] = kFlagPair;
                blob[2] = kSrcRoot;
                blob[3] = s1;
                blob[4] = kroot;
                blob[5] = k1;
                blob[6] = (uint32_t)xoff;
                blob[7] = nkc;
                blob[10] = nsc;
                blob[12] = droot;
                blob[13] = d1;
                blob[14] = (uint32_t)poff;
                blob[15] = ndc;
                if (an) {  // the node classifier covers PAIR tables too (build_node)
                    auto* a = new TableAnalysis();
                    a->rules = rules;
                    a->rule_base = rule_base;
                    a->sb = sb;
                    a->sint_cls = sint_cls;
                    a->nsc = nsc;
                    a->kb = kb;
                    a->kseg_cls = kseg_cls;
                    a->nkc = nkc;
                    a->pair = true;
                    a->db = db;
                    a->dint_cls = dint_cls;
                    a->ndc = ndc;
                    a->npc = npc;
                    a->pmap.swap(pmap);
                    a->xv.swap(xv);
                    *an = a;
                }
                return true;
            }
        }
        return false;
    };

    // long dst lists: PAIR's two lookups beat a record scan (unless it does not fit)
    if (cross && lists && max_list > kPairListMin && tu.pair && n <= kPairMaxRules) {
        if (try_pair()) return true;
        blob_header_only();
    }
    if (cross) {
        const uint32_t nkc = (uint32_t)key_sets.size();
        const uint32_t s1 = std::min<uint32_t>(pick_stride(sb.size(), 32, tu), lc ? tu.lc_root_bits : 32u);
        if (build_trie(blob, sb, sint_cls, 32, s1, tu, lc) != kSrcRoot) return false;
        blob[2] = kSrcRoot;
        blob[3] = s1;
        const uint32_t k1 = pick_stride(kb.size(), 18, tu);
        blob[4] = build_trie(blob, kb, kseg_cls, 18, k1, tu, lc);
        if (blob[4] == kTrieFail) return false;
        blob[5] = k1;
        blob[7] = nkc;
        while (blob.size() % 4) blob.push_back(0);
        blob[6] = (uint32_t)blob.size();
        if (an) {
            auto* a = new TableAnalysis();
            a->rules = rules;
            a->rule_base = rule_base;
            a->sb = sb;
            a->sint_cls = sint_cls;
            a->nsc = nsc;
            a->kb = kb;
            a->kseg_cls = kseg_cls;
            a->nkc = nkc;
            a->cverd = cverd;
            if (lists) a->clist = clist;
            *an = a;
        }
        if (!lists) {
            blob[0] = kFlagCross;
            blob.insert(blob.end(), cverd.begin(), cverd.end());
            return true;
        }
        blob[0] = kFlagCross | kFlagLists;
        const size_t xoff = blob.size();
        blob.resize(blob.size() + 2 * cverd.size(), 0);
        while (blob.size() % 4) blob.push_back(0);
        for (size_t e = 0; e < cverd.size(); e++) {
            blob[xoff + 2 * e] = cverd[e];
            const auto& L = clist[e];
            if (L.empty()) continue;
            if (blob.size() >= 0x7FFFFFF0u) return false;
            blob[xoff + 2 * e + 1] = (uint32_t)blob.size();
            for (uint32_t r : L) {
                uint32_t l = 0;
                dlen(rules[r].dmask, &l);
                put_rec(rules[r].dnet, l, 0, kRecKeyAll, verdict(r));  // key already covered by the class
            }
            put_rec(0, 0, 0, kRecKeyAll, cverd[e]);  // fall through to the pair's verdict
        }
        return true;
    }

    if (!cross && tu.pair && n <= kPairMaxRules && try_pair()) return true;
    blob_header_only();

    // ---- CANDI: a candidate table read from HBM whose live rules test no dst ------------------
    // Below the 4-B src root (staged in LDS by the launch) every trie entry is 8 B (blobwalk.hpp
    // candi_walk): an internal entry, a leaf whose src class has at most one candidate carrying
    // that candidate (key range, action, rule) -- or the table's default -- itself, or a leaf
    // pointing at the class's record list (classes of two or more candidates). A lookup then
    // ends with its last trie read instead of a further record gather; on MI355X a gather costs
    // the same for 4 and 16 B, per active lane (tools/gather_probe.hip), so one gather less per
    // tuple is the lever for tables over LDS. Root leaves keep the record form.
    // Window (Tuning::candi_window_bits, blobwalk.hpp candi_walk): right after the root, staged
    // with it, the terminal 8-B entry of every address of one aligned 2^w-address window -- the
    // window where the table's earliest rules sit (a first-match table's leading rules decide
    // the most lookups: the reference's own scan cost is the matched rule's index) -- so a
    // lookup there reads LDS only (an inline candidate) or goes straight to its record list.
    bool cand_dst_free = true;
    for (uint32_t i = 0; i < n; i++) cand_dst_free &= !live(rules[i]) || rules[i].dmask == 0;
    if (lc && tu.candi && cand_dst_free && n < kCandiDefault) {
        std::vector<uint32_t> tmp;  // the 4-B trie (kEncBlob, leaf = kLeaf | src class)
        // the window: score 1 / (r + 1) per rule r whose src prefix fits in a window, summed per
        // aligned window; the best one (the lower address on a tie)
        uint32_t wbase = 0, wsize = 0;
        const uint32_t wb = tu.candi_window_bits;
        if (wb) {
            std::map<uint32_t, double> score;
            for (uint32_t r = 0; r < n && r < (1u << 16); r++) {
                const DevRule& R = rules[r];
                if (!live(R) || (uint32_t)__builtin_popcount(R.smask) < 32u - wb) continue;
                score[R.snet & ~((1u << wb) - 1u)] += 1.0 / (r + 1.0);
            }
            double best = 0;
            for (const auto& kv : score)
                if (kv.second > best) best = kv.second, wbase = kv.first, wsize = 1u << wb;
        }
        // with a window the root takes at most candi_window_root_bits (12): header + root + a 2^11
        // window = 32 KiB, so four 512-thread workgroups still fit a CU's LDS (A/B on MI355X,
        // config 4: 13-bit root without a window 190 Gpps, with a 2^10 window (three per CU) 176,
        // 12-bit root + 2^11 window 194); the window is left out when it does not stage with the root
        const uint32_t s1 = std::min<uint32_t>(std::min<uint32_t>(pick_stride(sb.size(), 32, tu), tu.lc_root_bits),
                                               wsize ? tu.candi_window_root_bits : 32u);
        if (wsize && candi_window_off(s1) + 2ull * wsize > tu.stage_root_max_words) wbase = wsize = 0;
        if (build_trie(tmp, sb, sint_cls, 32, s1, tu, lc) == 0) {
            std::vector<int64_t> rec_of(nsc, -1);  // record list index of a class (root leaves, pointers)
            std::vector<uint32_t> rec_cls;
            auto rec = [&](uint32_t c) {
                if (rec_of[c] < 0) rec_of[c] = (int64_t)rec_cls.size(), rec_cls.push_back(c);
                return (uint32_t)rec_of[c];
            };
            // blocks: (old offset, stride) -> new word offset; breadth-first from the root
            blob.resize(wsize ? candi_window_off(s1) + 2u * wsize : kSrcRoot + (1u << s1), 0);
            struct Blk {
                uint32_t old_off, stride, new_off;
            };
            std::vector<Blk> q{{0, s1, kSrcRoot}};
            bool ok = true;
            std::vector<uint32_t> rec_at;  // record index per referenced class, assigned below
            for (size_t qi = 0; qi < q.size() && ok; qi++) {
                const Blk b = q[qi];
                for (uint32_t e = 0; e < (1u << b.stride) && ok; e++) {
                    const uint32_t x = tmp[b.old_off + e];
                    uint32_t w0 = 0, w1 = 0;
                    if (!(x & kLeaf)) {  // internal: allocate the child's 8-B block
                        const uint32_t st = trie_stride(x);
                        const uint64_t child = blob.size();
                        if (child + (2ull << st) > kTrieChildMask) {
                            ok = false;
                            break;
                        }
                        blob.resize(blob.size() + (2u << st), 0);
                        q.push_back({trie_child(x), st, (uint32_t)child});
                        w0 = (uint32_t)child;
                        w1 = kCandiNode | kCandiInternal | st;
                        if (qi == 0) {  // root entries stay 4 B
                            blob[b.new_off + e] = (uint32_t)child | (st << kTrieStrideShift);
                            continue;
                        }
                    } else {
                        const uint32_t c = x & ~kLeaf;
                        const std::vector<uint32_t>& L = src_lists[c];
                        if (qi == 0) {
                            blob[b.new_off + e] = kLeaf | rec(c);
                            continue;
                        }
                        if (L.size() >= 2) {
                            w0 = rec(c);
                            w1 = kCandiNode;
                        } else if (L.empty()) {
                            w0 = 0 | (kRecKeyAll & 0x3FFFu) << 18;
                            w1 = (kRecKeyAll >> 14) | kCandiDefault << 6;
                        } else {
                            const DevRule& R = rules[L[0]];
                            w0 = R.klo | (R.khi & 0x3FFFu) << 18;
                            w1 = (R.khi >> 14) | (R.act & 3u) << 4 | L[0] << 6;
                        }
                    }
                    blob[b.new_off + 2 * e] = w0;
                    blob[b.new_off + 2 * e + 1] = w1;
                }
            }
            // window entries: the address's src class (its elementary interval) -> its terminal
            // entry (never internal), list numbers like the leaves' (turned into records below)
            const uint32_t w0ff = candi_window_off(s1);
            for (uint32_t d = 0; ok && d < wsize; d++) {
                const uint64_t a = (uint64_t)wbase + d;
                const size_t k = (size_t)(std::upper_bound(sb.begin(), sb.end(), a) - sb.begin()) - 1;
                const uint32_t c = sint_cls[k];
                const std::vector<uint32_t>& L = src_lists[c];
                uint32_t w0, w1;
                if (L.size() >= 2) {
                    w0 = rec(c);
                    w1 = kCandiNode;
                } else if (L.empty()) {
                    w0 = 0 | (kRecKeyAll & 0x3FFFu) << 18;
                    w1 = (kRecKeyAll >> 14) | kCandiDefault << 6;
                } else {
                    const DevRule& R = rules[L[0]];
                    w0 = R.klo | (R.khi & 0x3FFFu) << 18;
                    w1 = (R.khi >> 14) | (R.act & 3u) << 4 | L[0] << 6;
                }
                blob[w0ff + 2 * d] = w0;
                blob[w0ff + 2 * d + 1] = w1;
            }
            if (ok) {
                blob[0] = kFlagCandI;
                blob[2] = kSrcRoot;
                blob[3] = s1;
                blob[4] = wbase;  // DevTable kroot / nkc: the window's first address and size (0: none)
                blob[7] = wsize;
                while (blob.size() % 4) blob.push_back(0);
                blob[6] = (uint32_t)blob.size();
                // record lists of the referenced classes, in reference order; rec(c) numbered the
                // lists, so list k starts at record first[k]
                std::vector<uint32_t> first(rec_cls.size());
                uint64_t nrec = 0;
                for (size_t k = 0; k < rec_cls.size(); k++) {
                    first[k] = (uint32_t)nrec;
                    nrec += std::max<size_t>(src_lists[rec_cls[k]].size(), 1);
                }
                if (nrec < (1ull << 29)) {
                    // leaves and pointers hold list numbers: turn them into record indices
                    for (uint32_t e = 0; e < (1u << s1); e++)
                        if (blob[kSrcRoot + e] & kLeaf) blob[kSrcRoot + e] = kLeaf | first[blob[kSrcRoot + e] & ~kLeaf];
                    for (size_t qi = 1; qi < q.size(); qi++)
                        for (uint32_t e = 0; e < (1u << q[qi].stride); e++) {
                            uint32_t* v = &blob[q[qi].new_off + 2 * e];
                            if ((v[1] & kCandiNode) && !(v[1] & kCandiInternal)) v[0] = first[v[0]];
                        }
                    for (uint32_t d = 0; d < wsize; d++) {
                        uint32_t* v = &blob[w0ff + 2 * d];
                        if (v[1] & kCandiNode) v[0] = first[v[0]];
                    }
                    for (uint32_t c : rec_cls) {
                        const std::vector<uint32_t>& L = src_lists[c];
                        for (size_t i = 0; i < L.size(); i++) {
                            const uint32_t r = L[i];
                            put_rec(0, i + 1 == L.size() ? kRecLast >> 18 : 0u, rules[r].klo, rules[r].khi, verdict(r));
                        }
                        if (L.empty()) put_rec(0, 0, 0, kRecKeyAll, dflt);
                    }
                    return true;
                }
            }
        }
        blob_header_only();
    }

    // ---- candidate mode: src trie leaves point at the class's record list -------------------
    std::vector<uint32_t> first_rec(nsc);
    uint64_t nrec = 0;
    for (uint32_t s = 0; s < nsc; s++) {
        first_rec[s] = (uint32_t)nrec;
        nrec += std::max<size_t>(src_lists[s].size(), 1);
    }
    if (nrec >= (1ull << 29)) return false;
    std::vector<uint32_t> leaf(sb.size());
    for (size_t k = 0; k < sb.size(); k++) leaf[k] = first_rec[sint_cls[k]];
    const uint32_t s1 = std::min<uint32_t>(pick_stride(sb.size(), 32, tu), lc ? tu.lc_root_bits : 32u);
    if (build_trie(blob, sb, leaf, 32, s1, tu, lc) != kSrcRoot) return false;
    blob[0] = kFlagCand;
    blob[2] = kSrcRoot;
    blob[3] = s1;
    while (blob.size() % 4) blob.push_back(0);  // 16-byte records
    blob[6] = (uint32_t)blob.size();
    for (uint32_t s = 0; s < nsc; s++) {
        const std::vector<uint32_t>& L = src_lists[s];
        for (size_t i = 0; i < L.size(); i++) {
            const uint32_t r = L[i];
            uint32_t l = 0;
            dlen(rules[r].dmask, &l);
            // the last candidate carries kRecLast: no match -> the table's default deny
            put_rec(rules[r].dnet, l | (i + 1 == L.size() ? kRecLast >> 18 : 0u), rules[r].klo, rules[r].khi, verdict(r));
        }
        if (L.empty()) put_rec(0, 0, 0, kRecKeyAll, dflt);  // no candidate: the table's default deny
    }
    return true;
}

// ---- node tries: depth and fixed-depth leaves (kEncNode / kEncNodeA) -------------------------
namespace {
// visits every leaf (kLeaf | class) of a node trie with its level (root = 1)
template <class F>
void node_trie_leaves(const std::vector<uint32_t>& b, uint32_t root, uint32_t s1, bool aligned, F&& f) {
    struct J {
        uint32_t at, n, depth;
    };
    std::vector<J> st{{root, 1u << s1, 1}};
    while (!st.empty()) {
        J j = st.back();
        st.pop_back();
        for (uint32_t e = 0; e < j.n; e++) {
            const uint32_t v = b[j.at + e];
            if (v & kLeaf) f(j.at + e, v & ~kLeaf, j.depth);
            else st.push_back({(aligned ? v : v >> 5) / 4u, 1u << (v & 31u), j.depth + 1});
        }
    }
}
uint32_t node_trie_depth(const std::vector<uint32_t>& b, uint32_t root, uint32_t s1, bool aligned) {
    uint32_t d = 1;
    node_trie_leaves(b, root, s1, aligned, [&](uint32_t, uint32_t, uint32_t depth) { d = std::max(d, depth); });
    return d;
}
// leaves (kLeaf | class) -> their class records (class c at rec0 + (c << shift) bytes, the
// address itself or shifted: blobwalk.hpp node_child_byte)
void node_point_leaves(std::vector<uint32_t>& b, uint32_t root, uint32_t s1, bool aligned, uint32_t rec0_bytes,
                       uint32_t shift) {
    std::vector<std::pair<uint32_t, uint32_t>> at;
    node_trie_leaves(b, root, s1, aligned, [&](uint32_t pos, uint32_t c, uint32_t) { at.push_back({pos, c}); });
    for (auto& p : at) b[p.first] = node_entry((rec0_bytes + (p.second << shift)) / 4u, 0u, aligned);
}
}  // namespace

// ---- FD blob: the fixed-depth form of a dst-independent CROSS table --------------------------
// Layout (u32 words; trie entries hold WORD offsets, kEncWords, so a blob is < 16 MiB):
//   [0] kFlagFD  [1] default verdict  [2] src root (16)  [3] s1  [4] key root  [5] k1
//   [6] depths (reads per field, root included): src trie in bits 0-7, key trie in bits 8-15
//       (equal when both walks run in lockstep; blobwalk.hpp fd_walk)  [7] bias = 1 - KSELF
//   [8] n_key_classes
//   [9] stage words (the prefix below)  [10] n_src_classes
//   prefix: header | src root block | key trie (all levels) | KSELF: one self word per key class
//   then:   src trie levels below the root | rows: per src class c {self word, verdict[c][0..nkc-1]}
// A self word at word A holds A << 10 (stride 0: reading "its child" reads itself). Trie leaves
// point at self words: src -> its class's row head, key -> its class's self word. Every lookup
// is exactly its field's depth in reads plus one verdict read at
//   (src self) + 1 + key class = (src self) + (key self) + bias,
// with no per-lane branch (fd_walk). The prefix -- everything a key lookup and the src root
// read touch -- is what a launch stages in LDS when the whole blob does not fit (device.hip
// STAGE 5). Only tables no rule of which tests dst qualify (engine.cpp): the kernel then does
// not read the dst stream.
namespace {
// depth (reads, root included) of a kEncWords trie rooted at word `root` with 2^s1 entries
uint32_t words_trie_depth(const std::vector<uint32_t>& b, uint32_t root, uint32_t s1) {
    uint32_t d = 1;
    struct J {
        uint32_t at, n, depth;
    };
    std::vector<J> st{{root, 1u << s1, 1}};
    while (!st.empty()) {
        J j = st.back();
        st.pop_back();
        d = std::max(d, j.depth);
        for (uint32_t e = 0; e < j.n; e++) {
            const uint32_t v = b[j.at + e];
            if (v & kLeaf) continue;
            st.push_back({v >> 10, 1u << ((v >> 5) & 31u), j.depth + 1});
        }
    }
    return d;
}
// entries of a kEncWords trie: leaves (kLeaf | class) -> self-word pointers (class c: base +
// c * step), child offsets at or above `from` moved by `delta`
void fd_fix_trie(std::vector<uint32_t>& b, uint32_t root, uint32_t s1, uint32_t base, uint32_t step, uint32_t from,
                 uint32_t delta) {
    std::vector<std::pair<uint32_t, uint32_t>> st{{root, 1u << s1}};
    while (!st.empty()) {
        auto j = st.back();
        st.pop_back();
        for (uint32_t e = 0; e < j.second; e++) {
            uint32_t& v = b[j.first + e];
            if (v & kLeaf) {
                v = (base + (v & ~kLeaf) * step) << 10;
                continue;
            }
            const uint32_t child = v >> 10;
            st.push_back({child, 1u << ((v >> 5) & 31u)});  // still at its pre-move offset
            if (child >= from) v += delta << 10;
        }
    }
}
}  // namespace

bool build_fd_blob(const TableAnalysis& A, uint32_t dflt, const Tuning& tu, std::vector<uint32_t>& blob,
                   uint32_t max_words, uint32_t lds_words) {
    if (A.pair || !A.clist.empty() || A.nsc == 0 || A.nkc == 0) return false;  // dst lists: the verdict reads dst
    // trie shapes, fewest levels first: the first whose blob fits LDS (lds_words) is taken;
    // if none does, of those that fit max_words (read from HBM, its prefix staged) the one with
    // the fewest dependent reads, then the smallest
    struct Shape {
        bool lc;
        uint32_t s1max, cstride;
    };
    const Shape shapes[] = {{true, 12, 8}, {false, 12, 8}, {false, 10, 6}, {false, 8, 4}};
    std::vector<uint32_t> best;
    uint64_t best_key = ~0ull;
    for (const Shape& sh : shapes) {
        const bool lc = sh.lc;
        const uint32_t s1 = std::min<uint32_t>(pick_stride(A.sb.size(), 32, tu), sh.s1max);
        const uint32_t k1 = std::min<uint32_t>(pick_stride(A.kb.size(), 18, tu), sh.s1max);
        const uint32_t P = kSrcRoot + (1u << s1);  // end of the src root block
        std::vector<uint32_t> st(kSrcRoot, 0), kt(P, 0);
        if (build_trie(st, A.sb, A.sint_cls, 32, s1, tu, lc, kEncWords, sh.cstride) != kSrcRoot) continue;
        if (build_trie(kt, A.kb, A.kseg_cls, 18, k1, tu, lc, kEncWords, sh.cstride) != P) continue;
        const uint32_t ds = words_trie_depth(st, kSrcRoot, s1), dk = words_trie_depth(kt, P, k1);
        const uint32_t kself = (uint32_t)kt.size();
        const uint32_t K = kself + A.nkc - P;  // key region: trie + self words
        const uint32_t below = (uint32_t)st.size() - P;  // src levels below the root
        const uint32_t row0 = P + K + below, rstep = A.nkc + 1;
        const uint64_t words = (uint64_t)row0 + (uint64_t)A.nsc * rstep;
        if (words > max_words || words >= kWordsChildMax) continue;
        fd_fix_trie(st, kSrcRoot, s1, row0, rstep, P, K);  // src children move up by K
        fd_fix_trie(kt, P, k1, kself, 1, 0, 0);
        blob.assign(words, 0);
        std::copy(st.begin(), st.begin() + P, blob.begin());
        std::copy(kt.begin() + P, kt.end(), blob.begin() + P);
        for (uint32_t k = 0; k < A.nkc; k++) blob[kself + k] = (kself + k) << 10;
        std::copy(st.begin() + P, st.end(), blob.begin() + P + K);
        for (uint32_t c = 0; c < A.nsc; c++) {
            const uint32_t r = row0 + c * rstep;
            blob[r] = r << 10;
            for (uint32_t k = 0; k < A.nkc; k++) blob[r + 1 + k] = A.cverd[(size_t)c * A.nkc + k];
        }
        blob[0] = kFlagFD;
        blob[1] = dflt;
        blob[2] = kSrcRoot;
        blob[3] = s1;
        blob[4] = P;
        blob[5] = k1;
        // reads per walk (fd_walk): each its own trie's depth when that saves 3+ reads (A/B on
        // MI355X: the 10k-rule sweep table, src 7 / key 4 levels, 448 -> 487 Gpps; config 2's
        // table, 4 / 2, 521 -> 510: its loop control costs more than two LDS re-reads of a self
        // word), else both the deeper one's
        const uint32_t dmax = std::max(ds, dk);
        blob[6] = (dmax - std::min(ds, dk) >= 3) ? (ds | dk << 8) : (dmax | dmax << 8);
        blob[7] = 1u - kself;
        blob[8] = A.nkc;
        blob[9] = (P + K + 3u) & ~3u;
        blob[10] = A.nsc;
        if (std::getenv("PG_FD_DEBUG")) {  // measurement aid: where an FD blob's words go
            std::set<std::vector<uint32_t>> rows;
            for (uint32_t c = 0; c < A.nsc; c++)
                rows.insert(std::vector<uint32_t>(A.cverd.begin() + (size_t)c * A.nkc,
                                                  A.cverd.begin() + (size_t)(c + 1) * A.nkc));
            std::fprintf(stderr, "fd: lc %d s1 %u k1 %u depths %u/%u | words: prefix %u, src levels %u, rows %u, total %zu "
                                 "(%u classes, %zu distinct rows, %u key classes)\n",
                         (int)lc, s1, k1, ds, dk, P + K, below, A.nsc * rstep, blob.size(), A.nsc, rows.size(), A.nkc);
        }
        if (blob.size() <= lds_words) return true;
        // read from HBM / L2: the fewest dependent reads, then the smallest blob -- a wider
        // (level-compressed) shape of the same depth only spreads the gathers over more bytes
        // than an XCD's L2 holds (config 7: 6.3 MB level-compressed vs 4.2 MB, both 4 / 3 reads)
        const uint64_t key = (uint64_t)std::max(ds, dk) << 40 | (uint64_t)(ds + dk) << 32 | blob.size();
        if (best.empty() || key < best_key) best.swap(blob), best_key = key;
    }
    if (best.empty()) return false;
    blob.swap(best);
    return true;
}

// ---- node classifier -------------------------------------------------------------------------
// One IPv4 partition for the whole node: cut at every covered table's src interval boundary
// and around every local pod address; elementary intervals with the same end point
// (interface + its tables) and the same src class in every covered table share a node IP
// class. Likewise one L4-key partition, node key class -> each table's key class by `kmap`.
// Then cross[t][ip class][local key class] is table t's cross entry for (its src class of
// that IP class, key class): an evaluation is two LDS trie walks (shared by every table and
// both directions of a connection) and one global load.
// Common-row section of the node image (device.hpp DevNode): per covered table, the cross row
// (over its key classes) shared by the most node IP classes -- typically "no rule admits this
// source": the default deny -- and a bitmap of the (table, IP class) pairs whose row equals it.
// Those evaluations read their entry from the LDS-staged image instead of gathering it from
// the cross table. Appended after the base image; the kernels stage and use it when the LDS
// budget allows (device.hip). Skipped when the bitmap would exceed kCommonMapMaxBits.
constexpr uint64_t kCommonMapMaxBits = 1ull << 20;  // 128 KiB
void build_common_rows(HostTableSet& h, const std::vector<uint32_t>& cov, const std::vector<TableAnalysis*>& an,
                       const Tuning& tu, bool uni) {
    std::vector<uint32_t>& img = h.node_img;
    std::vector<uint32_t>& TI = uni ? h.node_aux : h.node_img;  // tabinfo (build_node)
    DevNode& N = h.node;
    const uint32_t T = (uint32_t)h.tabs.size(), G = N.n_ipc;
    uint32_t rs = 0;  // bitmap row: G bits in 2^rs words
    while ((32ull << rs) < G) rs++;
    const uint64_t bits = (uint64_t)T << (rs + 5);
    if (!tu.node_common || bits > kCommonMapMaxBits) return;
    const std::vector<uint32_t>& X = h.node_cross;
    std::vector<uint32_t> sec, map(uni ? 0 : (size_t)(bits / 32), 0);
    // uniform layout: the marks as one 64-bit mask per IP class (uint2 {tables 0-31, 32-63}), so a
    // connection reads its two classes' masks once instead of one bitmap word per evaluation. Past
    // 64 tables a bit covers a group of 2^gshift consecutive tables (bit t >> gshift): set when the
    // class's row is the common one in every table of the group, so an evaluation whose group bit
    // is clear gathers its entry from the cross table, which holds every row
    // (wide records, DevNode wide: one 32-bit mark word, so T <= 32 << gshift); the uniform
    // layout's "no ACL" pseudo-table tnil (build_node) takes the group after the tables
    const uint32_t mbits = N.wide ? 32u : 64u;
    uint32_t gshift = 0;
    while (uni && (mbits << gshift) < T) gshift++;
    if (uni && !N.wide)
        while ((N.tnil >> gshift) >= mbits) gshift++;
    // (the pseudo-table's group must hold no table: tnil a multiple of 2^gshift, past T)
    if (uni && !N.wide && (N.tnil < T || (N.tnil & ((1u << gshift) - 1u)) != 0)) return;
    N.gshift = gshift;
    std::vector<uint32_t> masks(uni ? 2 * (size_t)G : 0, 0);
    std::vector<uint8_t> grp_common(uni ? (size_t)G * 64 : 0, 1);  // [g][group]: every table common
    std::vector<uint32_t> crow(T, 0);
    for (uint32_t t : cov) {
        const uint32_t base = TI[N.tabinfo + 4 * t], nk = uni ? N.gk : an[t]->nkc;
        // most frequent row: rows hashed, candidates compared word by word
        std::unordered_map<uint64_t, std::pair<uint32_t, uint32_t>> freq;  // hash -> (first ip class, count)
        auto row = [&](uint32_t g) { return X.data() + base + (size_t)g * nk; };
        auto hrow = [&](uint32_t g) {
            uint64_t x = 1469598103934665603ull;
            for (uint32_t k = 0; k < nk; k++) x = (x ^ row(g)[k]) * 1099511628211ull;
            return x;
        };
        uint32_t best = 0, best_n = 0;
        for (uint32_t g = 0; g < G; g++) {
            auto& f = freq.emplace(hrow(g), std::make_pair(g, 0u)).first->second;
            if (!std::equal(row(g), row(g) + nk, row(f.first))) continue;  // hash collision: not counted
            if (++f.second > best_n) best_n = f.second, best = f.first;
        }
        crow[t] = (uint32_t)sec.size();
        sec.insert(sec.end(), row(best), row(best) + nk);
        for (uint32_t g = 0; g < G; g++) {
            const bool same = std::equal(row(g), row(g) + nk, row(best));
            if (uni && !same) grp_common[(size_t)g * 64 + (t >> gshift)] = 0;
            if (!uni && same) map[((size_t)t << rs) + (g >> 5)] |= 1u << (g & 31u);
        }
    }
    if (uni)
        for (uint32_t g = 0; g < G; g++)
            for (uint32_t b = 0; b < mbits && (b << gshift) < T; b++)
                if (grp_common[(size_t)g * 64 + b]) masks[2 * (size_t)g + (b >> 5)] |= 1u << (b & 31u);
    if (uni && !N.wide) {  // rows up to tnil (unused ones zero), then tnil's: PERMIT, the "no ACL" slot
        const uint32_t noacl = (uint32_t)h.rules.size() + T;
        sec.resize((size_t)N.tnil * N.gk, 0u);
        sec.insert(sec.end(), N.gk, (kActPermit << 30) | noacl);
        for (uint32_t g = 0; g < G; g++) {
            const uint32_t b = N.tnil >> gshift;
            masks[2 * (size_t)g + (b >> 5)] |= 1u << (b & 31u);
        }
    }
    while (sec.size() % 4) sec.push_back(0);
    const uint32_t s0 = (uint32_t)img.size();
    for (uint32_t t : cov) TI[N.tabinfo + 4 * t + 2] = s0 + crow[t];
    img.insert(img.end(), sec.begin(), sec.end());
    if (uni) {  // the masks live in the class records (words 2-3; wide records: word 2, word 3 holds
                // the end point's tables): class g's at word cmap + (g << 2)
        N.cmap = N.ipinfo + 2u;
        N.cmap_shift = 2u;
        for (uint32_t g = 0; g < G; g++) {
            img[N.cmap + 4 * (size_t)g] = masks[2 * (size_t)g];
            if (!N.wide) img[N.cmap + 4 * (size_t)g + 1] = masks[2 * (size_t)g + 1];
        }
    } else {
        N.cmap = (uint32_t)img.size();
        N.cmap_shift = rs;
        img.insert(img.end(), map.begin(), map.end());
    }
    while (img.size() % 4) img.push_back(0);
    N.img_words = (uint32_t)img.size();
}

bool build_node(HostTableSet& h, const std::vector<TableAnalysis*>& an, const std::vector<NodePod>& pods,
                const NodePod& node_end, const Tuning& tu) {
    h.node_img.clear();
    h.node_aux.clear();
    h.node_cross.clear();
    h.node = DevNode{};
    h.node_rec_words = 0;
    const uint32_t T = (uint32_t)h.tabs.size();
    if (!tu.node_build || T == 0 || T >= 0xFFFFu) return false;
    std::vector<uint32_t> cov;
    for (uint32_t t = 0; t < T; t++)
        if (an[t] && an[t]->nkc <= 0xFFFFu && (!an[t]->pair || (an[t]->nsc <= 0xFFFFu && an[t]->ndc <= 0xFFFFu)))
            cov.push_back(t);
    if (cov.empty()) return false;
    // PAIR tables among them: the IPv4 partition also separates their dst classes
    std::vector<size_t> pcov;  // indices into cov
    for (size_t c = 0; c < cov.size(); c++)
        if (an[cov[c]]->pair) pcov.push_back(c);
    // List tables (cross-product tables with dst-specific rules in front of some verdicts,
    // clist): with Tuning::node_list_table (uniform layout) the IPv4 partition also separates every address
    // range those rules' dst prefixes tell apart (the class key holds, per list table, which of
    // them contain the class), so a list resolves by the rule-dst-side address's class alone: one
    // entry of a list-verdict table [list][node IP class] instead of a walk over its records
    std::vector<size_t> lcov;  // indices into cov
    std::vector<std::vector<uint64_t>> lb;   // per list table: its dst interval starts
    std::vector<std::vector<uint32_t>> lcl;  // ... and their classes (set of containing prefixes)
    if (tu.node_list_table && tu.node_uniform && cov.size() == T && pcov.empty())
        for (size_t c = 0; c < cov.size(); c++) {
            const TableAnalysis& A = *an[cov[c]];
            if (A.pair) continue;
            std::vector<uint32_t> lr;  // the table's list rules
            for (const auto& l : A.clist) lr.insert(lr.end(), l.begin(), l.end());
            if (lr.empty()) continue;
            std::sort(lr.begin(), lr.end());
            lr.erase(std::unique(lr.begin(), lr.end()), lr.end());
            std::vector<uint64_t> b{0};
            for (uint32_t r : lr) {
                const DevRule& R = A.rules[r];
                b.push_back(R.dnet & R.dmask);
                b.push_back((uint64_t)(R.dnet & R.dmask) + (uint64_t)(~R.dmask) + 1u);
            }
            std::sort(b.begin(), b.end());
            b.erase(std::unique(b.begin(), b.end()), b.end());
            while (!b.empty() && b.back() >= (1ull << 32)) b.pop_back();
            std::map<std::vector<uint32_t>, uint32_t> ids;
            std::vector<uint32_t> cl(b.size());
            std::vector<uint32_t> in;
            for (size_t k = 0; k < b.size(); k++) {
                in.clear();
                for (uint32_t r : lr)
                    if (((uint32_t)b[k] & A.rules[r].dmask) == (A.rules[r].dnet & A.rules[r].dmask)) in.push_back(r);
                cl[k] = ids.emplace(in, (uint32_t)ids.size()).first->second;
            }
            lcov.push_back(c);
            lb.push_back(std::move(b));
            lcl.push_back(std::move(cl));
        }

    // IPv4 partition
    std::vector<uint64_t> gb{0};
    for (uint32_t t : cov) gb.insert(gb.end(), an[t]->sb.begin(), an[t]->sb.end());
    for (size_t c : pcov) gb.insert(gb.end(), an[cov[c]]->db.begin(), an[cov[c]]->db.end());
    for (const auto& b : lb) gb.insert(gb.end(), b.begin(), b.end());
    if ((uint64_t)h.rules.size() + T + 2 >= kNodeList) return false;  // verdict slots below the list flag
    std::map<uint32_t, NodePod> by_ip;  // a repeated address: the last pod wins, as in the iphash
    for (const NodePod& p : pods) by_ip[p.ip] = p;
    std::vector<NodePod> ps;
    for (auto& kv : by_ip) ps.push_back(kv.second);
    for (const NodePod& p : ps) {
        gb.push_back(p.ip);
        if ((uint64_t)p.ip + 1 < (1ull << 32)) gb.push_back((uint64_t)p.ip + 1);
    }
    std::sort(gb.begin(), gb.end());
    gb.erase(std::unique(gb.begin(), gb.end()), gb.end());
    const size_t C = cov.size();
    const size_t PC = pcov.size();
    const size_t LC = lcov.size();
    std::vector<size_t> at(C, 0), atd(PC, 0), atl(LC, 0);
    std::unordered_map<std::vector<uint32_t>, uint32_t, VecHash> ipc_of;
    // class -> {ifc, tin, tout, src class per covered table..., dst class per PAIR table...,
    // list-dst class per list table...}
    std::vector<std::vector<uint32_t>> ipc_key;
    std::vector<uint32_t> ipc_rep;  // per class: an address in it (list verdicts)
    std::vector<uint32_t> gcls(gb.size());
    size_t pi = 0;
    std::vector<uint32_t> key(3 + C + PC + LC);
    for (size_t k = 0; k < gb.size(); k++) {
        const uint64_t a = gb[k];
        while (pi < ps.size() && ps[pi].ip < a) pi++;
        const NodePod& e = (pi < ps.size() && ps[pi].ip == a) ? ps[pi] : node_end;
        key[0] = (uint32_t)e.ifc, key[1] = (uint32_t)e.tin, key[2] = (uint32_t)e.tout;
        for (size_t c = 0; c < C; c++) {
            const TableAnalysis& A = *an[cov[c]];
            while (at[c] + 1 < A.sb.size() && A.sb[at[c] + 1] <= a) at[c]++;
            key[3 + c] = A.sint_cls[at[c]];
        }
        for (size_t q = 0; q < PC; q++) {
            const TableAnalysis& A = *an[cov[pcov[q]]];
            while (atd[q] + 1 < A.db.size() && A.db[atd[q] + 1] <= a) atd[q]++;
            key[3 + C + q] = A.dint_cls[atd[q]];
        }
        for (size_t q = 0; q < LC; q++) {
            while (atl[q] + 1 < lb[q].size() && lb[q][atl[q] + 1] <= a) atl[q]++;
            key[3 + C + PC + q] = lcl[q][atl[q]];
        }
        auto it = ipc_of.find(key);
        if (it == ipc_of.end()) {
            it = ipc_of.emplace(key, (uint32_t)ipc_key.size()).first;
            ipc_key.push_back(key);
            ipc_rep.push_back((uint32_t)a);
        }
        gcls[k] = it->second;
    }
    uint32_t G = (uint32_t)ipc_key.size();
    uint64_t entries = 0;
    for (uint32_t t : cov)
        entries += an[t]->pair ? (uint64_t)an[t]->nsc * an[t]->ndc + (uint64_t)an[t]->npc * an[t]->nkc
                               : (uint64_t)G * an[t]->nkc;
    if (entries > kNodeCrossBudget) return false;

    // L4-key partition
    std::vector<uint64_t> kb{0};
    for (uint32_t t : cov) kb.insert(kb.end(), an[t]->kb.begin(), an[t]->kb.end());
    std::sort(kb.begin(), kb.end());
    kb.erase(std::unique(kb.begin(), kb.end()), kb.end());
    std::fill(at.begin(), at.end(), 0);
    std::unordered_map<std::vector<uint32_t>, uint32_t, VecHash> kc_of;
    std::vector<std::vector<uint32_t>> kc_key;
    std::vector<uint32_t> kcls(kb.size());
    std::vector<uint32_t> kk(C);
    for (size_t k = 0; k < kb.size(); k++) {
        for (size_t c = 0; c < C; c++) {
            const TableAnalysis& A = *an[cov[c]];
            while (at[c] + 1 < A.kb.size() && A.kb[at[c] + 1] <= kb[k]) at[c]++;
            kk[c] = A.kseg_cls[at[c]];
        }
        auto it = kc_of.find(kk);
        if (it == kc_of.end()) {
            it = kc_of.emplace(kk, (uint32_t)kc_key.size()).first;
            kc_key.push_back(kk);
        }
        kcls[k] = it->second;
    }
    const uint32_t GK = (uint32_t)kc_key.size();
    // image: IPv4 trie (root at word 0), key trie, class records, tabinfo, kmap
    std::vector<uint32_t>& img = h.node_img;
    DevNode& N = h.node;
    // end points pack into the class record (classify.hpp node_end_packed): interface indices
    // below 2^14; fewer than 255 tables in one word with the interface, else (wide records,
    // DevNode wide) 16-bit table ids in a word of their own, beside 32-bit common-row marks
    bool pack_ok = true;
    for (const auto& k : ipc_key)
        if ((int32_t)k[0] >= 0 && (k[0] & ~(3u << kEndKindShift)) >= 0x4000u) pack_ok = false;
    // "no ACL" is a pseudo-table id tnil: the first id of a group of common-row marks past the
    // tables (T rounded up to 2^gshift), whose common row holds PERMIT with the "no ACL" slot in
    // every column and whose mark is set in every class (build_common_rows), so an evaluation of
    // it reads that row like any common row -- no test of the id in the kernels that stage the
    // section (classify.hpp uni_eval). Narrow records need tnil below 255.
    auto gshift_for = [](uint32_t tabs, uint32_t mbits) {
        uint32_t g = 0;
        while (((((tabs + (1u << g) - 1u) >> g) << g) >> g) >= mbits) g++;  // tnil's group index < mbits
        return g;
    };
    // Wide records keep 0xFFFF for "no ACL", tested in their kernels (their 32-bit marks have no
    // group to spare).
    const uint32_t gs_nil = gshift_for(T, 64);
    const uint32_t tnil_narrow = ((T + (1u << gs_nil) - 1u) >> gs_nil) << gs_nil;
    const bool wide = tnil_narrow >= 255;  // (build_node: T < 0xFFFF)
    const uint32_t tnil = wide ? 0xFFFFu : tnil_narrow;
    // uniform layout (DevNode uniform): every table covered, none in PAIR form -- rows over the
    // node key classes at cross[(t * G + ip class) * GK + key class], so an evaluation computes
    // its entry's address from (t, classes) instead of reading tabinfo and kmap (at most 64
    // tables: the common-row marks are then one 64-bit mask per IP class). Its tries take the
    // aligned encoding (blobwalk.hpp: one VALU less per step, strides of 8 and 4 only); other
    // node sets the shifted one, whose strides are free (config 6: a 4-KiB smaller image keeps
    // three workgroups per CU)
    // (and it resolves lists by the list-verdict table: its kernels carry no record walk)
    bool has_lists = false;
    for (uint32_t t : cov)
        for (const auto& l : an[t]->clist) has_lists |= !l.empty();
    // (more than 64 tables: the common-row marks cover groups of 2^gshift tables, DevNode gshift)
    const bool aligned = tu.node_uniform && C == T && PC == 0 && pack_ok && (tu.node_list_table || !has_lists);
    const int enc = aligned ? kEncNodeA : kEncNode;
    // IPv4 trie root: the smallest trie among the root strides that give the fewest levels (a
    // walk reads exactly depth words; a smaller image leaves LDS for the counter histogram --
    // config 5: 12 -> 10 bits keeps image + histogram within two workgroups per CU); aligned:
    // strides of 8 and 4 below the root, so 32 - root is a multiple of 4
    {
        const uint32_t top = std::min(pick_stride(gb.size(), 32, tu), tu.node_root_bits);
        uint32_t best_d = ~0u;
        std::vector<uint32_t> tmp;
        for (uint32_t s1 = aligned ? top - top % 4u : top; s1 >= 4 && (aligned || s1 + 4 > top); s1 -= aligned ? 4 : 1) {
            tmp.clear();
            if (build_trie(tmp, gb, gcls, 32, s1, tu, false, enc, kNodeStride) != 0) return false;
            const uint32_t d = node_trie_depth(tmp, 0, s1, aligned);
            if (d < best_d || (d == best_d && tmp.size() < img.size())) {
                best_d = d;
                N.ip_s1 = s1;
                img.swap(tmp);
            }
        }
        if (best_d == ~0u) return false;
    }
    N.ip_depth = node_trie_depth(img, 0, N.ip_s1, aligned);
    // class records (blobwalk.hpp node_ip_rec_shift): uniform 16 B (IPv4) / 32 B (key), else
    // 4-B self words
    const uint32_t rshift = aligned ? node_ip_rec_shift<true>() : node_ip_rec_shift<false>();
    const uint32_t kshift = aligned ? node_key_rec_shift<true>() : node_key_rec_shift<false>();
    if (aligned) {
        // a class with a leaf above the last level needs its record on a 32-byte boundary (a
        // finished lookup re-reads it at stride 0), so those classes take every other record
        // slot; the rest fill the others (slots past the classes: never reached)
        const uint32_t align = 32u >> rshift;
        std::vector<uint8_t> early(G, 0);
        node_trie_leaves(img, 0, N.ip_s1, true, [&](uint32_t, uint32_t c, uint32_t d) {
            if (d < N.ip_depth) early[c] = 1;
        });
        uint32_t ne = 0;
        for (uint32_t g = 0; g < G; g++) ne += early[g];
        const uint32_t S = std::max<uint32_t>(G, ne ? (ne - 1) * align + 1 : 0);
        std::vector<uint32_t> slot(G);
        std::vector<uint8_t> used(S, 0);
        uint32_t k = 0, nx = 0;
        for (uint32_t g = 0; g < G; g++)
            if (early[g]) slot[g] = align * k++, used[slot[g]] = 1;
        for (uint32_t g = 0; g < G; g++) {
            if (early[g]) continue;
            while (used[nx]) nx++;
            slot[g] = nx, used[nx] = 1;
        }
        std::vector<std::vector<uint32_t>> rk(S, ipc_key[0]);
        std::vector<uint32_t> rr(S, ipc_rep[0]);
        for (uint32_t g = 0; g < G; g++) rk[slot[g]] = ipc_key[g], rr[slot[g]] = ipc_rep[g];
        ipc_key.swap(rk);
        ipc_rep.swap(rr);
        std::vector<std::pair<uint32_t, uint32_t>> lv;
        node_trie_leaves(img, 0, N.ip_s1, true, [&](uint32_t pos, uint32_t c, uint32_t) { lv.push_back({pos, c}); });
        for (auto& x : lv) img[x.first] = kLeaf | slot[x.second];
        if (std::getenv("PG_NODE_DEBUG"))  // measurement aid: record slots
            std::fprintf(stderr, "node: %u classes, %u with a leaf above the last level, %u record slots\n", G, ne, S);
        G = S;
    }
    entries = 0;
    for (uint32_t t : cov)
        entries += an[t]->pair ? (uint64_t)an[t]->nsc * an[t]->ndc + (uint64_t)an[t]->npc * an[t]->nkc
                               : (uint64_t)G * an[t]->nkc;
    if (entries > kNodeCrossBudget) return false;
    const bool uni = aligned && (uint64_t)T * G < (1u << 24) && (uint64_t)T * G * GK <= kNodeCrossBudget &&
                     (uint64_t)G * GK < (1u << 24);  // (24-bit products: classify.hpp mad24)
    if (aligned && !uni) {  // (the aligned tries are the uniform layout's): the other layout
        Tuning t2 = tu;
        t2.node_uniform = 0;
        return build_node(h, an, pods, node_end, t2);
    }
    if (uni) entries = (uint64_t)T * G * GK;
    // L4-key trie: aligned, the root stride (18 - root a multiple of 4, at most
    // Tuning::node_key_root_bits) with the fewest levels, then the smallest trie
    if (aligned) {
        const size_t k0 = img.size();
        std::vector<uint32_t> best;
        uint32_t best_d = ~0u;
        for (uint32_t k1 = 2; k1 <= std::min(tu.node_root_bits, tu.node_key_root_bits); k1 += 4) {
            img.resize(k0);
            const uint32_t root = build_trie(img, kb, kcls, 18, k1, tu, false, enc, kNodeStride);
            if (root == kTrieFail) continue;
            const uint32_t d = node_trie_depth(img, root, k1, true);
            if (d < best_d || (d == best_d && img.size() < k0 + best.size())) {
                best_d = d;
                N.key_k1 = k1;
                N.key_root = root;
                best.assign(img.begin() + k0, img.end());
            }
        }
        if (best_d == ~0u) return false;
        img.resize(k0);
        img.insert(img.end(), best.begin(), best.end());
    } else {
        N.key_k1 = std::min(pick_stride(kb.size(), 18, tu), tu.node_root_bits);
        N.key_root = build_trie(img, kb, kcls, 18, N.key_k1, tu, false, enc, kNodeStride);
        if (N.key_root == kTrieFail) return false;
    }
    N.key_depth = node_trie_depth(img, N.key_root, N.key_k1, aligned);
    // records: uniform IPv4 classes {self, packed end point, common-row mask lo, hi} (16 B), key
    // classes {self} (32 B); otherwise 4-B self words and ipinfo {interface, tin | tout << 16}
    // per class; self = the leaf value pointing at the record (blobwalk.hpp)
    const uint32_t rw = (1u << rshift) / 4u, kw = (1u << kshift) / 4u;  // record words
    while (img.size() % 8) img.push_back(0);
    const uint32_t irec0 = (uint32_t)img.size();
    img.resize(img.size() + rw * (size_t)G, 0);
    while (img.size() % 8) img.push_back(0);
    const uint32_t krec0 = (uint32_t)img.size();
    img.resize(img.size() + kw * (size_t)GK, 0);
    if ((uint64_t)img.size() * 4 >= kNodeChildMaxWords * 4ull) return false;
    node_point_leaves(img, 0, N.ip_s1, aligned, irec0 * 4u, rshift);
    node_point_leaves(img, N.key_root, N.key_k1, aligned, krec0 * 4u, kshift);
    for (uint32_t g = 0; g < G; g++) {
        const auto& k = ipc_key[g];
        uint32_t* r = img.data() + irec0 + rw * (size_t)g;
        r[0] = node_entry(irec0 + rw * g, 0u, aligned);
        if (aligned) {
            auto t8 = [&](uint32_t t) { return (int32_t)t < 0 ? tnil : t; };
            auto t16 = [&](uint32_t t) { return (int32_t)t < 0 ? tnil : t; };
            const uint32_t f = (int32_t)k[0] < 0 ? 0xFFFFu : ((k[0] & 0x3FFFu) | ((k[0] >> kEndKindShift) & 3u) << 14);
            if (wide) {
                r[1] = f;
                r[3] = t16(k[1]) | t16(k[2]) << 16;
            } else {
                r[1] = f | t8(k[1]) << 16 | t8(k[2]) << 24;
            }
        }
    }
    for (uint32_t k = 0; k < GK; k++) img[krec0 + kw * k] = node_entry(krec0 + kw * k, 0u, aligned);
    N.ipself = irec0 * 4u >> rshift;  // class = (record byte address >> record shift) - ipself
    N.kself = krec0 * 4u >> kshift;
    N.ipinfo = irec0;
    if (!aligned) {
        while (img.size() % 2) img.push_back(0);
        N.ipinfo = (uint32_t)img.size();
        auto t16 = [](uint32_t t) { return (int32_t)t < 0 ? 0xFFFFu : t; };
        for (uint32_t g = 0; g < G; g++) {
            img.push_back(ipc_key[g][0]);
            img.push_back(t16(ipc_key[g][1]) | (t16(ipc_key[g][2]) << 16));
        }
        while (img.size() % 4) img.push_back(0);
    }
    // (the uniform layout's kernels never read tabinfo and kmap: the builder keeps them off the
    // image, in h.node_aux)
    std::vector<uint32_t>& TI = uni ? h.node_aux : img;
    N.tabinfo = (uint32_t)TI.size();
    TI.resize(TI.size() + 4 * (size_t)T, 0);
    N.gk_shift = 0;
    while ((1u << N.gk_shift) < GK) N.gk_shift++;
    N.kmap = (uint32_t)TI.size();
    TI.resize(TI.size() + (((size_t)T << N.gk_shift) + 1) / 2, 0);
    while (img.size() % 4) img.push_back(0);
    // PAIR tables: per node IP class, the table's src class | dst class << 16
    std::vector<uint32_t> pmap_off(PC);
    for (size_t q = 0; q < PC; q++) {
        pmap_off[q] = (uint32_t)img.size();
        for (uint32_t g = 0; g < G; g++) img.push_back(ipc_key[g][3 + pcov[q]] | (ipc_key[g][3 + C + q] << 16));
    }
    while (img.size() % 4) img.push_back(0);
    if (img.size() >= 0xFFFFu) return false;  // map offsets are 16-bit (tabinfo.w)
    N.gk = GK;
    N.n_ipc = G;
    N.n_pair = (uint32_t)PC;
    N.wide = aligned && wide;
    N.tnil = aligned ? tnil : 0xFFFFFFFFu;
    N.img_words = N.img_words_base = (uint32_t)img.size();
    N.cmap = 0;

    // cross entries, then the dst records of the pairs with a list (or the list-verdict table)
    std::vector<uint32_t>& X = h.node_cross;
    X.reserve(entries + 16);
    std::vector<uint32_t> recs;
    const size_t rec0 = (entries + 3) & ~(uint64_t)3;
    // the list-verdict table is the uniform layout's list form; the others keep the records
    const bool ltab = uni && tu.node_list_table != 0;  // (every list table is in lcov then)
    struct ListRef {
        size_t c, e;  // the list of (covered table cov[c], src class x key class e)
    };
    std::vector<ListRef> lists;
    size_t q = 0;
    for (size_t c = 0; c < C; c++) {
        const uint32_t t = cov[c];
        const TableAnalysis& A = *an[t];
        TI[N.tabinfo + 4 * t] = (uint32_t)X.size();
        TI[N.tabinfo + 4 * t + 1] = A.nkc | 0x80000000u;
        for (uint32_t g = 0; g < GK; g++) {
            const uint32_t ki = (t << N.gk_shift) + g;
            TI[N.kmap + ki / 2] |= kc_key[g][c] << ((ki & 1u) * 16u);
        }
        if (A.pair) {  // {pair map base, nkc | covered | PAIR, verdicts base, class map | ndc << 16}
            TI[N.tabinfo + 4 * t + 1] |= kNodePairFlag;
            X.insert(X.end(), A.pmap.begin(), A.pmap.end());
            TI[N.tabinfo + 4 * t + 2] = (uint32_t)X.size();
            X.insert(X.end(), A.xv.begin(), A.xv.end());
            TI[N.tabinfo + 4 * t + 3] = pmap_off[q++] | (A.ndc << 16);
            continue;
        }
        std::vector<uint32_t> first(A.clist.empty() ? 0 : A.cverd.size(), 0xFFFFFFFFu);
        const uint32_t nkr = uni ? GK : A.nkc;  // row width: node key classes (uniform) or the table's
        for (uint32_t g = 0; g < G; g++) {
            const uint32_t sc = ipc_key[g][3 + c];
            for (uint32_t x = 0; x < nkr; x++) {
                const uint32_t lk = uni ? kc_key[x][c] : x;
                const size_t e = (size_t)sc * A.nkc + lk;
                if (A.clist.empty() || A.clist[e].empty()) {
                    X.push_back(A.cverd[e]);
                    continue;
                }
                if (first[e] == 0xFFFFFFFFu && ltab) {  // list id
                    if (lists.size() >= kNodeRecMask) return false;
                    first[e] = (uint32_t)lists.size();
                    lists.push_back(ListRef{c, e});
                } else if (first[e] == 0xFFFFFFFFu) {
                    const uint64_t ri = (rec0 + recs.size()) / 4;
                    if (ri >= kNodeRecMask) return false;
                    first[e] = (uint32_t)ri;
                    for (uint32_t r : A.clist[e]) {
                        const DevRule& R = A.rules[r];
                        recs.push_back(R.dnet);
                        recs.push_back((uint32_t)__builtin_popcount(R.dmask) << 18);
                        recs.push_back(kRecKeyAll);
                        recs.push_back(((R.act & 3u) << 30) | (A.rule_base + r));
                    }
                    recs.push_back(0);
                    recs.push_back(0);
                    recs.push_back(kRecKeyAll);
                    recs.push_back(A.cverd[e]);
                }
                X.push_back(kNodeList | first[e]);
            }
        }
    }
    std::vector<uint32_t> xcov;  // the cross-product tables (common rows); PAIR tables have none
    for (uint32_t t : cov)
        if (!an[t]->pair) xcov.push_back(t);
    build_common_rows(h, xcov, an, tu, uni);
    N.uniform = uni;
    N.tstride = uni ? G * GK : 0;
    N.crow0 = uni && N.cmap ? TI[N.tabinfo + 2] : 0;  // table 0's common row: table t's at crow0 + t * GK
    X.resize(rec0, 0);
    X.insert(X.end(), recs.begin(), recs.end());
    // list-verdict table (DevNode lv0): list L's verdict for node IP class g at lv0 + L * G + g --
    // its first rule whose dst prefix contains the class (every address of a class lies in the
    // same prefixes of every list table: the class key), else the verdict behind the list
    N.lv0 = 0;
    h.node_list_tab_words = 0;
    if (!lists.empty()) {
        if ((uint64_t)lists.size() * G > kNodeListTabBudget) {  // the record form instead (so not uniform)
            Tuning t2 = tu;
            t2.node_list_table = 0;
            t2.node_uniform = 0;
            return build_node(h, an, pods, node_end, t2);
        }
        N.lv0 = (uint32_t)X.size();
        h.node_list_tab_words = (uint32_t)(lists.size() * G);
        X.reserve(X.size() + lists.size() * G);
        for (const ListRef& L : lists) {
            const TableAnalysis& A = *an[cov[L.c]];
            for (uint32_t g = 0; g < G; g++) {
                uint32_t v = A.cverd[L.e];
                for (uint32_t r : A.clist[L.e]) {
                    const DevRule& R = A.rules[r];
                    if ((ipc_rep[g] & R.dmask) == R.dnet) {
                        v = ((R.act & 3u) << 30) | (A.rule_base + r);
                        break;
                    }
                }
                X.push_back(v);
            }
        }
    }
    // dst records, also at the end of the image when they fit node_list_words: a launch that
    // stages them walks a list in LDS instead of one dependent gather per record (config 3:
    // +17 % with the lists not walked at all, measured); launches that do not stage them read
    // the cross-array copy (device.hip)
    N.rec0 = (uint32_t)rec0;
    h.node_rec_words = (uint32_t)recs.size();
    N.lrec = 0;
    if (!recs.empty() && recs.size() <= tu.node_list_words) {
        while (img.size() % 4) img.push_back(0);
        N.lrec = (uint32_t)img.size();
        img.insert(img.end(), recs.begin(), recs.end());
        N.img_words = (uint32_t)img.size();
    }
    if (X.empty()) X.resize(4, 0);
    if ((uint64_t)X.size() * 4u >= kMaxLoaderBytes || (uint64_t)img.size() * 4u >= kMaxLoaderBytes) {
        h.node_img.clear();  // (the loaders' 32-bit byte offsets: no node; the per-table path)
        h.node_aux.clear();
        h.node_cross.clear();
        h.node = DevNode{};
        h.node_rec_words = 0;
        return false;
    }
    if (std::getenv("PG_NODE_DEBUG"))  // measurement aid: the image's shape
        std::fprintf(stderr,
                     "node: T %u G %u GK %u uniform %u | ip root %u depth %u, key root %u depth %u | words: "
                     "ip trie %u, key trie %u, ip rec %u, key rec %u, tabinfo+kmap %u, common %u, lists %u, total %u\n",
                     T, N.n_ipc, N.gk, N.uniform, N.ip_s1, N.ip_depth, N.key_k1, N.key_depth, N.key_root,
                     irec0 - N.key_root, krec0 - irec0, uni ? 0u : N.tabinfo - krec0, uni ? 0u : N.img_words_base - N.tabinfo,
                     (N.lrec ? N.lrec : N.img_words) - N.img_words_base, N.lrec ? N.img_words - N.lrec : 0,
                     N.img_words);
    return true;
}

}  // namespace pg
