/*
 * CPU oracle in C -- TEST INFRASTRUCTURE ONLY (tests/, smoke(), bench.py cpu_baseline leg).
 *
 * Restates, for bulk parity checks and the CPU baseline, the per-packet semantics of
 * /root/reference/mock/aclengine/aclengine_mock.go:
 *   evalACL          :503-652   (ora_eval_faithful: parses the CIDR strings on every rule
 *                                visit exactly like the Go loop; ora_eval: same loop over
 *                                rules parsed once per ACL, multi-threaded)
 *   testConnection   :424-501   (ora_conn; optionally every evaluation it makes, in order:
 *                                the hit-counter histogram of a connection batch;
 *                                ora_conn_faithful / ora_perpod_faithful: testConnection and
 *                                the per-pod evalACL over ora_eval_faithful's string-parsing
 *                                rule loop, the reference-shaped CPU baseline of those modes)
 * and Go 1.11 net.ParseCIDR / IPNet.Contains for IPv4 packets (src/net/ip.go), which the
 * evalACL loop calls per rule visit.  Independent of the product code in vpp_amd/csrc.
 * Pinned through oracle/aclengine.py (itself pinned by the reference's KATs) by
 * tests/test_oracle_c.py.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
    int32_t action;
    uint8_t has_macip, has_ip_rule, has_ip, has_icmp;
    const char* src;
    const char* dst;
    uint8_t tcp_present, tcp_has_src, tcp_has_dst, udp_present, udp_has_src, udp_has_dst, pad0, pad1;
    uint32_t tcp_src_lo, tcp_src_hi, tcp_dst_lo, tcp_dst_hi;
    uint32_t udp_src_lo, udp_src_hi, udp_dst_lo, udp_dst_hi;
} ora_rule;

typedef struct {  /* the raw rules of one ACL (the faithful variants) */
    const ora_rule* r;
    int n;
} ora_facl;

enum { A_DENY = 0, A_PERMIT = 1, A_REFLECT = 2, A_FAILURE = 3 };
enum { P_TCP = 0, P_UDP = 1, P_OTHER = 2 };

/* ---------------- Go 1.11 net.ParseCIDR (v4 + v6 syntax) -------------------------------- */
#define BIG 0xFFFFFF
static int dtoi(const char* s, int len, int* n, int* used) {
    int v = 0, i = 0;
    for (; i < len && s[i] >= '0' && s[i] <= '9'; i++) {
        v = v * 10 + (s[i] - '0');
        if (v >= BIG) { *n = BIG; *used = i; return 0; }
    }
    if (i == 0) { *n = 0; *used = 0; return 0; }
    *n = v; *used = i;
    return 1;
}
static int xtoi(const char* s, int len, int* n, int* used) {
    int v = 0, i = 0;
    for (; i < len; i++) {
        char c = s[i];
        if (c >= '0' && c <= '9') v = v * 16 + (c - '0');
        else if (c >= 'a' && c <= 'f') v = v * 16 + (c - 'a' + 10);
        else if (c >= 'A' && c <= 'F') v = v * 16 + (c - 'A' + 10);
        else break;
        if (v >= BIG) { *n = 0; *used = i; return 0; }
    }
    if (i == 0) { *n = 0; *used = 0; return 0; }
    *n = v; *used = i;
    return 1;
}
/* ip: 16 bytes (Go's IPv4() form for v4) */
static int parse_v4(const char* s, int len, uint8_t ip[16]) {
    uint8_t p[4];
    for (int i = 0; i < 4; i++) {
        if (len == 0) return 0;
        if (i > 0) { if (s[0] != '.') return 0; s++; len--; }
        int n, c;
        if (!dtoi(s, len, &n, &c) || n > 0xFF) return 0;
        s += c; len -= c; p[i] = (uint8_t)n;
    }
    if (len != 0) return 0;
    memset(ip, 0, 10); ip[10] = ip[11] = 0xFF;
    memcpy(ip + 12, p, 4);
    return 1;
}
static int parse_v6(const char* s, int len, uint8_t ip[16]) {
    memset(ip, 0, 16);
    int ellipsis = -1;
    if (len >= 2 && s[0] == ':' && s[1] == ':') {
        ellipsis = 0; s += 2; len -= 2;
        if (len == 0) return 1;
    }
    int i = 0;
    while (i < 16) {
        int n, c;
        if (!xtoi(s, len, &n, &c) || n > 0xFFFF) return 0;
        if (c < len && s[c] == '.') {
            if (ellipsis < 0 && i != 12) return 0;
            if (i + 4 > 16) return 0;
            uint8_t v4[16];
            if (!parse_v4(s, len, v4)) return 0;
            memcpy(ip + i, v4 + 12, 4);
            len = 0; i += 4;
            break;
        }
        ip[i] = (uint8_t)(n >> 8); ip[i + 1] = (uint8_t)n; i += 2;
        s += c; len -= c;
        if (len == 0) break;
        if (s[0] != ':' || len == 1) return 0;
        s++; len--;
        if (s[0] == ':') {
            if (ellipsis >= 0) return 0;
            ellipsis = i; s++; len--;
            if (len == 0) break;
        }
    }
    if (len != 0) return 0;
    if (i < 16) {
        if (ellipsis < 0) return 0;
        int n = 16 - i;
        for (int j = i - 1; j >= ellipsis; j--) ip[j + n] = ip[j];
        for (int j = ellipsis + n - 1; j >= ellipsis; j--) ip[j] = 0;
    } else if (ellipsis >= 0) {
        return 0;
    }
    return 1;
}
/* ParseCIDR + "can this network contain an IPv4 address, and with which (net, mask)".
 * returns: -1 parse error, 0 never contains IPv4, 1 ok */
static int parse_cidr_v4(const char* s, uint32_t* net, uint32_t* mask) {
    int len = (int)strlen(s);
    const char* slash = memchr(s, '/', len);
    if (!slash) return -1;
    int alen = (int)(slash - s);
    const char* m = slash + 1;
    int mlen = len - alen - 1;
    uint8_t ip[16];
    int iplen = 4;
    int ok = parse_v4(s, alen, ip);
    int v4syntax = ok;
    if (!ok) { iplen = 16; ok = parse_v6(s, alen, ip); }
    int n, used;
    int okm = dtoi(m, mlen, &n, &used);
    if (!ok || !okm || used != mlen || n < 0 || n > 8 * iplen) return -1;
    if (v4syntax) {
        uint32_t k = n ? (0xFFFFFFFFu << (32 - n)) : 0u;
        uint32_t a = ((uint32_t)ip[12] << 24) | ((uint32_t)ip[13] << 16) | ((uint32_t)ip[14] << 8) | ip[15];
        *mask = k; *net = a & k;
        return 1;
    }
    /* IPv6 syntax: 128-bit mask; the IPNet is IPv4-usable iff the masked address is
     * IPv4-mapped (To4 != nil), and then Contains uses mask[12:] (Go networkNumberAndMask) */
    uint8_t mk[16];
    for (int i = 0, r = n; i < 16; i++) {
        if (r >= 8) { mk[i] = 0xFF; r -= 8; } else { mk[i] = (uint8_t)(~(0xFFu >> r)); r = 0; }
    }
    for (int i = 0; i < 16; i++) ip[i] &= mk[i];
    for (int i = 0; i < 10; i++) if (ip[i]) return 0;
    if (ip[10] != 0xFF || ip[11] != 0xFF) return 0;
    uint32_t k = ((uint32_t)mk[12] << 24) | ((uint32_t)mk[13] << 16) | ((uint32_t)mk[14] << 8) | mk[15];
    uint32_t a = ((uint32_t)ip[12] << 24) | ((uint32_t)ip[13] << 16) | ((uint32_t)ip[14] << 8) | ip[15];
    *mask = k; *net = a & k;
    return 1;
}

/* ---------------- evalACL, faithful: strings parsed per rule visit -------------------- */
static int eval_faithful_one(const ora_rule* R, int n, uint32_t src, uint32_t dst, int proto, uint32_t dport,
                             int32_t* idx) {
    for (int i = 0; i < n; i++) {
        const ora_rule* r = &R[i];
        *idx = i;
        if (r->has_macip || !r->has_ip_rule) return A_FAILURE;
        if (r->has_icmp || !r->has_ip) return A_FAILURE;
        if (r->udp_present && r->tcp_present) return A_FAILURE;
        if (r->src && r->src[0]) {
            uint32_t net, mask;
            int k = parse_cidr_v4(r->src, &net, &mask);
            if (k < 0) return A_FAILURE;
            if (k == 0 || (src & mask) != net) continue;
        }
        if (r->dst && r->dst[0]) {
            uint32_t net, mask;
            int k = parse_cidr_v4(r->dst, &net, &mask);
            if (k < 0) return A_FAILURE;
            if (k == 0 || (dst & mask) != net) continue;
        }
        if (proto == P_TCP || proto == P_UDP) {
            int mine = proto == P_TCP ? r->tcp_present : r->udp_present;
            int other = proto == P_TCP ? r->udp_present : r->tcp_present;
            if (other) continue;
            if (mine) {
                int hs = proto == P_TCP ? r->tcp_has_src : r->udp_has_src;
                int hd = proto == P_TCP ? r->tcp_has_dst : r->udp_has_dst;
                uint32_t slo = proto == P_TCP ? r->tcp_src_lo : r->udp_src_lo;
                uint32_t shi = proto == P_TCP ? r->tcp_src_hi : r->udp_src_hi;
                uint32_t dlo = proto == P_TCP ? r->tcp_dst_lo : r->udp_dst_lo;
                uint32_t dhi = proto == P_TCP ? r->tcp_dst_hi : r->udp_dst_hi;
                if (!hs) return A_FAILURE;
                if (slo != 0 || shi != 0xFFFF) return A_FAILURE;
                if (!hd) return A_FAILURE;
                if (dport < (dlo & 0xFFFF) || dport > (dhi & 0xFFFF)) continue;
            }
        } else if (proto == P_OTHER) {
            if (r->tcp_present || r->udp_present) continue;
        }
        switch (r->action) {
            case A_DENY: return A_DENY;
            case A_PERMIT: return A_PERMIT;
            case A_REFLECT: return A_REFLECT;
            default: return A_FAILURE;
        }
    }
    *idx = -1;
    return A_DENY;
}

/* Threads of the faithful variants: one engine per thread over a contiguous slice of the tuples,
 * as BASELINE.md's B1 row runs the Go classifier with one engine per goroutine at
 * GOMAXPROCS=1 and GOMAXPROCS=$(nproc). Nothing is shared but the read-only rule strings. */
typedef struct {
    const ora_rule* rules;
    int n_rules;
    const uint32_t *src, *dst;
    const uint16_t* dport;
    const uint8_t* proto;
    int32_t *act, *idx;
    size_t lo, hi;
} faithful_job;

static void* faithful_worker(void* p) {
    faithful_job* j = (faithful_job*)p;
    for (size_t i = j->lo; i < j->hi; i++)
        j->act[i] = eval_faithful_one(j->rules, j->n_rules, j->src[i], j->dst[i], j->proto[i], j->dport[i], &j->idx[i]);
    return NULL;
}

int ora_eval_faithful(const ora_rule* rules, int n_rules, const uint32_t* src, const uint32_t* dst,
                      const uint16_t* dport, const uint8_t* proto, size_t n, int32_t* out_action, int32_t* out_idx,
                      int threads) {
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t th[256];
    faithful_job jobs[256];
    size_t per = (n + threads - 1) / threads;
    for (int t = 0; t < threads; t++) {
        size_t lo = t * per, hi = (t + 1) * per < n ? (t + 1) * per : n;
        if (lo > hi) lo = hi;
        jobs[t] = (faithful_job){rules, n_rules, src, dst, dport, proto, out_action, out_idx, lo, hi};
        if (threads == 1) faithful_worker(&jobs[t]);
        else pthread_create(&th[t], NULL, faithful_worker, &jobs[t]);
    }
    if (threads > 1)
        for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
    return 0;
}

/* ---------------- evalACL over rules parsed once -------------------------------------- */
typedef struct {
    int8_t pre_fail;   /* structural FAILURE before any test */
    int8_t src_state;  /* 0 any, 1 v4 net, 2 never, -1 parse error */
    int8_t dst_state;
    uint8_t tcp, udp, tcp_bad, udp_bad, action;
    uint32_t snet, smask, dnet, dmask;
    uint32_t tlo, thi, ulo, uhi;
} prule;

typedef struct ora_acl {
    int n;
    prule* r;
} ora_acl;

ora_acl* ora_acl_new(const ora_rule* rules, int n) {
    ora_acl* a = (ora_acl*)calloc(1, sizeof(ora_acl));
    a->n = n;
    a->r = (prule*)calloc(n > 0 ? n : 1, sizeof(prule));
    for (int i = 0; i < n; i++) {
        const ora_rule* s = &rules[i];
        prule* p = &a->r[i];
        p->pre_fail = s->has_macip || !s->has_ip_rule || s->has_icmp || !s->has_ip || (s->udp_present && s->tcp_present);
        if (s->src && s->src[0]) {
            int k = parse_cidr_v4(s->src, &p->snet, &p->smask);
            p->src_state = k < 0 ? -1 : (k == 0 ? 2 : 1);
        }
        if (s->dst && s->dst[0]) {
            int k = parse_cidr_v4(s->dst, &p->dnet, &p->dmask);
            p->dst_state = k < 0 ? -1 : (k == 0 ? 2 : 1);
        }
        p->tcp = s->tcp_present;
        p->udp = s->udp_present;
        p->tcp_bad = !s->tcp_has_src || s->tcp_src_lo != 0 || s->tcp_src_hi != 0xFFFF || !s->tcp_has_dst;
        p->udp_bad = !s->udp_has_src || s->udp_src_lo != 0 || s->udp_src_hi != 0xFFFF || !s->udp_has_dst;
        p->tlo = s->tcp_dst_lo & 0xFFFF; p->thi = s->tcp_dst_hi & 0xFFFF;
        p->ulo = s->udp_dst_lo & 0xFFFF; p->uhi = s->udp_dst_hi & 0xFFFF;
        p->action = (s->action >= 0 && s->action <= 2) ? (uint8_t)s->action : A_FAILURE;
    }
    return a;
}

void ora_acl_free(ora_acl* a) {
    if (!a) return;
    free(a->r);
    free(a);
}

static inline int eval_one(const ora_acl* a, uint32_t src, uint32_t dst, int proto, uint32_t port, int32_t* idx) {
    if (!a) { *idx = -1; return A_PERMIT; }
    for (int i = 0; i < a->n; i++) {
        const prule* r = &a->r[i];
        *idx = i;
        if (r->pre_fail) return A_FAILURE;
        if (r->src_state == -1) return A_FAILURE;
        if (r->src_state == 2 || (r->src_state == 1 && (src & r->smask) != r->snet)) continue;
        if (r->dst_state == -1) return A_FAILURE;
        if (r->dst_state == 2 || (r->dst_state == 1 && (dst & r->dmask) != r->dnet)) continue;
        if (proto == P_TCP) {
            if (r->udp) continue;
            if (r->tcp) {
                if (r->tcp_bad) return A_FAILURE;
                if (port < r->tlo || port > r->thi) continue;
            }
        } else if (proto == P_UDP) {
            if (r->tcp) continue;
            if (r->udp) {
                if (r->udp_bad) return A_FAILURE;
                if (port < r->ulo || port > r->uhi) continue;
            }
        } else if (proto == P_OTHER) {
            if (r->tcp || r->udp) continue;
        }
        return r->action;
    }
    *idx = -1;
    return A_DENY;
}

typedef struct {
    const ora_acl* acl;
    const uint32_t *src, *dst;
    const uint16_t* dport;
    const uint8_t* proto;
    int32_t *act, *idx;
    size_t lo, hi;
} eval_job;

static void* eval_worker(void* p) {
    eval_job* j = (eval_job*)p;
    for (size_t i = j->lo; i < j->hi; i++)
        j->act[i] = eval_one(j->acl, j->src[i], j->dst[i], j->proto[i], j->dport[i], &j->idx[i]);
    return NULL;
}

int ora_eval(const ora_acl* acl, const uint32_t* src, const uint32_t* dst, const uint16_t* dport,
             const uint8_t* proto, size_t n, int32_t* out_action, int32_t* out_idx, int threads) {
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t th[256];
    eval_job jobs[256];
    size_t per = (n + threads - 1) / threads;
    for (int t = 0; t < threads; t++) {
        jobs[t] = (eval_job){acl, src, dst, dport, proto, out_action, out_idx, t * per,
                             (t + 1) * per < n ? (t + 1) * per : n};
        if (jobs[t].lo > jobs[t].hi) jobs[t].lo = jobs[t].hi;
        pthread_create(&th[t], NULL, eval_worker, &jobs[t]);
    }
    for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
    return 0;
}

/* ---------------- testConnection (aclengine_mock.go:424-501) -------------------------- */
typedef struct {
    const ora_acl* const* acls; /* per table */
    const int32_t *if_in, *if_out;  /* per interface: table or -1 */
    const int32_t *sif, *dif;       /* per tuple: interface or -1 (unresolved -> FAILURE) */
    const uint32_t *src, *dst;
    const uint16_t *sport, *dport;
    const uint8_t* proto;
    int32_t *conn, *last_table, *last_idx;
    int32_t *ev_table, *ev_idx; /* optional: every evaluation, 4 per tuple (-3 = none) */
    size_t lo, hi;
    const ora_facl* facls;      /* set: the reference-faithful evaluation (strings parsed per
                                   rule visit) of these raw rules instead of acls */
} conn_job;

/* one evalACL of table t (-1 = nil ACL: PERMIT, aclengine_mock.go:506-508) */
static inline int eval_tab(const conn_job* j, int32_t t, uint32_t x, uint32_t y, int pr, uint32_t port, int32_t* li) {
    if (j->facls) {
        if (t < 0) { *li = -1; return A_PERMIT; }
        return eval_faithful_one(j->facls[t].r, j->facls[t].n, x, y, pr, port, li);
    }
    return eval_one(t >= 0 ? j->acls[t] : NULL, x, y, pr, port, li);
}

/* Every evalACL a connection makes is recorded in order (ev_table/ev_idx, up to 4 per
 * tuple, -3 = not made) when the caller asks for it: the per-rule hit counters of
 * testConnection count exactly these (the unresolved-interface FAILURE counts once, as
 * table -2). */
static int conn_one(const conn_job* j, size_t i, int32_t* lt, int32_t* li) {
    int32_t si = j->sif[i], di = j->dif[i];
    int32_t* evt = j->ev_table ? j->ev_table + 4 * i : NULL;
    int32_t* evi = j->ev_idx ? j->ev_idx + 4 * i : NULL;
    int nev = 0;
    if (evt)
        for (int k = 0; k < 4; k++) evt[k] = -3, evi[k] = -1;
    *lt = -2; *li = -1;
    if (si < 0 || di < 0) {
        if (evt) evt[0] = -2;
        return 3;
    }
    int same = si == di;
    int srefl = 0, drefl = 0, a;
    int pr = j->proto[i];
    uint32_t s = j->src[i], d = j->dst[i];
#define EV(tab, x, y, port)                                                      \
    do {                                                                         \
        int32_t t_ = (tab);                                                      \
        *lt = t_;                                                                \
        a = eval_tab(j, t_, x, y, pr, port, li);                                 \
        if (evt) evt[nev] = t_, evi[nev] = *li;                                  \
        nev++;                                                                   \
    } while (0)
    EV(j->if_in[si], s, d, j->dport[i]);
    if (a == A_FAILURE) return 3;
    if (a == A_DENY) return 0;
    if (a == A_REFLECT) { srefl = 1; if (same) drefl = 1; }
    if (!drefl) {
        EV(j->if_out[di], s, d, j->dport[i]);
        if (a == A_FAILURE) return 3;
        if (a == A_DENY) return 0;
        if (a == A_REFLECT) { drefl = 1; if (same) srefl = 1; }
    }
    if (!drefl) {
        EV(j->if_in[di], d, s, j->sport[i]);
        if (a == A_FAILURE) return 3;
        if (a == A_DENY) return 1;
    }
    if (!srefl) {
        EV(j->if_out[si], d, s, j->sport[i]);
        if (a == A_FAILURE) return 3;
        if (a == A_DENY) return 1;
    }
    return 2;
#undef EV
}

static void* conn_worker(void* p) {
    conn_job* j = (conn_job*)p;
    for (size_t i = j->lo; i < j->hi; i++) j->conn[i] = conn_one(j, i, &j->last_table[i], &j->last_idx[i]);
    return NULL;
}

int ora_conn(const ora_acl* const* acls, const int32_t* if_in, const int32_t* if_out, const int32_t* sif,
             const int32_t* dif, const uint32_t* src, const uint32_t* dst, const uint16_t* sport, const uint16_t* dport,
             const uint8_t* proto, size_t n, int32_t* out_conn, int32_t* out_last_table, int32_t* out_last_idx,
             int32_t* ev_table, int32_t* ev_idx, int threads) {
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t th[256];
    conn_job jobs[256];
    size_t per = (n + threads - 1) / threads;
    for (int t = 0; t < threads; t++) {
        size_t lo = t * per, hi = (t + 1) * per < n ? (t + 1) * per : n;
        if (lo > hi) lo = hi;
        jobs[t] = (conn_job){acls, if_in, if_out, sif, dif, src, dst, sport, dport, proto, out_conn, out_last_table,
                             out_last_idx, ev_table, ev_idx, lo, hi, NULL};
        pthread_create(&th[t], NULL, conn_worker, &jobs[t]);
    }
    for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
    return 0;
}

/* ---------------- per-pod mode: evalACL(outbound ACL of dst's interface) ---------------- */
static void* perpod_worker(void* p) {
    conn_job* j = (conn_job*)p;
    for (size_t i = j->lo; i < j->hi; i++) {
        const int32_t di = j->dif[i];
        if (di < 0) { /* interface not resolvable: FAILURE */
            j->conn[i] = A_FAILURE; j->last_table[i] = -2; j->last_idx[i] = -1;
            continue;
        }
        const int32_t t = j->if_out[di];
        j->last_table[i] = t;
        j->conn[i] = eval_tab(j, t, j->src[i], j->dst[i], j->proto[i], j->dport[i], &j->last_idx[i]);
    }
    return NULL;
}

int ora_perpod(const ora_acl* const* acls, const int32_t* if_out, const int32_t* dif, const uint32_t* src,
               const uint32_t* dst, const uint16_t* dport, const uint8_t* proto, size_t n, int32_t* out_action,
               int32_t* out_table, int32_t* out_idx, int threads) {
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t th[256];
    conn_job jobs[256];
    size_t per = (n + threads - 1) / threads;
    for (int t = 0; t < threads; t++) {
        size_t lo = t * per, hi = (t + 1) * per < n ? (t + 1) * per : n;
        if (lo > hi) lo = hi;
        jobs[t] = (conn_job){acls, NULL, if_out, NULL, dif, src, dst, NULL, dport, proto, out_action, out_table,
                             out_idx, NULL, NULL, lo, hi, NULL};
        pthread_create(&th[t], NULL, perpod_worker, &jobs[t]);
    }
    for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
    return 0;
}

/* ---------------- the same, reference-faithful: CIDR strings parsed on every rule visit ----------
 * (evalACL as aclengine_mock.go:535, 549 runs it: net.ParseCIDR per rule per packet), over the raw
 * rules of every table; at one thread and at every core (one engine per thread over a slice of the
 * tuples: BASELINE.md B1, GOMAXPROCS=1 and GOMAXPROCS=$(nproc)). */
static void run_jobs(conn_job* jobs, int threads, void* (*worker)(void*)) {
    pthread_t th[256];
    if (threads == 1) {
        worker(&jobs[0]);
        return;
    }
    for (int t = 0; t < threads; t++) pthread_create(&th[t], NULL, worker, &jobs[t]);
    for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
}

int ora_conn_faithful(const ora_facl* facls, const int32_t* if_in, const int32_t* if_out, const int32_t* sif,
                      const int32_t* dif, const uint32_t* src, const uint32_t* dst, const uint16_t* sport,
                      const uint16_t* dport, const uint8_t* proto, size_t n, int32_t* out_conn,
                      int32_t* out_last_table, int32_t* out_last_idx, int threads) {
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    conn_job jobs[256];
    size_t per = (n + threads - 1) / threads;
    for (int t = 0; t < threads; t++) {
        size_t lo = t * per, hi = (t + 1) * per < n ? (t + 1) * per : n;
        if (lo > hi) lo = hi;
        jobs[t] = (conn_job){NULL, if_in, if_out, sif, dif, src, dst, sport, dport, proto, out_conn, out_last_table,
                             out_last_idx, NULL, NULL, lo, hi, facls};
    }
    run_jobs(jobs, threads, conn_worker);
    return 0;
}

int ora_perpod_faithful(const ora_facl* facls, const int32_t* if_out, const int32_t* dif, const uint32_t* src,
                        const uint32_t* dst, const uint16_t* dport, const uint8_t* proto, size_t n,
                        int32_t* out_action, int32_t* out_table, int32_t* out_idx, int threads) {
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    conn_job jobs[256];
    size_t per = (n + threads - 1) / threads;
    for (int t = 0; t < threads; t++) {
        size_t lo = t * per, hi = (t + 1) * per < n ? (t + 1) * per : n;
        if (lo > hi) lo = hi;
        jobs[t] = (conn_job){NULL, NULL, if_out, NULL, dif, src, dst, NULL, dport, proto, out_action, out_table,
                             out_idx, NULL, NULL, lo, hi, facls};
    }
    run_jobs(jobs, threads, perpod_worker);
    return 0;
}
