/*
 * sentinel_oracle.c -- TEST INFRASTRUCTURE ONLY (see sentinel_oracle.h).
 *
 * Single-threaded CPU restatement of Sentinel 1.6.0's statistics-and-rule-check
 * path, clocked by event time (the reference's own AbstractTimeBasedTest mocks
 * TimeUtil the same way: core-test/test/AbstractTimeBasedTest.java:30-57).
 * Every function cites the Java it restates; paths use the SURVEY.md §0.1
 * prefixes (core/, param/, csrv/).  Concurrency machinery (CAS retry loops,
 * LongAdder striping, tryLock/yield) collapses to its single-thread outcome.
 *
 * Build: oracle/Makefile -> oracle/liboracle.so (gcc -O2 -ffp-contract=off).
 */
#include "sentinel_oracle.h"

#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <strings.h>

/* ======================================================================= */
/* Java arithmetic                                                          */
/* ======================================================================= */

/* (long) d -- JLS 5.1.3 narrowing: NaN -> 0, saturating, truncation */
static int64_t j_d2l(double d) {
    if (d != d) return 0;
    if (d >= 9223372036854775807.0) return INT64_MAX;
    if (d <= -9223372036854775808.0) return INT64_MIN;
    return (int64_t)d;
}
/* (int) d */
static int32_t j_d2i(double d) {
    if (d != d) return 0;
    if (d >= 2147483647.0) return INT32_MAX;
    if (d <= -2147483648.0) return INT32_MIN;
    return (int32_t)d;
}
static int32_t j_iadd(int32_t a, int32_t b) { return (int32_t)((uint32_t)a + (uint32_t)b); }
static int32_t j_imul(int32_t a, int32_t b) { return (int32_t)((uint32_t)a * (uint32_t)b); }
static int32_t j_idiv(int32_t a, int32_t b) {
    if (b == 0) return 0; /* ArithmeticException in Java; never reached with valid rules */
    if (a == INT32_MIN && b == -1) return INT32_MIN;
    return a / b;
}

/* java.lang.Math.round(double) (Java 8+: floor(a + 1/2) computed exactly) */
static int64_t j_round(double a) {
    union { double d; int64_t l; } u;
    u.d = a;
    int64_t bits = u.l;
    int64_t biased_exp = (bits & 0x7ff0000000000000LL) >> 52;
    int64_t shift = (52 - 1 + 1023) - biased_exp;
    if ((shift & -64) == 0) {
        int64_t r = (bits & 0x000fffffffffffffLL) | (0x000fffffffffffffLL + 1);
        if (bits < 0) r = -r;
        return ((r >> shift) + 1) >> 1;
    }
    return j_d2l(a);
}
/* java.lang.Math.nextUp(double) */
static double j_next_up(double d) {
    if (d != d || d == INFINITY) return d;
    return nextafter(d, INFINITY);
}
/* Double.doubleToLongBits -> Double.hashCode */
static int32_t j_double_hash(double d) {
    union { double d; uint64_t l; } u;
    u.d = d;
    if (d != d) u.l = 0x7ff8000000000000ULL;
    return (int32_t)(uint32_t)(u.l ^ (u.l >> 32));
}
/* java.lang.String.hashCode over the UTF-16 code units of a UTF-8 string */
static int32_t j_string_hash(const char* s) {
    if (!s) return 0;
    uint32_t h = 0;
    const unsigned char* p = (const unsigned char*)s;
    while (*p) {
        uint32_t cp;
        if (*p < 0x80) { cp = *p++; }
        else if ((*p & 0xE0) == 0xC0 && p[1]) { cp = ((p[0] & 0x1Fu) << 6) | (p[1] & 0x3Fu); p += 2; }
        else if ((*p & 0xF0) == 0xE0 && p[1] && p[2]) { cp = ((p[0] & 0x0Fu) << 12) | ((p[1] & 0x3Fu) << 6) | (p[2] & 0x3Fu); p += 3; }
        else if (p[1] && p[2] && p[3]) { cp = ((p[0] & 0x07u) << 18) | ((p[1] & 0x3Fu) << 12) | ((p[2] & 0x3Fu) << 6) | (p[3] & 0x3Fu); p += 4; }
        else { cp = *p++; }
        if (cp >= 0x10000) {
            cp -= 0x10000;
            h = 31u * h + (0xD800u + (cp >> 10));
            h = 31u * h + (0xDC00u + (cp & 0x3FFu));
        } else {
            h = 31u * h + cp;
        }
    }
    return (int32_t)h;
}
static int str_blank(const char* s) { /* StringUtil.isBlank */
    if (!s) return 1;
    for (; *s; ++s) if (*s != ' ' && *s != '\t' && *s != '\n' && *s != '\r' && *s != '\f' && *s != '\v') return 0;
    return 1;
}
static int str_eq(const char* a, const char* b) {
    if (!a || !b) return a == b;
    return strcmp(a, b) == 0;
}
static char* str_dup(const char* s) {
    if (!s) return NULL;
    size_t n = strlen(s) + 1;
    char* d = (char*)malloc(n);
    memcpy(d, s, n);
    return d;
}

/* ======================================================================= */
/* small hash map u64 -> i64 (open addressing, exact keys)                  */
/* ======================================================================= */
typedef struct {
    uint64_t* keys;
    int64_t* vals;
    uint8_t* used;          /* 0 empty, 1 live, 2 tombstone */
    uint64_t cap, n, tomb;
} u64map;

static uint64_t mix64(uint64_t x) {
    x ^= x >> 30; x *= 0xbf58476d1ce4e5b9ULL;
    x ^= x >> 27; x *= 0x94d049bb133111ebULL;
    x ^= x >> 31; return x;
}
static void m_free(u64map* m) { free(m->keys); free(m->vals); free(m->used); memset(m, 0, sizeof(*m)); }
static int64_t* m_find(u64map* m, uint64_t k) {
    if (!m->cap) return NULL;
    uint64_t i = mix64(k) & (m->cap - 1);
    while (m->used[i]) {
        if (m->used[i] == 1 && m->keys[i] == k) return &m->vals[i];
        i = (i + 1) & (m->cap - 1);
    }
    return NULL;
}
static void m_rehash(u64map* m, uint64_t cap);
static int64_t* m_put(u64map* m, uint64_t k, int64_t v) { /* insert or overwrite */
    if ((m->n + m->tomb + 1) * 2 > m->cap) /* live + tombstones at most half: probes always end */
        m_rehash(m, (m->n + 1) * 4 > m->cap ? (m->cap ? m->cap * 2 : 16) : m->cap);
    uint64_t i = mix64(k) & (m->cap - 1);
    while (m->used[i] == 1) {
        if (m->keys[i] == k) { m->vals[i] = v; return &m->vals[i]; }
        i = (i + 1) & (m->cap - 1);
    }
    /* may land on a tombstone (2) or empty (0); check the rest of the chain for k first */
    uint64_t j = i;
    while (m->used[j]) {
        if (m->used[j] == 1 && m->keys[j] == k) { m->vals[j] = v; return &m->vals[j]; }
        j = (j + 1) & (m->cap - 1);
    }
    if (m->used[i] == 2) m->tomb--;
    m->used[i] = 1; m->keys[i] = k; m->vals[i] = v; m->n++;
    return &m->vals[i];
}
static void m_del(u64map* m, uint64_t k) {
    if (!m->cap) return;
    uint64_t i = mix64(k) & (m->cap - 1);
    while (m->used[i]) {
        if (m->used[i] == 1 && m->keys[i] == k) { m->used[i] = 2; m->n--; m->tomb++; return; }
        i = (i + 1) & (m->cap - 1);
    }
}
static void m_rehash(u64map* m, uint64_t cap) {
    u64map o = *m;
    m->cap = cap;
    m->keys = (uint64_t*)calloc(m->cap, 8);
    m->vals = (int64_t*)calloc(m->cap, 8);
    m->used = (uint8_t*)calloc(m->cap, 1);
    m->n = 0;
    m->tomb = 0;
    for (uint64_t i = 0; i < o.cap; ++i)
        if (o.used[i] == 1) m_put(m, o.keys[i], o.vals[i]);
    free(o.keys); free(o.vals); free(o.used);
}

/* ======================================================================= */
/* CacheMap: ConcurrentLinkedHashMapWrapper(capacity) as ParameterMetric    */
/* uses it (param/.../ParameterMetric.java:37-114).  Access order = LRU:     */
/* get and putIfAbsent of a present key move it to the most-recently-used    */
/* end; an insert beyond the capacity evicts the least recently used entry   */
/* (ConcurrentLinkedHashMap's eviction deque, exact for one caller thread).  */
/* The library itself is not in /root/reference: restated, parity unpinned  */
/* (SURVEY Q13).                                                            */
/* ======================================================================= */
typedef struct {
    u64map idx;               /* key -> node */
    uint64_t* key;
    int64_t* val;
    int64_t *prev, *next;     /* -1 at the ends */
    int64_t head, tail;       /* head = most recently used */
    int64_t n_nodes, cap_nodes, free_head;
    uint64_t n, cap;          /* live entries, maximum */
} lrumap;

static void lm_init(lrumap* m, uint64_t cap) { memset(m, 0, sizeof(*m)); m->head = m->tail = m->free_head = -1; m->cap = cap; }
static void lm_free(lrumap* m) {
    m_free(&m->idx); free(m->key); free(m->val); free(m->prev); free(m->next);
    memset(m, 0, sizeof(*m)); m->head = m->tail = m->free_head = -1;
}
static void lm_unlink(lrumap* m, int64_t i) {
    if (m->prev[i] >= 0) m->next[m->prev[i]] = m->next[i]; else m->head = m->next[i];
    if (m->next[i] >= 0) m->prev[m->next[i]] = m->prev[i]; else m->tail = m->prev[i];
}
static void lm_front(lrumap* m, int64_t i) {
    m->prev[i] = -1; m->next[i] = m->head;
    if (m->head >= 0) m->prev[m->head] = i; else m->tail = i;
    m->head = i;
}
static int64_t lm_node(lrumap* m, uint64_t k) {
    int64_t* p = m_find(&m->idx, k);
    return p ? *p : -1;
}
static void lm_drop(lrumap* m, int64_t i) {
    lm_unlink(m, i);
    m_del(&m->idx, m->key[i]);
    m->next[i] = m->free_head; m->free_head = i;
    m->n--;
}
/* CacheMap.get: the value (touched) or NULL */
static int64_t* lm_get(lrumap* m, uint64_t k) {
    int64_t i = lm_node(m, k);
    if (i < 0) return NULL;
    if (m->head != i) { lm_unlink(m, i); lm_front(m, i); }
    return &m->val[i];
}
/* CacheMap.putIfAbsent: the present value (touched), or inserts v (*inserted = 1) and evicts beyond capacity */
static int64_t* lm_put_absent(lrumap* m, uint64_t k, int64_t v, int* inserted) {
    int64_t* p = lm_get(m, k);
    if (inserted) *inserted = p == NULL;
    if (p) return p;
    int64_t i = m->free_head;
    if (i >= 0) m->free_head = m->next[i];
    else {
        if (m->n_nodes == m->cap_nodes) {
            m->cap_nodes = m->cap_nodes ? m->cap_nodes * 2 : 16;
            m->key = (uint64_t*)realloc(m->key, 8 * (size_t)m->cap_nodes);
            m->val = (int64_t*)realloc(m->val, 8 * (size_t)m->cap_nodes);
            m->prev = (int64_t*)realloc(m->prev, 8 * (size_t)m->cap_nodes);
            m->next = (int64_t*)realloc(m->next, 8 * (size_t)m->cap_nodes);
        }
        i = m->n_nodes++;
    }
    m->key[i] = k; m->val[i] = v;
    m_put(&m->idx, k, i);
    lm_front(m, i);
    m->n++;
    while (m->n > m->cap && m->tail >= 0 && m->tail != i) lm_drop(m, m->tail);
    return &m->val[i];
}
/* CacheMap.put: insert or overwrite (touched) */
static void lm_put(lrumap* m, uint64_t k, int64_t v) { *lm_put_absent(m, k, v, NULL) = v; }
static void lm_remove(lrumap* m, uint64_t k) {
    int64_t i = lm_node(m, k);
    if (i >= 0) lm_drop(m, i);
}

/* string interning: name -> dense id */
typedef struct {
    u64map idx;     /* fnv(name) -> first id with that hash (chained via next) */
    char** names;
    int64_t* next;
    uint32_t n, cap;
} strtab;
static uint64_t fnv64(const char* s) {
    uint64_t h = 1469598103934665603ULL;
    for (; *s; ++s) { h ^= (unsigned char)*s; h *= 1099511628211ULL; }
    return h;
}
static int64_t st_find(strtab* t, const char* s) {
    int64_t* p = m_find(&t->idx, fnv64(s));
    if (!p) return -1;
    for (int64_t id = *p; id >= 0; id = t->next[id])
        if (strcmp(t->names[id], s) == 0) return id;
    return -1;
}
static uint32_t st_intern(strtab* t, const char* s) {
    int64_t id = st_find(t, s);
    if (id >= 0) return (uint32_t)id;
    if (t->n == t->cap) {
        t->cap = t->cap ? t->cap * 2 : 64;
        t->names = (char**)realloc(t->names, t->cap * sizeof(char*));
        t->next = (int64_t*)realloc(t->next, t->cap * sizeof(int64_t));
    }
    uint32_t nid = t->n++;
    t->names[nid] = str_dup(s);
    uint64_t h = fnv64(s);
    int64_t* p = m_find(&t->idx, h);
    t->next[nid] = p ? *p : -1;
    m_put(&t->idx, h, nid);
    return nid;
}
static void st_free(strtab* t) {
    for (uint32_t i = 0; i < t->n; ++i) free(t->names[i]);
    free(t->names); free(t->next); m_free(&t->idx);
    memset(t, 0, sizeof(*t));
}

/* ======================================================================= */
/* MetricBucket + LeapArray                                                 */
/* core/slots/statistic/data/MetricBucket.java:28-139                      */
/* core/slots/statistic/base/LeapArray.java:42-429                         */
/* ======================================================================= */
enum { EV_PASS = 0, EV_BLOCK, EV_EXC, EV_SUCC, EV_RT, EV_OCC, EV_N }; /* MetricEvent order */

typedef struct {
    int64_t ws;
    int64_t c[EV_N];
    int64_t min_rt;
    int present;
} obucket;

enum { LEAP_PLAIN = 0, LEAP_OCCUPIABLE = 1, LEAP_FUTURE = 2 };

typedef struct oleap {
    int kind, n, interval, wlen;
    int max_rt;              /* TIME_DROP_VALVE: MetricBucket.initMinRt */
    obucket* b;
    struct oleap* borrow;    /* OccupiableBucketLeapArray.borrowArray */
    obucket scratch;         /* detached bucket for a backwards clock */
} oleap;

static void leap_init(oleap* a, int kind, int n, int interval, int max_rt) {
    memset(a, 0, sizeof(*a));
    a->kind = kind; a->n = n; a->interval = interval; a->wlen = interval / n; a->max_rt = max_rt;
    a->b = (obucket*)calloc((size_t)n, sizeof(obucket));
    if (kind == LEAP_OCCUPIABLE) {
        a->borrow = (oleap*)malloc(sizeof(oleap));
        leap_init(a->borrow, LEAP_FUTURE, n, interval, max_rt);
    }
}
static void leap_free(oleap* a) {
    if (a->borrow) { leap_free(a->borrow); free(a->borrow); }
    free(a->b);
    memset(a, 0, sizeof(*a));
}
static void bucket_zero(obucket* b, int max_rt) { /* MetricBucket.reset() */
    for (int i = 0; i < EV_N; ++i) b->c[i] = 0;
    b->min_rt = max_rt;
}
/* LeapArray.isWindowDeprecated; FutureBucketLeapArray overrides (FutureBucketLeapArray.java:48-52) */
static int leap_deprecated(const oleap* a, int64_t t, const obucket* w) {
    if (a->kind == LEAP_FUTURE) return t >= w->ws;
    return t - w->ws > a->interval;
}
/* LeapArray.getWindowValue (LeapArray.java:251-264) + WindowWrap.isTimeInWindow (WindowWrap.java:88-90) */
static obucket* leap_window_value(oleap* a, int64_t t) {
    if (t < 0) return NULL;
    int idx = (int)((t / a->wlen) % a->n);
    obucket* b = &a->b[idx];
    if (!b->present || !(b->ws <= t && t < b->ws + a->wlen)) return NULL;
    return b;
}
/* newEmptyBucket: Occupiable copies ALL events of the borrow bucket (OccupiableBucketLeapArray.java:40-49) */
static void leap_new_empty(oleap* a, int64_t t, obucket* out) {
    bucket_zero(out, a->max_rt);
    if (a->kind == LEAP_OCCUPIABLE) {
        obucket* bb = leap_window_value(a->borrow, t);
        if (bb) { for (int i = 0; i < EV_N; ++i) out->c[i] = bb->c[i]; } /* MetricBucket.reset(bucket) */
    }
}
/* resetWindowTo: Occupiable zeroes then adds the borrow PASS only (OccupiableBucketLeapArray.java:52-64) */
static void leap_reset_to(oleap* a, obucket* w, int64_t ws) {
    w->ws = ws;
    bucket_zero(w, a->max_rt);
    if (a->kind == LEAP_OCCUPIABLE) {
        obucket* bb = leap_window_value(a->borrow, ws);
        if (bb) w->c[EV_PASS] += bb->c[EV_PASS];
    }
}
/* LeapArray.currentWindow(t) (LeapArray.java:117-208) */
static obucket* leap_current(oleap* a, int64_t t) {
    if (t < 0) return NULL;
    int idx = (int)((t / a->wlen) % a->n);
    int64_t ws = t - t % a->wlen;
    obucket* old = &a->b[idx];
    if (!old->present) {
        leap_new_empty(a, t, old);
        old->ws = ws; old->present = 1;
        return old;
    }
    if (ws == old->ws) return old;
    if (ws > old->ws) { leap_reset_to(a, old, ws); return old; }
    /* clock went back: a detached fresh bucket, updates are lost (Q3) */
    leap_new_empty(a, t, &a->scratch);
    a->scratch.ws = ws; a->scratch.present = 1;
    return &a->scratch;
}
static int leap_slot_of(const oleap* a, const obucket* b) {
    if (b == &a->scratch) return -2;
    return (int)(b - a->b);
}
/* sum of one event over values(t) (LeapArray.values, LeapArray.java:337-353) */
static int64_t leap_sum(oleap* a, int64_t t, int ev) {
    if (t < 0) return 0;
    int64_t s = 0;
    for (int i = 0; i < a->n; ++i) {
        obucket* w = &a->b[i];
        if (!w->present || leap_deprecated(a, t, w)) continue;
        s += w->c[ev];
    }
    return s;
}
/* LeapArray.getPreviousWindow(t) (LeapArray.java:216-234); isWindowDeprecated uses TimeUtil (= now) */
static obucket* leap_previous(oleap* a, int64_t t, int64_t now) {
    if (t < 0) return NULL;
    int64_t time_id = (t - a->wlen) / a->wlen;
    int idx = (int)(time_id % a->n);
    t = t - a->wlen;
    obucket* w = &a->b[idx];
    if (!w->present || leap_deprecated(a, now, w)) return NULL;
    if (w->ws + a->wlen < t) return NULL;
    return w;
}
/* LeapArray.getValidHead(t) (LeapArray.java:362-372) */
static obucket* leap_valid_head(oleap* a, int64_t t, int64_t now) {
    int idx = (int)(((t + a->wlen) / a->wlen) % a->n);
    obucket* w = &a->b[idx];
    if (!w->present || leap_deprecated(a, now, w)) return NULL;
    return w;
}

/* ======================================================================= */
/* ArrayMetric + StatisticNode                                              */
/* core/slots/statistic/metric/ArrayMetric.java:58-313                     */
/* core/node/StatisticNode.java:95-342                                      */
/* ======================================================================= */
typedef struct {
    oleap sec;     /* rollingCounterInSecond = ArrayMetric(SAMPLE_COUNT, INTERVAL) (occupiable) */
    oleap min;     /* rollingCounterInMinute = ArrayMetric(60, 60*1000, false) */
    int32_t thread;
    int64_t last_fetch;
    int created;
} onode;

typedef struct {
    int sample_count, interval, max_rt, cold_factor, occupy_timeout;
} ocfg;

static void node_init(onode* nd, const ocfg* c) {
    memset(nd, 0, sizeof(*nd));
    leap_init(&nd->sec, LEAP_OCCUPIABLE, c->sample_count, c->interval, c->max_rt);
    leap_init(&nd->min, LEAP_PLAIN, 60, 60 * 1000, c->max_rt);
    nd->last_fetch = -1;
    nd->created = 1;
}
static void node_free(onode* nd) {
    if (!nd->created) return;
    leap_free(&nd->sec); leap_free(&nd->min);
    nd->created = 0;
}
/* ArrayMetric reads: data.currentWindow() then a reduction over values() */
static int64_t am_sum(oleap* a, int64_t now, int ev) { leap_current(a, now); return leap_sum(a, now, ev); }
static double interval_sec(const oleap* a) { return a->interval / 1000.0; }

static double nd_pass_qps(onode* n, int64_t now) { return am_sum(&n->sec, now, EV_PASS) / interval_sec(&n->sec); }
static double nd_block_qps(onode* n, int64_t now) { return am_sum(&n->sec, now, EV_BLOCK) / interval_sec(&n->sec); }
static double nd_success_qps(onode* n, int64_t now) { return am_sum(&n->sec, now, EV_SUCC) / interval_sec(&n->sec); }
static double nd_exception_qps(onode* n, int64_t now) { return am_sum(&n->sec, now, EV_EXC) / interval_sec(&n->sec); }
static double nd_occupied_qps(onode* n, int64_t now) { return am_sum(&n->sec, now, EV_OCC) / interval_sec(&n->sec); }
static double nd_total_qps(onode* n, int64_t now) { return nd_pass_qps(n, now) + nd_block_qps(n, now); }
static double nd_avg_rt(onode* n, int64_t now) { /* StatisticNode.avgRt */
    int64_t succ = am_sum(&n->sec, now, EV_SUCC);
    if (succ == 0) return 0;
    return am_sum(&n->sec, now, EV_RT) * 1.0 / succ;
}
static double nd_min_rt(onode* n, int64_t now, int max_rt) { /* ArrayMetric.minRt (Q5) */
    leap_current(&n->sec, now);
    int64_t rt = max_rt;
    for (int i = 0; i < n->sec.n; ++i) {
        obucket* w = &n->sec.b[i];
        if (!w->present || leap_deprecated(&n->sec, now, w)) continue;
        if (w->min_rt < rt) rt = w->min_rt;
    }
    return (double)(rt > 1 ? rt : 1);
}
static double nd_max_success_qps(onode* n, int64_t now) {
    leap_current(&n->sec, now);
    int64_t s = 0;
    for (int i = 0; i < n->sec.n; ++i) {
        obucket* w = &n->sec.b[i];
        if (!w->present || leap_deprecated(&n->sec, now, w)) continue;
        if (w->c[EV_SUCC] > s) s = w->c[EV_SUCC];
    }
    if (s < 1) s = 1;
    return (double)s * n->sec.n;
}
/* ArrayMetric.previousWindowPass/Block on the minute window */
static double nd_previous(onode* n, int64_t now, int ev) {
    leap_current(&n->min, now);
    obucket* w = leap_previous(&n->min, now, now);
    return w ? (double)w->c[ev] : 0.0;
}
static int64_t nd_total(onode* n, int64_t now, int ev) { return am_sum(&n->min, now, ev); }
static int64_t nd_waiting(onode* n, int64_t now) { /* OccupiableBucketLeapArray.currentWaiting */
    leap_current(n->sec.borrow, now);
    return leap_sum(n->sec.borrow, now, EV_PASS);
}
static void am_add(oleap* a, int64_t now, int ev, int64_t v) {
    obucket* w = leap_current(a, now);
    if (w) w->c[ev] += v;
}
static void am_add_rt(oleap* a, int64_t now, int64_t rt) { /* MetricBucket.addRT (MetricBucket.java:126-133) */
    obucket* w = leap_current(a, now);
    if (!w) return;
    w->c[EV_RT] += rt;
    if (rt < w->min_rt) w->min_rt = rt;
}
static void nd_add_pass(onode* n, int64_t now, int c) { am_add(&n->sec, now, EV_PASS, c); am_add(&n->min, now, EV_PASS, c); }
static void nd_add_block(onode* n, int64_t now, int c) { am_add(&n->sec, now, EV_BLOCK, c); am_add(&n->min, now, EV_BLOCK, c); }
static void nd_add_exception(onode* n, int64_t now, int c) { am_add(&n->sec, now, EV_EXC, c); am_add(&n->min, now, EV_EXC, c); }
static void nd_add_rt_success(onode* n, int64_t now, int64_t rt, int c) { /* StatisticNode.addRtAndSuccess */
    am_add(&n->sec, now, EV_SUCC, c); am_add_rt(&n->sec, now, rt);
    am_add(&n->min, now, EV_SUCC, c); am_add_rt(&n->min, now, rt);
}
/* StatisticNode.tryOccupyNext (StatisticNode.java:293-325) */
static int64_t nd_try_occupy_next(onode* n, const ocfg* c, int64_t now, int acquire, double threshold) {
    double max_count = threshold * c->interval / 1000;
    int64_t cur_borrow = nd_waiting(n, now);
    if (cur_borrow >= max_count) return c->occupy_timeout;
    int wlen = c->interval / c->sample_count;
    int64_t earliest = now - now % wlen + wlen - c->interval;
    int idx = 0;
    int64_t cur_pass = am_sum(&n->sec, now, EV_PASS);
    while (earliest < now) {
        int64_t wait = (int64_t)idx * wlen + wlen - now % wlen;
        if (wait >= c->occupy_timeout) break;
        obucket* wb = leap_window_value(&n->sec, earliest);
        int64_t wpass = wb ? wb->c[EV_PASS] : 0;
        if (cur_pass + cur_borrow + acquire - wpass <= max_count) return wait;
        earliest += wlen;
        cur_pass -= wpass;
        idx++;
    }
    return c->occupy_timeout;
}
static void nd_add_waiting(onode* n, int64_t future_time, int acquire) {
    obucket* w = leap_current(n->sec.borrow, future_time);
    if (w) w->c[EV_PASS] += acquire;
}
static void nd_add_occupied_pass(onode* n, int64_t now, int acquire) {
    am_add(&n->min, now, EV_OCC, acquire);
    am_add(&n->min, now, EV_PASS, acquire);
}

/* ======================================================================= */
/* Traffic shaping controllers                                              */
/* core/slots/block/flow/controller/{Default,WarmUp,RateLimiter,WarmUpRateLimiter}Controller.java */
/* ======================================================================= */
struct or_ctrl {
    int behavior, grade;
    double count;
    int cold_factor;
    int32_t warning_token, max_token;
    double slope;
    int64_t stored, last_filled;      /* WarmUpController.storedTokens/lastFilledTime */
    int max_queue;
    int64_t latest;                   /* RateLimiter/WarmUpRateLimiter latestPassedTime */
};

/* WarmUpController.construct (WarmUpController.java:100-117) */
static void ctrl_init(or_ctrl* c, int behavior, int grade, double count, int warm, int max_queue, int cold) {
    memset(c, 0, sizeof(*c));
    c->behavior = behavior; c->grade = grade; c->count = count; c->max_queue = max_queue;
    c->latest = -1;
    if (behavior == SG_CONTROL_BEHAVIOR_WARM_UP || behavior == SG_CONTROL_BEHAVIOR_WARM_UP_RATE_LIMITER) {
        c->cold_factor = cold;
        c->warning_token = j_idiv(j_d2i(warm * count), cold - 1);
        c->max_token = j_iadd(c->warning_token, j_d2i(j_imul(2, warm) * count / (1.0 + cold)));
        c->slope = (cold - 1.0) / count / (double)(c->max_token - c->warning_token);
    }
}
/* WarmUpController.coolDownTokens (WarmUpController.java:161-174) */
static int64_t warm_cool_down(or_ctrl* c, int64_t cur, int64_t pass_qps) {
    int64_t old = c->stored, nv = old;
    if (old < c->warning_token) {
        nv = j_d2l(old + (cur - c->last_filled) * c->count / 1000);
    } else if (old > c->warning_token) {
        if (pass_qps < j_idiv(j_d2i(c->count), c->cold_factor))
            nv = j_d2l(old + (cur - c->last_filled) * c->count / 1000);
    }
    return nv < c->max_token ? nv : c->max_token;
}
/* WarmUpController.syncToken (WarmUpController.java:141-159) */
static void warm_sync(or_ctrl* c, int64_t now, int64_t pass_qps) {
    int64_t cur = now - now % 1000;
    if (cur <= c->last_filled) return;
    int64_t nv = warm_cool_down(c, cur, pass_qps);
    c->stored = nv;
    int64_t v = c->stored - pass_qps;
    c->stored = v < 0 ? 0 : v;
    c->last_filled = cur;
}
/* Math.nextUp(1.0 / (aboveToken * slope + 1.0 / count)) */
static double warm_qps(const or_ctrl* c, int64_t rest) {
    int64_t above = rest - c->warning_token;
    return j_next_up(1.0 / (above * c->slope + 1.0 / c->count));
}
/* Rate limiter core shared by RateLimiterController.canPass (RateLimiterController.java:46-91)
 * and WarmUpRateLimiterController.canPass (WarmUpRateLimiterController.java:43-87):
 * sleep() does not advance the replay clock (Q10); the wait is reported. */
static int rl_admit(int64_t* latest, int64_t cost, int64_t now, int max_queue, int64_t* wait_ms) {
    int64_t expected = cost + *latest;
    if (expected <= now) { *latest = now; return 1; }
    int64_t wait = cost + *latest - now;
    if (wait > max_queue) return 0;
    *latest += cost;
    wait = *latest - now;
    if (wait > max_queue) { *latest -= cost; return 0; }
    if (wait > 0 && wait_ms) *wait_ms = wait;
    return 1;
}

/* ======================================================================= */
/* rules                                                                    */
/* ======================================================================= */
typedef struct {
    sg_flow_rule r;          /* strings owned */
    char* limit_app_norm;    /* after "blank -> default" */
    int32_t hash;
    or_ctrl ctrl;
    int src_index;
} oflow;

typedef struct {
    sg_degrade_rule r;
    int32_t hash;
    int cut;
    int64_t pass_count;
    int64_t cut_until;
    int src_index;
} odegrade;

typedef struct {
    uint64_t key;
    int32_t count;
} ohot;

typedef struct {
    sg_param_rule r;
    sg_param_item* items;    /* owned copies */
    ohot* hot;               /* parsed hot items (ParamFlowRuleUtil.parseHotItems) */
    int n_hot;
    int32_t hash;
    int src_index;
} oparam;

/* per-(resource, rule) param state: ParameterMetric keeps maps keyed by rule *equality* */
typedef struct {
    oparam rule;             /* a copy used for equality only */
    lrumap time_map;         /* ruleTimeCounters[rule] */
    lrumap token_map;        /* ruleTokenCounter[rule] */
} oparam_state;

typedef struct {
    int32_t idx;
    lrumap map;              /* threadCountMap[paramIdx] */
} othread_map;

typedef struct {
    oparam_state* st; int n_st, cap_st;
    othread_map* tm; int n_tm, cap_tm;
    int exists;              /* ParamFlowSlot.metricsMap contains the resource */
} oparam_metric;

/* ---- equality (FlowRule.equals FlowRule.java:195-212, AbstractRule.equals AbstractRule.java:60-88) */
static int limit_app_equals(const char* s1, const char* s2) {
    if (s1 && strcmp(s1, "") == 0) return s2 && strcmp(s2, "default") == 0;
    if (s1 && strcmp(s1, "default") == 0) return !s2 || strcmp(s2, "") == 0 || strcmp(s1, s2) == 0;
    if (!s1) return !s2 || strcmp(s2, "default") == 0;
    return s2 && strcmp(s1, s2) == 0;
}
static int32_t abstract_rule_hash(const char* resource, const char* limit_app) {
    int32_t h = resource ? j_string_hash(resource) : 0;
    if (!(limit_app == NULL || strcmp(limit_app, "") == 0 || strcmp(limit_app, "default") == 0))
        h = j_iadd(j_imul(31, h), j_string_hash(limit_app));
    return h;
}
static int32_t long_hash(int64_t v) { return (int32_t)(uint32_t)((uint64_t)v ^ ((uint64_t)v >> 32)); }
/* ClusterFlowConfig.hashCode / ParamFlowClusterConfig.hashCode */
static int32_t cluster_cfg_hash(int64_t flow_id, int thr, int fallback, int strategy, int sc, int win, int has_strategy) {
    int32_t h = flow_id ? long_hash(flow_id) : 0;
    h = j_iadd(j_imul(31, h), thr);
    h = j_iadd(j_imul(31, h), fallback ? 1 : 0);
    if (has_strategy) h = j_iadd(j_imul(31, h), strategy);
    h = j_iadd(j_imul(31, h), sc);
    h = j_iadd(j_imul(31, h), win);
    return h;
}
/* FlowRule.hashCode (FlowRule.java:214-227) */
static int32_t flow_hash(const sg_flow_rule* r, const char* limit_app) {
    int32_t h = abstract_rule_hash(r->resource, limit_app);
    h = j_iadd(j_imul(31, h), r->grade);
    h = j_iadd(j_imul(31, h), j_double_hash(r->count));
    h = j_iadd(j_imul(31, h), r->strategy);
    h = j_iadd(j_imul(31, h), r->ref_resource ? j_string_hash(r->ref_resource) : 0);
    h = j_iadd(j_imul(31, h), r->control_behavior);
    h = j_iadd(j_imul(31, h), r->warm_up_period_sec);
    h = j_iadd(j_imul(31, h), r->max_queueing_time_ms);
    h = j_iadd(j_imul(31, h), r->cluster_mode ? 1 : 0);
    int32_t ch = 0;
    if (r->cluster_mode || r->cluster_flow_id) /* clusterConfig non-null */
        ch = cluster_cfg_hash(r->cluster_flow_id, r->cluster_threshold_type, r->cluster_fallback_to_local,
                              r->cluster_strategy, r->cluster_sample_count, r->cluster_window_interval_ms, 1);
    h = j_iadd(j_imul(31, h), ch);
    return h;
}
static int flow_equals(const oflow* a, const oflow* b) {
    if (!str_eq(a->r.resource, b->r.resource)) return 0;
    if (!limit_app_equals(a->limit_app_norm, b->limit_app_norm)) return 0;
    if (a->r.grade != b->r.grade) return 0;
    if (!(a->r.count == b->r.count || (a->r.count != a->r.count && b->r.count != b->r.count))) return 0;
    if (a->r.strategy != b->r.strategy || a->r.control_behavior != b->r.control_behavior) return 0;
    if (a->r.warm_up_period_sec != b->r.warm_up_period_sec) return 0;
    if (a->r.max_queueing_time_ms != b->r.max_queueing_time_ms) return 0;
    if ((a->r.cluster_mode != 0) != (b->r.cluster_mode != 0)) return 0;
    if (!str_eq(a->r.ref_resource, b->r.ref_resource)) return 0;
    int ac = a->r.cluster_mode || a->r.cluster_flow_id, bc = b->r.cluster_mode || b->r.cluster_flow_id;
    if (ac != bc) return 0;
    if (ac) {
        if (a->r.cluster_flow_id != b->r.cluster_flow_id) return 0;
        if (a->r.cluster_threshold_type != b->r.cluster_threshold_type) return 0;
        if ((a->r.cluster_fallback_to_local != 0) != (b->r.cluster_fallback_to_local != 0)) return 0;
        if (a->r.cluster_strategy != b->r.cluster_strategy) return 0;
        if (a->r.cluster_sample_count != b->r.cluster_sample_count) return 0;
        if (a->r.cluster_window_interval_ms != b->r.cluster_window_interval_ms) return 0;
    }
    return 1;
}
/* DegradeRule.hashCode/equals (DegradeRule.java:141-170) */
static int32_t degrade_hash(const sg_degrade_rule* r, const char* limit_app) {
    int32_t h = abstract_rule_hash(r->resource, limit_app);
    h = j_iadd(j_imul(31, h), j_double_hash(r->count));
    h = j_iadd(j_imul(31, h), r->time_window);
    h = j_iadd(j_imul(31, h), r->grade);
    return h;
}
static int degrade_equals(const odegrade* a, const odegrade* b) {
    return str_eq(a->r.resource, b->r.resource) && limit_app_equals(a->r.limit_app, b->r.limit_app) &&
           a->r.count == b->r.count && a->r.time_window == b->r.time_window && a->r.grade == b->r.grade;
}
/* ParamFlowItem.hashCode; ArrayList.hashCode (ParamFlowItem.java:97-103) */
static int32_t param_items_hash(const sg_param_item* it, int n) {
    int32_t h = 1;
    for (int i = 0; i < n; ++i) {
        int32_t e = it[i].object ? j_string_hash(it[i].object) : 0;
        e = j_iadd(j_imul(31, e), it[i].has_count ? it[i].count : 0);
        e = j_iadd(j_imul(31, e), it[i].class_type ? j_string_hash(it[i].class_type) : 0);
        h = j_iadd(j_imul(31, h), e);
    }
    return h;
}
/* ParamFlowRule.hashCode (ParamFlowRule.java:218-234) */
static int32_t param_hash(const sg_param_rule* r, const sg_param_item* items, const char* limit_app) {
    int32_t h = abstract_rule_hash(r->resource, limit_app);
    h = j_iadd(j_imul(31, h), r->grade);
    h = j_iadd(j_imul(31, h), r->has_param_idx ? r->param_idx : 0);
    h = j_iadd(j_imul(31, h), j_double_hash(r->count));
    h = j_iadd(j_imul(31, h), r->control_behavior);
    h = j_iadd(j_imul(31, h), r->max_queueing_time_ms);
    h = j_iadd(j_imul(31, h), r->burst_count);
    h = j_iadd(j_imul(31, h), long_hash(r->duration_in_sec));
    h = j_iadd(j_imul(31, h), param_items_hash(items, r->n_items));
    h = j_iadd(j_imul(31, h), r->cluster_mode ? 1 : 0);
    int32_t ch = 0;
    if (r->cluster_mode || r->cluster_flow_id)
        ch = cluster_cfg_hash(r->cluster_flow_id, r->cluster_threshold_type, r->cluster_fallback_to_local, 0,
                              r->cluster_sample_count, r->cluster_window_interval_ms, 0);
    h = j_iadd(j_imul(31, h), ch);
    return h;
}
static int param_items_equal(const sg_param_item* a, int na, const sg_param_item* b, int nb) {
    if (na != nb) return 0;
    for (int i = 0; i < na; ++i) {
        if (!str_eq(a[i].object, b[i].object) || !str_eq(a[i].class_type, b[i].class_type)) return 0;
        if ((a[i].has_count != 0) != (b[i].has_count != 0)) return 0;
        if (a[i].has_count && a[i].count != b[i].count) return 0;
    }
    return 1;
}
static int param_equals(const oparam* a, const oparam* b) {
    const sg_param_rule *x = &a->r, *y = &b->r;
    if (!str_eq(x->resource, y->resource) || !limit_app_equals(x->limit_app, y->limit_app)) return 0;
    if (x->grade != y->grade || !(x->count == y->count) || x->control_behavior != y->control_behavior) return 0;
    if (x->max_queueing_time_ms != y->max_queueing_time_ms || x->burst_count != y->burst_count) return 0;
    if (x->duration_in_sec != y->duration_in_sec || (x->cluster_mode != 0) != (y->cluster_mode != 0)) return 0;
    if ((x->has_param_idx != 0) != (y->has_param_idx != 0)) return 0;
    if (x->has_param_idx && x->param_idx != y->param_idx) return 0;
    if (!param_items_equal(a->items, x->n_items, b->items, y->n_items)) return 0;
    int xc = x->cluster_mode || x->cluster_flow_id, yc = y->cluster_mode || y->cluster_flow_id;
    if (xc != yc) return 0;
    if (xc && (x->cluster_flow_id != y->cluster_flow_id || x->cluster_threshold_type != y->cluster_threshold_type ||
               (x->cluster_fallback_to_local != 0) != (y->cluster_fallback_to_local != 0) ||
               x->cluster_sample_count != y->cluster_sample_count ||
               x->cluster_window_interval_ms != y->cluster_window_interval_ms))
        return 0;
    return 1;
}

/* java.util.HashSet iteration order (Q11): HashMap buckets (h ^ h>>>16) & (cap-1)
 * in table order, insertion order inside a bucket; capacity starts at 16 and
 * doubles when size exceeds cap*0.75, and when a bin would reach 9 nodes while
 * cap < 64 (HashMap.putVal/treeifyBin).  order[] holds insertion-ordered
 * element indices; it is permuted in place. */
static void java_hashset_order(const int32_t* hashes, int* order, int n) {
    if (n <= 1) return;
    int cap = 16;
    /* replay insertions to find the final capacity */
    int* bin_count = NULL;
    for (;;) {
        int grown = 0;
        free(bin_count);
        bin_count = (int*)calloc((size_t)cap, sizeof(int));
        int size = 0;
        for (int k = 0; k < n; ++k) {
            uint32_t h = (uint32_t)hashes[order[k]];
            h ^= h >> 16;
            int b = (int)(h & (uint32_t)(cap - 1));
            if (bin_count[b] >= 8 && cap < 64) { cap *= 2; grown = 1; break; }
            bin_count[b]++;
            if (++size > cap * 3 / 4) {
                if (k + 1 < n) { cap *= 2; grown = 1; break; }
            }
        }
        if (!grown) break;
    }
    free(bin_count);
    /* stable sort by bucket index */
    int* tmp = (int*)malloc(sizeof(int) * (size_t)n);
    int* key = (int*)malloc(sizeof(int) * (size_t)n);
    for (int k = 0; k < n; ++k) {
        uint32_t h = (uint32_t)hashes[order[k]];
        h ^= h >> 16;
        key[k] = (int)(h & (uint32_t)(cap - 1));
    }
    int m = 0;
    for (int b = 0; b < cap && m < n; ++b)
        for (int k = 0; k < n; ++k)
            if (key[k] == b) tmp[m++] = order[k];
    memcpy(order, tmp, sizeof(int) * (size_t)n);
    free(tmp); free(key);
}

/* ======================================================================= */
/* engine                                                                   */
/* ======================================================================= */
typedef struct {
    uint32_t ctx;      /* context name id */
    onode node;
} odefault;

typedef struct {
    uint32_t origin;   /* origin name id */
    onode node;
} oorigin;

typedef struct {
    int has_chain;
    int touched;       /* ClusterBuilderSlot created the ClusterNode */
    onode cluster;
    odefault* defs; int n_defs;
    oorigin* origins; int n_origins;
    /* compiled rules (indices into the engine's rule arrays), evaluation order */
    int* flow; int n_flow;
    int* degrade; int n_degrade;
    int* param; int n_param;
    oparam_metric pm;
} ores;

typedef struct {
    int64_t flow_id;
    double count;              /* FlowRule.count of the rule now mapped to this flowId */
    int32_t threshold_type;    /* ClusterFlowConfig.thresholdType */
    int live;                  /* still named by the loaded list */
    oleap metric;              /* ClusterMetricLeapArray (7 events) */
    int64_t occupy_pass, occupy_pass_req;
    int has_occupied;
    int32_t connected;
} ocluster;

/* token server view of a cluster-mode ParamFlowRule (ClusterParamFlowRuleManager) and its
 * ClusterParamMetric: a ClusterParameterLeapArray(sampleCount, windowIntervalMs) of per-bucket
 * value -> LongAdder maps (csrv/flow/statistic/metric/ClusterParamMetric.java:36-91,
 * ClusterParameterLeapArray.java:30-58).  A value's count in bucket j is live while its stamp equals
 * the bucket's window start (resetWindowTo clears the map).  Exact tables: the reference's CLHM
 * capacity of 4000 values per bucket (ClusterParamMetric.DEFAULT_CLUSTER_MAX_CAPACITY) is not
 * modelled -- parity unpinned beyond it. */
typedef struct { uint64_t key; int64_t* ws; int64_t* cnt; } ocpval;
typedef struct {
    int64_t flow_id;
    double count;
    int32_t threshold_type;
    int32_t connected;
    ohot* hot; int n_hot;
    int n; int64_t interval, wlen;
    int64_t* fws;               /* bucket window starts, -1 = never created */
    ocpval* vals; int n_vals;
    int live;
} ocparam;
static void cp_apply(void* e, const sg_param_rule* r, uint32_t n);

typedef struct {
    int64_t ts;
    uint8_t status;
    uint32_t res;
    uint32_t ctx;
    int32_t origin;        /* -1 none */
    int32_t count;
    int nargs;
    uint64_t key0;         /* args[0] key (scalar) */
    int key0_kind;
    int exited;
} oentry;

struct or_engine {
    ocfg c;
    int max_chain, switch_on;
    strtab names;          /* resource names */
    strtab ctx_names;      /* context names; 0 = sentinel_default_context */
    strtab origin_names;
    ores* res; uint32_t n_res, cap_res;
    uint32_t n_chains;
    oflow* flows; int n_flows;
    odegrade* degrades; int n_degrades;
    oparam* params; int n_params;
    /* last loaded lists (for the DynamicSentinelProperty equality no-op) */
    int flow_loaded, degrade_loaded, param_loaded;
    oflow* last_flow_list; int n_last_flow;
    odegrade* last_deg_list; int n_last_deg;
    oparam* last_par_list; int n_last_par;
    /* per-event entry records for EXIT/TRACE references */
    oentry* ents; uint64_t n_ents, cap_ents;
    uint64_t n_events;     /* global event counter (sg_event index) */
    u64map ev2ent;         /* global event index -> entry record */
    /* token server */
    ocluster* cl; int n_cl;
    ocparam* cp; int n_cp;
    oleap ns_limiter;      /* GlobalRequestLimiter (UnaryLeapArray(10, 1000)) */
    double max_allowed_qps;
    int cl_sample_count, cl_interval;
    double exceed_count, max_occupy_ratio;
};

static void free_flow(oflow* f) {
    free((char*)f->r.resource); free((char*)f->r.limit_app); free((char*)f->r.ref_resource);
    free(f->limit_app_norm);
}
static void free_param(oparam* p) {
    free((char*)p->r.resource); free((char*)p->r.limit_app);
    for (int i = 0; i < p->r.n_items; ++i) { free((char*)p->items[i].object); free((char*)p->items[i].class_type); }
    free(p->items); free(p->hot);
}

or_engine* or_create(const sg_config* cfg) {
    sg_config d;
    if (!cfg) { sg_config_default(&d); cfg = &d; }
    or_engine* e = (or_engine*)calloc(1, sizeof(or_engine));
    e->c.sample_count = cfg->sample_count;
    e->c.interval = cfg->interval_ms;
    e->c.max_rt = cfg->statistic_max_rt;
    e->c.cold_factor = cfg->cold_factor;
    e->c.occupy_timeout = cfg->occupy_timeout_ms;
    e->max_chain = cfg->max_slot_chain_size;
    e->switch_on = cfg->switch_on;
    st_intern(&e->ctx_names, "sentinel_default_context");
    leap_init(&e->ns_limiter, LEAP_PLAIN, 10, 1000, cfg->statistic_max_rt);
    e->max_allowed_qps = cfg->cluster_max_allowed_qps;
    e->cl_sample_count = cfg->cluster_sample_count;
    e->cl_interval = cfg->cluster_interval_ms;
    e->exceed_count = cfg->cluster_exceed_count;
    e->max_occupy_ratio = cfg->cluster_max_occupy_ratio;
    return e;
}

static void res_free(ores* r) {
    node_free(&r->cluster);
    for (int i = 0; i < r->n_defs; ++i) node_free(&r->defs[i].node);
    for (int i = 0; i < r->n_origins; ++i) node_free(&r->origins[i].node);
    free(r->defs); free(r->origins);
    free(r->flow); free(r->degrade); free(r->param);
    for (int i = 0; i < r->pm.n_st; ++i) {
        lm_free(&r->pm.st[i].time_map); lm_free(&r->pm.st[i].token_map);
        free_param(&r->pm.st[i].rule);
    }
    for (int i = 0; i < r->pm.n_tm; ++i) lm_free(&r->pm.tm[i].map);
    free(r->pm.st); free(r->pm.tm);
}

void or_destroy(or_engine* e) {
    if (!e) return;
    for (uint32_t i = 0; i < e->n_res; ++i) res_free(&e->res[i]);
    free(e->res);
    for (int i = 0; i < e->n_flows; ++i) free_flow(&e->flows[i]);
    free(e->flows);
    for (int i = 0; i < e->n_last_flow; ++i) free_flow(&e->last_flow_list[i]);
    free(e->last_flow_list);
    for (int i = 0; i < e->n_degrades; ++i) { free((char*)e->degrades[i].r.resource); free((char*)e->degrades[i].r.limit_app); }
    free(e->degrades);
    for (int i = 0; i < e->n_last_deg; ++i) { free((char*)e->last_deg_list[i].r.resource); free((char*)e->last_deg_list[i].r.limit_app); }
    free(e->last_deg_list);
    for (int i = 0; i < e->n_params; ++i) free_param(&e->params[i]);
    free(e->params);
    for (int i = 0; i < e->n_last_par; ++i) free_param(&e->last_par_list[i]);
    free(e->last_par_list);
    for (int i = 0; i < e->n_cl; ++i) leap_free(&e->cl[i].metric);
    free(e->cl);
    leap_free(&e->ns_limiter);
    cp_apply(e, NULL, 0);
    free(e->cp);
    free(e->ents);
    m_free(&e->ev2ent);
    st_free(&e->names); st_free(&e->ctx_names); st_free(&e->origin_names);
    free(e);
}

static ores* res_get(or_engine* e, uint32_t id) {
    while (id >= e->cap_res) {
        uint32_t nc = e->cap_res ? e->cap_res * 2 : 1024;
        e->res = (ores*)realloc(e->res, nc * sizeof(ores));
        memset(e->res + e->cap_res, 0, (nc - e->cap_res) * sizeof(ores));
        e->cap_res = nc;
    }
    if (id >= e->n_res) e->n_res = id + 1;
    return &e->res[id];
}

int or_register(or_engine* e, const char* name, uint32_t* out_id) {
    if (!e || !name) return SG_EINVAL;
    uint32_t id = st_intern(&e->names, name);
    res_get(e, id);
    if (out_id) *out_id = id;
    return SG_OK;
}

int or_register_many(or_engine* e, const char* const* names, uint32_t n) {
    for (uint32_t i = 0; i < n; ++i) {
        int rc = or_register(e, names[i], NULL);
        if (rc) return rc;
    }
    return SG_OK;
}

/* ---- FlowRuleUtil.isValidRule (FlowRuleUtil.java:174-228) -------------- */
static int flow_valid(const sg_flow_rule* r) {
    if (!r || str_blank(r->resource) || !(r->count >= 0) || r->grade < 0 || r->strategy < 0 || r->control_behavior < 0)
        return 0;
    if (r->cluster_mode) {
        if (r->cluster_flow_id <= 0) return 0;
        if (!(r->cluster_sample_count > 0 && r->cluster_window_interval_ms > 0 &&
              r->cluster_window_interval_ms % r->cluster_sample_count == 0))
            return 0;
        if (r->strategy != 0) return 0; /* switch (rule.getStrategy()) NORMAL only (FlowRuleUtil.java:189-194) */
    }
    if ((r->strategy == SG_STRATEGY_RELATE || r->strategy == SG_STRATEGY_CHAIN) && str_blank(r->ref_resource)) return 0;
    switch (r->control_behavior) {
    case SG_CONTROL_BEHAVIOR_WARM_UP: return r->warm_up_period_sec > 0;
    case SG_CONTROL_BEHAVIOR_RATE_LIMITER: return r->max_queueing_time_ms > 0;
    case SG_CONTROL_BEHAVIOR_WARM_UP_RATE_LIMITER: return r->warm_up_period_sec > 0 && r->max_queueing_time_ms > 0;
    default: return 1;
    }
}

/* FlowRuleComparator.compare (FlowRuleComparator.java:30-55) */
static int flow_cmp(const oflow* a, const oflow* b) {
    if (a->r.cluster_mode && !b->r.cluster_mode) return 1;
    if (!a->r.cluster_mode && b->r.cluster_mode) return -1;
    if (a->limit_app_norm == NULL) return 0;
    if (str_eq(a->limit_app_norm, b->limit_app_norm)) return 0;
    if (strcmp(a->limit_app_norm, "default") == 0) return 1;
    if (b->limit_app_norm && strcmp(b->limit_app_norm, "default") == 0) return -1;
    return 0;
}

static void copy_flow(oflow* d, const sg_flow_rule* s) {
    memset(d, 0, sizeof(*d));
    d->r = *s;
    d->r.resource = str_dup(s->resource);
    d->r.limit_app = str_dup(s->limit_app);
    d->r.ref_resource = str_dup(s->ref_resource);
    d->limit_app_norm = str_dup(str_blank(s->limit_app) ? "default" : s->limit_app);
}

static int flow_list_equal(or_engine* e, const sg_flow_rule* r, uint32_t n) {
    if (!e->flow_loaded || (int)n != e->n_last_flow) return 0;
    for (uint32_t i = 0; i < n; ++i) {
        oflow tmp;
        copy_flow(&tmp, &r[i]);
        int eq = flow_equals(&tmp, &e->last_flow_list[i]);
        free_flow(&tmp);
        if (!eq) return 0;
    }
    return 1;
}

/* FlowRuleManager.loadRules -> FlowRuleUtil.buildFlowRuleMap (FlowRuleUtil.java:89-137) */
int or_load_flow_rules(or_engine* e, const sg_flow_rule* r, uint32_t n, uint32_t* n_loaded) {
    if (!e || (n && !r)) return SG_EINVAL;
    if (flow_list_equal(e, r, n)) { /* DynamicSentinelProperty.updateValue no-op */
        if (n_loaded) {
            uint32_t k = 0;
            for (uint32_t i = 0; i < e->n_res; ++i) k += (uint32_t)e->res[i].n_flow;
            *n_loaded = k;
        }
        return SG_OK;
    }
    for (int i = 0; i < e->n_last_flow; ++i) free_flow(&e->last_flow_list[i]);
    free(e->last_flow_list);
    e->last_flow_list = (oflow*)calloc(n ? n : 1, sizeof(oflow));
    for (uint32_t i = 0; i < n; ++i) copy_flow(&e->last_flow_list[i], &r[i]);
    e->n_last_flow = (int)n;
    e->flow_loaded = 1;

    for (int i = 0; i < e->n_flows; ++i) free_flow(&e->flows[i]);
    free(e->flows);
    e->flows = (oflow*)calloc(n ? n : 1, sizeof(oflow));
    e->n_flows = 0;
    for (uint32_t i = 0; i < e->n_res; ++i) { free(e->res[i].flow); e->res[i].flow = NULL; e->res[i].n_flow = 0; }

    /* validate, default limitApp, build a fresh controller per rule, group per resource into HashSets */
    for (uint32_t i = 0; i < n; ++i) {
        if (!flow_valid(&r[i])) continue;
        oflow* f = &e->flows[e->n_flows];
        copy_flow(f, &r[i]);
        f->src_index = (int)i;
        f->hash = flow_hash(&f->r, f->limit_app_norm);
        ctrl_init(&f->ctrl, f->r.grade == SG_FLOW_GRADE_QPS ? f->r.control_behavior : SG_CONTROL_BEHAVIOR_DEFAULT,
                  f->r.grade, f->r.count, f->r.warm_up_period_sec, f->r.max_queueing_time_ms, e->c.cold_factor);
        uint32_t rid;
        or_register(e, f->r.resource, &rid);
        ores* rs = res_get(e, rid);
        /* HashSet.add: drop if an equal rule is already in this resource's set */
        int dup = 0;
        for (int k = 0; k < rs->n_flow; ++k)
            if (flow_equals(&e->flows[rs->flow[k]], f)) { dup = 1; break; }
        if (dup) { free_flow(f); memset(f, 0, sizeof(*f)); continue; }
        rs->flow = (int*)realloc(rs->flow, sizeof(int) * (size_t)(rs->n_flow + 1));
        rs->flow[rs->n_flow++] = e->n_flows;
        e->n_flows++;
    }
    int32_t* hs = (int32_t*)malloc(sizeof(int32_t) * (size_t)(e->n_flows > 0 ? (unsigned)e->n_flows : 1u));
    for (int k = 0; k < e->n_flows; ++k) hs[k] = e->flows[k].hash;
    for (uint32_t i = 0; i < e->n_res; ++i) {
        ores* rs = &e->res[i];
        if (rs->n_flow <= 1) continue;
        java_hashset_order(hs, rs->flow, rs->n_flow);   /* new ArrayList<>(HashSet) */
        /* Collections.sort(rules, FlowRuleComparator): stable insertion sort */
        for (int a = 1; a < rs->n_flow; ++a) {
            int v = rs->flow[a], b = a - 1;
            while (b >= 0 && flow_cmp(&e->flows[rs->flow[b]], &e->flows[v]) > 0) { rs->flow[b + 1] = rs->flow[b]; --b; }
            rs->flow[b + 1] = v;
        }
    }
    free(hs);
    if (n_loaded) *n_loaded = (uint32_t)e->n_flows;

    /* token server view: ClusterFlowRuleManager.applyClusterFlowRule (csrv/flow/rule/
     * ClusterFlowRuleManager.java:323-363) walks the list in order; cluster-mode rules that pass
     * FlowRuleUtil.isValidRule; ruleMap.put -> the last rule of a flowId wins; putMetricIfAbsent keeps
     * an existing metric (window shape included); clearAndResetRulesConditional drops the others. */
    for (int j = 0; j < e->n_cl; ++j) e->cl[j].live = 0;
    for (uint32_t i = 0; i < n; ++i) {
        const sg_flow_rule* q = &r[i];
        if (!q->cluster_mode || !flow_valid(q)) continue;
        int found = -1;
        for (int j = 0; j < e->n_cl; ++j) if (e->cl[j].flow_id == q->cluster_flow_id) found = j;
        if (found < 0) {
            e->cl = (ocluster*)realloc(e->cl, sizeof(ocluster) * (size_t)(e->n_cl + 1));
            ocluster* c = &e->cl[e->n_cl++];
            memset(c, 0, sizeof(*c));
            c->flow_id = q->cluster_flow_id;
            leap_init(&c->metric, LEAP_PLAIN, q->cluster_sample_count, q->cluster_window_interval_ms, e->c.max_rt);
            found = e->n_cl - 1;
        }
        e->cl[found].count = q->count;
        e->cl[found].threshold_type = q->cluster_threshold_type;
        e->cl[found].live = 1;
    }
    {
        int w = 0;
        for (int j = 0; j < e->n_cl; ++j) {
            if (e->cl[j].live) e->cl[w++] = e->cl[j];
            else leap_free(&e->cl[j].metric);
        }
        e->n_cl = w;
    }
    return SG_OK;
}

/* DegradeRuleManager.isValidRule (DegradeRuleManager.java:207-212) */
static int degrade_valid(const sg_degrade_rule* r) {
    return r && !str_blank(r->resource) && r->count >= 0 && r->time_window > 0;
}

int or_load_degrade_rules(or_engine* e, const sg_degrade_rule* r, uint32_t n, uint32_t* n_loaded) {
    if (!e || (n && !r)) return SG_EINVAL;
    /* DynamicSentinelProperty.updateValue: an equal list is a no-op (List.equals -> DegradeRule.equals) */
    if (e->degrade_loaded && (int)n == e->n_last_deg) {
        int eq = 1;
        for (uint32_t i = 0; i < n && eq; ++i) {
            odegrade t;
            memset(&t, 0, sizeof(t));
            t.r = r[i];
            eq = degrade_equals(&t, &e->last_deg_list[i]);
        }
        if (eq) { if (n_loaded) *n_loaded = (uint32_t)e->n_degrades; return SG_OK; }
    }
    for (int i = 0; i < e->n_last_deg; ++i) { free((char*)e->last_deg_list[i].r.resource); free((char*)e->last_deg_list[i].r.limit_app); }
    free(e->last_deg_list);
    e->last_deg_list = (odegrade*)calloc(n ? n : 1, sizeof(odegrade));
    for (uint32_t i = 0; i < n; ++i) {
        e->last_deg_list[i].r = r[i];
        e->last_deg_list[i].r.resource = str_dup(r[i].resource);
        e->last_deg_list[i].r.limit_app = str_dup(r[i].limit_app);
    }
    e->n_last_deg = (int)n;
    for (int i = 0; i < e->n_degrades; ++i) { free((char*)e->degrades[i].r.resource); free((char*)e->degrades[i].r.limit_app); }
    free(e->degrades);
    e->degrades = (odegrade*)calloc(n ? n : 1, sizeof(odegrade));
    e->n_degrades = 0;
    e->degrade_loaded = 1;
    for (uint32_t i = 0; i < e->n_res; ++i) { free(e->res[i].degrade); e->res[i].degrade = NULL; e->res[i].n_degrade = 0; }
    for (uint32_t i = 0; i < n; ++i) {
        if (!degrade_valid(&r[i])) continue;
        odegrade* d = &e->degrades[e->n_degrades];
        memset(d, 0, sizeof(*d));
        d->r = r[i];
        d->r.resource = str_dup(r[i].resource);
        d->r.limit_app = str_dup(str_blank(r[i].limit_app) ? "default" : r[i].limit_app);
        d->hash = degrade_hash(&d->r, d->r.limit_app);
        d->src_index = (int)i;
        uint32_t rid;
        or_register(e, d->r.resource, &rid);
        ores* rs = res_get(e, rid);
        int dup = 0;
        for (int k = 0; k < rs->n_degrade; ++k)
            if (degrade_equals(&e->degrades[rs->degrade[k]], d)) { dup = 1; break; }
        if (dup) { free((char*)d->r.resource); free((char*)d->r.limit_app); continue; }
        rs->degrade = (int*)realloc(rs->degrade, sizeof(int) * (size_t)(rs->n_degrade + 1));
        rs->degrade[rs->n_degrade++] = e->n_degrades;
        e->n_degrades++;
    }
    int32_t* hs = (int32_t*)malloc(sizeof(int32_t) * (size_t)(e->n_degrades > 0 ? (unsigned)e->n_degrades : 1u));
    for (int k = 0; k < e->n_degrades; ++k) hs[k] = e->degrades[k].hash;
    for (uint32_t i = 0; i < e->n_res; ++i)
        if (e->res[i].n_degrade > 1) java_hashset_order(hs, e->res[i].degrade, e->res[i].n_degrade);
    free(hs);
    if (n_loaded) *n_loaded = (uint32_t)e->n_degrades;
    return SG_OK;
}

/* ---- param values: type-tagged 64-bit keys -------------------------------
 * tag (top 4 bits): 1 String, 2 Integer, 3 Long, 4 Double, 5 Float, 6 Byte,
 * 7 Short, 8 Boolean, 9 Character.  Low 60 bits: the value (exact for the
 * 32-bit types and for Long in [-2^59, 2^59)), else a 60-bit FNV-1a hash of
 * the canonical text.  Restates ParamFlowRuleUtil.parseItemValue's typing
 * (param/slots/block/flow/param/ParamFlowRuleUtil.java:85-121). */
#define KEY_MASK 0x0FFFFFFFFFFFFFFFULL
static uint64_t tagged(uint64_t tag, uint64_t v) { return (tag << 60) | (v & KEY_MASK); }
static uint64_t fnv60(const char* s) { return fnv64(s) & KEY_MASK; }
uint64_t or_param_key(const char* value, const char* t) {
    if (!value) return 0;
    if (str_blank(t) || strcmp(t, "java.lang.String") == 0 || strcmp(t, "String") == 0) return tagged(1, fnv60(value));
    if (!strcmp(t, "int") || !strcmp(t, "java.lang.Integer")) return tagged(2, (uint32_t)(int32_t)strtol(value, NULL, 10));
    if (!strcmp(t, "long") || !strcmp(t, "java.lang.Long")) {
        long long v = strtoll(value, NULL, 10);
        if (v >= -(1LL << 59) && v < (1LL << 59)) return tagged(3, (uint64_t)v);
        return tagged(3, fnv60(value) | (1ULL << 59));
    }
    if (!strcmp(t, "double") || !strcmp(t, "java.lang.Double")) {
        double d = strtod(value, NULL);
        union { double d; uint64_t u; } u; u.d = d;
        return tagged(4, mix64(u.u));
    }
    if (!strcmp(t, "float") || !strcmp(t, "java.lang.Float")) {
        float f = strtof(value, NULL);
        union { float f; uint32_t u; } u; u.f = f;
        return tagged(5, u.u);
    }
    if (!strcmp(t, "byte") || !strcmp(t, "java.lang.Byte")) return tagged(6, (uint8_t)(int8_t)strtol(value, NULL, 10));
    if (!strcmp(t, "short") || !strcmp(t, "java.lang.Short")) return tagged(7, (uint16_t)(int16_t)strtol(value, NULL, 10));
    if (!strcmp(t, "boolean") || !strcmp(t, "java.lang.Boolean"))
        return tagged(8, (strcasecmp(value, "true") == 0) ? 1 : 0); /* Boolean.parseBoolean */
    if (!strcmp(t, "char")) return tagged(9, (unsigned char)value[0]);
    return tagged(1, fnv60(value)); /* unknown class type -> the String value */
}

/* ParamFlowRuleUtil.isValidRule (ParamFlowRuleUtil.java:32-38) */
static int param_valid(const sg_param_rule* r) {
    if (!r || str_blank(r->resource) || !(r->count >= 0) || r->grade < 0 || !r->has_param_idx || r->burst_count < 0 ||
        r->control_behavior < 0 || r->duration_in_sec <= 0 || r->max_queueing_time_ms < 0)
        return 0;
    if (r->cluster_mode) {
        if (!(r->cluster_sample_count > 0 && r->cluster_window_interval_ms > 0 &&
              r->cluster_window_interval_ms % r->cluster_sample_count == 0))
            return 0;
        if (r->cluster_flow_id <= 0) return 0;
    }
    return 1;
}

static void copy_param(oparam* d, const sg_param_rule* s) {
    memset(d, 0, sizeof(*d));
    d->r = *s;
    d->r.resource = str_dup(s->resource);
    d->r.limit_app = str_dup(str_blank(s->limit_app) ? "default" : s->limit_app);
    d->items = (sg_param_item*)calloc((size_t)(s->n_items > 0 ? s->n_items : 1), sizeof(sg_param_item));
    for (int i = 0; i < s->n_items; ++i) {
        d->items[i] = s->items[i];
        d->items[i].object = str_dup(s->items[i].object);
        d->items[i].class_type = str_dup(s->items[i].class_type);
    }
    d->r.items = d->items;
    /* ParamFlowRuleUtil.parseHotItems (ParamFlowRuleUtil.java:62-83): HashMap.put, later wins */
    d->hot = (ohot*)calloc((size_t)(s->n_items > 0 ? s->n_items : 1), sizeof(ohot));
    d->n_hot = 0;
    for (int i = 0; i < s->n_items; ++i) {
        const sg_param_item* it = &s->items[i];
        if (!it->object) continue;
        if (!it->has_count || it->count < 0) continue;
        uint64_t k = or_param_key(it->object, it->class_type);
        int j;
        for (j = 0; j < d->n_hot; ++j) if (d->hot[j].key == k) break;
        d->hot[j].key = k; d->hot[j].count = it->count;
        if (j == d->n_hot) d->n_hot++;
    }
}

static void pm_clear(oparam_metric* pm) { /* ParameterMetric removed from ParamFlowSlot.metricsMap */
    for (int i = 0; i < pm->n_st; ++i) { lm_free(&pm->st[i].time_map); lm_free(&pm->st[i].token_map); free_param(&pm->st[i].rule); }
    for (int i = 0; i < pm->n_tm; ++i) lm_free(&pm->tm[i].map);
    free(pm->st); free(pm->tm);
    memset(pm, 0, sizeof(*pm));
}

/* ParamFlowRuleManager.loadRules -> aggregateHotParamRules (ParamFlowRuleManager.java:103-166) */
int or_load_param_rules(or_engine* e, const sg_param_rule* r, uint32_t n, uint32_t* n_loaded) {
    if (!e || (n && !r)) return SG_EINVAL;
    if (e->param_loaded && (int)n == e->n_last_par) {
        int eq = 1;
        for (uint32_t i = 0; i < n && eq; ++i) {
            oparam tmp;
            copy_param(&tmp, &r[i]);
            eq = param_equals(&tmp, &e->last_par_list[i]);
            free_param(&tmp);
        }
        if (eq) { if (n_loaded) *n_loaded = (uint32_t)e->n_params; return SG_OK; }
    }
    for (int i = 0; i < e->n_last_par; ++i) free_param(&e->last_par_list[i]);
    free(e->last_par_list);
    e->last_par_list = (oparam*)calloc(n ? n : 1, sizeof(oparam));
    for (uint32_t i = 0; i < n; ++i) copy_param(&e->last_par_list[i], &r[i]);
    e->n_last_par = (int)n;
    uint32_t n_res_before = e->n_res;
    int* had = (int*)calloc(e->n_res ? e->n_res : 1, sizeof(int));
    for (uint32_t i = 0; i < e->n_res; ++i) had[i] = e->res[i].n_param > 0;
    for (int i = 0; i < e->n_params; ++i) free_param(&e->params[i]);
    free(e->params);
    e->params = (oparam*)calloc(n ? n : 1, sizeof(oparam));
    e->n_params = 0;
    e->param_loaded = 1;
    for (uint32_t i = 0; i < e->n_res; ++i) { free(e->res[i].param); e->res[i].param = NULL; e->res[i].n_param = 0; }
    cp_apply(e, r, n);  /* ClusterParamFlowRuleManager: the same list, its cluster-mode rules */
    if (n == 0) {
        /* "No parameter flow rules, so clear all the metrics" */
        for (uint32_t i = 0; i < e->n_res; ++i) pm_clear(&e->res[i].pm);
        free(had);
        if (n_loaded) *n_loaded = 0;
        return SG_OK;
    }
    for (uint32_t i = 0; i < n; ++i) {
        if (!param_valid(&r[i])) continue;
        oparam* p = &e->params[e->n_params];
        copy_param(p, &r[i]);
        p->hash = param_hash(&p->r, p->items, p->r.limit_app);
        p->src_index = (int)i;
        uint32_t rid;
        or_register(e, p->r.resource, &rid);
        ores* rs = res_get(e, rid);
        int dup = 0;
        for (int k = 0; k < rs->n_param; ++k)
            if (param_equals(&e->params[rs->param[k]], p)) { dup = 1; break; }
        if (dup) { free_param(p); memset(p, 0, sizeof(*p)); continue; }
        rs->param = (int*)realloc(rs->param, sizeof(int) * (size_t)(rs->n_param + 1));
        rs->param[rs->n_param++] = e->n_params;
        e->n_params++;
    }
    int32_t* hs = (int32_t*)malloc(sizeof(int32_t) * (size_t)(e->n_params > 0 ? (unsigned)e->n_params : 1u));
    for (int k = 0; k < e->n_params; ++k) hs[k] = e->params[k].hash;
    for (uint32_t i = 0; i < e->n_res; ++i)
        if (e->res[i].n_param > 1) java_hashset_order(hs, e->res[i].param, e->res[i].n_param);
    free(hs);
    /* clear unused hot param metrics (ParamFlowSlot.clearHotParamMetricForName) */
    for (uint32_t i = 0; i < n_res_before; ++i)
        if (had[i] && e->res[i].n_param == 0) pm_clear(&e->res[i].pm);
    free(had);
    if (n_loaded) *n_loaded = (uint32_t)e->n_params;
    return SG_OK;
}

int or_rule_order(or_engine* e, uint32_t res, int kind, int32_t* out, int cap) {
    if (!e || res >= e->n_res) return 0;
    ores* r = &e->res[res];
    int n = kind == 0 ? r->n_flow : kind == 1 ? r->n_degrade : r->n_param;
    int* l = kind == 0 ? r->flow : kind == 1 ? r->degrade : r->param;
    for (int i = 0; i < n && i < cap; ++i)
        out[i] = kind == 0 ? e->flows[l[i]].src_index : kind == 1 ? e->degrades[l[i]].src_index : e->params[l[i]].src_index;
    return n;
}

/* ======================================================================= */
/* node selection (FlowRuleChecker.selectNodeByRequesterAndStrategy,        */
/* core/slots/block/flow/FlowRuleChecker.java:67-124)                       */
/* ======================================================================= */
typedef struct {
    uint32_t res;
    uint32_t ctx;
    int32_t origin;            /* -1 = "" */
    onode* dnode;              /* DefaultNode (context, res) */
    onode* onode_;             /* origin StatisticNode or NULL */
    const char* origin_name;
    const char* ctx_name;
} octx;

static onode* default_node(or_engine* e, ores* r, uint32_t ctx) {
    for (int i = 0; i < r->n_defs; ++i) if (r->defs[i].ctx == ctx) return &r->defs[i].node;
    r->defs = (odefault*)realloc(r->defs, sizeof(odefault) * (size_t)(r->n_defs + 1));
    odefault* d = &r->defs[r->n_defs++];
    d->ctx = ctx;
    node_init(&d->node, &e->c);
    return &d->node;
}
static onode* origin_node(or_engine* e, ores* r, int32_t origin) {
    for (int i = 0; i < r->n_origins; ++i) if ((int32_t)r->origins[i].origin == origin) return &r->origins[i].node;
    r->origins = (oorigin*)realloc(r->origins, sizeof(oorigin) * (size_t)(r->n_origins + 1));
    oorigin* o = &r->origins[r->n_origins++];
    o->origin = (uint32_t)origin;
    node_init(&o->node, &e->c);
    return &o->node;
}

static int is_other_origin(or_engine* e, const octx* x) { /* FlowRuleManager.isOtherOrigin (FlowRuleManager.java:106-125) */
    if (!x->origin_name || !*x->origin_name) return 0;
    ores* r = &e->res[x->res];
    for (int i = 0; i < r->n_flow; ++i)
        if (str_eq(x->origin_name, e->flows[r->flow[i]].limit_app_norm)) return 0;
    return 1;
}
static onode* select_reference_node(or_engine* e, const oflow* f, const octx* x) {
    if (!f->r.ref_resource || !*f->r.ref_resource) return NULL;
    if (f->r.strategy == SG_STRATEGY_RELATE) {
        int64_t rid = st_find(&e->names, f->r.ref_resource);
        if (rid < 0 || (uint32_t)rid >= e->n_res || !e->res[rid].touched) return NULL;
        return &e->res[rid].cluster;
    }
    if (f->r.strategy == SG_STRATEGY_CHAIN) {
        if (!str_eq(f->r.ref_resource, x->ctx_name)) return NULL;
        return x->dnode;
    }
    return NULL;
}
static onode* select_node(or_engine* e, const oflow* f, const octx* x) {
    const char* la = f->limit_app_norm;
    const char* origin = x->origin_name ? x->origin_name : "";
    if (str_eq(la, origin) && strcmp(origin, "default") != 0 && strcmp(origin, "other") != 0) {
        if (f->r.strategy == SG_STRATEGY_DIRECT) return x->onode_;
        return select_reference_node(e, f, x);
    } else if (strcmp(la, "default") == 0) {
        if (f->r.strategy == SG_STRATEGY_DIRECT) return &e->res[x->res].cluster;
        return select_reference_node(e, f, x);
    } else if (strcmp(la, "other") == 0 && is_other_origin(e, x)) {
        if (f->r.strategy == SG_STRATEGY_DIRECT) return x->onode_;
        return select_reference_node(e, f, x);
    }
    return NULL;
}

/* ======================================================================= */
/* checks                                                                    */
/* ======================================================================= */
enum { R_PASS = 0, R_BLOCK = 1, R_WAIT = 2 };

/* TrafficShapingController.canPass on a real node */
static int ctrl_can_pass(or_engine* e, or_ctrl* c, onode* node, int64_t now, int acquire, int prioritized,
                         int64_t* wait_ms) {
    switch (c->behavior) {
    case SG_CONTROL_BEHAVIOR_WARM_UP: { /* WarmUpController.canPass (WarmUpController.java:119-139) */
        int64_t pass_qps = j_d2l(nd_pass_qps(node, now));
        int64_t prev_qps = j_d2l(nd_previous(node, now, EV_PASS));
        warm_sync(c, now, prev_qps);
        int64_t rest = c->stored;
        if (rest >= c->warning_token) {
            double wq = warm_qps(c, rest);
            if ((double)(pass_qps + acquire) <= wq) return R_PASS;
        } else {
            if ((double)(pass_qps + acquire) <= c->count) return R_PASS;
        }
        return R_BLOCK;
    }
    case SG_CONTROL_BEHAVIOR_RATE_LIMITER: { /* RateLimiterController.canPass */
        if (acquire <= 0) return R_PASS;
        if (c->count <= 0) return R_BLOCK;
        int64_t cost = j_round(1.0 * acquire / c->count * 1000);
        return rl_admit(&c->latest, cost, now, c->max_queue, wait_ms) ? R_PASS : R_BLOCK;
    }
    case SG_CONTROL_BEHAVIOR_WARM_UP_RATE_LIMITER: { /* WarmUpRateLimiterController.canPass */
        int64_t prev_qps = j_d2l(nd_previous(node, now, EV_PASS));
        warm_sync(c, now, prev_qps);
        int64_t rest = c->stored, cost;
        if (rest >= c->warning_token) {
            double wq = warm_qps(c, rest);
            cost = j_round(1.0 * acquire / wq * 1000);
        } else {
            cost = j_round(1.0 * acquire / c->count * 1000);
        }
        return rl_admit(&c->latest, cost, now, c->max_queue, wait_ms) ? R_PASS : R_BLOCK;
    }
    default: { /* DefaultController.canPass (DefaultController.java:49-81) */
        int32_t cur = c->grade == SG_FLOW_GRADE_THREAD ? node->thread : j_d2i(nd_pass_qps(node, now));
        if ((double)j_iadd(cur, acquire) > c->count) {
            if (prioritized && c->grade == SG_FLOW_GRADE_QPS) {
                int64_t wait = nd_try_occupy_next(node, &e->c, now, acquire, c->count);
                if (wait < e->c.occupy_timeout) {
                    nd_add_waiting(node, now + wait, acquire);
                    nd_add_occupied_pass(node, now, acquire);
                    if (wait_ms) *wait_ms = wait;
                    return R_WAIT; /* PriorityWaitException */
                }
            }
            return R_BLOCK;
        }
        return R_PASS;
    }
    }
}

/* FlowRuleChecker.passCheck (FlowRuleChecker.java:43-65); a cluster-mode rule
 * finds no TokenService in this process (pickClusterService() == null) and so
 * falls back to local checking or passes (fallbackToLocalOrPass). */
static int flow_pass_check(or_engine* e, oflow* f, const octx* x, int64_t now, int acquire, int prioritized,
                           int64_t* wait_ms) {
    if (f->limit_app_norm == NULL) return R_PASS;
    if (f->r.cluster_mode && !f->r.cluster_fallback_to_local) return R_PASS;
    onode* sel = select_node(e, f, x);
    if (!sel) return R_PASS;
    return ctrl_can_pass(e, &f->ctrl, sel, now, acquire, prioritized, wait_ms);
}

/* DegradeRule.passCheck (DegradeRule.java:172-223) with the replay reset rule (Q12) */
static int degrade_check_values(odegrade* d, int64_t now, double avg_rt, double exc_qps, double succ_qps,
                                double total_qps, double total_exc) {
    if (d->cut && now >= d->cut_until) { d->cut = 0; d->pass_count = 0; } /* ResetTask ran */
    if (d->cut) return 0;
    if (d->r.grade == SG_DEGRADE_GRADE_RT) {
        if (avg_rt < d->r.count) { d->pass_count = 0; return 1; }
        if (++d->pass_count < 5) return 1;
    } else if (d->r.grade == SG_DEGRADE_GRADE_EXCEPTION_RATIO) {
        if (total_qps < 5) return 1;
        double real_success = succ_qps - exc_qps;
        if (real_success <= 0 && exc_qps < 5) return 1;
        if (exc_qps / succ_qps < d->r.count) return 1;
    } else if (d->r.grade == SG_DEGRADE_GRADE_EXCEPTION_COUNT) {
        if (total_exc < d->r.count) return 1;
    }
    d->cut = 1;
    d->cut_until = now + (int64_t)d->r.time_window * 1000;
    return 0;
}
static int degrade_pass_check(odegrade* d, onode* cn, int cn_exists, int64_t now) {
    if (d->cut && now >= d->cut_until) { d->cut = 0; d->pass_count = 0; }
    if (d->cut) return 0;
    if (!cn_exists) return 1;
    /* read only the values the grade needs, in the Java order */
    double avg = 0, exc = 0, succ = 0, tot = 0, texc = 0;
    if (d->r.grade == SG_DEGRADE_GRADE_RT) avg = nd_avg_rt(cn, now);
    else if (d->r.grade == SG_DEGRADE_GRADE_EXCEPTION_RATIO) {
        exc = nd_exception_qps(cn, now); succ = nd_success_qps(cn, now); tot = nd_total_qps(cn, now);
    } else if (d->r.grade == SG_DEGRADE_GRADE_EXCEPTION_COUNT) texc = (double)nd_total(cn, now, EV_EXC);
    return degrade_check_values(d, now, avg, exc, succ, tot, texc);
}

/* ---- ParameterMetric (param/slots/block/flow/param/ParameterMetric.java:37-241) */
static oparam_state* pm_state(oparam_metric* pm, const oparam* rule) {
    for (int i = 0; i < pm->n_st; ++i) if (param_equals(&pm->st[i].rule, rule)) return &pm->st[i];
    return NULL;
}
static lrumap* pm_thread_map(oparam_metric* pm, int32_t idx) {
    for (int i = 0; i < pm->n_tm; ++i) if (pm->tm[i].idx == idx) return &pm->tm[i].map;
    return NULL;
}
static void pm_initialize(oparam_metric* pm, const oparam* rule) { /* ParameterMetric.initialize */
    pm->exists = 1;
    if (!pm_state(pm, rule)) {
        if (pm->n_st == pm->cap_st) {
            pm->cap_st = pm->cap_st ? pm->cap_st * 2 : 4;
            pm->st = (oparam_state*)realloc(pm->st, sizeof(oparam_state) * (size_t)pm->cap_st);
        }
        oparam_state* s = &pm->st[pm->n_st++];
        memset(s, 0, sizeof(*s));
        copy_param(&s->rule, &rule->r);
        s->rule.r.param_idx = rule->r.param_idx;
        /* Math.min(BASE_PARAM_MAX_CAPACITY * durationInSec, TOTAL_MAX_CAPACITY) (ParameterMetric.java:91,100) */
        int64_t cap = 4000 * rule->r.duration_in_sec;
        if (cap > 200000) cap = 200000;
        lm_init(&s->time_map, (uint64_t)cap);
        lm_init(&s->token_map, (uint64_t)cap);
    }
    if (!pm_thread_map(pm, rule->r.param_idx)) {
        if (pm->n_tm == pm->cap_tm) {
            pm->cap_tm = pm->cap_tm ? pm->cap_tm * 2 : 4;
            pm->tm = (othread_map*)realloc(pm->tm, sizeof(othread_map) * (size_t)pm->cap_tm);
        }
        othread_map* t = &pm->tm[pm->n_tm++];
        t->idx = rule->r.param_idx;
        lm_init(&t->map, 4000);  /* THREAD_COUNT_MAX_CAPACITY (ParameterMetric.java:37) */
    }
}
static int64_t pm_thread_count(oparam_metric* pm, int32_t idx, uint64_t v) {
    lrumap* m = pm_thread_map(pm, idx);
    if (!m) return 0;
    int64_t* p = lm_get(m, v);
    return p ? *p : 0;
}
static const ohot* hot_find(const oparam* p, uint64_t v) {
    for (int i = 0; i < p->n_hot; ++i) if (p->hot[i].key == v) return &p->hot[i];
    return NULL;
}

/* ParamFlowChecker.passDefaultLocalCheck (ParamFlowChecker.java:121-196) */
static int param_default_check(oparam_metric* pm, oparam* rule, int acquire, uint64_t v, int64_t now) {
    oparam_state* s = pm_state(pm, rule);
    if (!s) return 1;
    int32_t token_count = j_d2i(rule->r.count);
    const ohot* h = hot_find(rule, v);
    if (h) token_count = h->count;
    if (token_count == 0) return 0;
    int32_t max_count = j_iadd(token_count, rule->r.burst_count);
    if (acquire > max_count) return 0;
    int ins;
    int64_t* last = lm_put_absent(&s->time_map, v, now, &ins);  /* timeCounters.putIfAbsent(value, now) */
    if (ins) {
        lm_put_absent(&s->token_map, v, j_iadd(max_count, -acquire), NULL);
        return 1;
    }
    int64_t pass_time = now - *last;
    if (pass_time > rule->r.duration_in_sec * 1000) {
        int64_t* old = lm_put_absent(&s->token_map, v, j_iadd(max_count, -acquire), &ins);
        if (ins) {
            *last = now;
            return 1;
        }
        int32_t rest = (int32_t)*old;
        int32_t to_add = (int32_t)((pass_time * token_count) / (rule->r.duration_in_sec * 1000));
        int32_t sum = j_iadd(rest, to_add);
        int32_t nq = sum > max_count ? j_iadd(max_count, -acquire) : j_iadd(sum, -acquire);
        if (nq < 0) return 0;
        *old = nq;
        *last = now;
        return 1;
    }
    int64_t* old = lm_get(&s->token_map, v);
    if (old) {
        int32_t ov = (int32_t)*old;
        if (j_iadd(ov, -acquire) >= 0) { *old = j_iadd(ov, -acquire); return 1; }
        return 0;
    }
    return 1; /* unreachable: both maps see the same key sequence, so they hold the same keys (the Java loop
                 would spin until the window passes) */
}
/* ParamFlowChecker.passThrottleLocalCheck (ParamFlowChecker.java:198-248) */
static int param_throttle_check(oparam_metric* pm, oparam* rule, int acquire, uint64_t v, int64_t now, int64_t* wait_ms) {
    oparam_state* s = pm_state(pm, rule);
    if (!s) return 1;
    int64_t token_count = j_d2l(rule->r.count);
    const ohot* h = hot_find(rule, v);
    if (h) token_count = h->count;
    if (token_count == 0) return 0;
    int64_t cost = j_round(1.0 * 1000 * acquire * (double)rule->r.duration_in_sec / (double)token_count);
    int ins;
    int64_t* rec = lm_put_absent(&s->time_map, v, now, &ins);  /* timeRecorderMap.putIfAbsent(value, now) */
    if (ins) return 1;
    int64_t last = *rec;
    int64_t expected = last + cost;
    if (expected <= now || expected - now < rule->r.max_queueing_time_ms) {
        *rec = now;
        int64_t wait = expected - now;
        if (wait > 0) { *rec = expected; if (wait_ms) *wait_ms += wait; }  /* each element's check sleeps */
        return 1;
    }
    return 0;
}
/* ParamFlowChecker.passSingleValueCheck (ParamFlowChecker.java:101-119) */
static int param_single_check(oparam_metric* pm, oparam* rule, int acquire, uint64_t v, int64_t now, int64_t* wait_ms) {
    if (rule->r.grade == SG_FLOW_GRADE_QPS) {
        if (rule->r.control_behavior == SG_CONTROL_BEHAVIOR_RATE_LIMITER)
            return param_throttle_check(pm, rule, acquire, v, now, wait_ms);
        return param_default_check(pm, rule, acquire, v, now);
    } else if (rule->r.grade == SG_FLOW_GRADE_THREAD) {
        int64_t tc = pm_thread_count(pm, rule->r.param_idx, v);
        const ohot* h = hot_find(rule, v);
        if (h) return ++tc <= h->count;
        int64_t threshold = j_d2l(rule->r.count);
        return ++tc <= threshold;
    }
    return 1;
}

/* The args of one call: args[i] = a[i] (SG_ARG_NULL / SCALAR / LIST); a LIST's elements are
 * table[a[i].key .. a[i].key + a[i].len), each SCALAR or NULL (include/sentinel_gpu.h sg_arg). */
typedef struct {
    int n;
    const sg_arg* a;
    const sg_arg* table;
} oargs;

/* ParamFlowChecker.passCheck/passLocalCheck (ParamFlowChecker.java:48-99).  A null element of a
 * Collection/array reaches passSingleValueCheck, whose map lookup throws; passLocalCheck catches
 * Throwable and returns true, so the value passes and its later elements are not checked. */
static int param_pass_check(oparam_metric* pm, oparam* rule, int acquire, const oargs* a, int64_t now, int64_t* wait_ms) {
    int idx = rule->r.param_idx;
    if (a->n <= idx) return 1;
    const sg_arg* v = &a->a[idx];
    if (v->kind == SG_ARG_NULL) return 1;
    if (rule->r.cluster_mode && rule->r.grade == SG_FLOW_GRADE_QPS) {
        /* passClusterCheck: no TokenService -> fallbackToLocalOrPass */
        if (!rule->r.cluster_fallback_to_local) return 1;
    }
    if (v->kind == SG_ARG_LIST) {
        for (uint32_t i = 0; i < v->len; ++i) {
            const sg_arg* el = &a->table[v->key + i];
            if (el->kind != SG_ARG_SCALAR) return 1;
            if (!param_single_check(pm, rule, acquire, el->key, now, wait_ms)) return 0;
        }
        return 1;
    }
    return param_single_check(pm, rule, acquire, v->key, now, wait_ms);
}

/* ParameterMetric.addThreadCount / decreaseThreadCount (ParameterMetric.java:126-241): every index
 * with a thread-count map; a null element throws inside the try around the whole loop, so the
 * remaining elements and indices are skipped. */
static void pm_thread_one(lrumap* m, uint64_t v, int add) {
    int ins;
    int64_t* p = lm_put_absent(m, v, 0, &ins);  /* putIfAbsent(value, new AtomicInteger()) */
    if (add) {
        if (ins) lm_put(m, v, 1);               /* put(value, new AtomicInteger(1)) */
        else (*p)++;
    } else if (!ins) {
        if (--(*p) <= 0) lm_remove(m, v);
    }
}
static void pm_thread_args(oparam_metric* pm, const oargs* a, int add) {
    for (int i = 0; i < a->n; ++i) {
        lrumap* m = pm_thread_map(pm, i);
        const sg_arg* v = &a->a[i];
        if (!m || v->kind == SG_ARG_NULL) continue;
        if (v->kind == SG_ARG_LIST) {
            for (uint32_t k = 0; k < v->len; ++k) {
                const sg_arg* el = &a->table[v->key + k];
                if (el->kind != SG_ARG_SCALAR) return;
                pm_thread_one(m, el->key, add);
            }
        } else {
            pm_thread_one(m, v->key, add);
        }
    }
}

/* ======================================================================= */
/* the slot chain                                                           */
/* ======================================================================= */
static uint32_t mk_decision(int status, int rule, int64_t wait) {
    if (wait < 0) wait = 0;
    if (wait > 0xFFFF) wait = 0xFFFF;
    return (uint32_t)status | ((uint32_t)(rule & 0xFF) << 8) | ((uint32_t)wait << 16);
}

/* CtSph.lookProcessChain cap (core/CtSph.java:206-227, Q1) */
static int ensure_chain(or_engine* e, ores* r) {
    if (r->has_chain) return 1;
    if (e->max_chain > 0 && e->n_chains >= (uint32_t)e->max_chain) return 0;
    r->has_chain = 1;
    e->n_chains++;
    return 1;
}

/* CtSph.entryWithPriority -> DefaultProcessorSlotChain.entry -> ... */
static uint32_t do_entry(or_engine* e, int64_t now, uint32_t res, int32_t count, int prioritized, uint32_t ctx,
                         int32_t origin, const oargs* a, int upstream, uint8_t* status_out) {
    /* NullContext: more than MAX_CONTEXT_NAME_SIZE contexts (ContextUtil.trueEnter, CtSph.java:120-127) */
    if (ctx > SG_MAX_CONTEXTS) { *status_out = SG_NO_CHECK; return mk_decision(SG_NO_CHECK, 0, 0); }
    if (!e->switch_on) { *status_out = SG_NO_CHECK; return mk_decision(SG_NO_CHECK, 0, 0); }
    ores* r = res_get(e, res);
    if (!ensure_chain(e, r)) { *status_out = SG_NO_CHECK; return mk_decision(SG_NO_CHECK, 0, 0); }
    /* NodeSelectorSlot / ClusterBuilderSlot */
    onode* dn = default_node(e, r, ctx);
    if (!r->touched) { node_init(&r->cluster, &e->c); r->touched = 1; }
    onode* on = origin >= 0 ? origin_node(e, r, origin) : NULL;
    octx x;
    x.res = res; x.ctx = ctx; x.origin = origin; x.dnode = dn; x.onode_ = on;
    x.origin_name = origin >= 0 ? e->origin_names.names[origin] : "";
    x.ctx_name = e->ctx_names.names[ctx];

    int status = SG_PASS, rule_slot = 0;
    int64_t wait = 0;
    /* ParamFlowSlot (ParamFlowSlot.java:49-101) */
    if (r->n_param > 0) {
        for (int i = 0; i < r->n_param && status == SG_PASS; ++i) {
            oparam* p = &e->params[r->param[i]];
            /* applyRealParamIdx: mutates the rule */
            if (p->r.param_idx < 0) {
                if (-p->r.param_idx <= a->n) p->r.param_idx = a->n + p->r.param_idx;
                else p->r.param_idx = -p->r.param_idx;
            }
            pm_initialize(&r->pm, p);
            int64_t w = 0;
            if (!param_pass_check(&r->pm, p, count, a, now, &w)) { status = SG_BLOCK_PARAM; rule_slot = i; }
            else wait += w; /* the Java thread sleeps once per queueing check */
        }
    }
    /* SystemSlot / AuthoritySlot of the caller (after ParamFlowSlot, before FlowSlot) */
    if (status == SG_PASS && upstream) { status = SG_BLOCK_UPSTREAM; rule_slot = 0; }
    /* FlowSlot.checkFlow (FlowSlot.java:146-158) */
    if (status == SG_PASS) {
        for (int i = 0; i < r->n_flow; ++i) {
            int64_t w = 0;
            int rc = flow_pass_check(e, &e->flows[r->flow[i]], &x, now, count, prioritized, &w);
            if (rc == R_BLOCK) { status = SG_BLOCK_FLOW; rule_slot = i; break; }
            if (rc == R_WAIT) { status = SG_PASS_WAIT; rule_slot = i; wait += w; break; }
            wait += w;
        }
    }
    /* DegradeSlot -> DegradeRuleManager.checkDegrade (DegradeRuleManager.java:72-85) */
    if (status == SG_PASS) {
        for (int i = 0; i < r->n_degrade; ++i) {
            if (!degrade_pass_check(&e->degrades[r->degrade[i]], &r->cluster, r->touched, now)) {
                status = SG_BLOCK_DEGRADE; rule_slot = i; break;
            }
        }
    }
    /* StatisticSlot.entry bookkeeping (StatisticSlot.java:54-133) */
    if (status == SG_PASS) {
        dn->thread++; r->cluster.thread++;             /* DefaultNode.increaseThreadNum -> ClusterNode */
        nd_add_pass(dn, now, count); nd_add_pass(&r->cluster, now, count);
        if (on) { on->thread++; nd_add_pass(on, now, count); }
        if (r->pm.exists) pm_thread_args(&r->pm, a, 1);   /* ParamFlowStatisticEntryCallback.onPass */
    } else if (status == SG_PASS_WAIT) {
        dn->thread++; r->cluster.thread++;
        if (on) on->thread++;
        if (r->pm.exists) pm_thread_args(&r->pm, a, 1);
    } else {
        nd_add_block(dn, now, count); nd_add_block(&r->cluster, now, count);
        if (on) nd_add_block(on, now, count);
        wait = 0;
    }
    *status_out = (uint8_t)status;
    return mk_decision(status, rule_slot, wait);
}

/* CtEntry.exit -> StatisticSlot.exit (StatisticSlot.java:136-173) */
static void do_exit(or_engine* e, int64_t now, oentry* en, int32_t count, int64_t rt_raw, int with_args,
                    const oargs* a) {
    if (en->status != SG_PASS && en->status != SG_PASS_WAIT) return; /* error != null or no chain */
    ores* r = res_get(e, en->res);
    onode* dn = default_node(e, r, en->ctx);
    onode* on = en->origin >= 0 ? origin_node(e, r, en->origin) : NULL;
    int64_t rt = rt_raw > e->c.max_rt ? e->c.max_rt : rt_raw;
    nd_add_rt_success(dn, now, rt, count); nd_add_rt_success(&r->cluster, now, rt, count);
    if (on) nd_add_rt_success(on, now, rt, count);
    dn->thread--; r->cluster.thread--;
    if (on) on->thread--;
    /* ParamFlowStatisticExitCallback.onExit: only exit(count, args) carries args (Q14) */
    if (with_args && r->pm.exists && a) pm_thread_args(&r->pm, a, 0);
}

static oentry* new_entry(or_engine* e) {
    if (e->n_ents == e->cap_ents) {
        e->cap_ents = e->cap_ents ? e->cap_ents * 2 : 1024;
        e->ents = (oentry*)realloc(e->ents, sizeof(oentry) * e->cap_ents);
    }
    oentry* en = &e->ents[e->n_ents++];
    memset(en, 0, sizeof(*en));
    return en;
}

/* one batch of sg_submit / sg_submit_ex (ext and args may be NULL) */
static int submit_impl(or_engine* e, const sg_event* ev, const sg_event_ext* ext, uint64_t n, const sg_arg* args,
                       uint64_t n_args, uint32_t* out) {
    if (!e || (n && !ev)) return SG_EINVAL;
    for (uint64_t i = 0; i < n; ++i) {
        const sg_event* v = &ev[i];
        const sg_event_ext* x = ext ? &ext[i] : NULL;
        if (x && (x->n_args > SG_MAX_ARGS || (x->n_args && (!args || x->arg_off + (uint64_t)x->n_args > n_args))))
            return SG_EINVAL;
        uint32_t ctx = x ? x->context_id : 0;
        int32_t origin = x && x->origin_id ? (int32_t)x->origin_id - 1 : -1;
        uint64_t gidx = e->n_events++;
        uint32_t d = SG_NOT_ENTRY;
        sg_arg one = {v->aux, SG_ARG_SCALAR, 0};
        oargs a = {0, NULL, args};
        if (x && x->n_args) { a.n = (int)x->n_args; a.a = args + x->arg_off; }
        if (v->kind == SG_EV_ENTRY) {
            if (!(x && x->n_args) && (v->flags & SG_F_HAS_ARG)) { a.n = 1; a.a = &one; }
            oentry* en = new_entry(e);
            en->ts = v->ts; en->res = v->res_id; en->ctx = ctx; en->origin = origin; en->count = v->count;
            en->key0_kind = a.n && a.a[0].kind == SG_ARG_SCALAR ? 1 : 0;
            en->nargs = a.n ? 1 : 0;
            en->key0 = en->key0_kind ? a.a[0].key : 0;
            d = do_entry(e, v->ts, v->res_id, v->count, (v->flags & SG_F_PRIORITIZED) != 0, ctx, origin, &a,
                         (v->flags & SG_F_BLOCKED_UPSTREAM) != 0, &en->status);
            m_put(&e->ev2ent, gidx, (int64_t)(en - e->ents));
        } else if (v->kind == SG_EV_EXIT) {
            uint64_t ref = v->aux & SG_REF_NONE;
            int64_t rt_raw = (int64_t)(v->aux >> 48);
            oentry tmp, *en = NULL;
            if (ref != SG_REF_NONE) {
                int64_t* p = m_find(&e->ev2ent, ref);
                if (p) en = &e->ents[*p];
            }
            if (!en) { /* caller asserts the entry passed */
                memset(&tmp, 0, sizeof(tmp));
                ores* r = res_get(e, v->res_id);
                tmp.status = r->has_chain && e->switch_on && ctx <= SG_MAX_CONTEXTS ? SG_PASS : SG_NO_CHECK;
                tmp.res = v->res_id; tmp.ctx = ctx; tmp.origin = origin;
                en = &tmp;
            }
            /* Entry.exit(count, args): the exit's own args; without a table, the ENTRY's args[0] (Q14) */
            sg_arg k0 = {en->key0, en->key0_kind ? SG_ARG_SCALAR : SG_ARG_NULL, 0};
            oargs ea = a;
            if (!(x && x->n_args)) { ea.n = en->nargs; ea.a = &k0; }
            do_exit(e, v->ts, en, v->count, rt_raw, (v->flags & SG_F_EXIT_ARGS) != 0, &ea);
        } else if (v->kind == SG_EV_TRACE) {
            uint64_t ref = v->aux & SG_REF_NONE;
            int ok;
            if (ref != SG_REF_NONE) {
                int64_t* p = m_find(&e->ev2ent, ref);
                ok = p && (e->ents[*p].status == SG_PASS || e->ents[*p].status == SG_PASS_WAIT);
            } else {
                ok = v->res_id < e->n_res && e->res[v->res_id].has_chain && ctx <= SG_MAX_CONTEXTS;
            }
            ores* r = v->res_id < e->n_res ? &e->res[v->res_id] : NULL;
            /* Tracer.traceExceptionToNode -> ClusterNode.trace (ClusterNode.java:99-106) */
            if (ok && r && r->touched && v->count > 0) nd_add_exception(&r->cluster, v->ts, v->count);
        }
        if (out) out[i] = d;
    }
    return SG_OK;
}

int or_submit(or_engine* e, const sg_event* ev, uint64_t n, uint32_t* out) {
    return submit_impl(e, ev, NULL, n, NULL, 0, out);
}

int or_submit_ex(or_engine* e, const sg_event* ev, const sg_event_ext* ext, uint64_t n, const sg_arg* args,
                 uint64_t n_args, uint32_t* out) {
    return submit_impl(e, ev, ext, n, args, n_args, out);
}

int or_intern_origin(or_engine* e, const char* origin, uint32_t* out_id) {
    if (!e || !out_id) return SG_EINVAL;
    *out_id = (!origin || !*origin) ? 0 : st_intern(&e->origin_names, origin) + 1;
    return SG_OK;
}

int or_intern_context(or_engine* e, const char* context, uint32_t* out_id) {
    if (!e || !out_id) return SG_EINVAL;
    *out_id = st_intern(&e->ctx_names, context && *context ? context : "sentinel_default_context");
    return SG_OK;
}

uint32_t or_entry_ex(or_engine* e, int64_t now, uint32_t res, int32_t count, int prioritized, const char* context,
                     const char* origin, int nargs, const int32_t* arg_kind, const uint64_t* arg_key,
                     const uint64_t* const* arg_list, const int32_t* arg_len, uint64_t* handle) {
    uint32_t ctx = context ? st_intern(&e->ctx_names, context) : 0;
    int32_t org = (origin && *origin) ? (int32_t)st_intern(&e->origin_names, origin) : -1;
    /* the kinds/keys/lists of the call as an sg_arg table: args first, list elements after them */
    int total = nargs;
    for (int i = 0; i < nargs; ++i) if (arg_kind[i] == 2) total += arg_len[i];
    sg_arg* t = (sg_arg*)calloc((size_t)(total > 0 ? total : 1), sizeof(sg_arg));
    int off = nargs;
    for (int i = 0; i < nargs; ++i) {
        if (arg_kind[i] == 1) { t[i].kind = SG_ARG_SCALAR; t[i].key = arg_key[i]; }
        else if (arg_kind[i] == 2) {
            t[i].kind = SG_ARG_LIST; t[i].key = (uint64_t)off; t[i].len = (uint32_t)arg_len[i];
            for (int k = 0; k < arg_len[i]; ++k, ++off) {  /* UINT64_MAX stands for a null element */
                t[off].kind = arg_list[i][k] == UINT64_MAX ? SG_ARG_NULL : SG_ARG_SCALAR;
                t[off].key = arg_list[i][k];
            }
        }
    }
    oargs a = {nargs, t, t};
    oentry* en = new_entry(e);
    en->ts = now; en->res = res; en->ctx = ctx; en->origin = org; en->count = count;
    en->nargs = nargs > 0 ? 1 : 0;
    en->key0_kind = nargs > 0 && arg_kind[0] == 1 ? 1 : 0;
    en->key0 = en->key0_kind ? arg_key[0] : 0;
    uint32_t d = do_entry(e, now, res, count, prioritized, ctx, org, &a, 0, &en->status);
    free(t);
    if (handle) *handle = (uint64_t)(en - e->ents);
    return d;
}

int or_exit_ex(or_engine* e, int64_t now, uint64_t handle, int32_t count, int with_args) {
    if (handle >= e->n_ents) return SG_EINVAL;
    oentry* en = &e->ents[handle];
    if (en->exited) return SG_ESTATE;
    en->exited = 1;
    sg_arg k0 = {en->key0, en->key0_kind ? SG_ARG_SCALAR : SG_ARG_NULL, 0};
    oargs a = {en->nargs, &k0, &k0};
    do_exit(e, now, en, count, now - en->ts, with_args, &a);
    return SG_OK;
}

int or_trace_ex(or_engine* e, int64_t now, uint64_t handle, int32_t count) {
    if (handle >= e->n_ents) return SG_EINVAL;
    oentry* en = &e->ents[handle];
    if (en->status != SG_PASS && en->status != SG_PASS_WAIT) return SG_OK;
    ores* r = res_get(e, en->res);
    if (r->touched && count > 0) nd_add_exception(&r->cluster, now, count);
    return SG_OK;
}

/* ======================================================================= */
/* read-back, snapshots                                                     */
/* ======================================================================= */
static void export_bucket(const obucket* b, sg_bucket* o) {
    if (!b->present) { memset(o, 0, sizeof(*o)); o->window_start = -1; return; }
    o->window_start = b->ws;
    o->pass = b->c[EV_PASS]; o->block = b->c[EV_BLOCK]; o->exception = b->c[EV_EXC];
    o->success = b->c[EV_SUCC]; o->rt = b->c[EV_RT]; o->occupied_pass = b->c[EV_OCC];
    o->min_rt = b->min_rt;
}
static void export_node(const onode* n, int has_chain, sg_node_state* out) {
    memset(out, 0, sizeof(*out));
    for (int i = 0; i < 8; ++i) { out->second[i].window_start = -1; out->borrow[i].window_start = -1; }
    for (int i = 0; i < 60; ++i) out->minute[i].window_start = -1;
    if (n && n->created) {
        for (int i = 0; i < n->sec.n && i < 8; ++i) export_bucket(&n->sec.b[i], &out->second[i]);
        for (int i = 0; i < n->sec.n && i < 8; ++i) export_bucket(&n->sec.borrow->b[i], &out->borrow[i]);
        for (int i = 0; i < 60; ++i) export_bucket(&n->min.b[i], &out->minute[i]);
        out->cur_thread_num = n->thread;
    }
    out->has_chain = has_chain;
}
int or_read_node(or_engine* e, uint32_t res, sg_node_state* out) {
    if (!e || !out) return SG_EINVAL;
    if (res >= e->n_res) { export_node(NULL, 0, out); return SG_OK; }
    ores* r = &e->res[res];
    export_node(r->touched ? &r->cluster : NULL, r->has_chain, out);
    return SG_OK;
}
int or_read_origin_node(or_engine* e, uint32_t res, const char* origin, sg_node_state* out) {
    if (!e || !out || res >= e->n_res) return SG_EINVAL;
    int64_t o = st_find(&e->origin_names, origin);
    ores* r = &e->res[res];
    for (int i = 0; i < r->n_origins && o >= 0; ++i)
        if ((int64_t)r->origins[i].origin == o) { export_node(&r->origins[i].node, r->has_chain, out); return SG_OK; }
    export_node(NULL, r->has_chain, out);
    return SG_ENOTFOUND;
}
int or_read_default_node(or_engine* e, uint32_t res, const char* context, sg_node_state* out) {
    if (!e || !out || res >= e->n_res) return SG_EINVAL;
    int64_t c = st_find(&e->ctx_names, context ? context : "sentinel_default_context");
    ores* r = &e->res[res];
    for (int i = 0; i < r->n_defs && c >= 0; ++i)
        if ((int64_t)r->defs[i].ctx == c) { export_node(&r->defs[i].node, r->has_chain, out); return SG_OK; }
    export_node(NULL, r->has_chain, out);
    return SG_ENOTFOUND;
}

double or_node_metric(or_engine* e, uint32_t res, int64_t now, int which) {
    if (!e || res >= e->n_res || !e->res[res].touched) return 0;
    onode* n = &e->res[res].cluster;
    switch (which) {
    case 0: return nd_pass_qps(n, now);
    case 1: return nd_block_qps(n, now);
    case 2: return nd_success_qps(n, now);
    case 3: return nd_exception_qps(n, now);
    case 4: return nd_total_qps(n, now);
    case 5: return nd_avg_rt(n, now);
    case 6: return nd_min_rt(n, now, e->c.max_rt);
    case 7: return nd_previous(n, now, EV_PASS);
    case 8: return nd_previous(n, now, EV_BLOCK);
    case 9: return (double)nd_total(n, now, EV_EXC);
    case 10: return (double)nd_total(n, now, EV_PASS);
    case 11: return (double)(nd_total(n, now, EV_PASS) + nd_total(n, now, EV_BLOCK));
    case 12: return (double)nd_total(n, now, EV_SUCC);
    case 13: return nd_max_success_qps(n, now);
    case 14: return nd_occupied_qps(n, now);
    case 15: return n->thread;
    case 16: return (double)nd_waiting(n, now);
    }
    return 0;
}

/* StatisticNode.metrics (StatisticNode.java:124-151) over every ClusterNode */
int or_snapshot_metrics(or_engine* e, int64_t now, sg_metric_node* out, uint64_t cap, uint64_t* n) {
    if (!e) return SG_EINVAL;
    uint64_t k = 0;
    int64_t cur = now - now % 1000;
    for (uint32_t i = 0; i < e->n_res; ++i) {
        ores* r = &e->res[i];
        if (!r->touched) continue;
        onode* nd = &r->cluster;
        leap_current(&nd->min, now); /* details(): data.currentWindow() */
        int64_t new_last = nd->last_fetch;
        for (int s = 0; s < nd->min.n; ++s) {
            obucket* w = &nd->min.b[s];
            if (!w->present || leap_deprecated(&nd->min, now, w)) continue;
            sg_metric_node m;
            memset(&m, 0, sizeof(m));
            m.timestamp = w->ws;
            m.pass_qps = w->c[EV_PASS]; m.block_qps = w->c[EV_BLOCK]; m.exception_qps = w->c[EV_EXC];
            m.success_qps = w->c[EV_SUCC];
            m.rt = w->c[EV_SUCC] != 0 ? w->c[EV_RT] / w->c[EV_SUCC] : w->c[EV_RT];
            m.occupied_pass_qps = w->c[EV_OCC];
            m.res_id = i;
            int in_time = m.timestamp > nd->last_fetch && m.timestamp < cur;
            int valid = m.pass_qps > 0 || m.block_qps > 0 || m.success_qps > 0 || m.exception_qps > 0 || m.rt > 0 ||
                        m.occupied_pass_qps > 0;
            if (in_time && valid) {
                if (k < cap && out) out[k] = m;
                k++;
                if (m.timestamp > new_last) new_last = m.timestamp;
            }
        }
        nd->last_fetch = new_last;
    }
    if (n) *n = k;
    return SG_OK;
}

int or_param_set_thread_count(or_engine* e, uint32_t res, int32_t param_idx, uint64_t key, int64_t v) {
    if (!e || res >= e->n_res) return SG_EINVAL;
    oparam_metric* pm = &e->res[res].pm;
    lrumap* m = pm_thread_map(pm, param_idx);
    if (!m) {
        if (pm->n_tm == pm->cap_tm) {
            pm->cap_tm = pm->cap_tm ? pm->cap_tm * 2 : 4;
            pm->tm = (othread_map*)realloc(pm->tm, sizeof(othread_map) * (size_t)pm->cap_tm);
        }
        othread_map* t = &pm->tm[pm->n_tm++];
        t->idx = param_idx;
        lm_init(&t->map, 4000);
        m = &t->map;
    }
    lm_put(m, key, v);
    return SG_OK;
}

int or_param_thread_count(or_engine* e, uint32_t res, int32_t param_idx, uint64_t key, int64_t* out) {
    if (!e || res >= e->n_res || !out) return SG_EINVAL;
    *out = pm_thread_count(&e->res[res].pm, param_idx, key);
    return SG_OK;
}

/* ======================================================================= */
/* token server: ClusterFlowChecker.acquireClusterToken (csrv/flow/ClusterFlowChecker.java:55-112) */
/* ClusterMetric/ClusterMetricLeapArray (csrv/flow/statistic/metric/)         */
/* ======================================================================= */
enum { CF_PASS = 0, CF_BLOCK, CF_PASS_REQ, CF_BLOCK_REQ, CF_OCC_PASS, CF_OCC_BLOCK, CF_WAITING, CF_N };
/* ClusterMetricBucket has 7 counters; obucket has 6 + min_rt: store WAITING in min_rt slot */
static int64_t* cf_slot(obucket* b, int ev) { return ev < EV_N ? &b->c[ev] : &b->min_rt; }

static obucket* cl_current(ocluster* c, int64_t now) {
    oleap* a = &c->metric;
    int idx = (int)((now / a->wlen) % a->n);
    int64_t ws = now - now % a->wlen;
    obucket* old = &a->b[idx];
    if (!old->present) {
        memset(old, 0, sizeof(*old));
        old->ws = ws; old->present = 1;
        return old;
    }
    if (ws == old->ws) return old;
    if (ws > old->ws) {
        /* resetWindowTo + transferOccupyToBucket (ClusterMetricLeapArray.java:47-64) */
        memset(old, 0, sizeof(*old));
        old->ws = ws; old->present = 1;
        if (c->has_occupied) {
            *cf_slot(old, CF_OCC_PASS) += c->occupy_pass;
            *cf_slot(old, CF_PASS) += c->occupy_pass; c->occupy_pass = 0;
            *cf_slot(old, CF_PASS_REQ) += c->occupy_pass_req; c->occupy_pass_req = 0;
            c->has_occupied = 0;
        }
        return old;
    }
    memset(&a->scratch, 0, sizeof(a->scratch));
    a->scratch.ws = ws; a->scratch.present = 1;
    return &a->scratch;
}
static int64_t cl_sum(ocluster* c, int64_t now, int ev) {
    cl_current(c, now);
    int64_t s = 0;
    for (int i = 0; i < c->metric.n; ++i) {
        obucket* w = &c->metric.b[i];
        if (!w->present || now - w->ws > c->metric.interval) continue;
        s += *cf_slot(w, ev);
    }
    return s;
}
static double cl_avg(ocluster* c, int64_t now, int ev) { return cl_sum(c, now, ev) / (c->metric.interval / 1000.0); }
static void cl_add(ocluster* c, int64_t now, int ev, int64_t v) { *cf_slot(cl_current(c, now), ev) += v; }

/* ClusterParamFlowRuleManager.applyClusterParamRules (csrv/flow/rule/ClusterParamFlowRuleManager.java:318-369):
 * cluster-mode rules passing ParamFlowRuleUtil.isValidRule, in list order; ruleMap.put -> the last rule of
 * a flowId wins; putMetricIfAbsent keeps an existing ClusterParamMetric (window shape included);
 * metrics of flowIds no longer named are removed. */
static void cp_free_one(ocparam* c) {
    for (int i = 0; i < c->n_vals; ++i) { free(c->vals[i].ws); free(c->vals[i].cnt); }
    free(c->vals); free(c->fws); free(c->hot);
    memset(c, 0, sizeof(*c));
}
static void cp_apply(void* ev, const sg_param_rule* r, uint32_t n) {
    or_engine* e = (or_engine*)ev;
    for (int j = 0; j < e->n_cp; ++j) e->cp[j].live = 0;
    for (uint32_t i = 0; i < n; ++i) {
        const sg_param_rule* q = &r[i];
        if (!q->cluster_mode || !param_valid(q)) continue;
        int found = -1;
        for (int j = 0; j < e->n_cp; ++j) if (e->cp[j].flow_id == q->cluster_flow_id) found = j;
        if (found < 0) {
            e->cp = (ocparam*)realloc(e->cp, sizeof(ocparam) * (size_t)(e->n_cp + 1));
            ocparam* c = &e->cp[e->n_cp++];
            memset(c, 0, sizeof(*c));
            c->flow_id = q->cluster_flow_id;
            c->n = q->cluster_sample_count;
            c->interval = q->cluster_window_interval_ms;
            c->wlen = c->interval / c->n;
            c->fws = (int64_t*)malloc(sizeof(int64_t) * (size_t)c->n);
            for (int k = 0; k < c->n; ++k) c->fws[k] = -1;
            found = e->n_cp - 1;
        }
        ocparam* c = &e->cp[found];
        c->count = q->count;
        c->threshold_type = q->cluster_threshold_type;
        /* ParamFlowRuleUtil.fillExceptionFlowItems: the parsed hot items of this rule */
        oparam tmp;
        copy_param(&tmp, q);
        free(c->hot);
        c->hot = (ohot*)calloc((size_t)(tmp.n_hot > 0 ? tmp.n_hot : 1), sizeof(ohot));
        memcpy(c->hot, tmp.hot, sizeof(ohot) * (size_t)tmp.n_hot);
        c->n_hot = tmp.n_hot;
        free_param(&tmp);
        c->live = 1;
    }
    int w = 0;
    for (int j = 0; j < e->n_cp; ++j) {
        if (e->cp[j].live) e->cp[w++] = e->cp[j];
        else cp_free_one(&e->cp[j]);
    }
    e->n_cp = w;
}
/* LeapArray.currentWindow of the ClusterParameterLeapArray: create / reset (map cleared) */
static int cp_current(ocparam* c, int64_t now) {
    int idx = (int)((now / c->wlen) % c->n);
    int64_t ws = now - now % c->wlen;
    if (c->fws[idx] < 0 || ws > c->fws[idx]) c->fws[idx] = ws;
    return idx;  /* requests are time-ordered: ws < fws (a detached bucket) cannot occur */
}
static ocpval* cp_val(ocparam* c, uint64_t key, int create) {
    for (int i = 0; i < c->n_vals; ++i) if (c->vals[i].key == key) return &c->vals[i];
    if (!create) return NULL;
    c->vals = (ocpval*)realloc(c->vals, sizeof(ocpval) * (size_t)(c->n_vals + 1));
    ocpval* v = &c->vals[c->n_vals++];
    v->key = key;
    v->ws = (int64_t*)malloc(sizeof(int64_t) * (size_t)c->n);
    v->cnt = (int64_t*)calloc((size_t)c->n, sizeof(int64_t));
    for (int k = 0; k < c->n; ++k) v->ws[k] = -1;
    return v;
}
/* ClusterParamMetric.getSum: currentWindow(), then the value's count over the valid buckets */
static int64_t cp_sum(ocparam* c, int64_t now, uint64_t key) {
    cp_current(c, now);
    ocpval* v = cp_val(c, key, 0);
    if (!v) return 0;
    int64_t s = 0;
    for (int j = 0; j < c->n; ++j) {
        if (c->fws[j] < 0 || now - c->fws[j] > c->interval) continue;  /* isWindowDeprecated (strict >) */
        if (v->ws[j] == c->fws[j]) s += v->cnt[j];
    }
    return s;
}
static void cp_add(ocparam* c, int64_t now, uint64_t key, int64_t count) {
    int idx = cp_current(c, now);
    ocpval* v = cp_val(c, key, 1);
    if (v->ws[idx] != c->fws[idx]) { v->ws[idx] = c->fws[idx]; v->cnt[idx] = 0; }
    v->cnt[idx] += count;
}
/* GlobalRequestLimiter.tryPass (limit/GlobalRequestLimiter.java:46-54, RequestLimiter.java:72-87) */
static int ns_try_pass(or_engine* e, int64_t now) {
    if (e->max_allowed_qps < 0) return 1;  /* no limiter registered -> tryPass true */
    obucket* w = leap_current(&e->ns_limiter, now);
    int64_t s = leap_sum(&e->ns_limiter, now, EV_PASS);
    if (!((double)s / (e->ns_limiter.interval / 1000.0) + 1 <= e->max_allowed_qps)) return 0;
    if (w) w->c[EV_PASS] += 1;
    return 1;
}

/* DefaultTokenService.requestParamToken (csrv/flow/DefaultTokenService.java:50-61) ->
 * ClusterParamFlowChecker.acquireClusterToken (csrv/flow/ClusterParamFlowChecker.java:42-88) */
int or_cluster_request_param_tokens(or_engine* e, const sg_param_token_req* reqs, uint64_t n, const uint64_t* values,
                                    uint64_t n_values, sg_token_result* out) {
    for (uint64_t i = 0; i < n; ++i) {
        const sg_param_token_req* q = &reqs[i];
        sg_token_result* o = &out[i];
        memset(o, 0, sizeof(*o));
        if (q->value_off + q->n_values > n_values) return SG_EINVAL;
        if (q->flow_id <= 0 || q->acquire_count <= 0 || q->n_values == 0) { o->status = SG_TOKEN_BAD_REQUEST; continue; }
        ocparam* c = NULL;
        for (int k = 0; k < e->n_cp; ++k) if (e->cp[k].flow_id == q->flow_id) c = &e->cp[k];
        if (!c) { o->status = SG_TOKEN_NO_RULE_EXISTS; continue; }
        const int64_t now = q->ts;
        if (!ns_try_pass(e, now)) { o->status = SG_TOKEN_TOO_MANY_REQUEST; continue; }
        const uint64_t* v = values + q->value_off;
        double remaining = -1;
        int passed = 1;
        for (uint32_t k = 0; k < q->n_values; ++k) {
            double latest = (double)cp_sum(c, now, v[k]) / (c->interval / 1000.0);  /* getAvg */
            double raw = c->count;                                                     /* getRawThreshold */
            for (int h = 0; h < c->n_hot; ++h) if (c->hot[h].key == v[k]) { raw = c->hot[h].count; break; }
            double thr = c->threshold_type == SG_CLUSTER_THRESHOLD_GLOBAL ? raw : raw * c->connected;
            double next = thr - latest - q->acquire_count;
            remaining = next;
            if (next < 0) { passed = 0; break; }
        }
        if (passed)
            for (uint32_t k = 0; k < q->n_values; ++k) cp_add(c, now, v[k], q->acquire_count);
        if (q->n_values > 1) remaining = -1;  /* "Remaining field is unsupported for multi-values" */
        if (passed) { o->status = SG_TOKEN_OK; o->remaining = j_d2i(remaining); }
        else o->status = SG_TOKEN_BLOCKED;
    }
    return SG_OK;
}

int or_cluster_set_connected_count(or_engine* e, int64_t flow_id, int32_t connected) {
    /* ClusterFlowRuleManager / ClusterParamFlowRuleManager.getConnectedCount: the namespace's count */
    int hit = 0;
    for (int i = 0; i < e->n_cl; ++i) if (e->cl[i].flow_id == flow_id) { e->cl[i].connected = connected; hit = 1; }
    for (int i = 0; i < e->n_cp; ++i) if (e->cp[i].flow_id == flow_id) { e->cp[i].connected = connected; hit = 1; }
    return hit ? SG_OK : SG_ENOTFOUND;
}

int or_cluster_request_tokens(or_engine* e, const sg_token_req* reqs, uint64_t n, sg_token_result* out) {
    for (uint64_t i = 0; i < n; ++i) {
        const sg_token_req* q = &reqs[i];
        sg_token_result* o = &out[i];
        memset(o, 0, sizeof(*o));
        /* DefaultTokenService.requestToken (csrv/flow/DefaultTokenService.java:37-48) */
        if (q->flow_id <= 0 || q->acquire_count <= 0) { o->status = SG_TOKEN_BAD_REQUEST; continue; }
        ocluster* c = NULL;
        for (int k = 0; k < e->n_cl; ++k) if (e->cl[k].flow_id == q->flow_id) c = &e->cl[k];
        if (!c) { o->status = SG_TOKEN_NO_RULE_EXISTS; continue; }
        int64_t now = q->ts;
        if (!ns_try_pass(e, now)) { o->status = SG_TOKEN_TOO_MANY_REQUEST; continue; }
        double latest_qps = cl_avg(c, now, CF_PASS_REQ);
        double thr = c->threshold_type == SG_CLUSTER_THRESHOLD_GLOBAL ? c->count : c->count * c->connected;
        double global_threshold = thr * e->exceed_count;
        double next_remaining = global_threshold - latest_qps - q->acquire_count;
        if (next_remaining >= 0) {
            cl_add(c, now, CF_PASS, q->acquire_count);
            cl_add(c, now, CF_PASS_REQ, 1);
            if (q->prioritized) cl_add(c, now, CF_OCC_PASS, q->acquire_count);
            o->status = SG_TOKEN_OK;
            o->remaining = j_d2i(next_remaining);
            o->wait_in_ms = 0;
            continue;
        }
        if (q->prioritized) {
            double occupy_avg = cl_avg(c, now, CF_WAITING);
            if (occupy_avg <= e->max_occupy_ratio * global_threshold) {
                /* ClusterMetric.tryOccupyNext (ClusterMetric.java:78-98) */
                double lq = cl_avg(c, now, CF_PASS);
                cl_current(c, now);
                obucket* head = NULL;
                {
                    oleap* a = &c->metric;
                    int idx = (int)(((now + a->wlen) / a->wlen) % a->n);
                    obucket* w = &a->b[idx];
                    if (w->present && !(now - w->ws > a->interval)) head = w;
                }
                int64_t head_pass = head ? *cf_slot(head, CF_PASS) : 0;
                int64_t occupied = c->occupy_pass;
                if (lq + (q->acquire_count + occupied) - head_pass <= global_threshold) {
                    c->occupy_pass += q->acquire_count;
                    c->occupy_pass_req += 1;
                    c->has_occupied = 1;
                    cl_add(c, now, CF_WAITING, q->acquire_count);
                    int wait = 1000 / c->metric.n;
                    if (wait > 0) { o->status = SG_TOKEN_SHOULD_WAIT; o->remaining = 0; o->wait_in_ms = wait; continue; }
                }
            }
        }
        cl_add(c, now, CF_BLOCK, q->acquire_count);
        cl_add(c, now, CF_BLOCK_REQ, 1);
        if (q->prioritized) cl_add(c, now, CF_OCC_BLOCK, q->acquire_count);
        o->status = SG_TOKEN_BLOCKED;
    }
    return SG_OK;
}

/* ======================================================================= */
/* unit-level hooks                                                          */
/* ======================================================================= */
or_ctrl* or_ctrl_new(int behavior, int grade, double count, int warm, int max_queue, int cold) {
    or_ctrl* c = (or_ctrl*)malloc(sizeof(or_ctrl));
    ctrl_init(c, behavior, grade, count, warm, max_queue, cold);
    return c;
}
void or_ctrl_free(or_ctrl* c) { free(c); }
int or_ctrl_can_pass(or_ctrl* c, int64_t now, double pass_qps, double prev_qps, int32_t cur_thread, int32_t acquire,
                     int64_t* wait_ms) {
    if (wait_ms) *wait_ms = 0;
    switch (c->behavior) {
    case SG_CONTROL_BEHAVIOR_WARM_UP: {
        int64_t pq = j_d2l(pass_qps), prev = j_d2l(prev_qps);
        warm_sync(c, now, prev);
        int64_t rest = c->stored;
        if (rest >= c->warning_token) return (double)(pq + acquire) <= warm_qps(c, rest);
        return (double)(pq + acquire) <= c->count;
    }
    case SG_CONTROL_BEHAVIOR_RATE_LIMITER: {
        if (acquire <= 0) return 1;
        if (c->count <= 0) return 0;
        int64_t cost = j_round(1.0 * acquire / c->count * 1000);
        return rl_admit(&c->latest, cost, now, c->max_queue, wait_ms);
    }
    case SG_CONTROL_BEHAVIOR_WARM_UP_RATE_LIMITER: {
        int64_t prev = j_d2l(prev_qps);
        warm_sync(c, now, prev);
        int64_t rest = c->stored, cost;
        if (rest >= c->warning_token) cost = j_round(1.0 * acquire / warm_qps(c, rest) * 1000);
        else cost = j_round(1.0 * acquire / c->count * 1000);
        return rl_admit(&c->latest, cost, now, c->max_queue, wait_ms);
    }
    default: {
        int32_t cur = c->grade == SG_FLOW_GRADE_THREAD ? cur_thread : j_d2i(pass_qps);
        return !((double)j_iadd(cur, acquire) > c->count);
    }
    }
}
int64_t or_ctrl_state(or_ctrl* c, int which) {
    switch (which) {
    case 0: return c->stored;
    case 1: return c->last_filled;
    case 2: return c->latest;
    case 3: return c->warning_token;
    case 4: return c->max_token;
    }
    return 0;
}
double or_ctrl_slope(or_ctrl* c) { return c->slope; }

struct or_degrade { odegrade d; };
or_degrade* or_degrade_new(int grade, double count, int time_window) {
    or_degrade* d = (or_degrade*)calloc(1, sizeof(or_degrade));
    d->d.r.grade = grade; d->d.r.count = count; d->d.r.time_window = time_window;
    return d;
}
void or_degrade_free(or_degrade* d) { free(d); }
int or_degrade_pass_check(or_degrade* d, int64_t now, double avg_rt, double exc_qps, double succ_qps, double total_qps,
                          double total_exc) {
    return degrade_check_values(&d->d, now, avg_rt, exc_qps, succ_qps, total_qps, total_exc);
}

struct or_leap { oleap a; };
or_leap* or_leap_new(int kind, int sample_count, int interval_ms) {
    or_leap* l = (or_leap*)calloc(1, sizeof(or_leap));
    leap_init(&l->a, kind, sample_count, interval_ms, 4900);
    return l;
}
void or_leap_free(or_leap* l) { if (l) { leap_free(&l->a); free(l); } }
int or_leap_current(or_leap* l, int64_t t, int64_t* ws) {
    obucket* b = leap_current(&l->a, t);
    if (!b) return -1;
    if (ws) *ws = b->ws;
    return leap_slot_of(&l->a, b);
}
int or_leap_add(or_leap* l, int64_t t, int ev, int64_t v) {
    obucket* b = leap_current(&l->a, t);
    if (!b) return -1;
    if (ev == EV_RT) { b->c[EV_RT] += v; if (v < b->min_rt) b->min_rt = v; }
    else b->c[ev] += v;
    return leap_slot_of(&l->a, b);
}
int64_t or_leap_get(or_leap* l, int slot, int ev) {
    if (slot == -2) return l->a.scratch.c[ev];
    if (slot < 0 || slot >= l->a.n) return 0;
    return l->a.b[slot].c[ev];
}
int or_leap_values_count(or_leap* l, int64_t t) {
    int k = 0;
    for (int i = 0; i < l->a.n; ++i)
        if (l->a.b[i].present && !leap_deprecated(&l->a, t, &l->a.b[i])) k++;
    return k;
}
int64_t or_leap_values_sum(or_leap* l, int64_t t, int ev) { return leap_sum(&l->a, t, ev); }
int or_leap_previous(or_leap* l, int64_t t, int64_t* ws) {
    obucket* b = leap_previous(&l->a, t, t);
    if (!b) return -1;
    if (ws) *ws = b->ws;
    return leap_slot_of(&l->a, b);
}
int or_leap_valid_head(or_leap* l, int64_t t, int64_t* ws) {
    obucket* b = leap_valid_head(&l->a, t, t);
    if (!b) return -1;
    if (ws) *ws = b->ws;
    return leap_slot_of(&l->a, b);
}
void or_leap_add_waiting(or_leap* l, int64_t t, int64_t n) {
    if (!l->a.borrow) return;
    obucket* b = leap_current(l->a.borrow, t);
    if (b) b->c[EV_PASS] += n;
}
int64_t or_leap_current_waiting(or_leap* l, int64_t now) {
    if (!l->a.borrow) return 0;
    leap_current(l->a.borrow, now);
    return leap_sum(l->a.borrow, now, EV_PASS);
}

/* defaults shared with the engine's sg_config_default (restated here so the
 * oracle library has no dependency on the product library) */
#ifndef OR_NO_CONFIG_DEFAULT
void sg_config_default(sg_config* c) {
    memset(c, 0, sizeof(*c));
    c->sample_count = 2;
    c->interval_ms = 1000;
    c->statistic_max_rt = 4900;
    c->cold_factor = 3;
    c->occupy_timeout_ms = 500;
    c->max_slot_chain_size = 6000;
    c->switch_on = 1;
    c->device = 0;
    c->max_resources = 1u << 20;
    c->max_rules = 1u << 21;
    c->param_table_log2 = 22;
    c->status_ring_log2 = 28;
    c->max_batch_events = 1u << 25;
    c->cluster_sample_count = 10;
    c->cluster_interval_ms = 1000;
    c->cluster_exceed_count = 1.0;
    c->cluster_max_occupy_ratio = 1.0;
    c->cluster_max_allowed_qps = 30000;
    c->aux_node_capacity = 65536;
}
#endif
