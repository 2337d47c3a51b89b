// engine.cpp -- host side of the MI355X decision engine: the C ABI of
// include/sentinel_gpu.h, the rule managers (validation, de-duplication,
// java.util.HashSet ordering, FlowRuleComparator sort) and the per-batch
// launch pipeline.  All decisions are taken by the HIP kernels in kernels.hip;
// nothing here evaluates a rule.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <set>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/sentinel_gpu.h"
#include "dev_types.h"
#include "pmap.h"  // (pm_buckets: sg_param_thread_count)

namespace sg {
// kernels.hip
hipError_t launch_rs_first(const sg_event* ev, uint64_t n, uint32_t max_res, uint64_t gbase, const uint8_t* ring,
                           uint64_t ring_mask, int32_t max_rt, SEv* rec_o, uint32_t* keys, uint32_t* vals,
                           uint32_t* ghist, uint32_t nblocks, uint32_t* bflags, int64_t* t0_out, uint32_t* prio,
                           uint64_t* key_ring, const uint32_t* comp, const sg_event_ext* ext, const sg_arg* args,
                           uint64_t n_args, uint32_t max_ctx, hipStream_t st);
// db = digit bits (8 or 10)
hipError_t launch_radix_hist(const uint32_t* keys, uint64_t n, int shift, uint32_t* ghist, uint32_t nblocks,
                             hipStream_t st);
hipError_t launch_radix_hist_n(const uint32_t* keys, uint64_t n, const uint32_t* ndev, int shift, uint32_t* ghist,
                               uint32_t nblocks, hipStream_t st);
hipError_t launch_radix_scatter_n(const uint32_t* kin, const uint32_t* vin, uint64_t n, const uint32_t* ndev, int shift,
                                  const uint32_t* goff, uint32_t nblocks, uint32_t* kout, uint32_t* vout, hipStream_t st);
hipError_t launch_radix_scatter_x(const uint32_t* kin, const uint32_t* vin, uint64_t n, const uint32_t* ndev,
                                  const uint32_t* tcnt, const uint32_t* dbase, int shift, const uint32_t* goff,
                                  uint32_t nblocks, uint32_t* kout, uint32_t* vout, uint32_t* pos_of, hipStream_t st);
hipError_t launch_grp_first(const sg_event* ev, uint64_t n, uint32_t max_res, uint64_t gbase, uint64_t ring_mask,
                            uint32_t* bflags, int64_t* t0_out, uint32_t* prio, uint64_t* key_ring, const uint32_t* comp,
                            const sg_event_ext* ext, const sg_arg* args, uint64_t n_args, uint32_t max_ctx,
                            const uint16_t* hot_tab, uint32_t nhot, uint32_t nblocks, uint32_t* words,
                            uint32_t* hot_hist, uint32_t* ckeys, uint32_t* cvals, uint32_t* ccnt, uint32_t* chist,
                            hipStream_t st);
hipError_t launch_hot_scan(uint32_t* C, uint32_t nblocks, uint32_t nhot, uint32_t* part, uint32_t* hb, uint32_t* total,
                           hipStream_t st);
hipError_t launch_grp_records(const sg_event* ev, uint64_t n, uint64_t gbase, uint64_t ring_mask, int32_t max_rt,
                              const uint32_t* words, const uint32_t* P, uint32_t nhot, uint32_t nblocks,
                              const uint32_t* hb, SEv* recs, uint32_t* svals, uint32_t* prev,
                              uint32_t* nprev, uint32_t* bst, uint32_t* bflags, const sg_event_ext* ext,
                              const sg_arg* args, uint32_t max_ctx, Link* link, uint32_t epoch, hipStream_t st);
hipError_t launch_hot_segs(const uint32_t* hb, uint32_t nhot, const uint32_t* hot_list, Seg* segs, uint32_t* out,
                           hipStream_t st);
hipError_t launch_hot_build(const Seg* segs, const uint32_t* mp, uint32_t mb, uint32_t min_len, uint32_t max_res, uint16_t* hot_tab,
                            uint32_t* hot_list, uint32_t nhot_old, uint32_t* hot_n, hipStream_t st);
hipError_t launch_cold_n(uint64_t n, const uint32_t* hot_total, uint32_t* out, hipStream_t st);
hipError_t launch_cold_small(const uint32_t* kin, const uint32_t* vin, const uint32_t* cnt, const uint32_t* dbase,
                             uint32_t* kout, uint32_t* vout, uint32_t* words, hipStream_t st);
uint32_t hot_max();
hipError_t launch_seg_cold(const uint32_t* keys, uint64_t n, const uint32_t* lo, const uint32_t* sbase, uint32_t* flag,
                           uint32_t* pos, Seg* segs, hipStream_t st,
                           hipError_t (*scan)(const uint32_t*, uint32_t*, uint64_t, uint32_t*, uint32_t*, hipStream_t),
                           uint32_t* part, uint32_t* ccount, uint32_t* nseg);
hipError_t launch_block_sums(const SEv* recs, uint64_t n, uint32_t* bst, Link* link, uint32_t epoch, uint32_t* bflags,
                             const uint32_t* skeys, const uint32_t* lo, hipStream_t st);
hipError_t launch_radix_scatter(const uint32_t* kin, const uint32_t* vin, uint64_t n, int shift, const uint32_t* goff,
                                uint32_t nblocks, uint32_t* kout, uint32_t* vout, uint32_t* pos_of, hipStream_t st);
uint32_t radix_tile();
hipError_t launch_scan(const uint32_t*, uint32_t*, uint64_t, uint32_t*, uint32_t*, hipStream_t);
hipError_t launch_snapshot(Bkt*, NodeInfo*, uint32_t, int64_t, int32_t, uint32_t*, uint32_t*, uint32_t*, uint32_t*,
                           sg_metric_node*, uint64_t, hipStream_t);
hipError_t launch_init_state(Bkt* sec, Bkt* minb, NodeInfo* info, int64_t* borrow, uint32_t nres, hipStream_t st);
hipError_t launch_set_flags(NodeInfo* info, const uint64_t* upd, uint32_t n, hipStream_t st);
hipError_t launch_region_copy(const uint64_t* src, uint64_t* dst, const uint64_t* tri, uint32_t n, hipStream_t st);
// decide.hip
hipError_t launch_seg(const uint32_t* keys, uint64_t n, uint32_t* flag, uint32_t* pos, Seg* segs, hipStream_t st,
                      hipError_t (*scan)(const uint32_t*, uint32_t*, uint64_t, uint32_t*, uint32_t*, hipStream_t),
                      uint32_t* part, uint32_t* nseg);
hipError_t launch_seg_bin(Seg* segs, const uint32_t* mp, uint32_t mb, uint64_t n, const Prog* prog, const uint32_t* prio,
                          uint32_t lane_max, uint32_t j1_max, uint32_t j4_max, uint32_t force_lane, uint32_t* blkcnt,
                          uint32_t pq_ok, uint32_t pq_wide, uint32_t* aux, uint32_t* ashort, uint64_t* along,
                          uint64_t* amulti, uint32_t* mixc, uint32_t* mix, uint32_t mix_cap, uint32_t* mixlen,
                          uint32_t mix_wide, uint32_t head_min,
                          hipStream_t st);
// aux.hip
hipError_t launch_aux(const SEv* recs, const Seg* segs, const uint32_t* aux, const uint32_t* ashort,
                      const uint64_t* along, uint64_t* apiece, const uint64_t* amulti, const DevState& S, const DevCfg& cfg,
                      int64_t t0, const uint32_t* dec, AuxAcc* pool, uint32_t pool_cap, uint32_t* pool_n, uint64_t* meta,
                      uint32_t* bflags, hipStream_t st);
hipError_t launch_aux_cold(const SEv* recs, const Seg* segs, const uint32_t* aux, const uint32_t* ashort, const DevState& S,
                           const DevCfg& cfg, int64_t t0, const uint32_t* dec, uint32_t* bflags, hipStream_t st);
// param.hip
hipError_t launch_pq(int wide, const SEv* recs, const sg_event* ev, const uint32_t* vals, const Seg* segs,
                     const uint32_t* order, uint32_t m, const DevState& S, const DevCfg& cfg, int64_t t0, uint32_t* dec,
                     uint32_t* bflags, hipStream_t st);
hipError_t launch_pm_grow(const Seg* segs, const uint32_t* mp, uint32_t mb, const DevState& S, unsigned long long* pool_next,
                          uint64_t pool_nb, uint32_t* bflags, uint4* mv, uint32_t* nmv, uint32_t mcap, uint32_t epoch,
                          uint32_t nm, PBucket* b2, PData* d2, uint32_t* sz, uint32_t* off, uint32_t* part,
                          hipError_t (*scan)(const uint32_t*, uint32_t*, uint64_t, uint32_t*, uint32_t*, hipStream_t),
                          hipStream_t st);
hipError_t launch_pm_compact(PMap* pm, uint32_t n, const PBucket* ob, const PData* od, PBucket* nbk, PData* nd,
                             uint32_t* sz, uint32_t* off, uint32_t* part, unsigned long long* pool_next,
                             hipError_t (*scan)(const uint32_t*, uint32_t*, uint64_t, uint32_t*, uint32_t*, hipStream_t),
                             hipStream_t st);
hipError_t launch_pm_grow_ids(const uint32_t* ids, uint32_t n, const DevState& S, unsigned long long* pool_next,
                              uint64_t pool_nb, uint32_t* bflags, hipStream_t st);
hipError_t launch_pv_a(SEv* recs, const uint32_t* vals, Seg* segs, const uint32_t* list, uint32_t m,
                       const DevState& S, const DevCfg& cfg, uint32_t* dec, PvSeg* pv, PvBuf B, uint32_t cap,
                       uint32_t* tot, uint32_t* hist, uint32_t* part, hipStream_t st,
                       hipError_t (*radix_hist)(const uint32_t*, uint64_t, const uint32_t*, int, uint32_t*, uint32_t, hipStream_t),
                       hipError_t (*radix_scatter)(const uint32_t*, const uint32_t*, uint64_t, const uint32_t*, int,
                                                   const uint32_t*, uint32_t, uint32_t*, uint32_t*, hipStream_t),
                       hipError_t (*scan)(const uint32_t*, uint32_t*, uint64_t, uint32_t*, uint32_t*, hipStream_t),
                       uint32_t tile, uint32_t* rest, uint32_t grant_all);
hipError_t launch_pv_b(SEv* recs, Seg* segs, const uint32_t* list, uint32_t m, const DevState& S, int64_t t0,
                       uint32_t* dec, uint32_t* bflags, PvSeg* pv, PvBuf B, uint32_t cap, uint32_t* tot, uint32_t* part,
                       uint32_t jumps, hipStream_t st,
                       hipError_t (*scan)(const uint32_t*, uint32_t*, uint64_t, uint32_t*, uint32_t*, hipStream_t),
                       uint32_t* rest);
hipError_t launch_pvt(SEv* recs, const sg_event* ev, const uint32_t* vals, Seg* segs, const uint32_t* list, uint32_t m,
                      const DevState& S, const DevCfg& cfg, uint32_t* dec, uint32_t* bflags, PvSeg* pv, PvBuf B,
                      uint32_t cap, uint32_t* tot, uint32_t* hist, uint32_t* part, hipStream_t st,
                      hipError_t (*radix_hist)(const uint32_t*, uint64_t, const uint32_t*, int, uint32_t*, uint32_t, hipStream_t),
                      hipError_t (*radix_scatter)(const uint32_t*, const uint32_t*, uint64_t, const uint32_t*, int,
                                                      const uint32_t*, uint32_t, uint32_t*, uint32_t*, hipStream_t),
                      hipError_t (*scan)(const uint32_t*, uint32_t*, uint64_t, uint32_t*, uint32_t*, hipStream_t),
                      uint32_t tile, uint32_t* rest);
hipError_t launch_pq_mix(int post, SEv* recs, const sg_event* ev, const uint32_t* vals, const Seg* segs,
                         const uint32_t* list, uint32_t n_narrow, uint64_t wide_off, uint32_t n_wide, const DevState& S,
                         const DevCfg& cfg, int64_t t0, uint32_t* dec, uint32_t* bflags, hipStream_t st,
                         const uint32_t* rest, const uint32_t* rest_n);
hipError_t launch_seg_order(Seg* segs, const uint32_t* mp, uint32_t mb, const uint32_t* off, uint32_t* order,
                            uint32_t* bin_off, hipStream_t st);
hipError_t launch_gather(const SEv* rec_o, const uint32_t* vals, const uint32_t* skeys, uint64_t n,
                         const uint32_t* pos_of, SEv* recs, uint32_t* prev, uint32_t* nprev, Link* link, uint32_t* bst,
                         uint32_t epoch, uint32_t* bflags, hipStream_t st);
hipError_t launch_fill(const Span* spans, const uint32_t* nspan, uint32_t cap, const SEv* recs, const Prog* prog,
                       const DRule* rules, uint32_t* dec, hipStream_t st);
hipError_t launch_resolve(const uint32_t* prev, uint32_t np, const uint8_t* ring, SEv* recs, const uint32_t* vals,
                          const sg_event_ext* ext, hipStream_t st);
hipError_t launch_post_w(const uint32_t* words, const uint32_t* P, uint32_t nhot, const uint32_t* dec, uint64_t n,
                         uint64_t gbase, uint8_t* ring, uint64_t ring_mask, uint32_t* out, hipStream_t st);
hipError_t launch_post(const uint32_t* pos_of, const uint32_t* dec, uint64_t n, uint64_t gbase, uint8_t* ring,
                       uint64_t ring_mask, uint32_t* out, hipStream_t st);
hipError_t launch_chain(const SEv* recs, const uint32_t* vals, const Seg* segs, uint32_t m, NodeInfo* info,
                        uint32_t grant_all, uint32_t* ncand, uint64_t* cand, const sg_event* ev, const Prog* prog,
                        const sg_event_ext* ext, uint32_t max_ctx, hipStream_t st);
hipError_t launch_tiny(const sg_event* ev, uint32_t n, const DevState& S, const DevCfg& cfg, uint32_t max_res,
                       uint32_t* prio_w, const uint32_t* comp, uint64_t n_args, uint32_t grant_all,
                       unsigned long long* pool_next, uint64_t pool_nb, uint32_t epoch, SEv* recs, uint32_t* vals,
                       uint32_t* dec, Seg* segs, uint32_t* bflags, uint32_t* out, hipStream_t st);
uint32_t tiny_max();
hipError_t launch_decide_bin(int bin, const SEv* recs, const sg_event* ev, const uint32_t* vals, const Seg* segs,
                             const uint32_t* order, uint32_t m, const DevState& S, const DevCfg& cfg, int64_t t0,
                             uint32_t* dec, uint32_t* bflags, hipStream_t st);
// cluster.hip
hipError_t launch_tok_classify(const sg_token_req* req, uint64_t n, const CSlot* tab, uint32_t mask, uint32_t* fidx,
                               sg_token_result* res, uint32_t* flags, hipStream_t st);
hipError_t launch_tok_limiter_par(const sg_token_req* req, uint64_t n, const uint32_t* fidx, uint32_t nflows,
                                  NsLimiter* lim, double allowed, uint32_t* keys, uint32_t* vals, sg_token_result* res,
                                  uint32_t* bflag, uint32_t* cflag, uint32_t* bidx, uint32_t* cexcl, uint32_t* bstart,
                                  uint32_t* kpass, uint32_t* part, uint32_t* small,
                                  hipError_t (*scan)(const uint32_t*, uint32_t*, uint64_t, uint32_t*, uint32_t*, hipStream_t),
                                  hipStream_t st);
hipError_t launch_tok_limiter(const sg_token_req* req, uint64_t n, const uint32_t* fidx, uint32_t nflows,
                              NsLimiter* lim, double allowed, uint32_t* keys, uint32_t* vals, sg_token_result* res,
                              hipStream_t st);
hipError_t launch_tok_flow(const uint32_t* skeys, const uint32_t* svals, uint64_t n, const sg_token_req* req,
                           CFlow* flows, uint32_t nflows, CBkt* bkts, double exceed, double max_occ_ratio,
                           sg_token_result* res, uint32_t* bounds, uint32_t light, uint32_t wide, hipStream_t st,
                           hipStream_t hs, hipEvent_t fork, hipEvent_t join);
hipError_t launch_ptok_flow(const uint32_t* skeys, const uint32_t* svals, uint64_t n, const sg_param_token_req* req,
                            const uint64_t* values, PFlow* flows, uint32_t nflows, const PHot* hot, PVal* tab,
                            uint32_t mask, sg_token_result* res, uint32_t* flags, hipStream_t st);
} // namespace sg

using namespace sg;

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

#define HIPCHK(x)                                                                                        \
    do {                                                                                                 \
        hipError_t _e = (x);                                                                             \
        if (_e != hipSuccess) return fail(SG_EDEVICE, std::string(#x ": ") + hipGetErrorString(_e));    \
    } while (0)

// ----------------------------------------------------------------- Java helpers
int32_t j_string_hash(const char* s) {
    if (!s) return 0;
    uint32_t h = 0;
    const unsigned char* p = (const unsigned char*)s;
    while (*p) {
        uint32_t cp;
        if (*p < 0x80) cp = *p++;
        else if ((*p & 0xE0) == 0xC0 && p[1]) { cp = ((p[0] & 0x1Fu) << 6) | (p[1] & 0x3Fu); p += 2; }
        else if ((*p & 0xF0) == 0xE0 && p[1] && p[2]) { cp = ((p[0] & 0x0Fu) << 12) | ((p[1] & 0x3Fu) << 6) | (p[2] & 0x3Fu); p += 3; }
        else if (p[1] && p[2] && p[3]) { cp = ((p[0] & 0x07u) << 18) | ((p[1] & 0x3Fu) << 12) | ((p[2] & 0x3Fu) << 6) | (p[3] & 0x3Fu); p += 4; }
        else cp = *p++;
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
inline int32_t h31(int32_t h, int32_t v) { return (int32_t)(31u * (uint32_t)h + (uint32_t)v); }
int32_t j_double_hash(double d) {
    uint64_t u;
    std::memcpy(&u, &d, 8);
    if (d != d) u = 0x7ff8000000000000ULL;
    return (int32_t)(uint32_t)(u ^ (u >> 32));
}
uint64_t dbl_bits(double d) {
    uint64_t u;
    std::memcpy(&u, &d, 8);
    if (d != d) u = 0x7ff8000000000000ULL;
    return u;
}
int32_t long_hash(int64_t v) { return (int32_t)(uint32_t)((uint64_t)v ^ ((uint64_t)v >> 32)); }
bool blank(const char* s) {
    if (!s) return true;
    for (; *s; ++s)
        if (*s != ' ' && *s != '\t' && *s != '\n' && *s != '\r' && *s != '\f' && *s != '\v') return false;
    return true;
}
std::string sv(const char* s) { return s ? std::string(s) : std::string(); }
// AbstractRule.limitAppEquals normal form: null, "" and "default" are interchangeable
std::string la_norm(const char* s) { return (!s || !*s || std::strcmp(s, "default") == 0) ? "default" : std::string(s); }
int32_t abstract_hash(const char* res, const char* la) {
    int32_t h = res ? j_string_hash(res) : 0;
    if (!(la == nullptr || !*la || std::strcmp(la, "default") == 0)) h = h31(h, j_string_hash(la));
    return h;
}
int32_t cluster_hash(int64_t fid, int thr, int fb, int strat, int sc, int win, bool has_strat) {
    int32_t h = fid ? long_hash(fid) : 0;
    h = h31(h, thr);
    h = h31(h, fb ? 1 : 0);
    if (has_strat) h = h31(h, strat);
    h = h31(h, sc);
    h = h31(h, win);
    return h;
}

// java.util.HashSet iteration order of elements inserted in `order` (see oracle Q11 note):
// bucket index (h ^ h>>>16) & (cap-1) ascending, insertion order inside a bucket.
void hashset_order(const std::vector<int32_t>& hashes, std::vector<int>& order) {
    size_t n = order.size();
    if (n <= 1) return;
    int cap = 16;
    for (;;) {
        bool grown = false;
        std::vector<int> bin(cap, 0);
        size_t size = 0;
        for (size_t k = 0; k < n; ++k) {
            uint32_t h = (uint32_t)hashes[order[k]];
            h ^= h >> 16;
            int b = (int)(h & (uint32_t)(cap - 1));
            if (bin[b] >= 8 && cap < 64) { cap *= 2; grown = true; break; }
            bin[b]++;
            if (++size > (size_t)cap * 3 / 4 && k + 1 < n) { cap *= 2; grown = true; break; }
        }
        if (!grown) break;
    }
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) {
        uint32_t ha = (uint32_t)hashes[a], hb = (uint32_t)hashes[b];
        ha ^= ha >> 16; hb ^= hb >> 16;
        return (ha & (uint32_t)(cap - 1)) < (hb & (uint32_t)(cap - 1));
    });
}

// ---- param value keys (ParamFlowRuleUtil.parseItemValue typing, ParamFlowRuleUtil.java:85-121)
constexpr uint64_t KEY_MASK = 0x0FFFFFFFFFFFFFFFULL;
uint64_t fnv64(const char* s) {
    uint64_t h = 1469598103934665603ULL;
    for (; *s; ++s) { h ^= (unsigned char)*s; h *= 1099511628211ULL; }
    return h;
}
uint64_t mix64(uint64_t x) {
    x ^= x >> 30; x *= 0xbf58476d1ce4e5b9ULL;
    x ^= x >> 27; x *= 0x94d049bb133111ebULL;
    x ^= x >> 31; return x;
}
uint64_t tagged(uint64_t tag, uint64_t v) { return (tag << 60) | (v & KEY_MASK); }
bool ieq(const char* a, const char* b) {
    for (; *a && *b; ++a, ++b) if (std::tolower((unsigned char)*a) != std::tolower((unsigned char)*b)) return false;
    return *a == *b;
}
uint64_t param_key(const char* v, const char* t) {
    if (!v) return 0;
    auto is = [&](const char* a, const char* b) { return t && (!std::strcmp(t, a) || !std::strcmp(t, b)); };
    if (blank(t) || !std::strcmp(t, "java.lang.String") || !std::strcmp(t, "String")) return tagged(1, fnv64(v) & KEY_MASK);
    if (is("int", "java.lang.Integer")) return tagged(2, (uint32_t)(int32_t)std::strtol(v, nullptr, 10));
    if (is("long", "java.lang.Long")) {
        long long x = std::strtoll(v, nullptr, 10);
        if (x >= -(1LL << 59) && x < (1LL << 59)) return tagged(3, (uint64_t)x);
        return tagged(3, (fnv64(v) & KEY_MASK) | (1ULL << 59));
    }
    if (is("double", "java.lang.Double")) {
        double d = std::strtod(v, nullptr);
        uint64_t u;
        std::memcpy(&u, &d, 8);
        return tagged(4, mix64(u));
    }
    if (is("float", "java.lang.Float")) {
        float f = std::strtof(v, nullptr);
        uint32_t u;
        std::memcpy(&u, &f, 4);
        return tagged(5, u);
    }
    if (is("byte", "java.lang.Byte")) return tagged(6, (uint8_t)(int8_t)std::strtol(v, nullptr, 10));
    if (is("short", "java.lang.Short")) return tagged(7, (uint16_t)(int16_t)std::strtol(v, nullptr, 10));
    if (is("boolean", "java.lang.Boolean")) return tagged(8, ieq(v, "true") ? 1 : 0);
    if (!std::strcmp(t, "char")) return tagged(9, (unsigned char)v[0]);
    return tagged(1, fnv64(v) & KEY_MASK);
}

// ----------------------------------------------------------------- rule records
struct FlowR {
    sg_flow_rule r;
    std::string res, la, ref;
    int32_t hash;
    std::string eqkey;  // FlowRule.equals
};
struct DegR {
    sg_degrade_rule r;
    std::string res, la;
    int32_t hash;
    std::string eqkey;
};
struct ParamItemR {
    std::string obj, ct;
    bool has_obj, has_ct;
    int32_t count, has_count;
};
struct ParamR {
    sg_param_rule r;
    std::string res, la;
    std::vector<ParamItemR> items;
    std::vector<std::pair<uint64_t, int32_t>> hot;
    int32_t hash;
    std::string eqkey;
};

std::string flow_eqkey(const sg_flow_rule& r) {
    char buf[512];
    bool cc = r.cluster_mode || r.cluster_flow_id;
    std::snprintf(buf, sizeof(buf), "%d|%016llx|%d|%d|%d|%d|%d|", r.grade, (unsigned long long)dbl_bits(r.count),
                  r.strategy, r.control_behavior, r.warm_up_period_sec, r.max_queueing_time_ms, r.cluster_mode ? 1 : 0);
    std::string k = std::string(buf) + sv(r.resource) + "\x01" + la_norm(r.limit_app) + "\x01" +
                    (r.ref_resource ? "1" + std::string(r.ref_resource) : "0") + "\x01";
    if (cc) {
        std::snprintf(buf, sizeof(buf), "C%lld|%d|%d|%d|%d|%d", (long long)r.cluster_flow_id, r.cluster_threshold_type,
                      r.cluster_fallback_to_local ? 1 : 0, r.cluster_strategy, r.cluster_sample_count,
                      r.cluster_window_interval_ms);
        k += buf;
    }
    return k;
}
int32_t flow_hash(const sg_flow_rule& r) {
    int32_t h = abstract_hash(r.resource, r.limit_app && !blank(r.limit_app) ? r.limit_app : "default");
    h = h31(h, r.grade);
    h = h31(h, j_double_hash(r.count));
    h = h31(h, r.strategy);
    h = h31(h, r.ref_resource ? j_string_hash(r.ref_resource) : 0);
    h = h31(h, r.control_behavior);
    h = h31(h, r.warm_up_period_sec);
    h = h31(h, r.max_queueing_time_ms);
    h = h31(h, r.cluster_mode ? 1 : 0);
    int32_t ch = 0;
    if (r.cluster_mode || r.cluster_flow_id)
        ch = cluster_hash(r.cluster_flow_id, r.cluster_threshold_type, r.cluster_fallback_to_local, r.cluster_strategy,
                          r.cluster_sample_count, r.cluster_window_interval_ms, true);
    return h31(h, ch);
}
bool flow_valid(const sg_flow_rule& r) { // FlowRuleUtil.isValidRule (FlowRuleUtil.java:174-228)
    if (blank(r.resource) || !(r.count >= 0) || r.grade < 0 || r.strategy < 0 || r.control_behavior < 0) return false;
    if (r.cluster_mode) {
        if (r.cluster_flow_id <= 0) return false;
        if (!(r.cluster_sample_count > 0 && r.cluster_window_interval_ms > 0 &&
              r.cluster_window_interval_ms % r.cluster_sample_count == 0))
            return false;
        if (r.strategy != 0) return false;
    }
    if ((r.strategy == SG_STRATEGY_RELATE || r.strategy == SG_STRATEGY_CHAIN) && blank(r.ref_resource)) return false;
    switch (r.control_behavior) {
    case SG_CONTROL_BEHAVIOR_WARM_UP: return r.warm_up_period_sec > 0;
    case SG_CONTROL_BEHAVIOR_RATE_LIMITER: return r.max_queueing_time_ms > 0;
    case SG_CONTROL_BEHAVIOR_WARM_UP_RATE_LIMITER: return r.warm_up_period_sec > 0 && r.max_queueing_time_ms > 0;
    default: return true;
    }
}
std::string deg_eqkey(const sg_degrade_rule& r, int uniq) {
    char buf[256];
    // DegradeRule.equals compares count with != (NaN never equal): give NaN rules a unique key
    if (r.count != r.count) std::snprintf(buf, sizeof(buf), "NaN#%d|", uniq);
    else std::snprintf(buf, sizeof(buf), "%.17g|%d|%d|", r.count == 0 ? 0.0 : r.count, r.time_window, r.grade);
    return std::string(buf) + sv(r.resource) + "\x01" + la_norm(r.limit_app);
}
int32_t deg_hash(const sg_degrade_rule& r) {
    int32_t h = abstract_hash(r.resource, r.limit_app && !blank(r.limit_app) ? r.limit_app : "default");
    h = h31(h, j_double_hash(r.count));
    h = h31(h, r.time_window);
    return h31(h, r.grade);
}
bool param_valid(const sg_param_rule& r) { // ParamFlowRuleUtil.isValidRule (ParamFlowRuleUtil.java:32-55)
    if (blank(r.resource) || !(r.count >= 0) || r.grade < 0 || !r.has_param_idx || r.burst_count < 0 ||
        r.control_behavior < 0 || r.duration_in_sec <= 0 || r.max_queueing_time_ms < 0)
        return false;
    if (r.cluster_mode) {
        if (!(r.cluster_sample_count > 0 && r.cluster_window_interval_ms > 0 &&
              r.cluster_window_interval_ms % r.cluster_sample_count == 0))
            return false;
        if (r.cluster_flow_id <= 0) return false;
    }
    return true;
}
ParamR make_param(const sg_param_rule& s) {
    ParamR p;
    p.r = s;
    p.res = sv(s.resource);
    p.la = la_norm(s.limit_app);
    for (int i = 0; i < s.n_items; ++i) {
        const sg_param_item& it = s.items[i];
        ParamItemR q;
        q.has_obj = it.object != nullptr;
        q.obj = sv(it.object);
        q.has_ct = it.class_type != nullptr;
        q.ct = sv(it.class_type);
        q.count = it.count;
        q.has_count = it.has_count;
        p.items.push_back(q);
        // ParamFlowRuleUtil.parseHotItems (ParamFlowRuleUtil.java:62-83)
        if (!it.object || !it.has_count || it.count < 0) continue;
        uint64_t k = param_key(it.object, it.class_type);
        bool found = false;
        for (auto& h : p.hot) if (h.first == k) { h.second = it.count; found = true; }
        if (!found) p.hot.push_back({k, it.count});
    }
    // ParamFlowRule.hashCode (ParamFlowRule.java:218-234)
    int32_t h = abstract_hash(s.resource, s.limit_app && !blank(s.limit_app) ? s.limit_app : "default");
    h = h31(h, s.grade);
    h = h31(h, s.has_param_idx ? s.param_idx : 0);
    h = h31(h, j_double_hash(s.count));
    h = h31(h, s.control_behavior);
    h = h31(h, s.max_queueing_time_ms);
    h = h31(h, s.burst_count);
    h = h31(h, long_hash(s.duration_in_sec));
    int32_t lh = 1;
    for (auto& q : p.items) {
        int32_t e = q.has_obj ? j_string_hash(q.obj.c_str()) : 0;
        e = h31(e, q.has_count ? q.count : 0);
        e = h31(e, q.has_ct ? j_string_hash(q.ct.c_str()) : 0);
        lh = h31(lh, e);
    }
    h = h31(h, lh);
    h = h31(h, s.cluster_mode ? 1 : 0);
    int32_t ch = 0;
    if (s.cluster_mode || s.cluster_flow_id)
        ch = cluster_hash(s.cluster_flow_id, s.cluster_threshold_type, s.cluster_fallback_to_local, 0,
                          s.cluster_sample_count, s.cluster_window_interval_ms, false);
    p.hash = h31(h, ch);
    // ParamFlowRule.equals
    char buf[512];
    std::snprintf(buf, sizeof(buf), "%d|%016llx|%d|%d|%d|%lld|%d|%d:%d|", s.grade, (unsigned long long)dbl_bits(s.count),
                  s.control_behavior, s.max_queueing_time_ms, s.burst_count, (long long)s.duration_in_sec,
                  s.cluster_mode ? 1 : 0, s.has_param_idx, s.has_param_idx ? s.param_idx : 0);
    std::string k = std::string(buf) + p.res + "\x01" + p.la + "\x01";
    for (auto& q : p.items) {
        std::snprintf(buf, sizeof(buf), "[%d%d%d:%d]", q.has_obj, q.has_ct, q.has_count, q.has_count ? q.count : 0);
        k += buf + q.obj + "\x02" + q.ct + "\x03";
    }
    if (s.cluster_mode || s.cluster_flow_id) {
        std::snprintf(buf, sizeof(buf), "C%lld|%d|%d|%d|%d", (long long)s.cluster_flow_id, s.cluster_threshold_type,
                      s.cluster_fallback_to_local ? 1 : 0, s.cluster_sample_count, s.cluster_window_interval_ms);
        k += buf;
    }
    p.eqkey = k;
    return p;
}

template <class T> void dfree(T*& p) {
    if (p) (void)hipFree(p);
    p = nullptr;
}

} // namespace

// =====================================================================================
#define TMAP_KEY (1ull << 63)  // pmap_key of a thread-count map: TMAP_KEY | res << 8 | paramIdx
struct sg_engine {
    sg_config cfg;
    int device = 0;
    hipStream_t stream = nullptr;
    double last_ms[4] = {0, 0, 0, 0};

    // resources
    std::unordered_map<std::string, uint32_t> ids;
    std::vector<std::string> names;
    uint32_t n_chains = 0;

    // rule managers
    bool flow_loaded = false, deg_loaded = false, par_loaded = false;
    std::vector<std::string> last_flow, last_deg, last_par; // equality keys of the last loaded lists
    std::vector<FlowR> flows;
    std::vector<DegR> degs;
    std::vector<ParamR> params;
    std::vector<std::vector<int>> res_flow, res_deg, res_par; // compiled order per resource
    std::map<std::string, uint32_t> psid_of;                   // "res\x00eqkey" -> param state id
    uint32_t next_psid = 1;
    // ParameterMetric maps (dev_types.h PMap): one region per rule state (psid) and per (resource, paramIdx)
    // thread-count map, laid out in one slot pool rebuilt whenever the set of maps changes
    std::map<uint32_t, uint32_t> rmap_cap;                      // psid -> CacheMap capacity
    std::set<uint64_t> tmaps;                                   // res << 8 | paramIdx
    std::vector<uint64_t> pmap_key;                             // map index -> psid, or TMAP_KEY | res << 8 | idx
    std::unordered_map<uint32_t, uint32_t> pmap_index;         // psid -> map index
    std::vector<uint32_t> tm_base;                              // per resource: Prog.tm_base
    uint64_t n_pslot = 0;                                       // bucket slots in the pool (param_table_log2 bound)
    uint64_t pool_nb = 0;                                       // pool buckets (regions grow into it: k_pm_grow)
    unsigned long long* d_pool_next = nullptr;
    uint4* d_pmoves = nullptr;  // k_pm_grow's move list (one entry a map) + its count word at [pmoves_cap]
    PBucket* d_pbkt2 = nullptr;  // the other pool of the device compaction (compact_pmaps), and its values
    PData* d_pdat2 = nullptr;
    uint32_t* d_pcwork = nullptr;  // its scratch: sizes, offsets, scan partials (3 x pmoves_cap + 4096 words)
    uint64_t pmoves_cap = 0;                  // next free pool bucket
    unsigned long long* h_pool_next = nullptr;                  // pinned copy, refreshed by every batch (compaction)
    uint64_t n_compact = 0;                                     // pool compactions (diagnostics)
    uint64_t pool2_nb = 0;                                      // buckets of d_pbkt2 / d_pdat2 (= pool_nb once laid out)
    uint32_t n_dev_rules = 0;

    // device state
    Bkt* d_sec = nullptr;
    Bkt* d_minb = nullptr;
    NodeInfo* d_info = nullptr;
    Prog* d_prog = nullptr;
    DRule* d_rules = nullptr;
    RState* d_rstate = nullptr;
    DHot* d_hot = nullptr;
    PMap* d_pmap = nullptr;
    PBucket* d_pbkt = nullptr;
    PData* d_pdat = nullptr;
    uint64_t* d_pbm = nullptr;
    uint32_t* d_ppre = nullptr;
    uint32_t* d_tmid = nullptr;
    uint8_t* d_ring = nullptr;
    uint32_t rules_cap = 0, hot_cap = 0;

    // batch scratch: two slots, so that the group stage of batch k+1 (on gstream) runs while the
    // decide stage of batch k (on stream) is still in flight.  The d_* fields below alias the slot
    // being filled (activate()).
    struct BatchSlot {
        sg_event* d_ev = nullptr;
        uint32_t* d_out = nullptr;
        uint32_t *d_k0 = nullptr, *d_v0 = nullptr, *d_k1 = nullptr, *d_v1 = nullptr;
        uint32_t *d_hist = nullptr, *d_part = nullptr, *d_flag = nullptr, *d_pos = nullptr, *d_order = nullptr;
        uint32_t *d_posof = nullptr, *d_dec = nullptr, *d_blkcnt = nullptr, *d_prev = nullptr;
        SEv *d_recs = nullptr, *d_rec_o = nullptr;
        uint32_t* d_ccnt = nullptr;    // hot / cold group stage: per-tile cold counts, the cold segments' tile scratch
        bool radix = false;            // this batch took the radix group stage (d_posof), else the hot / cold one
        uint32_t nhot = 0;             // ... with these hot ids (its words and P in d_flag / d_pos)
        Seg* d_segs = nullptr;
        uint64_t* d_cand = nullptr;
        uint32_t* d_bsmall = nullptr;  // [0] bflags [1] nseg [2] ncand [3] nprev [4..5] t0 [8..8+N_BINS] bin offsets
                                       // [120] frozen spans recorded
        sg_event_ext* d_ext = nullptr; // sg_submit_ex host inputs staged in HBM
        sg_arg* d_args = nullptr;
        uint64_t ext_cap = 0, args_cap = 0;
        // sg_submit_ex: the aux.hip post-pass lists k_seg_bin builds (counts in d_bsmall[130..133])
        uint32_t* d_ashort = nullptr;
        uint64_t *d_apiece = nullptr, *d_amulti = nullptr, *d_along = nullptr;
        uint64_t aux_cap_n = 0;
        uint32_t* d_mix = nullptr;     // XF_MIX segments of the cooperative bins: [0, nmix0) narrow, [mix_cap, ..) wide
        uint64_t mix_cap = 0;
        Link* d_link = nullptr;        // frozen-stretch skipping side tables (DevState.link/bst/pend/spans)
        uint32_t *d_bst = nullptr, *d_pend = nullptr;
        Span* d_spans = nullptr;
        hipEvent_t ev[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};  // group start/end, decide start/end, post end
        bool pending = false;  // decide enqueued, not yet collected (timings, flags)
    } slot[2];
    int cur = 0;                 // slot of the next batch
    int last = -1;               // slot of the last batch submitted
    hipStream_t gstream = nullptr;
    std::vector<std::array<double, 4>> tlog;  // per batch [group, decide, post, total] ms, by collect()
    std::string fatal;           // non-empty: a batch left device state inconsistent; every later submit fails
    uint32_t* d_prio = nullptr;  // [res] sticky PM_* marks (DevState.prio)
    // hot / cold group stage (kernels.hip k_grp_*): [sort key] -> hot id of the next batch (0xFFFF: cold), the ids'
    // keys, and how many (the host learns it with the batch's head)
    uint16_t* d_hot_tab = nullptr;
    uint32_t* d_hot_list = nullptr;
    uint32_t nhot = 0;
    uint32_t* d_hot_part = nullptr;  // the hot scan's per-chunk partials ((max tiles / 64 + 2) x HOT_MAX words)
    uint32_t* d_hot_hb = nullptr;    // per hot id: first sorted position, total (2 x HOT_MAX words)
    bool radix_group = false;    // SG_DEBUG_FLAGS & 8192: the all-radix group stage (A/B)
    uint64_t radix_below = 1u << 18;  // SG_RADIX_BELOW: batches of fewer events take the radix group stage (the drop-in's
                                      // 65,536-event batches: 36 vs 30-32 M entries/s on the hot / cold one)
    uint32_t tok_light = 8192;   // SG_TOK_LIGHT: token flows of at most this many requests a call on one-wave workgroups
    uint32_t tok_wide = 1024;    // SG_TOK_WIDE: 1024 or 512 lanes for the other token flows (1024: 7.3 vs 8.0 ms a call)
    bool tiny_on = true;         // SG_TINY=0: synchronous batches of <= 256 events through the batched path too
    // sg_submit_ex: host-side ext / args are staged here (per batch slot, below); origin / context nodes
    AuxNode* d_auxtab = nullptr;
    uint32_t* d_auxcnt = nullptr;
    uint64_t aux_mask = 0;
    // the aux.hip post-pass: partial node results of the pieces of long segments (decide stage: one set)
    AuxAcc* d_auxpool = nullptr;
    uint64_t* d_auxmeta = nullptr;
    uint32_t auxpool_cap = 0;
    uint64_t auxmeta_cap = 0;
    // ContextUtil names: origins (0 = "") and contexts (0 = sentinel_default_context), first-intern order
    std::unordered_map<std::string, uint32_t> origin_ids, context_ids;
    std::unordered_map<std::string, int> rule_names;  // limitApp / CHAIN ref strings the flow rules name
    uint32_t* d_comp = nullptr;  // [res] STRATEGY_RELATE component representative (sort key); null: none
    uint32_t* d_prev = nullptr;
    uint32_t* d_bsmall = nullptr;
    Link* d_link = nullptr;
    uint32_t *d_bst = nullptr, *d_pend = nullptr;
    Span* d_spans = nullptr;
    uint32_t span_cap = 0;
    uint32_t epoch = 0;          // link tag of the batch being grouped
    uint64_t spans_total = 0;    // frozen span slots taken by the cooperative kernels (diagnostics)
    uint64_t cap_n = 0;
    sg_event* d_ev = nullptr;
    uint32_t* d_out = nullptr;
    uint32_t *d_k0 = nullptr, *d_v0 = nullptr, *d_k1 = nullptr, *d_v1 = nullptr;
    uint32_t *d_hist = nullptr, *d_part = nullptr, *d_flag = nullptr, *d_pos = nullptr, *d_order = nullptr;
    uint32_t *d_posof = nullptr, *d_dec = nullptr, *d_blkcnt = nullptr;
    SEv *d_recs = nullptr, *d_rec_o = nullptr;
    Seg* d_segs = nullptr;
    // d_small: [0] bflags [1] nseg [2] ncand [3] snapshot total [8..8+N_BINS) bin counts
    //          [64..64+N_BINS) bin cursors
    uint32_t* d_small = nullptr;
    uint32_t* d_sink = nullptr;  // 1024 words, DevState.sink
    int64_t* d_borrow = nullptr;  // [res][2]{ws, pass}: second-window borrow rings (prioritized entries)
    uint64_t* d_keyring = nullptr;  // ENTRY arg keys by global index (exit(count, args)); once param rules exist
    uint64_t* d_cand = nullptr;
    uint32_t dbg_flags = 0;
    int prof_bin = 0;            // SG_PROF_BIN: which cooperative bin (0 J16, 1 J4, 2 J1) fills the SG_DEBUG counters
    unsigned long long* d_dbg = nullptr;  // SG_DEBUG=1: [0..63] counters of the J16 bin
    uint64_t cap_hist = 0;
    uint64_t gbase = 0;
    // decide bins run concurrently: one stream per cooperative bin, the lane bins on the main stream
    // decide streams: J16 on bin_stream[0], J4 then J1 on bin_stream[1] (together shorter than J16), the
    // lane bins on stream; with gstream that is four streams for the four hardware queues a process
    // gets (GPU_MAX_HW_QUEUES): a fifth stream would share a queue and serialise behind another's kernels
    hipStream_t bin_stream[2] = {nullptr, nullptr};
    hipEvent_t fork = nullptr, join[2] = {nullptr, nullptr};
    hipEvent_t fork0 = nullptr;  // XF_MIX batches: the pre passes on bin_stream[1] start here, beside the lane bins
    hipEvent_t grown = nullptr;  // ... and their map-touching part after the maps' growth
    bool pipeline = true;   // the group stage of batch k+1 overlaps the decide stage of batch k (SG_PIPELINE=0: off)
    int j1_stream = -1;     // SG_J1_STREAM=1 / 0: J1 after J16 / J8 on bin_stream[0] / after the lane bins (default:
                            // bin_stream[0] when the short aux nodes take the main stream, else the main stream)
    uint32_t lane_max = 256, j1_max = 4096, j4_max = 65536;
    uint32_t head_min = 0;       // SG_HEAD_MIN: single-rule THREAD / rate-limiter head segments longer than this leave
                                 // the lane bins for the event-driven head owner (0: the lane bins keep up to lane_max;
                                 // C3 A/B: 64 -> 1.15, 128 -> 1.27, 0 -> 1.27 G entries/s)
    bool bins_pinned = false;  // SG_LANE_MAX / SG_J1_MAX / SG_J4_MAX set: no per-batch adaptation
    uint32_t skip_min = 32768;  // frozen stretches shorter than this (x NW/16) are streamed, not skipped
    bool pq_on = true;          // PF_PQ segments to k_pq (SG_PQ=0: the per-lane kernel, as before round 3)
    uint32_t pq_wide = 8192;    // PF_PQ segments longer than this get the 1024-lane k_pq
    bool mix_on = true;         // XF_MIX programs (SG_MIX=0: every param + flow / degrade resource one lane)
    bool mix_pq = false;        // SG_MIX_PQ=1: param-only programs of the XF_MIX shape decided as XF_MIX too
    bool pv_pq = true;          // SG_PV_PQ (default 1): XF_PVPQ programs' long segments through the value-parallel passes
    bool has_mix = false;       // some resource's program is XF_MIX (the batches keep the pre / post pass lists)
    bool has_head = false;      // some resource's program is XF_HEADT / XF_HEADR (head.hip k_head is launched)
    bool pv_on = true;          // SG_PV (default 1): the value-parallel pre pass (pvalue.hip) for the long XF_MIX segments
    PvBuf pvb{};                // its scratch: the pre pass's (launch_pv_a / _b) ...
    PvBuf pvbt{};               // ... and the post pass's (launch_pvt), so that the next batch's extraction and sort
                                // (launch_pv_a, early on bin_stream[1]) can run beside this batch's post pass
    bool has_multi = false;     // some STRATEGY_RELATE component exists (PX_MULTI): launch_pv_a waits for the grants
    uint64_t pv_cap = 0;
    PvSeg* d_pvseg = nullptr;
    PvSeg* d_pvtseg = nullptr;  // the post pass's (pvalue.hip launch_pvt)
    uint32_t* d_pvrest = nullptr;  // the wide segments the passes left to k_pq: pre [0, pvseg_cap], post after
    bool pvt_on = false;        // SG_PVT (default: SG_PV): the value-parallel post pass (thread-count maps)
    uint64_t pvseg_cap = 0;
    uint64_t pvch_cap = 0;      // pvalue.hip's extraction chunk arrays
    uint32_t *d_pvtot = nullptr, *d_pvhist = nullptr, *d_pvpart = nullptr, *d_pvthist = nullptr, *d_pvtpart = nullptr;
    uint32_t pv_last_m = 0;     // listed segments of the last batch that ran it (diagnostics)
    bool skip_pinned = false;   // SG_SKIP_MIN set: no per-batch adaptation
    // token server (cluster.hip): flowId table and ClusterMetric state in HBM, host mirror of the
    // configuration (ClusterFlowRuleManager.FLOW_RULES / ClusterMetricStatistics roles)
    std::vector<CFlow> cflows;                    // host copy of the config part (state lives on the device)
    std::unordered_map<int64_t, uint32_t> cmap;   // flowId -> flow index
    CFlow* d_cflow = nullptr;
    CBkt* d_cbkt = nullptr;
    CSlot* d_ctab = nullptr;
    uint32_t ctab_mask = 0;
    uint64_t ncbkt = 0;
    NsLimiter* d_nslim = nullptr;
    sg_token_req* d_treq = nullptr;
    sg_token_result* d_tres = nullptr;
    uint32_t* d_tfidx = nullptr;
    uint32_t* d_tbounds = nullptr;  // the flows' first sorted positions (nflows + 1 words)
    uint32_t tbounds_cap = 0;
    uint64_t tcap = 0;
    // cluster param flows (ClusterParamFlowRuleManager / ClusterParamMetricStatistics roles)
    std::vector<PFlow> pflows;                    // host copy of the config part
    std::unordered_map<int64_t, uint32_t> pmap;   // flowId -> param flow index
    PFlow* d_pflow = nullptr;
    PHot* d_phot = nullptr;
    CSlot* d_pftab = nullptr;
    uint32_t pftab_mask = 0;
    PVal* d_pvtab = nullptr;                      // (flow, value) counts, 2^PV_LOG2 slots
    uint32_t pv_mask = 0;
    sg_param_token_req* d_preq = nullptr;
    uint64_t* d_pvals = nullptr;
    uint64_t pcap = 0, pvcap = 0;
    // snapshot scratch
    uint32_t *d_snap_cnt = nullptr, *d_snap_off = nullptr;
    sg_metric_node* d_snap_out = nullptr;
    uint64_t snap_cap = 0;
};

namespace {

constexpr uint64_t SHARD_BATCH = 3ull << 21;  // batches of fewer events take the shard-sized bins and skip threshold

static void activate(sg_engine* e, int k) {
    auto& B = e->slot[k];
    e->d_ev = B.d_ev; e->d_out = B.d_out;
    e->d_k0 = B.d_k0; e->d_v0 = B.d_v0; e->d_k1 = B.d_k1; e->d_v1 = B.d_v1;
    e->d_hist = B.d_hist; e->d_part = B.d_part; e->d_flag = B.d_flag; e->d_pos = B.d_pos; e->d_order = B.d_order;
    e->d_posof = B.d_posof; e->d_dec = B.d_dec; e->d_blkcnt = B.d_blkcnt; e->d_prev = B.d_prev;
    e->d_recs = B.d_recs; e->d_rec_o = B.d_rec_o; e->d_segs = B.d_segs; e->d_cand = B.d_cand;
    e->d_bsmall = B.d_bsmall;
    e->d_link = B.d_link; e->d_bst = B.d_bst; e->d_pend = B.d_pend; e->d_spans = B.d_spans;
}
static void free_slot(sg_engine::BatchSlot& B) {
    dfree(B.d_ev); dfree(B.d_out); dfree(B.d_k0); dfree(B.d_v0); dfree(B.d_k1); dfree(B.d_v1);
    dfree(B.d_hist); dfree(B.d_part); dfree(B.d_flag); dfree(B.d_pos); dfree(B.d_order); dfree(B.d_segs);
    dfree(B.d_cand); dfree(B.d_posof); dfree(B.d_dec); dfree(B.d_recs); dfree(B.d_rec_o); dfree(B.d_blkcnt);
    dfree(B.d_prev); dfree(B.d_bsmall); dfree(B.d_ccnt);
    B.d_ccnt = nullptr;
    dfree(B.d_link); dfree(B.d_bst); dfree(B.d_pend); dfree(B.d_spans); dfree(B.d_ext); dfree(B.d_args);
    dfree(B.d_ashort); dfree(B.d_apiece); dfree(B.d_amulti); dfree(B.d_along); dfree(B.d_mix);
    B.d_mix = nullptr;
    B.ext_cap = B.args_cap = B.aux_cap_n = B.mix_cap = 0;
    B.d_link = nullptr; B.d_bst = B.d_pend = nullptr; B.d_spans = nullptr;
    B.d_ev = nullptr; B.d_out = nullptr; B.d_k0 = B.d_v0 = B.d_k1 = B.d_v1 = nullptr;
    B.d_hist = B.d_part = B.d_flag = B.d_pos = B.d_order = nullptr;
    B.d_posof = B.d_dec = B.d_blkcnt = B.d_prev = B.d_bsmall = nullptr;
    B.d_recs = B.d_rec_o = nullptr; B.d_segs = nullptr; B.d_cand = nullptr;
}
int ensure_batch(sg_engine* e, uint64_t n) {
    if (n <= e->cap_n) return SG_OK;
    uint64_t c = std::max<uint64_t>(n, 1u << 20);
    HIPCHK(hipStreamSynchronize(e->stream));  // no batch may use the old buffers
    uint64_t nblocks = (c + radix_tile() - 1) / radix_tile();
    e->cap_hist = nblocks * 256;  // 8-bit digit histograms
    for (auto& B : e->slot) {
        free_slot(B);
        HIPCHK(hipMalloc(&B.d_ev, c * sizeof(sg_event)));
        HIPCHK(hipMalloc(&B.d_out, c * 4));
        HIPCHK(hipMalloc(&B.d_k0, c * 4));
        HIPCHK(hipMalloc(&B.d_v0, c * 4));
        HIPCHK(hipMalloc(&B.d_k1, c * 4));
        HIPCHK(hipMalloc(&B.d_v1, c * 4));
        HIPCHK(hipMalloc(&B.d_hist, e->cap_hist * 4));
        HIPCHK(hipMalloc(&B.d_part, (e->cap_hist / 4096 + c / 4096 + 64) * 4));
        HIPCHK(hipMalloc(&B.d_flag, c * 4));
        HIPCHK(hipMalloc(&B.d_pos, c * 4));
        HIPCHK(hipMalloc(&B.d_order, c * 4));
        HIPCHK(hipMalloc(&B.d_segs, c * sizeof(Seg)));
        HIPCHK(hipMalloc(&B.d_cand, c * 8));
        HIPCHK(hipMalloc(&B.d_posof, c * 4));
        HIPCHK(hipMalloc(&B.d_dec, c * 4));
        HIPCHK(hipMalloc(&B.d_recs, c * sizeof(SEv)));
        // (radix stage only: every batch, or those below radix_below)
        const uint64_t co = (e->radix_group || c >= (1ull << 30)) ? c : std::min<uint64_t>(c, e->radix_below);
        if (co) HIPCHK(hipMalloc(&B.d_rec_o, co * sizeof(SEv)));
        HIPCHK(hipMalloc(&B.d_ccnt, 3 * (nblocks + 64) * 4));
    }
    dfree(e->d_hot_part);
    dfree(e->d_hot_hb);
    HIPCHK(hipMalloc(&e->d_hot_part, (nblocks / 16 + 2) * hot_max() * 4));  // (HS_TC >= 16 tiles a chunk)
    HIPCHK(hipMalloc(&e->d_hot_hb, 2 * hot_max() * 4));
    for (auto& B : e->slot) {
        HIPCHK(hipMalloc(&B.d_blkcnt, ((c + 255) / 256 + 1) * N_BINS * 4));
        HIPCHK(hipMalloc(&B.d_prev, c * 4));
        HIPCHK(hipMalloc(&B.d_bsmall, 256 * 4));
        HIPCHK(hipMemset(B.d_bsmall, 0, 256 * 4));
        HIPCHK(hipMalloc(&B.d_link, c * sizeof(Link)));
        HIPCHK(hipMemset(B.d_link, 0, c * sizeof(Link)));  // tag 0 is never a batch's epoch
        HIPCHK(hipMalloc(&B.d_bst, ((c + 1023) / 1024 + 1) * 4));
        HIPCHK(hipMalloc(&B.d_pend, c * 4));
        HIPCHK(hipMalloc(&B.d_spans, (c / SPAN_CHUNK + 65536) * sizeof(Span)));
    }
    e->span_cap = (uint32_t)(c / SPAN_CHUNK + 65536);
    e->cap_n = c;
    activate(e, e->cur);
    return SG_OK;
}

// The slot's batch: wait for its decide stage, record its stage times and check its device flags.
static int collect(sg_engine* e, int k) {
    auto& B = e->slot[k];
    if (!B.pending) return SG_OK;
    B.pending = false;
    HIPCHK(hipEventSynchronize(B.ev[4]));
    float g = 0, d = 0, p = 0;
    (void)hipEventElapsedTime(&g, B.ev[0], B.ev[1]);
    (void)hipEventElapsedTime(&d, B.ev[2], B.ev[3]);
    (void)hipEventElapsedTime(&p, B.ev[3], B.ev[4]);
    (void)hipGetLastError();
    e->last_ms[0] = g; e->last_ms[1] = d; e->last_ms[2] = p; e->last_ms[3] = (double)g + d + p;
    e->tlog.push_back({(double)g, (double)d, (double)p, (double)g + d + p});
    if (e->tlog.size() > 4096) e->tlog.erase(e->tlog.begin(), e->tlog.begin() + 2048);
    uint32_t bflags = 0;  // on gstream: a null-stream copy could share a queue with a decide kernel
    HIPCHK(hipMemcpyAsync(&bflags, B.d_bsmall, 4, hipMemcpyDeviceToHost, e->gstream));
    uint32_t nspan = 0;
    HIPCHK(hipMemcpyAsync(&nspan, B.d_bsmall + 120, 4, hipMemcpyDeviceToHost, e->gstream));
    HIPCHK(hipStreamSynchronize(e->gstream));
    e->spans_total += nspan;
    // Flags the decide kernels raise (the group stage's own checks return before the decide stage runs):
    // an EXIT/TRACE whose reference names an event that is not an earlier ENTRY of its resource, and a
    // batch starting before the last window a resource already holds (the clock went back).
    if (bflags & BF_BAD_REF)
        return fail(SG_EINVAL, "an EXIT/TRACE references an event that is not an earlier ENTRY of the same resource");
    if (bflags & BF_BACKWARD)
        return fail(SG_EINVAL, "event timestamps must be non-decreasing across batches (SURVEY Q3)");
    if (bflags & BF_AUX_FULL) return fail(SG_ECAPACITY, "origin/context node pool full (raise aux_node_capacity)");
    // A map that could not place a key has already committed its ring bit and live count (a ghost entry), and a
    // failed k_pq invariant leaves its maps in an unknown state: the engine refuses every later batch.
    if (bflags & BF_PQ_INVARIANT)
        e->fatal = "internal error: a k_pq tile's presorted key subset did not match its accesses";
    else if (bflags & BF_POOL_FULL)  // a map that could not grow may have lost a key (a ghost entry, as below)
        e->fatal = "the hot-parameter map pool is used up (raise param_table_log2)";
    else if (bflags & BF_PTAB_FULL)
        e->fatal = "a hot-parameter map table could not place a key (its map holds a ghost entry)";
    if (bflags & (BF_PQ_INVARIANT | BF_PTAB_FULL | BF_POOL_FULL)) return fail(SG_ECAPACITY, e->fatal + " -- engine unusable");
    return SG_OK;
}
// every batch in flight done (called by the API functions that read or write engine state)
static int drain(sg_engine* e) {
    int rc = SG_OK;
    for (int i = 0; i < 2; ++i) {  // oldest first
        int r = collect(e, (e->cur + i) & 1);
        if (r && !rc) rc = r;
    }
    HIPCHK(hipStreamSynchronize(e->stream));
    return rc;
}


// CacheMap capacity of a rule's time/token maps (ParameterMetric.initialize, ParameterMetric.java:87-104)
static uint32_t rule_map_cap(int64_t duration_sec) {
    const int64_t c = (int64_t)PM_BASE_CAP * std::max<int64_t>(duration_sec, 1);
    return (uint32_t)std::min<int64_t>(c, PM_TOTAL_CAP);
}

// Build the device rule program of every resource from the compiled host lists.
int upload_rules(sg_engine* e, bool reset_flow_state, bool reset_deg_state, bool reset_par_state) {
    uint32_t R = e->cfg.max_resources;
    std::vector<Prog> prog(R);
    std::vector<DRule> rules;
    std::vector<RState> rst;
    std::vector<DHot> hot;
    // previous rule states to carry over when a kind was not reloaded
    std::vector<RState> old_rst;
    std::vector<Prog> old_prog;
    if ((!reset_flow_state || !reset_deg_state || !reset_par_state) && e->n_dev_rules) {
        old_rst.resize(e->n_dev_rules);
        old_prog.resize(R);
        HIPCHK(hipMemcpy(old_rst.data(), e->d_rstate, e->n_dev_rules * sizeof(RState), hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(old_prog.data(), e->d_prog, R * sizeof(Prog), hipMemcpyDeviceToHost));
    }
    size_t nres = e->names.size();
    bool any_mix = false, any_head = false;
    std::vector<std::pair<uint32_t, uint32_t>> relate;  // (resource, referenced resource) of RELATE rules
    for (size_t r = 0; r < nres && r < R; ++r) {
        Prog p;
        std::memset(&p, 0, sizeof(p));
        p.rule_off = (uint32_t)rules.size();
        p.tm_base = r < e->tm_base.size() ? e->tm_base[r] : NO_ID;
        // param rules: HashSet order (ParamFlowSlot.checkFlow iterates them, ParamFlowSlot.java:84-100)
        const auto& pl = r < e->res_par.size() ? e->res_par[r] : std::vector<int>();
        for (size_t i = 0; i < pl.size(); ++i) {
            const ParamR& q = e->params[pl[i]];
            DRule d;
            std::memset(&d, 0, sizeof(d));
            d.kind = RK_PARAM;
            d.grade = (uint8_t)q.r.grade;
            d.behavior = (uint8_t)q.r.control_behavior;
            // cluster mode + QPS without fallback: passClusterCheck finds no TokenService in this process and
            // passes -- the rule's metric is still initialised (ParamFlowSlot.initHotParamMetricsFor)
            if (q.r.cluster_mode && q.r.grade == SG_FLOW_GRADE_QPS && !q.r.cluster_fallback_to_local) {
                d.behavior = PB_INIT_ONLY;
                // a run of such rules with fixed indices is one pseudo-rule: the set of maps it initialises
                if (q.r.param_idx >= 0 && p.n_param && rules.back().behavior == PB_INIT_ONLY &&
                    rules.back().param_idx >= 0) {
                    if (q.r.param_idx < SG_MAX_ARGS) rules.back().burst |= (int32_t)(1u << q.r.param_idx);
                    continue;
                }
            }
            d.slot = (uint8_t)i;
            d.max_queue = q.r.max_queueing_time_ms;
            d.count = q.r.count;
            d.burst = q.r.burst_count;
            if (d.behavior == PB_INIT_ONLY && q.r.param_idx >= 0)  // the pseudo-rule's map set
                d.burst = q.r.param_idx < SG_MAX_ARGS ? (int32_t)(1u << q.r.param_idx) : 0;
            double c = q.r.count;
            d.token_count = (c != c) ? 0 : c >= 2147483647.0 ? INT32_MAX : (int32_t)c;
            d.token_count_l = (c != c) ? 0 : c >= 9.2e18 ? INT64_MAX : (int64_t)c;
            d.duration_sec = q.r.duration_in_sec;
            d.hot_off = (uint32_t)hot.size();
            d.hot_n = (uint32_t)q.hot.size();
            for (auto& h : q.hot) hot.push_back(DHot{h.first, h.second, 0});
            d.pmap = e->pmap_index.at(e->psid_of.at(q.res + std::string("\0", 1) + q.eqkey));
            d.param_idx = q.r.param_idx;
            d.ref = NO_REF;
            rules.push_back(d);
            rst.push_back(RState{0, 0, 0, 0});  // a: paramIdx resolved by applyRealParamIdx + 1 (0 = not yet)
            p.n_param++;
        }
        // flow rules: FlowRuleComparator order; limitApp and strategy pick the node each rule checks
        // (FlowRuleChecker.selectNodeByRequesterAndStrategy, FlowRuleChecker.java:90-124)
        const auto& fl = r < e->res_flow.size() ? e->res_flow[r] : std::vector<int>();
        // FlowRuleManager.isOtherOrigin reads every rule of the resource, the cluster-only ones included
        std::vector<uint32_t> skipped_origins;
        for (size_t i = 0; i < fl.size(); ++i) {
            const FlowR& f = e->flows[fl[i]];
            if (!(f.r.cluster_mode && !f.r.cluster_fallback_to_local) || f.la == "default" || f.la == "other") continue;
            auto oi = e->origin_ids.find(f.la);
            if (oi != e->origin_ids.end()) skipped_origins.push_back(oi->second);
        }
        for (size_t i = 0; i < fl.size(); ++i) {
            const FlowR& f = e->flows[fl[i]];
            if (f.r.cluster_mode && !f.r.cluster_fallback_to_local) continue; // no TokenService -> pass
            DRule d;
            std::memset(&d, 0, sizeof(d));
            d.kind = RK_FLOW;
            d.grade = (uint8_t)f.r.grade;
            d.behavior = (uint8_t)(f.r.grade == SG_FLOW_GRADE_QPS ? f.r.control_behavior : SG_CONTROL_BEHAVIOR_DEFAULT);
            if (d.behavior > 3) d.behavior = SG_CONTROL_BEHAVIOR_DEFAULT;
            d.slot = (uint8_t)i;
            d.max_queue = f.r.max_queueing_time_ms;
            d.count = f.r.count;
            d.ref = NO_REF;
            d.la_kind = f.la == "default" ? LA_DEFAULT : f.la == "other" ? LA_OTHER : LA_ORIGIN;
            auto oi = e->origin_ids.find(f.la);
            d.la_origin = oi == e->origin_ids.end() ? NO_ID : oi->second;
            if (d.la_kind == LA_OTHER && !skipped_origins.empty()) {
                d.hot_off = (uint32_t)hot.size();
                d.hot_n = (uint32_t)skipped_origins.size();
                for (uint32_t o : skipped_origins) hot.push_back(DHot{o, 0, 0});
            }
            d.strategy = (uint32_t)f.r.strategy;
            d.chain_ctx = NO_ID;
            if (f.r.strategy == SG_STRATEGY_RELATE) {  // another resource's ClusterNode (same node if itself)
                auto it = e->ids.find(f.ref);
                const uint32_t b = it == e->ids.end() ? NO_REF : it->second;
                if (b != NO_REF && b != (uint32_t)r && b < R) { d.ref = b; relate.emplace_back((uint32_t)r, b); }
            } else if (f.r.strategy == SG_STRATEGY_CHAIN) {  // the DefaultNode of the context named refResource
                if (f.ref == "sentinel_default_context") d.chain_ctx = 0;
                else {
                    auto ci = e->context_ids.find(f.ref);
                    if (ci != e->context_ids.end()) d.chain_ctx = ci->second;
                }
                p.multi |= PX_CHAIN;
            }
            if (d.la_kind != LA_DEFAULT && f.r.strategy == SG_STRATEGY_DIRECT) p.multi |= PX_ORIGIN;
            if (d.la_kind != LA_DEFAULT || f.r.strategy == SG_STRATEGY_CHAIN || f.r.strategy > SG_STRATEGY_CHAIN)
                p.pflags |= PF_SERIAL;  // node selection beyond the ClusterNode: the per-lane kernel
            if (d.behavior == SG_CONTROL_BEHAVIOR_WARM_UP || d.behavior == SG_CONTROL_BEHAVIOR_WARM_UP_RATE_LIMITER) {
                // WarmUpController.construct (WarmUpController.java:100-117)
                int cold = e->cfg.cold_factor;
                double c = f.r.count;
                auto d2i = [](double v) -> int32_t {
                    if (v != v) return 0;
                    if (v >= 2147483647.0) return INT32_MAX;
                    if (v <= -2147483648.0) return INT32_MIN;
                    return (int32_t)v;
                };
                int32_t wt = d2i(f.r.warm_up_period_sec * c) / (cold - 1);
                int32_t mt = (int32_t)((uint32_t)wt + (uint32_t)d2i((double)(2 * f.r.warm_up_period_sec) * c / (1.0 + cold)));
                d.warning_token = wt;
                d.max_token = mt;
                d.slope = (cold - 1.0) / c / (double)(mt - wt);
                d.count_div_cold = d2i(c) / cold;
                p.pflags |= PF_WARM;
            }
            rules.push_back(d);
            rst.push_back(RState{0, 0, -1, 0});
            p.n_flow++;
        }
        const auto& dl = r < e->res_deg.size() ? e->res_deg[r] : std::vector<int>();
        for (size_t i = 0; i < dl.size(); ++i) {
            const DegR& g = e->degs[dl[i]];
            DRule d;
            std::memset(&d, 0, sizeof(d));
            d.kind = RK_DEGRADE;
            d.grade = (uint8_t)g.r.grade;
            d.slot = (uint8_t)i;
            d.count = g.r.count;
            d.time_window = g.r.time_window;
            if (g.r.grade == SG_DEGRADE_GRADE_EXCEPTION_COUNT) p.pflags |= PF_EXC_COUNT;
            if (g.r.grade == SG_DEGRADE_GRADE_RT) p.pflags |= PF_RT;
            rules.push_back(d);
            rst.push_back(RState{0, 0, 0, 0});
            p.n_degrade++;
        }
        if ((int)p.n_param + p.n_flow + p.n_degrade > 16)
            return fail(SG_ENOTSUP, "more than 16 rules on one resource: " + e->names[r]);
        {  // limits of the cooperative decide kernels (decide.hip JMAX_*); else one lane decides it
            int n_rl = 0;
            for (int i = 0; i < p.n_flow; ++i) {
                uint8_t b = rules[p.rule_off + p.n_param + i].behavior;
                if (b == SG_CONTROL_BEHAVIOR_RATE_LIMITER || b == SG_CONTROL_BEHAVIOR_WARM_UP_RATE_LIMITER) ++n_rl;
            }
            if (n_rl) p.pflags |= PF_RL;
            // param rules beside flow / degrade rules (XF_MIX): QPS DefaultController-style token buckets on
            // paramIdx 0 with LDS-sized maps only -- their verdicts are then a function of earlier checks of the
            // same (rule, value) alone (no THREAD grade: its count moves with full-chain passes; no throttle:
            // its wait would add to the flow stages')
            bool mix = p.n_param >= 1 && p.n_param <= 4 && ((p.n_flow + p.n_degrade) > 0 || e->mix_pq) && !p.multi;
            for (int i = 0; i < p.n_param && mix; ++i) {
                const DRule& d = rules[p.rule_off + i];
                if (d.param_idx < 0) mix = false;
                else if (d.behavior == PB_INIT_ONLY) { if (d.burst & ~1) mix = false; }
                else if (d.param_idx != 0 || d.grade != SG_FLOW_GRADE_QPS ||
                         d.behavior != SG_CONTROL_BEHAVIOR_DEFAULT || rule_map_cap(d.duration_sec) > PQ_MAX_CAP)
                    mix = false;
            }
            if (mix) {  // a thread-count map of another index is k_lane's
                auto it = e->tmaps.lower_bound(((uint64_t)r << 8) | 1);
                if (it != e->tmaps.end() && (*it >> 8) == (uint64_t)r) mix = false;
            }
            if (mix && e->mix_on) { p.xf |= XF_MIX; any_mix = true; }
            if ((p.xf & XF_MIX) && p.n_param == 1 && rules[p.rule_off].behavior != PB_INIT_ONLY) p.xf |= XF_PLITE;
            if ((p.n_param && !(p.xf & XF_MIX)) || p.n_flow > 4 || p.n_degrade > 4 || n_rl > 2 || p.multi)
                p.pflags |= PF_SERIAL;
            bool all_default_qps = true;
            for (int i = 0; i < p.n_flow; ++i) {
                const DRule& d = rules[p.rule_off + p.n_param + i];
                if (d.behavior != SG_CONTROL_BEHAVIOR_DEFAULT || d.grade != SG_FLOW_GRADE_QPS) all_default_qps = false;
            }
            if (all_default_qps) p.pflags |= PF_FROZEN;
            // k_pq (param.hip): param rules with a fixed paramIdx and LDS-sized rings, nothing else; QPS-grade
            // rules, and at most one THREAD-grade rule on paramIdx 0 checked last (its check and the entry's
            // thread-count increment are one access of the thread-count map)
            bool pq = p.n_param >= 1 && p.n_param <= 4 && p.n_flow == 0 && p.n_degrade == 0 && !p.multi;
            int last_checked = -1, n_thread = 0, thread_at = -1;
            for (int i = 0; i < p.n_param && pq; ++i) {
                const DRule& d = rules[p.rule_off + i];
                if (d.param_idx < 0) pq = false;
                else if (d.behavior == PB_INIT_ONLY) { if (d.burst & ~1) pq = false; }  // maps on other indices
                else if (d.param_idx != 0) pq = false;  // sg_submit_ex args beyond [0] are k_lane's
                else if (d.grade == SG_FLOW_GRADE_THREAD) { ++n_thread; thread_at = i; last_checked = i; }
                else if (d.grade != SG_FLOW_GRADE_QPS || rule_map_cap(d.duration_sec) > PQ_MAX_CAP) pq = false;
                else last_checked = i;
            }
            if (n_thread > 1 || (n_thread == 1 && thread_at != last_checked)) pq = false;
            if (n_thread) p.xf |= XF_PTHREAD;
            // a thread-count map of another index (an earlier rule set's, kept with the metric) is k_lane's too
            if (pq) {
                auto it = e->tmaps.lower_bound(((uint64_t)r << 8) | 1);
                if (it != e->tmaps.end() && (*it >> 8) == (uint64_t)r) pq = false;
            }
            if (pq && !(p.xf & XF_MIX)) p.pflags |= PF_PQ;
            // one checked QPS rule (DefaultController or throttle), no THREAD grade: the value-parallel passes
            if ((p.pflags & PF_PQ) && e->pv_pq && e->pv_on && p.n_param == 1 && n_thread == 0 &&
                rules[p.rule_off].behavior != PB_INIT_ONLY) {
                p.xf |= XF_PVPQ;
                any_mix = true;
            }
            if (p.n_flow <= 2 && p.n_degrade <= 2 && n_rl == 0) p.pflags |= PF_J16;
            // one flow rule and nothing else on the ClusterNode: a THREAD-grade DefaultController or a QPS
            // RateLimiter head is decided by the event-driven head owner (head.hip k_head)
            if (p.n_param == 0 && p.n_flow == 1 && p.n_degrade == 0 && !p.multi && !(p.pflags & PF_SERIAL)) {
                const DRule& d = rules[p.rule_off];
                if (d.strategy == SG_STRATEGY_DIRECT && d.la_kind == LA_DEFAULT) {
                    if (d.grade == SG_FLOW_GRADE_THREAD && d.behavior == SG_CONTROL_BEHAVIOR_DEFAULT) p.xf |= XF_HEADT;
                    else if (d.grade == SG_FLOW_GRADE_QPS && (d.behavior == SG_CONTROL_BEHAVIOR_RATE_LIMITER ||
                                                              (d.behavior == SG_CONTROL_BEHAVIOR_WARM_UP_RATE_LIMITER && d.count > 0)))
                        p.xf |= XF_HEADR;
                }
                if (p.xf & (XF_HEADT | XF_HEADR)) any_head = true;
            }
        }
        // carry controller / breaker state of kinds that were not reloaded
        if (!old_rst.empty()) {
            const Prog& op = old_prog[r];
            if (!reset_par_state && op.n_param == p.n_param)
                for (int i = 0; i < p.n_param; ++i) rst[p.rule_off + i] = old_rst[op.rule_off + i];
            if (!reset_flow_state && op.n_flow == p.n_flow)
                for (int i = 0; i < p.n_flow; ++i) rst[p.rule_off + p.n_param + i] = old_rst[op.rule_off + op.n_param + i];
            if (!reset_deg_state && op.n_degrade == p.n_degrade)
                for (int i = 0; i < p.n_degrade; ++i)
                    rst[p.rule_off + p.n_param + p.n_flow + i] = old_rst[op.rule_off + op.n_param + op.n_flow + i];
        }
        prog[r] = p;
    }
    // STRATEGY_RELATE components (co-locate the rule graph's connected components):
    // union-find over the references; every member sorts under the representative, one segment
    std::vector<uint32_t> comp;
    bool any_multi = false;
    if (!relate.empty()) {
        comp.resize(R);
        for (uint32_t x = 0; x < R; ++x) comp[x] = x;
        std::function<uint32_t(uint32_t)> find = [&](uint32_t x) { return comp[x] == x ? x : comp[x] = find(comp[x]); };
        for (auto& pr : relate) {
            uint32_t a = find(pr.first), b = find(pr.second);
            if (a != b) comp[std::max(a, b)] = std::min(a, b);
        }
        for (uint32_t x = 0; x < R; ++x) comp[x] = find(x);
        std::vector<uint32_t> members;
        for (uint32_t x = 0; x < R; ++x)
            if (comp[x] != x) { members.push_back(x); members.push_back(comp[x]); }
        std::sort(members.begin(), members.end());
        members.erase(std::unique(members.begin(), members.end()), members.end());
        for (uint32_t x : members) {
            if (comp[x] == x) { prog[x].multi |= PX_MULTI; prog[x].pflags |= PF_SERIAL; }
        }
        any_multi = !members.empty();
        // ClusterNode existence of the members from here on: NI_TOUCHED (a chain grant means an ENTRY of
        // the resource was decided in a finished batch: no batch is in flight during a rule load)
        std::vector<NodeInfo> ni(members.size());
        for (size_t k = 0; k < members.size(); ++k)
            HIPCHK(hipMemcpy(&ni[k], e->d_info + members[k], sizeof(NodeInfo), hipMemcpyDeviceToHost));
        for (size_t k = 0; k < members.size(); ++k) {
            if (ni[k].flags & NI_CHAIN) ni[k].flags |= NI_TOUCHED;
            HIPCHK(hipMemcpy(e->d_info + members[k], &ni[k], sizeof(NodeInfo), hipMemcpyHostToDevice));
        }
        // their param maps at full size: a member's events sort under the representative, so the per-segment
        // growth (k_pm_grow) never sees them
        if (e->d_pmap) {
            const std::set<uint32_t> ms(members.begin(), members.end());
            std::vector<uint32_t> ids;
            for (uint32_t i = 0; i < (uint32_t)e->pmap_key.size(); ++i)
                if ((e->pmap_key[i] & TMAP_KEY) && ms.count((uint32_t)(e->pmap_key[i] >> 8))) ids.push_back(i);
            for (const auto& kv : e->psid_of) {
                auto it = e->ids.find(kv.first.substr(0, kv.first.find('\0')));
                auto pi = e->pmap_index.find(kv.second);
                if (it != e->ids.end() && ms.count(it->second) && pi != e->pmap_index.end()) ids.push_back(pi->second);
            }
            if (!ids.empty()) {
                uint32_t* d_ids = nullptr;
                HIPCHK(hipMalloc(&d_ids, ids.size() * 4));
                HIPCHK(hipMemcpy(d_ids, ids.data(), ids.size() * 4, hipMemcpyHostToDevice));
                DevState Sg{};
                std::memset(&Sg, 0, sizeof(Sg));
                Sg.pmap = e->d_pmap; Sg.pbkt = e->d_pbkt; Sg.pdat = e->d_pdat; Sg.pbm = e->d_pbm;
                HIPCHK(hipMemset(e->d_small, 0, 4));
                HIPCHK(launch_pm_grow_ids(d_ids, (uint32_t)ids.size(), Sg, e->d_pool_next, e->pool_nb, e->d_small, e->stream));
                uint32_t fl = 0;
                HIPCHK(hipMemcpyAsync(&fl, e->d_small, 4, hipMemcpyDeviceToHost, e->stream));
                HIPCHK(hipStreamSynchronize(e->stream));
                (void)hipFree(d_ids);
                if (fl & (BF_POOL_FULL | BF_PTAB_FULL))
                    return fail(SG_ECAPACITY, "hot-parameter map pool too small for the maps of STRATEGY_RELATE members "
                                              "(raise param_table_log2)");
            }
        }
    }
    if (rules.size() > e->cfg.max_rules) return fail(SG_ECAPACITY, "compiled rule table exceeds max_rules");
    if (rules.size() > e->rules_cap) {
        dfree(e->d_rules); dfree(e->d_rstate);
        e->rules_cap = (uint32_t)std::max<size_t>(rules.size(), 1024);
        HIPCHK(hipMalloc(&e->d_rules, e->rules_cap * sizeof(DRule)));
        HIPCHK(hipMalloc(&e->d_rstate, e->rules_cap * sizeof(RState)));
    }
    if (hot.size() > e->hot_cap) {
        dfree(e->d_hot);
        e->hot_cap = (uint32_t)std::max<size_t>(hot.size(), 1024);
        HIPCHK(hipMalloc(&e->d_hot, e->hot_cap * sizeof(DHot)));
    }
    HIPCHK(hipDeviceSynchronize());
    if (!rules.empty()) {
        HIPCHK(hipMemcpy(e->d_rules, rules.data(), rules.size() * sizeof(DRule), hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(e->d_rstate, rst.data(), rst.size() * sizeof(RState), hipMemcpyHostToDevice));
    }
    if (!hot.empty()) HIPCHK(hipMemcpy(e->d_hot, hot.data(), hot.size() * sizeof(DHot), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(e->d_prog, prog.data(), R * sizeof(Prog), hipMemcpyHostToDevice));
    e->n_dev_rules = (uint32_t)rules.size();
    e->has_mix = any_mix;
    e->has_head = any_head;
    e->has_multi = any_multi;
    if (comp.empty()) {
        dfree(e->d_comp);
        e->d_comp = nullptr;
    } else {
        if (!e->d_comp) HIPCHK(hipMalloc(&e->d_comp, (uint64_t)R * 4));
        HIPCHK(hipMemcpy(e->d_comp, comp.data(), (uint64_t)R * 4, hipMemcpyHostToDevice));
    }
    return SG_OK;
}

uint32_t intern(sg_engine* e, const std::string& name) {
    auto it = e->ids.find(name);
    if (it != e->ids.end()) return it->second;
    uint32_t id = (uint32_t)e->names.size();
    e->ids.emplace(name, id);
    e->names.push_back(name);
    return id;
}

template <class V> void resize_lists(sg_engine* e, V& v) {
    if (v.size() < e->names.size()) v.resize(e->names.size());
}

} // namespace

// =====================================================================================
extern "C" {

const char* sg_last_error(void) { return g_err.c_str(); }

void sg_config_default(sg_config* c) {
    std::memset(c, 0, sizeof(*c));
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
    c->param_table_log2 = 28;
    c->status_ring_log2 = 28;
    c->max_batch_events = 1u << 25;
    c->cluster_sample_count = 10;
    c->cluster_interval_ms = 1000;
    c->cluster_exceed_count = 1.0;
    c->cluster_max_occupy_ratio = 1.0;
    c->cluster_max_allowed_qps = 30000;
    c->aux_node_capacity = 65536;
}

int sg_engine_create(const sg_config* cfg_in, sg_engine** out) {
    if (!out) return fail(SG_EINVAL, "out is null");
    sg_config cfg;
    if (cfg_in) cfg = *cfg_in;
    else sg_config_default(&cfg);
    if (cfg.sample_count != 2 || cfg.interval_ms != 1000)
        return fail(SG_ENOTSUP, "the device path implements SAMPLE_COUNT=2, INTERVAL=1000 (the reference defaults)");
    if (cfg.cold_factor <= 1) return fail(SG_EINVAL, "cold factor must be > 1");
    if (cfg.max_resources == 0 || cfg.param_table_log2 < 4 || cfg.param_table_log2 > 34 || cfg.status_ring_log2 < 10 ||
        cfg.status_ring_log2 > 36)
        return fail(SG_EINVAL, "bad capacity in sg_config");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(SG_EDEVICE, "no HIP device visible");
    if (cfg.device < 0 || cfg.device >= ndev) return fail(SG_EDEVICE, "device ordinal out of range");
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, cfg.device) != hipSuccess) return fail(SG_EDEVICE, "hipGetDeviceProperties failed");
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(SG_EDEVICE, std::string("this build targets gfx950, found ") + prop.gcnArchName);
    sg_engine* e = new sg_engine();
    e->cfg = cfg;
    e->device = cfg.device;
    auto bad = [&](int rc) { sg_engine_destroy(e); return rc; };
    if (hipSetDevice(e->device) != hipSuccess) return bad(fail(SG_EDEVICE, "hipSetDevice failed"));
    // The group stage (the critical path of the two-slot pipeline) gets the highest stream priority,
    // so that its short bandwidth-bound kernels are dispatched into the CUs the long decide kernels
    // free (C4: 4.53 -> 4.34 ms per batch).  SG_STREAM_PRIO=0: default priorities; =1: decide first.
    int prio_lo = 0, prio_hi = 0;
    const char* sp = std::getenv("SG_STREAM_PRIO");
    if (!(sp && sp[0] == '0')) (void)hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi);
    if (!(sp && sp[0] == '1')) std::swap(prio_lo, prio_hi);
    if (hipStreamCreateWithPriority(&e->stream, hipStreamNonBlocking, prio_hi) != hipSuccess) return bad(fail(SG_EDEVICE, "stream"));
    if (hipStreamCreateWithPriority(&e->gstream, hipStreamNonBlocking, prio_lo) != hipSuccess) {
        return bad(fail(SG_EDEVICE, "stream"));
    }
    for (auto& B : e->slot)
        for (auto& v : B.ev) if (hipEventCreate(&v) != hipSuccess) return bad(fail(SG_EDEVICE, "event"));
    uint64_t R = cfg.max_resources;
    if (hipMalloc(&e->d_sec, R * 2 * sizeof(Bkt)) != hipSuccess || hipMalloc(&e->d_minb, R * 60 * sizeof(Bkt)) != hipSuccess ||
        hipMalloc(&e->d_info, R * sizeof(NodeInfo)) != hipSuccess || hipMalloc(&e->d_prog, R * sizeof(Prog)) != hipSuccess ||
        hipMalloc(&e->d_ring, 1ull << cfg.status_ring_log2) != hipSuccess || hipMalloc(&e->d_small, 256 * 4) != hipSuccess ||
        hipMalloc(&e->d_sink, 1024 * 4) != hipSuccess || hipMalloc(&e->d_borrow, R * 4 * sizeof(int64_t)) != hipSuccess ||
        hipMalloc(&e->d_prio, R * 4) != hipSuccess || hipMalloc(&e->d_hot_tab, R * 2) != hipSuccess ||
        hipMalloc(&e->d_hot_list, hot_max() * 4) != hipSuccess)
        return bad(fail(SG_ENOMEM, "device allocation of the engine state failed"));
    {   // origin / context node table (open addressing, load <= 2/3 at capacity, power of two)
        const uint64_t cap = std::max<uint32_t>(cfg.aux_node_capacity, 16u);
        uint64_t slots = 32;
        while (2 * slots < 3 * cap) slots <<= 1;
        e->aux_mask = slots - 1;
        e->cfg.aux_node_capacity = (uint32_t)cap;
        if (hipMalloc(&e->d_auxtab, slots * sizeof(AuxNode)) != hipSuccess || hipMalloc(&e->d_auxcnt, 4) != hipSuccess ||
            hipMemsetAsync(e->d_auxtab, 0xFF, slots * sizeof(AuxNode), e->stream) != hipSuccess ||
            hipMemsetAsync(e->d_auxcnt, 0, 4, e->stream) != hipSuccess)
            return bad(fail(SG_ENOMEM, "device allocation of the origin/context node table failed"));
    }
    if (hipMemsetAsync(e->d_prog, 0, R * sizeof(Prog), e->stream) != hipSuccess ||
        hipMemsetAsync(e->d_ring, 0xFF, 1ull << cfg.status_ring_log2, e->stream) != hipSuccess ||
        hipMemsetAsync(e->d_prio, 0, R * 4, e->stream) != hipSuccess ||
        hipMemsetAsync(e->d_hot_tab, 0xFF, R * 2, e->stream) != hipSuccess ||
        launch_init_state(e->d_sec, e->d_minb, e->d_info, e->d_borrow, (uint32_t)R, e->stream) != hipSuccess ||
        hipStreamSynchronize(e->stream) != hipSuccess)
        return bad(fail(SG_EDEVICE, "device initialisation failed"));
    for (auto& s : e->bin_stream)
        if (hipStreamCreateWithPriority(&s, hipStreamNonBlocking, prio_hi) != hipSuccess) return bad(fail(SG_EDEVICE, "stream"));
    if (hipEventCreateWithFlags(&e->fork, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&e->fork0, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&e->grown, hipEventDisableTiming) != hipSuccess)
        return bad(fail(SG_EDEVICE, "event"));
    for (auto& v : e->join)
        if (hipEventCreateWithFlags(&v, hipEventDisableTiming) != hipSuccess) return bad(fail(SG_EDEVICE, "event"));
    if (const char* d = std::getenv("SG_DEBUG")) {
        if (d[0] == '1' && hipMalloc(&e->d_dbg, 64 * 8) == hipSuccess) (void)hipMemset(e->d_dbg, 0, 64 * 8);
    }
    if (const char* f = std::getenv("SG_DEBUG_FLAGS")) e->dbg_flags = (uint32_t)std::strtoul(f, nullptr, 0);
    e->radix_group = (e->dbg_flags & 8192) != 0;
    if (const char* f = std::getenv("SG_PROF_BIN")) e->prof_bin = std::atoi(f);  // SG_DEBUG counters of J16/J4/J1
    // decide-bin thresholds (segment lengths); tuning knobs, the defaults are the measured best
    if (const char* v = std::getenv("SG_LANE_MAX")) { e->lane_max = (uint32_t)std::strtoul(v, nullptr, 0); e->bins_pinned = true; }
    if (const char* v = std::getenv("SG_J1_MAX")) { e->j1_max = (uint32_t)std::strtoul(v, nullptr, 0); e->bins_pinned = true; }
    if (const char* v = std::getenv("SG_HEAD_MIN")) e->head_min = (uint32_t)std::strtoul(v, nullptr, 0);
    if (const char* v = std::getenv("SG_J4_MAX")) { e->j4_max = (uint32_t)std::strtoul(v, nullptr, 0); e->bins_pinned = true; }
    if (const char* v = std::getenv("SG_PIPELINE")) e->pipeline = v[0] == '1';
    if (const char* v = std::getenv("SG_TINY")) e->tiny_on = v[0] != '0';
    if (const char* v = std::getenv("SG_RADIX_BELOW")) e->radix_below = std::strtoull(v, nullptr, 0);
    if (const char* v = std::getenv("SG_TOK_WIDE")) e->tok_wide = std::atoi(v) == 512 ? 512u : 1024u;
    if (const char* v = std::getenv("SG_TOK_LIGHT")) e->tok_light = (uint32_t)std::strtoul(v, nullptr, 0);
    if (const char* v = std::getenv("SG_J1_STREAM")) e->j1_stream = std::atoi(v);
    if (const char* v = std::getenv("SG_PQ")) e->pq_on = v[0] != '0';
    if (const char* v = std::getenv("SG_MIX")) e->mix_on = v[0] != '0';
    if (const char* v = std::getenv("SG_MIX_PQ")) e->mix_pq = v[0] != '0';
    if (const char* v = std::getenv("SG_PV_PQ")) e->pv_pq = v[0] != '0';
    if (const char* v = std::getenv("SG_PV")) e->pv_on = v[0] != '0';
    e->pvt_on = e->pv_on;
    if (const char* v = std::getenv("SG_PVT")) e->pvt_on = v[0] != '0';
    if (const char* v = std::getenv("SG_PQ_WIDE")) e->pq_wide = (uint32_t)std::strtoul(v, nullptr, 0);
    if (const char* v = std::getenv("SG_SKIP_MIN")) {
        e->skip_min = std::max<uint32_t>(1u, (uint32_t)std::strtoul(v, nullptr, 0));
        e->skip_pinned = true;
    }
    *out = e;
    return SG_OK;
}

// diagnostics export (not part of the ABI): SG_DEBUG=1 counters of the cooperative J16 bin,
// accumulated over batches (see decide.hip k_jac)
// diagnostics export (not part of the ABI): stage times of the batches collected since the last call,
// 4 doubles each ([group, decide, post, total] ms); returns the number of batches written
extern "C" int sgx_timing_log(sg_engine* e, double* out, int cap) {
    if (!e || !out) return 0;
    (void)drain(e);
    int k = 0;
    for (; k < cap && k < (int)e->tlog.size(); ++k)
        for (int j = 0; j < 4; ++j) out[4 * k + j] = e->tlog[k][j];
    e->tlog.clear();
    return k;
}
// diagnostics export (not part of the ABI): frozen span slots recorded by the cooperative kernels so far
extern "C" unsigned long long sgx_spans_total(sg_engine* e) {
    if (!e) return 0;
    (void)drain(e);
    return e->spans_total;
}
// diagnostics export: zero the SG_DEBUG counters ([20] is a running minimum)
extern "C" int sgx_debug_reset(sg_engine* e) {
    if (!e || !e->d_dbg) return 0;
    (void)drain(e);
    unsigned long long z[64] = {0};
    z[20] = ~0ull;
    return hipMemcpy(e->d_dbg, z, sizeof(z), hipMemcpyHostToDevice) == hipSuccess ? 1 : 0;
}
extern "C" int sgx_debug_counters(sg_engine* e, unsigned long long* out, int cap) {
    if (!e || !e->d_dbg || !out) return 0;
    int k = cap < 64 ? cap : 64;
    if (hipDeviceSynchronize() != hipSuccess) return 0;
    if (hipMemcpy(out, e->d_dbg, (size_t)k * 8, hipMemcpyDeviceToHost) != hipSuccess) return 0;
    return k;
}

// diagnostics export (not part of the ABI; parity tests): an origin (kind 0) / context (kind 1) node of res.
// out[0..15] = second window buckets {ws, pass, block, exc, succ, rt, occ, minRt} x 2, out[16] = curThreadNum,
// out[17..20] = minute pass history {ws, pass} per second parity; returns 1, 0 if the node does not exist.
extern "C" int sgx_read_aux_node(sg_engine* e, uint32_t res, uint32_t kind, uint32_t id, long long* out) {
    if (!e || !out || drain(e) != SG_OK) return -1;
    const unsigned long long key = ((unsigned long long)res << 32) | ((unsigned long long)kind << 31) | (id & 0x7FFFFFFFu);
    uint64_t h = mix64(key) & e->aux_mask;
    for (uint64_t probe = 0; probe <= e->aux_mask; ++probe) {
        AuxNode a;
        if (hipMemcpy(&a, e->d_auxtab + h, sizeof(a), hipMemcpyDeviceToHost) != hipSuccess) return -1;
        if (a.key == AUX_EMPTY) return 0;
        if (a.key == key) {
            for (int p = 0; p < 2; ++p) {
                const Bkt& b = a.sec[p];
                const int64_t v[8] = {b.ws, b.pass, b.block, b.exc, b.succ, b.rt, b.occ, b.minrt};
                for (int k = 0; k < 8; ++k) out[8 * p + k] = v[k];
            }
            out[16] = a.thread;
            out[17] = a.mws[0]; out[18] = a.mpass[0]; out[19] = a.mws[1]; out[20] = a.mpass[1];
            return 1;
        }
        h = (h + 1) & e->aux_mask;
    }
    return 0;
}
// diagnostics export: the last batch's value-parallel passes (pvalue.hip), out = {pre pass: listed segments it decided,
// accesses, blocked stretches the walk jumped; post pass: segments eligible, ops, segments committed; the pre
// pass's longest walk (steps, when over 256)}
extern "C" int sgx_pv_last(sg_engine* e, unsigned long long* out) {
    if (!e || !out || drain(e) != SG_OK) return -1;
    out[0] = out[1] = out[2] = out[3] = out[4] = out[5] = out[6] = 0;
    if (!e->d_pvseg || !e->d_pvtot || !e->pv_last_m) return 0;
    std::vector<PvSeg> v(e->pv_last_m);
    uint32_t tot[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (hipMemcpy(v.data(), e->d_pvseg, v.size() * sizeof(PvSeg), hipMemcpyDeviceToHost) != hipSuccess) return -1;
    if (hipMemcpy(tot, e->d_pvtot, 32, hipMemcpyDeviceToHost) != hipSuccess) return -1;
    for (const auto& s : v) out[0] += s.ok ? 1 : 0;
    out[1] = tot[0];
    out[2] = tot[2];
    out[6] = tot[3];
    if (e->pvt_on && e->d_pvtseg) {
        if (hipMemcpy(v.data(), e->d_pvtseg, v.size() * sizeof(PvSeg), hipMemcpyDeviceToHost) != hipSuccess) return -1;
        for (const auto& s : v) out[3] += s.ok ? 1 : 0;
        out[4] = tot[4];
        out[5] = tot[7];
    }
    if (!e->pv_on) out[0] = out[1] = out[2] = out[6] = 0;
    return 0;
}
// diagnostics export: the param map pool, out = {pool buckets, buckets taken, taken at the last compaction,
// compactions between batches, compactions inside a batch (on the device)}
extern "C" int sgx_param_pool(sg_engine* e, unsigned long long* out) {
    if (!e || !out || drain(e) != SG_OK) return -1;
    unsigned long long ctl[PC_WORDS] = {0, 0, 0, 0};
    if (e->d_pool_next && hipMemcpy(ctl, e->d_pool_next, sizeof(ctl), hipMemcpyDeviceToHost) != hipSuccess) return -1;
    out[0] = e->pool_nb; out[1] = ctl[PC_NEXT]; out[2] = ctl[PC_FLOOR]; out[3] = e->n_compact; out[4] = ctl[PC_RESCUES];
    return 0;
}

static int compact_pmaps(sg_engine* e);
// diagnostics export: compact the param map pool now, between batches (tests run the compaction at full size)
extern "C" int sgx_param_compact(sg_engine* e) {
    if (!e || drain(e) != SG_OK) return -1;
    if (!e->pool_nb) return 0;
    if (compact_pmaps(e) != SG_OK) return -1;
    ++e->n_compact;
    return 0;
}

static void free_pv(sg_engine* e);

int sg_engine_destroy(sg_engine* e) {
    if (!e) return SG_OK;
    (void)hipSetDevice(e->device);
    if (e->stream) (void)hipStreamSynchronize(e->stream);
    if (e->gstream) (void)hipStreamSynchronize(e->gstream);
    dfree(e->d_sec); dfree(e->d_minb); dfree(e->d_info); dfree(e->d_prog); dfree(e->d_rules); dfree(e->d_rstate);
    dfree(e->d_hot); dfree(e->d_pmap); dfree(e->d_pbkt); dfree(e->d_pdat); dfree(e->d_pbm); dfree(e->d_ppre); dfree(e->d_tmid); dfree(e->d_ring); dfree(e->d_small); dfree(e->d_sink);
    dfree(e->d_pool_next); dfree(e->d_pmoves); dfree(e->d_pbkt2); dfree(e->d_pdat2); dfree(e->d_pcwork);
    if (e->h_pool_next) (void)hipHostFree(e->h_pool_next);
    free_pv(e);
    dfree(e->d_pvseg); dfree(e->d_pvtseg); dfree(e->d_pvtot); dfree(e->d_pvrest);
    if (e->gstream) (void)hipStreamSynchronize(e->gstream);
    for (auto& B : e->slot) free_slot(B);
    dfree(e->d_prio); dfree(e->d_hot_tab); dfree(e->d_hot_list); dfree(e->d_hot_part); dfree(e->d_hot_hb); dfree(e->d_comp); dfree(e->d_auxtab); dfree(e->d_auxpool); dfree(e->d_auxcnt); dfree(e->d_auxmeta);
    dfree(e->d_pflow); dfree(e->d_phot); dfree(e->d_pftab); dfree(e->d_pvtab); dfree(e->d_preq); dfree(e->d_pvals);
    dfree(e->d_cflow); dfree(e->d_cbkt); dfree(e->d_ctab); dfree(e->d_nslim); dfree(e->d_borrow); dfree(e->d_keyring);
    dfree(e->d_treq); dfree(e->d_tres); dfree(e->d_tfidx); dfree(e->d_tbounds);
    dfree(e->d_snap_cnt); dfree(e->d_snap_off); dfree(e->d_snap_out); dfree(e->d_dbg);
    for (auto& B : e->slot)
        for (auto& v : B.ev) if (v) (void)hipEventDestroy(v);
    if (e->gstream) (void)hipStreamDestroy(e->gstream);
    for (auto& v : e->join) if (v) (void)hipEventDestroy(v);
    if (e->fork) (void)hipEventDestroy(e->fork);
    if (e->fork0) (void)hipEventDestroy(e->fork0);
    if (e->grown) (void)hipEventDestroy(e->grown);
    for (auto& s : e->bin_stream) if (s) (void)hipStreamDestroy(s);
    if (e->stream) (void)hipStreamDestroy(e->stream);
    delete e;
    return SG_OK;
}

int sg_register_resources(sg_engine* e, const char* const* names, uint32_t n, uint32_t* out_ids) {
    if (!e || (n && !names)) return fail(SG_EINVAL, "null argument");
    if (int rc = drain(e)) return rc;
    for (uint32_t i = 0; i < n; ++i) {
        if (!names[i]) return fail(SG_EINVAL, "null resource name");
        auto it = e->ids.find(names[i]);
        uint32_t id;
        if (it != e->ids.end()) id = it->second;
        else {
            if (e->names.size() >= e->cfg.max_resources) return fail(SG_ECAPACITY, "max_resources reached");
            id = intern(e, names[i]);
        }
        if (out_ids) out_ids[i] = id;
    }
    return SG_OK;
}

int sg_resource_id(sg_engine* e, const char* name, uint32_t* out_id) {
    if (!e || !name || !out_id) return fail(SG_EINVAL, "null argument");
    auto it = e->ids.find(name);
    if (it == e->ids.end()) return fail(SG_ENOTFOUND, std::string("unknown resource ") + name);
    *out_id = it->second;
    return SG_OK;
}

int sg_param_key(sg_engine* e, const char* value, const char* class_type, uint64_t* out_key) {
    (void)e;
    if (!out_key) return fail(SG_EINVAL, "null out_key");
    *out_key = param_key(value, class_type);
    return SG_OK;
}

static int register_rule_resource(sg_engine* e, const char* name, uint32_t* id) {
    auto it = e->ids.find(name);
    if (it != e->ids.end()) { *id = it->second; return SG_OK; }
    if (e->names.size() >= e->cfg.max_resources) return fail(SG_ECAPACITY, "max_resources reached");
    *id = intern(e, name);
    return SG_OK;
}

// FlowRuleManager.loadRules -> FlowRuleUtil.buildFlowRuleMap (core/slots/block/flow/FlowRuleUtil.java:89-137)
// ClusterFlowRuleManager.applyClusterFlowRule (csrv/flow/rule/ClusterFlowRuleManager.java:323-363): the
// cluster-mode rules of the list, in list order, FlowRuleUtil.isValidRule; a later rule with the same
// flowId replaces an earlier one (ruleMap.put).  ClusterMetricStatistics.putMetricIfAbsent keeps the
// metric (and its window shape) of a flowId that stays; clearAndResetRulesConditional drops the rest.
static uint64_t tab_hash_h(int64_t k) {  // same mix as cluster.hip tab_hash
    uint64_t z = (uint64_t)k + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static int rebuild_cluster(sg_engine* e, const sg_flow_rule* rules, uint32_t n) {
    std::vector<int64_t> order;                       // flowIds in first-appearance order
    std::unordered_map<int64_t, const sg_flow_rule*> rule_of;
    for (uint32_t i = 0; i < n; ++i) {
        const sg_flow_rule& r = rules[i];
        if (!r.cluster_mode || !flow_valid(r)) continue;
        if (!rule_of.count(r.cluster_flow_id)) order.push_back(r.cluster_flow_id);
        rule_of[r.cluster_flow_id] = &r;
    }
    // current device state of the flows that stay
    const uint32_t nold = (uint32_t)e->cflows.size();
    std::vector<CFlow> old_f(nold);
    std::vector<CBkt> old_b(e->ncbkt);
    if (nold) HIPCHK(hipMemcpy(old_f.data(), e->d_cflow, nold * sizeof(CFlow), hipMemcpyDeviceToHost));
    if (e->ncbkt) HIPCHK(hipMemcpy(old_b.data(), e->d_cbkt, e->ncbkt * sizeof(CBkt), hipMemcpyDeviceToHost));
    std::vector<CFlow> nf;
    std::vector<CBkt> nb;
    std::unordered_map<int64_t, uint32_t> nmap;
    for (int64_t fid : order) {
        const sg_flow_rule& r = *rule_of[fid];
        CFlow f;
        std::memset(&f, 0, sizeof(f));
        auto it = e->cmap.find(fid);
        if (it != e->cmap.end()) {  // metric kept, rule replaced
            f = old_f[it->second];
            const uint32_t ob = f.boff;
            f.boff = (uint32_t)nb.size();
            for (int k = 0; k < f.n; ++k) nb.push_back(old_b[ob + k]);
        } else {
            f.flow_id = fid;
            f.n = r.cluster_sample_count;
            f.interval = r.cluster_window_interval_ms;
            f.boff = (uint32_t)nb.size();
            CBkt z;
            std::memset(&z, 0, sizeof(z));
            z.ws = -1;
            for (int k = 0; k < f.n; ++k) nb.push_back(z);
        }
        f.count = r.count;
        f.thr_type = r.cluster_threshold_type;
        nmap[fid] = (uint32_t)nf.size();
        nf.push_back(f);
    }
    uint32_t cap = 16;
    while (cap < 2 * nf.size() + 2) cap <<= 1;
    std::vector<CSlot> tab(cap);
    for (auto& t : tab) { t.key = 0; t.idx = 0xFFFFFFFFu; t.pad = 0; }
    for (uint32_t i = 0; i < nf.size(); ++i) {
        uint64_t h = tab_hash_h(nf[i].flow_id) & (cap - 1);
        while (tab[h].idx != 0xFFFFFFFFu) h = (h + 1) & (cap - 1);
        tab[h].key = nf[i].flow_id;
        tab[h].idx = i;
    }
    dfree(e->d_cflow); dfree(e->d_cbkt); dfree(e->d_ctab);
    e->d_cflow = nullptr; e->d_cbkt = nullptr; e->d_ctab = nullptr;
    if (!nf.empty()) {
        HIPCHK(hipMalloc(&e->d_cflow, nf.size() * sizeof(CFlow)));
        HIPCHK(hipMemcpy(e->d_cflow, nf.data(), nf.size() * sizeof(CFlow), hipMemcpyHostToDevice));
        HIPCHK(hipMalloc(&e->d_cbkt, nb.size() * sizeof(CBkt)));
        HIPCHK(hipMemcpy(e->d_cbkt, nb.data(), nb.size() * sizeof(CBkt), hipMemcpyHostToDevice));
    }
    HIPCHK(hipMalloc(&e->d_ctab, cap * sizeof(CSlot)));
    HIPCHK(hipMemcpy(e->d_ctab, tab.data(), cap * sizeof(CSlot), hipMemcpyHostToDevice));
    e->ctab_mask = cap - 1;
    e->cflows = std::move(nf);
    e->ncbkt = nb.size();
    e->cmap = std::move(nmap);
    return SG_OK;
}

int sg_load_flow_rules(sg_engine* e, const sg_flow_rule* rules, uint32_t n, uint32_t* n_loaded) {
    if (!e || (n && !rules)) return fail(SG_EINVAL, "null argument");
    if (int rc = drain(e)) return rc;  // no batch in flight while the rule tables change
    std::vector<std::string> keys(n);
    for (uint32_t i = 0; i < n; ++i) keys[i] = flow_eqkey(rules[i]);
    if (e->flow_loaded && keys == e->last_flow) { // DynamicSentinelProperty.updateValue: equal -> no-op
        if (n_loaded) *n_loaded = (uint32_t)e->flows.size();
        return SG_OK;
    }
    std::vector<FlowR> flows;
    std::vector<std::vector<int>> per;
    std::unordered_map<std::string, int> seen;
    for (uint32_t i = 0; i < n; ++i) {
        const sg_flow_rule& r = rules[i];
        if (!flow_valid(r)) continue;
        uint32_t rid;
        int rc = register_rule_resource(e, r.resource, &rid);
        if (rc) return rc;
        if (r.strategy == SG_STRATEGY_RELATE && r.ref_resource && *r.ref_resource) {  // its ClusterNode is read
            uint32_t ref;
            rc = register_rule_resource(e, r.ref_resource, &ref);
            if (rc) return rc;
        }
        std::string k = std::to_string(rid) + "#" + keys[i];
        if (seen.count(k)) continue; // HashSet.add of an equal rule
        seen[k] = 1;
        FlowR f;
        f.r = r;
        f.res = r.resource;
        f.la = la_norm(r.limit_app);
        f.ref = sv(r.ref_resource);
        f.hash = flow_hash(r);
        f.eqkey = keys[i];
        flows.push_back(f);
        if (per.size() <= rid) per.resize(rid + 1);
        per[rid].push_back((int)flows.size() - 1);
    }
    std::vector<int32_t> hs(flows.size());
    for (size_t i = 0; i < flows.size(); ++i) hs[i] = flows[i].hash;
    for (auto& l : per) {
        hashset_order(hs, l);
        // Collections.sort(rules, FlowRuleComparator) -- stable (FlowRuleComparator.java:30-55)
        std::stable_sort(l.begin(), l.end(), [&](int a, int b) {
            const FlowR &x = flows[a], &y = flows[b];
            auto cmp = [](const FlowR& o1, const FlowR& o2) {
                if (o1.r.cluster_mode && !o2.r.cluster_mode) return 1;
                if (!o1.r.cluster_mode && o2.r.cluster_mode) return -1;
                if (o1.la == o2.la) return 0;
                if (o1.la == "default") return 1;
                if (o2.la == "default") return -1;
                return 0;
            };
            return cmp(x, y) < 0;
        });
    }
    // publish
    auto old_flows = std::move(e->flows);
    auto old_per = std::move(e->res_flow);
    e->flows = std::move(flows);
    e->res_flow = std::move(per);
    resize_lists(e, e->res_flow);
    e->rule_names.clear();  // the origin / context names the flow rules read (sg_intern_* recompiles on first sight)
    for (auto& f : e->flows) {
        e->rule_names["o\x01" + f.la] = 1;
        if (f.r.strategy == SG_STRATEGY_CHAIN) e->rule_names["c\x01" + f.ref] = 1;
    }
    int rc = upload_rules(e, true, false, false);
    if (rc) { e->flows = std::move(old_flows); e->res_flow = std::move(old_per); return rc; }
    e->last_flow = keys;
    e->flow_loaded = true;
    rc = rebuild_cluster(e, rules, n);
    if (rc) return rc;
    if (n_loaded) *n_loaded = (uint32_t)e->flows.size();
    return SG_OK;
}

// DegradeRuleManager.loadRules (core/slots/block/degrade/DegradeRuleManager.java:112-205)
int sg_load_degrade_rules(sg_engine* e, const sg_degrade_rule* rules, uint32_t n, uint32_t* n_loaded) {
    if (!e || (n && !rules)) return fail(SG_EINVAL, "null argument");
    if (int rc = drain(e)) return rc;  // no batch in flight while the rule tables change
    std::vector<std::string> keys(n);
    for (uint32_t i = 0; i < n; ++i) keys[i] = deg_eqkey(rules[i], (int)i);
    bool has_nan = false;
    for (uint32_t i = 0; i < n; ++i) has_nan |= rules[i].count != rules[i].count;
    if (e->deg_loaded && !has_nan && keys == e->last_deg) {
        if (n_loaded) *n_loaded = (uint32_t)e->degs.size();
        return SG_OK;
    }
    std::vector<DegR> degs;
    std::vector<std::vector<int>> per;
    std::unordered_map<std::string, int> seen;
    for (uint32_t i = 0; i < n; ++i) {
        const sg_degrade_rule& r = rules[i];
        if (blank(r.resource) || !(r.count >= 0) || r.time_window <= 0) continue; // isValidRule
        uint32_t rid;
        int rc = register_rule_resource(e, r.resource, &rid);
        if (rc) return rc;
        std::string k = std::to_string(rid) + "#" + keys[i];
        if (seen.count(k)) continue;
        seen[k] = 1;
        DegR d;
        d.r = r;
        d.res = r.resource;
        d.la = la_norm(r.limit_app);
        d.hash = deg_hash(r);
        d.eqkey = keys[i];
        degs.push_back(d);
        if (per.size() <= rid) per.resize(rid + 1);
        per[rid].push_back((int)degs.size() - 1);
    }
    std::vector<int32_t> hs(degs.size());
    for (size_t i = 0; i < degs.size(); ++i) hs[i] = degs[i].hash;
    for (auto& l : per) hashset_order(hs, l);
    auto od = std::move(e->degs);
    auto op = std::move(e->res_deg);
    e->degs = std::move(degs);
    e->res_deg = std::move(per);
    resize_lists(e, e->res_deg);
    int rc = upload_rules(e, false, true, false);
    if (rc) { e->degs = std::move(od); e->res_deg = std::move(op); return rc; }
    e->last_deg = keys;
    e->deg_loaded = true;
    if (n_loaded) *n_loaded = (uint32_t)e->degs.size();
    return SG_OK;
}

// ParamFlowRuleManager.loadRules (param/slots/block/flow/param/ParamFlowRuleManager.java:103-166)
// ClusterParamFlowRuleManager.applyClusterParamRules (csrv/flow/rule/ClusterParamFlowRuleManager.java:318-369):
// cluster-mode rules passing ParamFlowRuleUtil.isValidRule, in list order; the last rule of a flowId wins;
// putMetricIfAbsent keeps the metric (window shape and value counts) of a flowId that stays; the metrics of
// the others are dropped (their value slots leave the table).
#define PV_LOG2 17
static int rebuild_cluster_param(sg_engine* e, const sg_param_rule* rules, const std::vector<ParamR>& all, uint32_t n) {
    std::vector<int64_t> order;
    std::unordered_map<int64_t, uint32_t> rule_of;
    for (uint32_t i = 0; i < n; ++i) {
        const sg_param_rule& r = rules[i];
        if (!r.cluster_mode || !param_valid(r)) continue;
        if (r.cluster_sample_count > CP_MAXN)
            return fail(SG_ENOTSUP, "cluster param rules with sampleCount > 16 are not on the device path");
        if (!rule_of.count(r.cluster_flow_id)) order.push_back(r.cluster_flow_id);
        rule_of[r.cluster_flow_id] = i;
    }
    const uint32_t nold = (uint32_t)e->pflows.size();
    std::vector<PFlow> old_f(nold);
    if (nold) HIPCHK(hipMemcpy(old_f.data(), e->d_pflow, nold * sizeof(PFlow), hipMemcpyDeviceToHost));
    std::vector<PFlow> nf;
    std::vector<PHot> nh;
    std::unordered_map<int64_t, uint32_t> nmap;
    std::vector<uint32_t> remap(nold, PV_EMPTY);  // old flow index -> new (value slots that stay)
    for (int64_t fid : order) {
        const uint32_t ri = rule_of[fid];
        const sg_param_rule& r = rules[ri];
        PFlow f;
        std::memset(&f, 0, sizeof(f));
        auto it = e->pmap.find(fid);
        if (it != e->pmap.end()) {
            f = old_f[it->second];
            remap[it->second] = (uint32_t)nf.size();
        } else {
            f.flow_id = fid;
            f.n = r.cluster_sample_count;
            f.interval = r.cluster_window_interval_ms;
            for (int k = 0; k < CP_MAXN; ++k) f.fws[k] = -1;
        }
        f.count = r.count;
        f.thr_type = r.cluster_threshold_type;
        f.hoff = (uint32_t)nh.size();
        f.nhot = (uint32_t)all[ri].hot.size();  // ParamFlowRuleUtil.fillExceptionFlowItems
        for (auto& h : all[ri].hot) { PHot x; x.key = h.first; x.count = h.second; x.pad = 0; nh.push_back(x); }
        nmap[fid] = (uint32_t)nf.size();
        nf.push_back(f);
    }
    const uint32_t cap_v = 1u << PV_LOG2;
    const bool need_v = !nf.empty() || e->d_pvtab;  // no table until a cluster param rule exists
    std::vector<PVal> vt(need_v ? cap_v : 0);
    if (!need_v) {}
    else if (e->d_pvtab) HIPCHK(hipMemcpy(vt.data(), e->d_pvtab, cap_v * sizeof(PVal), hipMemcpyDeviceToHost));
    else for (auto& v : vt) v.flow = PV_EMPTY;
    // re-insert the value slots of the flows that stay, under their new flow index (same probe as pv_find)
    std::vector<PVal> keep;
    for (auto& v : vt) if (v.flow != PV_EMPTY && v.flow < nold && remap[v.flow] != PV_EMPTY) { keep.push_back(v); keep.back().flow = remap[v.flow]; }
    for (auto& v : vt) { v.flow = PV_EMPTY; v.key = 0; }
    for (auto& v : keep) {
        uint64_t h = tab_hash_h((int64_t)(v.key ^ ((uint64_t)v.flow * 0xD6E8FEB86659FD93ull))) & (cap_v - 1);
        while (vt[h].flow != PV_EMPTY) h = (h + 1) & (cap_v - 1);
        vt[h] = v;
    }
    uint32_t cap = 16;
    while (cap < 2 * nf.size() + 2) cap <<= 1;
    std::vector<CSlot> tab(cap);
    for (auto& t : tab) { t.key = 0; t.idx = 0xFFFFFFFFu; t.pad = 0; }
    for (uint32_t i = 0; i < nf.size(); ++i) {
        uint64_t h = tab_hash_h(nf[i].flow_id) & (cap - 1);
        while (tab[h].idx != 0xFFFFFFFFu) h = (h + 1) & (cap - 1);
        tab[h].key = nf[i].flow_id;
        tab[h].idx = i;
    }
    dfree(e->d_pflow); dfree(e->d_phot); dfree(e->d_pftab);
    e->d_pflow = nullptr; e->d_phot = nullptr; e->d_pftab = nullptr;
    if (!nf.empty()) {
        HIPCHK(hipMalloc(&e->d_pflow, nf.size() * sizeof(PFlow)));
        HIPCHK(hipMemcpy(e->d_pflow, nf.data(), nf.size() * sizeof(PFlow), hipMemcpyHostToDevice));
    }
    if (!nh.empty()) {
        HIPCHK(hipMalloc(&e->d_phot, nh.size() * sizeof(PHot)));
        HIPCHK(hipMemcpy(e->d_phot, nh.data(), nh.size() * sizeof(PHot), hipMemcpyHostToDevice));
    }
    if (need_v) {
        if (!e->d_pvtab) HIPCHK(hipMalloc(&e->d_pvtab, cap_v * sizeof(PVal)));
        HIPCHK(hipMemcpy(e->d_pvtab, vt.data(), cap_v * sizeof(PVal), hipMemcpyHostToDevice));
        e->pv_mask = cap_v - 1;
    }
    HIPCHK(hipMalloc(&e->d_pftab, cap * sizeof(CSlot)));
    HIPCHK(hipMemcpy(e->d_pftab, tab.data(), cap * sizeof(CSlot), hipMemcpyHostToDevice));
    e->pftab_mask = cap - 1;
    e->pflows = std::move(nf);
    e->pmap = std::move(nmap);
    return SG_OK;
}

// ---- ParameterMetric maps (dev_types.h PMap)
// A map's cuckoo table: two-choice buckets of PM_BKT slots at <= 50 % load; its live-stamp ring: >= 4 x cap bits
static uint32_t ring_log2(uint32_t cap) {
    uint32_t k = 10;
    while ((1ull << k) < 4ull * cap + 64) ++k;
    return k;
}

// Lay out one region per map in a fresh pool, carrying the entries, stamps, rings and counters of the maps that
// stay (each at its current size; a new map starts at PM_MIN_NB buckets and grows per batch, k_pm_grow).  The pool
// holds 2^param_table_log2 slots, or less when that is more than the maps could ever take (twice their full
// regions: they grow by doubling).  Everything that can fail (the capacity check, the allocations) happens before
// the engine changes: an SG_ECAPACITY leaves the old maps in place.  Called with the current maps it compacts the
// pool (the regions the maps grew out of are dropped).
static int rebuild_pmaps(sg_engine* e, const std::map<uint32_t, uint32_t>& rcap, const std::set<uint64_t>& tmaps) {
    std::vector<PMap> old(e->pmap_key.size());
    if (!old.empty()) HIPCHK(hipMemcpy(old.data(), e->d_pmap, old.size() * sizeof(PMap), hipMemcpyDeviceToHost));
    std::unordered_map<uint64_t, uint32_t> was;
    for (uint32_t i = 0; i < (uint32_t)e->pmap_key.size(); ++i) was[e->pmap_key[i]] = i;
    std::vector<uint64_t> keys;
    std::vector<PMap> hdr;
    uint64_t nbkt = 0, nword = 0, nfull = 0;
    auto add = [&](uint64_t key, uint32_t cap) {
        PMap m;
        std::memset(&m, 0, sizeof(m));
        m.base = nbkt;
        auto it = was.find(key);
        m.nb = it == was.end() ? PM_MIN_NB : old[it->second].nb;
        m.cap = cap;
        m.rb_log2 = ring_log2(cap);
        m.bm = nword;
        keys.push_back(key);
        hdr.push_back(m);
        nbkt += m.nb;
        nfull += 2ull * map_buckets(cap);
        nword += (1ull << m.rb_log2) / 64;
    };
    for (const auto& kv : rcap) add(kv.first, kv.second);
    for (uint64_t t : tmaps) add(TMAP_KEY | t, PM_BASE_CAP);
    const uint64_t total = nbkt * PM_BKT;
    if (total > (1ull << e->cfg.param_table_log2))
        return fail(SG_ECAPACITY, "hot-parameter maps need " + std::to_string(total) + " slots, param_table_log2 = " +
                                      std::to_string(e->cfg.param_table_log2) + " allows " +
                                      std::to_string(1ull << e->cfg.param_table_log2));
    const uint64_t pool_nb = keys.empty() ? 0 : std::max<uint64_t>(nbkt, std::min<uint64_t>((1ull << e->cfg.param_table_log2) / PM_BKT, nfull + nbkt));
    std::vector<uint64_t> tri_b, tri_d, tri_w;  // {source word, destination word, words} per pool
    for (size_t i = 0; i < keys.size(); ++i) {
        auto it = was.find(keys[i]);
        if (it == was.end()) continue;
        const PMap& o = old[it->second];
        if (o.rb_log2 != hdr[i].rb_log2) continue;  // cannot happen: fixed by the map's identity
        hdr[i].clock = o.clock;
        hdr[i].thr = o.thr;
        hdr[i].live = o.live;
        const uint64_t bw = sizeof(PBucket) / 8, dw = PM_BKT * sizeof(PData) / 8;
        tri_b.insert(tri_b.end(), {o.base * bw, hdr[i].base * bw, (uint64_t)o.nb * bw});
        tri_d.insert(tri_d.end(), {o.base * dw, hdr[i].base * dw, (uint64_t)o.nb * dw});
        tri_w.insert(tri_w.end(), {o.bm, hdr[i].bm, (1ull << o.rb_log2) / 64});
    }
    std::vector<uint32_t> tb(e->names.size(), NO_ID), tmid;
    for (size_t i = 0; i < keys.size(); ++i) {
        if (!(keys[i] & TMAP_KEY)) continue;
        const uint32_t r = (uint32_t)(keys[i] >> 8), idx = (uint32_t)(keys[i] & 0xFF);
        if (r >= tb.size()) tb.resize(r + 1, NO_ID);
        if (tb[r] == NO_ID) { tb[r] = (uint32_t)tmid.size(); tmid.resize(tmid.size() + SG_MAX_ARGS, NO_ID); }
        tmid[tb[r] + idx] = (uint32_t)i;
    }
    PBucket* nbk = nullptr;
    PData* ndt = nullptr;
    uint64_t* nbm = nullptr;
    uint32_t* npr = nullptr;
    PMap* nh = nullptr;
    uint32_t* nt = nullptr;
    uint64_t* dtri = nullptr;
    // the compactions' second pool and scratch, allocated with the pool (a compaction that is needed later cannot
    // fail for memory: ADVICE r4)
    PBucket* nbk2 = nullptr;
    PData* ndt2 = nullptr;
    uint32_t* nwork = nullptr;
    const uint64_t mcap = std::max<uint64_t>(e->pmoves_cap, keys.size());
    auto release = [&]() {
        dfree(nbk); dfree(ndt); dfree(nbm); dfree(npr); dfree(nh); dfree(nt); dfree(dtri); dfree(nbk2); dfree(ndt2);
        dfree(nwork);
    };
    const size_t ntri = std::max(tri_b.size(), std::max(tri_d.size(), tri_w.size()));
    if ((nbkt && (hipMalloc(&nbk, pool_nb * sizeof(PBucket)) != hipSuccess ||
                  hipMalloc(&ndt, pool_nb * PM_BKT * sizeof(PData)) != hipSuccess ||
                  hipMalloc(&nbm, nword * 8) != hipSuccess || hipMalloc(&npr, nword * 4) != hipSuccess ||
                  hipMalloc(&nbk2, pool_nb * sizeof(PBucket)) != hipSuccess ||
                  hipMalloc(&ndt2, pool_nb * PM_BKT * sizeof(PData)) != hipSuccess ||
                  hipMalloc(&nwork, (3ull * mcap + 4096) * 4) != hipSuccess)) ||
        (!hdr.empty() && hipMalloc(&nh, hdr.size() * sizeof(PMap)) != hipSuccess) ||
        (!tmid.empty() && hipMalloc(&nt, tmid.size() * 4) != hipSuccess) ||
        (ntri && hipMalloc(&dtri, 3 * ntri * 8) != hipSuccess)) {
        release();
        (void)hipGetLastError();
        return fail(SG_ECAPACITY, "device memory for " + std::to_string(pool_nb * PM_BKT) +
                                      " hot-parameter map slots and their compaction copy (lower param_table_log2)");
    }
    if (!e->d_pool_next) {
        HIPCHK(hipMalloc(&e->d_pool_next, PC_WORDS * 8));
        HIPCHK(hipMemset(e->d_pool_next, 0, PC_WORDS * 8));
        HIPCHK(hipHostMalloc(&e->h_pool_next, PC_WORDS * 8));
        std::memset(e->h_pool_next, 0, PC_WORDS * 8);
    }
    if (nbkt) {
        HIPCHK(hipMemsetAsync(nbk, 0xFF, pool_nb * sizeof(PBucket), e->stream));  // PK_EMPTY keys (regions grow into it)
        HIPCHK(hipMemsetAsync(ndt, 0, total * sizeof(PData), e->stream));
        HIPCHK(hipMemsetAsync(nbm, 0, nword * 8, e->stream));
    }
    if (!hdr.empty()) HIPCHK(hipMemcpyAsync(nh, hdr.data(), hdr.size() * sizeof(PMap), hipMemcpyHostToDevice, e->stream));
    if (!tmid.empty()) HIPCHK(hipMemcpyAsync(nt, tmid.data(), tmid.size() * 4, hipMemcpyHostToDevice, e->stream));
    auto copy = [&](const std::vector<uint64_t>& tri, const void* src, void* dst) -> int {
        if (tri.empty()) return SG_OK;
        HIPCHK(hipMemcpyAsync(dtri, tri.data(), tri.size() * 8, hipMemcpyHostToDevice, e->stream));
        HIPCHK(launch_region_copy(reinterpret_cast<const uint64_t*>(src), reinterpret_cast<uint64_t*>(dst), dtri,
                                  (uint32_t)(tri.size() / 3), e->stream));
        HIPCHK(hipStreamSynchronize(e->stream));  // dtri is reused by the next pool
        return SG_OK;
    };
    if (int rc = copy(tri_b, e->d_pbkt, nbk)) { release(); return rc; }
    if (int rc = copy(tri_d, e->d_pdat, ndt)) { release(); return rc; }
    if (int rc = copy(tri_w, e->d_pbm, nbm)) { release(); return rc; }
    HIPCHK(hipStreamSynchronize(e->stream));
    dfree(dtri);
    dfree(e->d_pbkt); dfree(e->d_pdat); dfree(e->d_pbm); dfree(e->d_ppre); dfree(e->d_pmap); dfree(e->d_tmid);
    dfree(e->d_pbkt2); dfree(e->d_pdat2); dfree(e->d_pcwork);
    e->d_pbkt2 = nbk2;
    e->d_pdat2 = ndt2;
    e->d_pcwork = nwork;
    e->pool2_nb = nbkt ? pool_nb : 0;
    e->d_pbkt = nbk;
    e->d_pdat = ndt;
    e->d_pbm = nbm;
    e->d_ppre = npr;
    e->d_pmap = nh;
    e->d_tmid = nt;
    e->n_pslot = total;
    e->pool_nb = pool_nb;
    {
        const unsigned long long next[2] = {nbkt, nbkt};  // PC_NEXT, PC_FLOOR
        HIPCHK(hipMemcpy(e->d_pool_next, next, 16, hipMemcpyHostToDevice));
        e->h_pool_next[PC_NEXT] = e->h_pool_next[PC_FLOOR] = nbkt;
    }
    e->pmap_key = keys;
    e->pmap_index.clear();
    for (uint32_t i = 0; i < (uint32_t)keys.size(); ++i)
        if (!(keys[i] & TMAP_KEY)) e->pmap_index[(uint32_t)keys[i]] = i;
    e->tm_base = tb;
    e->rmap_cap = rcap;
    e->tmaps = tmaps;
    if (keys.size() > e->pmoves_cap) {  // (the stream is drained: rebuild_pmaps synchronised it above)
        dfree(e->d_pmoves);
        e->pmoves_cap = keys.size();
        HIPCHK(hipMalloc(&e->d_pmoves, (e->pmoves_cap + 1) * sizeof(uint4)));
    }
    return SG_OK;
}

// The second pool of the compactions and their scratch exist whenever the pool does: laid out with the maps
// (rebuild_pmaps), so a compaction never allocates
static int ensure_pool2(sg_engine* e) {
    if (!e->pool_nb || (e->pool2_nb == e->pool_nb && e->d_pcwork)) return SG_OK;
    return fail(SG_ESTATE, "the hot-parameter map pool has no compaction copy");
}

// The pool's compaction between batches (drained): on the device, every map's region back to back into the
// other pool (kept allocated: a host relayout of ~2M maps took a second), then the pools swap.  Without the memory
// for a second pool, the host relayout (rebuild_pmaps).
static int compact_pmaps(sg_engine* e) {
    const uint32_t nm = (uint32_t)e->pmap_key.size();
    if (!nm) return SG_OK;
    if (int rc = ensure_pool2(e)) return rc;
    hipStream_t st = e->stream;
    HIPCHK(hipMemsetAsync(e->d_pbkt2, 0xFF, e->pool_nb * sizeof(PBucket), st));  // PK_EMPTY: regions grow into it
    HIPCHK(launch_pm_compact(e->d_pmap, nm, e->d_pbkt, e->d_pdat, e->d_pbkt2, e->d_pdat2, e->d_pcwork,
                             e->d_pcwork + e->pmoves_cap, e->d_pcwork + 2 * e->pmoves_cap, e->d_pool_next, launch_scan, st));
    HIPCHK(hipMemcpyAsync(e->h_pool_next, e->d_pool_next, PC_WORDS * 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    std::swap(e->d_pbkt, e->d_pbkt2);
    std::swap(e->d_pdat, e->d_pdat2);
    return SG_OK;
}

int sg_load_param_rules(sg_engine* e, const sg_param_rule* rules, uint32_t n, uint32_t* n_loaded) {
    if (!e || (n && !rules)) return fail(SG_EINVAL, "null argument");
    if (int rc = drain(e)) return rc;  // no batch in flight while the rule tables change
    std::vector<ParamR> all;
    std::vector<std::string> keys;
    for (uint32_t i = 0; i < n; ++i) {
        if (rules[i].n_items > 0 && !rules[i].items) return fail(SG_EINVAL, "param rule items pointer is null");
        all.push_back(make_param(rules[i]));
        keys.push_back(all.back().eqkey);
    }
    // a negative paramIdx is rewritten in the loaded rule objects (ParamFlowSlot.applyRealParamIdx), so the
    // property's equality check never matches the list that created them: such a list always reloads
    bool neg = false;
    for (uint32_t i = 0; i < n; ++i) neg |= rules[i].has_param_idx && rules[i].param_idx < 0;
    if (e->par_loaded && keys == e->last_par && !neg) {
        if (n_loaded) *n_loaded = (uint32_t)e->params.size();
        return SG_OK;
    }
    std::vector<ParamR> ps;
    std::vector<std::vector<int>> per;
    std::unordered_map<std::string, int> seen;
    for (uint32_t i = 0; i < n; ++i) {
        if (!param_valid(rules[i])) continue;
        uint32_t rid;
        int rc = register_rule_resource(e, rules[i].resource, &rid);
        if (rc) return rc;
        std::string k = std::to_string(rid) + "#" + keys[i];
        if (seen.count(k)) continue;
        seen[k] = 1;
        ps.push_back(all[i]);
        if (per.size() <= rid) per.resize(rid + 1);
        per[rid].push_back((int)ps.size() - 1);
    }
    std::vector<int32_t> hs(ps.size());
    for (size_t i = 0; i < ps.size(); ++i) hs[i] = ps[i].hash;
    for (auto& l : per) hashset_order(hs, l);
    // ParameterMetric lifetime: resources that had rules and now have none lose their metric
    // (ParamFlowRuleManager.java:150-159); all metrics are cleared for an empty list.  Work on copies: the maps
    // are rebuilt (and may fail with SG_ECAPACITY) before anything of the engine changes.
    std::vector<bool> now_has(e->names.size(), false);
    for (size_t r = 0; r < per.size(); ++r) now_has[r] = !per[r].empty();
    auto psid_of = e->psid_of;
    auto rcap = e->rmap_cap;
    auto tmaps = e->tmaps;
    uint32_t next_psid = e->next_psid;
    std::vector<uint64_t> clear_flags;
    for (size_t r = 0; r < e->res_par.size(); ++r) {
        bool had = !e->res_par[r].empty();
        if ((had && !now_has[r]) || n == 0) {
            const std::string pre = e->names[r] + std::string("\0", 1);
            for (auto it = psid_of.begin(); it != psid_of.end();) {
                if (it->first.compare(0, pre.size(), pre) == 0) { rcap.erase(it->second); it = psid_of.erase(it); }
                else ++it;
            }
            tmaps.erase(tmaps.lower_bound((uint64_t)r << 8), tmaps.lower_bound((uint64_t)(r + 1) << 8));
            clear_flags.push_back(((uint64_t)(NI_PM | (((1u << SG_MAX_ARGS) - 1) << NI_TM_SHIFT)) << 32) | r);
        }
    }
    for (auto& q : ps) {
        std::string k = q.res + std::string("\0", 1) + q.eqkey;
        if (!psid_of.count(k)) {
            psid_of[k] = next_psid;
            rcap[next_psid++] = rule_map_cap(q.r.duration_in_sec);
        }
    }
    // thread-count maps: ParameterMetric.initialize makes one per paramIdx a rule of the resource resolves to
    // (a negative index resolves per call: any index); a map stays while the resource keeps a metric
    for (size_t r = 0; r < per.size(); ++r)
        for (int i : per[r]) {
            const int32_t idx = ps[i].r.param_idx;
            for (int32_t k = 0; k < SG_MAX_ARGS; ++k)
                if (idx < 0 || idx == k) tmaps.insert(((uint64_t)r << 8) | (uint64_t)k);
        }
    // the capacity check first: with SG_ECAPACITY neither the cluster rules nor the maps change
    uint64_t need = (rcap.size() + tmaps.size()) * (uint64_t)PM_MIN_NB * PM_BKT;  // (new maps' first regions)
    if (need > (1ull << e->cfg.param_table_log2))
        return fail(SG_ECAPACITY, "hot-parameter maps need " + std::to_string(need) + " slots, param_table_log2 = " +
                                      std::to_string(e->cfg.param_table_log2) + " allows " +
                                      std::to_string(1ull << e->cfg.param_table_log2));
    if (int rc = rebuild_cluster_param(e, rules, all, n)) return rc;
    if (int rc = rebuild_pmaps(e, rcap, tmaps)) return rc;
    e->psid_of = std::move(psid_of);
    e->next_psid = next_psid;
    auto op = std::move(e->params);
    auto opr = std::move(e->res_par);
    e->params = std::move(ps);
    e->res_par = std::move(per);
    resize_lists(e, e->res_par);
    int rc = upload_rules(e, false, false, true);
    if (rc) { e->params = std::move(op); e->res_par = std::move(opr); return rc; }
    if (!clear_flags.empty()) {
        uint64_t* d = nullptr;
        HIPCHK(hipMalloc(&d, clear_flags.size() * 8));
        HIPCHK(hipMemcpy(d, clear_flags.data(), clear_flags.size() * 8, hipMemcpyHostToDevice));
        HIPCHK(launch_set_flags(e->d_info, d, (uint32_t)clear_flags.size(), e->stream));
        HIPCHK(hipStreamSynchronize(e->stream));
        (void)hipFree(d);
    }
    e->last_par = keys;
    e->par_loaded = true;
    if (!e->params.empty() && !e->d_keyring) {  // thread counts can exist from now on: remember ENTRY keys
        const uint64_t nk = 1ull << e->cfg.status_ring_log2;
        HIPCHK(hipMalloc(&e->d_keyring, nk * sizeof(uint64_t)));
        HIPCHK(hipMemset(e->d_keyring, 0xFF, nk * sizeof(uint64_t)));  // NO_KEY
    }
    if (n_loaded) *n_loaded = (uint32_t)e->params.size();
    return SG_OK;
}

// pvalue.hip's scratch for up to cap accesses of up to m listed segments (the decide stage's: a batch in flight may
// still use the old arrays, so the stream drains first)
static void free_pvbuf(PvBuf& B) {
    dfree(B.key); dfree(B.pos); dfree(B.dt); dfree(B.acq); dfree(B.tc); dfree(B.seg); dfree(B.gid); dfree(B.idx);
    dfree(B.gid2); dfree(B.idx2); dfree(B.prev); dfree(B.w); dfree(B.sprev); dfree(B.sw); dfree(B.fslot); dfree(B.hit);
    dfree(B.keep); dfree(B.flast); dfree(B.ftok); dfree(B.htab); dfree(B.chunk); dfree(B.ccnt); dfree(B.cof);
    dfree(B.gdt); dfree(B.gaw); dfree(B.gpos); dfree(B.range);
    B = PvBuf{};
}
static void free_pv(sg_engine* e) {
    free_pvbuf(e->pvb);
    free_pvbuf(e->pvbt);
    dfree(e->d_pvhist); dfree(e->d_pvpart); dfree(e->d_pvthist); dfree(e->d_pvtpart);
    e->d_pvhist = e->d_pvpart = e->d_pvthist = e->d_pvtpart = nullptr;
    e->pv_cap = 0;
    e->pvch_cap = 0;
}
// every stream that may still read the scratch: the decide stream and the pre pass's
static hipError_t drain_decide(sg_engine* e) {
    hipError_t r = hipStreamSynchronize(e->stream);
    for (auto s : e->bin_stream)
        if (r == hipSuccess && s) r = hipStreamSynchronize(s);
    return r;
}
// (grown with headroom: a reallocation drains the stream, so it must stay rare)
static int ensure_pv(sg_engine* e, uint64_t cap, uint64_t m) {
    if (m > e->pvseg_cap) {
        HIPCHK(drain_decide(e));
        dfree(e->d_pvseg);
        dfree(e->d_pvtseg);
        e->pvseg_cap = std::max<uint64_t>(m + m / 2, 1024);
        HIPCHK(hipMalloc(&e->d_pvseg, e->pvseg_cap * sizeof(PvSeg)));
        HIPCHK(hipMalloc(&e->d_pvtseg, e->pvseg_cap * sizeof(PvSeg)));
        dfree(e->d_pvrest);
        HIPCHK(hipMalloc(&e->d_pvrest, 2 * (e->pvseg_cap + 1) * 4));
    }
    if (!e->d_pvtot) HIPCHK(hipMalloc(&e->d_pvtot, 64));
    if (cap > e->pv_cap) {
        HIPCHK(drain_decide(e));
        free_pv(e);
        const uint64_t c = std::max<uint64_t>(cap + cap / 4, 1u << 16);
        for (PvBuf* Bp : {&e->pvb, &e->pvbt}) {
            PvBuf& B = *Bp;
            HIPCHK(hipMalloc(&B.key, c * 8)); HIPCHK(hipMalloc(&B.pos, c * 4)); HIPCHK(hipMalloc(&B.dt, c * 4));
            HIPCHK(hipMalloc(&B.acq, c * 4)); HIPCHK(hipMalloc(&B.tc, c * 4)); HIPCHK(hipMalloc(&B.seg, c * 4));
            HIPCHK(hipMalloc(&B.gid, c * 4)); HIPCHK(hipMalloc(&B.idx, c * 4)); HIPCHK(hipMalloc(&B.gid2, c * 4));
            HIPCHK(hipMalloc(&B.idx2, c * 4)); HIPCHK(hipMalloc(&B.prev, c * 4)); HIPCHK(hipMalloc(&B.w, c * 4));
            HIPCHK(hipMalloc(&B.sprev, c * 4)); HIPCHK(hipMalloc(&B.sw, c * 4)); HIPCHK(hipMalloc(&B.fslot, c * 4));
            HIPCHK(hipMalloc(&B.hit, c)); HIPCHK(hipMalloc(&B.keep, c)); HIPCHK(hipMalloc(&B.flast, c * 8));
            HIPCHK(hipMalloc(&B.ftok, c * 4)); HIPCHK(hipMalloc(&B.htab, c * 16));
            HIPCHK(hipMalloc(&B.gdt, c * 4)); HIPCHK(hipMalloc(&B.gaw, c * 4)); HIPCHK(hipMalloc(&B.gpos, c * 4));
            HIPCHK(hipMalloc(&B.range, c * 16));
        }
        const uint64_t nblocks = (c + radix_tile() - 1) / radix_tile();
        HIPCHK(hipMalloc(&e->d_pvhist, nblocks * 256 * 4));
        HIPCHK(hipMalloc(&e->d_pvpart, nblocks * 256 * 4 + 4096));
        HIPCHK(hipMalloc(&e->d_pvthist, nblocks * 256 * 4));
        HIPCHK(hipMalloc(&e->d_pvtpart, nblocks * 256 * 4 + 4096));
        e->pv_cap = c;
    }
    // chunks: cap / PV_CH (4096) + one per segment (launch_pv's grid: pv_cap / 4096 + m + 1)
    const uint64_t nch = e->pv_cap / 4096 + m + 16;
    if (nch > e->pvch_cap) {
        HIPCHK(drain_decide(e));
        e->pvch_cap = nch + nch / 2;
        for (PvBuf* Bp : {&e->pvb, &e->pvbt}) {
            PvBuf& B = *Bp;
            dfree(B.chunk); dfree(B.ccnt); dfree(B.cof);
            HIPCHK(hipMalloc(&B.chunk, e->pvch_cap * 8)); HIPCHK(hipMalloc(&B.ccnt, e->pvch_cap * 4));
            HIPCHK(hipMalloc(&B.cof, e->pvch_cap * 4 + 4));
        }
    }
    return SG_OK;
}

// The XF_MIX segment lists of slot B for up to mb segments (narrow, then wide at mix_cap)
static int ensure_mix(sg_engine::BatchSlot& B, uint64_t mb) {
    if (mb > B.mix_cap) {
        dfree(B.d_mix);
        B.mix_cap = std::max<uint64_t>(mb, 1u << 12);
        HIPCHK(hipMalloc(&B.d_mix, B.mix_cap * 2 * 4));
    }
    return SG_OK;
}

// Lists of the aux.hip post-pass for a batch of n events in slot B, and the engine's partial pool.
#define AUXPOOL_CAP (1u << 20)
static int ensure_aux(sg_engine* e, sg_engine::BatchSlot& B, uint64_t n) {
    const uint64_t npiece = n / AUX_PIECE + n / 257 + 64;  // pieces: every long segment's, <= n/P + n/(AUX_SHORT + 1)
    if (n > B.aux_cap_n) {
        dfree(B.d_ashort); dfree(B.d_apiece); dfree(B.d_amulti); dfree(B.d_along);
        const uint64_t c = std::max<uint64_t>(n, 1u << 16);
        HIPCHK(hipMalloc(&B.d_ashort, c * 4));
        HIPCHK(hipMalloc(&B.d_along, (c / 257 + 64) * 8));
        HIPCHK(hipMalloc(&B.d_apiece, (c / AUX_PIECE + c / 257 + 64) * 8));
        HIPCHK(hipMalloc(&B.d_amulti, (c / AUX_PIECE + 64) * 8));
        B.aux_cap_n = c;
    }
    if (!e->d_auxpool) {
        HIPCHK(hipMalloc(&e->d_auxpool, (uint64_t)AUXPOOL_CAP * sizeof(AuxAcc)));
        e->auxpool_cap = AUXPOOL_CAP;
    }
    if (npiece > e->auxmeta_cap) {
        HIPCHK(hipStreamSynchronize(e->stream));  // no decide stage may use the old buffer
        dfree(e->d_auxmeta);
        const uint64_t c = std::max<uint64_t>(npiece, B.aux_cap_n / AUX_PIECE + B.aux_cap_n / 257 + 64);
        HIPCHK(hipMalloc(&e->d_auxmeta, c * 8));
        e->auxmeta_cap = c;
    }
    return SG_OK;
}

static bool is_device_ptr(const void* p) {
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) { (void)hipGetLastError(); return false; }
    return a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeManaged;
}

// Batch pipeline: the group stage (records, sort, segments, bins) of this batch runs on gstream and
// the host waits for it only; the decide stage (reference resolution, chain grants, decide kernels,
// post) is enqueued on stream behind the previous batch's and the call returns.  So batch k+1's
// group stage overlaps batch k's decide stage.  Buffers must stay valid until sg_sync.
static int submit_impl(sg_engine* e, const sg_event* ev, const sg_event_ext* ext, uint64_t n, const sg_arg* args,
                       uint64_t n_args, uint32_t* out) {
    if (!e || (n && (!ev || !out))) return fail(SG_EINVAL, "null argument");
    if (n_args && !args) return fail(SG_EINVAL, "null args table");
    if (!e->fatal.empty()) return fail(SG_ESTATE, e->fatal + " -- engine unusable, recreate it");
    if (n == 0) return SG_OK;
    if (n > e->cfg.max_batch_events || n >= (1ull << 31)) return fail(SG_EINVAL, "batch larger than max_batch_events");
    HIPCHK(hipSetDevice(e->device));
    int rc = ensure_batch(e, n);
    if (rc) return rc;
    const int k = e->cur;
    rc = collect(e, k);  // the batch that last used this slot (two batches ago) is decided
    if (rc) return rc;
    // the param map pool: the regions maps grew out of are dropped by a compaction between batches once the growth
    // since the last one took half of what was free (the counts are a batch or two old); a batch that finds the pool
    // short before that compacts on the device itself (launch_pm_grow)
    if (int prc = ensure_pool2(e)) return prc;
    const unsigned long long pfloor = e->h_pool_next ? e->h_pool_next[PC_FLOOR] : 0;
    if (e->pool_nb && e->h_pool_next[PC_NEXT] > pfloor + (e->pool_nb - pfloor) / 2) {
        if (int drc = drain(e)) return drc;
        if (int crc = compact_pmaps(e)) return crc;
        ++e->n_compact;
    }
    activate(e, k);
    auto& B = e->slot[k];
    hipStream_t gs = e->gstream, st = e->stream;
    const sg_event* dev_ev = ev;
    bool host_in = !is_device_ptr(ev);
    bool host_out = !is_device_ptr(out);
    if (host_in) {
        HIPCHK(hipMemcpyAsync(e->d_ev, ev, n * sizeof(sg_event), hipMemcpyHostToDevice, gs));
        dev_ev = e->d_ev;
    }
    uint32_t* dev_out = host_out ? e->d_out : out;
    // sg_submit_ex: the Context and args tables in HBM (staged per batch slot when the caller's are host memory)
    const sg_event_ext* dev_ext = ext;
    const sg_arg* dev_args = n_args ? args : nullptr;
    if (ext && !is_device_ptr(ext)) {
        if (n > B.ext_cap) {
            dfree(B.d_ext);
            B.ext_cap = std::max<uint64_t>(n, 1u << 16);
            HIPCHK(hipMalloc(&B.d_ext, B.ext_cap * sizeof(sg_event_ext)));
        }
        HIPCHK(hipMemcpyAsync(B.d_ext, ext, n * sizeof(sg_event_ext), hipMemcpyHostToDevice, gs));
        dev_ext = B.d_ext;
    }
    if (n_args && !is_device_ptr(args)) {
        if (n_args > B.args_cap) {
            dfree(B.d_args);
            B.args_cap = std::max<uint64_t>(n_args, 1u << 16);
            HIPCHK(hipMalloc(&B.d_args, B.args_cap * sizeof(sg_arg)));
        }
        HIPCHK(hipMemcpyAsync(B.d_args, args, n_args * sizeof(sg_arg), hipMemcpyHostToDevice, gs));
        dev_args = B.d_args;
    }
    const uint64_t ring_mask = (1ull << e->cfg.status_ring_log2) - 1;
    // Overlapping this group stage with the previous batch's decide stage wins once the decide kernels
    // no longer stream frozen stretches through single CUs (C4 on MI355X: 6.45 -> 5.45 ms per batch);
    // SG_PIPELINE=0 runs the stages back to back.
    if (!e->pipeline && e->last >= 0 && e->slot[e->last].pending)
        HIPCHK(hipStreamWaitEvent(gs, e->slot[e->last].ev[4], 0));
    HIPCHK(hipEventRecord(B.ev[0], gs));
    // ---- 1. group: records + stable LSD radix sort on res_id (8-bit digits over the bits of max_resources-1)
    uint32_t R = e->cfg.max_resources;
    int bits = 1;
    while (bits < 32 && (1ull << bits) < R) ++bits;
    // 8-bit digits: measured faster than two 10-bit passes for 1M resources on MI355X (group stage
    // 2.99 vs 3.11 ms standalone; 1024 digit runs per 4096-item tile average 4 items, too short to
    // write coalesced).
    const int db = 8;
    int passes = (bits + db - 1) / db;
    uint32_t nblocks = (uint32_t)((n + radix_tile() - 1) / radix_tile());
    HIPCHK(hipMemsetAsync(e->d_bsmall, 0, 256 * 4, gs));
    int64_t* d_t0 = reinterpret_cast<int64_t*>(e->d_bsmall + 4);  // [4..5]
    uint32_t *kin = e->d_k1, *vin = e->d_v1, *kout = e->d_k0, *vout = e->d_v0;
    if (++e->epoch == 0) e->epoch = 1;
    // every event through the radix passes: SG_DEBUG_FLAGS & 8192 (A/B of the group stage), or a batch of 2^30 events
    // or more (the hot / cold stage's words hold a position in 30 bits)
    B.radix = e->radix_group || n >= (1ull << 30) || n < e->radix_below;
    if (B.radix) {
        HIPCHK(launch_rs_first(dev_ev, n, R, e->gbase, e->d_ring, ring_mask, e->cfg.statistic_max_rt, e->d_rec_o,
                               e->d_k1, e->d_v1, e->d_hist, nblocks, e->d_bsmall + 0, d_t0, e->d_prio, e->d_keyring,
                               e->d_comp, dev_ext, dev_args, n_args, SG_MAX_CONTEXTS, gs));
        for (int p = 0; p < passes; ++p) {
            if (p > 0) HIPCHK(launch_radix_hist(kin, n, p * db, e->d_hist, nblocks, gs));
            HIPCHK(launch_scan(e->d_hist, e->d_hist, (uint64_t)nblocks << db, e->d_part, nullptr, gs));
            HIPCHK(launch_radix_scatter(kin, vin, n, p * db, e->d_hist, nblocks, kout, vout,
                                        p == passes - 1 ? e->d_posof : nullptr, gs));
            std::swap(kin, kout);
            std::swap(vin, vout);
        }
        HIPCHK(launch_seg(kin, n, e->d_flag, e->d_pos, e->d_segs, gs, launch_scan, e->d_part, e->d_bsmall + 1));
        HIPCHK(launch_gather(e->d_rec_o, vin, kin, n, e->d_posof, e->d_recs, e->d_prev, e->d_bsmall + 3, e->d_link,
                             e->d_bst, e->epoch, e->d_bsmall + 0, gs));
    } else {
        // ---- hot / cold group stage (kernels.hip k_grp_*): [77] hot_total (the cold region's start), [78] cold
        // events, [80] hot segments, [81] (hot_total again), [82] cold segments, [76] the next batch's hot ids
        const uint32_t nhot = e->nhot;
        B.nhot = nhot;
        uint32_t* words = e->d_flag;    // per event: W_HOT | W_ENT? | hot id << 12 | rank in its tile's run of the id;
                                        // cold: W_ENT? | sorted position (the last cold pass)
        uint32_t* hot_off = e->d_pos;   // [hot id][tile] counts, scanned in place: the runs' sorted positions
        uint32_t* ccnt = B.d_ccnt;      // per tile: cold events (compacted at the tile's start in k1 / v1)
        HIPCHK(launch_grp_first(dev_ev, n, R, e->gbase, ring_mask, e->d_bsmall + 0, d_t0, e->d_prio, e->d_keyring,
                                e->d_comp, dev_ext, dev_args, n_args, SG_MAX_CONTEXTS, e->d_hot_tab, nhot, nblocks,
                                words, hot_off, e->d_k1, e->d_v1, ccnt, e->d_hist, gs));
        HIPCHK(launch_hot_scan(hot_off, nblocks, nhot, e->d_hot_part, e->d_hot_hb, e->d_bsmall + 77, gs));
        HIPCHK(launch_cold_n(n, e->d_bsmall + 77, e->d_bsmall + 78, gs));
        if (nblocks == 1) {  // one tile: the cold pairs sorted by one workgroup (k_cold_small), into k0 / v0
            HIPCHK(launch_cold_small(kin, vin, ccnt, e->d_bsmall + 77, kout, vout, words, gs));
            std::swap(kin, kout);
            std::swap(vin, vout);
        }
        for (int p = 0; p < passes && nblocks > 1; ++p) {  // the cold (key, index) pairs
            if (p > 0) HIPCHK(launch_radix_hist_n(kin, n, e->d_bsmall + 78, p * db, e->d_hist, nblocks, gs));
            HIPCHK(launch_scan(e->d_hist, e->d_hist, (uint64_t)nblocks << db, e->d_part, nullptr, gs));
            const bool last = p == passes - 1;
            HIPCHK(launch_radix_scatter_x(kin, vin, n, p ? e->d_bsmall + 78 : nullptr, p ? nullptr : ccnt,
                                          last ? e->d_bsmall + 77 : nullptr, p * db, e->d_hist, nblocks, kout, vout,
                                          last ? words : nullptr, gs));
            std::swap(kin, kout);
            std::swap(vin, vout);
        }
        // segments: the hot ids' (in id order), then the cold keys' [hot_total, n)
        HIPCHK(launch_hot_segs(e->d_hot_hb, nhot, e->d_hot_list, e->d_segs, e->d_bsmall + 80, gs));
        const uint64_t sc = nblocks + 64;
        HIPCHK(launch_seg_cold(kin, n, e->d_bsmall + 77, e->d_bsmall + 80, ccnt + sc, ccnt + 2 * sc, e->d_segs, gs,
                               launch_scan, e->d_part, e->d_bsmall + 82, e->d_bsmall + 1));
        HIPCHK(hipMemsetAsync(e->d_bst, 0, ((n + 1023) / 1024) * 4, gs));
        HIPCHK(launch_grp_records(dev_ev, n, e->gbase, ring_mask, e->cfg.statistic_max_rt, words, hot_off, nhot, nblocks,
                                  e->d_hot_hb, e->d_recs, vin, e->d_prev, e->d_bsmall + 3, e->d_bst,
                                  e->d_bsmall + 0, dev_ext, dev_args, SG_MAX_CONTEXTS, e->d_link, e->epoch, gs));
        HIPCHK(launch_block_sums(e->d_recs, n, e->d_bst, e->d_link, e->epoch, e->d_bsmall + 0, kin, e->d_bsmall + 77, gs));
    }
    // bins + bin-ordered dispatch list (per-block counts -> scan -> placement), sized by an upper bound of
    // the segment count so that the group stage needs one host round trip
    const bool force_lane = !e->cfg.switch_on || (e->dbg_flags & 2);
    const uint32_t mb = (uint32_t)std::min<uint64_t>(n, R);
    const uint32_t nblk = (mb + 255) / 256;
    // Bin thresholds by batch size: a full batch (C4: 2^25 events) keeps the decide stage busy with event
    // throughput, and wider owners for shorter segments cost more than they save (measured); in a batch of
    // fewer than SHARD_BATCH (6.3M) events -- one rank's shard of a multi-GPU step -- the longest owner chains bound it
    // instead, so segments get wider owners sooner (tools/shard_rehearsal.sh: 8-way shards of C4, mean
    // rank step 1.70 -> 1.33 ms, slowest 1.85 -> 1.73 ms).
    uint32_t lane_max = e->lane_max, j1_max = e->j1_max, j4_max = e->j4_max;
    // (below SHARD_BATCH events: an 8-way shard of a 2^25-event global batch is ~2^22; a 4-way shard's 2^23 runs
    // faster with the full-batch bins: 4-way rehearsal 2.24 -> 1.79 ms per global batch)
    if (!e->bins_pinned && n < SHARD_BATCH) {
        lane_max = std::min<uint32_t>(lane_max, 128);
        j1_max = std::min<uint32_t>(j1_max, 1024);
        j4_max = std::min<uint32_t>(j4_max, 4096);
    }
    if (ext) {  // the aux.hip post-pass lists of this slot
        if (int arc = ensure_aux(e, B, n)) return arc;
    }
    if (e->has_mix) {  // the XF_MIX lists of this slot
        if (int mrc = ensure_mix(B, mb)) return mrc;
    }
    HIPCHK(launch_seg_bin(e->d_segs, e->d_bsmall + 1, mb, n, e->d_prog, e->d_prio, lane_max, j1_max, j4_max,
                          force_lane ? 1 : 0, e->d_blkcnt, e->pq_on ? 1u : 0u, e->pq_wide, ext ? e->d_bsmall + 130 : nullptr,
                          B.d_ashort, B.d_along, B.d_amulti, e->d_bsmall + 6, e->has_mix ? B.d_mix : nullptr,
                          (uint32_t)B.mix_cap, e->d_bsmall + 72, (e->pv_on || e->pvt_on) ? 0u : e->pq_wide,
                          (e->dbg_flags & HEAD_OFF) ? 0u : e->head_min, gs));
    HIPCHK(launch_scan(e->d_blkcnt, e->d_blkcnt, (uint64_t)nblk * N_BINS, e->d_part, nullptr, gs));
    HIPCHK(launch_seg_order(e->d_segs, e->d_bsmall + 1, mb, e->d_blkcnt, e->d_order, e->d_bsmall + 8, gs));
    // the next batch's hot ids: this batch's resources of >= n / 8192 events (about one per 4096-event tile, so
    // that a tile's run of one hot id is more than a random write), at least 64
    const uint32_t hot_min = (uint32_t)std::max<uint64_t>(64, n / 8192);
    if (!B.radix)
        HIPCHK(launch_hot_build(e->d_segs, e->d_bsmall + 1, mb, hot_min, R, e->d_hot_tab, e->d_hot_list, e->nhot,
                                e->d_bsmall + 76, gs));
    // [0] bflags [1] nseg [3] nprev [4..5] t0 [6..7] XF_MIX lists [8..8+N_BINS] bin offsets [72] wide XF_MIX events
    // [76] the next batch's hot ids
    uint32_t head[77];
    static_assert(8 + N_BINS + 1 <= 72, "head layout");
    HIPCHK(hipMemcpyAsync(head, e->d_bsmall, sizeof(head), hipMemcpyDeviceToHost, gs));
    HIPCHK(hipEventRecord(B.ev[1], gs));
    HIPCHK(hipStreamSynchronize(gs));
    if (!B.radix) e->nhot = std::min<uint32_t>(head[76], hot_max());
    const uint32_t m = head[1];
    const uint32_t nprev = head[3];
    int64_t t0 = 0;
    std::memcpy(&t0, head + 4, 8);
    uint32_t bflags = head[0];
    if (bflags & BF_BAD_RES) return fail(SG_EINVAL, "event res_id >= max_resources");
    if (bflags & BF_BAD_REF)
        return fail(SG_EINVAL, "an EXIT/TRACE references an event that is not an earlier ENTRY of the same resource");
    if (bflags & BF_TSPAN) return fail(SG_EINVAL, "a batch must span less than 2^31 ms");
    if (bflags & BF_BACKWARD) return fail(SG_EINVAL, "event timestamps must be non-decreasing (SURVEY Q3)");
    if (bflags & BF_BAD_ARGS)
        return fail(SG_EINVAL, "an sg_event_ext names args outside the table (or more than SG_MAX_ARGS, or a bad kind)");
    const uint32_t* off = head + 8;
    uint32_t bin_n[N_BINS];
    for (int b = 0; b < N_BINS; ++b) bin_n[b] = off[b + 1] - off[b];
    // ---- 3. decide: cooperative bins on their own streams, lane bins on the main stream (state for every kernel)
    DevCfg dc;
    std::memset(&dc, 0, sizeof(dc));
    dc.max_rt = e->cfg.statistic_max_rt;
    dc.occupy_timeout = e->cfg.occupy_timeout_ms;
    dc.max_chain = e->cfg.max_slot_chain_size;
    dc.switch_on = e->cfg.switch_on;
    dc.ring_mask = ring_mask;
    dc.dbg_flags = e->dbg_flags;
    dc.heads = e->has_head ? 1u : 0u;
    DevState S{};
    std::memset(&S, 0, sizeof(S));
    S.sec = e->d_sec;
    S.minb = e->d_minb;
    S.info = e->d_info;
    S.prog = e->d_prog;
    S.rules = e->d_rules;
    S.rstate = e->d_rstate;
    S.hot = e->d_hot;
    S.pmap = e->d_pmap;
    S.pbkt = e->d_pbkt;
    S.pdat = e->d_pdat;
    S.pbm = e->d_pbm;
    S.ppre = e->d_ppre;
    S.tmid = e->d_tmid;
    S.ring = e->d_ring;
    S.sink = e->d_sink;
    S.borrow = e->d_borrow;
    S.prio = e->d_prio;
    S.key_ring = e->d_keyring;
    S.gbase = e->gbase;
    S.link = e->d_link;
    S.bst = e->d_bst;
    S.pend = e->d_pend;
    S.spans = e->d_spans;
    S.nspan = e->d_bsmall + 120;
    S.span_cap = e->span_cap;
    S.epoch = e->epoch;
    S.skip_ok = !(bflags & (BF_MULTI_LINK | BF_ZERO_CNT)) && !(e->dbg_flags & 4) ? 1u : 0u;
    // a shard-sized batch (see the bins above) is bound by its longest owners, whose frozen stretches are
    // cheaper skipped than streamed from 8192 positions on (8-way C4 shards: slowest rank 1.79 -> 1.69 ms)
    S.skip_min = (!e->skip_pinned && n < SHARD_BATCH) ? std::min<uint32_t>(e->skip_min, 8192) : e->skip_min;
    S.ext = dev_ext;
    S.args = dev_args;
    S.aux_tab = e->d_auxtab;
    S.aux_count = e->d_auxcnt;
    S.aux_cap = e->cfg.aux_node_capacity;
    S.aux_mask = e->aux_mask;
    S.max_ctx = SG_MAX_CONTEXTS;
    // ---- decide stage, in order after the previous batch's: references into earlier batches first
    HIPCHK(hipStreamWaitEvent(st, B.ev[1], 0));
    const uint32_t n_mix = e->has_mix ? head[6] : 0u, n_mixw = e->has_mix ? head[7] : 0u;
    // SG_DEBUG_FLAGS & 8 (diagnostics): every decide kernel on the main stream, one after the other
    const bool serial_bins = (e->dbg_flags & 8) != 0;
    const bool pre_split = (n_mix || n_mixw) && !serial_bins;
    hipStream_t ps = pre_split ? e->bin_stream[1] : st;
    // the value-parallel pre pass's extraction and sort (launch_pv_a) read only this batch's records and the rules,
    // so with every chain granted (k_pv_prep then knows the grants' outcome) they start as soon as this batch is
    // grouped, on bin_stream[1] beside the previous batch's post pass (their own scratch, pvb; the post pass has pvbt)
    const uint32_t grant_all = (e->cfg.switch_on && e->cfg.max_slot_chain_size <= 0) ? 1u : 0u;
    if (n_mixw && (e->pv_on || e->pvt_on) && head[72]) {
        if (int prc = ensure_pv(e, head[72], n_mixw)) return prc;
        e->pv_last_m = n_mixw;
    }
    const bool pv_ran = n_mixw && e->pv_on && head[72];
    const bool pv_early = pv_ran && pre_split && grant_all && !e->has_multi;
    if (pv_early) {
        HIPCHK(hipStreamWaitEvent(ps, B.ev[1], 0));
        HIPCHK(launch_pv_a(e->d_recs, vin, e->d_segs, B.d_mix + B.mix_cap, n_mixw, S, dc, e->d_dec, e->d_pvseg, e->pvb,
                           head[72], e->d_pvtot, e->d_pvhist, e->d_pvpart, ps, launch_radix_hist_n,
                           launch_radix_scatter_n, launch_scan, radix_tile(), e->d_pvrest, grant_all));
    }
    HIPCHK(launch_resolve(e->d_prev, nprev, e->d_ring, e->d_recs, vin, dev_ext, st));
    // ---- chain cap (CtSph.lookProcessChain): grant chains in order of first ENTRY.  First on the decide stream: the
    // pre pass's eligibility reads the chain flags (it ran beside the grants and raced them)
    if (e->cfg.switch_on && (e->cfg.max_slot_chain_size <= 0 || e->n_chains < (uint32_t)e->cfg.max_slot_chain_size)) {
        const bool grant_all = e->cfg.max_slot_chain_size <= 0;
        HIPCHK(launch_chain(e->d_recs, vin, e->d_segs, m, e->d_info, grant_all ? 1 : 0, e->d_bsmall + 2, e->d_cand,
                            dev_ev, e->d_prog, dev_ext, SG_MAX_CONTEXTS, st));
        if (!grant_all) {
            uint32_t ncand = 0;
            HIPCHK(hipMemcpyAsync(&ncand, e->d_bsmall + 2, 4, hipMemcpyDeviceToHost, st));
            HIPCHK(hipStreamSynchronize(st));
            if (ncand) {
                std::vector<uint64_t> cand(ncand);
                HIPCHK(hipMemcpy(cand.data(), e->d_cand, ncand * 8ull, hipMemcpyDeviceToHost));
                std::sort(cand.begin(), cand.end());  // by batch index of the first ENTRY
                std::vector<uint64_t> upd;
                std::unordered_map<uint32_t, int> seen;  // RELATE components list every ENTRY
                for (uint32_t i = 0; i < ncand; ++i) {
                    uint32_t res = (uint32_t)cand[i];
                    if (!seen.emplace(res, 1).second) continue;
                    bool grant = e->n_chains < (uint32_t)e->cfg.max_slot_chain_size;
                    if (grant) e->n_chains++;
                    upd.push_back(((uint64_t)(grant ? NI_CHAIN : NI_REJECTED) << 32) | res | (1ull << 63));
                }
                ncand = (uint32_t)upd.size();
                HIPCHK(hipMemcpyAsync(e->d_cand, upd.data(), ncand * 8ull, hipMemcpyHostToDevice, st));
                HIPCHK(launch_set_flags(e->d_info, e->d_cand, ncand, st));
                HIPCHK(hipStreamSynchronize(st));
            }
        }
    }
    // XF_MIX segments of the cooperative bins (and XF_PVPQ ones): their param checks first (the value-parallel pre
    // pass, else k_pq's), the owners then decide the flow / degrade chain on them.  The pre pass runs on
    // bin_stream[1] (whose J4 / J1 wait for it anyway); its extraction and sort touch no map region, so they start
    // after the chain grants, beside the maps' growth on the main stream; the rest waits for the growth.
    if (pre_split) {
        HIPCHK(hipEventRecord(e->fork0, st));
        HIPCHK(hipStreamWaitEvent(ps, e->fork0, 0));
    }
    if (pv_ran && !pv_early)
        HIPCHK(launch_pv_a(e->d_recs, vin, e->d_segs, B.d_mix + B.mix_cap, n_mixw, S, dc, e->d_dec, e->d_pvseg, e->pvb,
                           head[72], e->d_pvtot, e->d_pvhist, e->d_pvpart, ps, launch_radix_hist_n,
                           launch_radix_scatter_n, launch_scan, radix_tile(), e->d_pvrest, grant_all));
    // param map regions grown for this batch's segments before anything touches a map; the pool's use, for the
    // compaction check of a later submit
    if (e->pool_nb) {
        DevState Sg{};
        std::memset(&Sg, 0, sizeof(Sg));
        Sg.prog = e->d_prog; Sg.rules = e->d_rules; Sg.tmid = e->d_tmid; Sg.prio = e->d_prio;
        Sg.pmap = e->d_pmap; Sg.pbkt = e->d_pbkt; Sg.pdat = e->d_pdat; Sg.pbm = e->d_pbm;
        const uint32_t nm = (uint32_t)e->pmap_key.size();
        HIPCHK(launch_pm_grow(e->d_segs, e->d_bsmall + 1, mb, Sg, e->d_pool_next, e->pool_nb, e->d_bsmall + 0, e->d_pmoves,
                              e->d_pmoves ? reinterpret_cast<uint32_t*>(e->d_pmoves + e->pmoves_cap) : nullptr,
                              (uint32_t)e->pmoves_cap, e->epoch, nm, e->d_pbkt2, e->d_pdat2, e->d_pcwork,
                              e->d_pcwork + e->pmoves_cap, e->d_pcwork + 2 * e->pmoves_cap, launch_scan, st));
        HIPCHK(hipMemcpyAsync(e->h_pool_next, e->d_pool_next, PC_WORDS * 8, hipMemcpyDeviceToHost, st));
    }
    HIPCHK(hipEventRecord(B.ev[2], st));
    if (pre_split) {  // every map-touching pre-pass kernel after the maps grew (they move)
        HIPCHK(hipEventRecord(e->grown, st));
        HIPCHK(hipStreamWaitEvent(ps, e->grown, 0));
    }
    if (pv_ran) {  // the rest of the value-parallel pre pass
        HIPCHK(launch_pv_b(e->d_recs, e->d_segs, B.d_mix + B.mix_cap, n_mixw, S, t0, e->d_dec, e->d_bsmall + 0,
                           e->d_pvseg, e->pvb, head[72], e->d_pvtot, e->d_pvpart, (bflags & BF_ZERO_CNT) ? 0u : 1u, ps,
                           launch_scan, e->d_pvrest));
    }
    if (n_mix || n_mixw)
        HIPCHK(launch_pq_mix(0, e->d_recs, dev_ev, vin, e->d_segs, B.d_mix, n_mix, B.mix_cap, n_mixw, S, dc, t0,
                             e->d_dec, e->d_bsmall + 0, ps, pv_ran ? e->d_pvrest + 1 : nullptr, e->d_pvrest));
    HIPCHK(hipEventRecord(e->fork, ps));
    auto lane_bins = [&]() -> int {
        {
            DevState Sl = S;
            Sl.dbg = e->d_dbg;  // SG_KPROF builds: lane-kernel phase cycles in dbg[32..36]
            HIPCHK(launch_decide_bin(BIN_LANE, e->d_recs, dev_ev, vin, e->d_segs, e->d_order + off[BIN_LANE],
                                     off[BIN_LANE + LANE_BINS] - off[BIN_LANE], Sl, dc, t0, e->d_dec, e->d_bsmall + 0, st));
        }
        HIPCHK(launch_decide_bin(BIN_LANE16, e->d_recs, dev_ev, vin, e->d_segs, e->d_order + off[BIN_LANE16],
                                 off[BIN_LANE16 + LANE_BINS] - off[BIN_LANE16], S, dc, t0, e->d_dec, e->d_bsmall + 0, st));
        {
            DevState Sl = S;
            Sl.dbg = e->d_dbg;  // SG_KPROF builds: lane-kernel phase cycles in dbg[32..37]
            HIPCHK(launch_decide_bin(BIN_LITE, e->d_recs, dev_ev, vin, e->d_segs, e->d_order + off[BIN_LITE],
                                     off[BIN_LITE + LANE_BINS] - off[BIN_LITE], Sl, dc, t0, e->d_dec, e->d_bsmall + 0, st));
        }
        return SG_OK;
    };
    if (pre_split) {
        if (int lrc = lane_bins()) return lrc;
        HIPCHK(hipStreamWaitEvent(st, e->fork, 0));  // (J8 / J1 on the main stream read the pre passes' verdicts)
    }
    // J16 and J4 on their own streams; J1 after the lane bins on the main stream (J4 + J1 in series was the
    // longest chain of the decide stage)
    const int coop[2] = {BIN_J16, BIN_J4};
    // J8 (the QPS-DefaultController heads) takes J16's stream when every head is of that kind (C2, C4); beside
    // THREAD-grade / WarmUp heads (C3: J16 is the decide stage's longest chain) it runs first on the main stream
    const bool j8_own = bin_n[BIN_J8] && !bin_n[BIN_J16];
    for (int c = 0; c < 2; ++c) {
        const int b = coop[c];
        if (c == 0 && bin_n[BIN_J8]) {
            DevState Sb = S;
            Sb.dbg = (e->prof_bin == 0 && e->d_dbg) ? e->d_dbg : nullptr;
            hipStream_t bs = (serial_bins || !j8_own) ? st : e->bin_stream[0];
            if (bs != st) HIPCHK(hipStreamWaitEvent(bs, e->fork, 0));
            HIPCHK(launch_decide_bin(BIN_J8, e->d_recs, dev_ev, vin, e->d_segs, e->d_order + off[BIN_J8], bin_n[BIN_J8], Sb, dc,
                                     t0, e->d_dec, e->d_bsmall + 0, bs));
            if (bs != st) HIPCHK(hipEventRecord(e->join[0], bs));
        }
        if (!bin_n[b]) continue;
        DevState Sb = S;
        Sb.dbg = (c == e->prof_bin && e->d_dbg) ? e->d_dbg : nullptr;
        hipStream_t bs = serial_bins ? st : e->bin_stream[c];
        if (!serial_bins) HIPCHK(hipStreamWaitEvent(bs, e->fork, 0));
        HIPCHK(launch_decide_bin(b, e->d_recs, dev_ev, vin, e->d_segs, e->d_order + off[b], bin_n[b], Sb, dc, t0,
                                 e->d_dec, e->d_bsmall + 0, bs));
        HIPCHK(hipEventRecord(e->join[c], bs));
    }
    // hot-parameter owners (k_pq): the wide ones beside J16, the narrow ones beside J4
    for (int c = 0; c < 2; ++c) {
        const int b = c == 0 ? BIN_PQ16 : BIN_PQ4;
        if (!bin_n[b]) continue;
        hipStream_t bs = serial_bins ? st : e->bin_stream[c];
        if (!serial_bins && !bin_n[coop[c]] && !(c == 0 && j8_own)) HIPCHK(hipStreamWaitEvent(bs, e->fork, 0));
        DevState Sp = S;
        Sp.dbg = (c == 0 && e->prof_bin == 3) ? e->d_dbg : nullptr;  // SG_PROF_BIN=3: k_pq<16> phase cycles (kprof builds)
        HIPCHK(launch_pq(c == 0, e->d_recs, dev_ev, vin, e->d_segs, e->d_order + off[b], bin_n[b], Sp, dc, t0, e->d_dec,
                         e->d_bsmall + 0, bs));
        HIPCHK(hipEventRecord(e->join[c], bs));
    }
    if (!pre_split)
        if (int lrc = lane_bins()) return lrc;
    // sg_submit_ex: the short segments' origin / context nodes (aux.hip k_aux_cold) need only the lane bins' verdicts
    // when every short segment (<= AUX_SHORT = 256 events, decide.hip) is a lane one -- lane bins up to 256 events and
    // no k_pq<4> segment -- so they go right after them, beside the owners
    // (a short PF_PQ segment on k_pq<16>, SG_PQ_WIDE below 256, is not a lane one either: ADVICE r5)
    const bool aux_early = ext && !bin_n[BIN_PQ4] && !serial_bins && (force_lane || lane_max >= 256u) &&
                           (!bin_n[BIN_PQ16] || e->pq_wide >= 256u);
    if (aux_early)
        HIPCHK(launch_aux_cold(e->d_recs, e->d_segs, e->d_bsmall + 130, B.d_ashort, S, dc, t0, e->d_dec, e->d_bsmall + 0, st));
    // J1: after the lane bins on the main stream, or (SG_J1_STREAM=1, and with the short aux nodes on the main stream)
    // after J16 / J8 on bin_stream[0]
    const bool j1_b0 = bin_n[BIN_J1] && !serial_bins && (e->j1_stream == 1 || (e->j1_stream < 0 && aux_early));
    // SG_J1_STREAM=2: the J1 segments halved, one half after J16 / J8 on bin_stream[0], the other after J4 on
    // bin_stream[1] (A/B)
    const bool j1_split = bin_n[BIN_J1] > 1 && !serial_bins && e->j1_stream == 2;
    if (j1_split) {
        const uint32_t h = bin_n[BIN_J1] / 2;
        for (int c = 0; c < 2; ++c) {
            DevState Sj = S;
            Sj.dbg = nullptr;
            hipStream_t bs = e->bin_stream[c];
            const bool ran = c == 0 ? (bin_n[BIN_J16] || bin_n[BIN_J8] || bin_n[BIN_PQ16]) : (bin_n[BIN_J4] || bin_n[BIN_PQ4]);
            if (!ran) HIPCHK(hipStreamWaitEvent(bs, e->fork, 0));
            HIPCHK(launch_decide_bin(BIN_J1, e->d_recs, dev_ev, vin, e->d_segs, e->d_order + off[BIN_J1] + (c ? h : 0),
                                     c ? bin_n[BIN_J1] - h : h, Sj, dc, t0, e->d_dec, e->d_bsmall + 0, bs));
            HIPCHK(hipEventRecord(e->join[c], bs));
        }
    } else if (bin_n[BIN_J1]) {
        DevState Sj = S;
        Sj.dbg = (e->prof_bin == 2 && e->d_dbg) ? e->d_dbg : nullptr;
        hipStream_t bs = j1_b0 ? e->bin_stream[0] : st;
        if (j1_b0 && !(bin_n[BIN_J16] || bin_n[BIN_J8] || bin_n[BIN_PQ16])) HIPCHK(hipStreamWaitEvent(bs, e->fork, 0));
        HIPCHK(launch_decide_bin(BIN_J1, e->d_recs, dev_ev, vin, e->d_segs, e->d_order + off[BIN_J1], bin_n[BIN_J1], Sj, dc,
                                 t0, e->d_dec, e->d_bsmall + 0, bs));
        if (j1_b0) HIPCHK(hipEventRecord(e->join[0], bs));
    }
    for (int c = 0; c < 2; ++c)
        if (bin_n[coop[c]] || bin_n[c == 0 ? BIN_PQ16 : BIN_PQ4] || (c == 0 && (j8_own || j1_b0)) || j1_split)
            HIPCHK(hipStreamWaitEvent(st, e->join[c], 0));
    // verdicts of the frozen spans the cooperative kernels skipped
    if (S.skip_ok && (bin_n[BIN_J16] || bin_n[BIN_J8] || bin_n[BIN_J4]))
        HIPCHK(launch_fill(e->d_spans, S.nspan, e->span_cap, e->d_recs, e->d_prog, e->d_rules, e->d_dec, st));
    // XF_MIX: the thread-count maps and ParameterMetric bits from the final verdicts (the long ones value-parallel
    // where the maps do not overflow, pvalue.hip; the rest by k_pq's post pass)
    if (n_mixw && e->pvt_on && head[72])
        HIPCHK(launch_pvt(e->d_recs, dev_ev, vin, e->d_segs, B.d_mix + B.mix_cap, n_mixw, S, dc, e->d_dec,
                          e->d_bsmall + 0, e->d_pvtseg, e->pvbt, head[72], e->d_pvtot + 4, e->d_pvthist, e->d_pvtpart, st,
                          launch_radix_hist_n, launch_radix_scatter_n, launch_scan, radix_tile(),
                          e->d_pvrest + e->pvseg_cap + 1));
    const bool pvt_ran = n_mixw && e->pvt_on && head[72];
    uint32_t* prest = e->d_pvrest + e->pvseg_cap + 1;
    if (n_mix || n_mixw)
        HIPCHK(launch_pq_mix(1, e->d_recs, dev_ev, vin, e->d_segs, B.d_mix, n_mix, B.mix_cap, n_mixw, S, dc, t0,
                             e->d_dec, e->d_bsmall + 0, st, pvt_ran ? prest + 1 : nullptr, prest));
    // origin / context nodes of the segments decided off k_lane<16>, from the committed verdicts (aux.hip)
    if (ext)
        HIPCHK(launch_aux(e->d_recs, e->d_segs, e->d_bsmall + 130, aux_early ? nullptr : B.d_ashort, B.d_along, B.d_apiece,
                          B.d_amulti, S, dc, t0, e->d_dec, e->d_auxpool, e->auxpool_cap, e->d_bsmall + 134, e->d_auxmeta,
                          e->d_bsmall + 0, st));
    HIPCHK(hipEventRecord(B.ev[3], st));
    // ---- 4. decisions back to submission order + status ring
    if (B.radix) HIPCHK(launch_post(e->d_posof, e->d_dec, n, e->gbase, e->d_ring, ring_mask, dev_out, st));
    else HIPCHK(launch_post_w(e->d_flag, e->d_pos, B.nhot, e->d_dec, n, e->gbase, e->d_ring, ring_mask, dev_out, st));
    if (host_out) HIPCHK(hipMemcpyAsync(out, dev_out, n * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipEventRecord(B.ev[4], st));
    B.pending = true;
    e->last = k;
    e->cur = k ^ 1;
    e->gbase += n;
    return SG_OK;
}

// A synchronous batch of at most tiny_max() events in one kernel (decide.hip k_tiny: every stage in one workgroup):
// the drop-in's small calls.  Returns SG_OK, an error (as the batched path's, at the same points: a malformed batch is
// rejected before any decision), or TINY_FALLBACK when the batch needs the batched path (a chain grant under a finite
// cap, which the host orders; a param pool that must be compacted first) -- nothing was decided then.
constexpr int TINY_FALLBACK = 1;
static int tiny_impl(sg_engine* e, const sg_event* ev, const sg_event_ext* ext, uint64_t n, const sg_arg* args,
                     uint64_t n_args, uint32_t* out) {
    if (!e || !ev || !out) return fail(SG_EINVAL, "null argument");
    if (n_args && !args) return fail(SG_EINVAL, "null args table");
    if (!e->fatal.empty()) return fail(SG_ESTATE, e->fatal + " -- engine unusable, recreate it");
    if (n > e->cfg.max_batch_events) return fail(SG_EINVAL, "batch larger than max_batch_events");
    HIPCHK(hipSetDevice(e->device));
    int rc = ensure_batch(e, n);
    if (rc) return rc;
    if ((rc = drain(e))) return rc;  // every earlier batch decided: the status ring holds their verdicts
    if ((rc = ensure_pool2(e))) return rc;
    const unsigned long long pfloor = e->h_pool_next ? e->h_pool_next[PC_FLOOR] : 0;
    if (e->pool_nb && e->h_pool_next[PC_NEXT] > pfloor + (e->pool_nb - pfloor) / 2) return TINY_FALLBACK;  // compaction due
    const int k = e->cur;
    activate(e, k);
    auto& B = e->slot[k];
    hipStream_t st = e->stream;
    const sg_event* dev_ev = ev;
    const bool host_out = !is_device_ptr(out);
    if (!is_device_ptr(ev)) {
        HIPCHK(hipMemcpyAsync(e->d_ev, ev, n * sizeof(sg_event), hipMemcpyHostToDevice, st));
        dev_ev = e->d_ev;
    }
    uint32_t* dev_out = host_out ? e->d_out : out;
    const sg_event_ext* dev_ext = ext;
    const sg_arg* dev_args = n_args ? args : nullptr;
    if (ext && !is_device_ptr(ext)) {
        if (n > B.ext_cap) {
            dfree(B.d_ext);
            B.ext_cap = std::max<uint64_t>(n, 1u << 16);
            HIPCHK(hipMalloc(&B.d_ext, B.ext_cap * sizeof(sg_event_ext)));
        }
        HIPCHK(hipMemcpyAsync(B.d_ext, ext, n * sizeof(sg_event_ext), hipMemcpyHostToDevice, st));
        dev_ext = B.d_ext;
    }
    if (n_args && !is_device_ptr(args)) {
        if (n_args > B.args_cap) {
            dfree(B.d_args);
            B.args_cap = std::max<uint64_t>(n_args, 1u << 16);
            HIPCHK(hipMalloc(&B.d_args, B.args_cap * sizeof(sg_arg)));
        }
        HIPCHK(hipMemcpyAsync(B.d_args, args, n_args * sizeof(sg_arg), hipMemcpyHostToDevice, st));
        dev_args = B.d_args;
    }
    if (++e->epoch == 0) e->epoch = 1;
    DevCfg dc;
    std::memset(&dc, 0, sizeof(dc));
    dc.max_rt = e->cfg.statistic_max_rt;
    dc.occupy_timeout = e->cfg.occupy_timeout_ms;
    dc.max_chain = e->cfg.max_slot_chain_size;
    dc.switch_on = e->cfg.switch_on;
    dc.ring_mask = (1ull << e->cfg.status_ring_log2) - 1;
    dc.dbg_flags = e->dbg_flags;
    dc.heads = e->has_head ? 1u : 0u;
    DevState S{};
    std::memset(&S, 0, sizeof(S));
    S.sec = e->d_sec; S.minb = e->d_minb; S.info = e->d_info; S.prog = e->d_prog; S.rules = e->d_rules;
    S.rstate = e->d_rstate; S.hot = e->d_hot; S.pmap = e->d_pmap; S.pbkt = e->d_pbkt; S.pdat = e->d_pdat;
    S.pbm = e->d_pbm; S.ppre = e->d_ppre; S.tmid = e->d_tmid; S.ring = e->d_ring; S.sink = e->d_sink;
    S.borrow = e->d_borrow; S.prio = e->d_prio; S.key_ring = e->d_keyring; S.gbase = e->gbase; S.link = e->d_link;
    S.bst = e->d_bst; S.pend = e->d_pend; S.spans = e->d_spans; S.nspan = e->d_bsmall + 120; S.span_cap = e->span_cap;
    S.epoch = e->epoch; S.skip_ok = 0; S.skip_min = e->skip_min; S.ext = dev_ext; S.args = dev_args;
    S.aux_tab = e->d_auxtab; S.aux_count = e->d_auxcnt; S.aux_cap = e->cfg.aux_node_capacity; S.aux_mask = e->aux_mask;
    S.max_ctx = SG_MAX_CONTEXTS;
    // the chain grants: every one in place (no cap), none (a cap reached: CtSph.lookProcessChain then returns null),
    // or the host's, in first-ENTRY order (the batched path)
    const int cap = e->cfg.max_slot_chain_size;
    const uint32_t grants = cap <= 0 ? 1u : e->n_chains >= (uint32_t)cap ? 2u : 0u;
    HIPCHK(launch_tiny(dev_ev, (uint32_t)n, S, dc, e->cfg.max_resources, e->d_prio, e->d_comp, n_args, grants,
                       e->d_pool_next, e->pool_nb, e->epoch, e->d_recs, e->d_v0, e->d_dec, e->d_segs, e->d_bsmall,
                       dev_out, st));
    uint32_t bflags = 0;
    HIPCHK(hipMemcpyAsync(&bflags, e->d_bsmall, 4, hipMemcpyDeviceToHost, st));
    if (host_out) HIPCHK(hipMemcpyAsync(out, dev_out, n * 4, hipMemcpyDeviceToHost, st));
    if (e->pool_nb) HIPCHK(hipMemcpyAsync(e->h_pool_next, e->d_pool_next, PC_WORDS * 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    if (bflags & BF_TINY_FALLBACK) return TINY_FALLBACK;
    if (bflags & BF_TINY_REJECTED) {  // rejected before any decision: submit_impl's checks, in its order
        if (bflags & BF_BAD_RES) return fail(SG_EINVAL, "event res_id >= max_resources");
        if (bflags & BF_BAD_REF)
            return fail(SG_EINVAL, "an EXIT/TRACE references an event that is not an earlier ENTRY of the same resource");
        if (bflags & BF_TSPAN) return fail(SG_EINVAL, "a batch must span less than 2^31 ms");
        if (bflags & BF_BACKWARD) return fail(SG_EINVAL, "event timestamps must be non-decreasing (SURVEY Q3)");
        return fail(SG_EINVAL, "an sg_event_ext names args outside the table (or more than SG_MAX_ARGS, or a bad kind)");
    }
    e->gbase += n;
    // the decide stage's own flags (collect)
    if (bflags & BF_BAD_REF)
        return fail(SG_EINVAL, "an EXIT/TRACE references an event that is not an earlier ENTRY of the same resource");
    if (bflags & BF_BACKWARD) return fail(SG_EINVAL, "event timestamps must be non-decreasing across batches (SURVEY Q3)");
    if (bflags & BF_AUX_FULL) return fail(SG_ECAPACITY, "origin/context node pool full (raise aux_node_capacity)");
    if (bflags & BF_PQ_INVARIANT)
        e->fatal = "internal error: a k_pq tile's presorted key subset did not match its accesses";
    else if (bflags & BF_POOL_FULL)
        e->fatal = "the hot-parameter map pool is used up (raise param_table_log2)";
    else if (bflags & BF_PTAB_FULL)
        e->fatal = "a hot-parameter map table could not place a key (its map holds a ghost entry)";
    if (bflags & (BF_PQ_INVARIANT | BF_PTAB_FULL | BF_POOL_FULL)) return fail(SG_ECAPACITY, e->fatal + " -- engine unusable");
    return SG_OK;
}

int sg_submit_async(sg_engine* e, const sg_event* ev, uint64_t n, uint32_t* out) {
    return submit_impl(e, ev, nullptr, n, nullptr, 0, out);
}

int sg_submit_ex_async(sg_engine* e, const sg_event* ev, const sg_event_ext* ext, uint64_t n, const sg_arg* args,
                       uint64_t n_args, uint32_t* out) {
    return submit_impl(e, ev, ext, n, args, n_args, out);
}

int sg_submit_ex(sg_engine* e, const sg_event* ev, const sg_event_ext* ext, uint64_t n, const sg_arg* args,
                 uint64_t n_args, uint32_t* out) {
    if (e && e->tiny_on && n && n <= tiny_max() && !e->radix_group) {
        const int trc = tiny_impl(e, ev, ext, n, args, n_args, out);
        if (trc != TINY_FALLBACK) return trc;
    }
    int rc = submit_impl(e, ev, ext, n, args, n_args, out);
    if (rc) {
        if (e) (void)drain(e);
        return rc;
    }
    return sg_sync(e);
}

// ContextUtil.enter(name, origin) names (core/context/ContextUtil.java:118-166).  A flow rule naming an origin
// (limitApp) or a context (STRATEGY_CHAIN refResource) before it was interned was compiled to match nothing;
// the first intern of such a name recompiles the rule programs, keeping every controller / breaker state.
int sg_intern_origin(sg_engine* e, const char* origin, uint32_t* out_id) {
    if (!e || !out_id) return fail(SG_EINVAL, "null argument");
    if (!origin || !*origin) { *out_id = 0; return SG_OK; }
    auto it = e->origin_ids.find(origin);
    if (it != e->origin_ids.end()) { *out_id = it->second; return SG_OK; }
    const uint32_t id = (uint32_t)e->origin_ids.size() + 1;
    if (id >= 0x7FFFFFFFu) return fail(SG_ECAPACITY, "too many origins");
    e->origin_ids.emplace(origin, id);
    *out_id = id;
    if (e->rule_names.count(std::string("o\x01") + origin)) {
        if (int rc = drain(e)) return rc;
        return upload_rules(e, false, false, false);
    }
    return SG_OK;
}

int sg_intern_context(sg_engine* e, const char* context, uint32_t* out_id) {
    if (!e || !out_id) return fail(SG_EINVAL, "null argument");
    if (!context || !*context || !std::strcmp(context, "sentinel_default_context")) { *out_id = 0; return SG_OK; }
    auto it = e->context_ids.find(context);
    if (it != e->context_ids.end()) { *out_id = it->second; return SG_OK; }
    const uint32_t id = (uint32_t)e->context_ids.size() + 1;
    e->context_ids.emplace(context, id);
    *out_id = id;
    if (e->rule_names.count(std::string("c\x01") + context)) {
        if (int rc = drain(e)) return rc;
        return upload_rules(e, false, false, false);
    }
    return SG_OK;
}

int sg_sync(sg_engine* e) {
    if (!e) return fail(SG_EINVAL, "null engine");
    HIPCHK(hipSetDevice(e->device));
    return drain(e);
}

int sg_submit(sg_engine* e, const sg_event* ev, uint64_t n, uint32_t* out) {
    if (e && e->tiny_on && n && n <= tiny_max() && !e->radix_group) {
        const int trc = tiny_impl(e, ev, nullptr, n, nullptr, 0, out);
        if (trc != TINY_FALLBACK) return trc;
    }
    int rc = sg_submit_async(e, ev, n, out);
    if (rc) {
        if (e) (void)drain(e);
        return rc;
    }
    return sg_sync(e);
}

int sg_last_timings(sg_engine* e, double* ms, int cap) {
    if (!e || !ms) return 0;
    int k = 0;
    for (; k < cap && k < 4; ++k) ms[k] = e->last_ms[k];
    return k;
}

int sg_param_thread_count(sg_engine* e, uint32_t res, int32_t idx, uint64_t key, int64_t* count, int32_t* present) {
    if (!e || !count) return fail(SG_EINVAL, "null argument");
    if (res >= e->cfg.max_resources) return fail(SG_EINVAL, "res_id out of range");
    if (int rc = drain(e)) return rc;
    *count = 0;
    if (present) *present = 0;
    if (idx < 0 || idx >= SG_MAX_ARGS) return SG_OK;
    const uint64_t want = TMAP_KEY | ((uint64_t)res << 8) | (uint64_t)idx;
    uint32_t id = NO_ID;
    for (uint32_t i = 0; i < (uint32_t)e->pmap_key.size(); ++i)
        if (e->pmap_key[i] == want) { id = i; break; }
    if (id == NO_ID) return SG_OK;
    HIPCHK(hipSetDevice(e->device));
    HIPCHK(hipStreamSynchronize(e->stream));
    PMap m;
    HIPCHK(hipMemcpy(&m, e->d_pmap + id, sizeof(m), hipMemcpyDeviceToHost));
    uint32_t b[2];
    pm_buckets(m.nb, key, b[0], b[1]);
    for (int h = 0; h < 2; ++h) {
        PBucket bk;
        HIPCHK(hipMemcpy(&bk, e->d_pbkt + m.base + b[h], sizeof(bk), hipMemcpyDeviceToHost));
        for (int j = 0; j < PM_BKT; ++j) {
            if (bk.key[j] != key) continue;
            const int64_t st = bk.stamp[j];
            if (st < m.thr || st >= m.clock) continue;  // a dead slot
            const uint64_t p = (uint64_t)st & ((1ull << m.rb_log2) - 1);
            uint64_t w = 0;
            HIPCHK(hipMemcpy(&w, e->d_pbm + m.bm + (p >> 6), 8, hipMemcpyDeviceToHost));
            if (!((w >> (p & 63)) & 1ull)) continue;
            PData d;
            HIPCHK(hipMemcpy(&d, e->d_pdat + (m.base + b[h]) * PM_BKT + j, sizeof(d), hipMemcpyDeviceToHost));
            *count = d.v0;
            if (present) *present = 1;
            return SG_OK;
        }
    }
    return SG_OK;
}

int sg_read_node(sg_engine* e, uint32_t res, int64_t now_ms, sg_node_state* out) {
    (void)now_ms;
    if (!e || !out) return fail(SG_EINVAL, "null argument");
    if (res >= e->cfg.max_resources) return fail(SG_EINVAL, "res_id out of range");
    if (int rc = drain(e)) return rc;
    HIPCHK(hipSetDevice(e->device));
    HIPCHK(hipStreamSynchronize(e->stream));
    Bkt sec[2], mb[60];
    int64_t bor[4];
    NodeInfo ni;
    HIPCHK(hipMemcpy(bor, e->d_borrow + (uint64_t)res * 4, sizeof(bor), hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(sec, e->d_sec + (uint64_t)res * 2, sizeof(sec), hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(mb, e->d_minb + (uint64_t)res * 60, sizeof(mb), hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(&ni, e->d_info + res, sizeof(ni), hipMemcpyDeviceToHost));
    std::memset(out, 0, sizeof(*out));
    auto ex = [](const Bkt& b, sg_bucket& o) {
        if (b.ws < 0) { std::memset(&o, 0, sizeof(o)); o.window_start = -1; return; }
        o.window_start = b.ws; o.pass = b.pass; o.block = b.block; o.exception = b.exc; o.success = b.succ;
        o.rt = b.rt; o.occupied_pass = b.occ; o.min_rt = b.minrt;
    };
    for (int i = 0; i < 8; ++i) { out->second[i].window_start = -1; out->borrow[i].window_start = -1; }
    bool chain = (ni.flags & NI_CHAIN) != 0;
    if (chain) {
        ex(sec[0], out->second[0]);
        ex(sec[1], out->second[1]);
        for (int i = 0; i < 60; ++i) ex(mb[i], out->minute[i]);
        for (int i = 0; i < 2; ++i)  // FutureBucketLeapArray buckets: pass only (min_rt as created)
            if (bor[2 * i] >= 0) {
                out->borrow[i].window_start = bor[2 * i];
                out->borrow[i].pass = bor[2 * i + 1];
                out->borrow[i].min_rt = e->cfg.statistic_max_rt;
            }
    } else {
        for (int i = 0; i < 60; ++i) out->minute[i].window_start = -1;
    }
    out->cur_thread_num = chain ? ni.thread : 0;
    out->has_chain = chain ? 1 : 0;
    return SG_OK;
}

int sg_snapshot_metrics(sg_engine* e, int64_t now_ms, sg_metric_node* out, uint64_t cap, uint64_t* n) {
    if (!e || !n) return fail(SG_EINVAL, "null argument");
    HIPCHK(hipSetDevice(e->device));
    if (int rc = drain(e)) return rc;
    uint32_t R = (uint32_t)std::min<size_t>(e->names.size(), e->cfg.max_resources);
    if (R == 0) { *n = 0; return SG_OK; }
    if (!e->d_snap_cnt) {
        HIPCHK(hipMalloc(&e->d_snap_cnt, (uint64_t)e->cfg.max_resources * 4));
        HIPCHK(hipMalloc(&e->d_snap_off, (uint64_t)e->cfg.max_resources * 4));
    }
    // out may be device memory (e.g. the buffer an RCCL all-gather sends from): the kernels write it
    // directly, no staging buffer and no host round trip
    const bool dev_out = out && is_device_ptr(out);
    if (!dev_out && cap > e->snap_cap) {
        dfree(e->d_snap_out);
        HIPCHK(hipMalloc(&e->d_snap_out, std::max<uint64_t>(cap, 1) * sizeof(sg_metric_node)));
        e->snap_cap = cap;
    }
    if (!e->d_part) { int rc = ensure_batch(e, 1); if (rc) return rc; }
    HIPCHK(launch_snapshot(e->d_minb, e->d_info, R, now_ms, e->cfg.statistic_max_rt, e->d_snap_cnt, e->d_snap_off,
                           e->d_part, e->d_small + 3, dev_out ? out : e->d_snap_out, dev_out || out ? cap : 0,
                           e->stream));
    uint32_t total = 0;
    HIPCHK(hipMemcpyAsync(&total, e->d_small + 3, 4, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    uint64_t k = std::min<uint64_t>(total, cap);
    if (k && out && !dev_out)
        HIPCHK(hipMemcpy(out, e->d_snap_out, k * sizeof(sg_metric_node), hipMemcpyDeviceToHost));
    *n = total;
    return SG_OK;
}

int sg_cluster_set_connected_count(sg_engine* e, int64_t flow_id, int32_t connected) {
    if (!e) return fail(SG_EINVAL, "null engine");
    if (int rc = drain(e)) return rc;
    // ClusterFlowRuleManager / ClusterParamFlowRuleManager.getConnectedCount: the namespace's count
    auto it = e->cmap.find(flow_id);
    auto pt = e->pmap.find(flow_id);
    if (it == e->cmap.end() && pt == e->pmap.end()) return fail(SG_ENOTFOUND, "no cluster rule with this flowId");
    if (it != e->cmap.end()) {
        e->cflows[it->second].connected = connected;
        HIPCHK(hipMemcpy(&e->d_cflow[it->second].connected, &connected, sizeof(int32_t), hipMemcpyHostToDevice));
    }
    if (pt != e->pmap.end()) {
        e->pflows[pt->second].connected = connected;
        HIPCHK(hipMemcpy(&e->d_pflow[pt->second].connected, &connected, sizeof(int32_t), hipMemcpyHostToDevice));
    }
    return SG_OK;
}

// Batched DefaultTokenService.requestToken (see cluster.hip for the device steps).
int sg_cluster_request_tokens(sg_engine* e, const sg_token_req* reqs, uint64_t n, sg_token_result* out) {
    if (!e || (n && (!reqs || !out))) return fail(SG_EINVAL, "null argument");
    if (!n) return SG_OK;
    if (n > 0x7FFFFFFFull) return fail(SG_EINVAL, "too many token requests in one call");
    if (int rc = drain(e)) return rc;
    hipStream_t st = e->stream;
    int rc = ensure_batch(e, n);  // radix-sort scratch
    if (rc) return rc;
    if (n > e->tcap) {
        dfree(e->d_treq); dfree(e->d_tres); dfree(e->d_tfidx);
        uint64_t c = std::max<uint64_t>(n, 1u << 16);
        HIPCHK(hipMalloc(&e->d_treq, c * sizeof(sg_token_req)));
        HIPCHK(hipMalloc(&e->d_tres, c * sizeof(sg_token_result)));
        HIPCHK(hipMalloc(&e->d_tfidx, c * 4));
        e->tcap = c;
    }
    if (!e->d_nslim) {
        HIPCHK(hipMalloc(&e->d_nslim, sizeof(NsLimiter)));
        NsLimiter z;
        for (int k = 0; k < NS_BUCKETS; ++k) { z.ws[k] = -1; z.cnt[k] = 0; }
        HIPCHK(hipMemcpy(e->d_nslim, &z, sizeof(z), hipMemcpyHostToDevice));
    }
    if (!e->d_ctab) {  // no cluster rule loaded yet: an empty table
        CSlot t[16];
        for (auto& x : t) { x.key = 0; x.idx = 0xFFFFFFFFu; x.pad = 0; }
        HIPCHK(hipMalloc(&e->d_ctab, sizeof(t)));
        HIPCHK(hipMemcpy(e->d_ctab, t, sizeof(t), hipMemcpyHostToDevice));
        e->ctab_mask = 15;
    }
    const uint32_t nflows = (uint32_t)e->cflows.size();
    // requests and results may be host or device memory (dist.request_tokens keeps them in HBM under RCCL)
    HIPCHK(hipMemcpyAsync(e->d_treq, reqs, n * sizeof(sg_token_req), hipMemcpyDefault, st));
    HIPCHK(hipMemsetAsync(e->d_small, 0, 4, st));
    HIPCHK(launch_tok_classify(e->d_treq, n, e->d_ctab, e->ctab_mask, e->d_tfidx, e->d_tres, e->d_small, st));
    uint32_t flags = 0;
    HIPCHK(hipMemcpyAsync(&flags, e->d_small, 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    if (flags & 1) return fail(SG_EINVAL, "token requests must be ordered by ts (the replay clock)");
    // GlobalRequestLimiter: a negative qpsAllowed stands for "no limiter registered" (tryPass -> true)
    const double allowed = e->cfg.cluster_max_allowed_qps < 0 ? 1.0 / 0.0 : (double)e->cfg.cluster_max_allowed_qps;
    // the limiter (parallel per 100 ms bucket; the drained batch slot's arrays are its scratch), then the flows
    HIPCHK(launch_tok_limiter_par(e->d_treq, n, e->d_tfidx, nflows, e->d_nslim, allowed, e->d_k0, e->d_v0, e->d_tres,
                                  e->d_flag, e->d_pos, e->d_order, e->d_prev, e->d_dec, e->d_posof, e->d_part,
                                  e->d_small + 8, launch_scan, st));
    if (nflows) {
        int bits = 1;
        while (bits < 32 && (1ull << bits) <= nflows) ++bits;  // keys 0..nflows (nflows = not for a flow)
        const int passes = (bits + 7) / 8;
        const uint32_t nblocks = (uint32_t)((n + radix_tile() - 1) / radix_tile());
        uint32_t *kin = e->d_k0, *vin = e->d_v0, *kout = e->d_k1, *vout = e->d_v1;
        for (int p = 0; p < passes; ++p) {
            HIPCHK(launch_radix_hist(kin, n, p * 8, e->d_hist, nblocks, st));
            HIPCHK(launch_scan(e->d_hist, e->d_hist, (uint64_t)nblocks * 256, e->d_part, nullptr, st));
            HIPCHK(launch_radix_scatter(kin, vin, n, p * 8, e->d_hist, nblocks, kout, vout, nullptr, st));
            std::swap(kin, kout);
            std::swap(vin, vout);
        }
        if (nflows + 1 > e->tbounds_cap) {
            dfree(e->d_tbounds);
            e->tbounds_cap = std::max<uint32_t>(nflows + 1, 1u << 12);
            HIPCHK(hipMalloc(&e->d_tbounds, (uint64_t)e->tbounds_cap * 4));
        }
        // (the decide streams are idle: every batch was drained above)
        HIPCHK(launch_tok_flow(kin, vin, n, e->d_treq, e->d_cflow, nflows, e->d_cbkt, e->cfg.cluster_exceed_count,
                               e->cfg.cluster_max_occupy_ratio, e->d_tres, e->d_tbounds, e->tok_light, e->tok_wide, st,
                               e->bin_stream[0], e->fork, e->join[0]));
    }
    HIPCHK(hipMemcpyAsync(out, e->d_tres, n * sizeof(sg_token_result), hipMemcpyDefault, st));
    HIPCHK(hipStreamSynchronize(st));
    return SG_OK;
}

// Batched DefaultTokenService.requestParamToken: the flow path's classify and namespace limiter steps on a
// derived sg_token_req view (n_values == 0 -> acquire 0 -> BAD_REQUEST), then k_ptok_flow per param flow.
int sg_cluster_request_param_tokens(sg_engine* e, const sg_param_token_req* reqs, uint64_t n, const uint64_t* values,
                                    uint64_t n_values, sg_token_result* out) {
    if (!e || (n && (!reqs || !out)) || (n_values && !values)) return fail(SG_EINVAL, "null argument");
    if (!n) return SG_OK;
    if (n > 0x7FFFFFFFull) return fail(SG_EINVAL, "too many token requests in one call");
    for (uint64_t i = 0; i < n; ++i)
        if (reqs[i].value_off > n_values || reqs[i].n_values > n_values - reqs[i].value_off)
            return fail(SG_EINVAL, "param token request values out of range");
    if (int rc = drain(e)) return rc;
    hipStream_t st = e->stream;
    int rc = ensure_batch(e, n);
    if (rc) return rc;
    if (n > e->tcap) {
        dfree(e->d_treq); dfree(e->d_tres); dfree(e->d_tfidx);
        uint64_t c = std::max<uint64_t>(n, 1u << 16);
        HIPCHK(hipMalloc(&e->d_treq, c * sizeof(sg_token_req)));
        HIPCHK(hipMalloc(&e->d_tres, c * sizeof(sg_token_result)));
        HIPCHK(hipMalloc(&e->d_tfidx, c * 4));
        e->tcap = c;
    }
    if (n > e->pcap) {
        dfree(e->d_preq);
        e->pcap = std::max<uint64_t>(n, 1u << 16);
        HIPCHK(hipMalloc(&e->d_preq, e->pcap * sizeof(sg_param_token_req)));
    }
    if (n_values > e->pvcap) {
        dfree(e->d_pvals);
        e->pvcap = std::max<uint64_t>(n_values, 1u << 16);
        HIPCHK(hipMalloc(&e->d_pvals, e->pvcap * sizeof(uint64_t)));
    }
    if (!e->d_nslim) {
        HIPCHK(hipMalloc(&e->d_nslim, sizeof(NsLimiter)));
        NsLimiter z;
        for (int k = 0; k < NS_BUCKETS; ++k) { z.ws[k] = -1; z.cnt[k] = 0; }
        HIPCHK(hipMemcpy(e->d_nslim, &z, sizeof(z), hipMemcpyHostToDevice));
    }
    if (!e->d_pftab) {  // no cluster param rule loaded yet: an empty table
        CSlot t[16];
        for (auto& x : t) { x.key = 0; x.idx = 0xFFFFFFFFu; x.pad = 0; }
        HIPCHK(hipMalloc(&e->d_pftab, sizeof(t)));
        HIPCHK(hipMemcpy(e->d_pftab, t, sizeof(t), hipMemcpyHostToDevice));
        e->pftab_mask = 15;
    }
    std::vector<sg_token_req> tq(n);
    for (uint64_t i = 0; i < n; ++i) {
        tq[i].ts = reqs[i].ts;
        tq[i].flow_id = reqs[i].flow_id;
        tq[i].acquire_count = reqs[i].n_values ? reqs[i].acquire_count : 0;  // empty params -> badRequest
        tq[i].prioritized = 0;
    }
    const uint32_t nflows = (uint32_t)e->pflows.size();
    HIPCHK(hipMemcpyAsync(e->d_treq, tq.data(), n * sizeof(sg_token_req), hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(e->d_preq, reqs, n * sizeof(sg_param_token_req), hipMemcpyHostToDevice, st));
    if (n_values) HIPCHK(hipMemcpyAsync(e->d_pvals, values, n_values * sizeof(uint64_t), hipMemcpyHostToDevice, st));
    HIPCHK(hipMemsetAsync(e->d_small, 0, 4, st));
    HIPCHK(launch_tok_classify(e->d_treq, n, e->d_pftab, e->pftab_mask, e->d_tfidx, e->d_tres, e->d_small, st));
    uint32_t flags = 0;
    HIPCHK(hipMemcpyAsync(&flags, e->d_small, 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    if (flags & 1) return fail(SG_EINVAL, "token requests must be ordered by ts (the replay clock)");
    const double allowed = e->cfg.cluster_max_allowed_qps < 0 ? 1.0 / 0.0 : (double)e->cfg.cluster_max_allowed_qps;
    HIPCHK(launch_tok_limiter(e->d_treq, n, e->d_tfidx, nflows, e->d_nslim, allowed, e->d_k0, e->d_v0, e->d_tres, st));
    if (nflows) {
        int bits = 1;
        while (bits < 32 && (1ull << bits) <= nflows) ++bits;
        const int passes = (bits + 7) / 8;
        const uint32_t nblocks = (uint32_t)((n + radix_tile() - 1) / radix_tile());
        uint32_t *kin = e->d_k0, *vin = e->d_v0, *kout = e->d_k1, *vout = e->d_v1;
        for (int p = 0; p < passes; ++p) {
            HIPCHK(launch_radix_hist(kin, n, p * 8, e->d_hist, nblocks, st));
            HIPCHK(launch_scan(e->d_hist, e->d_hist, (uint64_t)nblocks * 256, e->d_part, nullptr, st));
            HIPCHK(launch_radix_scatter(kin, vin, n, p * 8, e->d_hist, nblocks, kout, vout, nullptr, st));
            std::swap(kin, kout);
            std::swap(vin, vout);
        }
        HIPCHK(launch_ptok_flow(kin, vin, n, e->d_preq, e->d_pvals, e->d_pflow, nflows, e->d_phot, e->d_pvtab,
                                e->pv_mask, e->d_tres, e->d_small, st));
    }
    HIPCHK(hipMemcpyAsync(out, e->d_tres, n * sizeof(sg_token_result), hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(&flags, e->d_small, 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    if (flags & 2) return fail(SG_ENOMEM, "cluster param value table is full");
    return SG_OK;
}

} // extern "C"
