// Host check of the device hot-parameter map (sentinel_amd/csrc/pmap.h): the exact __host__ __device__ code
// of the LRU CacheMap operations k_lane runs, driven by random put / get / remove sequences on the CPU and
// compared after every operation with a reference LRU (std::list + hash map: ParameterMetric's CacheMap as
// the oracle restates it, oracle/sentinel_oracle.c lm_*).  Built and run by tests/test_pmap_host.py.
//
// Mode "tile" checks the residency rule k_pq (param.hip pq_map_phase) decides a tile of accesses with -- the
// leaders' recency ranks, D = r + #earlier first accesses of older or absent keys < cap, the eviction of the
// oldest untouched keys and the placement of new keys -- restated step by step on the same representation.
//
// usage: pmap_host CAP OPS KEYSPACE SEED HOTKEYS [tile]   (exit 0 = every operation matched)
#include <cstdio>
#include <cstdlib>
#include <list>
#include <string>
#include <unordered_map>
#include <vector>

#include "../sentinel_amd/csrc/pmap.h"

using namespace sg;

struct RefLru {
    size_t cap;
    std::list<uint64_t> order;  // front = most recently used
    std::unordered_map<uint64_t, std::pair<std::list<uint64_t>::iterator, int64_t>> map;
    // putIfAbsent: true if present (touched); else inserted with value 0, evicting the LRU of a full map
    bool put(uint64_t k) {
        auto it = map.find(k);
        if (it != map.end()) {
            order.erase(it->second.first);
            order.push_front(k);
            it->second.first = order.begin();
            return true;
        }
        if (map.size() >= cap) {
            map.erase(order.back());
            order.pop_back();
        }
        order.push_front(k);
        map[k] = {order.begin(), 0};
        return false;
    }
    int64_t* get(uint64_t k) {
        auto it = map.find(k);
        if (it == map.end()) return nullptr;
        order.erase(it->second.first);
        order.push_front(k);
        it->second.first = order.begin();
        return &it->second.second;
    }
    void erase(uint64_t k) {
        auto it = map.find(k);
        if (it == map.end()) return;
        order.erase(it->second.first);
        map.erase(it);
    }
};

static uint64_t rng_state = 1;
static uint64_t rnd() {
    rng_state ^= rng_state << 13; rng_state ^= rng_state >> 7; rng_state ^= rng_state << 17;
    return rng_state;
}

#include <algorithm>
#include <map>

// k_pq's tile rule for a put-only access sequence (the rule maps and the thread-count map's adds)
static int tile_mode(PMap& m, const PRef& R, RefLru& ref, long ops, uint64_t keyspace, uint64_t hot) {
    const int64_t RB = pm_rbits(m);
    const uint32_t W = (uint32_t)(RB >> 6);
    long tiles = 0, exact = 0;
    for (long done = 0; done < ops;) {
        const uint32_t na = (uint32_t)std::min<long>(1 + rnd() % std::min<uint32_t>(2048, m.cap - 1), ops - done);
        std::vector<uint64_t> key(na);
        for (auto& k : key) k = (3ull << 60) | ((hot && rnd() % 4 != 0) ? rnd() % hot : rnd() % keyspace);
        // reserve (pq_reserve): the pmap.h lane version has the same effect
        pm_reserve(m, R, na);
        const int64_t clock0 = m.clock;
        const uint32_t live0 = m.live;
        // ranks: live stamps before each ring word, stamp order from thr
        std::vector<uint32_t> wpre(W);
        const uint32_t w0 = (uint32_t)(((uint64_t)m.thr & (uint64_t)(RB - 1)) >> 6);
        uint32_t acc = 0;
        for (uint32_t l = 0; l < W; ++l) { const uint32_t w = (w0 + l) & (W - 1); wpre[w] = acc; acc += __builtin_popcountll(R.bm[w]); }
        // groups (sorted by key, then position) and their leaders' probes
        std::map<uint64_t, std::vector<uint32_t>> groups;
        for (uint32_t e = 0; e < na; ++e) groups[key[e]].push_back(e);
        std::vector<int32_t> lrank(na, -1);
        struct G { int32_t slot; bool live; int64_t st; uint32_t last; };
        std::map<uint64_t, G> gi;
        for (auto& kv : groups) {
            G g{pm_lookup(m, R.B, kv.first), false, 0, kv.second.back()};
            int32_t rank = 0x7FFFFFFF;
            if (g.slot >= 0) {
                g.st = R.B[g.slot / PM_BKT].stamp[g.slot % PM_BKT];
                g.live = pm_live(m, R.bm, g.st);
                if (g.live) {
                    const uint64_t p = (uint64_t)g.st & (uint64_t)(RB - 1);
                    const uint32_t below = wpre[p >> 6] + __builtin_popcountll(R.bm[p >> 6] & ((1ull << (p & 63)) - 1ull));
                    rank = (int32_t)(live0 - below - 1);
                }
            }
            lrank[kv.second[0]] = rank;
            gi[kv.first] = g;
        }
        // residency of every access against the reference, in tile order
        uint32_t F = 0;
        for (uint32_t e = 0; e < na; ++e) {
            bool hit = true;  // a repeat inside the tile
            const int32_t rk = lrank[e];
            if (rk != -1) {
                if (rk == 0x7FFFFFFF) hit = false;
                else if ((uint32_t)rk + F < m.cap) hit = true;
                else {
                    ++exact;
                    uint32_t d = (uint32_t)rk;
                    for (uint32_t j = 0; j < e; ++j) if (lrank[j] != -1 && lrank[j] > rk) ++d;
                    hit = d < m.cap;
                }
                ++F;
            }
            const bool rp = ref.put(key[e]);
            if (rp != hit) { printf("tile %ld access %u key %llx: tile rule %d reference %d (rank %d, F %u)\n", tiles, e,
                                    (unsigned long long)key[e], hit, rp, rk, F); return 1; }
        }
        // commit: touched keys leave their old stamps, the oldest untouched keys beyond cap are evicted, new stamps
        uint32_t nnew = 0;
        for (auto& kv : gi) { if (kv.second.live) pm_clrbit(R.bm, m, kv.second.st); else ++nnew; }
        const uint32_t E = live0 + nnew > m.cap ? live0 + nnew - m.cap : 0u;
        if (E) {
            uint32_t before = 0;
            for (uint32_t l = 0; l < W; ++l) {
                const uint32_t w = (w0 + l) & (W - 1);
                const uint32_t c = __builtin_popcountll(R.bm[w]);
                if (before < E && R.bm[w]) { uint64_t x = R.bm[w]; uint32_t k = E - before; while (x && k) { x &= x - 1; --k; } R.bm[w] = x; }
                before += c;
            }
        }
        std::vector<uint8_t> claim(m.nb * PM_BKT, 0);
        std::vector<std::pair<uint64_t, int64_t>> need;
        for (auto& kv : gi) {
            const int64_t ns = clock0 + kv.second.last;  // every event is an access here: tA(e) = e
            pm_setbit(R.bm, m, ns);
            if (kv.second.slot >= 0) { R.B[kv.second.slot / PM_BKT].stamp[kv.second.slot % PM_BKT] = ns; claim[kv.second.slot] = 1; }
            else need.push_back({kv.first, ns});
        }
        m.clock = clock0 + na;
        m.live = live0 + nnew - E;
        for (auto& nk : need) {
            uint32_t b1, b2;
            pm_buckets(m.nb, nk.first, b1, b2);
            int f1 = -1, f2 = -1, n1 = 0, n2 = 0;
            for (int j = 0; j < PM_BKT; ++j) {
                const bool fr1 = !claim[b1 * PM_BKT + j] && (R.B[b1].key[j] == PK_EMPTY || !pm_live(m, R.bm, R.B[b1].stamp[j]));
                const bool fr2 = !claim[b2 * PM_BKT + j] && (R.B[b2].key[j] == PK_EMPTY || !pm_live(m, R.bm, R.B[b2].stamp[j]));
                if (fr1) { if (f1 < 0) f1 = j; } else ++n1;
                if (fr2) { if (f2 < 0) f2 = j; } else ++n2;
            }
            const bool u1 = f1 >= 0 && (f2 < 0 || n1 <= n2);
            if (!u1 && f2 < 0) { printf("tile %ld: no free slot (displacement walk not modelled)\n", tiles); return 1; }
            const uint32_t i = u1 ? b1 * PM_BKT + f1 : b2 * PM_BKT + f2;
            claim[i] = 1;
            R.B[i / PM_BKT].key[i % PM_BKT] = nk.first;
            R.B[i / PM_BKT].stamp[i % PM_BKT] = nk.second;
        }
        if (m.live != ref.map.size()) { printf("tile %ld: live %u vs %zu\n", tiles, m.live, ref.map.size()); return 1; }
        std::vector<std::pair<int64_t, uint64_t>> dev;
        for (uint32_t b = 0; b < m.nb; ++b)
            for (int j = 0; j < PM_BKT; ++j)
                if (R.B[b].key[j] != PK_EMPTY && pm_live(m, R.bm, R.B[b].stamp[j])) dev.push_back({R.B[b].stamp[j], R.B[b].key[j]});
        if (dev.size() != ref.order.size()) { printf("tile %ld: %zu live slots vs %zu\n", tiles, dev.size(), ref.order.size()); return 1; }
        std::sort(dev.rbegin(), dev.rend());
        size_t q = 0;
        for (uint64_t kk : ref.order)
            if (dev[q++].second != kk) { printf("tile %ld: recency order differs at %zu\n", tiles, q - 1); return 1; }
        done += na;
        ++tiles;
    }
    printf("ok: tile rule, %ld ops in %ld tiles, cap %u, live %u, exact counts %ld\n", ops, tiles, m.cap, m.live, exact);
    return 0;
}

int main(int argc, char** argv) {
    const uint32_t cap = argc > 1 ? (uint32_t)atoi(argv[1]) : 16;
    const long ops = argc > 2 ? atol(argv[2]) : 200000;
    const uint64_t keyspace = argc > 3 ? strtoull(argv[3], nullptr, 10) : 64;
    rng_state = argc > 4 ? strtoull(argv[4], nullptr, 10) | 1 : 1;
    const uint64_t hot = argc > 5 ? strtoull(argv[5], nullptr, 10) : 0;
    // one map laid out as engine.cpp rebuild_pmaps does
    PMap m{};
    m.nb = std::max<uint32_t>(2u, (2u * cap + PM_BKT - 1) / PM_BKT);
    m.cap = cap;
    uint32_t k = 10;
    while ((1ull << k) < 4ull * cap + 64) ++k;
    m.rb_log2 = k;
    std::vector<PBucket> B(m.nb);
    for (auto& b : B)
        for (int j = 0; j < PM_BKT; ++j) { b.key[j] = PK_EMPTY; b.stamp[j] = -1; }
    std::vector<PData> D(m.nb * PM_BKT);
    std::vector<uint64_t> bm((1ull << k) / 64, 0);
    std::vector<uint32_t> pre((1ull << k) / 64, 0);
    PRef R{B.data(), D.data(), bm.data(), pre.data()};
    RefLru ref;
    ref.cap = cap;
    uint32_t bflags = 0;
    long compactions = 0;
    if (argc > 6 && std::string(argv[6]) == "tile") return tile_mode(m, R, ref, ops, keyspace, hot);
    for (long op = 0; op < ops; ++op) {
        // keys: a few hot ones (keep old keys alive, forcing ring compactions), the rest uniform
        const uint64_t key = (3ull << 60) | ((hot && rnd() % 4 != 0) ? rnd() % hot : rnd() % keyspace);
        const int kind = (int)(rnd() % 10);  // 0-5 put, 6-7 get, 8-9 thread-count decrement (erase at <= 0)
        const int64_t span0 = m.clock - m.thr;
        if (kind <= 5) {
            bool present;
            const int32_t i = pm_put(m, R, key, &present, &bflags);
            const bool rp = ref.put(key);
            if (present != rp) { printf("op %ld put %llx: device present=%d ref=%d\n", op, (unsigned long long)key, present, rp); return 1; }
            if (!rp) ref.map[key].second = 1;
            else ref.map[key].second += 1;
            D[i].v0 = present ? D[i].v0 + 1 : 1;
        } else if (kind <= 7) {
            const int32_t i = pm_get(m, R, key);
            int64_t* rv = ref.get(key);
            if ((i >= 0) != (rv != nullptr)) { printf("op %ld get %llx: device %d ref %d\n", op, (unsigned long long)key, i >= 0, rv != nullptr); return 1; }
            if (rv && D[i].v0 != *rv) { printf("op %ld get: value %lld vs %lld\n", op, (long long)D[i].v0, (long long)*rv); return 1; }
        } else {  // decreaseThreadCount: putIfAbsent(v, 0); present -> decrement, removed at <= 0
            bool present;
            const int32_t i = pm_put(m, R, key, &present, &bflags);
            const bool rp = ref.put(key);
            if (present != rp) { printf("op %ld dec %llx: device present=%d ref=%d\n", op, (unsigned long long)key, present, rp); return 1; }
            if (!present) { D[i].v0 = 0; ref.map[key].second = 0; }
            else {
                const int64_t c = D[i].v0 - 1;
                if (c <= 0) { pm_erase(m, R, i); ref.erase(key); }
                else { D[i].v0 = c; ref.map[key].second = c; }
            }
        }
        if (span0 > (int64_t)m.live + 64 && m.clock - m.thr <= (int64_t)m.live) ++compactions;  // pm_compact ran
        if (m.live != ref.map.size()) { printf("op %ld: live %u vs %zu\n", op, m.live, ref.map.size()); return 1; }
        if (op % 997 == 0) {  // the live key set and its recency order
            std::vector<std::pair<int64_t, uint64_t>> dev;
            for (uint32_t b = 0; b < m.nb; ++b)
                for (int j = 0; j < PM_BKT; ++j)
                    if (B[b].key[j] != PK_EMPTY && pm_live(m, bm.data(), B[b].stamp[j])) dev.push_back({B[b].stamp[j], B[b].key[j]});
            if (dev.size() != ref.order.size()) { printf("op %ld: %zu live slots vs %zu\n", op, dev.size(), ref.order.size()); return 1; }
            std::sort(dev.rbegin(), dev.rend());
            size_t q = 0;
            for (uint64_t kk : ref.order)
                if (dev[q++].second != kk) { printf("op %ld: recency order differs at %zu\n", op, q - 1); return 1; }
        }
    }
    if (bflags) { printf("bflags %x\n", bflags); return 1; }
    printf("ok: %ld ops, cap %u, live %u, clock %lld, compactions %ld\n", ops, cap, m.live, (long long)m.clock, compactions);
    return 0;
}
