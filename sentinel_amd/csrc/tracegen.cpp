// tracegen.cpp -- seeded synthetic Sentinel workloads (north_star's
// >= 1M resources with mixed flow / degrade / param rules).
//
// Host-only C++ (no GPU).  Produces the resource names, the rules of each
// config and a time-ordered sg_event trace; bench.py and the tests hand the
// buffers straight to sg_submit / the oracle.  Everything is a deterministic
// function of (config, seed, sizes): xoshiro256** seeded by splitmix64, Zipf via
// Walker alias tables, exponential RT with mean 20 ms clipped at 4900 ms.
//
// Trace model (open loop): entries arrive as a Poisson stream
// at `rate` entries/s; every entry gets an EXIT at t + RT that refers to it
// (SG_AUX_EXIT(ref, rt)), and C4 entries get a TRACE with p = 0.05 just before
// their exit.  EXIT/TRACE of an entry that was blocked are no-ops in both the
// engine and the oracle, which is exactly what CtSph does when it exits a
// blocked entry internally (core/CtSph.java:157-162).  Within one millisecond
// the order is: entries, traces, exits.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/sentinel_gpu.h"

namespace {

struct Rng {
    uint64_t s[4];
    static uint64_t splitmix(uint64_t& x) {
        uint64_t z = (x += 0x9e3779b97f4a7c15ULL);
        z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
        z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
        return z ^ (z >> 31);
    }
    explicit Rng(uint64_t seed) {
        uint64_t x = seed;
        for (auto& v : s) v = splitmix(x);
    }
    static uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
    uint64_t next() {
        uint64_t r = rotl(s[1] * 5, 7) * 9, t = s[1] << 17;
        s[2] ^= s[0]; s[3] ^= s[1]; s[1] ^= s[2]; s[0] ^= s[3]; s[2] ^= t; s[3] = rotl(s[3], 45);
        return r;
    }
    double uniform() { return (next() >> 11) * (1.0 / 9007199254740992.0); }        // [0,1)
    double uniform_pos() { return ((next() >> 11) + 1) * (1.0 / 9007199254740993.0); } // (0,1]
    uint64_t below(uint64_t n) { return n ? next() % n : 0; }
};

// Walker alias table for Zipf(s) over ranks 0..n-1 (P(k) ~ (k+1)^-s)
struct Alias {
    std::vector<float> prob;
    std::vector<uint32_t> alias;
    void build(uint64_t n, double s) {
        std::vector<double> p(n);
        double sum = 0;
        for (uint64_t k = 0; k < n; ++k) { p[k] = std::pow((double)(k + 1), -s); sum += p[k]; }
        prob.assign(n, 0); alias.assign(n, 0);
        std::vector<uint32_t> small, large;
        small.reserve(n); large.reserve(n);
        for (uint64_t k = 0; k < n; ++k) {
            p[k] = p[k] * n / sum;
            (p[k] < 1.0 ? small : large).push_back((uint32_t)k);
        }
        while (!small.empty() && !large.empty()) {
            uint32_t a = small.back(); small.pop_back();
            uint32_t b = large.back();
            prob[a] = (float)p[a]; alias[a] = b;
            p[b] = (p[b] + p[a]) - 1.0;
            if (p[b] < 1.0) { large.pop_back(); small.push_back(b); }
        }
        for (uint32_t a : large) { prob[a] = 1.0f; alias[a] = a; }
        for (uint32_t a : small) { prob[a] = 1.0f; alias[a] = a; }
    }
    uint32_t sample(Rng& r) const {
        uint64_t k = r.below(prob.size());
        return r.uniform() < prob[k] ? (uint32_t)k : alias[k];
    }
};

struct Workload {
    int config = 0;
    std::vector<std::string> name_store;
    std::vector<const char*> names;
    std::vector<sg_flow_rule> flow;
    std::vector<sg_degrade_rule> degrade;
    std::vector<sg_param_rule> param;
    std::vector<sg_event> events;
    uint64_t n_entries = 0;
    int64_t t0 = 0, t_end = 0;
    std::string la_default = "default";
    // hot items of the param rules (variant TG_V_HOT): the strings the sg_param_item pointers name
    std::vector<std::string> item_text;
    std::vector<std::vector<sg_param_item>> items;
};

// trace variants (tg_create `variant` bits), on top of the SURVEY.md configs:
enum : uint32_t {
    TG_V_WARM_RL = 1,   // C3: a fifth of the flow rules become WarmUpRateLimiter (control behaviour 3)
    TG_V_HOT = 2,       // C5: every param rule gets 3 hot items (popular values, counts 0..19)
    TG_V_THREAD = 4,    // C5: a fifth of the param rules are THREAD grade; every EXIT releases its ENTRY's
                        // argument (Entry.exit(count, args): SG_F_EXIT_ARGS)
    TG_V_UNIFORM = 8    // C5: half of the parameter values uniform over n_param_values, half Zipf(1.1): many
                        // distinct values churn the maps while the popular ones repeat (and get blocked)
};

sg_flow_rule flow_default(const char* res, double count) {
    sg_flow_rule r;
    std::memset(&r, 0, sizeof(r));
    r.resource = res;
    r.limit_app = "default";
    r.count = count;
    r.grade = SG_FLOW_GRADE_QPS;
    r.strategy = SG_STRATEGY_DIRECT;
    r.control_behavior = SG_CONTROL_BEHAVIOR_DEFAULT;
    r.warm_up_period_sec = 10;
    r.max_queueing_time_ms = 500;
    r.cluster_threshold_type = SG_CLUSTER_THRESHOLD_AVG_LOCAL;
    r.cluster_fallback_to_local = 1;
    r.cluster_sample_count = 10;
    r.cluster_window_interval_ms = 1000;
    return r;
}

double log_uniform(Rng& r, double lo, double hi) {
    return std::floor(std::exp(std::log(lo) + r.uniform() * (std::log(hi) - std::log(lo))));
}

// Raw, unsorted event with its final-order key.
struct Raw {
    uint64_t key;      // (ms - t0) * 4 + kind_rank
    uint64_t entry_id; // entries: own id; exit/trace: referenced entry id
    uint32_t res;
    uint16_t count;
    uint8_t kind;
    uint8_t flags;
    uint64_t aux;      // entry: param key; exit: rt
};

void finalize(Workload& w, std::vector<Raw>& raw) {
    // counting sort by key (stable): entries (rank 0) < traces (1) < exits (2) within a ms
    uint64_t max_key = 0;
    for (auto& x : raw) max_key = std::max(max_key, x.key);
    std::vector<uint64_t> cnt(max_key + 2, 0);
    for (auto& x : raw) cnt[x.key + 1]++;
    for (size_t i = 1; i < cnt.size(); ++i) cnt[i] += cnt[i - 1];
    std::vector<uint64_t> pos(raw.size());
    for (size_t i = 0; i < raw.size(); ++i) pos[i] = cnt[raw[i].key]++;
    // final index of every entry
    std::vector<uint64_t> entry_pos(w.n_entries, SG_REF_NONE);
    for (size_t i = 0; i < raw.size(); ++i)
        if (raw[i].kind == SG_EV_ENTRY) entry_pos[raw[i].entry_id] = pos[i];
    w.events.resize(raw.size());
    for (size_t i = 0; i < raw.size(); ++i) {
        const Raw& x = raw[i];
        sg_event& e = w.events[pos[i]];
        e.ts = w.t0 + (int64_t)(x.key >> 2);
        e.res_id = x.res;
        e.count = x.count;
        e.kind = x.kind;
        e.flags = x.flags;
        if (x.kind == SG_EV_ENTRY) e.aux = x.aux;
        else if (x.kind == SG_EV_EXIT) e.aux = SG_AUX_EXIT(entry_pos[x.entry_id], x.aux);
        else e.aux = entry_pos[x.entry_id] & SG_REF_NONE;
    }
}

int64_t exp_rt(Rng& r) {
    double v = -20.0 * std::log(r.uniform_pos());
    int64_t rt = (int64_t)v;
    return rt > 4900 ? 4900 : rt;
}

// C1: FlowQpsDemo (sentinel-demo-basic .../flow/FlowQpsDemo.java:37-160): 32 threads,
// entry -> exit in the same ms -> sleep U{0..49}, for `seconds` seconds.
void gen_c1(Workload& w, uint64_t seed, int seconds) {
    Rng rng(seed);
    w.name_store = {"abc"};
    w.names = {w.name_store[0].c_str()};
    w.flow.push_back(flow_default(w.names[0], 20));
    std::vector<Raw> raw;
    uint64_t id = 0;
    for (int th = 0; th < 32; ++th) {
        int64_t t = rng.below(50);
        while (t < (int64_t)seconds * 1000) {
            Raw e{(uint64_t)t * 4 + 0, id, 0, 1, SG_EV_ENTRY, 0, 0};
            Raw x{(uint64_t)t * 4 + 2, id, 0, 1, SG_EV_EXIT, 0, 0};
            raw.push_back(e);
            raw.push_back(x);
            ++id;
            t += (int64_t)rng.below(50);
        }
    }
    // entry ids must follow the final order of entries for readability: re-key by time
    std::stable_sort(raw.begin(), raw.end(), [](const Raw& a, const Raw& b) { return a.key < b.key; });
    uint64_t k = 0;
    std::vector<uint64_t> remap(id);
    for (auto& x : raw) if (x.kind == SG_EV_ENTRY) remap[x.entry_id] = k++;
    for (auto& x : raw) x.entry_id = remap[x.entry_id];
    w.n_entries = id;
    w.t_end = w.t0 + (int64_t)seconds * 1000;
    finalize(w, raw);
}

// C2-C6: Zipf(1.1) resources, Poisson arrivals at `rate` entries/s.
void gen_zipf(Workload& w, int config, uint64_t seed, uint32_t n_res, uint64_t n_entries, double rate,
              uint64_t n_param_values, uint32_t variant) {
    Rng rng(seed);
    w.name_store.resize(n_res);
    w.names.resize(n_res);
    for (uint32_t i = 0; i < n_res; ++i) {
        char buf[32];
        std::snprintf(buf, sizeof(buf), "res-%u", i);
        w.name_store[i] = buf;
    }
    for (uint32_t i = 0; i < n_res; ++i) w.names[i] = w.name_store[i].c_str();

    // rules
    for (uint32_t i = 0; i < n_res; ++i) {
        const char* nm = w.names[i];
        if (config == 2) {
            w.flow.push_back(flow_default(nm, log_uniform(rng, 10, 1e4)));
        } else if (config == 3) {
            double u = rng.uniform();
            sg_flow_rule r = flow_default(nm, log_uniform(rng, 10, 1e4));
            if (u < 0.4) {
            } else if (u < 0.6) {
                r.grade = SG_FLOW_GRADE_THREAD;
                r.count = (double)(4 + rng.below(61));
            } else if (u < 0.8) {
                r.control_behavior = SG_CONTROL_BEHAVIOR_WARM_UP;
                r.warm_up_period_sec = 10;
            } else if ((variant & TG_V_WARM_RL) && u < 0.9) {
                r.control_behavior = SG_CONTROL_BEHAVIOR_WARM_UP_RATE_LIMITER;
                r.warm_up_period_sec = 10;
                r.max_queueing_time_ms = 500;
            } else {
                r.control_behavior = SG_CONTROL_BEHAVIOR_RATE_LIMITER;
                r.max_queueing_time_ms = 500;
            }
            w.flow.push_back(r);
        } else if (config == 4) {
            w.flow.push_back(flow_default(nm, log_uniform(rng, 10, 1e4)));
            sg_degrade_rule d;
            std::memset(&d, 0, sizeof(d));
            d.resource = nm;
            d.limit_app = "default";
            d.time_window = 10;
            switch (i % 3) {
            case 0: d.grade = SG_DEGRADE_GRADE_RT; d.count = 50; break;
            case 1: d.grade = SG_DEGRADE_GRADE_EXCEPTION_RATIO; d.count = 0.2; break;
            default: d.grade = SG_DEGRADE_GRADE_EXCEPTION_COUNT; d.count = 20; break;
            }
            w.degrade.push_back(d);
        } else if (config == 6) {  // C4's flow + degrade rules and a C5-style QPS param rule on args[0]
            w.flow.push_back(flow_default(nm, log_uniform(rng, 10, 1e4)));
            sg_degrade_rule d;
            std::memset(&d, 0, sizeof(d));
            d.resource = nm;
            d.limit_app = "default";
            d.time_window = 10;
            switch (i % 3) {
            case 0: d.grade = SG_DEGRADE_GRADE_RT; d.count = 50; break;
            case 1: d.grade = SG_DEGRADE_GRADE_EXCEPTION_RATIO; d.count = 0.2; break;
            default: d.grade = SG_DEGRADE_GRADE_EXCEPTION_COUNT; d.count = 20; break;
            }
            w.degrade.push_back(d);
            sg_param_rule p;
            std::memset(&p, 0, sizeof(p));
            p.resource = nm;
            p.limit_app = "default";
            p.count = (double)(5 + rng.below(46));
            p.duration_in_sec = 1;
            p.grade = SG_FLOW_GRADE_QPS;
            p.param_idx = 0;
            p.has_param_idx = 1;
            p.burst_count = (int32_t)rng.below(6);
            p.cluster_sample_count = 10;
            p.cluster_window_interval_ms = 1000;
            w.param.push_back(p);
        } else if (config == 5) {
            sg_param_rule p;
            std::memset(&p, 0, sizeof(p));
            p.resource = nm;
            p.limit_app = "default";
            p.count = (double)(5 + rng.below(46));
            p.duration_in_sec = 1;
            p.grade = SG_FLOW_GRADE_QPS;
            p.param_idx = 0;
            p.has_param_idx = 1;
            p.burst_count = (int32_t)rng.below(6);
            if (rng.uniform() < 0.2) {
                p.control_behavior = SG_CONTROL_BEHAVIOR_RATE_LIMITER;
                p.max_queueing_time_ms = 100;
            }
            if ((variant & TG_V_THREAD) && rng.uniform() < 0.2) {
                p.grade = SG_FLOW_GRADE_THREAD;
                p.control_behavior = SG_CONTROL_BEHAVIOR_DEFAULT;
                p.count = (double)(3 + rng.below(8));
            }
            p.cluster_sample_count = 10;
            p.cluster_window_interval_ms = 1000;
            w.param.push_back(p);
        }
    }

    // popularity: Zipf rank -> random resource id
    Alias za;
    za.build(n_res, 1.1);
    std::vector<uint32_t> perm(n_res);
    for (uint32_t i = 0; i < n_res; ++i) perm[i] = i;
    for (uint32_t i = n_res; i > 1; --i) std::swap(perm[i - 1], perm[rng.below(i)]);
    Alias pa;
    std::vector<uint64_t> pkey;
    if (config == 5 || config == 6) {
        pa.build(n_param_values, 1.1);
        pkey.resize(n_param_values);
        Rng kr(seed ^ 0x5eed5eedULL);
        for (uint64_t i = 0; i < n_param_values; ++i) pkey[i] = (3ULL << 60) | (kr.next() & ((1ULL << 59) - 1)); // Long keys
        if (variant & TG_V_HOT) {  // hot items: three of the 16 most popular values, as ("<long>", "long")
            Rng hr(seed ^ 0x407e11ULL);
            w.items.resize(w.param.size());
            w.item_text.reserve(w.param.size() * 3);
            for (size_t k = 0; k < w.param.size(); ++k) {
                for (int j = 0; j < 3; ++j) {
                    const uint64_t v = pkey[hr.below(std::min<uint64_t>(16, n_param_values))] & ((1ULL << 59) - 1);
                    w.item_text.push_back(std::to_string(v));
                }
            }
            for (size_t k = 0; k < w.param.size(); ++k) {
                for (int j = 0; j < 3; ++j) {
                    sg_param_item it;
                    std::memset(&it, 0, sizeof(it));
                    it.object = w.item_text[3 * k + j].c_str();
                    it.class_type = "long";
                    it.count = (int32_t)hr.below(20);
                    it.has_count = 1;
                    w.items[k].push_back(it);
                }
                w.param[k].items = w.items[k].data();
                w.param[k].n_items = 3;
            }
        }
    }
    const uint8_t exit_flags = (config == 5 && (variant & TG_V_THREAD)) ? SG_F_EXIT_ARGS : 0;

    std::vector<Raw> raw;
    raw.reserve(n_entries * (config == 4 || config == 6 ? 21 : 20) / 10);
    double t_us = 0;
    const double mean_gap_us = 1e6 / rate;
    for (uint64_t i = 0; i < n_entries; ++i) {
        t_us += -mean_gap_us * std::log(rng.uniform_pos());
        uint64_t ms = (uint64_t)(t_us / 1000.0);
        uint32_t res = perm[za.sample(rng)];
        Raw e{ms * 4 + 0, i, res, 1, SG_EV_ENTRY, 0, 0};
        if (config == 5 || config == 6) {
            e.flags = SG_F_HAS_ARG;
            e.aux = pkey[(variant & TG_V_UNIFORM) && rng.uniform() < 0.5 ? rng.below(n_param_values) : pa.sample(rng)];
        }
        raw.push_back(e);
        int64_t rt = exp_rt(rng);
        uint64_t xms = ms + (uint64_t)rt;
        if ((config == 4 || config == 6) && rng.uniform() < 0.05) raw.push_back(Raw{xms * 4 + 1, i, res, 1, SG_EV_TRACE, 0, 0});
        raw.push_back(Raw{xms * 4 + 2, i, res, 1, SG_EV_EXIT, exit_flags, (uint64_t)rt});
    }
    w.n_entries = n_entries;
    w.t_end = w.t0 + (int64_t)(t_us / 1000.0) + 1;
    finalize(w, raw);
}

} // namespace

extern "C" {

typedef struct tg_workload tg_workload;

// config 1..6; n_res/n_entries/rate = 0 pick the SURVEY.md defaults.
tg_workload* tg_create(int config, uint64_t seed, uint32_t n_res, uint64_t n_entries, double rate, int64_t t0,
                       uint64_t n_param_values, uint32_t variant) {
    Workload* w = new Workload();
    w->config = config;
    w->t0 = t0 ? t0 : 1700000000000LL;
    if (config == 1) {
        gen_c1(*w, seed, n_entries ? (int)n_entries : 100);
    } else {
        uint32_t dres = config == 2 ? 10000 : config == 3 ? 100000 : (config == 4 || config == 6) ? 1000000 : 10000;
        gen_zipf(*w, config, seed, n_res ? n_res : dres, n_entries ? n_entries : 100000000ULL,
                 rate > 0 ? rate : 1e6, n_param_values ? n_param_values : 10000000ULL, variant);
    }
    return reinterpret_cast<tg_workload*>(w);
}

void tg_destroy(tg_workload* h) { delete reinterpret_cast<Workload*>(h); }

const char* const* tg_names(tg_workload* h, uint32_t* n) {
    Workload* w = reinterpret_cast<Workload*>(h);
    *n = (uint32_t)w->names.size();
    return w->names.data();
}
const sg_flow_rule* tg_flow_rules(tg_workload* h, uint32_t* n) {
    Workload* w = reinterpret_cast<Workload*>(h);
    *n = (uint32_t)w->flow.size();
    return w->flow.data();
}
const sg_degrade_rule* tg_degrade_rules(tg_workload* h, uint32_t* n) {
    Workload* w = reinterpret_cast<Workload*>(h);
    *n = (uint32_t)w->degrade.size();
    return w->degrade.data();
}
const sg_param_rule* tg_param_rules(tg_workload* h, uint32_t* n) {
    Workload* w = reinterpret_cast<Workload*>(h);
    *n = (uint32_t)w->param.size();
    return w->param.data();
}
const sg_event* tg_events(tg_workload* h, uint64_t* n) {
    Workload* w = reinterpret_cast<Workload*>(h);
    *n = w->events.size();
    return w->events.data();
}
uint64_t tg_n_entries(tg_workload* h) { return reinterpret_cast<Workload*>(h)->n_entries; }
int64_t tg_t_end(tg_workload* h) { return reinterpret_cast<Workload*>(h)->t_end; }

} // extern "C"
