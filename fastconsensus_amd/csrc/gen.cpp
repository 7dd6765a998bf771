// gen.cpp -- host C++ utilities that feed the engine: LFR-like and SBM synthetic graphs
// (benchmark inputs) and a native edge-list parser (replaces
// nx.read_edgelist(f, nodetype=int), fast_consensus.py:434).  Not on the device path.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <numeric>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/fastconsensus_amd.h"

namespace fc {
void set_error(const std::string& msg);
}

namespace {

struct Rng {
    uint64_t s;
    explicit Rng(uint64_t seed) : s(seed * 0x9E3779B97F4A7C15ull + 0x632BE59BD9B4E019ull) {}
    uint64_t next() {
        uint64_t z = (s += 0x9E3779B97F4A7C15ull);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    }
    double uni() { return (next() >> 11) * (1.0 / 9007199254740992.0); }
    uint64_t below(uint64_t n) { return (uint64_t)(((unsigned __int128)next() * n) >> 64); }
};

// Continuous power law p(x) ~ x^-g on [a, b], sampled by inverse CDF.
double powerlaw(Rng& r, double g, double a, double b) {
    const double u = r.uni();
    if (std::fabs(g - 1.0) < 1e-12) return a * std::pow(b / a, u);
    const double e = 1.0 - g;
    return std::pow(std::pow(a, e) + u * (std::pow(b, e) - std::pow(a, e)), 1.0 / e);
}
double powerlaw_mean(double g, double a, double b) {
    // E[x] of the continuous law on [a,b]
    const double e1 = 1.0 - g, e2 = 2.0 - g;
    const double z = (std::pow(b, e1) - std::pow(a, e1)) / e1;
    const double m = (std::fabs(e2) < 1e-12) ? std::log(b / a) : (std::pow(b, e2) - std::pow(a, e2)) / e2;
    return m / z;
}

inline uint64_t key(int32_t a, int32_t b) {
    const uint32_t u = (uint32_t)std::min(a, b), v = (uint32_t)std::max(a, b);
    return ((uint64_t)u << 32) | v;
}

// pair a shuffled stub list; emits candidate edges (self loops dropped later)
void pair_stubs(std::vector<int32_t>& stubs, Rng& r, std::vector<uint64_t>& out,
                const std::vector<int32_t>* comm_of) {
    for (size_t i = stubs.size(); i > 1; --i) std::swap(stubs[i - 1], stubs[r.below(i)]);
    for (size_t i = 0; i + 1 < stubs.size(); i += 2) {
        const int32_t a = stubs[i], b = stubs[i + 1];
        if (a == b) continue;
        if (comm_of && (*comm_of)[a] == (*comm_of)[b]) continue;  // external stub pairs only
        out.push_back(key(a, b));
    }
}

}  // namespace

extern "C" {

int fc_generate_lfr(int64_t n, double tau1, double tau2, double mu, double avg_deg, int32_t max_deg,
                    int32_t min_comm, int32_t max_comm, uint64_t seed, int64_t m_cap, int32_t* u, int32_t* v,
                    int64_t* m_out, int32_t* planted) {
    if (n < 2 || n >= (int64_t(1) << 31) || mu < 0 || mu > 1 || avg_deg <= 0 || max_deg < 1 || min_comm < 2 ||
        max_comm < min_comm || !m_out) {
        fc::set_error("fc_generate_lfr: bad arguments");
        return FC_EINVAL;
    }
    Rng r(seed);
    // 1. degrees: power law tau1 on [kmin, max_deg], kmin solved so the mean is avg_deg
    double lo = 1.0, hi = (double)max_deg;
    if (powerlaw_mean(tau1, hi - 1e-9, (double)max_deg) < avg_deg) lo = hi - 1e-9;
    for (int it = 0; it < 100; ++it) {
        const double mid = 0.5 * (lo + hi);
        if (powerlaw_mean(tau1, mid, (double)max_deg) < avg_deg) lo = mid; else hi = mid;
    }
    const double kmin = 0.5 * (lo + hi);
    std::vector<int32_t> deg(n), kin(n);
    for (int64_t i = 0; i < n; ++i) {
        int32_t d = (int32_t)std::lround(powerlaw(r, tau1, kmin, (double)max_deg));
        deg[i] = std::max(1, std::min(d, max_deg));
        kin[i] = (int32_t)std::lround((1.0 - mu) * deg[i]);
    }
    // 2. community sizes: power law tau2 on [min_comm, max_comm] until they cover n
    std::vector<int64_t> sizes;
    int64_t tot = 0;
    while (tot < n) {
        int64_t s = std::lround(powerlaw(r, tau2, (double)min_comm, (double)max_comm));
        s = std::max<int64_t>(min_comm, std::min<int64_t>(s, max_comm));
        sizes.push_back(s);
        tot += s;
    }
    int64_t excess = tot - n;  // shave the excess off communities above min_comm
    for (size_t i = 0; excess > 0 && i < sizes.size(); ++i) {
        const int64_t take = std::min<int64_t>(excess, sizes[i] - min_comm);
        sizes[i] -= take;
        excess -= take;
    }
    if (excess > 0) sizes.back() -= excess;
    const int64_t C = (int64_t)sizes.size();
    // 3. assign nodes (largest internal degree first) to communities with room and size > kin
    std::vector<int32_t> order(n);
    std::iota(order.begin(), order.end(), 0);
    for (int64_t i = n; i > 1; --i) std::swap(order[i - 1], order[r.below(i)]);
    std::stable_sort(order.begin(), order.end(), [&](int32_t a, int32_t b) { return kin[a] > kin[b]; });
    std::vector<int64_t> room(sizes.begin(), sizes.end());
    std::vector<int32_t> comm(n, -1);
    std::vector<int32_t> cidx(C);
    std::iota(cidx.begin(), cidx.end(), 0);
    std::sort(cidx.begin(), cidx.end(), [&](int32_t a, int32_t b) { return sizes[a] > sizes[b]; });
    for (int32_t node : order) {
        // random probes first, then a scan over communities by decreasing size
        int32_t pick = -1;
        for (int t = 0; t < 32 && pick < 0; ++t) {
            const int32_t cc = (int32_t)r.below(C);
            if (room[cc] > 0 && sizes[cc] > kin[node]) pick = cc;
        }
        for (int64_t j = 0; j < C && pick < 0; ++j)
            if (room[cidx[j]] > 0) pick = cidx[j];
        comm[node] = pick;
        room[pick]--;
        if (kin[node] >= sizes[pick]) kin[node] = (int32_t)sizes[pick] - 1;
    }
    // 4. wire: internal configuration model per community, then external stubs globally
    std::vector<std::vector<int32_t>> members(C);
    for (int64_t i = 0; i < n; ++i) members[comm[i]].push_back((int32_t)i);
    std::vector<uint64_t> edges;
    edges.reserve((size_t)(n * avg_deg / 2 * 1.05));
    std::vector<int32_t> stubs;
    for (int64_t cc = 0; cc < C; ++cc) {
        stubs.clear();
        for (int32_t x : members[cc])
            for (int32_t k = 0; k < kin[x]; ++k) stubs.push_back(x);
        pair_stubs(stubs, r, edges, nullptr);
    }
    stubs.clear();
    for (int64_t i = 0; i < n; ++i)
        for (int32_t k = kin[i]; k < deg[i]; ++k) stubs.push_back((int32_t)i);
    pair_stubs(stubs, r, edges, &comm);
    std::sort(edges.begin(), edges.end());
    edges.erase(std::unique(edges.begin(), edges.end()), edges.end());
    // emit in a random order (the generator order must not leak structure into node order)
    for (size_t i = edges.size(); i > 1; --i) std::swap(edges[i - 1], edges[r.below(i)]);
    const int64_t m = (int64_t)edges.size();
    *m_out = m;
    if (u && v) {
        if (m > m_cap) {
            fc::set_error("fc_generate_lfr: m_cap too small");
            return FC_ELIMIT;
        }
        for (int64_t i = 0; i < m; ++i) {
            u[i] = (int32_t)(edges[i] >> 32);
            v[i] = (int32_t)(edges[i] & 0xffffffffu);
        }
    }
    if (planted)
        for (int64_t i = 0; i < n; ++i) planted[i] = comm[i];
    return FC_OK;
}

int fc_generate_sbm(int64_t n, int32_t block_size, double deg_in, double deg_out, uint64_t seed, int64_t m_cap,
                    int32_t* u, int32_t* v, int64_t* m_out) {
    if (n < 2 || block_size < 2 || n % block_size != 0 || !m_out) {
        fc::set_error("fc_generate_sbm: bad arguments (n must be a multiple of block_size)");
        return FC_EINVAL;
    }
    Rng r(seed ^ 0x5b5b5b5bull);
    const int64_t B = n / block_size;
    std::vector<uint64_t> edges;
    const int64_t m_in = std::llround(n * deg_in / 2.0), m_out_e = std::llround(n * deg_out / 2.0);
    edges.reserve((size_t)(m_in + m_out_e));
    for (int64_t i = 0; i < m_in; ++i) {  // uniform pairs inside a uniform block
        const int64_t b = (int64_t)r.below(B);
        const int32_t a = (int32_t)(b * block_size + (int64_t)r.below(block_size));
        const int32_t c = (int32_t)(b * block_size + (int64_t)r.below(block_size));
        if (a != c) edges.push_back(key(a, c));
    }
    for (int64_t i = 0; i < m_out_e; ++i) {
        const int32_t a = (int32_t)r.below(n), c = (int32_t)r.below(n);
        if (a / block_size != c / block_size) edges.push_back(key(a, c));
    }
    std::sort(edges.begin(), edges.end());
    edges.erase(std::unique(edges.begin(), edges.end()), edges.end());
    for (size_t i = edges.size(); i > 1; --i) std::swap(edges[i - 1], edges[r.below(i)]);
    const int64_t m = (int64_t)edges.size();
    *m_out = m;
    if (u && v) {
        if (m > m_cap) {
            fc::set_error("fc_generate_sbm: m_cap too small");
            return FC_ELIMIT;
        }
        for (int64_t i = 0; i < m; ++i) {
            u[i] = (int32_t)(edges[i] >> 32);
            v[i] = (int32_t)(edges[i] & 0xffffffffu);
        }
    }
    return FC_OK;
}

// Two-phase parser: sizes first (labels/u/v NULL), then fill.  Node order = first
// appearance in the file, as nx.read_edgelist builds it; '#' starts a comment.
int fc_read_edgelist(const char* path, int64_t* n_out, int64_t* m_out, int64_t* labels, int32_t* u,
                     int32_t* v) {
    FILE* f = std::fopen(path, "rb");
    if (!f) {
        fc::set_error(std::string("cannot open ") + (path ? path : "(null)"));
        return FC_EINVAL;
    }
    std::unordered_map<int64_t, int32_t> id;
    std::vector<int64_t> order;
    int64_t m = 0;
    char line[4096];
    int rc = FC_OK;
    int64_t lineno = 0;
    while (std::fgets(line, sizeof line, f)) {
        ++lineno;
        char* p = line;
        char* hash = std::strchr(p, '#');
        if (hash) *hash = 0;
        char* end;
        while (*p == ' ' || *p == '\t') ++p;
        if (*p == 0 || *p == '\n' || *p == '\r') continue;
        const long long a = std::strtoll(p, &end, 10);
        if (end == p) { rc = FC_EINVAL; break; }
        p = end;
        const long long b = std::strtoll(p, &end, 10);
        if (end == p) {
            if (*p == 0 || *p == '\n' || *p == '\r' || *p == ' ' || *p == '\t') continue;  // <2 columns: skipped
            rc = FC_EINVAL;
            break;
        }
        int32_t ia, ib;
        auto ita = id.find(a);
        if (ita == id.end()) { ia = (int32_t)order.size(); id.emplace(a, ia); order.push_back(a); } else ia = ita->second;
        auto itb = id.find(b);
        if (itb == id.end()) { ib = (int32_t)order.size(); id.emplace(b, ib); order.push_back(b); } else ib = itb->second;
        if (u && v) { u[m] = ia; v[m] = ib; }
        ++m;
    }
    std::fclose(f);
    if (rc != FC_OK) {
        fc::set_error("fc_read_edgelist: line " + std::to_string(lineno) + " is not an integer edge");
        return rc;
    }
    if (n_out) *n_out = (int64_t)order.size();
    if (m_out) *m_out = m;
    if (labels) std::memcpy(labels, order.data(), sizeof(int64_t) * order.size());
    return FC_OK;
}

}  // extern "C"
