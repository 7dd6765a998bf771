// graph.hip -- device-resident graph: ingest (replaces nx.read_edgelist + G.copy() +
// weight reset, fast_consensus.py:131-136, :434), deterministic CSR build, and the
// merge that turns nextgraph into graph (fast_consensus.py:198, :307).
#include <hipcub/hipcub.hpp>
#include <rocprim/device/device_merge.hpp>
#include <rocprim/iterator/discard_iterator.hpp>

#include "fc_ctx.h"
#include "fc_device.h"

#include <chrono>
#include <cstdio>

namespace fc {

static constexpr int TB = 256;
static inline unsigned nblk(int64_t n, int tb = TB) {
    int64_t b = (n + tb - 1) / tb;
    if (b < 1) b = 1;
    return (unsigned)b;
}

// ------------------------------------------------------------------ hipcub wrappers
template <class K, class V>
static void sort_pairs(Ctx& c, const K* kin, K* kout, const V* vin, V* vout, int64_t n, int end_bit) {
    if (n <= 0) return;
    size_t tmp = 0;
    FC_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp, kin, kout, vin, vout, (int)n, 0, end_bit, c.stream));
    c.sort_tmp.ensure(tmp);
    FC_HIP(hipcub::DeviceRadixSort::SortPairs(c.sort_tmp.p, tmp, kin, kout, vin, vout, (int)n, 0, end_bit,
                                              c.stream));
}
void sort_keys_public(Ctx& c, const uint64_t* kin, uint64_t* kout, int64_t n, int end_bit) {
    if (n <= 0) return;
    size_t tmp = 0;
    FC_HIP(hipcub::DeviceRadixSort::SortKeys(nullptr, tmp, kin, kout, (int)n, 0, end_bit, c.stream));
    c.sort_tmp.ensure(tmp);
    FC_HIP(hipcub::DeviceRadixSort::SortKeys(c.sort_tmp.p, tmp, kin, kout, (int)n, 0, end_bit, c.stream));
}
template <class T>
void exclusive_scan(Ctx& c, const T* in, T* out, int64_t n) {
    if (n <= 0) return;
    size_t tmp = 0;
    FC_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, in, out, (int)n, c.stream));
    c.sort_tmp.ensure(tmp);
    FC_HIP(hipcub::DeviceScan::ExclusiveSum(c.sort_tmp.p, tmp, in, out, (int)n, c.stream));
}
template void exclusive_scan<int64_t>(Ctx&, const int64_t*, int64_t*, int64_t);
template void exclusive_scan<int32_t>(Ctx&, const int32_t*, int32_t*, int64_t);
template <class K, class V>
void sort_pairs_public(Ctx& c, const K* kin, K* kout, const V* vin, V* vout, int64_t n, int end_bit) {
    sort_pairs(c, kin, kout, vin, vout, n, end_bit);
}
template void sort_pairs_public<uint64_t, int64_t>(Ctx&, const uint64_t*, uint64_t*, const int64_t*, int64_t*,
                                                   int64_t, int);
template void sort_pairs_public<uint32_t, int32_t>(Ctx&, const uint32_t*, uint32_t*, const int32_t*, int32_t*,
                                                   int64_t, int);
template void sort_pairs_public<uint64_t, int32_t>(Ctx&, const uint64_t*, uint64_t*, const int32_t*, int32_t*,
                                                   int64_t, int);

void sync(Ctx& c) { FC_HIP(hipStreamSynchronize(c.stream)); }

__global__ void k_reduce_shards(unsigned long long* base, int F, unsigned max_mask) {
    __shared__ unsigned long long s[CSH];
    for (int f = 0; f < F; ++f) {
        const bool mx = (max_mask >> f) & 1u;
        s[threadIdx.x] = base[(size_t)threadIdx.x * F + f];
        __syncthreads();
        for (int o = CSH / 2; o > 0; o >>= 1) {
            if ((int)threadIdx.x < o) {
                const unsigned long long a = s[threadIdx.x], b = s[threadIdx.x + o];
                s[threadIdx.x] = mx ? (a > b ? a : b) : a + b;
            }
            __syncthreads();
        }
        if (threadIdx.x == 0) base[(size_t)CSH * F + f] = s[0];
        __syncthreads();
    }
}
unsigned long long* shards_begin(Ctx& c, int F) {
    unsigned long long* base = (unsigned long long*)ensure<int64_t>(c.counters, (size_t)(CSH + 1) * F);
    FC_HIP(hipMemsetAsync(base, 0, sizeof(unsigned long long) * CSH * F, c.stream));
    return base;
}
void shards_fold(Ctx& c, int F, unsigned max_mask, int64_t* host_out) {
    unsigned long long* base = (unsigned long long*)c.counters.p;
    k_reduce_shards<<<1, CSH, 0, c.stream>>>(base, F, max_mask);
    FC_HIP(hipMemcpyAsync(c.hpin, base + (size_t)CSH * F, sizeof(int64_t) * F, hipMemcpyDeviceToHost, c.stream));
    sync(c);
    for (int f = 0; f < F; ++f) host_out[f] = c.hpin[f];
}
int64_t read_i64(Ctx& c, const int64_t* dev) {
    FC_HIP(hipMemcpyAsync(c.hpin, dev, sizeof(int64_t), hipMemcpyDeviceToHost, c.stream));
    sync(c);
    return c.hpin[0];
}

// ------------------------------------------------------------------ ingest kernels
// Internal numbering sigma[node] (a seeded Feistel bijection, or the identity), its inverse,
// and the identity label storage (store_order() replaces it).
// relabel = 2, second ingest: sigma'[node] = spos[sigma[node]] -- the numbering follows the
// storage order (community order of the one-replica ordering run), the storage is the identity
__global__ void k_sigma_compose(int64_t n, int32_t* sigma, int32_t* npos, int32_t* spos) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int32_t s = spos[sigma[i]];
    sigma[i] = s;
    npos[s] = (int32_t)i;
}
__global__ void k_identity(int64_t n, int32_t* p) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = (int32_t)i;
}
__global__ void k_sigma(int64_t n, Perm P, int relabel, int32_t* sigma, int32_t* npos, int32_t* spos) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int32_t s = relabel ? (int32_t)perm_apply(P, (uint32_t)i) : (int32_t)i;
    sigma[i] = s;
    npos[s] = (int32_t)i;
    spos[i] = (int32_t)i;
}
// Input edge i (node ids, file order) -> canonical key (min, max) in internal ids, or the
// sentinel for a self loop; endpoints outside [0, n) are counted (the load then fails).
__global__ void k_make_keys(int64_t m, int64_t n, const int32_t* u, const int32_t* v, const int32_t* sigma, int bits,
                            uint64_t* key, int64_t* idx, unsigned long long* bad) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    bool oob = false;
    if (i < m) {
        const int32_t a0 = u[i], b0 = v[i];
        const uint64_t sent = (bits >= 32) ? ~0ull : ((1ull << (2 * bits)) - 1ull);
        uint64_t k = sent;
        oob = (uint32_t)a0 >= (uint64_t)n || (uint32_t)b0 >= (uint64_t)n;
        if (!oob && a0 != b0) {
            const int32_t a = sigma[a0], b = sigma[b0];
            const uint64_t lo = (uint64_t)(a < b ? a : b), hi = (uint64_t)(a < b ? b : a);
            k = (lo << bits) | hi;
        }
        key[i] = k;
        idx[i] = i;
    }
    const unsigned long long bl = __ballot(oob);
    if ((threadIdx.x & 63) == 0 && bl) atomicAdd(shard(bad, 1, 0), (unsigned long long)__popcll(bl));
}

__global__ void k_unique_flags(int64_t m, const uint64_t* key, int bits, int64_t* flag) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    uint64_t sent = (bits >= 32) ? ~0ull : ((1ull << (2 * bits)) - 1ull);
    uint64_t k = key[i];
    flag[i] = (k != sent && (i == 0 || key[i - 1] != k)) ? 1 : 0;
}

__global__ void k_scatter_unique(int64_t m, const uint64_t* key, const int64_t* idx, const int64_t* flag,
                                 const int64_t* pos, int bits, int32_t* eu, int32_t* ev, int32_t* ew,
                                 int64_t* eage) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m || !flag[i]) return;
    int64_t p = pos[i];
    uint64_t k = key[i];
    eu[p] = (int32_t)(k >> bits);
    ev[p] = (int32_t)(k & ((1ull << bits) - 1ull));
    ew[p] = 1;          // fast_consensus.py:135-136: every weight reset to 1.0
    eage[p] = idx[i];   // first occurrence (stable sort) = networkx adjacency age
}

// Host edge arrays -> device graph.  Everything after the PCIe upload of u and v runs on the
// device: validation, internal numbering, canonical keys, dedupe (stable radix sort keeps
// the first occurrence = networkx adjacency age), CSR, label storage order.
void graph_load(Ctx& c, int64_t n, int64_t m, const int32_t* u, const int32_t* v) {
    c.clo_next = -1;   // a sharded closure sequence is sized for the old graph
    FC_REQUIRE(n >= 1 && n < (int64_t(1) << 31), FC_EINVAL, "node count out of range");
    FC_REQUIRE(m >= 0 && m < (int64_t(1) << 31), FC_EINVAL, "edge count out of range");
    auto t_last = std::chrono::steady_clock::now();
    auto mark = [&](const char* what) {   // FC_TRACE: per-phase wall time of the load
        if (!c.trace) return;
        sync(c);
        const auto t = std::chrono::steady_clock::now();
        fprintf(stderr, "[fc] load %-14s %8.2f ms\n", what,
                1e-6 * (double)std::chrono::duration_cast<std::chrono::nanoseconds>(t - t_last).count());
        t_last = t;
    };
    c.N = 0;   // no graph until this load completes
    const int64_t mm = m > 0 ? m : 1;
    int32_t* du = ensure<int32_t>(c.cu, mm);
    int32_t* dv = ensure<int32_t>(c.cv, mm);
    if (m > 0) {
        FC_HIP(hipMemcpyAsync(du, u, sizeof(int32_t) * m, hipMemcpyHostToDevice, c.stream));
        FC_HIP(hipMemcpyAsync(dv, v, sizeof(int32_t) * m, hipMemcpyHostToDevice, c.stream));
    }
    int32_t* sigma = ensure<int32_t>(c.sigma, n);
    int32_t* npos = ensure<int32_t>(c.npos, n);
    int32_t* spos = ensure<int32_t>(c.spos, n);
    k_sigma<<<nblk(n), TB, 0, c.stream>>>(n, make_perm((uint32_t)n, (uint32_t)mix64(c.seed ^ 0x51A7E5EDull)),
                                          c.relabel ? 1 : 0, sigma, npos, spos);
    int bits = 1;
    while ((int64_t(1) << bits) < n) ++bits;
    Graph& g = c.g;
    // canonical keys in the numbering sigma, sort + dedupe, CSR (run twice with relabel = 2)
    auto ingest = [&]() {
    uint64_t* k1 = ensure<uint64_t>(c.mkey, mm);
    uint64_t* k2 = ensure<uint64_t>(c.mkey2, mm);
    int64_t* i1 = ensure<int64_t>(c.midx, mm);
    int64_t* i2 = ensure<int64_t>(c.midx2, mm);
    int64_t* fl = ensure<int64_t>(c.ckey, mm + 1);
    int64_t* ps = ensure<int64_t>(c.ckey2, mm + 1);
    unsigned long long* bad = shards_begin(c, 1);
    if (m > 0) k_make_keys<<<nblk(m), TB, 0, c.stream>>>(m, n, du, dv, sigma, bits, k1, i1, bad);
    int64_t nbad = 0;
    shards_fold(c, 1, 0u, &nbad);
    FC_REQUIRE(nbad == 0, FC_EINVAL, std::to_string(nbad) + " edge endpoints out of range [0, n)");
    mark("upload+keys");
    c.N = n;
    c.key_bits = bits;
    sort_pairs(c, k1, k2, i1, i2, m, 2 * bits);
    k_unique_flags<<<nblk(m), TB, 0, c.stream>>>(m, k2, bits, fl);
    exclusive_scan(c, fl, ps, m);
    int64_t last_pos = 0, last_flag = 0;
    if (m > 0) {
        FC_HIP(hipMemcpyAsync(&c.hpin[0], ps + m - 1, 8, hipMemcpyDeviceToHost, c.stream));
        FC_HIP(hipMemcpyAsync(&c.hpin[1], fl + m - 1, 8, hipMemcpyDeviceToHost, c.stream));
        sync(c);
        last_pos = c.hpin[0];
        last_flag = c.hpin[1];
    }
    int64_t mu = last_pos + last_flag;
    g.m = mu;
    int64_t cap = mu > 0 ? mu : 1;
    ensure<int32_t>(g.eu, cap); ensure<int32_t>(g.ev, cap); ensure<int32_t>(g.ew, cap); ensure<int64_t>(g.eage, cap);
    k_scatter_unique<<<nblk(m), TB, 0, c.stream>>>(m, k2, i2, fl, ps, bits, g.eu.as<int32_t>(), g.ev.as<int32_t>(),
                                                    g.ew.as<int32_t>(), g.eage.as<int64_t>());
    c.m_original = mu;   // L = G.number_of_edges() (fast_consensus.py:132, :144)
    mark("sort+dedupe");
    graph_build_csr(c, g);
    slot_maps(c);        // identity storage (the ordering pass below runs on it)
    mark("csr");
    };
    ingest();
    if (c.relabel == 2 && g.M2 > 0) {
        // FC_OPT_RELABEL = 2: the internal numbering in community order (the storage-order run's
        // communities), for kernels that gather neighbour state by internal id -- Infomap's
        // union levels (leiden.hip), whose buckets are hashes of the id, not chunks of the visit
        // order (cd.hip / cd_rl.hip need a random numbering: chunked visit orders would put
        // neighbours in one bucket).  The storage is the identity afterwards.
        store_order(c);
        sigma = ensure<int32_t>(c.sigma, n);
        npos = ensure<int32_t>(c.npos, n);
        spos = ensure<int32_t>(c.spos, n);
        k_sigma_compose<<<nblk(n), TB, 0, c.stream>>>(n, sigma, npos, spos);
        k_identity<<<nblk(n), TB, 0, c.stream>>>(n, spos);
        du = ensure<int32_t>(c.cu, mm);
        dv = ensure<int32_t>(c.cv, mm);
        if (m > 0) {   // the ordering run may have reused the upload buffers: upload again
            FC_HIP(hipMemcpyAsync(du, u, sizeof(int32_t) * m, hipMemcpyHostToDevice, c.stream));
            FC_HIP(hipMemcpyAsync(dv, v, sizeof(int32_t) * m, hipMemcpyHostToDevice, c.stream));
        }
        ingest();
        mark("relabel");
    }
    c.h_sigma.resize(n);
    FC_HIP(hipMemcpyAsync(c.h_sigma.data(), sigma, 4 * n, hipMemcpyDeviceToHost, c.stream));
    if (c.store_order && c.relabel != 2 && g.M2 > 0) {
        store_order(c);
        graph_slots(c, g);
    }
    slot_maps(c);
    mark("store_order");
    graph_copy(c, c.g0, g);
    c.labT_valid = false;
    sync(c);
    mark("copy");
}

// ------------------------------------------------------------------ node-space export
__global__ void k_export_keys(int64_t m, const int32_t* u, const int32_t* v, const int32_t* npos, int bits,
                              uint64_t* key, int64_t* idx) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= m) return;
    const uint64_t a = (uint64_t)npos[u[e]], b = (uint64_t)npos[v[e]];
    key[e] = a < b ? (a << bits) | b : (b << bits) | a;
    idx[e] = e;
}
__global__ void k_export_gather(int64_t m, const uint64_t* key, const int64_t* idx, int bits, const int32_t* w,
                                const int64_t* age, int32_t* ou, int32_t* ov, int32_t* ow, int64_t* oage) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    ou[i] = (int32_t)(key[i] >> bits);
    ov[i] = (int32_t)(key[i] & ((1ull << bits) - 1ull));
    ow[i] = w[idx[i]];
    oage[i] = age[idx[i]];
}
// An edge list in internal ids -> node ids, canonical (u<v) and sorted, on the host.
void graph_to_host(Ctx& c, int64_t m, const int32_t* u, const int32_t* v, const int32_t* w, const int64_t* age,
                   int32_t* ou, int32_t* ov, int32_t* ow, int64_t* oage) {
    if (m <= 0) return;
    uint64_t* k1 = ensure<uint64_t>(c.mkey, m);
    uint64_t* k2 = ensure<uint64_t>(c.mkey2, m);
    int64_t* i1 = ensure<int64_t>(c.midx, m);
    int64_t* i2 = ensure<int64_t>(c.midx2, m);
    int32_t* su = ensure<int32_t>(c.st_u, m);
    int32_t* sv = ensure<int32_t>(c.st_v, m);
    int32_t* sw = ensure<int32_t>(c.st_w, m);
    int64_t* sa = ensure<int64_t>(c.st_age, m);
    k_export_keys<<<nblk(m), TB, 0, c.stream>>>(m, u, v, c.npos.as<int32_t>(), c.key_bits, k1, i1);
    sort_pairs(c, k1, k2, i1, i2, m, 2 * c.key_bits);
    k_export_gather<<<nblk(m), TB, 0, c.stream>>>(m, k2, i2, c.key_bits, w, age, su, sv, sw, sa);
    if (ou) FC_HIP(hipMemcpyAsync(ou, su, 4 * m, hipMemcpyDeviceToHost, c.stream));
    if (ov) FC_HIP(hipMemcpyAsync(ov, sv, 4 * m, hipMemcpyDeviceToHost, c.stream));
    if (ow) FC_HIP(hipMemcpyAsync(ow, sw, 4 * m, hipMemcpyDeviceToHost, c.stream));
    if (oage) FC_HIP(hipMemcpyAsync(oage, sa, 8 * m, hipMemcpyDeviceToHost, c.stream));
    sync(c);
}

// graph = G.copy() (fast_consensus.py:131): device-to-device, the input stays resident.
void graph_copy(Ctx& c, Graph& dst, const Graph& src) {
    c.clo_next = -1;
    const int64_t m = src.m > 0 ? src.m : 1, n = c.N;
    auto cp = [&](DevBuf& d, const DevBuf& s, size_t bytes) {
        d.ensure(bytes + 16);
        if (!s.p) return;   // edgeless graph: a per-entry array was never allocated
        FC_HIP(hipMemcpyAsync(d.p, s.p, std::min(bytes, s.bytes), hipMemcpyDeviceToDevice, c.stream));
    };
    cp(dst.eu, src.eu, 4 * m); cp(dst.ev, src.ev, 4 * m); cp(dst.ew, src.ew, 4 * m); cp(dst.eage, src.eage, 8 * m);
    cp(dst.rowptr, src.rowptr, 8 * (n + 1));
    cp(dst.col, src.col, 8 * m); cp(dst.cw, src.cw, 8 * m); cp(dst.ceid, src.ceid, 8 * m);
    cp(dst.crev, src.crev, 8 * m);
    cp(dst.colp, src.colp, 8 * m);
    cp(dst.vrec, src.vrec, 16 * n);
    cp(dst.kdeg, src.kdeg, 8 * n);
    dst.m = src.m; dst.M2 = src.M2; dst.max_deg = src.max_deg; dst.max_kdeg = src.max_kdeg; dst.max_w = src.max_w;
    c.labT_valid = false;
}

// ------------------------------------------------------------------ CSR build
// start[x] = first index i with key[i] >= x, x in [0, n], for sorted keys in [0, n): the
// exclusive prefix count of each node's edges, written once per node with no atomics
// (index i writes the nodes in (key[i-1], key[i]]).
template <class K>
__global__ void k_bounds(int64_t m, const K* key, int64_t n, int64_t* start) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i > m) return;
    const int64_t lo = i == 0 ? -1 : (int64_t)key[i - 1];
    const int64_t hi = i == m ? n : (int64_t)key[i];
    for (int64_t x = lo + 1; x <= hi; ++x) start[x] = i;
}
__global__ void k_rowptr(int64_t n, int64_t m, const int64_t* us, const int64_t* vs, int64_t* rowptr) {
    int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (x < n) rowptr[x] = us[x] + vs[x];
    if (x == n) rowptr[n] = 2 * m;
}
__global__ void k_iota_ev(int64_t m, const int32_t* ev, uint32_t* key, int32_t* idx) {
    int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= m) return;
    key[e] = (uint32_t)ev[e];
    idx[e] = (int32_t)e;
}
// Row x = [neighbours u < x, ascending] ++ [neighbours v > x, ascending]: fully sorted rows.
__global__ void k_fill_upper(int64_t m, const int32_t* eu, const int32_t* ev, const int32_t* ew,
                             const int64_t* rowptr, const int64_t* ustart, const int64_t* vstart,
                             int32_t* col, int32_t* cw, int32_t* ceid, int32_t* posu) {
    int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= m) return;
    int32_t u = eu[e];
    int64_t nlow = vstart[u + 1] - vstart[u];
    int64_t p = rowptr[u] + nlow + (e - ustart[u]);
    col[p] = ev[e]; cw[p] = ew[e]; ceid[p] = (int32_t)e;
    posu[e] = (int32_t)p;
}
__global__ void k_fill_lower(int64_t m, const int32_t* perm, const uint32_t* vsorted, const int32_t* eu,
                             const int32_t* ew, const int64_t* rowptr, const int64_t* vstart, int32_t* col,
                             int32_t* cw, int32_t* ceid, int32_t* posv) {
    int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= m) return;
    int32_t e = perm[f];
    int32_t v = (int32_t)vsorted[f];          // = ev[e], read in order
    int64_t p = rowptr[v] + (f - vstart[v]);
    col[p] = eu[e]; cw[p] = ew[e]; ceid[p] = e;
    posv[e] = (int32_t)p;
}
// rev[j] = position of the reverse adjacency entry (the same undirected edge seen from
// the other endpoint): moving vertex v updates nlab at rev[j] for each j in row(v).
__global__ void k_fill_rev(int64_t m, const int32_t* posu, const int32_t* posv, int32_t* rev) {
    int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= m) return;
    const int32_t a = posu[e], b = posv[e];
    rev[a] = b;
    rev[b] = a;
}
__global__ void k_kdeg(int64_t n, const int64_t* rowptr, const int32_t* cw, int64_t* kdeg, unsigned long long* red) {
    int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    int64_t s = 0, d = 0, mw = 0;
    if (x < n) {
        for (int64_t j = rowptr[x]; j < rowptr[x + 1]; ++j) { s += cw[j]; mw = max(mw, (int64_t)cw[j]); }
        kdeg[x] = s;
        d = rowptr[x + 1] - rowptr[x];
    }
    // block reduce: sum(kdeg), max(deg), max(kdeg), max(w)
    __shared__ long long ss[TB], sd[TB], sk[TB], sw[TB];
    ss[threadIdx.x] = s; sd[threadIdx.x] = d; sk[threadIdx.x] = s; sw[threadIdx.x] = mw;
    __syncthreads();
    for (int o = TB / 2; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) {
            ss[threadIdx.x] += ss[threadIdx.x + o];
            sd[threadIdx.x] = max(sd[threadIdx.x], sd[threadIdx.x + o]);
            sk[threadIdx.x] = max(sk[threadIdx.x], sk[threadIdx.x + o]);
            sw[threadIdx.x] = max(sw[threadIdx.x], sw[threadIdx.x + o]);
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        atomicAdd(shard(red, 4, 0), (unsigned long long)ss[0]);
        atomicMax(shard(red, 4, 1), (unsigned long long)sd[0]);
        atomicMax(shard(red, 4, 2), (unsigned long long)sk[0]);
        atomicMax(shard(red, 4, 3), (unsigned long long)sw[0]);
    }
}

__global__ void k_slots(int64_t m2, const int32_t* col, const int32_t* spos, int32_t* colp) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j < m2) colp[j] = spos[col[j]];
}
// One 16-byte record per vertex for the CD kernels: row start, degree, k_v, storage slot --
// one load where a list-order visit would touch three random lines (rowptr, kdeg, spos).
__global__ void k_vrec(int64_t n, const int64_t* rowptr, const int64_t* kdeg, const int32_t* spos, int4* vrec) {
    const int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= n) return;
    const int64_t rb = rowptr[v];
    vrec[v] = make_int4((int32_t)(uint32_t)rb, (int32_t)(rowptr[v + 1] - rb), (int32_t)kdeg[v], spos[v]);
}
void graph_slots(Ctx& c, Graph& g) {
    const int64_t m2 = 2 * g.m, n = c.N;
    int32_t* colp = ensure<int32_t>(g.colp, m2 > 0 ? m2 : 1);
    if (m2 > 0) k_slots<<<nblk(m2), TB, 0, c.stream>>>(m2, g.col.as<int32_t>(), c.spos.as<int32_t>(), colp);
    int4* vrec = ensure<int4>(g.vrec, n);
    k_vrec<<<nblk(n), TB, 0, c.stream>>>(n, g.rowptr.as<int64_t>(), g.kdeg.as<int64_t>(), c.spos.as<int32_t>(), vrec);
}

void graph_build_csr(Ctx& c, Graph& g) {
    const int64_t n = c.N, m = g.m;
    int64_t* us = ensure<int64_t>(c.nodetmp3, 2 * (n + 1));
    int64_t* vs = us + (n + 1);
    int64_t* rowptr = ensure<int64_t>(g.rowptr, n + 1);
    int64_t m2 = 2 * m > 0 ? 2 * m : 1;
    int32_t* col = ensure<int32_t>(g.col, m2);
    int32_t* cw = ensure<int32_t>(g.cw, m2);
    int32_t* ceid = ensure<int32_t>(g.ceid, m2);
    uint32_t* k1 = (uint32_t*)ensure<uint64_t>(c.mkey, m > 0 ? m : 1);
    uint32_t* k2 = (uint32_t*)ensure<uint64_t>(c.mkey2, m > 0 ? m : 1);
    int32_t* i1 = (int32_t*)ensure<int64_t>(c.midx, m > 0 ? m : 1);
    int32_t* i2 = (int32_t*)ensure<int64_t>(c.midx2, m > 0 ? m : 1);
    if (m > 0) {   // edges by v (stable: each v's run stays in u order)
        k_iota_ev<<<nblk(m), TB, 0, c.stream>>>(m, g.ev.as<int32_t>(), k1, i1);
        sort_pairs(c, (const uint32_t*)k1, k2, (const int32_t*)i1, i2, m, c.key_bits);
    }
    // row starts of the upper (u) and lower (v) halves: eu is sorted, k2 holds the sorted ev
    k_bounds<int32_t><<<nblk(m + 1), TB, 0, c.stream>>>(m, g.eu.as<int32_t>(), n, us);
    k_bounds<uint32_t><<<nblk(m + 1), TB, 0, c.stream>>>(m, k2, n, vs);
    k_rowptr<<<nblk(n + 1), TB, 0, c.stream>>>(n, m, us, vs, rowptr);
    if (m > 0) {
        int32_t* posu = (int32_t*)k1;   // sort inputs are dead once the sort is enqueued
        int32_t* posv = i1;
        int32_t* rev = ensure<int32_t>(g.crev, m2);
        k_fill_upper<<<nblk(m), TB, 0, c.stream>>>(m, g.eu.as<int32_t>(), g.ev.as<int32_t>(), g.ew.as<int32_t>(),
                                                    rowptr, us, vs, col, cw, ceid, posu);
        k_fill_lower<<<nblk(m), TB, 0, c.stream>>>(m, i2, k2, g.eu.as<int32_t>(), g.ew.as<int32_t>(), rowptr, vs,
                                                    col, cw, ceid, posv);
        k_fill_rev<<<nblk(m), TB, 0, c.stream>>>(m, posu, posv, rev);
    }
    int64_t* kdeg = ensure<int64_t>(g.kdeg, n);
    unsigned long long* red = shards_begin(c, 4);
    k_kdeg<<<nblk(n), TB, 0, c.stream>>>(n, rowptr, cw, kdeg, red);
    int64_t h[4];
    shards_fold(c, 4, 0xEu, h);
    g.M2 = h[0];
    g.max_deg = (int32_t)h[1];
    g.max_kdeg = h[2];
    g.max_w = (int32_t)h[3];
    graph_slots(c, g);
}

// ------------------------------------------------------------------ merge
// graph <- kept ++ closure ++ repair, re-sorted canonically (fast_consensus.py:198, :307).
__global__ void k_merge_keys(int64_t n0, int64_t n1, const int32_t* au, const int32_t* av, const int32_t* bu,
                             const int32_t* bv, int bits, uint64_t* key, int64_t* idx) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n0 + n1) return;
    int32_t u, v;
    if (i < n0) { u = au[i]; v = av[i]; } else { u = bu[i - n0]; v = bv[i - n0]; }
    key[i] = ((uint64_t)u << bits) | (uint64_t)v;
    idx[i] = i;
}
__global__ void k_merge_gather(int64_t n, int64_t n0, const int64_t* idx, const int32_t* au, const int32_t* av,
                               const int32_t* aw, const int64_t* aage, const int32_t* bu, const int32_t* bv,
                               const int32_t* bw, const int64_t* bage, int32_t* eu, int32_t* ev, int32_t* ew,
                               int64_t* eage) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    int64_t s = idx[i];
    if (s < n0) { eu[i] = au[s]; ev[i] = av[s]; ew[i] = aw[s]; eage[i] = aage[s]; }
    else { s -= n0; eu[i] = bu[s]; ev[i] = bv[s]; ew[i] = bw[s]; eage[i] = bage[s]; }
}

// kept (c.ku.., sorted) ++ added (c.cu.., n_cand closure + n_rep repair) -> c.g, then CSR.
// The three lists are disjoint (closure pairs are non-edges of the kept graph, repair pairs
// touch nodes isolated in both), so the canonical order is unique: only the added list is
// radix-sorted, then merged with the kept list (merge path).
void graph_merge_next(Ctx& c, int64_t n_added) {
    const int64_t n0 = c.kept_m, total = c.kept_m + n_added;
    int64_t cap = total > 0 ? total : 1;
    uint64_t* k1 = ensure<uint64_t>(c.mkey, cap);
    uint64_t* k2 = ensure<uint64_t>(c.mkey2, cap);
    int64_t* i1 = ensure<int64_t>(c.midx, cap);
    int64_t* i2 = ensure<int64_t>(c.midx2, cap);
    int64_t* im = ensure<int64_t>(c.cval, cap);
    Graph& g = c.g;
    ensure<int32_t>(g.eu, cap); ensure<int32_t>(g.ev, cap); ensure<int32_t>(g.ew, cap); ensure<int64_t>(g.eage, cap);
    if (total > 0) {
        k_merge_keys<<<nblk(total), TB, 0, c.stream>>>(n0, n_added, c.ku.as<int32_t>(), c.kv.as<int32_t>(),
                                                        c.cu.as<int32_t>(), c.cv.as<int32_t>(), c.key_bits, k1, i1);
        const int64_t* src = i1;
        if (n_added > 0) {
            sort_pairs(c, k1 + n0, k2 + n0, i1 + n0, i2 + n0, n_added, 2 * c.key_bits);
            if (n0 > 0) {
                size_t tmp = 0;
                auto disc = rocprim::make_discard_iterator();
                FC_HIP(rocprim::merge(nullptr, tmp, k1, k2 + n0, disc, i1, i2 + n0, im, (size_t)n0, (size_t)n_added,
                                      rocprim::less<uint64_t>(), c.stream));
                c.sort_tmp.ensure(tmp);
                FC_HIP(rocprim::merge(c.sort_tmp.p, tmp, k1, k2 + n0, disc, i1, i2 + n0, im, (size_t)n0,
                                      (size_t)n_added, rocprim::less<uint64_t>(), c.stream));
                src = im;
            } else {
                src = i2;
            }
        }
        k_merge_gather<<<nblk(total), TB, 0, c.stream>>>(
            total, n0, src, c.ku.as<int32_t>(), c.kv.as<int32_t>(), c.kw.as<int32_t>(), c.kage.as<int64_t>(),
            c.cu.as<int32_t>(), c.cv.as<int32_t>(), c.cw2.as<int32_t>(), c.cage.as<int64_t>(), g.eu.as<int32_t>(),
            g.ev.as<int32_t>(), g.ew.as<int32_t>(), g.eage.as<int64_t>());
    }
    g.m = total;
    graph_build_csr(c, g);
    c.labT_valid = false;
}

}  // namespace fc
