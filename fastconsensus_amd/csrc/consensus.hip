// consensus.hip -- the consensus-graph update of fast_consensus():
//   per-edge co-membership rule + tau threshold + delta check  (fast_consensus.py:150-173,
//   :273-288, check_consensus_graph :17-37), triadic closure (:175-190, :292-304) and
//   isolate repair (:193-195).  Integer/byte work, HBM/gather bound: no MFMA.
#include <hipcub/hipcub.hpp>

#include "fc_ctx.h"
#include "fc_device.h"

namespace fc {

template <class T> void exclusive_scan(Ctx& c, const T* in, T* out, int64_t n);
template <class K, class V>
void sort_pairs_public(Ctx& c, const K* kin, K* kout, const V* vin, V* vout, int64_t n, int end_bit);
void sort_keys_public(Ctx& c, const uint64_t* kin, uint64_t* kout, int64_t n, int end_bit);

static constexpr int TB = 256;
static inline unsigned nblk(int64_t n, int tb = TB) {
    int64_t b = (n + tb - 1) / tb;
    if (b < 1) b = 1;
    return (unsigned)b;
}

// ------------------------------------------------------------------ consensus partial
// One edge per group of G lanes; each lane compares 4 replicas per 16-byte load of the
// node-major label rows labT[node][ldT] (a 64-replica row is 256 B = one coalesced load
// by 16 lanes).  LOUVAIN: highest global replica index whose labels split (u,v), or -1.
// COUNT: number of replicas co-clustering (u,v).
template <int G, bool LOUVAIN>
__global__ __launch_bounds__(256) void k_pair_partial(int64_t m, const int32_t* __restrict__ eu,
                                                      const int32_t* __restrict__ ev,
                                                      const int32_t* __restrict__ labT, int ldT, int n_r,
                                                      int rbase, int32_t* __restrict__ out) {
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t e = gid / G;
    const int l = (int)(gid % G);
    if (e >= m) return;  // whole groups exit together (G divides 64)
    const int4* ru = reinterpret_cast<const int4*>(labT + (int64_t)eu[e] * ldT);
    const int4* rv = reinterpret_cast<const int4*>(labT + (int64_t)ev[e] * ldT);
    int res = LOUVAIN ? -1 : 0;
    for (int q = l; 4 * q < n_r; q += G) {
        const int4 a = ru[q], b = rv[q];
        const int base = 4 * q;
        if (LOUVAIN) {
            if (base + 3 < n_r && a.w != b.w) res = max(res, base + 3);
            else if (base + 2 < n_r && a.z != b.z) res = max(res, base + 2);
            else if (base + 1 < n_r && a.y != b.y) res = max(res, base + 1);
            else if (a.x != b.x) res = max(res, base);
        } else {
            res += (a.x == b.x);
            if (base + 1 < n_r) res += (a.y == b.y);
            if (base + 2 < n_r) res += (a.z == b.z);
            if (base + 3 < n_r) res += (a.w == b.w);
        }
    }
#pragma unroll
    for (int off = G / 2; off > 0; off >>= 1) {
        int o = __shfl_xor(res, off, G);
        res = LOUVAIN ? max(res, o) : res + o;
    }
    if (l == 0) out[e] = LOUVAIN ? (res < 0 ? -1 : res + rbase) : res;
}

template <bool LOUVAIN>
static void launch_pair_partial(Ctx& c, int64_t m, const int32_t* eu, const int32_t* ev, int32_t* out) {
    if (m <= 0) return;
    const int chunks = (c.n_r + 3) / 4;
    int G = 1;
    while (G < chunks && G < 16) G <<= 1;
    const int64_t threads = m * G;
    const unsigned grid = nblk(threads);
    const int32_t* labT = c.labT.as<int32_t>();
    switch (G) {
        case 1: k_pair_partial<1, LOUVAIN><<<grid, TB, 0, c.stream>>>(m, eu, ev, labT, c.ldT, c.n_r, c.rbase, out); break;
        case 2: k_pair_partial<2, LOUVAIN><<<grid, TB, 0, c.stream>>>(m, eu, ev, labT, c.ldT, c.n_r, c.rbase, out); break;
        case 4: k_pair_partial<4, LOUVAIN><<<grid, TB, 0, c.stream>>>(m, eu, ev, labT, c.ldT, c.n_r, c.rbase, out); break;
        case 8: k_pair_partial<8, LOUVAIN><<<grid, TB, 0, c.stream>>>(m, eu, ev, labT, c.ldT, c.n_r, c.rbase, out); break;
        default: k_pair_partial<16, LOUVAIN><<<grid, TB, 0, c.stream>>>(m, eu, ev, labT, c.ldT, c.n_r, c.rbase, out); break;
    }
}

void consensus_partial(Ctx& c, int algo, int32_t* out) {
    FC_REQUIRE(c.n_r > 0, FC_ESTATE, "no labelings: run fc_cd or fc_set_labels first");
    if (!c.labT_valid) labels_transpose(c);
    const int sl = timer_begin(c);
    if (algo == FC_ALGO_LOUVAIN)   // k_last; LPM and the new_consensus.py rule: co-membership count
        launch_pair_partial<true>(c, c.g.m, c.g.eu.as<int32_t>(), c.g.ev.as<int32_t>(), out);
    else
        launch_pair_partial<false>(c, c.g.m, c.g.eu.as<int32_t>(), c.g.ev.as<int32_t>(), out);
    timer_end(c, 1, sl);
}

// ------------------------------------------------------------------ consensus apply
// Closed form of the Louvain rule (fast_consensus.py:150-159), proven equal to the
// literal loop in tests/test_oracle_golden.py: w in {0,n_p} -> 0; no split -> n_p;
// else w + (n_p - 1 - k_last).  LPM (:273-280): the co-membership count.
// new_consensus.py rule (:155-163, FC_ALGO_LOUVAIN_NC): w in {0,n_p} -> w, else the count.
// keep iff !(w' < tau*n_p) in float64 (:165, :286).  Counts kept and "unconverged"
// (w' not in {0, n_p}, check_consensus_graph :30-32) per block -> one atomic per block.
__global__ __launch_bounds__(256) void k_consensus_apply(int algo, int64_t m, int n_p, double cut,
                                                         const int32_t* __restrict__ ew,
                                                         const int32_t* __restrict__ part,
                                                         int32_t* __restrict__ wnew, int64_t* __restrict__ flag,
                                                         unsigned long long* counters) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    int keep = 0, unc = 0;
    if (e < m) {
        int nw;
        if (algo == FC_ALGO_LOUVAIN) {
            const int w = ew[e];
            const int k = part[e];
            nw = (w == 0 || w == n_p) ? 0 : (k < 0 ? n_p : w + (n_p - 1 - k));
        } else if (algo == FC_ALGO_LOUVAIN_NC) {
            const int w = ew[e];
            nw = (w == 0 || w == n_p) ? w : part[e];
        } else {
            nw = part[e];
        }
        keep = !((double)nw < cut);
        unc = keep && nw != 0 && nw != n_p;
        wnew[e] = nw;
        flag[e] = keep;
    }
    // wave64 ballot counts -> LDS -> one sharded atomic per block and field
    __shared__ unsigned long long s_k, s_u;
    if (threadIdx.x == 0) { s_k = 0; s_u = 0; }
    __syncthreads();
    const unsigned long long bk = __ballot(keep), bu = __ballot(unc);
    if ((threadIdx.x & 63) == 0) {
        if (bk) atomicAdd(&s_k, (unsigned long long)__popcll(bk));
        if (bu) atomicAdd(&s_u, (unsigned long long)__popcll(bu));
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        if (s_k) atomicAdd(shard(counters, 2, 0), s_k);
        if (s_u) atomicAdd(shard(counters, 2, 1), s_u);
    }
}

__global__ void k_scatter_kept(int64_t m, const int64_t* flag, const int64_t* pos, const int32_t* eu,
                               const int32_t* ev, const int32_t* wnew, const int64_t* eage, int32_t* ku,
                               int32_t* kv, int32_t* kw, int64_t* kage) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= m || !flag[e]) return;
    const int64_t p = pos[e];
    ku[p] = eu[e]; kv[p] = ev[e]; kw[p] = wnew[e]; kage[p] = eage[e];
}
// Kept CSR = the current CSR filtered by the edge keep flags (rows stay sorted).
__global__ void k_csr_flags(int64_t m2, const int32_t* ceid, const int64_t* eflag, int64_t* f2) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j < m2) f2[j] = eflag[ceid[j]];
    else if (j == m2) f2[j] = 0;
}
__global__ void k_csr_compact(int64_t m2, const int64_t* f2, const int64_t* p2, const int32_t* col,
                              int32_t* kcol) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j < m2 && f2[j]) kcol[p2[j]] = col[j];
}
__global__ void k_krowptr(int64_t n, const int64_t* rowptr, const int64_t* p2, int64_t* krowptr) {
    const int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (x <= n) krowptr[x] = p2[rowptr[x]];
}

void consensus_apply(Ctx& c, int algo, int n_p, double tau, const int32_t* partial, int64_t* kept_out,
                     int64_t* unconv_out) {
    c.clo_next = -1;   // a sharded closure sequence (fc_closure_begin ...) read the previous kept graph
    c.clo_algo = algo;   // the closure's block count follows the loop (closure_blocks)
    const int sl = timer_begin(c);
    Graph& g = c.g;
    const int64_t m = g.m, cap = m + 1;
    int32_t* wnew = ensure<int32_t>(c.wnew, cap);
    int64_t* flag = ensure<int64_t>(c.flag, 2 * cap + 1);
    int64_t* pos = ensure<int64_t>(c.pos, 2 * cap + 1);
    unsigned long long* ctr = shards_begin(c, 2);
    const double cut = tau * (double)n_p;  // Python float64 product (fast_consensus.py:165)
    if (m > 0)
        k_consensus_apply<<<nblk(m), TB, 0, c.stream>>>(algo, m, n_p, cut, g.ew.as<int32_t>(),
                                                         partial, wnew, flag, ctr);
    FC_HIP(hipMemsetAsync(flag + m, 0, sizeof(int64_t), c.stream));
    exclusive_scan(c, flag, pos, m + 1);
    int64_t h[2];
    shards_fold(c, 2, 0u, h);
    const int64_t kept = h[0], unconv = h[1];
    c.kept_m = kept;
    const int64_t kc = kept > 0 ? kept : 1;
    int32_t* ku = ensure<int32_t>(c.ku, kc);
    int32_t* kv = ensure<int32_t>(c.kv, kc);
    int32_t* kw = ensure<int32_t>(c.kw, kc);
    int64_t* kage = ensure<int64_t>(c.kage, kc);
    if (m > 0)
        k_scatter_kept<<<nblk(m), TB, 0, c.stream>>>(m, flag, pos, g.eu.as<int32_t>(), g.ev.as<int32_t>(), wnew,
                                                      g.eage.as<int64_t>(), ku, kv, kw, kage);
    // kept CSR (for closure sampling and has_edge); flag[] holds edge flags, reuse wnew-free scratch
    const int64_t m2 = 2 * m;
    int64_t* f2 = ensure<int64_t>(c.nodetmp3, m2 + 1 > 2 * (c.N + 1) ? m2 + 1 : 2 * (c.N + 1));
    int64_t* p2 = ensure<int64_t>(c.ckey2, m2 + 1);
    k_csr_flags<<<nblk(m2 + 1), TB, 0, c.stream>>>(m2, g.ceid.as<int32_t>(), flag, f2);
    exclusive_scan(c, f2, p2, m2 + 1);
    int32_t* kcol = ensure<int32_t>(c.kcol, 2 * kc);
    int64_t* krowptr = ensure<int64_t>(c.krowptr, c.N + 1);
    k_csr_compact<<<nblk(m2), TB, 0, c.stream>>>(m2, f2, p2, g.col.as<int32_t>(), kcol);
    k_krowptr<<<nblk(c.N + 1), TB, 0, c.stream>>>(c.N, g.rowptr.as<int64_t>(), p2, krowptr);
    if (kept_out) *kept_out = kept;
    if (unconv_out) *unconv_out = unconv;
    timer_end(c, 1, sl);
}

// ------------------------------------------------------------------ closure
// b in the ascending row col[lo, end)
__device__ __forceinline__ bool has_edge_row(const int32_t* col, int64_t lo, int64_t end, int32_t b) {
    int64_t hi = end;
    if (hi - lo <= 16) {   // short row: 16 independent loads (one round trip), not a dependent search
        bool f = false;
#pragma unroll
        for (int q = 0; q < 16; ++q)
            if (lo + q < hi) f |= col[lo + q] == b;
        return f;
    }
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        const int32_t x = col[mid];
        if (x < b) lo = mid + 1;
        else hi = mid;
    }
    return lo < end && col[lo] == b;
}
__device__ __forceinline__ bool has_edge_sorted(const int64_t* rowptr, const int32_t* col, int32_t a,
                                                int32_t b) {
    return has_edge_row(col, rowptr[a], rowptr[a + 1], b);
}

// Attempt t (fast_consensus.py:175-184): node uniform over all N (np.random.choice over
// nextgraph.nodes(), :177); if it has >= 2 neighbours, two distinct neighbours uniformly
// (random.sample, :181); candidate iff not an edge (:183).  The reference's nextgraph GROWS
// while it samples (a closure edge is a neighbour for every later attempt); the attempts run
// here in closure_rounds consecutive blocks [t0, t1), and a block draws from the
// post-threshold graph (krowptr/kcol) plus the C graph of every closure edge the earlier
// blocks found (crowptr/ccol, ascending rows; null in the first block).  A node's neighbours
// are its kept row then its C row.  The CPU twin in oracle/fc_oracle.c restates it bit for bit.
// A block's candidates are deduplicated in an open-addressing table cleared per block (key
// (u << bits) | v, value the first attempt of the block that drew it, atomicMin); the thread
// whose CAS creates a slot lists it.  The table holds one block's pairs only (2x slots), so
// it stays in the Infinity Cache; earlier blocks' candidates are C edges (has_edge in C).
constexpr uint64_t CLO_EMPTY = ~0ull;
// A table slot: the pair key and the first attempt that drew it in one 16-byte record, so the
// attempt's atomicMin lands on the line its CAS just brought in (two arrays cost a second
// random line per candidate).  Cleared to all ones (key EMPTY, attempt UINT_MAX).
struct __align__(16) CloSlot {
    unsigned long long key;
    unsigned int att;
    unsigned int pad;
};
__device__ __forceinline__ uint64_t clo_slot(uint64_t key, uint64_t mask) { return mix64(key) & mask; }
// insert key with attempt a; returns the slot if this call created it, else -1
__device__ __forceinline__ int64_t clo_insert(CloSlot* tab, uint64_t hmask, uint64_t key, uint32_t a) {
    uint64_t h = clo_slot(key, hmask);
    while (true) {
        unsigned long long k = tab[h].key;
        if (k == CLO_EMPTY) {
            k = atomicCAS(&tab[h].key, (unsigned long long)CLO_EMPTY, (unsigned long long)key);
            if (k == CLO_EMPTY) {                 // created: a candidate of this block
                atomicMin(&tab[h].att, a);
                return (int64_t)h;
            }
        }
        if (k == key) { atomicMin(&tab[h].att, a); return -1; }   // drawn again in this block
        h = (h + 1) & hmask;
    }
}
// PK: the node's kept row and C row from one 16-byte record (rec[x] = {kept start, kept length,
// C start, C length}; 32-bit offsets, used while both graphs hold < 2^31 entries): one line per
// node lookup instead of krowptr's and crowptr's two.
template <bool PK>
__global__ __launch_bounds__(256) void k_closure_sample(int64_t t0, int64_t cnt, int64_t n, uint32_t k0, uint32_t k1,
                                                        uint32_t iter, const int64_t* __restrict__ krowptr,
                                                        const int32_t* __restrict__ kcol,
                                                        const int64_t* __restrict__ crowptr,
                                                        const int32_t* __restrict__ ccol,
                                                        const int4* __restrict__ rec, int bits,
                                                        CloSlot* tab, uint64_t hmask, int64_t* slot) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= cnt) return;
    slot[i] = -1;
    const int64_t t = t0 + i;
    U4 ctr = {(uint32_t)t, (uint32_t)(t >> 32), iter, 0x5eedu};
    const U4 r = philox(ctr, k0, k1);
    const int32_t x = (int32_t)below(r.x, (uint32_t)n);
    int64_t kb, dk, cb = 0, dc = 0;
    if (PK) {
        const int4 rx = rec[x];
        kb = (uint32_t)rx.x; dk = rx.y; cb = (uint32_t)rx.z; dc = rx.w;
    } else {
        kb = krowptr[x];
        dk = krowptr[x + 1] - kb;
        if (crowptr) { cb = crowptr[x]; dc = crowptr[x + 1] - cb; }
    }
    const int64_t d = dk + dc;
    if (d < 2) return;
    const uint32_t i1 = below(r.y, (uint32_t)d);
    uint32_t i2 = below(r.z, (uint32_t)(d - 1));
    if (i2 >= i1) ++i2;
    const int32_t a = (int64_t)i1 < dk ? kcol[kb + i1] : ccol[cb + i1 - dk];
    const int32_t b = (int64_t)i2 < dk ? kcol[kb + i2] : ccol[cb + i2 - dk];
    const int32_t u = a < b ? a : b, v = a < b ? b : a;
    if (PK) {
        const int4 ru = rec[u];
        if (has_edge_row(kcol, (uint32_t)ru.x, (int64_t)(uint32_t)ru.x + ru.y, v)) return;
        if (ru.w > 0 && has_edge_row(ccol, (uint32_t)ru.z, (int64_t)(uint32_t)ru.z + ru.w, v)) return;   // an earlier block's candidate
    } else {
        if (has_edge_sorted(krowptr, kcol, u, v)) return;
        if (crowptr && has_edge_sorted(crowptr, ccol, u, v)) return;   // an earlier block's candidate
    }
    const uint64_t key = ((uint64_t)u << bits) | (uint64_t)v;
    slot[i] = clo_insert(tab, hmask, key, (uint32_t)i);   // dense: no shared counter (one hot address serialised the block)
}
// rec[x] = {kept row start, kept length, 0, 0}: the closure's first block (empty C graph)
__global__ void k_clo_rec_init(int64_t n, const int64_t* krowptr, int4* rec) {
    const int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (x >= n) return;
    const int64_t kb = krowptr[x];
    rec[x] = make_int4((int32_t)kb, (int32_t)(krowptr[x + 1] - kb), 0, 0);
}
// This block's candidates (the attempts that created a slot, in attempt order) appended to
// the accumulated list at the device-side count *nacc (no host round trip per block).
// The running count is snapshotted here (nacc[1] = nacc[0]), one launch before k_append_cand
// reads it: reading and bumping nacc[0] inside one launch raced across workgroups.
__global__ void k_slot_flags(int64_t n, const int64_t* slot, int64_t* flag, int64_t* nacc) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i > n) return;
    flag[i] = (i < n && slot[i] >= 0) ? 1 : 0;
    if (i == n) nacc[1] = nacc[0];
}
__global__ void k_append_cand(int64_t n, const int64_t* slot, const int64_t* pos, const CloSlot* tab, int64_t t0,
                              int64_t* nacc, uint64_t* akey, int64_t* aval) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t base = nacc[1];                  // the block's first entry (k_slot_flags); not written here
    if (i < n && slot[i] >= 0) {
        const CloSlot e = tab[slot[i]];
        akey[base + pos[i]] = e.key;
        aval[base + pos[i]] = t0 + (int64_t)e.att;
    }
    if (i == n) nacc[0] = base + pos[n];           // nobody in this launch reads [0]
}
// C graph, grown block by block: the new block's entries (both directions) are counted and
// scattered per node (int32 atomics, their owner beside them), then the grown graph is written
// into the other buffer entry by entry: an old entry of row x moves up by the new entries of the
// rows before x (nrow[x], an exclusive prefix sum) and those of x with smaller ids; a new entry
// lands after the old and new entries of its row with smaller ids.  Rows stay ascending, every
// pass is coalesced (round 5 merged row by row, one thread per node walking its row: ~0.35 ms
// per block at 4 M nodes, which 16 lpm blocks would pay 15 times).  Each entry carries its row
// (own[]) so no search over the row starts is needed.
__global__ void k_cgraph_ndeg(const int64_t* nacc, const uint64_t* akey, int bits, int32_t* ndeg) {
    const int64_t i = nacc[1] + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;   // this block's candidates
    if (i >= nacc[0]) return;
    atomicAdd(&ndeg[akey[i] >> bits], 1);
    atomicAdd(&ndeg[akey[i] & ((1ull << bits) - 1ull)], 1);
}
__global__ void k_cgraph_nfill(const int64_t* nacc, const uint64_t* akey, int bits, const int32_t* nrow, int32_t* cur,
                               int32_t* ncol, int32_t* nown) {
    const int64_t i = nacc[1] + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nacc[0]) return;
    const int32_t u = (int32_t)(akey[i] >> bits), v = (int32_t)(akey[i] & ((1ull << bits) - 1ull));
    const int32_t pu = nrow[u] + atomicAdd(&cur[u], 1), pv = nrow[v] + atomicAdd(&cur[v], 1);
    ncol[pu] = v; nown[pu] = u;
    ncol[pv] = u; nown[pv] = v;
}
// row starts of the grown graph (and the C half of the packed node records)
__global__ void k_cgraph_rows(int64_t n, const int64_t* crow, const int32_t* nrow, int64_t* crow2, int4* rec) {
    const int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (x > n) return;
    const int64_t o = crow[x] + nrow[x];
    crow2[x] = o;
    if (x < n && rec) {   // the node's C row in its closure record (k_closure_sample<true>)
        int2* rc = (int2*)(rec + x) + 1;
        *rc = make_int2((int32_t)o, (int32_t)(crow[x + 1] - crow[x] + (nrow[x + 1] - nrow[x])));
    }
}
// old entries (crow[n] of them), grid-stride over a fixed grid: the count is on the device
__global__ void k_cgraph_old(int64_t n, const int64_t* crow, const int32_t* col, const int32_t* own, const int32_t* nrow,
                             const int32_t* ncol, int32_t* col2, int32_t* own2) {
    const int64_t m = crow[n];
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < m; j += (int64_t)gridDim.x * blockDim.x) {
        const int32_t x = own[j], y = col[j];
        const int32_t nb = nrow[x], ne = nrow[x + 1];
        int32_t k = 0;
        for (int32_t q = nb; q < ne; ++q) k += ncol[q] < y ? 1 : 0;   // a row gains a few entries per block
        const int64_t p = j + nb + k;
        col2[p] = y;
        own2[p] = x;
    }
}
// new entries (nrow[n] of them)
__global__ void k_cgraph_new(int64_t n, const int64_t* crow, const int32_t* col, const int32_t* nrow,
                             const int32_t* ncol, const int32_t* nown, int32_t* col2, int32_t* own2) {
    const int64_t m = nrow[n];
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x) {
        const int32_t x = nown[i], y = ncol[i];
        int64_t lo = crow[x], hi = crow[x + 1];
        const int64_t b0 = lo;
        while (lo < hi) {                         // old entries of x below y (the row is ascending)
            const int64_t mid = (lo + hi) >> 1;
            if (col[mid] < y) lo = mid + 1;
            else hi = mid;
        }
        const int32_t nb = nrow[x], ne = nrow[x + 1];
        int32_t k = 0;
        for (int32_t q = nb; q < ne; ++q) k += ncol[q] < y ? 1 : 0;
        const int64_t p = b0 + nb + (lo - b0) + k;
        col2[p] = y;
        own2[p] = x;
    }
}
__global__ void k_pairs_keys(int64_t np_, const int32_t* pairs, const int64_t* krowptr, const int32_t* kcol,
                             int bits, uint64_t* key, int64_t* val) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= np_) return;
    const uint64_t sent = (1ull << (2 * bits)) - 1ull;
    const int32_t a = pairs[2 * t], b = pairs[2 * t + 1];
    uint64_t k = sent;
    if (a != b) {
        const int32_t u = a < b ? a : b, v = a < b ? b : a;
        if (!has_edge_sorted(krowptr, kcol, u, v)) k = ((uint64_t)u << bits) | (uint64_t)v;
    }
    key[t] = k;
    val[t] = t;
}
// first occurrence of each candidate (stable radix sort keeps sample order in a key run)
__global__ void k_first_flags(int64_t n, const uint64_t* key, int bits, int64_t* flag) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i > n) return;
    if (i == n) { flag[i] = 0; return; }
    const uint64_t sent = (1ull << (2 * bits)) - 1ull;
    flag[i] = (key[i] != sent && (i == 0 || key[i - 1] != key[i])) ? 1 : 0;
}
__global__ void k_scatter_cand(int64_t n, const int64_t* flag, const int64_t* pos, const uint64_t* key,
                               const int64_t* val, int bits, int64_t age_base, int32_t* cu, int32_t* cv,
                               int64_t* cage) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || !flag[i]) return;
    const int64_t p = pos[i];
    cu[p] = (int32_t)(key[i] >> bits);
    cv[p] = (int32_t)(key[i] & ((1ull << bits) - 1ull));
    cage[p] = age_base + val[i];  // creation order = first sample index
}

static void finish_candidates(Ctx& c, int64_t n, uint64_t* k1, int64_t* v1, int iteration) {
    const int64_t cap = n > 0 ? n : 1;
    uint64_t* k2 = ensure<uint64_t>(c.mkey2, cap);
    int64_t* v2 = ensure<int64_t>(c.midx2, cap);
    sort_pairs_public(c, (const uint64_t*)k1, k2, (const int64_t*)v1, v2, n, 2 * c.key_bits);
    int64_t* fl = ensure<int64_t>(c.flag, n + 1 > 2 * (c.g.m + 1) + 1 ? n + 1 : 2 * (c.g.m + 1) + 1);
    int64_t* ps = ensure<int64_t>(c.pos, n + 1 > 2 * (c.g.m + 1) + 1 ? n + 1 : 2 * (c.g.m + 1) + 1);
    k_first_flags<<<nblk(n + 1), TB, 0, c.stream>>>(n, k2, c.key_bits, fl);
    exclusive_scan(c, fl, ps, n + 1);
    c.n_cand = read_i64(c, ps + n);
    // closure + (up to N) repair edges share the "added" arrays
    const int64_t acap = c.n_cand + c.N + 1;
    int32_t* cu = ensure<int32_t>(c.cu, acap);
    int32_t* cv = ensure<int32_t>(c.cv, acap);
    ensure<int32_t>(c.cw2, acap);
    int64_t* cage = ensure<int64_t>(c.cage, acap);
    const int64_t base = (int64_t)(iteration + 1) << AGE_ITER_SHIFT;
    k_scatter_cand<<<nblk(n), TB, 0, c.stream>>>(n, fl, ps, k2, v2, c.key_bits, base, cu, cv, cage);
}

// Buffers of a closure over `attempts` (sized for the whole run: no reallocation between blocks)
namespace {
struct Clo {
    int R;
    int64_t rcap;
    uint64_t hsize;
    CloSlot* tab;
    int4* rec;                     // packed node records, or null (graphs past 2^31 entries)
    int64_t *slot, *fl, *ps, *aval, *nacc;
    uint64_t* akey;
    int32_t *nrow, *ncur, *ncol, *nown;
};
}  // namespace
static Clo clo_bufs(Ctx& c, int64_t attempts) {
    Clo b;
    const int64_t cap = attempts > 0 ? attempts : 1;
    b.R = (int)std::max<int64_t>(1, std::min<int64_t>(closure_blocks(c), cap));
    b.rcap = (cap + b.R - 1) / b.R + 1;                            // attempts per block (at most)
    const int64_t N = c.N;
    b.hsize = 1024;
    while (b.hsize < 2 * (uint64_t)b.rcap) b.hsize <<= 1;          // one block's pairs, load <= 1/2
    b.tab = ensure<CloSlot>(c.clo_hkey, b.hsize);
    // the kept graph holds 2 * kept_m entries (consensus_apply), the C graph at most 2 * attempts
    b.rec = (c.clo_pack && 2 * c.kept_m < ((int64_t)1 << 31) && 2 * cap < ((int64_t)1 << 31))
                ? ensure<int4>(c.clo_rec, N) : nullptr;
    b.slot = ensure<int64_t>(c.clo_list, b.rcap);
    b.fl = ensure<int64_t>(c.nodetmp, std::max<int64_t>(b.rcap + 1, N + 1));
    b.ps = ensure<int64_t>(c.nodetmp2, std::max<int64_t>(b.rcap + 1, N + 1));
    b.akey = ensure<uint64_t>(c.clo_akey, cap);
    b.aval = ensure<int64_t>(c.clo_aval, cap);
    b.nacc = ensure<int64_t>(c.clo_cnt, 4);                         // [0] candidates so far, [1] this block's first, [2..3] scratch
    // the C graph (ping-pong; sized for every candidate: no reallocation inside the loop)
    b.nrow = ensure<int32_t>(c.clo_nrow, 2 * (N + 1));             // a block's new-entry offsets | cursors
    b.ncur = b.nrow + (N + 1);
    b.ncol = ensure<int32_t>(c.clo_ncol, 4 * b.rcap);   // a block's new entries | their rows
    b.nown = b.ncol + 2 * b.rcap;
    if (b.R > 1)
        for (DevBuf* d : {&c.clo_col, &c.clo_col2, &c.clo_own, &c.clo_own2}) ensure<int32_t>(*d, 2 * cap);
    for (DevBuf* d : {&c.clo_rowptr, &c.clo_rowptr2}) ensure<int64_t>(*d, N + 1);
    return b;
}
static void clo_reset(Ctx& c, const Clo& b) {
    FC_HIP(hipMemsetAsync(b.nacc, 0, 2 * sizeof(int64_t), c.stream));
    FC_HIP(hipMemsetAsync(c.clo_rowptr.p, 0, sizeof(int64_t) * (c.N + 1), c.stream));   // empty C graph
    if (b.rec) k_clo_rec_init<<<nblk(c.N), TB, 0, c.stream>>>(c.N, c.krowptr.as<int64_t>(), b.rec);
}
static void clo_clear_table(Ctx& c, const Clo& b) {
    FC_HIP(hipMemsetAsync(b.tab, 0xff, sizeof(CloSlot) * b.hsize, c.stream));
}
// attempts [t0, t0 + n) of block r drawn into the (cleared) table; slot[i] >= 0 lists a new pair
static void clo_draw(Ctx& c, const Clo& b, int64_t t0, int64_t n, int iteration, int r) {
    const uint64_t s = mix64(c.seed ^ 0xC105u);
    const int64_t* crow = r > 0 ? c.clo_rowptr.as<int64_t>() : nullptr;
    const int32_t* ccol = r > 0 ? c.clo_col.as<int32_t>() : nullptr;
    if (b.rec)
        k_closure_sample<true><<<nblk(n), TB, 0, c.stream>>>(t0, n, c.N, (uint32_t)s, (uint32_t)(s >> 32),
                                                             (uint32_t)iteration, c.krowptr.as<int64_t>(),
                                                             c.kcol.as<int32_t>(), crow, ccol, b.rec, c.key_bits, b.tab,
                                                             b.hsize - 1, b.slot);
    else
        k_closure_sample<false><<<nblk(n), TB, 0, c.stream>>>(t0, n, c.N, (uint32_t)s, (uint32_t)(s >> 32),
                                                              (uint32_t)iteration, c.krowptr.as<int64_t>(),
                                                              c.kcol.as<int32_t>(), crow, ccol, nullptr, c.key_bits,
                                                              b.tab, b.hsize - 1, b.slot);
}
// the listed slots of the table (slot[0..n)) appended to the accumulated candidates; unless r is
// the last block, the C graph grows by them (rows ascending) for the next block
static void clo_append(Ctx& c, const Clo& b, int64_t n, int64_t t0, int r) {
    const int bits = c.key_bits;
    const int64_t N = c.N;
    k_slot_flags<<<nblk(n + 1), TB, 0, c.stream>>>(n, b.slot, b.fl, b.nacc);
    exclusive_scan(c, b.fl, b.ps, n + 1);
    k_append_cand<<<nblk(n + 1), TB, 0, c.stream>>>(n, b.slot, b.ps, b.tab, t0, b.nacc, b.akey, b.aval);
    if (r + 1 == b.R) return;
    FC_HIP(hipMemsetAsync(b.nrow, 0, sizeof(int32_t) * 2 * (N + 1), c.stream));
    k_cgraph_ndeg<<<nblk(n), TB, 0, c.stream>>>(b.nacc, b.akey, bits, b.ncur);
    exclusive_scan(c, b.ncur, b.nrow, N + 1);
    FC_HIP(hipMemsetAsync(b.ncur, 0, sizeof(int32_t) * (N + 1), c.stream));
    k_cgraph_nfill<<<nblk(n), TB, 0, c.stream>>>(b.nacc, b.akey, bits, b.nrow, b.ncur, b.ncol, b.nown);
    const int64_t* crow = c.clo_rowptr.as<int64_t>();
    k_cgraph_rows<<<nblk(N + 1), TB, 0, c.stream>>>(N, crow, b.nrow, c.clo_rowptr2.as<int64_t>(), b.rec);
    // old entries: at most 2 x the attempts before this block; new ones: 2 x this block's
    const unsigned og = (unsigned)std::max<int64_t>(1, std::min<int64_t>(nblk(2 * t0), 2048));
    const unsigned ng = (unsigned)std::max<int64_t>(1, std::min<int64_t>(nblk(2 * n), 2048));
    if (t0 > 0)
        k_cgraph_old<<<og, TB, 0, c.stream>>>(N, crow, c.clo_col.as<int32_t>(), c.clo_own.as<int32_t>(), b.nrow, b.ncol,
                                               c.clo_col2.as<int32_t>(), c.clo_own2.as<int32_t>());
    k_cgraph_new<<<ng, TB, 0, c.stream>>>(N, crow, c.clo_col.as<int32_t>(), b.nrow, b.ncol, b.nown,
                                           c.clo_col2.as<int32_t>(), c.clo_own2.as<int32_t>());
    std::swap(c.clo_rowptr, c.clo_rowptr2);
    std::swap(c.clo_col, c.clo_col2);
    std::swap(c.clo_own, c.clo_own2);
}

void closure_sample(Ctx& c, int64_t attempts, int iteration) {
    c.clo_next = -1;   // it resets the candidate table a sharded sequence was filling
    const int sl = timer_begin(c);
    const Clo b = clo_bufs(c, attempts);
    clo_reset(c, b);
    for (int r = 0; r < b.R; ++r) {
        const int64_t t0 = attempts * r / b.R, t1 = attempts * (r + 1) / b.R, n = t1 - t0;
        if (n <= 0) continue;
        clo_clear_table(c, b);
        clo_draw(c, b, t0, n, iteration, r);
        clo_append(c, b, n, t0, r);
    }
    // candidates in key order (first-sample ages ride along; the keys are distinct)
    finish_candidates(c, read_i64(c, b.nacc), b.akey, b.aval, iteration);
    timer_end(c, 2, sl);
}

// ---- the same closure with each block's attempts split over ranks (multi-GPU) ----------------
// A block's draws depend only on the attempt index (Philox counter) and on the graph the block
// draws from (kept graph + the C graph of the earlier blocks), so rank g can draw any sub-range
// [t_lo, t_hi) of block r.  Its pairs (deduplicated, first attempt each) go out as int64
// (key, attempt); the ranks' lists, all-gathered, are re-inserted into the table keeping the
// smallest attempt per key (atomicMin, as a single rank drawing the whole block does), and
// appended and grown exactly as closure_sample does: every rank ends with the same candidates.
__global__ void k_emit_cand(int64_t n, const int64_t* slot, const int64_t* pos, const CloSlot* tab, int64_t t0,
                            int64_t* out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || slot[i] < 0) return;
    const CloSlot e = tab[slot[i]];
    const int64_t p = pos[i];
    out[2 * p] = (int64_t)e.key;
    out[2 * p + 1] = t0 + (int64_t)e.att;
}
__global__ void k_closure_insert(int64_t cnt, const int64_t* __restrict__ in, int64_t t0, CloSlot* tab, uint64_t hmask,
                                 int64_t* slot) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= cnt) return;
    slot[i] = clo_insert(tab, hmask, (uint64_t)in[2 * i], (uint32_t)(in[2 * i + 1] - t0));
}

int closure_begin(Ctx& c, int64_t attempts, int iteration) {
    const int sl = timer_begin(c);
    const Clo b = clo_bufs(c, attempts);
    clo_reset(c, b);
    c.clo_attempts = attempts;
    c.clo_R = b.R;
    c.clo_next = 0;
    c.clo_iter = iteration;
    timer_end(c, 2, sl);
    return b.R;
}

int64_t closure_block_sample(Ctx& c, int r, int64_t t_lo, int64_t t_hi, int64_t* out, int64_t capacity) {
    const int sl = timer_begin(c);
    const Clo b = clo_bufs(c, c.clo_attempts);
    const int64_t n = t_hi - t_lo;
    int64_t count = 0;
    if (n > 0) {
        clo_clear_table(c, b);
        clo_draw(c, b, t_lo, n, c.clo_iter, r);
        k_slot_flags<<<nblk(n + 1), TB, 0, c.stream>>>(n, b.slot, b.fl, b.nacc + 2);   // its count snapshot into scratch
        exclusive_scan(c, b.fl, b.ps, n + 1);
        count = read_i64(c, b.ps + n);
        FC_REQUIRE(count <= capacity, FC_EINVAL,
                   "closure block output holds " + std::to_string(capacity) + " pairs; " + std::to_string(count) +
                       " drawn");
        if (count > 0) k_emit_cand<<<nblk(n), TB, 0, c.stream>>>(n, b.slot, b.ps, b.tab, t_lo, out);
    }
    timer_end(c, 2, sl);
    return count;
}

void closure_block_add(Ctx& c, int r, const int64_t* in, int64_t count) {
    const int sl = timer_begin(c);
    const Clo b = clo_bufs(c, c.clo_attempts);
    const int64_t t0 = c.clo_attempts * r / b.R;
    if (count > 0) {
        clo_clear_table(c, b);
        k_closure_insert<<<nblk(count), TB, 0, c.stream>>>(count, in, t0, b.tab, b.hsize - 1, b.slot);
        clo_append(c, b, count, t0, r);
    }
    c.clo_next = r + 1;
    timer_end(c, 2, sl);
}

int64_t closure_finish(Ctx& c) {
    const int sl = timer_begin(c);
    const Clo b = clo_bufs(c, c.clo_attempts);
    finish_candidates(c, read_i64(c, b.nacc), b.akey, b.aval, c.clo_iter);
    c.clo_next = -1;
    timer_end(c, 2, sl);
    return c.n_cand;
}

void closure_from_pairs(Ctx& c, int64_t npairs, const int32_t* pairs, int iteration) {
    c.clo_next = -1;
    const int64_t cap = npairs > 0 ? npairs : 1;
    int32_t* dp = ensure<int32_t>(c.ckey, 2 * cap);
    if (npairs > 0) FC_HIP(hipMemcpyAsync(dp, pairs, sizeof(int32_t) * 2 * npairs, hipMemcpyHostToDevice, c.stream));
    uint64_t* k1 = ensure<uint64_t>(c.mkey, cap);
    int64_t* v1 = ensure<int64_t>(c.midx, cap);
    if (npairs > 0)
        k_pairs_keys<<<nblk(npairs), TB, 0, c.stream>>>(npairs, dp, c.krowptr.as<int64_t>(), c.kcol.as<int32_t>(),
                                                         c.key_bits, k1, v1);
    finish_candidates(c, npairs, k1, v1, iteration);
}

void closure_partial(Ctx& c, int32_t* out) {
    if (!c.labT_valid) labels_transpose(c);
    launch_pair_partial<false>(c, c.n_cand, c.cu.as<int32_t>(), c.cv.as<int32_t>(), out);
}

// ------------------------------------------------------------------ repair
__global__ void k_closure_weights(int64_t n, int louvain, const int32_t* counts, int32_t* cw) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) cw[i] = louvain ? counts[i] : 0;  // lpm closure weight is always 0 (:302-304)
}
__global__ void k_deg_next(int64_t n, const int64_t* krowptr, int64_t* deg) {
    const int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (x < n) deg[x] = krowptr[x + 1] - krowptr[x];
}
// Only deg == 0 matters (isolates): a closure edge marks both ends with a plain store.
__global__ void k_deg_add(int64_t k, const int32_t* cu, const int32_t* cv, int64_t* deg) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= k) return;
    deg[cu[i]] = 1;
    deg[cv[i]] = 1;
}
// Indexed by NODE ORDER t (x = sigma[t]): nx.isolates visits nodes in node order.
__global__ void k_iso_flags(int64_t n, const int32_t* sigma, const int64_t* deg, const int64_t* rowptr,
                            int64_t* flag) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t > n) return;
    if (t == n) { flag[t] = 0; return; }
    const int32_t x = sigma[t];
    // isolated in nextgraph and has a neighbour in graph (else the reference raises)
    flag[t] = (deg[x] == 0 && rowptr[x + 1] > rowptr[x]) ? 1 : 0;
}
// Isolate bookkeeping in node order t: isoidx[x] = its index among the isolates (or -1).
__global__ void k_iso_index(int64_t n, const int32_t* sigma, const int64_t* flag, const int64_t* pos, int32_t* iso,
                            int64_t* isoidx) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    const int32_t x = sigma[t];
    if (!flag[t]) { isoidx[x] = -1; return; }
    const int64_t i = pos[t];
    isoidx[x] = i;
    iso[i] = x;
}
// Target of isolated node x: its neighbour in the OLD graph with the minimum old weight;
// ties -> first in networkx adjacency order = earlier neighbours ascending, then later
// neighbours by creation age (proof: DESIGN.md; pinned by tests/golden adj snapshots).
// One wave per isolate: lanes stride the row, then a lexicographic (w, sec, j) min over the
// wave -- a row walk of a hub in the old graph was one thread's serial dependent loads.
__global__ __launch_bounds__(256) void k_iso_target(int64_t k, const int32_t* npos, const int32_t* iso,
                                                    const int64_t* rowptr, const int32_t* col, const int32_t* cw,
                                                    const int32_t* ceid, const int64_t* eage, int32_t* target,
                                                    int32_t* tw) {
    const int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int lane = threadIdx.x & 63;
    if (i >= k) return;                       // wave-uniform
    const int32_t x = iso[i];
    const int32_t t = npos[x];
    int32_t bw = 0x7fffffff;
    int64_t bs = 0x7fffffffffffffffll, bj = 0x7fffffffffffffffll;
    for (int64_t j = rowptr[x] + lane; j < rowptr[x + 1]; j += 64) {
        const int32_t w = cw[j];
        const int32_t py = npos[col[j]];
        const int64_t sec = (py < t) ? (int64_t)py : ((int64_t)1 << 62) + eage[ceid[j]];
        if (w < bw || (w == bw && (sec < bs || (sec == bs && j < bj)))) { bw = w; bs = sec; bj = j; }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const int32_t ow = __shfl_xor(bw, off);
        const int64_t os = __shfl_xor(bs, off), oj = __shfl_xor(bj, off);
        if (ow < bw || (ow == bw && (os < bs || (os == bs && oj < bj)))) { bw = ow; bs = os; bj = oj; }
    }
    if (lane == 0) {
        target[i] = bj != 0x7fffffffffffffffll ? col[bj] : -1;
        tw[i] = bw;
    }
}
// Sequential live-isolates semantics (nx.isolates is a lazy generator): x is skipped iff
// an earlier repaired node chose x.  Resolved by Jacobi sweeps over the DAG x' -> T(x').
__global__ void k_iso_hit(int64_t k, const int32_t* npos, const int32_t* iso, const int64_t* isoidx,
                          const int32_t* target, const int32_t* active, int32_t* hit) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= k || !active[i]) return;
    const int32_t y = target[i];
    const int64_t j = isoidx[y];
    if (j >= 0 && npos[y] > npos[iso[i]]) hit[j] = 1;   // y comes later in node order
}
__global__ void k_iso_update(int64_t k, const int32_t* hit, int32_t* active, int32_t* changed) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= k) return;
    const int32_t a = hit[i] ? 0 : 1;
    if (a != active[i]) { active[i] = a; *changed = 1; }
}
// The same fixpoint in ONE workgroup with the state in LDS (k <= ISO_LDS isolates): no host
// round trip per Jacobi sweep (round 1 synchronised the host once per sweep, unbounded in the
// DAG depth).
constexpr int ISO_LDS = 16384;
__global__ __launch_bounds__(1024) void k_iso_resolve(int64_t k, const int32_t* npos, const int32_t* iso,
                                                      const int64_t* isoidx, const int32_t* target, int32_t* active) {
    __shared__ uint8_t s_act[ISO_LDS], s_hit[ISO_LDS];
    __shared__ int s_changed;
    for (int64_t i = threadIdx.x; i < k; i += blockDim.x) s_act[i] = 0;   // all-zero start: the first pass flips all
    for (int64_t it = 0; it <= k + 1; ++it) {
        for (int64_t i = threadIdx.x; i < k; i += blockDim.x) s_hit[i] = 0;
        if (threadIdx.x == 0) s_changed = 0;
        __syncthreads();
        if (it > 0)
            for (int64_t i = threadIdx.x; i < k; i += blockDim.x) {
                if (!s_act[i]) continue;
                const int32_t y = target[i];
                const int64_t j = isoidx[y];
                if (j >= 0 && npos[y] > npos[iso[i]]) s_hit[j] = 1;
            }
        __syncthreads();
        for (int64_t i = threadIdx.x; i < k; i += blockDim.x) {
            const uint8_t a = s_hit[i] ? 0 : 1;
            if (a != s_act[i]) { s_act[i] = a; s_changed = 1; }
        }
        __syncthreads();
        const bool done = !s_changed && it > 0;   // block-uniform
        __syncthreads();
        if (done) break;
    }
    for (int64_t i = threadIdx.x; i < k; i += blockDim.x) active[i] = s_act[i];
}
__global__ void k_iso_flag64(int64_t k, const int32_t* active, int64_t* f) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < k) f[i] = active[i];
    else if (i == k) f[i] = 0;
}
__global__ void k_repair_edges(int64_t k, const int32_t* npos, const int64_t* f, const int64_t* p,
                               const int32_t* iso, const int32_t* target, const int32_t* tw, int64_t base, int64_t off,
                               int32_t* cu, int32_t* cv, int32_t* cw, int64_t* cage) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= k || !f[i]) return;
    const int32_t x = iso[i], y = target[i];
    const int64_t q = off + p[i];
    cu[q] = x < y ? x : y;
    cv[q] = x < y ? y : x;
    cw[q] = tw[i];                 // carries the old weight (:195)
    cage[q] = base + AGE_REPAIR_OFFSET + npos[x];   // added in node order
}

static int64_t repair(Ctx& c, int iteration) {
    const int64_t n = c.N;
    Graph& g = c.g;  // still the OLD graph here
    int64_t* deg = ensure<int64_t>(c.deg_next, n + 1);
    k_deg_next<<<nblk(n), TB, 0, c.stream>>>(n, c.krowptr.as<int64_t>(), deg);
    if (c.n_cand > 0) k_deg_add<<<nblk(c.n_cand), TB, 0, c.stream>>>(c.n_cand, c.cu.as<int32_t>(), c.cv.as<int32_t>(), deg);
    int64_t* fl = ensure<int64_t>(c.nodetmp, n + 1);
    int64_t* ps = ensure<int64_t>(c.nodetmp2, n + 1);
    const int32_t* sigma = c.sigma.as<int32_t>();
    const int32_t* npos = c.npos.as<int32_t>();
    k_iso_flags<<<nblk(n + 1), TB, 0, c.stream>>>(n, sigma, deg, g.rowptr.as<int64_t>(), fl);
    exclusive_scan(c, fl, ps, n + 1);
    const int64_t k = read_i64(c, ps + n);
    c.n_iso = k;
    if (k == 0) return 0;
    int32_t* iso = ensure<int32_t>(c.iso, k);
    int64_t* isoidx = ensure<int64_t>(c.isoflag, n);
    int32_t* target = ensure<int32_t>(c.target, k);
    int32_t* tw = ensure<int32_t>(c.tw, k);
    k_iso_index<<<nblk(n), TB, 0, c.stream>>>(n, sigma, fl, ps, iso, isoidx);
    k_iso_target<<<nblk(k * 64), TB, 0, c.stream>>>(k, npos, iso, g.rowptr.as<int64_t>(), g.col.as<int32_t>(),
                                                     g.cw.as<int32_t>(), g.ceid.as<int32_t>(), g.eage.as<int64_t>(),
                                                     target, tw);
    int32_t* active = ensure<int32_t>(c.active, k);
    int32_t* hit = ensure<int32_t>(c.hit, k + 1);
    int32_t* changed = hit + k;
    if (k <= ISO_LDS) {
        k_iso_resolve<<<1, 1024, 0, c.stream>>>(k, npos, iso, isoidx, target, active);
    } else {
        // many isolates: multi-block Jacobi sweeps, the host checking for a fixpoint every 8
        FC_HIP(hipMemsetAsync(active, 0, sizeof(int32_t) * k, c.stream));  // all-zero start: first pass flips all
        for (int64_t it = 0; it <= k + 8; ) {
            FC_HIP(hipMemsetAsync(changed, 0, sizeof(int32_t), c.stream));
            for (int s = 0; s < 8; ++s, ++it) {
                FC_HIP(hipMemsetAsync(hit, 0, sizeof(int32_t) * k, c.stream));
                if (it > 0) k_iso_hit<<<nblk(k), TB, 0, c.stream>>>(k, npos, iso, isoidx, target, active, hit);
                if (s == 7) FC_HIP(hipMemsetAsync(changed, 0, sizeof(int32_t), c.stream));   // the last sweep decides
                k_iso_update<<<nblk(k), TB, 0, c.stream>>>(k, hit, active, changed);
            }
            int32_t ch = 0;
            FC_HIP(hipMemcpyAsync(&ch, changed, sizeof(int32_t), hipMemcpyDeviceToHost, c.stream));
            sync(c);
            if (!ch) break;
        }
    }
    int64_t* f = ensure<int64_t>(c.nodetmp, k + 1);   // fl no longer needed
    int64_t* p = ensure<int64_t>(c.nodetmp2, k + 1);
    k_iso_flag64<<<nblk(k + 1), TB, 0, c.stream>>>(k, active, f);
    exclusive_scan(c, f, p, k + 1);
    const int64_t nrep = read_i64(c, p + k);
    const int64_t base = (int64_t)(iteration + 1) << AGE_ITER_SHIFT;
    k_repair_edges<<<nblk(k), TB, 0, c.stream>>>(k, npos, f, p, iso, target, tw, base, c.n_cand, c.cu.as<int32_t>(),
                                                  c.cv.as<int32_t>(), c.cw2.as<int32_t>(), c.cage.as<int64_t>());
    return nrep;
}

// ------------------------------------------------------------------ convergence check
__global__ __launch_bounds__(256) void k_count_unconv(int64_t m, int n_p, const int32_t* w,
                                                      unsigned long long* out) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int u = (e < m) && w[e] != 0 && w[e] != n_p;
    __shared__ unsigned long long s_u;
    if (threadIdx.x == 0) s_u = 0;
    __syncthreads();
    const unsigned long long b = __ballot(u);
    if ((threadIdx.x & 63) == 0 && b) atomicAdd(&s_u, (unsigned long long)__popcll(b));
    __syncthreads();
    if (threadIdx.x == 0 && s_u) atomicAdd(shard(out, 1, 0), s_u);
}
int64_t count_unconverged(Ctx& c, const int32_t* w, int64_t m, int n_p) {
    unsigned long long* ctr = shards_begin(c, 1);
    if (m > 0) k_count_unconv<<<nblk(m), TB, 0, c.stream>>>(m, n_p, w, ctr);
    int64_t h[1];
    shards_fold(c, 1, 0u, h);
    return h[0];
}

void closure_apply(Ctx& c, int algo, int n_p, const int32_t* counts, int iteration) {
    int sl = timer_begin(c);
    if (c.n_cand > 0)
        k_closure_weights<<<nblk(c.n_cand), TB, 0, c.stream>>>(c.n_cand, is_louvain(algo), counts,
                                                               c.cw2.as<int32_t>());
    int64_t nrep = 0;
    if (is_louvain(algo)) nrep = repair(c, iteration);  // lpm has no repair (:260-310)
    timer_end(c, 2, sl);
    sl = timer_begin(c);
    graph_merge_next(c, c.n_cand + nrep);
    timer_end(c, 3, sl);
    (void)n_p;
}

}  // namespace fc
