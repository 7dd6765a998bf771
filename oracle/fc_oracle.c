/*
 * fc_oracle.c -- CPU restatement of ytabatabaee/fastconsensus's consensus inner loop.
 *
 *   *** TEST INFRASTRUCTURE ONLY ***
 *   Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 *   this library, and only as the CHECKER (or the timed CPU baseline).  The product
 *   path (fastconsensus_amd) never links, imports or falls back to it.
 *
 * Parity status: the deterministic parts (consensus rule, threshold, convergence
 * check, closure given samples, isolate repair, adjacency order) are PINNED against
 * golden vectors produced by the reference itself (tests/golden/make_golden.py).
 * The community-detection arithmetic (python-louvain 0.15 level 0, igraph 0.9.7 LPA)
 * is restated from the published algorithms; those libraries are absent from the
 * container, so that part is "parity unpinned" (statistical comparisons only).
 *
 * Every function cites the reference line it restates (fast_consensus.py).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

typedef int32_t i32;
typedef int64_t i64;
typedef uint64_t u64;
typedef uint8_t u8;

/* ------------------------------------------------------------------ RNG (oracle's own) */
static inline u64 splitmix64(u64* s) {
    u64 z = (*s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static inline u64 rng_below(u64* s, u64 n) { /* unbiased enough for tests: 128-bit multiply */
    return (u64)(((unsigned __int128)splitmix64(s) * n) >> 64);
}
static void shuffle_i32(i32* a, i64 n, u64* s) {
    for (i64 i = n - 1; i > 0; --i) {
        i64 j = (i64)rng_below(s, (u64)(i + 1));
        i32 t = a[i]; a[i] = a[j]; a[j] = t;
    }
}

/* ------------------------------------------------------------------ consensus rule
 * Louvain branch, fast_consensus.py:150-159 (literal loop, not the closed form):
 *   nextgraph weight starts at 0 (:145-146); if graph weight not in (0, n_p) (:153):
 *   for each partition i: same community -> += 1 (:156-157), else -> = old weight (:159).
 * LPM branch, fast_consensus.py:273-280: count of partitions with u, v co-clustered.
 * algo 2: the new_consensus.py fork's louvain rule (new_consensus.py:155-163, literal):
 *   nextgraph weight starts at 0 (:149-150); if graph weight not in (0, n_p) (:157):
 *   += 1 per partition that co-clusters (:158-160); else (:161-163) -> = graph weight.
 * labels are replica-major [n_p][N].  algo: 0 = louvain, 1 = lpm, 2 = louvain (new rule).
 */
void orc_consensus(int algo, i64 m, const i32* eu, const i32* ev, const i32* w_in, int n_p,
                   i64 N, const i32* lab, i32* w_out) {
#pragma omp parallel for schedule(static)
    for (i64 e = 0; e < m; ++e) {
        const i32 u = eu[e], v = ev[e];
        i32 nw = 0;
        if (algo == 0) {
            const i32 w = w_in[e];
            if (w != 0 && w != n_p) {
                for (int i = 0; i < n_p; ++i) {
                    if (lab[(i64)i * N + u] == lab[(i64)i * N + v]) nw += 1;
                    else nw = w;
                }
            }
        } else if (algo == 2) {
            const i32 w = w_in[e];
            if (w != 0 && w != n_p) {
                for (int i = 0; i < n_p; ++i)
                    if (lab[(i64)i * N + u] == lab[(i64)i * N + v]) nw += 1;
            } else {
                nw = w;
            }
        } else {
            for (int i = 0; i < n_p; ++i) nw += (lab[(i64)i * N + u] == lab[(i64)i * N + v]);
        }
        w_out[e] = nw;
    }
}

/* threshold: remove iff weight < thresh*n_p (fast_consensus.py:163-168, :284-288),
 * Python float64 product and compare.  Returns the kept count. */
i64 orc_threshold(i64 m, const i32* w, double tau, int n_p, u8* keep) {
    const double cut = tau * (double)n_p;
    i64 kept = 0;
    for (i64 e = 0; e < m; ++e) {
        keep[e] = !((double)w[e] < cut);
        kept += keep[e];
    }
    return kept;
}

/* check_consensus_graph (fast_consensus.py:17-37): count weights not in {0, n_p};
 * not converged iff count > delta * number_of_edges.  keep may be NULL. */
int orc_check(i64 m, const i32* w, const u8* keep, int n_p, double delta, i64* count_out) {
    i64 count = 0, mm = 0;
    for (i64 e = 0; e < m; ++e) {
        if (keep && !keep[e]) continue;
        ++mm;
        if (w[e] != 0 && w[e] != n_p) ++count;
    }
    if (count_out) *count_out = count;
    return ((double)count > delta * (double)mm) ? 0 : 1;
}

/* ------------------------------------------------------------------ sorted edge sets */
static inline u64 ekey(i32 u, i32 v) { return ((u64)(uint32_t)u << 32) | (uint32_t)v; }

static i64 find_key(const i32* eu, const i32* ev, i64 m, u64 key) {
    i64 lo = 0, hi = m;
    while (lo < hi) {
        i64 mid = (lo + hi) >> 1;
        u64 k = ekey(eu[mid], ev[mid]);
        if (k < key) lo = mid + 1; else hi = mid;
    }
    return (lo < m && ekey(eu[lo], ev[lo]) == key) ? lo : -1;
}

typedef struct { u64 key; i64 idx; } kv_t;
static int cmp_kv(const void* a, const void* b) {
    const kv_t* x = (const kv_t*)a; const kv_t* y = (const kv_t*)b;
    if (x->key != y->key) return x->key < y->key ? -1 : 1;
    return x->idx < y->idx ? -1 : (x->idx > y->idx);
}
static int cmp_idx(const void* a, const void* b) {
    const kv_t* x = (const kv_t*)a; const kv_t* y = (const kv_t*)b;
    return x->idx < y->idx ? -1 : (x->idx > y->idx);
}

/* Triadic closure given the recorded sample pairs (fast_consensus.py:175-190 louvain,
 * :292-304 lpm).  Sequential semantics: pair t adds (a,b) iff it is absent from the
 * post-threshold graph (eu,ev sorted canonical) and from the pairs already added.
 * Weight: louvain = #partitions with a, b co-clustered (:186-190); lpm = 0 always
 * (`a in communities[i]` compares an int with a set of frozensets, :302-304).
 * Output in first-occurrence order; out_first[k] = sample index t of edge k.
 * Returns the number of new edges. */
i64 orc_closure_pairs(int algo, i64 m, const i32* eu, const i32* ev, i64 npairs,
                      const i32* pairs, int n_p, i64 N, const i32* lab, i32* out_u,
                      i32* out_v, i32* out_w, i64* out_first) {
    kv_t* kv = (kv_t*)malloc(sizeof(kv_t) * (size_t)(npairs > 0 ? npairs : 1));
    i64 n = 0;
    for (i64 t = 0; t < npairs; ++t) {
        i32 a = pairs[2 * t], b = pairs[2 * t + 1];
        i32 u = a < b ? a : b, v = a < b ? b : a;
        if (u == v) continue;
        kv[n].key = ekey(u, v); kv[n].idx = t; ++n;
    }
    qsort(kv, (size_t)n, sizeof(kv_t), cmp_kv);
    i64 k = 0;
    for (i64 i = 0; i < n; ++i) {
        if (i > 0 && kv[i].key == kv[i - 1].key) continue;         /* later duplicate */
        i32 u = (i32)(kv[i].key >> 32), v = (i32)(kv[i].key & 0xffffffffu);
        if (find_key(eu, ev, m, kv[i].key) >= 0) continue;          /* has_edge (:183) */
        kv[k++] = kv[i];
        (void)u; (void)v;
    }
    qsort(kv, (size_t)k, sizeof(kv_t), cmp_idx);
    for (i64 i = 0; i < k; ++i) {
        i32 u = (i32)(kv[i].key >> 32), v = (i32)(kv[i].key & 0xffffffffu);
        i32 w = 0;
        if (algo == 0)
            for (int r = 0; r < n_p; ++r) w += (lab[(i64)r * N + u] == lab[(i64)r * N + v]);
        out_u[i] = u; out_v[i] = v; out_w[i] = w; out_first[i] = kv[i].idx;
    }
    free(kv);
    return k;
}

/* ------------------------------------------------------------------ adjacency order
 * networkx adjacency order of `graph` (always produced by Graph.copy(), :131, :198):
 * neighbours earlier in node order first, ascending; then later neighbours in edge
 * creation order (age).  Proven in DESIGN.md §"adjacency order"; pinned by the
 * adj* snapshots in the golden fixtures.  Writes a CSR in that order. */
typedef struct { i32 nbr; i64 key; i32 w; } adj_t;
static int cmp_adj(const void* a, const void* b) {
    const adj_t* x = (const adj_t*)a; const adj_t* y = (const adj_t*)b;
    if (x->key != y->key) return x->key < y->key ? -1 : 1;
    return 0;
}
void orc_adjacency_order(i64 N, i64 m, const i32* eu, const i32* ev, const i32* w,
                         const i64* age, const i32* npos, i64* ptr, i32* nbr, i32* nw) {
    memset(ptr, 0, sizeof(i64) * (size_t)(N + 1));
    for (i64 e = 0; e < m; ++e) { ptr[eu[e] + 1]++; ptr[ev[e] + 1]++; }
    for (i64 x = 0; x < N; ++x) ptr[x + 1] += ptr[x];
    adj_t* tmp = (adj_t*)malloc(sizeof(adj_t) * (size_t)(2 * m + 1));
    i64* fill = (i64*)malloc(sizeof(i64) * (size_t)(N + 1));
    memcpy(fill, ptr, sizeof(i64) * (size_t)N);
    for (i64 e = 0; e < m; ++e) {
        /* ids may be an internal numbering; node order is npos[] (NULL: the ids themselves) */
        i32 u = eu[e], v = ev[e];
        if (npos && npos[u] > npos[v]) { i32 t = u; u = v; v = t; }     /* u earlier in node order */
        const i64 pu = npos ? npos[u] : u;
        /* in row v, u is an earlier neighbour: key = its node position (ascending) */
        adj_t a = {u, pu, w[e]};
        tmp[fill[v]++] = a;
        /* in row u, v is a later neighbour: key = N + age (after all earlier ones) */
        adj_t b = {v, (i64)N + age[e], w[e]};
        tmp[fill[u]++] = b;
    }
    for (i64 x = 0; x < N; ++x)
        qsort(tmp + ptr[x], (size_t)(ptr[x + 1] - ptr[x]), sizeof(adj_t), cmp_adj);
    for (i64 j = 0; j < 2 * m; ++j) { nbr[j] = tmp[j].nbr; if (nw) nw[j] = tmp[j].w; }
    free(tmp); free(fill);
}

/* Isolate repair (fast_consensus.py:193-195).  For each node x in node order that has
 * degree 0 in nextgraph AT VISIT TIME (nx.isolates is a lazy generator), connect it to
 * the neighbour y of x in the OLD graph with the minimum old weight -- stable sort, so
 * ties go to the first neighbour in networkx adjacency order -- carrying that weight.
 * old graph: (m_old, ou, ov, ow, oage); nextgraph degrees: deg[N] (updated in place).
 * Returns the number of repair edges written to out_u/out_v/out_w (canonical u<v) in
 * the order they are added; out_x (may be NULL) receives the repaired node x. */
i64 orc_repair(i64 N, i64 m_old, const i32* ou, const i32* ov, const i32* ow, const i64* oage,
               const i32* sigma, i64* deg, i32* out_u, i32* out_v, i32* out_w, i64* out_x) {
    /* sigma (may be NULL): node position -> id; nodes are visited in node order */
    i64* ptr = (i64*)malloc(sizeof(i64) * (size_t)(N + 1));
    i32* nbr = (i32*)malloc(sizeof(i32) * (size_t)(2 * m_old + 1));
    i32* nw = (i32*)malloc(sizeof(i32) * (size_t)(2 * m_old + 1));
    i32* npos = NULL;
    if (sigma) {
        npos = (i32*)malloc(sizeof(i32) * (size_t)(N ? N : 1));
        for (i64 t = 0; t < N; ++t) npos[sigma[t]] = (i32)t;
    }
    orc_adjacency_order(N, m_old, ou, ov, ow, oage, npos, ptr, nbr, nw);
    i64 k = 0;
    for (i64 t = 0; t < N; ++t) {
        const i64 x = sigma ? sigma[t] : t;
        if (deg[x] != 0) continue;
        if (ptr[x + 1] == ptr[x]) continue;        /* reference would raise IndexError */
        i64 best = ptr[x];
        for (i64 j = ptr[x] + 1; j < ptr[x + 1]; ++j)
            if (nw[j] < nw[best]) best = j;          /* strict: first minimum wins */
        i32 y = nbr[best];
        out_u[k] = (i32)(x < y ? x : y); out_v[k] = (i32)(x < y ? y : x); out_w[k] = nw[best];
        if (out_x) out_x[k] = t;   /* creation order of repair edges = node order of x */
        ++k;
        deg[x]++; deg[y]++;
    }
    free(ptr); free(nbr); free(nw); free(npos);
    return k;
}

/* Sort + merge: canonical sorted edge list from an unsorted one (stable on equal keys
 * never happens: edge sets are simple).  perm receives the source index order. */
void orc_sort_edges(i64 m, const i32* eu, const i32* ev, i64* perm) {
    kv_t* kv = (kv_t*)malloc(sizeof(kv_t) * (size_t)(m > 0 ? m : 1));
    for (i64 e = 0; e < m; ++e) { kv[e].key = ekey(eu[e], ev[e]); kv[e].idx = e; }
    qsort(kv, (size_t)m, sizeof(kv_t), cmp_kv);
    for (i64 e = 0; e < m; ++e) perm[e] = kv[e].idx;
    free(kv);
}

/* ------------------------------------------------------------------ python-louvain level 0
 * Restatement of python-louvain 0.15 `generate_dendrogram(graph, randomize=True)` level 0
 * = `status.init` + `__one_level` (called at fast_consensus.py:148, :384), from the
 * published package source (not vendored; not line-citable here):
 *   passes over a freshly shuffled node order; per node: remove from own community,
 *   incr = remove_cost + dnc - deg(com)*k_i/(2*tw) over neighbour communities in a
 *   shuffled order, strict > best (starting at 0 = stay); stop when a pass improves
 *   modularity by < 1e-7 (__MIN) or moves nothing.  float64 arithmetic as in Python.
 * Output labels are renumbered 0..k-1 by first appearance in node order.
 * CSR: symmetric, no self loops.  Returns the number of passes. */
static double modularity_status(i64 N, const double* internals, const double* degrees, double tw) {
    double q = 0.0;
    if (tw <= 0) return 0.0;
    for (i64 c = 0; c < N; ++c) {
        if (degrees[c] == 0.0 && internals[c] == 0.0) continue;
        q += internals[c] / tw - (degrees[c] / (2.0 * tw)) * (degrees[c] / (2.0 * tw));
    }
    return q;
}

static void renumber(i64 N, i32* lab, i32* map) {
    for (i64 i = 0; i < N; ++i) map[i] = -1;
    i32 next = 0;
    for (i64 i = 0; i < N; ++i) {
        if (map[lab[i]] < 0) map[lab[i]] = next++;
        lab[i] = map[lab[i]];
    }
}

int orc_louvain_level0(i64 N, const i64* rowptr, const i32* col, const i32* w, u64 seed,
                       i32* lab) {
    u64 s = seed ^ 0xD1B54A32D192ED03ull;
    double* gdeg = (double*)calloc((size_t)N, sizeof(double));
    double* degrees = (double*)calloc((size_t)N, sizeof(double));
    double* internals = (double*)calloc((size_t)N, sizeof(double));
    double* neighw = (double*)calloc((size_t)N, sizeof(double));
    i32* order = (i32*)malloc(sizeof(i32) * (size_t)(N ? N : 1));
    i32* ncoms = (i32*)malloc(sizeof(i32) * (size_t)(N ? N : 1));
    u8* seen = (u8*)calloc((size_t)N, 1);
    double tw = 0.0;
    for (i64 i = 0; i < N; ++i) {
        double d = 0.0;
        for (i64 j = rowptr[i]; j < rowptr[i + 1]; ++j) d += (double)w[j];
        gdeg[i] = d; degrees[i] = d; internals[i] = 0.0; lab[i] = (i32)i; order[i] = (i32)i;
        tw += d;
    }
    tw *= 0.5;                       /* graph.size(weight): each edge once */
    int passes = 0;
    if (tw > 0.0) {
        double new_mod = modularity_status(N, internals, degrees, tw), cur_mod;
        int modified = 1;
        while (modified) {
            cur_mod = new_mod;
            modified = 0;
            ++passes;
            shuffle_i32(order, N, &s);
            for (i64 t = 0; t < N; ++t) {
                const i32 node = order[t];
                const i32 com_node = lab[node];
                const double degc_totw = gdeg[node] / (tw * 2.0);
                i64 nc = 0;
                for (i64 j = rowptr[node]; j < rowptr[node + 1]; ++j) {
                    const i32 c = lab[col[j]];
                    if (col[j] == node) continue;
                    if (!seen[c]) { seen[c] = 1; ncoms[nc++] = c; neighw[c] = 0.0; }
                    neighw[c] += (double)w[j];
                }
                const double own_w = seen[com_node] ? neighw[com_node] : 0.0;
                const double remove_cost = -own_w + (degrees[com_node] - gdeg[node]) * degc_totw;
                degrees[com_node] -= gdeg[node];               /* __remove */
                internals[com_node] -= own_w;
                i32 best_com = com_node;
                double best_inc = 0.0;
                shuffle_i32(ncoms, nc, &s);
                for (i64 q = 0; q < nc; ++q) {
                    const i32 c = ncoms[q];
                    const double incr = remove_cost + neighw[c] - degrees[c] * degc_totw;
                    if (incr > best_inc) { best_inc = incr; best_com = c; }
                }
                const double bw = seen[best_com] ? neighw[best_com] : 0.0;
                degrees[best_com] += gdeg[node];                /* __insert */
                internals[best_com] += bw;
                lab[node] = best_com;
                if (best_com != com_node) modified = 1;
                for (i64 q = 0; q < nc; ++q) seen[ncoms[q]] = 0;
            }
            new_mod = modularity_status(N, internals, degrees, tw);
            if (new_mod - cur_mod < 1e-7) break;
        }
    }
    renumber(N, lab, ncoms);
    free(gdeg); free(degrees); free(internals); free(neighw); free(order); free(ncoms); free(seen);
    return passes;
}

/* ------------------------------------------------------------------ igraph 0.9.7 LPA
 * Restatement of igraph_community_label_propagation as called at fast_consensus.py:270
 * (no weights => every neighbour counts 1): unique initial labels; each sweep visits
 * nodes in a fresh random order and assigns a uniformly random dominant neighbour
 * label; another sweep is needed iff some visited node's current label was not
 * dominant.  Isolated nodes keep their label.  Returns the number of sweeps. */
int orc_lpa(i64 N, const i64* rowptr, const i32* col, u64 seed, i32* lab, int max_sweeps) {
    u64 s = seed ^ 0x8CB92BA72F3D8DD7ull;
    i32* order = (i32*)malloc(sizeof(i32) * (size_t)(N ? N : 1));
    i32* cnt = (i32*)calloc((size_t)N, sizeof(i32));
    i32* dom = (i32*)malloc(sizeof(i32) * (size_t)(N ? N : 1));
    i32* touched = (i32*)malloc(sizeof(i32) * (size_t)(N ? N : 1));
    for (i64 i = 0; i < N; ++i) { lab[i] = (i32)i; order[i] = (i32)i; }
    int sweeps = 0, running = 1;
    while (running && sweeps < max_sweeps) {
        running = 0;
        ++sweeps;
        shuffle_i32(order, N, &s);
        for (i64 t = 0; t < N; ++t) {
            const i32 v = order[t];
            i64 nt = 0, nd = 0;
            i32 maxc = 0;
            for (i64 j = rowptr[v]; j < rowptr[v + 1]; ++j) {
                const i32 l = lab[col[j]];
                if (cnt[l] == 0) touched[nt++] = l;
                const i32 c = ++cnt[l];
                if (c > maxc) { maxc = c; nd = 0; dom[nd++] = l; }
                else if (c == maxc) dom[nd++] = l;
            }
            if (nd > 0) {
                if (cnt[lab[v]] != maxc) running = 1;
                lab[v] = dom[rng_below(&s, (u64)nd)];
            }
            for (i64 q = 0; q < nt; ++q) cnt[touched[q]] = 0;
        }
    }
    renumber(N, lab, dom);
    free(order); free(cnt); free(dom); free(touched);
    return sweeps;
}

/* ------------------------------------------------------------------ leidenalg Leiden
 * Restatement of leidenalg.find_partition(G, ModularityVertexPartition, weights='weight',
 * seed=i, n_iterations=1) as called at fast_consensus.py:121-123 (n_p times, :210-211 and
 * :386-387).  leidenalg is not vendored and not installed here, so this follows its
 * published algorithm (Traag, Waltman & van Eck, Sci. Rep. 9:5233, 2019) and the package's
 * documented defaults -- parity unpinned (statistical comparisons only):
 *   move_nodes: a queue holding every node in random order; the popped node moves to the
 *     neighbour community -- or an empty one -- of largest modularity gain when that gain
 *     is positive; its neighbours outside the new community re-enter the queue.
 *   refine: singletons; in random order a node still alone joins the neighbour refined
 *     community inside its own move-phase community of largest positive gain.
 *   aggregate by the refined partition, every aggregate node starting in the move-phase
 *     community of its members; repeat while the refinement merged anything.
 * Gains in exact int64 (w_vc*2M - k_v*Sigma_c): integer weights.  Output labels are
 * renumbered 0..k-1 by first node (leidenalg orders communities by size; the host layer
 * does that for both the oracle and the engine).  Returns the number of levels. */
typedef struct { i64 n; i64* rp; i32* col; i64* w; i64* kv; } ld_graph;

static void ld_free(ld_graph* g) { free(g->rp); free(g->col); free(g->w); free(g->kv); }

static void ld_move(const ld_graph* g, i64 M2, i32* P, i64* tot, i32* csize, u64* s, i64* nw, u8* seen,
                    i32* cands) {
    const i64 n = g->n;
    i32* q = (i32*)malloc(sizeof(i32) * (size_t)(n ? n : 1));
    u8* inq = (u8*)calloc((size_t)n + 1, 1);
    i32* empt = (i32*)malloc(sizeof(i32) * (size_t)(n ? n : 1));
    i64 ne = 0;
    for (i64 c = 0; c < n; ++c) if (csize[c] == 0) empt[ne++] = (i32)c;
    for (i64 i = 0; i < n; ++i) { q[i] = (i32)i; inq[i] = 1; }
    shuffle_i32(q, n, s);
    i64 head = 0, len = n;
    while (len > 0) {
        const i32 v = q[head];
        head = (head + 1 == n) ? 0 : head + 1;
        --len;
        inq[v] = 0;
        const i32 own = P[v];
        const i64 kv = g->kv[v];
        i64 nc = 0;
        for (i64 j = g->rp[v]; j < g->rp[v + 1]; ++j) {
            const i32 c = P[g->col[j]];
            if (!seen[c]) { seen[c] = 1; nw[c] = 0; cands[nc++] = c; }
            nw[c] += g->w[j];
        }
        const i64 wown = seen[own] ? nw[own] : 0;
        i32 best = own;
        long long bs = (long long)wown * M2 - (long long)kv * (tot[own] - kv);
        shuffle_i32(cands, nc, s);
        for (i64 k = 0; k < nc; ++k) {
            const i32 c = cands[k];
            if (c == own) continue;
            const long long sc = (long long)nw[c] * M2 - (long long)kv * tot[c];
            if (sc > bs) { bs = sc; best = c; }
        }
        for (i64 k = 0; k < nc; ++k) seen[cands[k]] = 0;
        if (csize[own] > 1 && bs < 0 && ne > 0) { best = empt[ne - 1]; bs = 0; }   /* the empty community */
        if (best == own) continue;
        if (csize[best] == 0) --ne;   /* best was the empty community on the stack top */
        tot[own] -= kv; tot[best] += kv;
        csize[own]--; csize[best]++;
        P[v] = best;
        if (csize[own] == 0) empt[ne++] = own;
        for (i64 j = g->rp[v]; j < g->rp[v + 1]; ++j) {
            const i32 u = g->col[j];
            if (P[u] != best && !inq[u]) {
                i64 tail = head + len;
                if (tail >= n) tail -= n;
                q[tail] = u; inq[u] = 1; ++len;
            }
        }
    }
    free(q); free(inq); free(empt);
}

/* one refinement pass; returns the number of refined communities */
static i64 ld_refine(const ld_graph* g, i64 M2, const i32* P, i32* R, i64* rtot, i32* rsize, u64* s, i64* nw,
                     u8* seen, i32* cands, i32* order) {
    const i64 n = g->n;
    for (i64 v = 0; v < n; ++v) { R[v] = (i32)v; rtot[v] = g->kv[v]; rsize[v] = 1; order[v] = (i32)v; }
    shuffle_i32(order, n, s);
    i64 ncom = n;
    for (i64 t = 0; t < n; ++t) {
        const i32 v = order[t];
        if (rsize[R[v]] != 1) continue;
        const i64 kv = g->kv[v];
        i64 nc = 0;
        for (i64 j = g->rp[v]; j < g->rp[v + 1]; ++j) {
            const i32 u = g->col[j];
            if (P[u] != P[v]) continue;
            const i32 c = R[u];
            if (!seen[c]) { seen[c] = 1; nw[c] = 0; cands[nc++] = c; }
            nw[c] += g->w[j];
        }
        i32 best = -1;
        long long bs = 0;
        shuffle_i32(cands, nc, s);
        for (i64 k = 0; k < nc; ++k) {
            const i32 c = cands[k];
            if (c == R[v]) continue;
            const long long sc = (long long)nw[c] * M2 - (long long)kv * rtot[c];
            if (sc > bs) { bs = sc; best = c; }
        }
        for (i64 k = 0; k < nc; ++k) seen[cands[k]] = 0;
        if (best < 0) continue;
        const i32 old = R[v];
        rtot[old] -= kv; rsize[old]--;
        rtot[best] += kv; rsize[best]++;
        R[v] = best;
        --ncom;
    }
    return ncom;
}

int orc_leiden(i64 N, const i64* rowptr, const i32* col, const i32* w, u64 seed, i32* lab) {
    u64 s = seed ^ 0x2545F4914F6CDD1Dull;
    ld_graph g;
    g.n = N;
    g.rp = (i64*)malloc(sizeof(i64) * (size_t)(N + 1));
    const i64 E = rowptr[N];
    g.col = (i32*)malloc(sizeof(i32) * (size_t)(E ? E : 1));
    g.w = (i64*)malloc(sizeof(i64) * (size_t)(E ? E : 1));
    g.kv = (i64*)calloc((size_t)(N ? N : 1), sizeof(i64));
    i64 M2 = 0;
    for (i64 v = 0; v <= N; ++v) g.rp[v] = rowptr[v];
    for (i64 v = 0; v < N; ++v)
        for (i64 j = rowptr[v]; j < rowptr[v + 1]; ++j) {
            g.col[j] = col[j]; g.w[j] = w ? w[j] : 1; g.kv[v] += g.w[j]; M2 += g.w[j];
        }
    const size_t nn = (size_t)(N ? N : 1);
    i32* P = (i32*)malloc(sizeof(i32) * nn);
    i32* R = (i32*)malloc(sizeof(i32) * nn);
    i64* tot = (i64*)malloc(sizeof(i64) * nn);
    i64* rtot = (i64*)malloc(sizeof(i64) * nn);
    i32* csize = (i32*)malloc(sizeof(i32) * nn);
    i32* rsize = (i32*)malloc(sizeof(i32) * nn);
    i64* nw = (i64*)malloc(sizeof(i64) * nn);
    u8* seen = (u8*)calloc(nn, 1);
    i32* cands = (i32*)malloc(sizeof(i32) * nn);
    i32* order = (i32*)malloc(sizeof(i32) * nn);
    i32* memb = (i32*)malloc(sizeof(i32) * nn);
    i32* nid = (i32*)malloc(sizeof(i32) * nn);
    i32* prep = (i32*)malloc(sizeof(i32) * nn);
    for (i64 v = 0; v < N; ++v) { P[v] = (i32)v; tot[v] = g.kv[v]; csize[v] = 1; memb[v] = (i32)v; }
    int levels = 0;
    while (1) {
        ++levels;
        ld_move(&g, M2, P, tot, csize, &s, nw, seen, cands);
        const i64 nR = ld_refine(&g, M2, P, R, rtot, rsize, &s, nw, seen, cands, order);
        if (nR == g.n || levels >= 64) break;
        /* aggregate by R: new ids in refined-community id order */
        i64 k = 0;
        for (i64 c = 0; c < g.n; ++c) nid[c] = rsize[c] > 0 ? (i32)k++ : -1;
        for (i64 c = 0; c < g.n; ++c) prep[c] = INT32_MAX;
        for (i64 v = 0; v < g.n; ++v) if (nid[R[v]] < prep[P[v]]) prep[P[v]] = nid[R[v]];
        ld_graph h;
        h.n = k;
        h.rp = (i64*)calloc((size_t)k + 1, sizeof(i64));
        h.kv = (i64*)calloc((size_t)(k ? k : 1), sizeof(i64));
        i32* np = (i32*)malloc(sizeof(i32) * (size_t)(k ? k : 1));
        /* members of each new node (counting sort) */
        i64* moff = (i64*)calloc((size_t)k + 1, sizeof(i64));
        i32* ml = (i32*)malloc(sizeof(i32) * (size_t)(g.n ? g.n : 1));
        for (i64 v = 0; v < g.n; ++v) moff[nid[R[v]] + 1]++;
        for (i64 x = 0; x < k; ++x) moff[x + 1] += moff[x];
        i64* cur = (i64*)malloc(sizeof(i64) * (size_t)(k ? k : 1));
        for (i64 x = 0; x < k; ++x) cur[x] = moff[x];
        for (i64 v = 0; v < g.n; ++v) ml[cur[nid[R[v]]]++] = (i32)v;
        i64 cap = g.rp[g.n] ? g.rp[g.n] : 1;
        h.col = (i32*)malloc(sizeof(i32) * (size_t)cap);
        h.w = (i64*)malloc(sizeof(i64) * (size_t)cap);
        i64 e = 0;
        for (i64 x = 0; x < k; ++x) {
            i64 nc = 0;
            for (i64 q = moff[x]; q < moff[x + 1]; ++q) {
                const i32 v = ml[q];
                h.kv[x] += g.kv[v];
                np[x] = prep[P[v]];
                for (i64 j = g.rp[v]; j < g.rp[v + 1]; ++j) {
                    const i32 y = nid[R[g.col[j]]];
                    if (y == x) continue;
                    if (!seen[y]) { seen[y] = 1; nw[y] = 0; cands[nc++] = y; }
                    nw[y] += g.w[j];
                }
            }
            /* rows sorted by column (canonical) */
            for (i64 a = 1; a < nc; ++a) {
                i32 t = cands[a]; i64 b = a - 1;
                while (b >= 0 && cands[b] > t) { cands[b + 1] = cands[b]; --b; }
                cands[b + 1] = t;
            }
            for (i64 q = 0; q < nc; ++q) { h.col[e] = cands[q]; h.w[e] = nw[cands[q]]; ++e; seen[cands[q]] = 0; }
            h.rp[x + 1] = e;
        }
        for (i64 v = 0; v < N; ++v) memb[v] = nid[R[memb[v]]];
        for (i64 x = 0; x < k; ++x) { P[x] = np[x]; tot[x] = 0; csize[x] = 0; }
        for (i64 x = 0; x < k; ++x) { tot[P[x]] += h.kv[x]; csize[P[x]]++; }
        free(np); free(moff); free(ml); free(cur);
        ld_free(&g);
        g = h;
    }
    for (i64 v = 0; v < N; ++v) lab[v] = P[memb[v]];
    renumber(N, lab, nid);
    ld_free(&g);
    free(P); free(R); free(tot); free(rtot); free(csize); free(rsize); free(nw); free(seen); free(cands);
    free(order); free(memb); free(nid); free(prep);
    return levels;
}

/* ------------------------------------------------------------------ igraph Infomap (core)
 * Restatement of the CORE of igraph_community_infomap (python-igraph 0.9.7
 * Graph.community_infomap(), trials=10), as called unweighted at fast_consensus.py:268 and
 * :390 (igraph absent: parity unpinned).  The two-level map equation for an undirected
 * graph, with node flow p_a = k_a/2M and module exit flow q_i = o_i/2M (o_i: weight of the
 * edges leaving module i),
 *   L = plogp(sum_i q_i) - 2 sum_i plogp(q_i) - sum_a plogp(p_a) + sum_i plogp(q_i + p_i),
 * is minimised by igraph's greedy core: passes over the nodes in random order, each node
 * moving to the neighbour module of the most negative delta-L (< -1e-10), passes until one
 * moves nothing (igraph: until the codelength stops improving); then the modules become the nodes of the next level
 * (aggregation), until a level merges nothing.  The best of `trials` runs (smallest L) is
 * kept.  igraph's alternating sub-module / single-node re-partitioning rounds around this
 * core are not part of this function or of the engine; orc_infomap_full (below) restates them
 * to measure the gap (0 to 0.01 % of the codelength).  log base 2 as igraph.
 * Output labels renumbered 0..k-1 by first node.  Returns the codelength (bits). */
static inline double plogp2(double p) { return p > 0.0 ? p * log(p) * 1.4426950408889634 : 0.0; }

static double im_delta(double inv, long long Q, long long oA, long long tA, long long oB, long long tB,
                       long long kv, long long sv, long long wA, long long wB) {
    const long long oA2 = oA - sv + 2 * wA, tA2 = tA - kv, oB2 = oB + sv - 2 * wB, tB2 = tB + kv;
    const long long Q2 = Q + (oA2 - oA) + (oB2 - oB);
    return (plogp2(Q2 * inv) - plogp2(Q * inv))
           - 2.0 * (plogp2(oA2 * inv) - plogp2(oA * inv) + plogp2(oB2 * inv) - plogp2(oB * inv))
           + (plogp2((oA2 + tA2) * inv) - plogp2((oA + tA) * inv) + plogp2((oB2 + tB2) * inv) - plogp2((oB + tB) * inv));
}

static double im_trial(i64 N, const i64* rowptr, const i32* col, u64* s, i32* lab) {
    ld_graph g;
    g.n = N;
    const i64 E = rowptr[N];
    g.rp = (i64*)malloc(sizeof(i64) * (size_t)(N + 1));
    g.col = (i32*)malloc(sizeof(i32) * (size_t)(E ? E : 1));
    g.w = (i64*)malloc(sizeof(i64) * (size_t)(E ? E : 1));
    g.kv = (i64*)calloc((size_t)(N ? N : 1), sizeof(i64));
    const size_t nn = (size_t)(N ? N : 1);
    i64* sv = (i64*)malloc(sizeof(i64) * nn);
    for (i64 v = 0; v <= N; ++v) g.rp[v] = rowptr[v];
    for (i64 j = 0; j < E; ++j) { g.col[j] = col[j]; g.w[j] = 1; }
    for (i64 v = 0; v < N; ++v) { g.kv[v] = rowptr[v + 1] - rowptr[v]; sv[v] = g.kv[v]; }
    const long long M2 = E;
    const double inv = M2 > 0 ? 1.0 / (double)M2 : 0.0;
    i32* P = (i32*)malloc(sizeof(i32) * nn);
    i64* tot = (i64*)malloc(sizeof(i64) * nn);
    i64* out = (i64*)malloc(sizeof(i64) * nn);
    i64* nw = (i64*)malloc(sizeof(i64) * nn);
    u8* seen = (u8*)calloc(nn, 1);
    i32* cands = (i32*)malloc(sizeof(i32) * nn);
    i32* order = (i32*)malloc(sizeof(i32) * nn);
    i32* memb = (i32*)malloc(sizeof(i32) * nn);
    i32* nid = (i32*)malloc(sizeof(i32) * nn);
    for (i64 v = 0; v < N; ++v) memb[v] = (i32)v;
    long long Q = 0;
    for (i64 v = 0; v < N; ++v) Q += sv[v];
    while (M2 > 0) {
        for (i64 v = 0; v < g.n; ++v) { P[v] = (i32)v; tot[v] = g.kv[v]; out[v] = sv[v]; order[v] = (i32)v; }
        for (int pass = 0; pass < 200; ++pass) {   /* igraph: until the codelength stops improving */
            shuffle_i32(order, g.n, s);
            i64 moved = 0;
            for (i64 t = 0; t < g.n; ++t) {
                const i32 v = order[t];
                const i32 A = P[v];
                i64 nc = 0;
                for (i64 j = g.rp[v]; j < g.rp[v + 1]; ++j) {
                    const i32 c = P[g.col[j]];
                    if (!seen[c]) { seen[c] = 1; nw[c] = 0; cands[nc++] = c; }
                    nw[c] += g.w[j];
                }
                const i64 wA = seen[A] ? nw[A] : 0;
                i32 best = -1;
                double bd = -1e-10;
                shuffle_i32(cands, nc, s);
                for (i64 k = 0; k < nc; ++k) {
                    const i32 B = cands[k];
                    if (B == A) continue;
                    const double d = im_delta(inv, Q, out[A], tot[A], out[B], tot[B], g.kv[v], sv[v], wA, nw[B]);
                    if (d < bd) { bd = d; best = B; }
                }
                if (best >= 0) {
                    const i64 wB = nw[best];
                    const long long dA = -sv[v] + 2 * wA, dB = sv[v] - 2 * wB;
                    out[A] += dA; out[best] += dB; Q += dA + dB;
                    tot[A] -= g.kv[v]; tot[best] += g.kv[v];
                    P[v] = best;
                    ++moved;
                }
                for (i64 k = 0; k < nc; ++k) seen[cands[k]] = 0;
            }
            if (!moved) break;
        }
        i64 k = 0;
        for (i64 c = 0; c < g.n; ++c) nid[c] = -1;
        for (i64 v = 0; v < g.n; ++v) nid[P[v]] = 0;
        for (i64 c = 0; c < g.n; ++c) if (nid[c] == 0) nid[c] = (i32)k++;
        if (k == g.n) break;
        /* aggregate by modules: kv' = tot, sv' = out, rows = inter-module weights */
        ld_graph h;
        h.n = k;
        h.rp = (i64*)calloc((size_t)k + 1, sizeof(i64));
        h.kv = (i64*)calloc((size_t)(k ? k : 1), sizeof(i64));
        i64* moff = (i64*)calloc((size_t)k + 1, sizeof(i64));
        i32* ml = (i32*)malloc(sizeof(i32) * (size_t)(g.n ? g.n : 1));
        for (i64 v = 0; v < g.n; ++v) moff[nid[P[v]] + 1]++;
        for (i64 x = 0; x < k; ++x) moff[x + 1] += moff[x];
        i64* cur = (i64*)malloc(sizeof(i64) * (size_t)(k ? k : 1));
        for (i64 x = 0; x < k; ++x) cur[x] = moff[x];
        for (i64 v = 0; v < g.n; ++v) ml[cur[nid[P[v]]]++] = (i32)v;
        const i64 cap = g.rp[g.n] ? g.rp[g.n] : 1;
        h.col = (i32*)malloc(sizeof(i32) * (size_t)cap);
        h.w = (i64*)malloc(sizeof(i64) * (size_t)cap);
        i64 e = 0;
        for (i64 c = 0; c < g.n; ++c) if (nid[c] >= 0) { h.kv[nid[c]] = tot[c]; sv[nid[c]] = out[c]; }
        for (i64 x = 0; x < k; ++x) {
            i64 nc = 0;
            for (i64 q = moff[x]; q < moff[x + 1]; ++q) {
                const i32 v = ml[q];
                for (i64 j = g.rp[v]; j < g.rp[v + 1]; ++j) {
                    const i32 y = nid[P[g.col[j]]];
                    if (y == x) continue;
                    if (!seen[y]) { seen[y] = 1; nw[y] = 0; cands[nc++] = y; }
                    nw[y] += g.w[j];
                }
            }
            for (i64 q = 0; q < nc; ++q) { h.col[e] = cands[q]; h.w[e] = nw[cands[q]]; ++e; seen[cands[q]] = 0; }
            h.rp[x + 1] = e;
        }
        for (i64 v = 0; v < N; ++v) memb[v] = nid[P[memb[v]]];
        free(moff); free(ml); free(cur);
        ld_free(&g);
        g = h;
    }
    /* codelength of the final modules (P over the last level) */
    double L = plogp2(Q * inv);
    for (i64 c = 0; c < g.n; ++c) L += -2.0 * plogp2(out[c] * inv) + plogp2((out[c] + tot[c]) * inv);
    for (i64 v = 0; v < N; ++v) L -= plogp2((double)(rowptr[v + 1] - rowptr[v]) * inv);
    for (i64 v = 0; v < N; ++v) lab[v] = M2 > 0 ? P[memb[v]] : (i32)v;
    renumber(N, lab, nid);
    ld_free(&g);
    free(sv); free(P); free(tot); free(out); free(nw); free(seen); free(cands); free(order); free(memb); free(nid);
    return L;
}

double orc_infomap(i64 N, const i64* rowptr, const i32* col, u64 seed, int trials, i32* lab) {
    u64 s = seed ^ 0x9FB21C651E98DF25ull;
    i32* tmp = (i32*)malloc(sizeof(i32) * (size_t)(N ? N : 1));
    double best = 1e300;
    for (int t = 0; t < (trials > 0 ? trials : 1); ++t) {
        const double L = im_trial(N, rowptr, col, &s, tmp);
        if (L < best) { best = L; memcpy(lab, tmp, sizeof(i32) * (size_t)N); }
    }
    free(tmp);
    return best;
}

/* Batch helper: n_r independent runs (replicas) in parallel over host threads.
 * algo 0 = louvain level 0, 1 = lpa, 3 = leiden, 4 = infomap (10 trials).  lab is [n_r][N]. */
void orc_cd_batch(int algo, int n_r, i64 N, const i64* rowptr, const i32* col, const i32* w,
                  u64 seed, i32* lab, int* sweeps, int nthreads) {
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#else
    (void)nthreads;
#endif
#pragma omp parallel for schedule(dynamic, 1)
    for (int r = 0; r < n_r; ++r) {
        u64 sd = seed * 0x9E3779B97F4A7C15ull + (u64)r * 0xC2B2AE3D27D4EB4Full + 1;
        int sw = algo == 0   ? orc_louvain_level0(N, rowptr, col, w, sd, lab + (i64)r * N)
                 : algo == 3 ? orc_leiden(N, rowptr, col, w, sd, lab + (i64)r * N)
                 : algo == 4 ? (int)orc_infomap(N, rowptr, col, sd, 10, lab + (i64)r * N)
                             : orc_lpa(N, rowptr, col, sd, lab + (i64)r * N, 10000);
        if (sweeps) sweeps[r] = sw;
    }
}

/* Modularity of a labelling (for statistical tests): Q = sum_c in_c/M - (tot_c/2M)^2. */
double orc_modularity(i64 N, const i64* rowptr, const i32* col, const i32* w, const i32* lab) {
    double* tot = (double*)calloc((size_t)N, sizeof(double));
    double in = 0.0, tw = 0.0;
    for (i64 i = 0; i < N; ++i)
        for (i64 j = rowptr[i]; j < rowptr[i + 1]; ++j) {
            const double ww = w ? (double)w[j] : 1.0;
            tot[lab[i]] += ww;
            tw += ww;
            if (lab[col[j]] == lab[i]) in += ww;
        }
    double q = 0.0;
    if (tw > 0) {
        q = in / tw;
        for (i64 c = 0; c < N; ++c) q -= (tot[c] / tw) * (tot[c] / tw);
    }
    free(tot);
    return q;
}

/* Symmetric CSR (neighbours ascending) from a canonical edge list. */
void orc_build_csr(i64 N, i64 m, const i32* eu, const i32* ev, const i32* w, i64* rowptr,
                   i32* col, i32* cw) {
    memset(rowptr, 0, sizeof(i64) * (size_t)(N + 1));
    for (i64 e = 0; e < m; ++e) { rowptr[eu[e] + 1]++; rowptr[ev[e] + 1]++; }
    for (i64 x = 0; x < N; ++x) rowptr[x + 1] += rowptr[x];
    i64* fill = (i64*)malloc(sizeof(i64) * (size_t)(N + 1));
    memcpy(fill, rowptr, sizeof(i64) * (size_t)N);
    /* lower neighbours first (ascending u, because eu is sorted), then upper ones */
    for (i64 e = 0; e < m; ++e) { i64 p = fill[ev[e]]++; col[p] = eu[e]; if (cw) cw[p] = w ? w[e] : 1; }
    for (i64 e = 0; e < m; ++e) { i64 p = fill[eu[e]]++; col[p] = ev[e]; if (cw) cw[p] = w ? w[e] : 1; }
    free(fill);
}

/* ==================================================================================
 * CPU twin of the engine's bucketed community detection (fastconsensus_amd/csrc/cd.hip).
 * This is NOT the reference algorithm: it restates, sequentially, the device algorithm
 * (random bucketed order, synchronous decisions inside a bucket, integer gains, hashed
 * tie-breaks) so that the HIP kernels can be checked bit-exactly on the same seed.
 * Statistical closeness to the reference's sequential algorithms is tested separately
 * against orc_louvain_level0 / orc_lpa above.
 * ================================================================================== */
static inline uint32_t tw_hash32(uint32_t x) {
    x ^= x >> 16; x *= 0x85ebca6bu; x ^= x >> 13; x *= 0xc2b2ae35u; x ^= x >> 16; return x;
}
static inline uint32_t tw_hash2(uint32_t a, uint32_t b) { return tw_hash32(a ^ tw_hash32(b + 0x9e3779b9u)); }
static inline u64 tw_mix64(u64 z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static inline uint32_t tw_stream_key(u64 seed, uint32_t rg, uint32_t iter, uint32_t sweep, uint32_t salt) {
    u64 z = tw_mix64(seed ^ (0x9E3779B97F4A7C15ull * (1 + (u64)rg)));
    z = tw_mix64(z ^ ((u64)iter << 32 | sweep) ^ ((u64)salt << 56));
    return (uint32_t)(z ^ (z >> 32));
}
typedef struct { uint32_t n, hb, mask, k0, k1, k2, k3; } tw_perm;
static tw_perm tw_make_perm(uint32_t n, uint32_t key) {
    tw_perm p;
    uint32_t bits = 1;
    while (bits < 32 && (1u << bits) < n) ++bits;
    uint32_t hb = (bits + 1) / 2;
    if (hb < 1) hb = 1;
    p.n = n; p.hb = hb; p.mask = (1u << hb) - 1u;
    p.k0 = tw_hash2(key, 0x1234567u); p.k1 = tw_hash2(key, 0x89abcdefu);
    p.k2 = tw_hash2(key, 0x2468aceu); p.k3 = tw_hash2(key, 0x13579bdu);
    return p;
}
static uint32_t tw_perm_apply(const tw_perm* p, uint32_t x) {
    do {
        uint32_t L = x >> p->hb, R = x & p->mask, t;
        t = R; R = L ^ (tw_hash32(R ^ p->k0) & p->mask); L = t;
        t = R; R = L ^ (tw_hash32(R ^ p->k1) & p->mask); L = t;
        t = R; R = L ^ (tw_hash32(R ^ p->k2) & p->mask); L = t;
        t = R; R = L ^ (tw_hash32(R ^ p->k3) & p->mask); L = t;
        x = (L << p->hb) | R;
    } while (x >= p->n);
    return x;
}
/* Vertex at sweep position p (or >= N: a padding slot).  Chunked orders visit chunks of
 * `chunk` consecutive vertices; the chunk grid is shifted by a per-(replica, sweep) offset
 * off in [0, chunk) (engine cd.hip pos_vertex), so two vertices closer than `chunk` do not
 * share a chunk -- and decide simultaneously -- in every sweep: a fixed grid kept such a pair
 * swapping communities forever (a dyad whose ends each join the other's singleton). */
static inline i64 tw_pos_vertex(const tw_perm* P, int chunk, uint32_t off, i64 N, i64 p) {
    if (!chunk) return (i64)tw_perm_apply(P, (uint32_t)p);
    const i64 w = (i64)tw_perm_apply(P, (uint32_t)(p / chunk)) * chunk + p % chunk - (i64)off;
    return (w < 0 || w >= N) ? N : w;
}
static inline uint32_t tw_chunk_off(int chunk, u64 seed, uint32_t rg, uint32_t iter, uint32_t sweep) {
    return chunk ? tw_stream_key(seed, rg, iter, sweep, 3) & (uint32_t)(chunk - 1) : 0u;
}
static inline uint32_t tw_tie(uint32_t tbk, i32 v, i32 c) { return tw_hash32(tw_hash32(tbk ^ (uint32_t)v) ^ (uint32_t)c); }
static inline int tw_better(long long s1, uint32_t h1, i32 c1, long long s2, uint32_t h2, i32 c2) {
    if (s1 != s2) return s1 > s2;
    if (h1 != h2) return h1 > h2;
    return c1 < c2;
}

/* One replica.  algo 0 = louvain local moving, 1 = lpa.  Returns sweeps executed. */
/* Bucket of list entry q (lists are concatenated per bucket, offsets loff). */
static int bucket_of_entry(const i64* loff, int k0, int k1, i64 q) {
    int k = k0;
    while (k + 1 < k1 && loff[k + 1] <= q) ++k;
    return k;
}

/* Coarsening of a filtered sweep (engine cd.hip k_list_offsets): its V listed vertices are
 * decided in rounds of g consecutive buckets, g the largest power of two <= B with V*g <= N,
 * so a round holds about as many decisions as one bucket of a full sweep (N/B); g <= gmax. */
static int tw_coarse(i64 N, i64 V, int B, int gmax) {
    int g = 1;
    while (2 * g <= B && 2 * g <= gmax && V * 2 * (i64)g <= N) g *= 2;
    return g;
}

/* shared: 1 the replica-lane engine (cd_rl.hip) -- every replica visits the vertices in the SAME
 * per-(iteration, sweep) order (its stream key uses TW_SHARED_RG in place of the replica
 * index); tie keys stay per replica.  0: the classic engine's per-replica orders.  2: the
 * hybrid (FC_OPT_CD_ENGINE=2) -- the shared order while the replica's sweep visits every vertex
 * or at least N/dense_div of them (a dense filtered sweep, run without coarse rounds), its own
 * order (and coarse rounds) once its filtered list is sparser. */
#define TW_SHARED_RG 0xffffffffu
/* LPA tie revisits under pruning (see tw_replica); settable for the semantics study */
static int tw_lpa_ties = 1;
void orc_set_lpa_ties(int on) { tw_lpa_ties = on; }
static int tw_lpa_coarsen = 0;   /* semantics study: LPA coarse rounds up to this g (0: none) */
void orc_set_lpa_coarsen(int g) { tw_lpa_coarsen = g; }
static int tw_replica(int algo, i64 N, const i64* rowptr, const i32* col, const i32* cw, const i64* kdeg, i64 M2,
                      u64 seed, uint32_t rg, uint32_t iter, int buckets, int max_sweeps, int chunk, int prune,
                      int coarsen, int lm, int shared, int dense_div, i32* lab) {
    const int louv = algo == 0;
    i64* tot = (i64*)malloc(sizeof(i64) * (size_t)N);
    i32* csz = (i32*)malloc(sizeof(i32) * (size_t)N);
    i64* acc = (i64*)calloc((size_t)N, sizeof(i64));
    u8* seen = (u8*)calloc((size_t)N, 1);
    i32* keys = (i32*)malloc(sizeof(i32) * (size_t)(N + 1));
    /* visit order: vertices, or chunks of `chunk` consecutive vertices, in random order */
    const i64 NC = chunk ? (N + 2 * (i64)chunk - 2) / chunk : N;   /* room for the chunk-grid shift */
    const i64 PN = chunk ? NC * chunk : N;
    const int B = (int)(buckets < NC ? buckets : NC);
    const i64 S = chunk ? ((NC + B - 1) / B) * chunk : (N + B - 1) / B;
    i32* dec = (i32*)malloc(sizeof(i32) * (size_t)(PN + 1));
    u8* aff = (u8*)calloc((size_t)N, 1);
    u8* mvf = lm ? (u8*)calloc((size_t)N, 1) : NULL;   /* movers of a tracked sweep (lm) */
    i64* lists = (i64*)malloc(sizeof(i64) * (size_t)(PN + 1));   /* per-bucket visit lists */
    i64* loff = (i64*)malloc(sizeof(i64) * (size_t)(B + 1));
    for (i64 v = 0; v < N; ++v) { lab[v] = (i32)v; tot[v] = kdeg[v]; csz[v] = 1; }
    int active = M2 > 0, sweep = 0;
    int track_now = 0, prune_now = 0;   /* adaptive pruning state (engine: k_sweep_end) */
    for (; sweep < max_sweeps && active; ++sweep) {
        const int filtered = prune && sweep > 0 && prune_now;
        /* hybrid: a filtered sweep that still visits >= N/dense_div vertices ("dense") keeps the
         * shared order, in single-bucket rounds (no coarsening); dense_div = 0: never */
        int dense = 0;
        if (shared == 2 && filtered && dense_div > 0) {
            i64 V = 0;
            for (i64 v = 0; v < N; ++v) V += aff[v] != 0;
            dense = (i64)dense_div * V >= N;
        }
        /* experimental (semantics study): shared == 3 -- sweep 0 in the replica's own order, then
         * as 2; shared >= 0x100 -- as 2 with replicas grouped by (shared & 0xff): the group's
         * shared order (key TW_SHARED_RG - group) */
        uint32_t prg;
        if (shared >= 0x100) {
            const uint32_t gs = (uint32_t)(shared & 0xff);
            prg = (!filtered || dense) ? TW_SHARED_RG - rg / gs : rg;
        } else if (shared == 3) {
            prg = (sweep > 0 && (!filtered || dense)) ? TW_SHARED_RG : rg;
        } else {
            prg = (shared == 1 || (shared == 2 && (!filtered || dense))) ? TW_SHARED_RG : rg;
        }
        const tw_perm P = tw_make_perm((uint32_t)NC, tw_stream_key(seed, prg, iter, (uint32_t)sweep, 1));
        const uint32_t tbk = tw_stream_key(seed, rg, iter, (uint32_t)sweep, 2);
        const uint32_t off = tw_chunk_off(chunk, seed, prg, iter, (uint32_t)sweep);
        unsigned long long dq = 0, moves = 0, unstable = 0;
        const int listed = prune && sweep > 0;
        if (listed) {   /* all lists are built (and flags cleared) at the sweep start;
                           unfiltered (every position) until moves have been tracked */
            i64 n = 0;
            for (int k = 0; k < B; ++k) {
                loff[k] = n;
                i64 blen = PN - (i64)k * S;
                if (blen > S) blen = S;
                for (i64 i = 0; i < blen; ++i) {
                    const i64 vv = tw_pos_vertex(&P, chunk, off, N, (i64)k * S + i);
                    if (vv < N) {
                        if (!prune_now || aff[vv]) lists[n++] = i;
                        aff[vv] = 0;
                    }
                }
            }
            loff[B] = n;
        }
        /* rounds: one bucket each, or g consecutive buckets of a filtered sweep */
        /* Louvain only: LPA's tied vertices redraw at every visit, and rounds of several
         * buckets let adjacent tied vertices flip together sweep after sweep (a replica on
         * LFR-100k at average degree 8 never stopped) */
        const int g = ((louv || tw_lpa_coarsen) && listed && prune_now && coarsen && !dense)
                          ? tw_coarse(N, loff[B], B, louv ? coarsen : (coarsen < tw_lpa_coarsen ? coarsen : tw_lpa_coarsen)) : 1;
        for (int k = 0; k < B; k += g) {
            const int k1 = k + g < B ? k + g : B;
            i64 blen = PN - (i64)k * S;
            if (blen > S) blen = S;
            if (blen <= 0) continue;
            const i64 ne = listed ? loff[k1] - loff[k] : blen;   /* g > 1 only when listed */
            for (i64 e = 0; e < ne; ++e) {
                const i64 i = listed ? lists[loff[k] + e] : e;
                dec[e] = -1;
                /* position: listed entries of round [k, k1) carry their own bucket */
                const int kb = listed ? bucket_of_entry(loff, k, k1, loff[k] + e) : k;
                const i64 vv = tw_pos_vertex(&P, chunk, off, N, (i64)kb * S + i);
                if (vv >= N) continue;
                const i32 v = (i32)vv;
                const i64 rb = rowptr[v], re = rowptr[v + 1];
                if (re == rb) continue;
                i64 nk = 0;
                for (i64 j = rb; j < re; ++j) {
                    const i32 c = lab[col[j]];
                    if (!seen[c]) { seen[c] = 1; acc[c] = 0; keys[nk++] = c; }
                    acc[c] += louv ? cw[j] : 1;
                }
                const i32 own = lab[v];
                const i64 kown = seen[own] ? acc[own] : 0;
                const i64 kv = kdeg[v];
                long long best_s = 0; uint32_t best_h = 0; i32 best_c = 0x7fffffff; int have = 0;
                for (i64 q = 0; q < nk; ++q) {
                    const i32 c = keys[q];
                    long long sc;
                    if (louv) { if (c == own) continue; sc = (long long)acc[c] * M2 - kv * tot[c]; }
                    else sc = acc[c];
                    const uint32_t h = tw_tie(tbk, v, c);
                    if (!have || tw_better(sc, h, c, best_s, best_h, best_c)) { best_s = sc; best_h = h; best_c = c; have = 1; }
                }
                /* LPA: a vertex with several dominant labels redraws among them at every visit
                 * (igraph visits every node each sweep), so pruning must keep visiting it: it
                 * flags itself for the next sweep.  A vertex with one dominant label and an
                 * unchanged neighbourhood would redraw the same label -- skipping it is exact. */
                int ntie = 0;
                if (!louv && have && track_now && tw_lpa_ties)
                    for (i64 q = 0; q < nk; ++q) ntie += acc[keys[q]] == best_s;
                for (i64 q = 0; q < nk; ++q) seen[keys[q]] = 0;
                if (!have) continue;
                if (ntie >= 2) aff[v] = 1;
                if (louv) {
                    const long long G = best_s - kown * M2 + kv * (tot[own] - kv);
                    if (G <= 0) continue;
                    const double d = (double)G * 2.0 / ((double)M2 * (double)M2);
                    dq += (unsigned long long)llrint(d * 1099511627776.0);
                    dec[e] = best_c;
                } else {
                    unstable += (kown != best_s);
                    if (best_c != own) dec[e] = best_c;
                }
            }
            for (i64 e = 0; e < ne; ++e) {
                if (dec[e] < 0) continue;
                const i64 i = listed ? lists[loff[k] + e] : e;
                const int kb = listed ? bucket_of_entry(loff, k, k1, loff[k] + e) : k;
                const i32 v = (i32)tw_pos_vertex(&P, chunk, off, N, (i64)kb * S + i);
                const i32 old = lab[v], nw = dec[e];
                lab[v] = nw;
                if (louv) { tot[old] -= kdeg[v]; tot[nw] += kdeg[v]; csz[old]--; csz[nw]++; }
                if (track_now && lm) mvf[v] = 1;
                else if (track_now)
                    for (i64 j = rowptr[v]; j < rowptr[v + 1]; ++j) aff[col[j]] = 1;
                ++moves;
            }
        }
        /* lm (engine k_mark_lm): at the end of a tracked sweep each mover marks the neighbours
         * whose label differs from its own, as the sweep left them */
        if (track_now && lm)
            for (i64 v = 0; v < N; ++v) {
                if (!mvf[v]) continue;
                mvf[v] = 0;
                for (i64 j = rowptr[v]; j < rowptr[v + 1]; ++j)
                    if (lab[col[j]] != lab[v]) aff[col[j]] = 1;
            }
        if (prune) {
            prune_now = track_now;
            if (lm || moves * 4 < (unsigned long long)N) track_now = 1;
        }
        if (louv) { if (moves == 0 || ((double)dq / 1099511627776.0) < 1e-7) active = 0; }
        else if (unstable == 0) active = 0;
    }
    free(tot); free(csz); free(acc); free(seen); free(keys); free(dec); free(aff); free(mvf); free(lists); free(loff);
    return sweep;
}

/* The engine's internal vertex numbering (graph.hip k_sigma, FC_OPT_RELABEL=1): node i ->
 * perm_apply(make_perm(n, (uint32_t)mix64(seed ^ 0x51A7E5ED)), i).  With it the CPU model
 * (tests/cpu_engine.py, sigma=...) reproduces a device run of the same seed exactly. */
void orc_device_sigma(i64 n, u64 seed, i32* sigma) {
    const tw_perm P = tw_make_perm((uint32_t)n, (uint32_t)tw_mix64(seed ^ 0x51A7E5EDull));
    for (i64 i = 0; i < n; ++i) sigma[i] = (i32)tw_perm_apply(&P, (uint32_t)i);
}

/* Replicas [rbase, rbase+n_r) of the engine's bucketed CD on a symmetric CSR.
 * lab: [n_r][N] raw community ids (not renumbered), sweeps: [n_r]. */
void orc_engine_cd(int algo, i64 N, const i64* rowptr, const i32* col, const i32* cw, int n_r, int rbase,
                   int iteration, u64 seed, int buckets, int max_sweeps, int chunk, int prune, int coarsen,
                   int prune_mark, int shared, int dense_div, i32* lab, int* sweeps) {
    i64* kdeg = (i64*)malloc(sizeof(i64) * (size_t)(N ? N : 1));
    i64 M2 = 0;
    i32 max_w = 0;
    for (i64 v = 0; v < N; ++v) {
        i64 s = 0;
        for (i64 j = rowptr[v]; j < rowptr[v + 1]; ++j) { s += cw[j]; if (cw[j] > max_w) max_w = cw[j]; }
        kdeg[v] = s;
        M2 += s;
    }
    /* engine cd_run: Leiden-style marks on consensus graphs (weights > 1; LPA too) */
    const int lm = (max_w > 1 || prune_mark == 2) && prune && prune_mark >= 1;
    (void)algo;
#pragma omp parallel for schedule(dynamic, 1)
    for (int r = 0; r < n_r; ++r) {
        int sw = tw_replica(algo, N, rowptr, col, cw, kdeg, M2, seed, (uint32_t)(rbase + r), (uint32_t)iteration,
                            buckets, max_sweeps, chunk, prune, coarsen, lm, shared, dense_div, lab + (i64)r * N);
        if (sweeps) sweeps[r] = sw;
    }
    free(kdeg);
}

/* CPU twin of the engine's counter-based closure sampler (consensus.hip k_closure_sample):
 * attempt t draws Philox4x32-10(counter = {t_lo, t_hi, iteration, 0x5eed}); node
 * x = uniform over N; if x has >= 2 neighbours in the post-threshold CSR (sorted rows),
 * two distinct positions i1 != i2 uniformly.  Writes the pair (a, b) or (-1, -1).
 * Feeding these pairs to orc_closure_pairs reproduces the device's candidates. */
typedef struct { uint32_t x, y, z, w; } tw_u4;
static tw_u4 tw_philox(tw_u4 c, uint32_t k0, uint32_t k1) {
    for (int i = 0; i < 10; ++i) {
        u64 p0 = (u64)0xD2511F53u * c.x, p1 = (u64)0xCD9E8D57u * c.z;
        tw_u4 n;
        n.x = (uint32_t)(p1 >> 32) ^ c.y ^ k0;
        n.y = (uint32_t)p1;
        n.z = (uint32_t)(p0 >> 32) ^ c.w ^ k1;
        n.w = (uint32_t)p0;
        c = n;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
    return c;
}
static inline uint32_t tw_below(uint32_t r, uint32_t n) { return (uint32_t)(((u64)r * n) >> 32); }
static int cmp_u64(const void* a, const void* b) {
    const u64 x = *(const u64*)a, y = *(const u64*)b;
    return x < y ? -1 : x > y;
}
static int tw_has_edge(const i64* rowptr, const i32* col, i32 a, i32 b) {
    i64 lo = rowptr[a], hi = rowptr[a + 1];
    while (lo < hi) {
        const i64 mid = (lo + hi) >> 1;
        if (col[mid] < b) lo = mid + 1;
        else hi = mid;
    }
    return lo < rowptr[a + 1] && col[lo] == b;
}
/* The engine's closure sampler (consensus.hip closure_sample), restated.  The reference
 * draws its L = m attempts SEQUENTIALLY from the growing nextgraph (fast_consensus.py:175-190,
 * :292-304): a closure edge is a neighbour for every later attempt.  The engine runs the
 * attempts in `rounds` consecutive blocks; a block draws in parallel from the post-threshold
 * graph plus every closure edge the earlier blocks found (the "C" graph, sorted rows).
 * Attempt t draws Philox4x32-10(counter = {t_lo, t_hi, iteration, 0x5eed}): node x uniform
 * over N; if x has d >= 2 neighbours (kept row ++ C row, both ascending), two distinct
 * positions uniformly.  pairs[t] = (a, b), or (-1, -1).  orc_closure_pairs on these pairs
 * (has_edge in the kept graph, first occurrence of each pair) gives the engine's candidates:
 * a pair that repeats an earlier block's candidate is a duplicate there. */
void orc_closure_sample(i64 N, const i64* krowptr, const i32* kcol, i64 attempts, u64 seed, int iteration,
                        int rounds, i32* pairs) {
    const u64 s = tw_mix64(seed ^ 0xC105u);
    const uint32_t k0 = (uint32_t)s, k1 = (uint32_t)(s >> 32);
    if (rounds < 1) rounds = 1;
    if (attempts > 0 && rounds > attempts) rounds = (int)attempts;
    i64* crow = (i64*)calloc((size_t)N + 1, sizeof(i64));   /* C graph: empty */
    i32* ccol = (i32*)malloc(sizeof(i32));
    u64* cand = (u64*)malloc(sizeof(u64) * (size_t)(attempts > 0 ? attempts : 1));   /* all C edges (u << 32 | v) */
    u64* rk = (u64*)malloc(sizeof(u64) * (size_t)(attempts > 0 ? attempts : 1));
    i64 nc = 0;
    for (int r = 0; r < rounds; ++r) {
        const i64 t0 = attempts * r / rounds, t1 = attempts * (r + 1) / rounds;
        i64 nr = 0;
        for (i64 t = t0; t < t1; ++t) {
            tw_u4 ctr = {(uint32_t)t, (uint32_t)((u64)t >> 32), (uint32_t)iteration, 0x5eedu};
            const tw_u4 q = tw_philox(ctr, k0, k1);
            const i32 x = (i32)tw_below(q.x, (uint32_t)N);
            const i64 kb = krowptr[x], dk = krowptr[x + 1] - kb;
            const i64 cb = crow[x], d = dk + (crow[x + 1] - cb);
            pairs[2 * t] = pairs[2 * t + 1] = -1;
            if (d < 2) continue;
            const uint32_t i1 = tw_below(q.y, (uint32_t)d);
            uint32_t i2 = tw_below(q.z, (uint32_t)(d - 1));
            if (i2 >= i1) ++i2;
            const i32 a = (i64)i1 < dk ? kcol[kb + i1] : ccol[cb + i1 - dk];
            const i32 b = (i64)i2 < dk ? kcol[kb + i2] : ccol[cb + i2 - dk];
            pairs[2 * t] = a;
            pairs[2 * t + 1] = b;
            const i32 u = a < b ? a : b, v = a < b ? b : a;
            if (!tw_has_edge(krowptr, kcol, u, v) && !tw_has_edge(crow, ccol, u, v))
                rk[nr++] = ((u64)(uint32_t)u << 32) | (uint32_t)v;
        }
        if (r + 1 == rounds) break;
        qsort(rk, (size_t)nr, sizeof(u64), cmp_u64);
        for (i64 i = 0; i < nr; ++i)
            if (i == 0 || rk[i] != rk[i - 1]) cand[nc++] = rk[i];
        /* rebuild C as a symmetric CSR with ascending rows */
        u64* dk2 = (u64*)malloc(sizeof(u64) * (size_t)(2 * nc + 1));
        for (i64 i = 0; i < nc; ++i) {
            const u64 u = cand[i] >> 32, v = cand[i] & 0xffffffffull;
            dk2[2 * i] = (u << 32) | v;
            dk2[2 * i + 1] = (v << 32) | u;
        }
        qsort(dk2, (size_t)(2 * nc), sizeof(u64), cmp_u64);
        free(ccol);
        ccol = (i32*)malloc(sizeof(i32) * (size_t)(2 * nc + 1));
        memset(crow, 0, sizeof(i64) * ((size_t)N + 1));
        for (i64 i = 0; i < 2 * nc; ++i) {
            crow[(dk2[i] >> 32) + 1]++;
            ccol[i] = (i32)(dk2[i] & 0xffffffffull);
        }
        for (i64 x = 0; x < N; ++x) crow[x + 1] += crow[x];
        free(dk2);
    }
    free(crow); free(ccol); free(cand); free(rk);
}

/* ------------------------------------------------------------------ sequential closure
 * The reference's closure loop itself (fast_consensus.py:175-184, :292-300), one attempt after
 * the other on a GROWING nextgraph: node x uniform over all N (np.random.choice, :177); if
 * it has >= 2 neighbours, two distinct ones uniformly (random.sample(set(...), 2), :181); if
 * a-b is absent (:183) it is added and is a neighbour / an edge for every later attempt.  The
 * RNG is the oracle's own (the reference's numpy/random streams cannot be reproduced), so
 * this is the reference's sampling DISTRIBUTION.  Used only as the reference-semantics
 * baseline of the engine's blocked sampler (tests/golden/make_refsem.py c3).
 * pairs_out: the added pairs in attempt order; returns their count (<= attempts). */
typedef struct { i32* a; i32 n, cap; } seq_row;
static void seq_push(seq_row* r, i32 x) {
    if (r->n == r->cap) { r->cap = r->cap ? 2 * r->cap : 4; r->a = (i32*)realloc(r->a, sizeof(i32) * (size_t)r->cap); }
    r->a[r->n++] = x;
}
static inline u64 seq_key(i32 a, i32 b) {
    const u64 u = (u64)(uint32_t)(a < b ? a : b), v = (u64)(uint32_t)(a < b ? b : a);
    return (u << 32) | v;
}
static int seq_insert(u64* tab, u64 mask, u64 k) {   /* 1 when newly inserted */
    u64 h = tw_mix64(k) & mask;
    while (tab[h] != ~0ull) {
        if (tab[h] == k) return 0;
        h = (h + 1) & mask;
    }
    tab[h] = k;
    return 1;
}
i64 orc_closure_sequential(i64 N, i64 m, const i32* eu, const i32* ev, i64 attempts, u64 seed, i32* pairs_out) {
    seq_row* rows = (seq_row*)calloc((size_t)(N > 0 ? N : 1), sizeof(seq_row));
    u64 tsize = 1024;
    while (tsize < 2 * (u64)(m + attempts + 1)) tsize <<= 1;
    u64* tab = (u64*)malloc(sizeof(u64) * tsize);
    memset(tab, 0xff, sizeof(u64) * tsize);
    for (i64 i = 0; i < m; ++i) {
        seq_push(&rows[eu[i]], ev[i]);
        seq_push(&rows[ev[i]], eu[i]);
        seq_insert(tab, tsize - 1, seq_key(eu[i], ev[i]));
    }
    u64 s = seed ^ 0x5E9C105Eull;
    i64 k = 0;
    for (i64 t = 0; t < attempts && N > 0; ++t) {
        const i32 x = (i32)rng_below(&s, (u64)N);
        const i32 d = rows[x].n;
        if (d < 2) continue;
        const i32 i1 = (i32)rng_below(&s, (u64)d);
        i32 i2 = (i32)rng_below(&s, (u64)(d - 1));
        if (i2 >= i1) ++i2;
        const i32 a = rows[x].a[i1], b = rows[x].a[i2];
        if (!seq_insert(tab, tsize - 1, seq_key(a, b))) continue;
        seq_push(&rows[a], b);
        seq_push(&rows[b], a);
        pairs_out[2 * k] = a;
        pairs_out[2 * k + 1] = b;
        ++k;
    }
    for (i64 x = 0; x < N; ++x) free(rows[x].a);
    free(rows); free(tab);
    return k;
}

/* ------------------------------------------------------------------ Infomap outer loop
 * igraph's infomap_partition() around the greedy core (restated from the published igraph
 * 0.9 infomap.cc, itself a port of Rosvall & Bergstrom's code; igraph absent: parity
 * unpinned).  The engine (leiden.hip MODE_INFO) and orc_infomap run the CORE only; this
 * fuller restatement exists to MEASURE what the re-partition rounds change
 * (tests/test_infomap.py::test_core_vs_repartition_rounds_gap):
 *   iteration 0: the core from singletons (passes + aggregation while the codelength improves);
 *   odd iterations: single-node movements -- the core again on the original nodes, starting
 *     from the current modules;
 *   even iterations >= 2: sub-module movements -- every module of > 1 node is partitioned by
 *     a recursive infomap_partition on its induced subgraph (a standalone graph: flows from
 *     the subgraph's degrees), the original nodes are grouped into those sub-modules, and the
 *     core runs on the sub-modules starting from their modules;
 *   repeat while an iteration lowers the codelength by > 1e-10.
 * The two-level map equation, flows and the greedy core are orc_infomap's. */
typedef struct {
    i64 n;
    i64* rp; i32* col; i64* w;      /* symmetric weighted CSR (no self entries) */
    i64* kv;                        /* node flow weight (weighted degree at the base level) */
    i64* sv;                        /* node exit weight (== kv at the base level) */
} im_graph;

static void im_free(im_graph* g) { free(g->rp); free(g->col); free(g->w); free(g->kv); free(g->sv); }

/* codelength (bits) of partition lab over g, with base-node flows kv0 (the original nodes
 * the codelength's node term counts) */
static double im_codelength(const im_graph* g, const i32* lab, double inv, double node_term) {
    const i64 n = g->n;
    i64* tot = (i64*)calloc((size_t)(n ? n : 1), sizeof(i64));
    i64* out = (i64*)calloc((size_t)(n ? n : 1), sizeof(i64));
    for (i64 v = 0; v < n; ++v) {
        tot[lab[v]] += g->kv[v];
        out[lab[v]] += g->sv[v];
        for (i64 j = g->rp[v]; j < g->rp[v + 1]; ++j)
            if (lab[g->col[j]] == lab[v]) out[lab[v]] -= g->w[j];
    }
    long long Q = 0;
    for (i64 c = 0; c < n; ++c) Q += out[c];
    double L = plogp2(Q * inv) - node_term;
    for (i64 c = 0; c < n; ++c)
        if (tot[c] || out[c]) L += -2.0 * plogp2(out[c] * inv) + plogp2((out[c] + tot[c]) * inv);
    free(tot); free(out);
    return L;
}

/* aggregate g by lab (ids 0..k-1): kv, sv summed / exit weights, inter-module rows */
static im_graph im_aggregate(const im_graph* g, const i32* lab, i64 k) {
    im_graph h;
    h.n = k;
    h.rp = (i64*)calloc((size_t)k + 1, sizeof(i64));
    h.kv = (i64*)calloc((size_t)(k ? k : 1), sizeof(i64));
    h.sv = (i64*)calloc((size_t)(k ? k : 1), sizeof(i64));
    i64* moff = (i64*)calloc((size_t)k + 1, sizeof(i64));
    i32* ml = (i32*)malloc(sizeof(i32) * (size_t)(g->n ? g->n : 1));
    for (i64 v = 0; v < g->n; ++v) moff[lab[v] + 1]++;
    for (i64 x = 0; x < k; ++x) moff[x + 1] += moff[x];
    i64* cur = (i64*)malloc(sizeof(i64) * (size_t)(k ? k : 1));
    for (i64 x = 0; x < k; ++x) cur[x] = moff[x];
    for (i64 v = 0; v < g->n; ++v) ml[cur[lab[v]]++] = (i32)v;
    const i64 cap = g->rp[g->n] ? g->rp[g->n] : 1;
    h.col = (i32*)malloc(sizeof(i32) * (size_t)cap);
    h.w = (i64*)malloc(sizeof(i64) * (size_t)cap);
    i64* nw = (i64*)calloc((size_t)(k ? k : 1), sizeof(i64));
    u8* seen = (u8*)calloc((size_t)(k ? k : 1), 1);
    i32* cands = (i32*)malloc(sizeof(i32) * (size_t)(k ? k : 1));
    i64 e = 0;
    for (i64 x = 0; x < k; ++x) {
        i64 nc = 0;
        for (i64 q = moff[x]; q < moff[x + 1]; ++q) {
            const i32 v = ml[q];
            h.kv[x] += g->kv[v];
            h.sv[x] += g->sv[v];
            for (i64 j = g->rp[v]; j < g->rp[v + 1]; ++j) {
                const i32 y = lab[g->col[j]];
                if (y == x) { h.sv[x] -= g->w[j]; continue; }
                if (!seen[y]) { seen[y] = 1; nw[y] = 0; cands[nc++] = y; }
                nw[y] += g->w[j];
            }
        }
        for (i64 q = 0; q < nc; ++q) { h.col[e] = cands[q]; h.w[e] = nw[cands[q]]; ++e; seen[cands[q]] = 0; }
        h.rp[x + 1] = e;
    }
    free(moff); free(ml); free(cur); free(nw); free(seen); free(cands);
    return h;
}

/* the greedy core (orc_infomap's im_trial) on g from partition init (NULL: singletons):
 * passes until one moves nothing, aggregation, repeat while a level merges; lab_out = module
 * of every node of g, renumbered 0..k-1 */
static void im_core(const im_graph* g0, const i32* init, double inv, u64* s, i32* lab_out) {
    const i64 N = g0->n;
    const size_t nn = (size_t)(N ? N : 1);
    im_graph g;
    g.n = N;
    g.rp = (i64*)malloc(sizeof(i64) * (size_t)(N + 1));
    const i64 E = g0->rp[N];
    g.col = (i32*)malloc(sizeof(i32) * (size_t)(E ? E : 1));
    g.w = (i64*)malloc(sizeof(i64) * (size_t)(E ? E : 1));
    g.kv = (i64*)malloc(sizeof(i64) * nn);
    g.sv = (i64*)malloc(sizeof(i64) * nn);
    memcpy(g.rp, g0->rp, sizeof(i64) * (size_t)(N + 1));
    if (E) { memcpy(g.col, g0->col, sizeof(i32) * (size_t)E); memcpy(g.w, g0->w, sizeof(i64) * (size_t)E); }
    memcpy(g.kv, g0->kv, sizeof(i64) * nn);
    memcpy(g.sv, g0->sv, sizeof(i64) * nn);
    i32* memb = (i32*)malloc(sizeof(i32) * nn);
    i32* P = (i32*)malloc(sizeof(i32) * nn);
    i64* tot = (i64*)malloc(sizeof(i64) * nn);
    i64* out = (i64*)malloc(sizeof(i64) * nn);
    i64* nw = (i64*)malloc(sizeof(i64) * nn);
    u8* seen = (u8*)calloc(nn, 1);
    i32* cands = (i32*)malloc(sizeof(i32) * nn);
    i32* order = (i32*)malloc(sizeof(i32) * nn);
    i32* nid = (i32*)malloc(sizeof(i32) * nn);
    for (i64 v = 0; v < N; ++v) memb[v] = (i32)v;
    int first = 1;
    while (1) {
        for (i64 v = 0; v < g.n; ++v) { P[v] = (first && init) ? init[v] : (i32)v; order[v] = (i32)v; tot[v] = 0; out[v] = 0; }
        for (i64 v = 0; v < g.n; ++v) {
            tot[P[v]] += g.kv[v];
            out[P[v]] += g.sv[v];
            for (i64 j = g.rp[v]; j < g.rp[v + 1]; ++j)
                if (P[g.col[j]] == P[v]) out[P[v]] -= g.w[j];
        }
        long long Q = 0;
        for (i64 c = 0; c < g.n; ++c) Q += out[c];
        for (int pass = 0; pass < 200; ++pass) {
            shuffle_i32(order, g.n, s);
            i64 moved = 0;
            for (i64 t = 0; t < g.n; ++t) {
                const i32 v = order[t];
                const i32 A = P[v];
                i64 nc = 0;
                for (i64 j = g.rp[v]; j < g.rp[v + 1]; ++j) {
                    const i32 c = P[g.col[j]];
                    if (!seen[c]) { seen[c] = 1; nw[c] = 0; cands[nc++] = c; }
                    nw[c] += g.w[j];
                }
                const i64 wA = seen[A] ? nw[A] : 0;
                i32 best = -1;
                double bd = -1e-10;
                shuffle_i32(cands, nc, s);
                for (i64 k = 0; k < nc; ++k) {
                    const i32 B = cands[k];
                    if (B == A) continue;
                    const double d = im_delta(inv, Q, out[A], tot[A], out[B], tot[B], g.kv[v], g.sv[v], wA, nw[B]);
                    if (d < bd) { bd = d; best = B; }
                }
                if (best >= 0) {
                    const i64 wB = nw[best];
                    const long long dA = -g.sv[v] + 2 * wA, dB = g.sv[v] - 2 * wB;
                    out[A] += dA; out[best] += dB; Q += dA + dB;
                    tot[A] -= g.kv[v]; tot[best] += g.kv[v];
                    P[v] = best;
                    ++moved;
                }
                for (i64 k = 0; k < nc; ++k) seen[cands[k]] = 0;
            }
            if (!moved) break;
        }
        i64 k = 0;
        for (i64 c = 0; c < g.n; ++c) nid[c] = -1;
        for (i64 v = 0; v < g.n; ++v) nid[P[v]] = 0;
        for (i64 c = 0; c < g.n; ++c) if (nid[c] == 0) nid[c] = (i32)k++;
        for (i64 v = 0; v < g.n; ++v) P[v] = nid[P[v]];
        for (i64 v = 0; v < N; ++v) memb[v] = P[memb[v]];
        if (k == g.n && !(first && init)) break;
        first = 0;
        if (k == g.n) break;
        im_graph h = im_aggregate(&g, P, k);
        im_free(&g);
        g = h;
    }
    for (i64 v = 0; v < N; ++v) lab_out[v] = memb[v];
    renumber(N, lab_out, nid);
    im_free(&g);
    free(memb); free(P); free(tot); free(out); free(nw); free(seen); free(cands); free(order); free(nid);
}

static double im_node_term(const im_graph* g, double inv) {
    double t = 0.0;
    for (i64 v = 0; v < g->n; ++v) t += plogp2(g->kv[v] * inv);
    return t;
}

/* infomap_partition(g, rcall): lab = the outer loop's final partition; returns its codelength */
static double im_partition(const im_graph* g, u64* s, i32* lab, int depth) {
    const i64 N = g->n;
    long long M2 = 0;
    for (i64 v = 0; v < N; ++v) M2 += g->kv[v];
    for (i64 v = 0; v < N; ++v) lab[v] = (i32)v;
    if (M2 <= 0 || N <= 1) return 0.0;
    const double inv = 1.0 / (double)M2, nt = im_node_term(g, inv);
    double L = im_codelength(g, lab, inv, nt);       /* singletons (calibrate() after initiate()) */
    i32* nl = (i32*)malloc(sizeof(i32) * (size_t)N);
    for (int iteration = 0;; ++iteration) {
        const double outer_old = L;
        if (iteration == 0) {
            im_core(g, NULL, inv, s, nl);
        } else if (iteration % 2 == 1 || depth > 30) {
            im_core(g, lab, inv, s, nl);              /* single-node movements from the modules */
        } else {
            /* sub-module movements: partition every module's induced subgraph recursively */
            i64 k = 0;
            for (i64 v = 0; v < N; ++v) if (lab[v] + 1 > k) k = lab[v] + 1;
            i64* moff = (i64*)calloc((size_t)k + 1, sizeof(i64));
            i32* ml = (i32*)malloc(sizeof(i32) * (size_t)N);
            i32* loc = (i32*)malloc(sizeof(i32) * (size_t)N);
            for (i64 v = 0; v < N; ++v) moff[lab[v] + 1]++;
            for (i64 x = 0; x < k; ++x) moff[x + 1] += moff[x];
            i64* cur = (i64*)malloc(sizeof(i64) * (size_t)(k ? k : 1));
            for (i64 x = 0; x < k; ++x) cur[x] = moff[x];
            for (i64 v = 0; v < N; ++v) { loc[v] = (i32)(cur[lab[v]] - moff[lab[v]]); ml[cur[lab[v]]++] = (i32)v; }
            i32* sub = (i32*)malloc(sizeof(i32) * (size_t)N);   /* node -> sub-module (global id) */
            i32* smod = (i32*)malloc(sizeof(i32) * (size_t)N);  /* sub-module -> its module */
            i32 next = 0;
            for (i64 x = 0; x < k; ++x) {
                const i64 sn = moff[x + 1] - moff[x];
                if (sn <= 1) {
                    for (i64 q = moff[x]; q < moff[x + 1]; ++q) { sub[ml[q]] = next; smod[next] = (i32)x; ++next; }
                    continue;
                }
                im_graph sg;                           /* induced subgraph, standalone flows */
                sg.n = sn;
                sg.rp = (i64*)calloc((size_t)sn + 1, sizeof(i64));
                i64 e = 0;
                for (i64 q = moff[x]; q < moff[x + 1]; ++q)
                    for (i64 j = g->rp[ml[q]]; j < g->rp[ml[q] + 1]; ++j) e += lab[g->col[j]] == x;
                sg.col = (i32*)malloc(sizeof(i32) * (size_t)(e ? e : 1));
                sg.w = (i64*)malloc(sizeof(i64) * (size_t)(e ? e : 1));
                sg.kv = (i64*)calloc((size_t)sn, sizeof(i64));
                sg.sv = (i64*)calloc((size_t)sn, sizeof(i64));
                e = 0;
                for (i64 q = moff[x]; q < moff[x + 1]; ++q) {
                    const i32 v = ml[q];
                    for (i64 j = g->rp[v]; j < g->rp[v + 1]; ++j)
                        if (lab[g->col[j]] == x) { sg.col[e] = loc[g->col[j]]; sg.w[e] = g->w[j]; sg.kv[q - moff[x]] += g->w[j]; ++e; }
                    sg.rp[q - moff[x] + 1] = e;
                    sg.sv[q - moff[x]] = sg.kv[q - moff[x]];
                }
                i32* sl = (i32*)malloc(sizeof(i32) * (size_t)sn);
                im_partition(&sg, s, sl, depth + 1);
                i32 sk = 0;
                for (i64 q = 0; q < sn; ++q) if (sl[q] + 1 > sk) sk = sl[q] + 1;
                for (i64 q = moff[x]; q < moff[x + 1]; ++q) sub[ml[q]] = next + sl[q - moff[x]];
                for (i32 t = 0; t < sk; ++t) smod[next + t] = (i32)x;
                next += sk;
                free(sl);
                im_free(&sg);
            }
            im_graph h = im_aggregate(g, sub, next);     /* the sub-modules become the nodes */
            i32* hl = (i32*)malloc(sizeof(i32) * (size_t)(next ? next : 1));
            im_core(&h, smod, inv, s, hl);               /* from the modules they came from */
            for (i64 v = 0; v < N; ++v) nl[v] = hl[sub[v]];
            renumber(N, nl, loc);
            im_free(&h);
            free(hl); free(moff); free(ml); free(loc); free(cur); free(sub); free(smod);
        }
        const double Ln = im_codelength(g, nl, inv, nt);
        memcpy(lab, nl, sizeof(i32) * (size_t)N);       /* igraph keeps the iteration's result */
        L = Ln;
        if (!(outer_old - Ln > 1e-10)) break;
    }
    free(nl);
    return L;
}

/* The fuller restatement: best of `trials` infomap_partition runs (unweighted topology).
 * Also returns, through core_L, the best core-only codelength of the same trials' first
 * iteration (what orc_infomap and the engine compute) for the gap measurement. */
double orc_infomap_full(i64 N, const i64* rowptr, const i32* col, u64 seed, int trials, i32* lab, double* core_L) {
    u64 s = seed ^ 0x9FB21C651E98DF25ull;
    im_graph g;
    g.n = N;
    const i64 E = rowptr[N];
    g.rp = (i64*)malloc(sizeof(i64) * (size_t)(N + 1));
    g.col = (i32*)malloc(sizeof(i32) * (size_t)(E ? E : 1));
    g.w = (i64*)malloc(sizeof(i64) * (size_t)(E ? E : 1));
    g.kv = (i64*)malloc(sizeof(i64) * (size_t)(N ? N : 1));
    g.sv = (i64*)malloc(sizeof(i64) * (size_t)(N ? N : 1));
    memcpy(g.rp, rowptr, sizeof(i64) * (size_t)(N + 1));
    if (E) memcpy(g.col, col, sizeof(i32) * (size_t)E);
    for (i64 j = 0; j < E; ++j) g.w[j] = 1;
    for (i64 v = 0; v < N; ++v) g.kv[v] = g.sv[v] = rowptr[v + 1] - rowptr[v];
    long long M2 = E;
    const double inv = M2 > 0 ? 1.0 / (double)M2 : 0.0, nt = im_node_term(&g, inv);
    i32* tmp = (i32*)malloc(sizeof(i32) * (size_t)(N ? N : 1));
    double best = 1e300, bcore = 1e300;
    for (int t = 0; t < (trials > 0 ? trials : 1); ++t) {
        u64 s2 = s;
        im_core(&g, NULL, inv, &s2, tmp);
        const double Lc = im_codelength(&g, tmp, inv, nt);
        if (Lc < bcore) bcore = Lc;
        const double L = im_partition(&g, &s, tmp, 0);
        if (L < best) { best = L; memcpy(lab, tmp, sizeof(i32) * (size_t)N); }
    }
    if (core_L) *core_L = bcore;
    im_free(&g);
    free(tmp);
    return best;
}
