// shud_partition.cpp — multilevel mesh partitioner, RCB fallback and per-rank halo plans (include/
// shud_partition.h).  Plain C++17, part of libshud_host.so.
//
// What is partitioned: the reference's RHS loops over all elements, segments and reaches in one process
// (src/ModelData/MD_f.cpp:9-50 serial, MD_f_omp.cpp:12-66 OpenMP).  Every flux is a one-hop function of y
// (element <-> 3 lateral neighbours, MD_ElementFlux.cpp:35-156; segment <-> (element, reach),
// MD_RiverFlux.cpp:100-126; reach <-> downstream / upstream reaches, MD_RiverFlux.cpp:5-63 and the junction
// sums of MD_f.cpp:236-240), so a k-way element partition plus one ghost layer lets each rank compute its owned
// DY exactly as one process would.  The partitioner minimises that ghost layer: the cut of the element dual
// graph, with river coupling edges so that a reach's segments stay with one rank where they can.
#include "shud_partition.h"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <numeric>
#include <random>
#include <string>
#include <thread>
#include <vector>

namespace {

thread_local std::string g_err;

int perr(int code, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

// ------------------------------------------------------------------------------------------------
// graphs
// ------------------------------------------------------------------------------------------------
struct Graph {
    int32_t n = 0;
    std::vector<int64_t> xadj;    // [n+1]
    std::vector<int32_t> adj;     // neighbours
    std::vector<int32_t> ew;      // edge weights (symmetric)
    std::vector<int32_t> vw;      // vertex weights
    int64_t tvw = 0;
};

// element dual graph + river coupling edges (weights summed where they coincide)
Graph dual_graph(const ShudMeshSoA *m) {
    const int NE = m->num_ele, NS = m->num_seg, NR = m->num_riv;
    Graph g;
    g.n = NE;
    g.vw.assign(NE, 1);
    for (int s = 0; s < NS; s++) g.vw[m->seg_ele[s]] += 1;
    // directed candidate edges (u -> v, w): each undirected edge appears once from each side
    std::vector<int64_t> cnt(NE + 1, 0);
    auto has_back = [&](int a, int b) {     // does a list b as a neighbour?
        for (int j = 0; j < 3; j++)
            if (m->nabr[(size_t)j * NE + a] == b) return true;
        return false;
    };
    // river coupling pairs: consecutive segments of one reach, last segment of a reach -> first of its downstream
    std::vector<std::pair<int32_t, int32_t>> rp;
    std::vector<int32_t> first_seg(NR, -1), last_seg(NR, -1);
    for (int s = 0; s < NS; s++) {
        const int r = m->seg_riv[s];
        if (first_seg[r] < 0) first_seg[r] = s;
        last_seg[r] = s;
    }
    for (int s = 0; s + 1 < NS; s++)
        if (m->seg_riv[s] == m->seg_riv[s + 1] && m->seg_ele[s] != m->seg_ele[s + 1])
            rp.emplace_back(m->seg_ele[s], m->seg_ele[s + 1]);
    for (int r = 0; r < NR; r++) {
        const int d = m->riv_down[r];
        if (d >= 0 && last_seg[r] >= 0 && first_seg[d] >= 0) {
            const int a = m->seg_ele[last_seg[r]], b = m->seg_ele[first_seg[d]];
            if (a != b) rp.emplace_back(a, b);
        }
    }
    for (int i = 0; i < NE; i++)
        for (int j = 0; j < 3; j++) {
            const int nb = m->nabr[(size_t)j * NE + i];
            if (nb < 0 || nb == i) continue;
            cnt[i + 1]++;
            if (!has_back(nb, i)) cnt[nb + 1]++;          // asymmetric adjacency: add the missing direction
        }
    for (auto &e : rp) { cnt[e.first + 1]++; cnt[e.second + 1]++; }
    for (int i = 0; i < NE; i++) cnt[i + 1] += cnt[i];
    std::vector<int32_t> tv(cnt[NE]), tw(cnt[NE]);
    std::vector<int64_t> pos(cnt.begin(), cnt.end() - 1);
    for (int i = 0; i < NE; i++)
        for (int j = 0; j < 3; j++) {
            const int nb = m->nabr[(size_t)j * NE + i];
            if (nb < 0 || nb == i) continue;
            tv[pos[i]] = nb; tw[pos[i]++] = 1;
            if (!has_back(nb, i)) { tv[pos[nb]] = i; tw[pos[nb]++] = 1; }
        }
    for (auto &e : rp) {
        tv[pos[e.first]] = e.second; tw[pos[e.first]++] = 1;
        tv[pos[e.second]] = e.first; tw[pos[e.second]++] = 1;
    }
    // merge duplicates per vertex (lateral + river on one pair, or two river links)
    g.xadj.assign(NE + 1, 0);
    g.adj.reserve(cnt[NE]);
    g.ew.reserve(cnt[NE]);
    std::vector<std::pair<int32_t, int32_t>> row;
    for (int i = 0; i < NE; i++) {
        row.clear();
        for (int64_t k = cnt[i]; k < cnt[i + 1]; k++) row.emplace_back(tv[k], tw[k]);
        std::sort(row.begin(), row.end());
        for (size_t k = 0; k < row.size(); k++) {
            if (k && row[k].first == row[k - 1].first) { g.ew.back() += row[k].second; continue; }
            g.adj.push_back(row[k].first);
            g.ew.push_back(row[k].second);
        }
        g.xadj[i + 1] = (int64_t)g.adj.size();
    }
    g.tvw = 0;
    for (int v : g.vw) g.tvw += v;
    return g;
}

// heavy-edge matching + contraction; returns false when the graph no longer shrinks
bool coarsen(const Graph &g, std::mt19937_64 &rng, int64_t maxvw, Graph &c, std::vector<int32_t> &cmap) {
    const int n = g.n;
    // visit order: blocks of 2048 consecutive vertices in a random order (block b_k = (off + k * stride) mod nb,
    // stride coprime to nb), vertices in index order inside a block — random enough for the matching, and the
    // adjacency of consecutive visits stays in cache (a fully scattered order costs a miss per vertex)
    constexpr int64_t B = 2048;
    const uint64_t nb = (uint64_t)((n + B - 1) / B);
    uint64_t stride = (rng() % nb) | 1;
    while (std::gcd(stride, nb) != 1) stride += 2;
    const uint64_t off = rng() % nb;
    std::vector<int32_t> match(n, -1);
    for (int64_t k = 0; k < (int64_t)nb * B; k++) {
        const int64_t blk = (int64_t)((off + (uint64_t)(k / B) * stride) % nb);
        const int64_t v64 = blk * B + k % B;
        if (v64 >= n) continue;
        const int v = (int)v64;
        if (match[v] >= 0) continue;
        int best = -1, bw = -1;
        for (int64_t k = g.xadj[v]; k < g.xadj[v + 1]; k++) {
            const int u = g.adj[k];
            if (match[u] >= 0 || u == v) continue;
            if ((int64_t)g.vw[v] + g.vw[u] > maxvw) continue;
            if (g.ew[k] > bw) { bw = g.ew[k]; best = u; }
        }
        if (best >= 0) { match[v] = best; match[best] = v; }
        else match[v] = v;
    }
    cmap.assign(n, -1);
    std::vector<int32_t> f1, f2;
    f1.reserve(n / 2 + 1);
    f2.reserve(n / 2 + 1);
    int cn = 0;
    for (int v = 0; v < n; v++) {
        if (cmap[v] >= 0) continue;
        cmap[v] = cn;
        cmap[match[v]] = cn;
        f1.push_back(v);
        f2.push_back(match[v]);
        cn++;
    }
    if (cn > (int64_t)n * 95 / 100) return false;
    c.n = cn;
    c.vw.assign(cn, 0);
    c.xadj.assign(cn + 1, 0);
    c.adj.clear();
    c.ew.clear();
    c.adj.reserve(g.adj.size() / 2 + cn);
    c.ew.reserve(g.adj.size() / 2 + cn);
    std::vector<int64_t> htab(cn, -1);
    for (int ci = 0; ci < cn; ci++) {
        const int64_t start = (int64_t)c.adj.size();
        const int fv[2] = {f1[ci], f2[ci]};
        const int nf = fv[0] == fv[1] ? 1 : 2;
        for (int t = 0; t < nf; t++) {
            const int v = fv[t];
            c.vw[ci] += g.vw[v];
            for (int64_t k = g.xadj[v]; k < g.xadj[v + 1]; k++) {
                const int cu = cmap[g.adj[k]];
                if (cu == ci) continue;
                if (htab[cu] < 0) {
                    htab[cu] = (int64_t)c.adj.size();
                    c.adj.push_back(cu);
                    c.ew.push_back(g.ew[k]);
                } else {
                    c.ew[htab[cu]] += g.ew[k];
                }
            }
        }
        for (int64_t k = start; k < (int64_t)c.adj.size(); k++) htab[c.adj[k]] = -1;
        c.xadj[ci + 1] = (int64_t)c.adj.size();
    }
    c.tvw = g.tvw;
    return true;
}

// ------------------------------------------------------------------------------------------------
// multilevel bisection: coarsen, grow + FM on the coarsest graph, FM at every uncoarsening level
// ------------------------------------------------------------------------------------------------
Graph induced(const Graph &g, const std::vector<int32_t> &verts, std::vector<int32_t> &l) {
    Graph s;
    s.n = (int32_t)verts.size();
    for (size_t i = 0; i < verts.size(); i++) l[verts[i]] = (int32_t)i;
    s.xadj.reserve(verts.size() + 1);
    s.xadj.push_back(0);
    s.vw.reserve(verts.size());
    for (int v : verts) {
        s.vw.push_back(g.vw[v]);
        s.tvw += g.vw[v];
        for (int64_t k = g.xadj[v]; k < g.xadj[v + 1]; k++)
            if (l[g.adj[k]] >= 0) { s.adj.push_back(l[g.adj[k]]); s.ew.push_back(g.ew[k]); }
        s.xadj.push_back((int64_t)s.adj.size());
    }
    for (int v : verts) l[v] = -1;
    return s;
}

int64_t bisect_cut(const Graph &s, const std::vector<int8_t> &side) {
    int64_t c = 0;
    for (int v = 0; v < s.n; v++)
        for (int64_t k = s.xadj[v]; k < s.xadj[v + 1]; k++)
            if (side[v] != side[s.adj[k]]) c += s.ew[k];
    return c / 2;
}

// Fiduccia–Mattheyses passes on a bisection (boundary vertices in a max-gain heap, lazy deletion): moves the
// best-gain vertex whose move keeps both sides within their caps (or relieves an overweight side), lets the
// cut rise for up to `climb` moves (hill climbing), then rolls back to the best state seen
void fm_refine(const Graph &s, std::vector<int8_t> &side, int64_t cap0, int64_t cap1, int passes, int climb) {
    const int n = s.n;
    int64_t w[2] = {0, 0};
    for (int v = 0; v < n; v++) w[side[v]] += s.vw[v];
    const int64_t cap[2] = {cap0, cap1};
    auto over = [&]() { return std::max<int64_t>(0, w[0] - cap[0]) + std::max<int64_t>(0, w[1] - cap[1]); };
    // gains are computed once per call and kept current through moves and rollbacks (O(E) once, then
    // O(moves x degree)); boundary vertices are those with gain > -degree
    std::vector<int64_t> gain(n), degw(n);
    int64_t cut = 0;
    for (int v = 0; v < n; v++) {
        int64_t ext = 0, in = 0;
        for (int64_t k = s.xadj[v]; k < s.xadj[v + 1]; k++) (side[s.adj[k]] != side[v] ? ext : in) += s.ew[k];
        gain[v] = ext - in;
        degw[v] = ext + in;
        cut += ext;
    }
    cut /= 2;
    std::vector<char> locked(n, 0);
    std::vector<int32_t> moves;
    auto flip = [&](int v) {                   // move v to the other side, updating weights, gains and cut
        const int from = side[v], to = from ^ 1;
        side[v] = (int8_t)to;
        w[from] -= s.vw[v];
        w[to] += s.vw[v];
        cut -= gain[v];
        for (int64_t k = s.xadj[v]; k < s.xadj[v + 1]; k++) {
            const int u = s.adj[k];
            gain[u] += (side[u] == to) ? -2 * (int64_t)s.ew[k] : 2 * (int64_t)s.ew[k];
        }
        gain[v] = -gain[v];
    };
    std::vector<std::pair<int64_t, int32_t>> heap;
    for (int pass = 0; pass < passes; pass++) {
        heap.clear();
        for (int v = 0; v < n; v++)
            if (gain[v] > -degw[v]) heap.emplace_back(gain[v], v);
        std::make_heap(heap.begin(), heap.end());
        for (int v : moves) locked[v] = 0;
        moves.clear();
        int64_t best_cut = cut, best_over = over();
        size_t best_len = 0;
        int since_best = 0;
        while (!heap.empty()) {
            std::pop_heap(heap.begin(), heap.end());
            const auto [gv, v] = heap.back();
            heap.pop_back();
            if (locked[v] || gv != gain[v]) continue;
            const int from = side[v], to = from ^ 1;
            if (w[to] + s.vw[v] > cap[to] && w[from] <= cap[from]) continue;
            flip(v);
            locked[v] = 1;
            moves.push_back(v);
            for (int64_t k = s.xadj[v]; k < s.xadj[v + 1]; k++) {
                const int u = s.adj[k];
                if (!locked[u]) { heap.emplace_back(gain[u], u); std::push_heap(heap.begin(), heap.end()); }
            }
            const int64_t ov = over();
            if (ov < best_over || (ov == best_over && cut < best_cut)) {
                best_over = ov; best_cut = cut; best_len = moves.size(); since_best = 0;
            } else if (++since_best > climb) {
                break;
            }
        }
        for (size_t k = moves.size(); k > best_len; k--) flip(moves[k - 1]);   // roll back past the best state
        if (best_len == 0) break;
    }
}

// greedy graph growing from `seed`: side 0 grows by the max-gain frontier vertex until its weight reaches
// target (coarsest graph only: a few hundred vertices)
void grow(const Graph &s, int seed, int64_t target, std::vector<int8_t> &side) {
    const int n = s.n;
    side.assign(n, 1);
    std::vector<int64_t> gain(n, 0);
    std::vector<char> front(n, 0);
    int64_t w0 = 0;
    int v = seed;
    while (true) {
        side[v] = 0;
        w0 += s.vw[v];
        front[v] = 0;
        for (int64_t k = s.xadj[v]; k < s.xadj[v + 1]; k++) {
            const int u = s.adj[k];
            if (side[u] == 1) { front[u] = 1; gain[u] += 2 * s.ew[k]; }
        }
        if (w0 >= target) break;
        int bv = -1;
        int64_t bg = INT64_MIN;
        for (int u = 0; u < n; u++)
            if (front[u] && gain[u] > bg) { bg = gain[u]; bv = u; }
        if (bv < 0) {                                  // disconnected: restart from any vertex on side 1
            for (int u = 0; u < n; u++)
                if (side[u] == 1) { bv = u; break; }
            if (bv < 0) break;
        }
        v = bv;
    }
}

// bisection of g into side 0 (weight fraction f0) and side 1, multilevel
void ml_bisect(const Graph &g, double f0, double ub, std::mt19937_64 &rng, std::vector<int8_t> &side,
               int *levels, int *coarse_n) {
    std::vector<Graph> lv;
    std::vector<std::vector<int32_t>> cm;
    const Graph *cur = &g;
    const int ctarget = 200;
    while (cur->n > ctarget && lv.size() < 64) {
        Graph c;
        std::vector<int32_t> cmap;
        const int64_t maxvw = std::max<int64_t>(2, (int64_t)(1.5 * (double)g.tvw / ctarget));
        if (!coarsen(*cur, rng, maxvw, c, cmap)) break;
        lv.push_back(std::move(c));
        cm.push_back(std::move(cmap));
        cur = &lv.back();
    }
    *levels = (int)lv.size();
    *coarse_n = cur->n;
    const int64_t t0 = (int64_t)((double)g.tvw * f0);
    const int64_t cap0 = (int64_t)std::ceil(ub * (double)g.tvw * f0);
    const int64_t cap1 = (int64_t)std::ceil(ub * (double)g.tvw * (1. - f0));
    std::vector<int8_t> best, s;
    int64_t best_cut = INT64_MAX, best_ov = INT64_MAX;
    for (int t = 0; t < 12; t++) {
        grow(*cur, (int)(rng() % (uint64_t)cur->n), t0, s);
        fm_refine(*cur, s, cap0, cap1, 8, std::max(50, cur->n / 4));
        int64_t w0 = 0;
        for (int v = 0; v < cur->n; v++) if (!s[v]) w0 += cur->vw[v];
        const int64_t ov = std::max<int64_t>(0, w0 - cap0) + std::max<int64_t>(0, cur->tvw - w0 - cap1);
        const int64_t c = bisect_cut(*cur, s);
        if (ov < best_ov || (ov == best_ov && c < best_cut)) { best_ov = ov; best_cut = c; best = s; }
    }
    for (int l = (int)lv.size() - 1; l >= 0; l--) {
        const Graph &fine = l ? lv[l - 1] : g;
        std::vector<int8_t> fs(fine.n);
        for (int v = 0; v < fine.n; v++) fs[v] = best[cm[l][v]];
        best.swap(fs);
        fm_refine(fine, best, cap0, cap1, 6, 200);
        lv.pop_back();
        cm.pop_back();
    }
    side.swap(best);
}

// multilevel recursive bisection: parts [p0, p0 + np) over the vertices `verts` of g.  Each sub-problem draws from
// its own generator seeded by (seed, p0, np), so the two halves can run on two threads and the result does not
// depend on scheduling; the first log2(8) levels fork (a k = 8 partition keeps up to 4 threads busy).
struct RbStats {
    std::mutex mu;
    int levels = 0, coarse_n = 0;
};
void recursive_bisect(const Graph &g, const std::vector<int32_t> &verts, int p0, int np, double ub, uint64_t seed,
                      std::vector<int32_t> &part, RbStats &st, int depth) {
    if (np == 1 || verts.size() <= 1) {
        for (int v : verts) part[v] = p0;
        return;
    }
    const int nl = np / 2;
    std::vector<int8_t> side;
    {
        std::mt19937_64 rng(seed ^ (0x9E3779B97F4A7C15ull * (uint64_t)(p0 + 1)) ^ ((uint64_t)np << 40));
        std::vector<int32_t> l(g.n, -1);
        Graph s = induced(g, verts, l);
        std::vector<int32_t>().swap(l);
        // the per-bisection slack compounds over log2(k) levels: split the 1.03 budget between them
        const double lvl_ub = std::pow(ub, 1.0 / std::max(1.0, std::ceil(std::log2((double)np))));
        int levels = 0, coarse_n = 0;
        ml_bisect(s, (double)nl / np, lvl_ub, rng, side, &levels, &coarse_n);
        std::lock_guard<std::mutex> lk(st.mu);
        st.levels = std::max(st.levels, levels);
        st.coarse_n = std::max(st.coarse_n, coarse_n);
    }
    std::vector<int32_t> L, R;
    for (size_t v = 0; v < verts.size(); v++) (side[v] == 0 ? L : R).push_back(verts[v]);
    std::vector<int8_t>().swap(side);
    if (depth < 3 && nl > 0 && np - nl > 1) {
        std::thread t([&] { recursive_bisect(g, L, p0, nl, ub, seed, part, st, depth + 1); });
        recursive_bisect(g, R, p0 + nl, np - nl, ub, seed, part, st, depth + 1);
        t.join();
    } else {
        recursive_bisect(g, L, p0, nl, ub, seed, part, st, depth + 1);
        recursive_bisect(g, R, p0 + nl, np - nl, ub, seed, part, st, depth + 1);
    }
}

// ------------------------------------------------------------------------------------------------
// k-way greedy boundary refinement (each level of the uncoarsening)
// ------------------------------------------------------------------------------------------------
// locked (optional): vertices that stay where they are (lake groups)
void kway_refine(const Graph &g, int k, double ub, int passes, std::vector<int32_t> &part,
                 const std::vector<char> *locked = nullptr) {
    const int n = g.n;
    std::vector<int64_t> pw(k, 0);
    for (int v = 0; v < n; v++) pw[part[v]] += g.vw[v];
    const int64_t maxpw = (int64_t)std::ceil(ub * (double)g.tvw / k);
    std::vector<int64_t> conn(k, 0);
    std::vector<int> touched;
    touched.reserve(64);
    for (int pass = 0; pass < passes; pass++) {
        int64_t moved = 0;
        for (int v = 0; v < n; v++) {
            if (locked && (*locked)[v]) continue;
            const int from = part[v];
            bool bnd = false;
            for (int64_t e = g.xadj[v]; e < g.xadj[v + 1]; e++)
                if (part[g.adj[e]] != from) { bnd = true; break; }
            if (!bnd) continue;
            touched.clear();
            for (int64_t e = g.xadj[v]; e < g.xadj[v + 1]; e++) {
                const int q = part[g.adj[e]];
                if (conn[q] == 0) touched.push_back(q);
                conn[q] += g.ew[e];
            }
            const int64_t id = conn[from];
            const int64_t vw = g.vw[v];
            int best = -1;
            int64_t bg = INT64_MIN;
            for (int q : touched) {
                if (q == from) continue;
                if (pw[q] + vw > maxpw) continue;
                const int64_t gq = conn[q] - id;
                if (gq > bg || (gq == bg && best >= 0 && pw[q] < pw[best])) { bg = gq; best = q; }
            }
            bool go = false;
            if (best >= 0) {
                if (bg > 0) go = true;
                else if (bg == 0 && pw[from] - vw > pw[best] + vw) go = true;    // balance-improving tie
                else if (pw[from] > maxpw) go = true;                           // overweight source
            }
            if (go) {
                part[v] = best;
                pw[from] -= vw;
                pw[best] += vw;
                moved++;
            }
            for (int q : touched) conn[q] = 0;
        }
        if (!moved) break;
    }
}

int64_t graph_cut(const Graph &g, const std::vector<int32_t> &part) {
    int64_t c = 0;
    for (int v = 0; v < g.n; v++)
        for (int64_t e = g.xadj[v]; e < g.xadj[v + 1]; e++)
            if (part[g.adj[e]] != part[v]) c += g.ew[e];
    return c / 2;
}

// ------------------------------------------------------------------------------------------------
// RCB (bit-identical to shud_rhs/partition.py rcb)
// ------------------------------------------------------------------------------------------------
void rcb_rec(const double *x, const double *y, const std::vector<double> &w, std::vector<int32_t> idx, int p0,
             int np, int32_t *part) {
    if (np == 1 || idx.empty()) {
        for (int i : idx) part[i] = p0;
        return;
    }
    const int nl = np / 2;
    double xmn = x[idx[0]], xmx = xmn, ymn = y[idx[0]], ymx = ymn;
    for (int i : idx) {
        xmn = std::min(xmn, x[i]); xmx = std::max(xmx, x[i]);
        ymn = std::min(ymn, y[i]); ymx = std::max(ymx, y[i]);
    }
    const double *key = (xmx - xmn) >= (ymx - ymn) ? x : y;
    std::vector<int32_t> order(idx.size());
    std::iota(order.begin(), order.end(), 0);
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return key[idx[a]] < key[idx[b]]; });
    std::vector<double> cw(idx.size());
    double acc = 0.;
    for (size_t k = 0; k < idx.size(); k++) { acc += w[idx[order[k]]]; cw[k] = acc; }
    const double target = cw.back() * nl / np;
    size_t cut = (size_t)(std::lower_bound(cw.begin(), cw.end(), target) - cw.begin());
    if (idx.size() > 1) cut = std::min(std::max(cut, (size_t)1), idx.size() - 1);
    else cut = 0;
    std::vector<int32_t> L, R;
    L.reserve(cut);
    R.reserve(idx.size() - cut);
    for (size_t k = 0; k < idx.size(); k++) (k < cut ? L : R).push_back(idx[order[k]]);
    std::vector<int32_t>().swap(idx);
    std::vector<int32_t>().swap(order);
    std::sort(L.begin(), L.end());
    std::sort(R.begin(), R.end());
    rcb_rec(x, y, w, std::move(L), p0, nl, part);
    rcb_rec(x, y, w, std::move(R), p0 + nl, np - nl, part);
}

// ---- lakes ----
bool has_lakes(const ShudMeshSoA *m) { return m->num_lake > 0 && m->ilake; }

// lake groups: lakes joined when elements of two lakes share an edge or a bank element (a non-lake element
// with an edge on a lake element) touches both; grp[i] = the group's smallest lake id for lake and bank
// elements, -1 elsewhere
std::vector<int32_t> lake_groups(const ShudMeshSoA *m) {
    const int NE = m->num_ele, NL = m->num_lake;
    std::vector<int32_t> uf(NL), grp(NE, -1), first(NE, -1);
    std::iota(uf.begin(), uf.end(), 0);
    auto find = [&](int a) {
        while (uf[a] != a) a = uf[a] = uf[uf[a]];
        return a;
    };
    auto unite = [&](int a, int b) {
        a = find(a);
        b = find(b);
        if (a != b) uf[std::max(a, b)] = std::min(a, b);
    };
    for (int i = 0; i < NE; i++) {
        const int li = m->ilake[i] - 1;
        for (int j = 0; j < 3; j++) {
            const int nb = m->nabr[(size_t)j * NE + i];
            if (nb < 0 || m->ilake[nb] <= 0) continue;
            const int lj = m->ilake[nb] - 1;
            if (li >= 0) unite(li, lj);
            else if (first[i] < 0) first[i] = lj;
            else unite(first[i], lj);
        }
    }
    for (int i = 0; i < NE; i++) {
        const int li = m->ilake[i] - 1;
        if (li >= 0) grp[i] = find(li);
        else if (first[i] >= 0) grp[i] = find(first[i]);
    }
    return grp;
}

// part of each lake (its elements' part; -1 for a lake without elements)
std::vector<int32_t> lake_parts(const ShudMeshSoA *m, const int32_t *ele_part) {
    std::vector<int32_t> lp(has_lakes(m) ? m->num_lake : 0, -1);
    if (lp.empty()) return lp;
    for (int i = 0; i < m->num_ele; i++)
        if (m->ilake[i] > 0) lp[m->ilake[i] - 1] = ele_part[i];
    return lp;
}

// move every lake group to the part holding most of its vertex weight (1 + #segments; lowest part on ties)
void constrain_lakes(const ShudMeshSoA *m, int nparts, int32_t *ele_part) {
    if (!has_lakes(m)) return;
    const int NE = m->num_ele, NL = m->num_lake;
    const std::vector<int32_t> grp = lake_groups(m);
    std::vector<int64_t> vw(NE, 1), w((size_t)NL * nparts, 0);
    for (int s = 0; s < m->num_seg; s++) vw[m->seg_ele[s]]++;
    for (int i = 0; i < NE; i++)
        if (grp[i] >= 0) w[(size_t)grp[i] * nparts + ele_part[i]] += vw[i];
    std::vector<int32_t> best(NL, 0);
    for (int g = 0; g < NL; g++)
        for (int p = 1; p < nparts; p++)
            if (w[(size_t)g * nparts + p] > w[(size_t)g * nparts + best[g]]) best[g] = p;
    for (int i = 0; i < NE; i++)
        if (grp[i] >= 0) ele_part[i] = best[grp[i]];
}

// reach owners: the part owning most of a reach's segments' elements (lowest on ties), part 0 without segments;
// with lakes, a reach with a segment on a lake element belongs to that lake's part (so lake elements are never
// segment ghosts of another rank)
std::vector<int32_t> reach_owners(const ShudMeshSoA *m, const int32_t *ele_part, int nparts) {
    const int NR = m->num_riv;
    std::vector<int32_t> cnt((size_t)NR * nparts, 0);
    for (int s = 0; s < m->num_seg; s++) cnt[(size_t)m->seg_riv[s] * nparts + ele_part[m->seg_ele[s]]]++;
    std::vector<int32_t> rp(NR, 0);
    for (int r = 0; r < NR; r++) {
        int best = 0;
        for (int p = 1; p < nparts; p++)
            if (cnt[(size_t)r * nparts + p] > cnt[(size_t)r * nparts + best]) best = p;
        rp[r] = best;
    }
    if (has_lakes(m))
        for (int s = 0; s < m->num_seg; s++)
            if (m->ilake[m->seg_ele[s]] > 0) rp[m->seg_riv[s]] = ele_part[m->seg_ele[s]];
    return rp;
}

// a plan with lakes needs every lake group on one part and every lake element's segments owned there
int check_lake_partition(const ShudMeshSoA *m, const int32_t *ele_part, const std::vector<int32_t> &rp) {
    if (!has_lakes(m)) return 0;
    const int NE = m->num_ele;
    const std::vector<int32_t> lp = lake_parts(m, ele_part);
    for (int i = 0; i < NE; i++) {
        if (m->ilake[i] <= 0) continue;
        if (ele_part[i] != lp[m->ilake[i] - 1])
            return perr(SHUD_ERR_UNSUPPORTED, "lake %d is split across parts (shud_partition_constrain)", m->ilake[i]);
        for (int j = 0; j < 3; j++) {
            const int nb = m->nabr[(size_t)j * NE + i];
            if (nb >= 0 && ele_part[nb] != ele_part[i])
                return perr(SHUD_ERR_UNSUPPORTED, "lake element %d and its neighbour %d lie on different parts "
                            "(shud_partition_constrain)", i, nb);
        }
    }
    for (int s = 0; s < m->num_seg; s++) {
        const int e = m->seg_ele[s];
        if (m->ilake[e] > 0 && rp[m->seg_riv[s]] != ele_part[e])
            return perr(SHUD_ERR_UNSUPPORTED, "reach %d has segments on lake elements of different parts", m->seg_riv[s]);
    }
    return 0;
}

void mesh_cuts(const ShudMeshSoA *m, const int32_t *ele_part, int nparts, int64_t *ec, int64_t *sc) {
    const int NE = m->num_ele;
    int64_t c = 0;
    for (int j = 0; j < 3; j++)
        for (int i = 0; i < NE; i++) {
            const int nb = m->nabr[(size_t)j * NE + i];
            if (nb > i && ele_part[nb] != ele_part[i]) c++;
        }
    *ec = c;
    const std::vector<int32_t> rp = reach_owners(m, ele_part, nparts);
    int64_t s = 0;
    for (int k = 0; k < m->num_seg; k++)
        if (ele_part[m->seg_ele[k]] != rp[m->seg_riv[k]]) s++;
    *sc = s;
}

// need masks: bit q set when rank q owns or ghosts the entity (one pass over elements, segments, reaches).
// Ghost elements of q: lateral neighbours of q's elements and elements of segments q holds (a segment is held
// by the owners of its element and of its reach); ghost reaches of q: reaches of segments q holds, downstream
// and upstream reaches of q's reaches (partition.py _ghost_sets)
void need_masks(const ShudMeshSoA *m, const int32_t *ele_part, const std::vector<int32_t> &rp,
                std::vector<uint64_t> &ne, std::vector<uint64_t> &nr) {
    const int NE = m->num_ele, NR = m->num_riv, NS = m->num_seg;
    ne.assign(NE, 0);
    nr.assign(NR, 0);
    for (int i = 0; i < NE; i++) {
        const uint64_t b = 1ull << ele_part[i];
        ne[i] |= b;
        for (int j = 0; j < 3; j++) {
            const int nb = m->nabr[(size_t)j * NE + i];
            if (nb >= 0) ne[nb] |= b;
        }
    }
    for (int s = 0; s < NS; s++) {
        const int e = m->seg_ele[s], r = m->seg_riv[s];
        const uint64_t b = (1ull << ele_part[e]) | (1ull << rp[r]);
        ne[e] |= b;
        nr[r] |= b;
    }
    const std::vector<int32_t> lp = lake_parts(m, ele_part);
    for (int r = 0; r < NR; r++) {
        nr[r] |= 1ull << rp[r];
        const int d = m->riv_down[r];
        if (d >= 0) {
            nr[d] |= 1ull << rp[r];          // downstream of an owned reach
            nr[r] |= 1ull << rp[d];          // upstream of an owned reach
        } else if (d <= -4 && !lp.empty()) {
            const int L = -3 - d - 1;        // flows into lake L: its QrivDown is summed by the lake's owner
            if (L < (int)lp.size() && lp[L] >= 0) nr[r] |= 1ull << lp[L];
        }
    }
}

// ghost elements / reaches per part of a partition; returns the largest per-part ghost count (elements +
// reaches), the size of the biggest halo one RHS must wait for
int64_t halo_counts(const ShudMeshSoA *m, const int32_t *ele_part, int nparts, std::vector<int64_t> &ge,
                    std::vector<int64_t> &gr) {
    const std::vector<int32_t> rp = reach_owners(m, ele_part, nparts);
    std::vector<uint64_t> ne, nr;
    need_masks(m, ele_part, rp, ne, nr);
    ge.assign(nparts, 0);
    gr.assign(nparts, 0);
    for (int i = 0; i < m->num_ele; i++) {
        uint64_t b = ne[i] & ~(1ull << ele_part[i]);
        while (b) { ge[__builtin_ctzll(b)]++; b &= b - 1; }
    }
    for (int r = 0; r < m->num_riv; r++) {
        uint64_t b = nr[r] & ~(1ull << rp[r]);
        while (b) { gr[__builtin_ctzll(b)]++; b &= b - 1; }
    }
    int64_t mx = 0;
    for (int p = 0; p < nparts; p++) mx = std::max(mx, ge[p] + gr[p]);
    return mx;
}

int check_mesh(const ShudMeshSoA *m) {
    if (!m || m->num_ele <= 0 || !m->nabr) return perr(SHUD_ERR_ARG, "empty mesh");
    if (m->num_seg > 0 && (!m->seg_ele || !m->seg_riv)) return perr(SHUD_ERR_ARG, "segments without indices");
    for (int s = 0; s < m->num_seg; s++)
        if (m->seg_ele[s] < 0 || m->seg_ele[s] >= m->num_ele || m->seg_riv[s] < 0 || m->seg_riv[s] >= m->num_riv)
            return perr(SHUD_ERR_ARG, "segment %d: index out of range", s);
    for (int64_t k = 0; k < 3 * (int64_t)m->num_ele; k++)
        if (m->nabr[k] >= m->num_ele) return perr(SHUD_ERR_ARG, "nabr out of range");
    for (int r = 0; r < m->num_riv; r++)
        if (m->riv_down && m->riv_down[r] >= m->num_riv) return perr(SHUD_ERR_ARG, "riv_down out of range");
    if (has_lakes(m))
        for (int i = 0; i < m->num_ele; i++)
            if (m->ilake[i] < 0 || m->ilake[i] > m->num_lake) return perr(SHUD_ERR_ARG, "ilake[%d] out of range", i);
    return 0;
}

}  // namespace

// ================================================================================================
// partitioner
// ================================================================================================
extern "C" const char *shud_partition_error(void) { return g_err.c_str(); }

extern "C" int shud_partition_constrain(const ShudMeshSoA *mesh, int32_t nparts, int32_t *ele_part) {
    int rc = check_mesh(mesh);
    if (rc) return rc;
    if (!ele_part || nparts < 1 || nparts > SHUD_PART_MAX_PARTS) return perr(SHUD_ERR_ARG, "bad partition");
    for (int i = 0; i < mesh->num_ele; i++)
        if (ele_part[i] < 0 || ele_part[i] >= nparts) return perr(SHUD_ERR_ARG, "ele_part[%d] out of range", i);
    constrain_lakes(mesh, nparts, ele_part);
    return 0;
}

extern "C" int shud_partition_cut(const ShudMeshSoA *mesh, const int32_t *ele_part, int32_t nparts, int64_t *ec,
                                  int64_t *sc) {
    int rc = check_mesh(mesh);
    if (rc) return rc;
    if (!ele_part || nparts < 1 || nparts > SHUD_PART_MAX_PARTS) return perr(SHUD_ERR_ARG, "bad partition");
    int64_t a = 0, b = 0;
    mesh_cuts(mesh, ele_part, nparts, &a, &b);
    if (ec) *ec = a;
    if (sc) *sc = b;
    return 0;
}

static int partition_one(const ShudMeshSoA *mesh, const double *cx, const double *cy, int nparts, int method,
                         uint64_t seed, int32_t *ele_part, ShudPartStats &S) {
    const int NE = mesh->num_ele;
    if (method == SHUD_PART_RCB) {
        if (!cx || !cy) return perr(SHUD_ERR_ARG, "RCB needs element centroids");
        std::vector<double> w(NE, 1.0);
        for (int s = 0; s < mesh->num_seg; s++) w[mesh->seg_ele[s]] += 1.0;
        std::vector<int32_t> idx(NE);
        std::iota(idx.begin(), idx.end(), 0);
        rcb_rec(cx, cy, w, std::move(idx), 0, nparts, ele_part);
        S.graph_cut = -1;                                       // reported for the multilevel graph only
    } else if (method == SHUD_PART_MULTILEVEL) {
        const double ub = 1.03;
        const bool verbose = getenv("SHUD_PART_VERBOSE") != nullptr;
        auto tk = std::chrono::steady_clock::now();
        auto lap = [&](const char *what) {
            const auto now = std::chrono::steady_clock::now();
            if (verbose) fprintf(stderr, "[partition] %s %.2fs\n", what, std::chrono::duration<double>(now - tk).count());
            tk = now;
        };
        Graph g = dual_graph(mesh);
        lap("dual graph");
        std::vector<int32_t> part(NE, 0), all(NE);
        std::iota(all.begin(), all.end(), 0);
        RbStats rb;
        recursive_bisect(g, all, 0, nparts, ub, seed, part, rb, 0);
        const int levels = rb.levels, coarse_n = rb.coarse_n;
        lap("recursive bisection");
        kway_refine(g, nparts, ub, 8, part);                    // k-way polish of the assembled partition
        lap("k-way refinement");
        if (has_lakes(mesh)) {
            // lake groups onto one part each, then rebalance around them (group vertices locked)
            constrain_lakes(mesh, nparts, part.data());
            const std::vector<int32_t> grp = lake_groups(mesh);
            std::vector<char> locked(NE, 0);
            for (int i = 0; i < NE; i++) locked[i] = grp[i] >= 0;
            kway_refine(g, nparts, ub, 16, part, &locked);
        }
        S.levels = levels;
        S.coarse_vertices = coarse_n;
        S.graph_cut = graph_cut(g, part);
        std::copy(part.begin(), part.end(), ele_part);
    } else {
        return perr(SHUD_ERR_ARG, "unknown method %d", method);
    }
    constrain_lakes(mesh, nparts, ele_part);                    // lake groups on one part each
    // every part must own at least one element
    std::vector<int64_t> pw(nparts, 0), pn(nparts, 0);
    int64_t tw = 0;
    std::vector<int64_t> vw(NE, 1);
    for (int s = 0; s < mesh->num_seg; s++) vw[mesh->seg_ele[s]]++;
    for (int i = 0; i < NE; i++) { pn[ele_part[i]]++; pw[ele_part[i]] += vw[i]; tw += vw[i]; }
    for (int p = 0; p < nparts; p++)
        if (!pn[p]) return perr(SHUD_ERR_ARG, "part %d is empty", p);
    S.imbalance = (double)*std::max_element(pw.begin(), pw.end()) / ((double)tw / nparts);
    mesh_cuts(mesh, ele_part, nparts, &S.edge_cut, &S.segment_cut);
    std::vector<int64_t> ge, gr;
    S.max_halo = halo_counts(mesh, ele_part, nparts, ge, gr);
    S.method_used = method;
    return 0;
}

extern "C" int shud_partition_mesh(const ShudMeshSoA *mesh, const double *cx, const double *cy, int32_t nparts,
                                   int32_t method, uint64_t seed, int32_t *ele_part, ShudPartStats *st) {
    const auto t0 = std::chrono::steady_clock::now();
    int rc = check_mesh(mesh);
    if (rc) return rc;
    if (!ele_part || nparts < 1 || nparts > SHUD_PART_MAX_PARTS) return perr(SHUD_ERR_ARG, "nparts must be 1..64");
    if (nparts > mesh->num_ele) return perr(SHUD_ERR_ARG, "more parts than elements");
    ShudPartStats S{};
    if (method == SHUD_PART_AUTO) {
        if ((rc = partition_one(mesh, cx, cy, nparts, SHUD_PART_MULTILEVEL, seed, ele_part, S))) return rc;
        if (cx && cy) {
            std::vector<int32_t> alt(mesh->num_ele);
            ShudPartStats A{};
            if ((rc = partition_one(mesh, cx, cy, nparts, SHUD_PART_RCB, seed, alt.data(), A))) return rc;
            if (A.max_halo < S.max_halo) {
                std::copy(alt.begin(), alt.end(), ele_part);
                S = A;
            }
        }
    } else if ((rc = partition_one(mesh, cx, cy, nparts, method, seed, ele_part, S))) {
        return rc;
    }
    S.seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (st) *st = S;
    return 0;
}

extern "C" int shud_partition_halo(const ShudMeshSoA *mesh, const int32_t *ele_part, int32_t nparts,
                                   int64_t *ghost_ele, int64_t *ghost_riv) {
    int rc = check_mesh(mesh);
    if (rc) return rc;
    if (!ele_part || nparts < 1 || nparts > SHUD_PART_MAX_PARTS) return perr(SHUD_ERR_ARG, "bad partition");
    std::vector<int64_t> ge, gr;
    halo_counts(mesh, ele_part, nparts, ge, gr);
    for (int p = 0; p < nparts; p++) {
        if (ghost_ele) ghost_ele[p] = ge[p];
        if (ghost_riv) ghost_riv[p] = gr[p];
    }
    return 0;
}

// ================================================================================================
// per-rank plan
// ================================================================================================
struct shud_plan {
    int rank = 0, nparts = 1;
    int NEg = 0, NRg = 0;
    std::vector<int32_t> ele_gid, riv_gid, seg_gid;      // local -> global
    int n_own_ele = 0, n_int = 0, n_own_riv = 0;
    std::vector<int32_t> riv_part;
    int NLg = 0;
    std::vector<int32_t> lake_gid;                        // owned lakes (0-based global ids), ascending
    std::vector<int32_t> l_bathy_off;
    std::vector<double> l_bathy_y, l_bathy_a;
    std::vector<int32_t> esend_off, esend_idx, erecv_off, rsend_off, rsend_idx, rrecv_off;
    // local mesh storage (shud_plan_local_mesh)
    std::vector<double> d_ele1[5], d_ele3[4], d_riv[9], d_seg[2], d_par[17];
    std::vector<int32_t> l_nabr, l_ibc, l_iss, l_ilake, l_down, l_rbc, l_sege, l_segr;
};

extern "C" int shud_plan_build(const ShudMeshSoA *m, const int32_t *ele_part, int32_t nparts, int32_t rank,
                               shud_plan_t *out) {
    int rc = check_mesh(m);
    if (rc) return rc;
    if (!out || !ele_part || nparts < 1 || nparts > SHUD_PART_MAX_PARTS || rank < 0 || rank >= nparts)
        return perr(SHUD_ERR_ARG, "bad plan arguments");
    const int NE = m->num_ele, NR = m->num_riv, NS = m->num_seg;
    for (int i = 0; i < NE; i++)
        if (ele_part[i] < 0 || ele_part[i] >= nparts) return perr(SHUD_ERR_ARG, "ele_part[%d] out of range", i);
    std::vector<int32_t> rp0 = reach_owners(m, ele_part, nparts);
    if ((rc = check_lake_partition(m, ele_part, rp0))) return rc;
    auto *P = new shud_plan;
    P->rank = rank;
    P->nparts = nparts;
    P->NEg = NE;
    P->NRg = NR;
    P->riv_part = std::move(rp0);
    const std::vector<int32_t> &rp = P->riv_part;
    if (has_lakes(m)) {
        P->NLg = m->num_lake;
        const std::vector<int32_t> lp = lake_parts(m, ele_part);
        for (int l = 0; l < m->num_lake; l++)
            if (lp[l] == rank) P->lake_gid.push_back(l);
    }
    std::vector<uint64_t> ne, nr;
    need_masks(m, ele_part, rp, ne, nr);
    const uint64_t me = 1ull << rank;
    // owned elements: [interior | boundary]; boundary = a lateral neighbour or an own segment's reach elsewhere
    std::vector<char> dep(NE, 0);
    for (int s = 0; s < NS; s++) {
        const int e = m->seg_ele[s];
        if (ele_part[e] == rank && rp[m->seg_riv[s]] != rank) dep[e] = 1;
    }
    std::vector<int32_t> own_int, own_bnd;
    for (int i = 0; i < NE; i++) {
        if (ele_part[i] != rank) continue;
        bool d = dep[i];
        for (int j = 0; j < 3 && !d; j++) {
            const int nb = m->nabr[(size_t)j * NE + i];
            if (nb >= 0 && ele_part[nb] != rank) d = true;
        }
        (d ? own_bnd : own_int).push_back(i);
    }
    P->n_int = (int)own_int.size();
    P->n_own_ele = (int)(own_int.size() + own_bnd.size());
    P->ele_gid = own_int;
    P->ele_gid.insert(P->ele_gid.end(), own_bnd.begin(), own_bnd.end());
    // ghosts grouped by source part, ascending global id inside a group
    P->erecv_off.assign(nparts + 1, 0);
    {
        std::vector<std::vector<int32_t>> g(nparts);
        for (int i = 0; i < NE; i++)
            if ((ne[i] & me) && ele_part[i] != rank) g[ele_part[i]].push_back(i);
        for (int q = 0; q < nparts; q++) {
            P->erecv_off[q + 1] = P->erecv_off[q] + (int32_t)g[q].size();
            P->ele_gid.insert(P->ele_gid.end(), g[q].begin(), g[q].end());
        }
    }
    for (int r = 0; r < NR; r++)
        if (rp[r] == rank) P->riv_gid.push_back(r);
    P->n_own_riv = (int)P->riv_gid.size();
    P->rrecv_off.assign(nparts + 1, 0);
    {
        std::vector<std::vector<int32_t>> g(nparts);
        for (int r = 0; r < NR; r++)
            if ((nr[r] & me) && rp[r] != rank) g[rp[r]].push_back(r);
        for (int q = 0; q < nparts; q++) {
            P->rrecv_off[q + 1] = P->rrecv_off[q] + (int32_t)g[q].size();
            P->riv_gid.insert(P->riv_gid.end(), g[q].begin(), g[q].end());
        }
    }
    for (int s = 0; s < NS; s++)
        if (ele_part[m->seg_ele[s]] == rank || rp[m->seg_riv[s]] == rank) P->seg_gid.push_back(s);
    // sends: to q, the entities this rank owns that q ghosts, in q's order (ascending global id) -> local index
    std::vector<int32_t> g2l(NE, -1);
    for (int k = 0; k < P->n_own_ele; k++) g2l[P->ele_gid[k]] = k;
    P->esend_off.assign(nparts + 1, 0);
    P->rsend_off.assign(nparts + 1, 0);
    for (int q = 0; q < nparts; q++) {
        P->esend_off[q + 1] = P->esend_off[q];
        P->rsend_off[q + 1] = P->rsend_off[q];
        if (q == rank) continue;
        const uint64_t bq = 1ull << q;
        for (int i = 0; i < NE; i++)
            if (ele_part[i] == rank && (ne[i] & bq)) { P->esend_idx.push_back(g2l[i]); P->esend_off[q + 1]++; }
        int lr = 0;
        for (int r = 0; r < NR; r++) {
            if (rp[r] != rank) continue;
            if (nr[r] & bq) { P->rsend_idx.push_back(lr); P->rsend_off[q + 1]++; }
            lr++;
        }
    }
    *out = P;
    return 0;
}

extern "C" void shud_plan_free(shud_plan_t p) { delete p; }

extern "C" int shud_plan_info(shud_plan_t p, ShudPlanInfo *I) {
    if (!p || !I) return perr(SHUD_ERR_ARG, "null argument");
    I->n_own_ele = p->n_own_ele;
    I->n_int_ele = p->n_int;
    I->n_ghost_ele = (int32_t)p->ele_gid.size() - p->n_own_ele;
    I->n_own_riv = p->n_own_riv;
    I->n_ghost_riv = (int32_t)p->riv_gid.size() - p->n_own_riv;
    I->n_seg = (int32_t)p->seg_gid.size();
    I->ele_gid = p->ele_gid.data();
    I->riv_gid = p->riv_gid.data();
    I->seg_gid = p->seg_gid.data();
    I->riv_part = p->riv_part.data();
    I->n_own_lake = (int32_t)p->lake_gid.size();
    I->lake_gid = p->lake_gid.data();
    return 0;
}

extern "C" int shud_plan_partition(shud_plan_t p, ShudPartition *o) {
    if (!p || !o) return perr(SHUD_ERR_ARG, "null argument");
    o->rank = p->rank;
    o->nranks = p->nparts;
    o->n_own_ele = p->n_own_ele;
    o->n_segghost_ele = (int32_t)p->ele_gid.size() - p->n_own_ele;
    o->n_own_riv = p->n_own_riv;
    o->ele_send_off = p->esend_off.data();
    o->ele_send_idx = p->esend_idx.data();
    o->ele_recv_off = p->erecv_off.data();
    o->riv_send_off = p->rsend_off.data();
    o->riv_send_idx = p->rsend_idx.data();
    o->riv_recv_off = p->rrecv_off.data();
    o->ele_gid = p->ele_gid.data();
    o->riv_gid = p->riv_gid.data();
    o->nccl_unique_id = nullptr;
    return 0;
}

extern "C" int shud_plan_local_mesh(shud_plan_t p, const ShudMeshSoA *g, const ShudParamsSoA *gp, ShudMeshSoA *L,
                                    ShudParamsSoA *lp) {
    if (!p || !g || !gp || !L || !lp) return perr(SHUD_ERR_ARG, "null argument");
    if (g->num_ele != p->NEg || g->num_riv != p->NRg) return perr(SHUD_ERR_ARG, "mesh does not match the plan");
    if (has_lakes(g) != (p->NLg > 0) || (p->NLg > 0 && g->num_lake != p->NLg))
        return perr(SHUD_ERR_ARG, "mesh lakes do not match the plan");
    const int NEg = g->num_ele;
    const int NEl = (int)p->ele_gid.size(), NRl = (int)p->riv_gid.size(), NSl = (int)p->seg_gid.size();
    const std::vector<int32_t> &le = p->ele_gid, &lr = p->riv_gid, &ls = p->seg_gid;
    std::vector<int32_t> g2le(NEg, -1), g2lr(g->num_riv, -1);
    for (int k = 0; k < NEl; k++) g2le[le[k]] = k;
    for (int k = 0; k < NRl; k++) g2lr[lr[k]] = k;
    auto gat1 = [&](const double *src, std::vector<double> &dst) -> const double * {
        if (!src) return nullptr;
        dst.resize(NEl);
        for (int k = 0; k < NEl; k++) dst[k] = src[le[k]];
        return dst.data();
    };
    auto gat3 = [&](const double *src, std::vector<double> &dst) -> const double * {
        if (!src) return nullptr;
        dst.resize(3 * (size_t)NEl);
        for (int j = 0; j < 3; j++)
            for (int k = 0; k < NEl; k++) dst[(size_t)j * NEl + k] = src[(size_t)j * NEg + le[k]];
        return dst.data();
    };
    auto gati = [&](const int32_t *src, std::vector<int32_t> &dst, const std::vector<int32_t> &idx) -> const int32_t * {
        if (!src) return nullptr;
        dst.resize(idx.size());
        for (size_t k = 0; k < idx.size(); k++) dst[k] = src[idx[k]];
        return dst.data();
    };
    auto gatr = [&](const double *src, std::vector<double> &dst) -> const double * {
        if (!src) return nullptr;
        dst.resize(NRl);
        for (int k = 0; k < NRl; k++) dst[k] = src[lr[k]];
        return dst.data();
    };
    memset(L, 0, sizeof *L);
    L->num_ele = NEl;
    L->num_riv = NRl;
    L->num_seg = NSl;
    L->close_boundary = g->close_boundary;
    L->area = gat1(g->area, p->d_ele1[0]);
    L->z_surf = gat1(g->z_surf, p->d_ele1[1]);
    L->z_bottom = gat1(g->z_bottom, p->d_ele1[2]);
    L->depression = gat1(g->depression, p->d_ele1[3]);
    L->rough = gat1(g->rough, p->d_ele1[4]);
    L->edge = gat3(g->edge, p->d_ele3[0]);
    L->dist2nabor = gat3(g->dist2nabor, p->d_ele3[1]);
    L->dist2edge = gat3(g->dist2edge, p->d_ele3[2]);
    L->avg_rough = gat3(g->avg_rough, p->d_ele3[3]);
    p->l_nabr.resize(3 * (size_t)NEl);
    for (int j = 0; j < 3; j++)
        for (int k = 0; k < NEl; k++) {
            const int nb = g->nabr[(size_t)j * NEg + le[k]];
            p->l_nabr[(size_t)j * NEl + k] = nb >= 0 ? g2le[nb] : -1;
        }
    L->nabr = p->l_nabr.data();
    L->ibc = gati(g->ibc, p->l_ibc, le);
    L->iss = gati(g->iss, p->l_iss, le);
    L->ilake = gati(g->ilake, p->l_ilake, le);
    // lakes: owned lakes renumbered 1..n_own_lake (lake elements are always owned, check_lake_partition)
    std::vector<int32_t> g2ll(p->NLg, -1);
    for (size_t k = 0; k < p->lake_gid.size(); k++) g2ll[p->lake_gid[k]] = (int32_t)k;
    if (p->NLg > 0) {
        for (int k = 0; k < NEl; k++) {
            const int v = p->l_ilake[k];
            if (v <= 0) continue;
            if (g2ll[v - 1] < 0) return perr(SHUD_ERR_ARG, "element %d of lake %d is local but the lake is not owned", le[k], v);
            p->l_ilake[k] = g2ll[v - 1] + 1;
        }
        const int nl = (int)p->lake_gid.size();
        p->l_bathy_off.assign(1, 0);
        p->l_bathy_y.clear();
        p->l_bathy_a.clear();
        for (int k = 0; k < nl; k++) {
            const int l = p->lake_gid[k];
            for (int q = g->lake_bathy_off[l]; q < g->lake_bathy_off[l + 1]; q++) {
                p->l_bathy_y.push_back(g->lake_bathy_y[q]);
                p->l_bathy_a.push_back(g->lake_bathy_a[q]);
            }
            p->l_bathy_off.push_back((int32_t)p->l_bathy_y.size());
        }
        L->num_lake = nl;
        L->lake_bathy_off = nl ? p->l_bathy_off.data() : nullptr;
        L->lake_bathy_y = nl ? p->l_bathy_y.data() : nullptr;
        L->lake_bathy_a = nl ? p->l_bathy_a.data() : nullptr;
    }
    p->l_down.resize(NRl);
    for (int k = 0; k < NRl; k++) {
        const int d = g->riv_down[lr[k]];
        if (d >= 0) {
            p->l_down[k] = g2lr[d] >= 0 ? g2lr[d] : -3;
        } else if (d <= -4 && p->NLg > 0) {            // into lake -3 - d: local id if owned, else the outlet code
            const int l = g2ll[-3 - d - 1];
            p->l_down[k] = l >= 0 ? -3 - (l + 1) : -3;
        } else {
            p->l_down[k] = d;
        }
    }
    L->riv_down = p->l_down.data();
    L->riv_bc = gati(g->riv_bc, p->l_rbc, lr);
    L->riv_length = gatr(g->riv_length, p->d_riv[0]);
    L->riv_bed_slope = gatr(g->riv_bed_slope, p->d_riv[1]);
    L->riv_dist2down = gatr(g->riv_dist2down, p->d_riv[2]);
    L->riv_avg_rough = gatr(g->riv_avg_rough, p->d_riv[3]);
    L->riv_depth = gatr(g->riv_depth, p->d_riv[4]);
    L->riv_bottom_width = gatr(g->riv_bottom_width, p->d_riv[5]);
    L->riv_bankslope = gatr(g->riv_bankslope, p->d_riv[6]);
    L->riv_ksath = gatr(g->riv_ksath, p->d_riv[7]);
    L->riv_bedthick = gatr(g->riv_bedthick, p->d_riv[8]);
    p->l_sege.resize(NSl);
    p->l_segr.resize(NSl);
    p->d_seg[0].resize(NSl);
    p->d_seg[1].resize(NSl);
    for (int k = 0; k < NSl; k++) {
        const int s = ls[k];
        p->l_sege[k] = g2le[g->seg_ele[s]];
        p->l_segr[k] = g2lr[g->seg_riv[s]];
        p->d_seg[0][k] = g->seg_length[s];
        p->d_seg[1][k] = g->seg_cwr[s];
    }
    L->seg_ele = p->l_sege.data();
    L->seg_riv = p->l_segr.data();
    L->seg_length = p->d_seg[0].data();
    L->seg_cwr = p->d_seg[1].data();
    const double *const *gsrc = (const double *const *)gp;          // ShudParamsSoA: 17 double pointers
    double const **ldst = (double const **)lp;
    static_assert(sizeof(ShudParamsSoA) == 17 * sizeof(const double *), "ShudParamsSoA layout");
    for (int f = 0; f < 17; f++) ldst[f] = gat1(gsrc[f], p->d_par[f]);
    return 0;
}

extern "C" int shud_plan_gather_ele(shud_plan_t p, const double *g, double *l) {
    if (!p || !g || !l) return perr(SHUD_ERR_ARG, "null argument");
    for (size_t k = 0; k < p->ele_gid.size(); k++) l[k] = g[p->ele_gid[k]];
    return 0;
}

extern "C" int shud_plan_gather_ele_i32(shud_plan_t p, const int32_t *g, int32_t *l) {
    if (!p || !g || !l) return perr(SHUD_ERR_ARG, "null argument");
    for (size_t k = 0; k < p->ele_gid.size(); k++) l[k] = g[p->ele_gid[k]];
    return 0;
}

extern "C" int shud_plan_owned_state(shud_plan_t p, const double *y, int32_t neg, double *o) {
    if (!p || !y || !o || neg != p->NEg) return perr(SHUD_ERR_ARG, "bad argument");
    const int no = p->n_own_ele, nro = p->n_own_riv;
    for (int b = 0; b < 3; b++)
        for (int k = 0; k < no; k++) o[(size_t)b * no + k] = y[(size_t)b * neg + p->ele_gid[k]];
    for (int k = 0; k < nro; k++) o[3 * (size_t)no + k] = y[3 * (size_t)neg + p->riv_gid[k]];
    for (size_t k = 0; k < p->lake_gid.size(); k++)
        o[3 * (size_t)no + nro + k] = y[3 * (size_t)neg + p->NRg + p->lake_gid[k]];
    return 0;
}

extern "C" int shud_plan_scatter_owned(shud_plan_t p, const double *o, int32_t neg, double *y) {
    if (!p || !y || !o || neg != p->NEg) return perr(SHUD_ERR_ARG, "bad argument");
    const int no = p->n_own_ele, nro = p->n_own_riv;
    for (int b = 0; b < 3; b++)
        for (int k = 0; k < no; k++) y[(size_t)b * neg + p->ele_gid[k]] = o[(size_t)b * no + k];
    for (int k = 0; k < nro; k++) y[3 * (size_t)neg + p->riv_gid[k]] = o[3 * (size_t)no + k];
    for (size_t k = 0; k < p->lake_gid.size(); k++)
        y[3 * (size_t)neg + p->NRg + p->lake_gid[k]] = o[3 * (size_t)no + nro + k];
    return 0;
}
