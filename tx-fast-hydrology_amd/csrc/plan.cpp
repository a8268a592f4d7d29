// Topology compiler: reference-walk replay, rank-ordered upstream lists, clustering, space-time
// schedule and workgroup packing.  See plan.hpp for the model.
#include "plan.hpp"

#include <algorithm>
#include <array>
#include <numeric>
#include <sstream>

namespace mcr {

namespace {

struct Cluster {
    int64_t root = -1;
    int64_t size = 0;
    int64_t ext = 0;        // cross-cluster inputs
    int64_t wg = -1;
    int32_t off = 0;        // G offset
    int32_t dmax = 0;       // deepest in-cluster distance to the root
    int64_t cnt[kMaxChain + 1] = {};   // lane chains by length
};

// Lanes of `chain` positions needed for chains of the given lengths (cnt[L] chains of length
// L), packed first-fit decreasing: the packing slot assignment (step 8) performs.
int64_t lanes_needed(const int64_t* c, int K) {
    switch (K) {
        case 1: return c[1];
        case 2: return c[2] + (c[1] + 1) / 2;
        case 3: return c[3] + c[2] + (std::max<int64_t>(0, c[1] - c[2]) + 2) / 3;
        default: {   // 4: a 3-chain leaves one free position, an odd 2-chain two
            const int64_t free1 = c[3] + (c[2] & 1) * 2;
            return c[4] + c[3] + (c[2] + 1) / 2 + (std::max<int64_t>(0, c[1] - free1) + 3) / 4;
        }
    }
}

int64_t lanes_sum(const int64_t* a, const int64_t* b, int K) {
    int64_t s[kMaxChain + 1];
    for (int L = 0; L <= kMaxChain; ++L) s[L] = a[L] + b[L];
    return lanes_needed(s, K);
}

}  // namespace

std::string build_plan(int64_t n, const int64_t* endnodes, const int64_t* indegree,
                       const int64_t* heads, int64_t n_heads, const PlanParams& params,
                       Plan& P) {
    P = Plan();
    P.n = n;
    P.p = params;
    const int64_t C = params.slots;
    const int32_t B = params.tile;
    if (n < 0) return "n must be >= 0";
    // fewer than 64 lanes: the member sweep's plans (sweep.hpp: a "lane" is a wave of members,
    // chain * slots node slots per workgroup); no lane-per-slot kernel runs them
    const bool member_plan = (C == 4 || C == 8 || C == 16 || C == 32) && C * params.chain <= 64;
    if (!member_plan && (C < 64 || C > 512 || (C % 64) != 0))
        return "slots must be a multiple of 64 in [64, 512]";
    if (B < 1 || B > 4096) return "tile must be in [1, 4096]";
    if (P.p.ext_cap < 1 || P.p.ext_cap > 0x7fff) return "ext_cap out of range";
    const int K = params.chain;
    if (K < 1 || K > kMaxChain) return "chain must be in [1, 4]";
    // hard cap of external inputs of the multi-launch kernel: what is left of its LDS after the
    // outflow double buffer (16 B) and forcing rows (24 B) of the chain * slots node slots and
    // the step-table window (kernels.hpp wavefront_lds_bytes; the dataflow kernel stages at most
    // kFlowMaxExt and checks max_ext_wg against it)
    {
        const int64_t left = kLdsBudget - 40 * (K * C + 1) - kTableEntryBytes * table_entries(C, B);
        const int64_t hard = std::min<int64_t>(left / (8 * (int64_t)B), 0x7fff);
        if (hard < 1) return "slots/tile too large for the 160 KiB LDS of a workgroup";
        P.ext_hard = (int32_t)hard;
        P.p.ext_cap = (int32_t)std::min<int64_t>(P.p.ext_cap, hard);
    }
    const int32_t soft = P.p.ext_cap;
    const int32_t hard = P.ext_hard;
    for (int64_t j = 0; j < n; ++j)
        if (endnodes[j] < 0 || endnodes[j] >= n) {
            std::ostringstream s;
            s << "endnodes[" << j << "] = " << endnodes[j] << " is out of range [0, " << n << ")";
            return s.str();
        }

    // ---- 1. replay the reference walk (nutils.py:72-88) -----------------------------------
    std::vector<int64_t> deg(indegree, indegree + n);
    P.rank.assign(n, -1);
    std::vector<int64_t> order;
    order.reserve(n);
    for (int64_t k = 0; k < n_heads; ++k) {
        int64_t s = heads[k];
        if (s < 0 || s >= n) {
            std::ostringstream m;
            m << "headwater index " << s << " out of range";
            return m.str();
        }
        while (deg[s] == 0) {
            if (P.rank[s] >= 0) {
                std::ostringstream m;
                m << "reach " << s << " would be processed twice in one step (duplicate or "
                  << "inconsistent headwater list / indegree)";
                return m.str();
            }
            P.rank[s] = (int64_t)order.size();
            order.push_back(s);
            const int64_t e = endnodes[s];
            deg[e] -= 1;
            s = e;
        }
    }
    P.n_routed = (int64_t)order.size();

    // ---- 2. rank-ordered upstream lists ---------------------------------------------------
    // contribution s -> e happens when s is processed (s routed, e != s).
    std::vector<int64_t> up_off(n + 1, 0);
    for (int64_t s : order)
        if (endnodes[s] != s) up_off[endnodes[s] + 1]++;
    for (int64_t j = 0; j < n; ++j) up_off[j + 1] += up_off[j];
    std::vector<int64_t> up_list(up_off[n]);
    {
        std::vector<int64_t> fill(up_off.begin(), up_off.end() - 1);
        for (int64_t s : order)  // rank order -> each list sorted by rank
            if (endnodes[s] != s) up_list[fill[endnodes[s]]++] = s;
    }
    P.in_off = up_off;   // kept: inflows are recomputed from outflows on the device
    P.in_list = up_list;
    for (int64_t s : order) {
        const int64_t e = endnodes[s];
        if (e != s && P.rank[e] >= 0 && P.rank[e] < P.rank[s]) {
            std::ostringstream m;
            m << "reach " << e << " is processed before its upstream reach " << s
              << " (indegree inconsistent with endnodes)";
            return m.str();
        }
    }
    // ---- 3. partial-sum nodes and heights -------------------------------------------------
    // A lane reads at most kUpInline upstream values per tick.  A reach with more routed
    // upstreams gets a left-deep chain of partial-sum nodes (ids n, n + 1, ...): a node outputs
    // ((0 + x1) + x2) + ... over at most kUpInline inputs, x1 possibly the previous partial sum.
    // Every value a lane publishes has the form 0 + (...) and is never -0.0, so 0 + prefix ==
    // prefix and the chain reproduces the reference's left fold bit for bit.  Where the chain is
    // cut is chosen per reach by a DP over the inputs' heights, so the deepest upstream enters
    // the fold as late as the rank order allows (usually no extra level on the critical path).
    std::vector<int32_t> h(n, 0);
    std::vector<int64_t> nodes;                 // topological compile order over all nodes
    nodes.reserve(n);
    std::vector<std::vector<int64_t>> vin;      // inputs of partial-sum node n + i
    std::vector<int64_t> rep_idx(n, -1);        // reaches whose input list was rewritten
    std::vector<std::vector<int64_t>> reps;
    {
        std::vector<int64_t> node_order(order);
        for (int64_t j = 0; j < n; ++j)
            if (P.rank[j] < 0) node_order.push_back(j);
        std::vector<int32_t> best;
        std::vector<int8_t> cut;
        std::vector<int64_t> chain;
        for (int64_t j : node_order) {
            const int64_t* u = up_list.data() + up_off[j];
            const int64_t k = up_off[j + 1] - up_off[j];
            int32_t hj = 0;
            if (k <= kUpInline) {
                for (int64_t q = 0; q < k; ++q) hj = std::max(hj, h[u[q]] + 1);
            } else {
                // best[p]: height of the value fold(u_1 .. u_p); cut[p]: how many raw inputs
                // the node of prefix p adds to fold(u_1 .. u_{p - cut[p]}) (0: one node over
                // u_1 .. u_p, only for p <= kUpInline); fold(u_1) is u_1 itself
                best.assign(k + 1, 0);
                cut.assign(k + 1, 0);
                best[1] = h[u[0]];
                int32_t pre = h[u[0]];
                for (int64_t p = 2; p <= k; ++p) {
                    pre = std::max(pre, h[u[p - 1]]);
                    if (p <= kUpInline) {
                        best[p] = pre + 1;
                        continue;
                    }
                    best[p] = INT32_MAX;
                    for (int s = kUpInline - 1; s >= 1; --s) {
                        int32_t m = best[p - s];
                        for (int64_t q = p - s; q < p; ++q) m = std::max(m, h[u[q]]);
                        if (m + 1 < best[p]) {
                            best[p] = m + 1;
                            cut[p] = (int8_t)s;
                        }
                    }
                }
                chain.clear();                 // prefixes that need a node, the reach first
                for (int64_t p = k;;) {
                    chain.push_back(p);
                    if (cut[p] == 0) break;
                    p -= cut[p];
                    if (p == 1) break;
                }
                int64_t prev = -1, plen = 1;   // value of the fold built so far (prefix plen)
                for (auto it = chain.rbegin(); it != chain.rend(); ++it) {
                    const int64_t p = *it;
                    const int64_t from = cut[p] == 0 ? 0 : p - cut[p];
                    std::vector<int64_t> x;
                    if (from > 0) {
                        if (from != plen) return "internal: partial-sum chain";
                        x.push_back(from == 1 ? u[0] : prev);
                    }
                    for (int64_t q = from; q < p; ++q) x.push_back(u[q]);
                    if ((int64_t)x.size() > kUpInline) return "internal: partial-sum fan-in";
                    int32_t hx = 0;
                    for (int64_t y : x) hx = std::max(hx, h[y] + 1);
                    if (p == k) {
                        hj = hx;
                        rep_idx[j] = (int64_t)reps.size();
                        reps.push_back(std::move(x));
                    } else {
                        prev = n + (int64_t)vin.size();
                        vin.push_back(std::move(x));
                        h.push_back(hx);
                        nodes.push_back(prev);
                    }
                    plen = p;
                }
            }
            h[j] = hj;
            nodes.push_back(j);
        }
    }
    const int64_t V = (int64_t)vin.size();
    const int64_t N = n + V;
    P.n_partial = V;
    // inputs of every node (CSR over [0, N)) and its consumer inside the schedule
    std::vector<int64_t> gin_off(N + 1, 0), gin_list;
    gin_list.reserve(up_list.size() + (size_t)V * kUpInline);
    for (int64_t x = 0; x < N; ++x) {
        if (x >= n)
            gin_list.insert(gin_list.end(), vin[x - n].begin(), vin[x - n].end());
        else if (rep_idx[x] >= 0)
            gin_list.insert(gin_list.end(), reps[rep_idx[x]].begin(), reps[rep_idx[x]].end());
        else
            gin_list.insert(gin_list.end(), up_list.begin() + up_off[x],
                            up_list.begin() + up_off[x + 1]);
        gin_off[x + 1] = (int64_t)gin_list.size();
    }
    std::vector<int64_t> cons(N, -1);
    for (int64_t x = 0; x < N; ++x)
        for (int64_t k = gin_off[x]; k < gin_off[x + 1]; ++k) cons[gin_list[k]] = x;
    for (int64_t x = 0; x < N; ++x) P.max_height = std::max(P.max_height, h[x]);

    // ---- 4. lane chains ----------------------------------------------------------------
    // A lane owns K = chain node slots (positions), computed in order within a tick.  A node at
    // position p >= 1 may consume the output of position p - 1 in the same tick (a chained
    // edge, no tick); every other input arrives from an earlier tick.  A run of up to K
    // consecutive nodes along a flow path therefore costs one tick (K = 2: fused lane pairs).
    // Only a node's LAST input in fold order may be chained: the device then folds the other
    // inputs (the chained code reads the zero slot) and adds the chained value last, which is
    // the reference's left fold bit for bit and needs no per-input selects (measured on the
    // Texas network: the same schedule length as chaining any input).
    // DP over the forest in topological order: F[x][k] = height (ticks) of x at position k of
    // its chain (k = 0: no chained input), fc[x][k] the chained input achieving it, bx = min
    // over k.  A node has one consumer, so it is chained into at most one node and the choices
    // of different consumers never conflict.
    std::vector<int32_t> F((size_t)N * K, INT32_MAX), bx(N, 0);
    std::vector<int64_t> fc((size_t)N * K, -1);
    for (int64_t x : nodes) {
        const int64_t k0 = gin_off[x], k1 = gin_off[x + 1];
        int32_t* Fx = &F[(size_t)x * K];
        int32_t s = 0;
        for (int64_t q = k0; q < k1; ++q) s = std::max(s, bx[gin_list[q]] + 1);
        Fx[0] = s;
        for (int k = 1; k < K && k1 > k0; ++k) {
            const int64_t c = gin_list[k1 - 1];
            int32_t m = F[(size_t)c * K + k - 1];
            if (m == INT32_MAX) continue;
            for (int64_t r = k0; r < k1 - 1; ++r) m = std::max(m, bx[gin_list[r]] + 1);
            if (m < Fx[k]) {
                Fx[k] = m;
                fc[(size_t)x * K + k] = c;
            }
        }
        int32_t b = Fx[0];
        for (int k = 1; k < K; ++k) b = std::min(b, Fx[k]);
        bx[x] = b;
    }
    // positions, downstream first: a node its consumer did not chain takes its best position
    // (the lowest on ties); below[x] = its chained input, above[x] = the node it is chained into
    std::vector<int8_t> cpos(N, -1);
    std::vector<int64_t> below(N, -1), above(N, -1), top(N, -1);
    for (auto it = nodes.rbegin(); it != nodes.rend(); ++it) {
        const int64_t x = *it;
        int k = cpos[x];
        if (k < 0) {
            const int32_t* Fx = &F[(size_t)x * K];
            k = 0;
            for (int j = 1; j < K; ++j)
                if (Fx[j] < Fx[k]) k = j;
            cpos[x] = (int8_t)k;
        }
        if (F[(size_t)x * K + k] == INT32_MAX) return "internal: lane chain position";
        if (k > 0) {
            const int64_t c = fc[(size_t)x * K + k];
            below[x] = c;
            above[c] = x;
            cpos[c] = (int8_t)(k - 1);
            P.n_pairs++;
        }
        top[x] = above[x] >= 0 ? top[above[x]] : x;
    }
    std::vector<int32_t>().swap(F);
    std::vector<int64_t>().swap(fc);
    // lane node of every node = the top (most downstream node) of its chain; a lane node's
    // inputs are the inputs of its chain members, bottom first, without the chained edges.
    // Every such input is itself the top of its chain (its one consumer did not chain it).
    auto lane_of = [&](int64_t x) { return top[x]; };
    std::vector<int64_t> lin_off(N + 1, 0), lin_list, chain_nodes;
    lin_list.reserve(gin_list.size());
    for (int64_t x = 0; x < N; ++x) {
        if (top[x] == x) {
            chain_nodes.clear();
            for (int64_t y = x; y >= 0; y = below[y]) chain_nodes.push_back(y);
            for (auto it = chain_nodes.rbegin(); it != chain_nodes.rend(); ++it)
                for (int64_t q = gin_off[*it]; q < gin_off[*it + 1]; ++q)
                    if (gin_list[q] != below[*it]) {
                        if (top[gin_list[q]] != gin_list[q]) return "internal: lane input";
                        lin_list.push_back(gin_list[q]);
                    }
        }
        lin_off[x + 1] = (int64_t)lin_list.size();
    }
    std::vector<int64_t> lnodes;            // lane nodes in topological order
    lnodes.reserve(N);
    for (int64_t x : nodes)
        if (top[x] == x) lnodes.push_back(x);
    auto lcons = [&](int64_t x) { return cons[x] < 0 ? -1 : lane_of(cons[x]); };
    auto weight = [&](int64_t x) -> int64_t { return (int64_t)cpos[x] + 1; };

    // ---- 5. clustering (bottom-up greedy) -------------------------------------------------
    // Each lane node starts a cluster that absorbs the clusters of its inputs while the lane
    // (`slots` lanes of K positions per workgroup) and external-input budgets allow.  The
    // deepest input is tried first; a shallow input whose value can arrive `tile` ticks late is
    // cut for free.
    const int64_t RS = (int64_t)K * C;
    const int64_t scap = span_cap(C);
    // cl: cluster (sync plans: wave cluster) of every lane node, grp: its group (the cluster
    // itself in classic plans); edges inside a cluster have unit slack, edges inside a group
    // between its wave clusters kWaveSlack, all others >= tile
    std::vector<int64_t> cl(N, -1), grp(N, -1);
    std::vector<int32_t> G(N, 0);
    // per workgroup: its lane bins (classic plans: one bin of `slots` lanes; sync plans: one per
    // wave), each a list of chain tops
    std::vector<std::vector<std::vector<int64_t>>> wg_bins;
    const int64_t bin_lanes = params.sync ? kWaveLanes : C;
    if (!params.sync) {
    std::vector<Cluster> clusters;
    std::vector<int32_t> eh(N, 0);          // critical-path estimate (ticks)
    std::vector<uint8_t> merged(N, 0);      // edge (x -> consumer) is inside a cluster
    std::vector<std::vector<int64_t>> members;
    std::vector<int64_t> ups;
    for (int64_t j : lnodes) {
        ups.assign(lin_list.begin() + lin_off[j], lin_list.begin() + lin_off[j + 1]);
        std::stable_sort(ups.begin(), ups.end(),
                         [&](int64_t a, int64_t b) { return eh[a] > eh[b]; });
        Cluster c;
        c.root = j;
        c.size = weight(j);
        c.cnt[weight(j)] = 1;
        std::vector<int64_t> absorb;
        int32_t best = ups.empty() ? -1 : eh[ups[0]];
        int32_t ehj = 0;
        bool first = true;
        for (int64_t u : ups) {
            const Cluster& cu = clusters[cl[u]];
            // merge the deepest input, any input a cut would delay, and any input once the
            // external-input budget is used up
            const bool want = first || (eh[u] + B > best + 1) || (c.ext + 1 > soft);
            first = false;
            // the cluster's tick span (in-cluster depth) must fit one workgroup's window
            if (want && lanes_sum(c.cnt, cu.cnt, K) <= C && c.ext + cu.ext <= hard &&
                cu.dmax + 1 <= scap) {
                c.size += cu.size;
                for (int L = 1; L <= kMaxChain; ++L) c.cnt[L] += cu.cnt[L];
                c.ext += cu.ext;
                c.dmax = std::max(c.dmax, cu.dmax + 1);
                absorb.push_back(cl[u]);
                merged[u] = 1;
                ehj = std::max(ehj, eh[u] + 1);
            } else {
                c.ext += 1;
                ehj = std::max(ehj, eh[u] + B);
            }
        }
        if (c.ext > hard) {
            // more external inputs than the LDS can stage: cannot be scheduled
            std::ostringstream m;
            m << "node " << j << " needs " << c.ext << " external inputs (LDS cap " << hard
              << " for slots=" << C << ", tile=" << B << ")";
            return m.str();
        }
        eh[j] = ehj;
        // merge small-to-large: the largest absorbed cluster keeps its id and member list
        int64_t id;
        if (absorb.empty()) {
            id = (int64_t)clusters.size();
            clusters.push_back(c);
            members.emplace_back();
        } else {
            id = absorb[0];
            for (int64_t a : absorb)
                if (clusters[a].size > clusters[id].size) id = a;
            for (int64_t a : absorb) {
                if (a == id) continue;
                for (int64_t v : members[a]) {
                    cl[v] = id;
                    members[id].push_back(v);
                }
                std::vector<int64_t>().swap(members[a]);
                clusters[a].size = 0;  // dead
            }
            clusters[id] = c;
        }
        members[id].push_back(j);
        cl[j] = id;
    }

    // ---- 6. schedule: local ALAP skew + cluster offsets -----------------------------------
    // distance to the cluster root: walk lane nodes in reverse (downstream first)
    std::vector<int32_t> dist(N, 0);
    for (Cluster& c : clusters) c.dmax = 0;      // recomputed exactly from the final clusters
    for (auto it = lnodes.rbegin(); it != lnodes.rend(); ++it) {
        const int64_t j = *it;
        const int64_t e = lcons(j);
        dist[j] = (e >= 0 && merged[j]) ? dist[e] + 1 : 0;
        Cluster& c = clusters[cl[j]];
        c.dmax = std::max(c.dmax, dist[j]);
    }
    // live clusters in root order (roots appear in `lnodes` order)
    std::vector<int64_t> live;
    for (int64_t j : lnodes)
        if (clusters[cl[j]].root == j) live.push_back(cl[j]);
    P.n_clusters = (int64_t)live.size();
    for (int64_t id : live) {
        Cluster& c = clusters[id];
        int64_t off = 0;
        for (int64_t v : members[id]) {
            const int32_t s = c.dmax - dist[v];
            for (int64_t k = lin_off[v]; k < lin_off[v + 1]; ++k) {
                const int64_t u = lin_list[k];
                if (cl[u] != id) off = std::max<int64_t>(off, (int64_t)G[u] + B - s);
            }
        }
        if (off > (int64_t)1 << 30) return "schedule overflow (network too deep)";
        c.off = (int32_t)off;
        for (int64_t v : members[id]) G[v] = c.off + c.dmax - dist[v];
    }

    // ---- 7. pack clusters into workgroups --------------------------------------------------
    // First fit in order of schedule offset, so a workgroup holds clusters that are active at
    // the same ticks; its G span is capped so the step-table window fits the LDS.
    std::vector<int64_t> by_off(live);
    std::stable_sort(by_off.begin(), by_off.end(), [&](int64_t a, int64_t b) {
        return clusters[a].off < clusters[b].off;
    });
    std::vector<int64_t> wg_fill, wg_ext, bin_lo, bin_hi;
    std::vector<std::array<int64_t, kMaxChain + 1>> wg_cnt;
    const int kProbe = 64;  // bounded first fit over the most recent bins keeps packing O(n)
    for (int64_t id : by_off) {
        Cluster& c = clusters[id];
        const int64_t lo = c.off, hi = (int64_t)c.off + c.dmax;
        int64_t w = -1;
        const int64_t nb = (int64_t)wg_fill.size();
        for (int64_t b = std::max<int64_t>(0, nb - kProbe); b < nb; ++b)
            if (lanes_sum(wg_cnt[b].data(), c.cnt, K) <= C &&
                wg_ext[b] + c.ext <= std::max<int64_t>(soft, c.ext) &&
                std::max(bin_hi[b], hi) - std::min(bin_lo[b], lo) <= scap) {
                w = b;
                break;
            }
        if (w < 0) {
            w = nb;
            wg_fill.push_back(0);
            wg_ext.push_back(0);
            wg_cnt.push_back({});
            bin_lo.push_back(lo);
            bin_hi.push_back(hi);
        }
        wg_fill[w] += c.size;
        wg_ext[w] += c.ext;
        for (int L = 1; L <= kMaxChain; ++L) wg_cnt[w][L] += c.cnt[L];
        bin_lo[w] = std::min(bin_lo[w], lo);
        bin_hi[w] = std::max(bin_hi[w], hi);
        c.wg = w;
    }
    P.nwg = (int32_t)wg_fill.size();
    wg_bins.assign(P.nwg, std::vector<std::vector<int64_t>>(1));
    for (int64_t id : live)
        for (int64_t v : members[id]) wg_bins[clusters[id].wg][0].push_back(v);
    for (int64_t x = 0; x < N; ++x) grp[x] = cl[x];
    } else {
    // ---- 5s. two-level clustering (sync plans) ---------------------------------------------
    // Same greedy as step 5, one level down: each lane node starts a wave cluster inside a new
    // group; for each input (deepest first) it tries (a) to absorb the input's wave cluster
    // (unit slack: one wave's lanes, the group's waves still pack into the workgroup), then
    // (b) to absorb the input's group over a local edge (slack kWaveSlack), else (c) cuts it
    // (slack tile, granules).  Inputs a cut would not delay are cut.
    const int W = (int)(C / kWaveLanes);
    if (W < 1 || W > 8 || C % kWaveLanes) return "sync plans need slots = 64 .. 512 lanes";
    const int64_t hardx = std::min<int64_t>(hard, 128);   // kFlowMaxExt (kernels.hpp)
    struct WaveCl {
        int64_t cnt[kMaxChain + 1] = {};
        int64_t grp = -1;
        std::vector<int64_t> mem;        // lane nodes
    };
    struct Group {
        std::vector<int64_t> waves;
        int64_t ext = 0, nloc = 0, root = -1, wg = -1;
        int32_t dmax = 0, off = 0;
        bool dead = false;
    };
    std::vector<WaveCl> wcl;
    std::vector<Group> grps;
    std::vector<int32_t> eh(N, 0);
    std::vector<int8_t> eslack(N, 0);   // slack of the edge x -> consumer inside its group
    std::vector<int64_t> ups, lanes_tmp;
    auto wave_lanes = [&](int64_t w) { return lanes_needed(wcl[w].cnt, K); };
    // first-fit decreasing of wave clusters (lane counts) into W waves of kWaveLanes
    auto ffd_fits = [&](std::vector<int64_t>& l) {
        std::sort(l.begin(), l.end(), std::greater<int64_t>());
        int64_t bins[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        for (int64_t x : l) {
            int b = 0;
            while (b < W && bins[b] + x > kWaveLanes) ++b;
            if (b == W) return false;
            bins[b] += x;
        }
        return true;
    };
    for (int64_t j : lnodes) {
        ups.assign(lin_list.begin() + lin_off[j], lin_list.begin() + lin_off[j + 1]);
        std::stable_sort(ups.begin(), ups.end(),
                         [&](int64_t a, int64_t b) { return eh[a] > eh[b]; });
        const int64_t wj = (int64_t)wcl.size();
        wcl.emplace_back();
        wcl[wj].cnt[weight(j)] = 1;
        wcl[wj].mem.push_back(j);
        const int64_t gj = (int64_t)grps.size();
        grps.emplace_back();
        grps[gj].waves.push_back(wj);
        grps[gj].root = j;
        wcl[wj].grp = gj;
        cl[j] = wj;
        const int32_t best = ups.empty() ? -1 : eh[ups[0]];
        int32_t ehj = 0;
        bool first = true;
        for (int64_t u : ups) {
            const int64_t wu = cl[u], gu = wcl[wu].grp;
            Group& A = grps[gj];
            Group& Bg = grps[gu];
            const int64_t xe = A.ext + A.nloc + Bg.ext + Bg.nloc;
            const bool want = first || (eh[u] + B > best + 1) || (A.ext + A.nloc + 1 > soft);
            first = false;
            bool done = false;
            if (want && xe <= hardx && Bg.dmax + 1 <= scap) {
                // (a) unit slack: u's wave cluster joins j's
                int64_t mc[kMaxChain + 1];
                for (int L = 0; L <= kMaxChain; ++L) mc[L] = wcl[wj].cnt[L] + wcl[wu].cnt[L];
                const int64_t lw = lanes_needed(mc, K);
                if (lw <= kWaveLanes) {
                    lanes_tmp.clear();
                    lanes_tmp.push_back(lw);
                    for (int64_t w : A.waves) if (w != wj) lanes_tmp.push_back(wave_lanes(w));
                    for (int64_t w : Bg.waves) if (w != wu) lanes_tmp.push_back(wave_lanes(w));
                    if (ffd_fits(lanes_tmp)) {
                        for (int L = 0; L <= kMaxChain; ++L) wcl[wj].cnt[L] = mc[L];
                        for (int64_t v : wcl[wu].mem) {
                            cl[v] = wj;
                            wcl[wj].mem.push_back(v);
                        }
                        std::vector<int64_t>().swap(wcl[wu].mem);
                        for (int64_t w : Bg.waves)
                            if (w != wu) {
                                A.waves.push_back(w);
                                wcl[w].grp = gj;
                            }
                        A.ext += Bg.ext;
                        A.nloc += Bg.nloc;
                        A.dmax = std::max(A.dmax, Bg.dmax + 1);
                        Bg.dead = true;
                        eslack[u] = 1;
                        ehj = std::max(ehj, eh[u] + 1);
                        done = true;
                    }
                }
            }
            if (!done && want && xe + 1 <= hardx && Bg.dmax + kWaveSlack <= scap &&
                eh[u] + kWaveSlack < eh[u] + B) {
                // (b) local edge: u's group joins j's, its wave clusters unchanged
                lanes_tmp.clear();
                for (int64_t w : A.waves) lanes_tmp.push_back(wave_lanes(w));
                for (int64_t w : Bg.waves) lanes_tmp.push_back(wave_lanes(w));
                if (ffd_fits(lanes_tmp)) {
                    for (int64_t w : Bg.waves) {
                        A.waves.push_back(w);
                        wcl[w].grp = gj;
                    }
                    A.ext += Bg.ext;
                    A.nloc += Bg.nloc + 1;
                    A.dmax = std::max(A.dmax, Bg.dmax + kWaveSlack);
                    Bg.dead = true;
                    eslack[u] = kWaveSlack;
                    ehj = std::max(ehj, eh[u] + kWaveSlack);
                    done = true;
                }
            }
            if (!done) {
                grps[gj].ext += 1;
                ehj = std::max(ehj, eh[u] + B);
            }
        }
        if (grps[gj].ext + grps[gj].nloc > hardx) {
            std::ostringstream m;
            m << "node " << j << " needs " << grps[gj].ext + grps[gj].nloc
              << " external inputs (cap " << hardx << ")";
            return m.str();
        }
        eh[j] = ehj;
    }
    // ---- 6s. schedule: distances inside groups (unit / kWaveSlack edges), group offsets -----
    std::vector<int32_t> dist(N, 0);
    for (auto it = lnodes.rbegin(); it != lnodes.rend(); ++it) {
        const int64_t j = *it;
        const int64_t e = lcons(j);
        dist[j] = (e >= 0 && eslack[j]) ? dist[e] + eslack[j] : 0;
        grp[j] = wcl[cl[j]].grp;
    }
    std::vector<int64_t> live;                   // live groups in root order
    for (int64_t j : lnodes)
        if (grps[grp[j]].root == j) live.push_back(grp[j]);
    P.n_clusters = (int64_t)live.size();
    for (int64_t id : live) {
        Group& g = grps[id];
        g.dmax = 0;
        for (int64_t w : g.waves)
            for (int64_t v : wcl[w].mem) g.dmax = std::max(g.dmax, dist[v]);
        int64_t off = 0;
        for (int64_t w : g.waves)
            for (int64_t v : wcl[w].mem) {
                const int32_t s = g.dmax - dist[v];
                for (int64_t k = lin_off[v]; k < lin_off[v + 1]; ++k) {
                    const int64_t u = lin_list[k];
                    if (grp[u] != id) off = std::max<int64_t>(off, (int64_t)G[u] + B - s);
                }
            }
        if (off > (int64_t)1 << 30) return "schedule overflow (network too deep)";
        g.off = (int32_t)off;
        for (int64_t w : g.waves)
            for (int64_t v : wcl[w].mem) G[v] = g.off + g.dmax - dist[v];
    }
    // ---- 7s. pack groups into workgroups: first fit by offset; a group's wave clusters go to
    // the workgroup's W waves first-fit decreasing (a wave may hold several wave clusters)
    std::vector<int64_t> by_off(live);
    std::stable_sort(by_off.begin(), by_off.end(),
                     [&](int64_t a, int64_t b) { return grps[a].off < grps[b].off; });
    struct Bin { int64_t cnt[kMaxChain + 1] = {}; };
    struct Wg {
        std::vector<Bin> bins;
        int64_t xe = 0, lo = 0, hi = 0;
        std::vector<int64_t> groups;
        bool dead = false;
    };
    std::vector<Wg> wgs;
    std::vector<std::vector<int>> gat(grps.size());       // wave of each of a group's waves
    auto sorted_waves = [&](int64_t id) {
        std::vector<int64_t> ws(grps[id].waves);
        std::stable_sort(ws.begin(), ws.end(), [&](int64_t a, int64_t b) {
            return wave_lanes(a) > wave_lanes(b);
        });
        grps[id].waves = ws;
    };
    // place group id into workgroup b (best fit of its wave clusters on b's waves); returns the
    // lanes b then uses, or -1 when it does not fit.  commit = false only tests.
    auto place_group = [&](int64_t id, int64_t b, bool commit) -> int64_t {
        const Group& g = grps[id];
        Wg& x = wgs[b];
        if (x.dead) return -1;
        const int64_t lo = g.off, hi = (int64_t)g.off + g.dmax;
        if (x.xe + g.ext + g.nloc > std::max<int64_t>(soft, g.ext + g.nloc)) return -1;
        if (!x.groups.empty() && std::max(x.hi, hi) - std::min(x.lo, lo) > scap) return -1;
        std::vector<Bin> tmp(x.bins);
        std::vector<int> at(g.waves.size(), -1);
        for (size_t q = 0; q < g.waves.size(); ++q) {
            int64_t bestl = -1;                          // best fit: the fullest wave it fits
            for (int v = 0; v < W; ++v) {
                int64_t c2[kMaxChain + 1];
                for (int L = 0; L <= kMaxChain; ++L) c2[L] = tmp[v].cnt[L] + wcl[g.waves[q]].cnt[L];
                const int64_t l2 = lanes_needed(c2, K);
                if (l2 <= kWaveLanes && l2 > bestl) {
                    bestl = l2;
                    at[q] = v;
                }
            }
            if (at[q] < 0) return -1;
            for (int L = 0; L <= kMaxChain; ++L) tmp[at[q]].cnt[L] += wcl[g.waves[q]].cnt[L];
        }
        int64_t used = 0;
        for (int v = 0; v < W; ++v) used += lanes_needed(tmp[v].cnt, K);
        if (commit) {
            x.lo = x.groups.empty() ? lo : std::min(x.lo, lo);
            x.hi = x.groups.empty() ? hi : std::max(x.hi, hi);
            x.bins = tmp;
            x.xe += g.ext + g.nloc;
            x.groups.push_back(id);
            gat[id] = at;
            grps[id].wg = b;
        }
        return used;
    };
    const int kProbe = 64;   // bounded first fit over the most recent workgroups keeps it O(n)
    for (int64_t id : by_off) {
        sorted_waves(id);
        int64_t w = -1, wfill = -1;
        const int64_t nb = (int64_t)wgs.size();
        for (int64_t b = std::max<int64_t>(0, nb - kProbe); b < nb; ++b) {
            const int64_t f = place_group(id, b, false);
            if (f > wfill) {                           // best fit over the probed workgroups
                w = b;
                wfill = f;
            }
        }
        if (w < 0) {
            w = nb;
            wgs.emplace_back();
            wgs[w].bins.assign(W, Bin());
        }
        if (place_group(id, w, true) < 0) return "internal: group does not fit a workgroup";
    }
    // repair: dissolve the emptiest workgroups into the others where every group of one finds
    // room (fragmentation at wave granularity costs ~2 % of the lanes; the dataflow kernel needs
    // every workgroup resident)
    {
        std::vector<int64_t> order(wgs.size());
        std::iota(order.begin(), order.end(), 0);
        auto lanes_of = [&](const Wg& x) {
            int64_t u = 0;
            for (const Bin& bn : x.bins) u += lanes_needed(bn.cnt, K);
            return u;
        };
        std::stable_sort(order.begin(), order.end(), [&](int64_t a, int64_t b) {
            return lanes_of(wgs[a]) < lanes_of(wgs[b]);
        });
        for (int64_t w : order) {
            if (wgs[w].dead || wgs[w].groups.empty()) continue;
            const std::vector<Wg> save(wgs);
            const std::vector<std::vector<int>> save_at(gat);
            std::vector<int64_t> gs(wgs[w].groups);
            std::vector<int64_t> gwg(gs.size());
            for (size_t q = 0; q < gs.size(); ++q) gwg[q] = grps[gs[q]].wg;
            wgs[w].dead = true;
            bool ok = true;
            for (int64_t id : gs) {
                int64_t bestb = -1, bf = -1;
                for (int64_t b = 0; b < (int64_t)wgs.size(); ++b) {
                    const int64_t f = place_group(id, b, false);
                    if (f > bf) {
                        bf = f;
                        bestb = b;
                    }
                }
                if (bestb < 0) {
                    ok = false;
                    break;
                }
                place_group(id, bestb, true);
            }
            if (!ok) {
                wgs = save;
                gat = save_at;
                for (size_t q = 0; q < gs.size(); ++q) grps[gs[q]].wg = gwg[q];
                for (int64_t b = 0; b < (int64_t)wgs.size(); ++b)
                    for (int64_t id : wgs[b].groups) grps[id].wg = b;
            }
        }
    }
    // compact: live workgroups in creation order
    std::vector<int64_t> wid(wgs.size(), -1);
    int32_t nw = 0;
    for (size_t b = 0; b < wgs.size(); ++b)
        if (!wgs[b].dead && !wgs[b].groups.empty()) wid[b] = nw++;
    P.nwg = nw;
    wg_bins.assign(P.nwg, std::vector<std::vector<int64_t>>(W));
    for (size_t b = 0; b < wgs.size(); ++b) {
        if (wid[b] < 0) continue;
        for (int64_t id : wgs[b].groups)
            for (size_t q = 0; q < grps[id].waves.size(); ++q)
                for (int64_t v : wcl[grps[id].waves[q]].mem)
                    wg_bins[wid[b]][gat[id][q]].push_back(v);
    }
    }
    P.nslots = (int64_t)P.nwg * RS;
    for (int64_t x = 0; x < N; ++x) {
        if (top[x] != x) {
            G[x] = G[top[x]];
            cl[x] = cl[top[x]];
            grp[x] = grp[top[x]];
        }
        P.gmax = std::max(P.gmax, G[x]);
    }

    // ---- 8. slot assignment ----------------------------------------------------------------
    // node slot of a workgroup: position * slots + lane.  The chains of each lane bin (the
    // workgroup, or one wave of it in sync plans) are packed into lanes first-fit decreasing
    // (longest first, best fit on the free positions: the packing lanes_needed counts), a chain
    // on consecutive positions bottom first; lanes are then ordered by their earliest G, so a
    // wave holds nodes that are active at the same ticks.
    P.slot_reach.assign(P.nslots, -1);
    P.G.assign(P.nslots, 0);
    P.flags.assign(P.nslots, kSlotPad);
    P.up_cnt.assign(P.nslots, 0);
    P.up4.assign(P.nslots, 0);
    P.pos.assign(n, -1);
    std::vector<int64_t> npos(N, -1);       // node -> slot
    P.wg_gmin.assign(P.nwg, 0);
    P.wg_gmax.assign(P.nwg, 0);
    auto place = [&](int64_t x, int64_t d) {
        npos[x] = d;
        P.G[d] = G[x];
        if (x < n) {
            P.slot_reach[d] = x;
            P.pos[x] = d;
            P.flags[d] = P.rank[x] >= 0 ? kSlotRouted : kSlotUnrouted;
        } else {
            P.flags[d] = kSlotSum;
        }
    };
    std::vector<std::vector<int64_t>> lanes;         // nodes of each lane, position order
    std::vector<int64_t> open[kMaxChain];            // lanes with f free positions
    std::vector<int64_t> lane_order;
    for (int32_t w = 0; w < P.nwg; ++w) {
      for (size_t bi = 0; bi < wg_bins[w].size(); ++bi) {
        auto& ch = wg_bins[w][bi];
        std::stable_sort(ch.begin(), ch.end(), [&](int64_t a, int64_t b) {
            return weight(a) != weight(b) ? weight(a) > weight(b) : G[a] < G[b];
        });
        lanes.clear();
        for (auto& o : open) o.clear();
        for (int64_t t : ch) {
            const int L = (int)weight(t);
            int64_t ln = -1;
            for (int f = L; f < K && ln < 0; ++f)
                if (!open[f].empty()) {
                    ln = open[f].back();
                    open[f].pop_back();
                }
            if (ln < 0) {
                ln = (int64_t)lanes.size();
                lanes.emplace_back();
            }
            const size_t at = lanes[ln].size();
            for (int64_t y = t; y >= 0; y = below[y]) lanes[ln].push_back(y);
            std::reverse(lanes[ln].begin() + at, lanes[ln].end());   // bottom first
            const int f = K - (int)lanes[ln].size();
            if (f > 0) open[f].push_back(ln);
        }
        if ((int64_t)lanes.size() > bin_lanes) return "internal: workgroup overfull";
        lane_order.resize(lanes.size());
        std::vector<int32_t> lane_g(lanes.size(), INT32_MAX);
        for (size_t l = 0; l < lanes.size(); ++l) {
            lane_order[l] = (int64_t)l;
            for (int64_t x : lanes[l]) lane_g[l] = std::min(lane_g[l], G[x]);
        }
        std::stable_sort(lane_order.begin(), lane_order.end(),
                         [&](int64_t a, int64_t b) { return lane_g[a] < lane_g[b]; });
        const int64_t base = (int64_t)w * RS + (int64_t)bi * bin_lanes;
        for (size_t l = 0; l < lane_order.size(); ++l) {
            const auto& nodes_l = lanes[lane_order[l]];
            for (size_t p = 0; p < nodes_l.size(); ++p)
                place(nodes_l[p], base + (int64_t)p * C + (int64_t)l);
        }
      }
        const int64_t base = (int64_t)w * RS;
        int32_t lo = INT32_MAX, hi = INT32_MIN;
        for (int64_t d = base; d < base + RS; ++d)
            if (P.flags[d] != kSlotPad) {
                lo = std::min(lo, P.G[d]);
                hi = std::max(hi, P.G[d]);
            }
        P.wg_gmin[w] = lo == INT32_MAX ? 0 : lo;
        P.wg_gmax[w] = lo == INT32_MAX ? 0 : hi;
        P.max_span = std::max(P.max_span, P.wg_gmax[w] - P.wg_gmin[w]);
        if ((int64_t)P.wg_gmax[w] - P.wg_gmin[w] > scap) return "internal: workgroup G span";
    }
    // input codes and external lists
    P.ext_off.assign(P.nwg + 1, 0);
    std::vector<std::vector<std::pair<int64_t, int32_t>>> ext(P.nwg);  // (src node, consumer G)
    std::vector<std::vector<int64_t>> loc(P.nwg);                       // local edges' sources
    struct LocRef { int64_t d; int k; int32_t li; };
    std::vector<LocRef> loc_ref;
    std::vector<int64_t> node_at(P.nslots, -1);
    for (int64_t x = 0; x < N; ++x) node_at[npos[x]] = x;
    for (int64_t d = 0; d < P.nslots; ++d) {
        const int64_t j = node_at[d];
        if (j < 0) continue;
        const int32_t w = (int32_t)(d / RS);
        const int64_t k0 = gin_off[j], k1 = gin_off[j + 1];
        if (k1 - k0 > kUpInline) return "internal: more than kUpInline inputs";
        P.up_cnt[d] = (uint8_t)(k1 - k0);
        uint64_t packed = 0;
        for (int64_t k = k0; k < k1; ++k) {
            const int64_t u = gin_list[k];
            uint16_t code;
            if (u == below[j]) {
                if (npos[u] != d - C || G[u] != G[j]) return "internal: lane chain layout";
                if (k != k1 - 1) return "internal: chained input is not the last input";
                code = kSelfCode;
            } else if (cl[u] == cl[j]) {
                if (G[j] != G[u] + 1) return "internal: in-cluster edge without unit slack";
                code = (uint16_t)(npos[u] - (int64_t)w * RS);
                if (P.p.sync && (npos[u] % RS) % C / kWaveLanes != (d % RS) % C / kWaveLanes)
                    return "internal: unit-slack edge across waves";
            } else if (grp[u] == grp[j]) {
                // local edge of a sync plan: column (granule inputs of w) + index, patched below
                if (G[j] != G[u] + kWaveSlack) return "internal: local edge without its slack";
                if (npos[u] / RS != w) return "internal: local edge across workgroups";
                loc[w].push_back(u);
                loc_ref.push_back({d, (int)(k - k0), (int32_t)(loc[w].size() - 1)});
                code = 0;
                P.n_local++;
            } else {
                if (G[j] < G[u] + B) return "internal: cross-cluster edge without tile slack";
                const size_t e = ext[w].size();
                if (e >= (size_t)hard) return "internal: external-input cap exceeded";
                ext[w].push_back({u, G[j]});
                code = (uint16_t)(kExtBit | e);
                P.n_cross++;
            }
            packed |= (uint64_t)code << (16 * (k - k0));
        }
        P.up4[d] = packed;
    }
    // each node has one consumer, so it feeds at most one external input; ext_src names the
    // source's row of the output arrays: the reach, or n + slot for a partial-sum node
    P.xid.assign(P.nslots, -1);
    P.lx.assign(P.nslots, -1);
    P.lx_off.assign(P.nwg + 1, 0);
    for (const LocRef& r : loc_ref) {
        const int32_t w = (int32_t)(r.d / RS);
        const int64_t e = (int64_t)ext[w].size() + r.li;
        if (e >= 0x7fff) return "internal: local input index";
        P.up4[r.d] |= (uint64_t)(kExtBit | (uint16_t)e) << (16 * r.k);
    }
    for (int32_t w = 0; w < P.nwg; ++w) {
        P.lx_off[w + 1] = P.lx_off[w] + (int32_t)loc[w].size();
        const int64_t xe = (int64_t)ext[w].size() + (int64_t)loc[w].size();
        if (xe > hard) return "internal: external-input cap exceeded";
        P.max_xe_wg = std::max(P.max_xe_wg, (int32_t)xe);
        for (size_t li = 0; li < loc[w].size(); ++li) {
            const int64_t src = npos[loc[w][li]];
            if (P.lx[src] != -1 || P.xid[src] != -1) return "internal: node feeds two inputs";
            P.lx[src] = (int16_t)(ext[w].size() + li);
            P.lx_src.push_back((int32_t)src);
        }
        P.ext_off[w + 1] = P.ext_off[w] + (int32_t)ext[w].size();
        P.max_ext_wg = std::max(P.max_ext_wg, (int32_t)ext[w].size());
        for (auto& pr : ext[w]) {
            const int64_t src = npos[pr.first];
            if (P.xid[src] != -1) return "internal: node feeds two external inputs";
            P.xid[src] = (int32_t)P.ext_src.size();
            P.ext_src.push_back(pr.first < n ? pr.first : n + src);
            P.ext_g.push_back(pr.second);
        }
    }
    return std::string();
}

int64_t active_schedule(const Plan& P, int64_t T, std::vector<int32_t>& list,
                        std::vector<int64_t>& off) {
    list.clear();
    off.assign(1, 0);
    if (T <= 0 || P.nwg == 0) return 0;
    const int64_t B = P.p.tile;
    const int64_t ticks = (int64_t)P.gmax + T;
    const int64_t nl = (ticks + B - 1) / B;
    // bucket each workgroup into the launches its window [gmin, gmax + T) overlaps
    std::vector<int64_t> cnt(nl + 1, 0);
    for (int32_t w = 0; w < P.nwg; ++w) {
        const int64_t a = P.wg_gmin[w] / B;
        const int64_t b = ((int64_t)P.wg_gmax[w] + T - 1) / B;
        for (int64_t k = a; k <= b && k < nl; ++k) cnt[k + 1]++;
    }
    for (int64_t k = 0; k < nl; ++k) cnt[k + 1] += cnt[k];
    off = cnt;
    list.assign(off[nl], 0);
    std::vector<int64_t> fill(off.begin(), off.end() - 1);
    for (int32_t w = 0; w < P.nwg; ++w) {
        const int64_t a = P.wg_gmin[w] / B;
        const int64_t b = ((int64_t)P.wg_gmax[w] + T - 1) / B;
        for (int64_t k = a; k <= b && k < nl; ++k) list[fill[k]++] = w;
    }
    return nl;
}

}  // namespace mcr
