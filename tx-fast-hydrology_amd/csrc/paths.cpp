// Path plan of the one-step member sweep (paths.hpp): heavy-path decomposition of the routed
// forest, small light subtrees absorbed into the chain that consumes them, tasks in a
// topological ticket order.  Host integer work only.
#include "paths.hpp"

#include <algorithm>
#include <queue>
#include <sstream>

namespace mcr {

std::string build_path_plan(const Plan& P, PathPlan& out) {
    const int64_t n = P.n;
    out = PathPlan{};
    out.n = n;
    if (n == 0) {
        out.task_off.assign(1, 0);
        return "";
    }
    // consumers: every routed reach feeds at most one reach (its endnode), through that reach's
    // inflow list; unrouted reaches feed nobody (the reference never adds their outflow)
    std::vector<int64_t> cons(n, -1);
    for (int64_t j = 0; j < n; ++j)
        for (int64_t k = P.in_off[j]; k < P.in_off[j + 1]; ++k) cons[P.in_list[k]] = j;
    // topological order: routed reaches by rank (upstreams finalise first), then the unrouted
    std::vector<int64_t> topo;
    topo.reserve(n);
    {
        std::vector<int64_t> byrank(n, -1);
        int64_t nr = 0;
        for (int64_t j = 0; j < n; ++j)
            if (P.rank[j] >= 0) {
                byrank[P.rank[j]] = j;
                ++nr;
            }
        for (int64_t r = 0; r < nr; ++r) topo.push_back(byrank[r]);
        for (int64_t j = 0; j < n; ++j)
            if (P.rank[j] < 0) topo.push_back(j);
    }
    std::vector<int64_t> tpos(n);
    for (int64_t k = 0; k < n; ++k) tpos[topo[k]] = k;
    // subtree sizes, heights, heavy inputs
    std::vector<int64_t> sz(n, 1), hc(n, -1);
    std::vector<int32_t> hgt(n, 1);
    for (int64_t j : topo) {
        int64_t best = -1, bs = 0;
        for (int64_t k = P.in_off[j]; k < P.in_off[j + 1]; ++k) {
            const int64_t u = P.in_list[k];
            if (tpos[u] >= tpos[j]) return "internal: inflow list not in topological order";
            sz[j] += sz[u];
            hgt[j] = std::max(hgt[j], hgt[u] + 1);
            if (sz[u] > bs) {
                bs = sz[u];
                best = u;
            }
        }
        hc[j] = best;
    }
    for (int64_t j = 0; j < n; ++j) out.crit = std::max(out.crit, hgt[j]);
    // nodes downstream of each node, itself included (priority of the ticket order)
    std::vector<int64_t> down(n, 1);
    for (int64_t k = n - 1; k >= 0; --k) {
        const int64_t j = topo[k];
        if (cons[j] >= 0) down[j] = 1 + down[cons[j]];
    }

    // absorbed light inputs: per node, its light inputs taken in reverse rank order while the
    // ring distance of the earliest absorbed root stays below kPathRing (the node itself comes
    // right after its absorbed subtrees)
    std::vector<char> absorbed_root(n, 0);
    for (int64_t j = 0; j < n; ++j) {
        int64_t later = 0;                   // nodes of absorbed subtrees after the current one
        for (int64_t k = P.in_off[j + 1] - 1; k >= P.in_off[j]; --k) {
            const int64_t u = P.in_list[k];
            if (u == hc[j] || sz[u] > kPathAbsorb) continue;
            if (later + sz[u] + 1 >= kPathRing) continue;
            absorbed_root[u] = 1;
            later += sz[u];
        }
    }
    // task of every node; tasks are built from chain bottoms that are not inside an absorbed
    // subtree.  Sequence of a task: per chain node (upstream first): its absorbed subtrees (each
    // in topological order, the subtrees in rank order of their roots), then the node.
    std::vector<int32_t> task(n, -1);
    std::vector<std::vector<int64_t>> tseq;
    std::vector<char> is_chain(n, 0);
    std::vector<int64_t> stack, sub;
    auto emit_subtree = [&](int64_t u, int32_t t, std::vector<int64_t>& seq) {
        sub.clear();
        stack.assign(1, u);
        while (!stack.empty()) {
            const int64_t x = stack.back();
            stack.pop_back();
            sub.push_back(x);
            for (int64_t k = P.in_off[x]; k < P.in_off[x + 1]; ++k) stack.push_back(P.in_list[k]);
        }
        std::sort(sub.begin(), sub.end(), [&](int64_t a, int64_t b) { return tpos[a] < tpos[b]; });
        for (int64_t x : sub) {
            task[x] = t;
            seq.push_back(x);
        }
    };
    // an absorbed subtree's nodes are inside it: mark them so their chain bottoms make no tasks
    std::vector<char> inside(n, 0);
    for (int64_t k = n - 1; k >= 0; --k) {
        const int64_t j = topo[k];
        if (absorbed_root[j] || (cons[j] >= 0 && inside[cons[j]])) inside[j] = 1;
    }
    std::vector<int64_t> chain;
    for (int64_t k = n - 1; k >= 0; --k) {        // downstream first: any order of tasks works
        const int64_t b = topo[k];
        if (inside[b]) continue;
        if (cons[b] >= 0 && hc[cons[b]] == b) continue;   // not a chain bottom
        const int32_t t = (int32_t)tseq.size();
        tseq.emplace_back();
        std::vector<int64_t>& seq = tseq.back();
        chain.clear();
        for (int64_t v = b; v >= 0; v = hc[v]) chain.push_back(v);
        std::reverse(chain.begin(), chain.end());
        for (int64_t v : chain) {
            for (int64_t q = P.in_off[v]; q < P.in_off[v + 1]; ++q) {
                const int64_t u = P.in_list[q];
                if (u != hc[v] && absorbed_root[u]) emit_subtree(u, t, seq);
            }
            task[v] = t;
            is_chain[v] = 1;
            seq.push_back(v);
        }
    }
    for (int64_t j = 0; j < n; ++j)
        if (task[j] < 0) return "internal: a reach belongs to no path task";
    const int32_t nt = (int32_t)tseq.size();

    // ticket order: Kahn over the task graph (producer -> consumer), longest remaining path first
    std::vector<std::vector<int32_t>> succ(nt);
    std::vector<int32_t> pending(nt, 0);
    std::vector<int64_t> prio(nt, 0);
    for (int32_t t = 0; t < nt; ++t) {
        const int64_t b = tseq[t].back();
        const int64_t c = cons[b];
        prio[t] = (int64_t)tseq[t].size() + (c >= 0 ? down[c] : 0);
        if (c >= 0) {
            if (task[c] == t) return "internal: a task feeds itself";
            succ[t].push_back(task[c]);
            ++pending[task[c]];
        }
        for (size_t q = 0; q + 1 < tseq[t].size(); ++q) {
            const int64_t x = tseq[t][q];
            if (cons[x] >= 0 && task[cons[x]] != t)
                return "internal: a task's inner node feeds another task";
        }
    }
    std::priority_queue<std::pair<int64_t, int32_t>> ready;
    for (int32_t t = 0; t < nt; ++t)
        if (pending[t] == 0) ready.push({prio[t], -t});
    std::vector<int32_t> order;
    order.reserve(nt);
    while (!ready.empty()) {
        const int32_t t = -ready.top().second;
        ready.pop();
        order.push_back(t);
        for (int32_t c : succ[t])
            if (--pending[c] == 0) ready.push({prio[c], -c});
    }
    if ((int32_t)order.size() != nt) return "internal: the task graph has a cycle";
    std::vector<int32_t> newid(nt);
    for (int32_t k = 0; k < nt; ++k) newid[order[k]] = k;

    // sequence, records
    out.n_tasks = nt;
    out.task_off.assign(nt + 1, 0);
    out.seq_reach.reserve(n);
    std::vector<int64_t> seqpos(n, -1);
    for (int32_t k = 0; k < nt; ++k) {
        const auto& s = tseq[order[k]];
        out.task_off[k] = (int32_t)out.seq_reach.size();
        out.max_task = std::max(out.max_task, (int32_t)s.size());
        for (int64_t x : s) {
            seqpos[x] = (int64_t)out.seq_reach.size();
            out.seq_reach.push_back(x);
        }
    }
    out.task_off[nt] = (int32_t)n;
    if (n >= (int64_t)kInPayload) return "network too large for the path plan";
    out.rec.assign((size_t)n * kPathRecWords, 0);
    std::vector<char> keep(n, 0);
    std::vector<uint32_t> codes;
    for (int64_t s = 0; s < n; ++s) {
        const int64_t x = out.seq_reach[s];
        const int32_t t = newid[task[x]];
        codes.clear();
        for (int64_t k = P.in_off[x]; k < P.in_off[x + 1]; ++k) {
            const int64_t u = P.in_list[k];
            const int32_t tu = newid[task[u]];
            const int64_t su = seqpos[u];
            if (tu != t) {
                if (su != out.task_off[tu + 1] - 1) return "internal: input from a task's inner node";
                codes.push_back(kInExt | (uint32_t)tu);
                ++out.n_ext;
            } else if (is_chain[x] && u == hc[x]) {
                codes.push_back(kInChain);
            } else if (su == s - 1) {
                codes.push_back(kInPrev);
            } else {
                if (s - su >= kPathRing || su > s) {
                    std::ostringstream m;
                    m << "internal: ring distance " << (s - su) << " of reach " << u;
                    return m.str();
                }
                codes.push_back(kInLocal | (uint32_t)su);
                keep[su] = 1;
            }
        }
        int32_t* r = &out.rec[(size_t)s * kPathRecWords];
        r[1] = (int32_t)P.pos[x];
        r[0] = (int32_t)codes.size() | (P.rank[x] >= 0 ? (int32_t)kRecRouted : 0) |
               (is_chain[x] ? (int32_t)kRecChain : 0) |
               (s == out.task_off[t + 1] - 1 && cons[x] >= 0 ? (int32_t)kRecPublish : 0);
        if (codes.size() > 0xffff) return "a reach has more than 65535 upstream reaches";
        for (size_t q = 0; q < codes.size(); ++q) {
            if ((int)q < kPathInline) {
                r[4 + q] = (int32_t)codes[q];
            } else {
                if (q == kPathInline) r[4 + kPathInline] = (int32_t)out.ovf.size();
                out.ovf.push_back((int32_t)codes[q]);
            }
        }
    }
    for (int64_t s = 0; s < n; ++s)
        if (keep[s]) out.rec[(size_t)s * kPathRecWords] |= (int32_t)kRecKeep;
    return "";
}

}  // namespace mcr
