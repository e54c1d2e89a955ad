/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * Restatement of the reference's small-buffer allreduce path: the tree that
 * TryAllreduceTree folds over (src/comm/communicator_collective.cc:6-13,14-43,
 * 71-78).  The fold order of that path is the iteration order of libstdc++
 * std::unordered_set / std::unordered_map containers the reference fills in a
 * particular sequence, so this file reproduces the SAME container operations
 * in the SAME sequence with the same libstdc++ (g++ 11 in this image and on
 * the GPU box) — it is not a copy of the reference's code, and compiling the
 * reference's own .cc files was refused.
 *
 * Steps restated (reference file:line):
 *  1. heap tree over ranks 0..n-1: neighbours of r are [parent (r+1)/2-1 if
 *     r>0, child 2r+1, child 2r+2] in that order; parent map r -> (r+1)/2-1
 *     (src/utils/topo.cc:3-30, maps filled for r = 0..n-1 in order);
 *  2. the ring list: DFS from 0, each node followed by the rings of its
 *     non-parent neighbours in order, the LAST child's list reversed
 *     (topo.cc:32-62); ring position of rank k = its index in that list
 *     (topo.cc:64-94: rmap walks ring_map's "next" from 0);
 *  3. the relabelled tree map: for every (key, neighbour-vector) of the heap
 *     tree map in ITS iteration order, append rmap[x] to _tree_map[rmap[key]]
 *     (topo.cc:95-106);
 *  4. Communicator::BuildTopology (src/comm/communicator_base.cc:113-150): a
 *     copy of that map is walked in iteration order, every (key, neighbour)
 *     becomes an edge; UndirectedGraph::_BuildAdjacentList
 *     (include/utils/graph.h:70-83) inserts `to` into adj[from] and — the
 *     reference's quirk — `to` (not `from`) into adj[to];
 *  5. TryReduceTree (communicator_collective.cc:14-43) with root 0: BFS
 *     distances (graph.h:45-67), then rank r's children are the neighbours
 *     one level further from the root, inserted in adj[r]'s iteration order
 *     into a fresh unordered_set `recv_from_nodes`, whose iteration order is
 *     the order r receives and folds them: own = OP(own, child's subtree)
 *     (reducer(src=received, dst=sendrecvbuf), :28-33).
 * The root then holds the reduction; every rank receives the root's bits
 * (TryBroadcast, :44-69 — whose stale forwarding for n >= 4, SURVEY finding
 * 6, is not reproduced: see DESIGN.md §6).
 */
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <queue>
#include <unordered_map>
#include <unordered_set>
#include <vector>

extern "C" int rdc_oracle_reducer(const void* src, void* dst, uint64_t len, int dtype, int op);
extern "C" size_t rdc_oracle_dtype_size(int dtype);

namespace {

typedef std::unordered_map<int, std::vector<int>> AdjVec;
typedef std::unordered_map<int, int> IntMap;

// step 1
void heap_tree(int n, AdjVec* tree, IntMap* parent) {
    for (int r = 0; r < n; ++r) {
        std::vector<int> nb;
        const int k = r + 1;
        if (k > 1) nb.push_back(k / 2 - 1);
        if (2 * k - 1 < n) nb.push_back(2 * k - 1);
        if (2 * k < n) nb.push_back(2 * k);
        (*tree)[r] = nb;
        (*parent)[r] = (r + 1) / 2 - 1;
    }
}

// step 2: DFS list, the last child's sub-list reversed
std::vector<int> ring_list(AdjVec& tree, IntMap& parent, int r) {
    std::vector<int> out(1, r);
    std::vector<int> kids;
    for (int x : tree[r])
        if (x != parent[r]) kids.push_back(x);
    for (size_t i = 0; i < kids.size(); ++i) {
        std::vector<int> sub = ring_list(tree, parent, kids[i]);
        if (i + 1 == kids.size()) std::reverse(sub.begin(), sub.end());
        out.insert(out.end(), sub.begin(), sub.end());
    }
    return out;
}

struct Tree {
    int n = 0;
    std::vector<std::vector<int>> children;  // fold order per rank (ring-relabelled ranks)
    std::vector<int> parent;
    std::vector<int> depth;
};

Tree build(int n) {
    Tree T;
    T.n = n;
    T.children.assign((size_t)n, std::vector<int>());
    T.parent.assign((size_t)n, -1);
    T.depth.assign((size_t)n, 0);
    if (n < 2) return T;
    AdjVec tree;
    IntMap parent;
    heap_tree(n, &tree, &parent);
    const std::vector<int> rl = ring_list(tree, parent, 0);
    IntMap rmap;  // heap index -> ring position
    for (int i = 0; i < n; ++i) rmap[rl[(size_t)i]] = i;
    // step 3: iterate the heap tree map (a copy iterates identically)
    AdjVec relabelled;
    {
        AdjVec copy = tree;
        for (const auto& kv : copy)
            for (int x : kv.second) relabelled[rmap[kv.first]].push_back(rmap[x]);
    }
    // step 4: edges in the iteration order of a copy of the relabelled map
    std::vector<std::pair<int, int>> edges;
    {
        AdjVec copy = relabelled;
        for (const auto& kv : copy)
            for (int x : kv.second) edges.emplace_back(kv.first, x);
    }
    std::unordered_map<int, std::unordered_set<int>> adj;
    for (const auto& e : edges) {
        std::unordered_set<int>& fa = adj[e.first];
        if (!fa.count(e.second)) fa.emplace(e.second);
        std::unordered_set<int>& ta = adj[e.second];
        if (!ta.count(e.first)) ta.emplace(e.second);  // graph.h:79-80 inserts `to` into adj[to]
    }
    // step 5: BFS distances from rank 0
    std::unordered_map<int, uint32_t> dist;
    {
        std::unordered_map<int, bool> seen;
        for (int v = 0; v < n; ++v) seen[v] = false;
        std::queue<int> q;
        q.push(0);
        seen[0] = true;
        dist[0] = 0;
        while (!q.empty()) {
            const int v = q.front();
            q.pop();
            for (int w : adj[v])
                if (!seen[w]) {
                    seen[w] = true;
                    dist[w] = dist[v] + 1;
                    q.push(w);
                }
        }
    }
    for (int r = 0; r < n; ++r) {
        const std::unordered_set<int> nb = adj[r];  // GetNeighbors returns a copy
        std::unordered_set<int> recv_from;
        const uint32_t d = dist[r];
        for (int x : nb) {
            if (dist[x] == d + 1) recv_from.insert(x);
            else if (dist[x] + 1 == d) T.parent[(size_t)r] = x;
        }
        for (int x : recv_from) T.children[(size_t)r].push_back(x);
        T.depth[(size_t)r] = (int)d;
    }
    return T;
}

// post-order fold program: (dst, src) pairs, own[dst] = OP(own[dst], own[src])
void program(const Tree& T, int v, std::vector<std::pair<int, int>>* out) {
    for (int c : T.children[(size_t)v]) {
        program(T, c, out);
        out->emplace_back(v, c);
    }
}

}  // namespace

extern "C" {

/* The tree TryReduceTree folds over for n ranks (root 0): children[r*16 + i]
 * = rank r's i-th child in fold order (nchild[r] of them), parent[r] (-1 at
 * the root), depth[r].  Returns 0, or -1 for n outside 1..16. */
int rdc_oracle_tree(int n, int* nchild, int* children, int* parent, int* depth) {
    if (n < 1 || n > 16) return -1;
    const Tree T = build(n);
    for (int r = 0; r < n; ++r) {
        nchild[r] = (int)T.children[(size_t)r].size();
        for (size_t i = 0; i < T.children[(size_t)r].size(); ++i) children[r * 16 + (int)i] = T.children[(size_t)r][i];
        parent[r] = T.parent[(size_t)r];
        depth[r] = T.depth[(size_t)r];
    }
    return 0;
}

/* The fold as a post-order program of n-1 (dst, src) rank pairs:
 * acc[dst] = OP(acc[dst], acc[src]) with acc[q] = rank q's input; the result
 * is acc[0].  Returns the number of pairs, or -1. */
int rdc_oracle_tree_program(int n, int* dst, int* src) {
    if (n < 1 || n > 16) return -1;
    const Tree T = build(n);
    std::vector<std::pair<int, int>> prog;
    program(T, 0, &prog);
    for (size_t i = 0; i < prog.size(); ++i) {
        dst[i] = prog[i].first;
        src[i] = prog[i].second;
    }
    return (int)prog.size();
}

/* TryAllreduceTree on n per-rank buffers (in place): every buffer receives
 * the root's tree reduction (reducer(src=child, dst=own) per fold). */
int rdc_oracle_allreduce_tree(void** bufs, int n, uint64_t count, int dtype, int op) {
    const size_t esz = rdc_oracle_dtype_size(dtype);
    if (esz == 0 || n < 1 || n > 16) return -1;
    if (n == 1 || count == 0) return 0;
    int dst[16], src[16];
    const int k = rdc_oracle_tree_program(n, dst, src);
    for (int i = 0; i < k; ++i) {
        const int rc = rdc_oracle_reducer(bufs[src[i]], bufs[dst[i]], count, dtype, op);
        if (rc) return rc;
    }
    for (int r = 1; r < n; ++r) memcpy(bufs[r], bufs[0], count * esz);
    return 0;
}

}  // extern "C"
