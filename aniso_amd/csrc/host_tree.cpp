// host_tree.cpp -- quadtree + U/V/W/X lists, bit-exact with bbfmm::tree
// (bbfmm.h:146-449), and the flattened per-shard work plan uploaded to HBM.
#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <functional>
#include <cmath>
#include <stdexcept>
#include <thread>
#include <unordered_map>

#include "host.hpp"

namespace aniso {

namespace {

struct Builder {
    Tree& t;
    const double* x;
    const double* y;
    int rank, maxLevelArg;
    std::vector<int> tmp;

    int new_node(int level, int slot) {
        t.parent.push_back(-1);
        t.level.push_back(level);
        t.slot.push_back(slot);
        t.isLeaf.push_back(0);
        t.isEmpty.push_back(0);
        t.child.push_back({-1, -1, -1, -1});
        t.ncx.push_back(0); t.ncy.push_back(0); t.nrx.push_back(0); t.nry.push_back(0);
        t.begin.push_back(0); t.count.push_back(0);
        return t.nn++;
    }

    // assignChildren (bbfmm.h:250-317); the children's point lists are a stable
    // 4-way partition of the parent's range of `perm` (same order as push_back).
    void assign(int id) {
        if (t.count[id] == 0) {
            t.isLeaf[id] = 1;
            t.isEmpty[id] = 1;
            return;
        }
        if (t.count[id] <= rank || t.level[id] == maxLevelArg) {
            t.isLeaf[id] = 1;
            t.maxLevel = std::max(t.maxLevel, t.level[id]);
            return;
        }
        for (int i = 0; i < 4; ++i) {
            int c = new_node(t.level[id] + 1, i);
            t.child[id][i] = c;
            t.parent[c] = id;
            t.ncx[c] = t.ncx[id] + ((i & 1) - 0.5) * t.nrx[id];
            t.ncy[c] = t.ncy[id] + (((i >> 1) & 1) - 0.5) * t.nry[id];
            t.nrx[c] = t.nrx[id] * 0.5;
            t.nry[c] = t.nry[id] * 0.5;
        }
        const int64_t b = t.begin[id], n = t.count[id];
        const double cx = t.ncx[id], cy = t.ncy[id];
        int64_t cnt[4] = {0, 0, 0, 0};
        for (int64_t k = b; k < b + n; ++k) {
            int idx = t.perm[k];
            int y_bit = y[idx] < cy ? 0 : 1;
            int x_bit = x[idx] < cx ? 0 : 1;
            cnt[2 * y_bit + x_bit]++;
        }
        int64_t off[4];
        off[0] = b;
        for (int i = 1; i < 4; ++i) off[i] = off[i - 1] + cnt[i - 1];
        for (int i = 0; i < 4; ++i) {
            t.begin[t.child[id][i]] = off[i];
            t.count[t.child[id][i]] = cnt[i];
        }
        for (int64_t k = b; k < b + n; ++k) {
            int idx = t.perm[k];
            int y_bit = y[idx] < cy ? 0 : 1;
            int x_bit = x[idx] < cx ? 0 : 1;
            tmp[off[2 * y_bit + x_bit]++] = idx;
        }
        std::copy(tmp.begin() + b, tmp.begin() + b + n, t.perm.begin() + b);
        for (int i = 0; i < 4; ++i) assign(t.child[id][i]);
    }
};

// findNode (bbfmm.h:416-429)
inline int find_node(const Tree& t, double px, double py) {
    int id = 0;
    for (;;) {
        if (std::fabs(t.ncx[id] - px) < kEps && std::fabs(t.ncy[id] - py) < kEps) return id;
        if (t.isLeaf[id]) return id;
        int x_bit = t.ncx[id] > px ? 0 : 1;
        int y_bit = t.ncy[id] > py ? 0 : 1;
        id = t.child[id][2 * y_bit + x_bit];
    }
}

// isAdjacent (bbfmm.h:431-447)
inline bool adjacent(const Tree& t, int a, int b) {
    double diff_x = std::fabs(t.ncx[a] - t.ncx[b]), diff_y = std::fabs(t.ncy[a] - t.ncy[b]);
    double r_x = std::fabs(t.nrx[a] + t.nrx[b]), r_y = std::fabs(t.nry[a] + t.nry[b]);
    bool rdx = r_x >= diff_x - kEps;
    bool rdy = r_y >= diff_y - kEps;
    bool x_adj = (std::fabs(diff_x - r_x) < kEps) && rdy;
    bool y_adj = (std::fabs(diff_y - r_y) < kEps) && rdx;
    return x_adj || y_adj;
}

inline void set_insert(std::vector<int>& v, int x) {
    auto it = std::lower_bound(v.begin(), v.end(), x);
    if (it == v.end() || *it != x) v.insert(it, x);
}

// buildNode (bbfmm.h:334-413)
void build_node(const Tree& t, int id, double minx, double miny, double maxx, double maxy, std::vector<int>& U,
                std::vector<int>& V, std::vector<int>& W, std::vector<int>& X, std::vector<int>& queue) {
    U.clear(); V.clear(); W.clear(); X.clear();
    if (t.parent[id] != -1) {
        int p = t.parent[id];
        double dx = t.nrx[id], dy = t.nry[id];
        double xs = t.ncx[p] - dx, ys = t.ncy[p] - dy;
        for (int x_id = -2; x_id < 4; x_id++)
            for (int y_id = -2; y_id < 4; y_id++) {
                double curx = xs + 2 * x_id * dx;
                double cury = ys + 2 * y_id * dy;
                bool le = (curx <= maxx + kEps) && (cury <= maxy + kEps);
                bool ge = (curx >= minx - kEps) && (cury >= miny - kEps);
                bool eq = std::fabs(curx - t.ncx[id]) < kEps && std::fabs(cury - t.ncy[id]) < kEps;
                if (!(le && ge && !eq)) continue;
                int cur = find_node(t, curx, cury);
                bool adj = adjacent(t, id, cur);
                if (t.level[cur] < t.level[id]) {
                    if (adj) {
                        if (t.isLeaf[cur]) set_insert(U, cur);
                    } else {
                        set_insert(X, cur);
                    }
                }
                if (t.level[cur] == t.level[id]) {
                    if (!adj) {
                        set_insert(V, cur);
                    } else if (t.isLeaf[id]) {
                        queue.clear();
                        queue.push_back(cur);
                        for (size_t h = 0; h < queue.size(); ++h) {
                            int f = queue[h];
                            if (!adjacent(t, f, id)) {
                                set_insert(W, f);
                            } else if (t.isLeaf[f]) {
                                set_insert(U, f);
                            } else {
                                for (int i = 0; i < 4; ++i) queue.push_back(t.child[f][i]);
                            }
                        }
                    }
                }
            }
    }
    if (t.isLeaf[id]) set_insert(U, id);
}

}  // namespace

void Tree::build(const double* x, const double* y, int64_t n, int rank, int maxLevelArg, int nthreads) {
    if (n <= 0) throw std::invalid_argument("tree needs at least one point");
    *this = Tree();
    // getCenterRadius (bbfmm.h:231-248)
    double x_max = x[0], x_min = x[0], y_max = y[0], y_min = y[0];
    for (int64_t i = 0; i < n; ++i) {
        x_max = std::max(x_max, x[i]); y_max = std::max(y_max, y[i]);
        x_min = std::min(x_min, x[i]); y_min = std::min(y_min, y[i]);
    }
    cx = (x_max + x_min) / 2.0;
    cy = (y_max + y_min) / 2.0;
    rx = (x_max - x_min) / 2.0;
    ry = (y_max - y_min) / 2.0;
    perm.resize(n);
    for (int64_t i = 0; i < n; ++i) perm[i] = (int)i;
    Builder b{*this, x, y, rank, maxLevelArg, std::vector<int>(n)};
    int root = b.new_node(0, 0);
    ncx[root] = cx; ncy[root] = cy; nrx[root] = rx; nry[root] = ry;
    begin[root] = 0; count[root] = n;
    b.assign(root);

    // lists, in parallel over nodes
    std::vector<std::vector<int>> L[4];
    for (auto& l : L) l.resize(nn);
    const double minx = cx - rx, miny = cy - ry, maxx = cx + rx, maxy = cy + ry;
    std::atomic<int> next{0};
    auto worker = [&]() {
        std::vector<int> q;
        for (;;) {
            int s = next.fetch_add(256);
            if (s >= nn) break;
            int e = std::min(nn, s + 256);
            for (int id = s; id < e; ++id) build_node(*this, id, minx, miny, maxx, maxy, L[0][id], L[1][id], L[2][id], L[3][id], q);
        }
    };
    int nt = std::max(1, std::min(nthreads, 64));
    std::vector<std::thread> th;
    for (int i = 1; i < nt; ++i) th.emplace_back(worker);
    worker();
    for (auto& h : th) h.join();
    std::vector<int64_t>* ptrs[4] = {&uPtr, &vPtr, &wPtr, &xPtr};
    std::vector<int>* idxs[4] = {&uIdx, &vIdx, &wIdx, &xIdx};
    for (int k = 0; k < 4; ++k) {
        ptrs[k]->assign(nn + 1, 0);
        for (int i = 0; i < nn; ++i) (*ptrs[k])[i + 1] = (*ptrs[k])[i] + (int64_t)L[k][i].size();
        idxs[k]->resize((*ptrs[k])[nn]);
        for (int i = 0; i < nn; ++i) std::copy(L[k][i].begin(), L[k][i].end(), idxs[k]->begin() + (*ptrs[k])[i]);
    }
}

// Shard boundaries (tree positions, nranks + 1 entries): the first level with at
// least 16 x nranks nodes (plus the leaves above it) is the frontier; its nodes,
// in tree order, are cut into nranks contiguous runs balanced by point count, so a
// boundary never splits a frontier node (nor, therefore, a leaf).  Depends only on
// the tree: every rank computes every rank's range.
std::vector<int64_t> shard_cuts(const Tree& t, int nranks) {
    if (nranks < 1) throw std::invalid_argument("nranks must be >= 1");
    const int64_t N = t.nn ? t.count[0] : 0;
    std::vector<int64_t> cuts(nranks + 1, N);
    cuts[0] = 0;
    if (nranks == 1) return cuts;
    int Lc = 0;
    std::vector<int> frontier;
    for (;;) {
        frontier.clear();
        for (int i = 0; i < t.nn; ++i)
            if (t.level[i] == Lc || (t.level[i] < Lc && t.isLeaf[i])) frontier.push_back(i);
        if ((int)frontier.size() >= 16 * nranks || Lc >= t.maxLevel) break;
        ++Lc;
    }
    std::sort(frontier.begin(), frontier.end(), [&](int a, int b) {
        return t.begin[a] != t.begin[b] ? t.begin[a] < t.begin[b] : t.count[a] < t.count[b];
    });
    int r = 1;
    for (int f : frontier) {
        while (r < nranks && t.begin[f] + t.count[f] / 2 >= (N * r) / nranks) {
            cuts[r] = t.begin[f];
            ++r;
        }
    }
    for (; r < nranks; ++r) cuts[r] = N;
    for (int k = 1; k <= nranks; ++k) cuts[k] = std::max(cuts[k], cuts[k - 1]);
    return cuts;
}

void Plan::build(const Tree& t, int np, int rank_, int nranks_) {
    (void)np;
    if (nranks_ < 1 || rank_ < 0 || rank_ >= nranks_) throw std::invalid_argument("bad shard rank/nranks");
    const bool symNear = nearSymmetric, symHs = nearSymHs, upIn = xUpPartialIn;
    const int capCanon = maxCanon;
    *this = Plan();
    nearSymmetric = symNear;
    nearSymHs = symHs;
    xUpPartialIn = upIn;
    maxCanon = std::max(0, std::min(kMaxCanon, capCanon));
    rank = rank_;
    nranks = nranks_;
    // ---- ownership: contiguous runs of a subtree frontier (DFS order == tree order)
    const std::vector<int64_t> cuts = shard_cuts(t, nranks);
    ownBegin = cuts[rank];
    ownEnd = cuts[rank + 1];
    auto intersects = [&](int n) { return t.begin[n] < ownEnd && t.begin[n] + t.count[n] > ownBegin; };
    // ---- tiers for the up / down passes (bbfmm.h:825-861 upPass, 1066-1106
    // downPass): subtrees of at most 4 levels (the top one up to 5), each one
    // workgroup with its nodes' expansions resident in LDS; roots of tier k-1
    // sit one level below tier k's bottom and are exchanged through HBM.
    {
        // the root (level 0) never interacts: its multipole is never a source and
        // its local is zero, so tiers cover levels 1 .. D (none for a lone leaf)
        const int D = t.maxLevel;
        tierRootLevel.clear();
        tierBottomLevel.clear();
        if (D >= 1) {
            const int bspan = 3;  // levels of the bottom tier (3: 4x the tasks at 1/4 the LDS; down 0.124 -> 0.090 ms, r01g)
            tierRootLevel.push_back(std::max(1, D - (bspan - 1)));
            tierBottomLevel.push_back(D);
            const int span = 2;  // levels per upper tier (1, 3 and 4 measured equal or slower, r01g; 3 and 4 on a rank of 8 +9 % / +35 %, r04ac)
            while (tierRootLevel.back() > 1) {
                tierBottomLevel.push_back(tierRootLevel.back() - 1);
                tierRootLevel.push_back(std::max(1, tierRootLevel.back() - span));
            }
        }
    }
    buildUpTasks(t);
    // ---- M2L over V then X (bbfmm.h:1051-1065), active non-empty targets.
    // V is a symmetric relation and K_{B<-A} = (-1)^m K_{A<-B}^T (tau is symmetric,
    // g_m(-d) = (-1)^m g_m(d)), so when both ends are targets here only the block
    // of the smaller id is stored (up to kMaxCanon per target, the rest directed):
    // its owner also produces the transposed product into a partial slot; slots
    // are numbered receiver-contiguously so k_m2l_gather reads one range per node.
    const char* symEnv = std::getenv("ANISO_SYMMETRIC");
    symmetric = !(symEnv && symEnv[0] == '0');
    std::vector<char> m2lActive(t.nn, 0);
    for (int i = 0; i < t.nn; ++i) m2lActive[i] = !t.isEmpty[i] && t.parent[i] != -1 && intersects(i);
    std::vector<std::vector<int>> inCanon(t.nn), inFrom(t.nn);  // per receiver: canonical ids, their senders
    m2lPtr.push_back(0);
    attPtr.assign(1, 0);
    attSrc.clear();
    attBlk.clear();
    attOwner.clear();
    attOther.clear();
    std::unordered_map<int64_t, int> attStored;  // (owner << 32 | other) -> stored V block
    auto attDirected = [&](int i, int b) {
        attSrc.push_back(b);
        attBlk.push_back((int)attOwner.size());
        attOwner.push_back(i);
        attOther.push_back(b);
    };
    int canon = 0;
    std::vector<int> canonSrc;
    for (int i = 0; i < t.nn; ++i) {
        if (!m2lActive[i]) continue;
        m2lTgt.push_back(i);
        canonSrc.clear();
        for (int64_t k = t.vPtr[i]; k < t.vPtr[i + 1]; ++k) {
            int b = t.vIdx[k];
            if (t.isEmpty[b]) continue;
            ++pairsM2L;
            if (symmetric && m2lActive[b] && b < i) {
                auto it = attStored.find(((int64_t)b << 32) | (uint32_t)i);
                if (it != attStored.end()) {
                    attSrc.push_back(b);
                    attBlk.push_back(~it->second);
                } else {
                    attDirected(i, b);
                }
            } else {
                if (symmetric && m2lActive[b]) attStored[((int64_t)i << 32) | (uint32_t)b] = (int)attOwner.size();
                attDirected(i, b);
            }
            if (symmetric && m2lActive[b]) {
                if (i < b && (int)canonSrc.size() < maxCanon) {
                    canonSrc.push_back(b);
                    continue;
                }
                if (i > b && std::find(inFrom[i].begin(), inFrom[i].end(), b) != inFrom[i].end())
                    continue;  // arrives through b's transposed product
            }
            m2lSrc.push_back(b);
        }
        for (int64_t k = t.xPtr[i]; k < t.xPtr[i + 1]; ++k)
            if (!t.isEmpty[t.xIdx[k]]) {
                m2lSrc.push_back(t.xIdx[k]);
                attDirected(i, t.xIdx[k]);
                ++pairsM2L;
            }
        attPtr.push_back((int64_t)attSrc.size());
        m2lNDir.push_back((int)(m2lSrc.size() - m2lPtr.back()));
        m2lCanonBase.push_back(canon);
        m2lMaxCanon = std::max<int>(m2lMaxCanon, (int)canonSrc.size());
        for (int b : canonSrc) {
            m2lSrc.push_back(b);
            inCanon[b].push_back(canon++);
            inFrom[b].push_back(i);
        }
        m2lPtr.push_back((int64_t)m2lSrc.size());
    }
    m2lCanon = canon;
    buildClusters(t);
    storedM2L = (int64_t)m2lSrc.size();
    m2lOutSlot.assign(canon, -1);
    m2lInPtr.push_back(0);
    int slot = 0;
    for (int i : m2lTgt) {
        for (int c : inCanon[i]) m2lOutSlot[c] = slot++;
        m2lInPtr.push_back(slot);
    }
    if (slot != canon) throw std::logic_error("symmetric M2L: canonical pair without an active receiver");
    // ---- near field over U then W (bbfmm.h:1081-1099), owned non-empty leaves.
    // U is symmetric as well: per leaf the stored sources are [directed | canonical]
    // (self block, W members and unowned U members first; then the U members with a
    // larger id); the transposed products land in a contiguous partial range.
    std::vector<int> leafIdx(t.nn, -1);
    for (int i = 0; i < t.nn; ++i) {
        if (!t.isLeaf[i] || t.isEmpty[i] || !intersects(i)) continue;
        if (t.begin[i] < ownBegin || t.begin[i] + t.count[i] > ownEnd)
            throw std::logic_error("shard boundary splits a leaf");
        leafIdx[i] = (int)leaves.size();
        leaves.push_back(i);
    }
    std::vector<std::vector<int>> nearInRef(leaves.size());  // per receiver: partial offsets of its blocks
    nearPtr.push_back(0);
    int64_t partTotal = 0;
    for (size_t li = 0; li < leaves.size(); ++li) {
        const int i = leaves[li];
        nearKOff.push_back(nearKTotal);
        int64_t S = 0, Sdir = 0;
        canonSrc.clear();
        for (int64_t k = t.uPtr[i]; k < t.uPtr[i + 1]; ++k) {
            int b = t.uIdx[k];
            if (t.isEmpty[b]) continue;
            pairsNear += t.count[i] * t.count[b];
            // k_near reduces a canonical column within one pass of <= 64 row quads
            if (symmetric && nearSymmetric && b != i && leafIdx[b] >= 0 && t.count[i] <= 128 && t.count[b] <= 128) {
                if (i < b) canonSrc.push_back(b);
                continue;
            }
            nearSrc.push_back(b);
            S += t.count[b];
        }
        for (int64_t k = t.wPtr[i]; k < t.wPtr[i + 1]; ++k) {
            int b = t.wIdx[k];
            if (t.isEmpty[b]) continue;
            pairsNear += t.count[i] * t.count[b];
            nearSrc.push_back(b);
            S += t.count[b];
        }
        Sdir = S;
        const int64_t partBase = partTotal;
        for (int b : canonSrc) {
            nearSrc.push_back(b);
            nearInRef[leafIdx[b]].push_back((int)partTotal);  // sender-contiguous partials
            partTotal += t.count[b];
            S += t.count[b];
        }
        nearPtr.push_back((int64_t)nearSrc.size());
        nearKTotal += S * ((t.count[i] + 3) & ~(int64_t)3);  // rows padded to a multiple of 4: 32-B row quads
        storedNear += S * t.count[i];
        if (S > (int64_t)1 << 30 || partTotal > ((int64_t)1 << 31) - 1)
            throw std::invalid_argument("leaf neighbourhood too large");
        leafInfo.push_back({i, (int)t.begin[i], (int)t.count[i], (int)S});
        nearMaxLeaf = std::max<int>(nearMaxLeaf, (int)t.count[i]);
        nearSym.push_back({(int)Sdir, (int)partBase});
    }
    nearPartTotal = partTotal;
    nearInPtr.assign(1, 0);
    nearInOff.clear();
    for (auto& v : nearInRef) {
        nearInOff.insert(nearInOff.end(), v.begin(), v.end());
        nearInPtr.push_back((int)nearInOff.size());
    }
    nearPtsPtr.push_back(0);
    for (size_t li = 0; li < leaves.size(); ++li) {
        for (int64_t j = nearPtr[li]; j < nearPtr[li + 1]; ++j) {
            int s = nearSrc[j];
            for (int64_t k = 0; k < t.count[s]; ++k) nearPts.push_back((int)(t.begin[s] + k));
        }
        nearPtsPtr.push_back((int64_t)nearPts.size());
    }
    // staged near field: one source table per 16 consecutive leaves (a 4 x 4 leaf
    // block on the uniform grids: a 6 x 6 leaf union instead of 16 x 9 per-leaf reads)
    nsPtr.assign(1, 0);
    nsPts.clear();
    nearLoc.clear();
    nsMax = 0;
    if (nearMaxLeaf <= 16 && !leaves.empty()) {
        nearLoc.resize(nearPts.size());
        std::vector<int> u;
        for (size_t g0 = 0; g0 < leaves.size(); g0 += 16) {
            const size_t g1 = std::min(leaves.size(), g0 + 16);
            u.assign(nearPts.begin() + nearPtsPtr[g0], nearPts.begin() + nearPtsPtr[g1]);
            std::sort(u.begin(), u.end());
            u.erase(std::unique(u.begin(), u.end()), u.end());
            if (u.size() > 65535) {  // the table index is 16 bits: no staging
                nsPtr.assign(1, 0);
                nsPts.clear();
                nearLoc.clear();
                nsMax = 0;
                break;
            }
            for (int64_t j = nearPtsPtr[g0]; j < nearPtsPtr[g1]; ++j)
                nearLoc[j] = (uint16_t)(std::lower_bound(u.begin(), u.end(), nearPts[j]) - u.begin());

            nsPts.insert(nsPts.end(), u.begin(), u.end());
            nsPtr.push_back((int64_t)nsPts.size());
            nsMax = std::max<int>(nsMax, (int)u.size());
        }
    }
    buildNearHs(t, leafIdx);
    buildDownTasks(t);
    buildNearUp(t);
}

void Plan::buildNearUp(const Tree& t) {
    nearUpGrp.clear();
    nearUpOk = false;
    const size_t ng = nsPtr.size() - 1;
    if (nranks != 1 || nsMax <= 0 || ng == 0 || leaves.size() != 16 * ng || upTierTask.size() < 2 ||
        (size_t)(upTierTask[1] - upTierTask[0]) != ng)
        return;
    std::vector<int> taskOf(t.nn, -1);
    for (int k = upTierTask[0]; k < upTierTask[1]; ++k) taskOf[upTaskRoot[k]] = k;
    for (size_t g = 0; g < ng; ++g) {
        const int* L = leaves.data() + 16 * g;
        if (t.parent[L[0]] < 0 || t.parent[t.parent[L[0]]] < 0) return;
        const int A = t.parent[t.parent[L[0]]];
        const int k = taskOf[A];
        if (k < 0 || upTaskPtr[k + 1] - upTaskPtr[k] != 21) return;  // a 3-level tier-0 task rooted at A
        std::array<int, 25> G{};
        int found = 0;
        for (int c = 0; c < 16; ++c) {
            const int p = t.parent[L[c]];
            if (t.parent[p] != A || !t.isLeaf[L[c]] || t.isEmpty[L[c]]) return;
            int m = -1, q = -1;
            for (int i = 0; i < 4; ++i) {
                if (t.child[A][i] == p) m = i;
                if (t.child[p][i] == L[c]) q = i;
            }
            if (m < 0 || q < 0 || m != c / 4) return;  // wave m of the group holds parent m's leaves
            G[c] = (m << 2) | q;
            found |= 1 << (4 * m + q);
        }
        if (found != 0xFFFF) return;  // the 16 leaves are all of A's grandchildren
        for (int m = 0; m < 4; ++m) {
            G[16 + m] = m;
            G[20 + m] = t.child[A][m];
        }
        G[24] = A;
        nearUpGrp.insert(nearUpGrp.end(), G.begin(), G.end());
    }
    nearUpOk = true;
}

// The staged near field of the harmonic block apply with symmetric U storage (see
// Plan::nearSymHs; bbfmm.h:1081-1099): its own column lists beside the directed ones
// (which the per-mode kernels keep), over the same source tables.  Per leaf the columns
// are [directed: itself, W, U members not both owned here | canonical: owned U members
// with a larger id], the canonical ones in one block per partner leaf.
void Plan::buildNearHs(const Tree& t, const std::vector<int>& leafIdx) {
    hsPtsPtr.assign(1, 0);
    hsLoc.clear();
    hsKOff.clear();
    hsSym.clear();
    hsSrcPtr.assign(1, 0);
    hsSrc.clear();
    hsDst.clear();
    nearSelfRow.clear();
    hsKTotal = 0;
    hsPartTotal = 0;
    hsStored = 0;
    nearGrpInPtr.assign(1, 0);
    nearGrpIn.clear();
    nearGrpSlots = 0;
    nearSymHsOn = nearSymHs && !nearSymmetric && nearMaxLeaf <= 16 && !leaves.empty() &&
                  nsPtr.size() == (leaves.size() + 15) / 16 + 1 &&
                  (size_t)nsMax * 11 * 8 <= 64 * 1024;  // near_hs_staged's test (K <= 8)
    if (!nearSymHsOn) return;
    std::vector<std::vector<int>> inRef(leaves.size()), grpIn(16);
    std::vector<int> u, dir, can;
    for (size_t g0 = 0; g0 < leaves.size(); g0 += 16) {
        const size_t g1 = std::min(leaves.size(), g0 + 16);
        int q = 0;  // the group's LDS slots: one per in-group canonical block, in (leaf, partner) order
        for (auto& v : grpIn) v.clear();
        u.assign(nsPts.begin() + nsPtr[g0 / 16], nsPts.begin() + nsPtr[g0 / 16 + 1]);  // sorted unique
        auto row = [&](int64_t pos) {
            auto it = std::lower_bound(u.begin(), u.end(), (int)pos);
            if (it == u.end() || *it != (int)pos) throw std::logic_error("staged near field: source not in its table");
            return (uint16_t)(it - u.begin());
        };
        for (size_t li = g0; li < g1; ++li) {
            const int i = leaves[li];
            dir.clear();
            can.clear();
            for (int64_t k = t.uPtr[i]; k < t.uPtr[i + 1]; ++k) {
                const int b = t.uIdx[k];
                if (t.isEmpty[b]) continue;
                if (b != i && leafIdx[b] >= 0) {  // both leaves owned: stored once, by the smaller id
                    if (i < b) can.push_back(b);
                    continue;
                }
                dir.push_back(b);
            }
            for (int64_t k = t.wPtr[i]; k < t.wPtr[i + 1]; ++k)
                if (!t.isEmpty[t.wIdx[k]]) dir.push_back(t.wIdx[k]);
            hsKOff.push_back(hsKTotal);
            int S = 0;
            for (int b : dir) {
                hsSrc.push_back(b);
                for (int64_t u0 = 0; u0 < t.count[b]; ++u0) {
                    hsLoc.push_back(row(t.begin[b] + u0));
                    hsDst.push_back(0);  // directed: no partner product
                }
                S += (int)t.count[b];
            }
            const int Sdir = S;
            for (int b : can) {
                const int lb = leafIdx[b];
                if (lb / 16 == (int)li / 16 && q < kNearGrpSlots) {
                    grpIn[lb % 16].push_back(q);  // the partner is in this group: an LDS slot
#ifdef ANISO_NEAR_SYM_ATOMIC  // A/B builds only: the partner's own LDS rows, added atomically
                    for (int64_t u0 = 0; u0 < t.count[b]; ++u0) hsDst.push_back(~(int)((lb % 16) * 16 + u0));
#else
                    for (int64_t u0 = 0; u0 < t.count[b]; ++u0) hsDst.push_back(~(int)(q * 16 + u0));
#endif
                    ++q;
                } else {
                    inRef[lb].push_back((int)hsPartTotal);  // else its partial slots, sender-contiguous
                    for (int64_t u0 = 0; u0 < t.count[b]; ++u0) hsDst.push_back((int)(hsPartTotal + u0));
                    hsPartTotal += t.count[b];
                }
                hsSrc.push_back(b);
                for (int64_t u0 = 0; u0 < t.count[b]; ++u0) hsLoc.push_back(row(t.begin[b] + u0));
                S += (int)t.count[b];
            }
            hsSym.push_back({Sdir, S});
            hsKTotal += (int64_t)S * ((t.count[i] + 3) & ~(int64_t)3);
            hsStored += (int64_t)S * t.count[i];
            hsPtsPtr.push_back((int64_t)hsLoc.size());
            hsSrcPtr.push_back((int64_t)hsSrc.size());
            nearSelfRow.push_back(row(t.begin[i]));  // the leaf's own points: one run of table rows
        }
        // per leaf its incoming slots, ascending (= by sender): summed in that order
        for (size_t li = g0; li < g1; ++li) {
            const auto& v = grpIn[li - g0];
            nearGrpIn.insert(nearGrpIn.end(), v.begin(), v.end());
            nearGrpInPtr.push_back((int)nearGrpIn.size());
        }
        nearGrpSlots = std::max(nearGrpSlots, q);
#ifdef ANISO_NEAR_SYM_ATOMIC
        nearGrpSlots = 16;
#endif
    }
    if (hsPartTotal > ((int64_t)1 << 31) - 1) throw std::invalid_argument("near partials overflow");
    // the down pass gathers the partials through the same per-leaf lists as the
    // single-RHS symmetric near field (a block handle has none of those)
    nearInPtr.assign(1, 0);
    nearInOff.clear();
    for (auto& v : inRef) {
        nearInOff.insert(nearInOff.end(), v.begin(), v.end());
        nearInPtr.push_back((int)nearInOff.size());
    }
}


// Nodes of the subtree of `root` down to level `bottom`, level by level (keep()
// filters nodes; children of leaves do not exist).
static std::vector<std::vector<int>> task_levels(const Tree& t, int root, int bottom,
                                                 const std::function<bool(int)>& keep) {
    std::vector<std::vector<int>> lv{{root}};
    while (t.level[lv.back()[0]] < bottom) {
        std::vector<int> next;
        for (int n : lv.back())
            if (!t.isLeaf[n])
                for (int q = 0; q < 4; ++q) {
                    const int c = t.child[n][q];
                    if (c >= 0 && keep(c)) next.push_back(c);
                }
        if (next.empty()) break;
        lv.push_back(std::move(next));
    }
    return lv;
}

void Plan::buildUpTasks(const Tree& t) {
    std::vector<int> slotOf(t.nn, -1);
    auto keep = [&](int n) { return !t.isEmpty[n]; };
    upTierTask.assign(1, 0);
    upTaskRoot.clear();
    upTaskPtr.assign(1, 0);
    upGrpPtr.assign(1, 0);
    upGrp.clear();
    upNode.clear();
    upCode.clear();
    upDesc.clear();
    upGrpFix.clear();
    upGeom.clear();
    upLeaf.clear();
    upMaxTask = 1;
    upTierMaxTask.assign(tierRootLevel.size(), 1);
    for (size_t k = 0; k < tierRootLevel.size(); ++k) {  // bottom-up
        for (int r = 0; r < t.nn; ++r) {
            if (t.level[r] != tierRootLevel[k] || t.isEmpty[r]) continue;
            auto lv = task_levels(t, r, tierBottomLevel[k], keep);
            const int base = (int)upNode.size();
            for (int L = (int)lv.size() - 1; L >= 0; --L) {  // deepest level first
                upGrp.push_back((int)upNode.size());
                for (int n : lv[L]) {
                    slotOf[n] = (int)upNode.size() - base;
                    upNode.push_back(n);
                }
            }
            for (int i = base; i < (int)upNode.size(); ++i) {
                const int n = upNode[i];
                std::array<int, 4> c{kLeafCode, kLeafCode, kLeafCode, kLeafCode};
                if (!t.isLeaf[n])
                    for (int q = 0; q < 4; ++q) {
                        const int ch = t.child[n][q];
                        c[q] = (ch < 0 || t.isEmpty[ch]) ? -1
                               : t.level[ch] <= tierBottomLevel[k] ? slotOf[ch]
                                                                   : -(ch + 2);  // root of the tier below
                    }
                upCode.push_back(c);
            }
            // per-task record and per-node records (one round of independent loads)
            const int nt = (int)upNode.size() - base, ng = (int)lv.size();
            if (ng > kTaskLevels) throw std::logic_error("up task deeper than its record");
            const int64_t b0 = t.begin[r];
            upDesc.push_back({base, nt, (int)b0, ng});
            std::array<int, kTaskLevels + 1> gs{};
            for (int g = 0; g < ng; ++g) gs[g] = upGrp[upGrp.size() - ng + g] - base;
            gs[ng] = nt;
            upGrpFix.insert(upGrpFix.end(), gs.begin(), gs.end());
            for (int i = base; i < (int)upNode.size(); ++i) {
                const int n = upNode[i];
                upGeom.push_back({t.ncx[n], t.ncy[n], 1.0 / t.nrx[n], 1.0 / t.nry[n]});
                upLeaf.push_back({(int)(t.begin[n] - b0), (int)t.count[n]});
            }
            upGrpPtr.push_back((int)upGrp.size());
            upTaskPtr.push_back((int)upNode.size());
            upTaskRoot.push_back(r);
            upMaxTask = std::max(upMaxTask, (int)upNode.size() - base);
            upTierMaxTask[k] = std::max(upTierMaxTask[k], (int)upNode.size() - base);
        }
        upTierTask.push_back((int)upTaskPtr.size() - 1);
    }
    upLastLeafTier = 0;
    for (size_t k = 0; k + 1 < upTierTask.size(); ++k)
        for (int task = upTierTask[k]; task < upTierTask[k + 1]; ++task)
            for (int i = upTaskPtr[task]; i < upTaskPtr[task + 1]; ++i)
                if (upCode[i][0] == kLeafCode) upLastLeafTier = (int)k;
    upGrp.push_back((int)upNode.size());  // sentinel: group g spans [upGrp[g], upGrp[g+1])
}

void Plan::buildDownTasks(const Tree& t) {
    auto intersects = [&](int n) { return t.begin[n] < ownEnd && t.begin[n] + t.count[n] > ownBegin; };
    auto keep = [&](int n) { return !t.isEmpty[n] && intersects(n); };
    std::vector<int> slotOf(t.nn, -1), leafOf(t.nn, -1);
    for (size_t i = 0; i < leaves.size(); ++i) leafOf[leaves[i]] = (int)i;
    dnTierTask.assign(1, 0);
    dnTaskPtr.assign(1, 0);
    dnGrpPtr.assign(1, 0);
    dnGrp.clear();
    dnNode.clear();
    dnLeafPtr.assign(1, 0);
    dnLeafSlot.clear();
    dnLeafIdx.clear();
    dnLeafPts.clear();
    dnLeafNear.clear();
    dnNearOff.clear();
    dnNearPtr.assign(1, 0);
    dnMaxNear = 1;
    dnPtsRange.clear();
    dnDesc.clear();
    dnGrpFix.clear();
    dnLeafGeom.clear();
    dnMaxTask = 1;
    dnMaxLeaves = 1;
    // Every task with owned leaves is independent: it rebuilds its root's parent
    // total from the ancestors' locals (L2L chain from level 1; the root's total is
    // zero), so the tasks of all tiers go in ONE launch and leafless tasks are dropped.
    dnChainPtr.assign(1, 0);
    dnChain.clear();
    dnChainFold.clear();
    dnMaxChain = 1;
    std::vector<int> anc;
    for (int k = (int)tierRootLevel.size() - 1; k >= 0; --k) {  // top-down
        for (int r = 0; r < t.nn; ++r) {
            if (t.level[r] != tierRootLevel[k] || !keep(r)) continue;
            auto lv = task_levels(t, r, tierBottomLevel[k], keep);
            bool hasLeaf = false;
            for (auto& level : lv)
                for (int n : level) hasLeaf |= leafOf[n] >= 0;
            if (!hasLeaf) continue;
            const int base = (int)dnNode.size();
            for (auto& level : lv) {  // shallowest level first
                dnGrp.push_back((int)dnNode.size());
                for (int n : level) {
                    slotOf[n] = (int)dnNode.size() - base;
                    const int p = t.parent[n];  // the root's total is zero
                    const int pc = (p < 0 || t.parent[p] < 0) ? -1 : n == r ? -2 : slotOf[p];
                    dnNode.push_back({n, pc, t.slot[n], hmFoldOf.empty() ? 0 : hmFoldOf[n]});
                }
            }
            anc.clear();  // ancestors of r below the root, top-down
            for (int a = t.parent[r]; a >= 0 && t.parent[a] >= 0; a = t.parent[a]) anc.push_back(a);
            for (auto it = anc.rbegin(); it != anc.rend(); ++it) {
                dnChain.push_back({*it, t.slot[*it]});
                dnChainFold.push_back(hmFoldOf.empty() ? 0 : hmFoldOf[*it]);
            }
            dnChainPtr.push_back((int)dnChain.size());
            dnMaxChain = std::max(dnMaxChain, (int)anc.size());
            const int nearBase = (int)dnNearOff.size();
            // owned leaves in tree order: they tile [ptsBegin, ptsEnd) contiguously
            std::vector<int> lf;
            for (int i = base; i < (int)dnNode.size(); ++i)
                if (leafOf[dnNode[i][0]] >= 0) lf.push_back(i - base);
            std::sort(lf.begin(), lf.end(), [&](int a, int b) { return t.begin[dnNode[base + a][0]] < t.begin[dnNode[base + b][0]]; });
            int64_t pb = -1, pe = -1;
            for (int sl : lf) {
                const int n = dnNode[base + sl][0];
                if (pe >= 0 && t.begin[n] != pe) throw std::logic_error("down task: owned leaves not contiguous");
                if (pb < 0) pb = t.begin[n];
                pe = t.begin[n] + t.count[n];
                dnLeafSlot.push_back(sl);
                dnLeafIdx.push_back(leafOf[n]);
                dnLeafPts.push_back((int)t.begin[n]);
                const int li = leafOf[n];
                dnLeafNear.push_back({(int)dnNearOff.size() - nearBase, nearInPtr[li + 1] - nearInPtr[li]});
                dnNearOff.insert(dnNearOff.end(), nearInOff.begin() + nearInPtr[li], nearInOff.begin() + nearInPtr[li + 1]);
            }
            const int nl = (int)lf.size();
            for (int sl : lf) {
                const int n = dnNode[base + sl][0];
                dnLeafGeom.push_back({t.ncx[n], t.ncy[n], 1.0 / t.nrx[n], 1.0 / t.nry[n]});
            }
            const int ng = (int)lv.size();
            if (ng > kTaskLevels) throw std::logic_error("down task deeper than its record");
            const int nt = (int)dnNode.size() - base;
            dnDesc.push_back({base, nt, (int)dnLeafSlot.size() - nl, nl});
            dnDesc.push_back({(int)std::max<int64_t>(pb, 0), (int)std::max<int64_t>(pe, 0),
                              dnChainPtr[dnChainPtr.size() - 2], (int)anc.size()});
            dnDesc.push_back({nearBase, (int)dnNearOff.size() - nearBase, ng, 0});
            std::array<int, kTaskLevels + 1> gs{};
            for (int g = 0; g < ng; ++g) gs[g] = dnGrp[dnGrp.size() - ng + g] - base;
            gs[ng] = nt;
            dnGrpFix.insert(dnGrpFix.end(), gs.begin(), gs.end());
            dnPtsRange.push_back({(int)std::max<int64_t>(pb, 0), (int)std::max<int64_t>(pe, 0)});
            dnLeafPtr.push_back((int)dnLeafSlot.size());
            dnNearPtr.push_back((int)dnNearOff.size());
            dnMaxNear = std::max(dnMaxNear, (int)dnNearOff.size() - nearBase);
            dnGrpPtr.push_back((int)dnGrp.size());
            dnTaskPtr.push_back((int)dnNode.size());
            dnMaxTask = std::max(dnMaxTask, (int)dnNode.size() - base);
            dnMaxLeaves = std::max(dnMaxLeaves, nl);
        }
    }
    dnTierTask.push_back((int)dnTaskPtr.size() - 1);  // one launch
    dnGrp.push_back((int)dnNode.size());
}

// Cluster plan of the harmonic M2L from the att lists.
void Plan::buildClusters(const Tree& t) {
    hmClPtr.assign(1, 0);
    hmTgt.clear();
    hmPtr.assign(1, 0);
    hmSrc.clear();
    hmBlk.clear();
    hmSlot.clear();
    hmMaxCl = 0;
    hmMaxLds = 0;
    hmDual = 0;
    hmCopyOwner.clear();
    hmCopyOther.clear();
    const int nt = (int)m2lTgt.size();
    if (nt == 0) return;
    // cluster key: (level, ancestor kClusterDepth levels up); targets keep id order
    std::vector<int> widx(t.nn, -1);
    for (int w = 0; w < nt; ++w) widx[m2lTgt[w]] = w;
    // cluster depth: the deepest (largest clusters, most in-cluster pairs) that still
    // gives >= kMinClusters workgroups, so a shard of an N-GPU run keeps the chip
    // busy (1M points, 8 ranks: depth 3 = 174 clusters, M2L 0.31 ms; depth 2 = 685,
    // 0.17 ms; one rank: depth 3 = 1,367 clusters is best; tools/shard_time.py)
    auto clusterCount = [&](int dp) {
        std::unordered_map<int64_t, char> seen;
        for (int w = 0; w < nt; ++w) {
            int a = m2lTgt[w];
            for (int k = 0; k < dp && t.parent[a] != -1; ++k) a = t.parent[a];
            seen[((int64_t)t.level[m2lTgt[w]] << 32) | (uint32_t)a] = 1;
        }
        return (int)seen.size();
    };
    if (const char* e = std::getenv("ANISO_HM_HALO")) hmHalo = e[0] != '0';
    // the halo form reads every stored block once whatever the cluster size, so its
    // clusters are 16 targets (depth 2: 44 LDS slots at most, 3 workgroups per CU)
    // where the copy form needs 64 for its in-cluster share (1M points, one GPU:
    // 1.225 against 1.273 ms per block matvec, M2L alone 0.73 against 0.84 ms, r04c)
    int depth = hmHalo ? 2 : kClusterDepth;
    while (depth > 1 && clusterCount(depth) < kMinClusters) --depth;
    if (const char* e = std::getenv("ANISO_HM_CLDEPTH"))  // tuning/experiments only (1..kClusterDepth)
        depth = std::max(1, std::min(kClusterDepth, std::atoi(e)));
    hmDepth = depth;
    // targets above the bottom up tier (at or above it on a shard: its roots arrive
    // by the all-gather) read multipoles the upper tiers produce; in the fused launch
    // their clusters may wait for them, so they form small clusters (<= 16 targets)
    // that go last
    const int upperBelow = tierRootLevel.empty() ? 0 : tierRootLevel[0] + (nranks > 1 ? 1 : 0);
    auto upper = [&](int w) { return t.level[m2lTgt[w]] < upperBelow; };
    // their clusters wait for the tier chain, so their run time is the launch's tail:
    // on a shard 4-target clusters, one target per wave (8 shards: 0.267-0.271 ms per
    // block matvec against 0.279-0.289 with 16-target ones, r03t); on one GPU they are
    // 6 % of the clusters and 16-target ones stay
    int upperDepth = nranks > 1 ? 1 : 2;
    if (const char* e = std::getenv("ANISO_HM_UPPER_DEPTH"))  // experiments only (0..2)
        upperDepth = std::max(0, std::min(2, std::atoi(e)));
    std::vector<int64_t> key(nt);
    auto keyAt = [&](int w, int dp) {
        int a = m2lTgt[w];
        for (int k = 0; k < dp && t.parent[a] != -1; ++k) a = t.parent[a];
        return ((int64_t)t.level[m2lTgt[w]] << 32) | (uint32_t)a;
    };
    for (int w = 0; w < nt; ++w) key[w] = keyAt(w, upper(w) ? std::min(depth, upperDepth) : depth);
    // the launch's tail: its last round of clusters drains over one cluster run time
    // (one GPU: 768 slots, 5,462 near-equal clusters of ~106 us; r05zo trace).  The
    // tailSplit lightest regular clusters are split into depth-1 (4-target) ones that
    // run after the upper clusters, so the last units are ~4x shorter: min(400, 1/4 of
    // the regular clusters) -- one GPU 1.155 -> 1.122 ms per block matvec (300-600 alike),
    // a rank of 8 (812 clusters) 0.202 -> 0.200 / 0.210 -> 0.206 ms with 200 (r05zq, r05zr)
    std::vector<char> split(nt, 0);
    if (depth > 1) {
        std::unordered_map<int64_t, int64_t> wk;
        for (int w = 0; w < nt; ++w)
            if (!upper(w)) wk[key[w]] += attPtr[w + 1] - attPtr[w];
        int tailSplit = std::min(400, (int)wk.size() / 4);
        if (const char* e = std::getenv("ANISO_HM_TAIL")) tailSplit = std::max(0, std::atoi(e));  // experiments
        std::vector<std::pair<int64_t, int64_t>> ws(wk.begin(), wk.end());  // key, weight
        std::sort(ws.begin(), ws.end(), [](const auto& a, const auto& b) {
            return a.second != b.second ? a.second < b.second : a.first < b.first;
        });
        std::unordered_map<int64_t, char> lite;
        for (size_t i = 0; i < ws.size() && (int)i < tailSplit; ++i) lite[ws[i].first] = 1;
        for (int w = 0; w < nt; ++w)
            if (!upper(w) && lite.count(key[w])) {
                split[w] = 1;
                key[w] = keyAt(w, 1);
            }
    }
    std::vector<int> order(nt);
    for (int w = 0; w < nt; ++w) order[w] = w;
    std::stable_sort(order.begin(), order.end(), [&](int x, int y) { return key[x] < key[y]; });
    {
        // launch order: heaviest cluster first (its att pairs), so the workgroups
        // dispatched last are short ones and the tail of the launch stays full; the
        // upper-level clusters after the others, the split tail clusters last
        std::vector<std::array<int64_t, 4>> seg;  // class, -weight, begin, end in `order`
        for (int k = 0; k < nt;) {
            int e = k;
            int64_t wgt = 0;
            for (; e < nt && key[order[e]] == key[order[k]]; ++e) wgt += attPtr[order[e] + 1] - attPtr[order[e]];
            seg.push_back({split[order[k]] ? 2 : upper(order[k]) ? 1 : 0, -wgt, k, e});
            k = e;
        }
        std::stable_sort(seg.begin(), seg.end(), [](const auto& a, const auto& b) {
            return a[0] != b[0] ? a[0] < b[0] : a[1] < b[1];
        });
        std::vector<int> o2;
        o2.reserve(nt);
        for (const auto& g : seg) o2.insert(o2.end(), order.begin() + g[2], order.begin() + g[3]);
        order.swap(o2);
    }
    std::vector<int> clOf(t.nn, -1), slotOf(t.nn, -1);
    int nc = 0;
    for (int k = 0; k < nt; ++k) {
        if (k > 0 && key[order[k]] != key[order[k - 1]]) {
            hmClPtr.push_back(k);
            ++nc;
        }
        const int n = m2lTgt[order[k]];
        clOf[n] = nc;
        slotOf[n] = k - hmClPtr.back();
        hmTgt.push_back(n);
    }
    hmClPtr.push_back(nt);
    for (size_t c = 0; c + 1 < hmClPtr.size(); ++c) hmMaxCl = std::max(hmMaxCl, hmClPtr[c + 1] - hmClPtr[c]);
    hmNDir.clear();
    hmHaloPtr.assign(1, 0);
    hmHaloNode.clear();
    hmFoldPtr.assign(1, 0);
    hmFoldNode.clear();
    hmFoldIdx.clear();
    std::vector<int> dSrc, dBlk, dSlot;
    std::vector<int> haloOf(t.nn, -1);
    for (size_t c = 0; c + 1 < hmClPtr.size(); ++c) {
        const int ncl = hmClPtr[c + 1] - hmClPtr[c], h0 = (int)hmHaloNode.size();
        for (int k = hmClPtr[c]; k < hmClPtr[c + 1]; ++k) {
            const int n = hmTgt[k], w = widx[n];
            dSrc.clear();
            dBlk.clear();
            dSlot.clear();
            for (int64_t e = attPtr[w]; e < attPtr[w + 1]; ++e) {
                const int b = attSrc[e];
                // a V pair with both ends targets (X pairs join different levels)
                const bool vt = clOf[b] >= 0 && t.level[b] == t.level[n];
                const bool same = vt && clOf[b] == clOf[n];
                if (vt && b > n && attBlk[e] >= 0 && (same || hmHalo)) {  // canonical end: one read, both products
                    dSrc.push_back(b);
                    dBlk.push_back(attBlk[e]);
                    if (same) {
                        dSlot.push_back(slotOf[b]);
                    } else {  // the partner's product goes to a halo slot of this cluster
                        if (haloOf[b] < 0) {
                            haloOf[b] = (int)hmHaloNode.size() - h0;
                            hmHaloNode.push_back(b);
                        }
                        dSlot.push_back(ncl + haloOf[b]);
                    }
                    continue;
                }
                if (vt && b < n && (same || hmHalo)) continue;  // applied by b's wave (dual)
                hmSrc.push_back(b);
                if (attBlk[e] < 0) {  // a transposed read: read a directed copy of the block instead
                    hmBlk.push_back((int)(attOwner.size() + hmCopyOwner.size()));
                    hmCopyOwner.push_back(n);
                    hmCopyOther.push_back(b);
                } else {
                    hmBlk.push_back(attBlk[e]);
                }
                hmSlot.push_back(-1);
            }
            hmNDir.push_back((int)(hmSrc.size() - hmPtr.back()));
            hmSrc.insert(hmSrc.end(), dSrc.begin(), dSrc.end());
            hmBlk.insert(hmBlk.end(), dBlk.begin(), dBlk.end());
            hmSlot.insert(hmSlot.end(), dSlot.begin(), dSlot.end());
            hmDual += (int64_t)dSrc.size();
            hmPtr.push_back((int64_t)hmSrc.size());
        }
        for (size_t h = h0; h < hmHaloNode.size(); ++h) haloOf[hmHaloNode[h]] = -1;
        hmHaloPtr.push_back((int)hmHaloNode.size());
        hmMaxLds = std::max(hmMaxLds, ncl + (int)hmHaloNode.size() - h0);
    }
    // the fold: per receiving node, its halo slots in cluster order (a fixed order),
    // stored receiver-contiguously (hmHaloPos)
    std::vector<std::vector<int>> recv(t.nn);
    for (size_t h = 0; h < hmHaloNode.size(); ++h) recv[hmHaloNode[h]].push_back((int)h);
    hmHaloPos.assign(hmHaloNode.size(), -1);
    hmFoldOf.assign(t.nn, 0);
    for (int n = 0; n < t.nn; ++n) {
        if (recv[n].empty()) continue;
        if (recv[n].size() > 7 || hmFoldIdx.size() >= (1u << 27)) throw std::logic_error("halo fold record overflow");
        hmFoldOf[n] = (int)((hmFoldIdx.size() << 3) | recv[n].size());
        for (size_t j = 0; j < recv[n].size(); ++j) hmHaloPos[recv[n][j]] = (int)(hmFoldIdx.size() + j);
        hmFoldNode.push_back(n);
        hmFoldIdx.insert(hmFoldIdx.end(), recv[n].begin(), recv[n].end());
        hmFoldPtr.push_back((int)hmFoldIdx.size());
    }
}

// Exchange plan of the sharded up pass (the reference
// runs upPass over the whole tree, bbfmm.h:825-861, and M2L reads src.nodeCharge
// of any V/X member, bbfmm.h:1051-1065).  What this rank reads below the tier-0
// root level L0 -- multipoles of its M2L sources there, the weighted charges of its
// near-field sources, of its correction stencil's 3x3 squares and of its own
// points -- lives in a few tier-0 subtrees around its range; it runs those tasks.
// Everything at or above L0 comes from the tier-0 roots, which each rank receives
// from their owners (the rank holding the root's first point).
// Fused top-of-tree launch (harmonic.hip k_top_m2l_hc): the upper up tier whose
// multipoles each cluster reads, its targets' own (the in-cluster dual products)
// included.  Tier k >= 1 writes its tasks' nodes; a sharded apply's tier 1 also
// stores the gathered tier-0 roots (up_task's recv copy), so those count as tier 1.
void Plan::buildTopWait(const Tree& t) {
    hmClWait.assign(hmClPtr.empty() ? 0 : hmClPtr.size() - 1, 0);
    const int ntier = (int)upTierTask.size() - 1;
    if (ntier < 2 || hmClWait.empty()) return;
    std::vector<int> prod(t.nn, 0);
    for (int k = 1; k < ntier; ++k)
        for (int task = upTierTask[k]; task < upTierTask[k + 1]; ++task)
            for (int i = upDesc[task][0]; i < upDesc[task][0] + upDesc[task][1]; ++i) prod[upNode[i]] = k;
    if (nranks > 1)
        for (int task = upTierTask[0]; task < upTierTask[1]; ++task) prod[upTaskRoot[task]] = 1;
    for (size_t c = 0; c + 1 < hmClPtr.size(); ++c) {
        int w = 0;
        for (int k = hmClPtr[c]; k < hmClPtr[c + 1]; ++k) {
            w = std::max(w, prod[hmTgt[k]]);
            for (int64_t e = hmPtr[k]; e < hmPtr[k + 1]; ++e) w = std::max(w, prod[hmSrc[e]]);
        }
        hmClWait[c] = w;
    }
}

void Plan::buildExchange(const Tree& t, int sz, int d2) {
    const int64_t N = t.count[0];
    // the fused corrections of the staged near field (d = 1: a square is one point)
    nearCorrRow.clear();
    nearCorrOk = false;
    if (d2 == 1 && sz > 0 && nsMax > 0 && !leaves.empty()) {
        std::vector<int> ip(N), rowTmp(N, -1);
        for (int64_t k = 0; k < N; ++k) ip[t.perm[k]] = (int)k;
        nearCorrRow.assign(leaves.size() * 16 * 9, 0xFFFF);
        bool ok = true;
        for (size_t g0 = 0; g0 < leaves.size() && ok; g0 += 16) {
            const int64_t r0 = nsPtr[g0 / 16], r1 = nsPtr[g0 / 16 + 1];
            for (int64_t r = r0; r < r1; ++r) rowTmp[nsPts[r]] = (int)(r - r0);
            for (size_t l = g0; l < std::min(leaves.size(), g0 + 16) && ok; ++l)
                for (int64_t r = 0; r < t.count[leaves[l]] && ok; ++r) {
                    const int tt = t.perm[t.begin[leaves[l]] + r], i = tt / sz, j = tt % sz;
                    for (int q9 = 0; q9 < 9; ++q9) {
                        const int di = q9 / 3 - 1, dj = q9 % 3 - 1;
                        if (i + di < 0 || i + di >= sz || j + dj < 0 || j + dj >= sz) continue;
                        const int row = rowTmp[ip[tt + di * sz + dj]];
                        if (row < 0) {
                            ok = false;
                            break;
                        }
                        nearCorrRow[(l * 16 + r) * 9 + q9] = (uint16_t)row;
                    }
                }
            for (int64_t r = r0; r < r1; ++r) rowTmp[nsPts[r]] = -1;
        }
        nearCorrOk = ok;
        if (!ok) nearCorrRow.clear();
    }
    xT0Tasks.clear();
    xOwnT0Tasks.clear();
    nearGrpEarly.clear();
    nearGrpLate.clear();
    xNeedNodes.clear();
    xOneHalo.clear();
    xOneHaloPoints = 0;
    xOneOk = false;
    xUpPartial = false;
    xUpTop = 0;
    xUpTask.clear();
    xUpRecNode.clear();
    xT0Part.clear();
    xUpRoots.clear();
    xRootSend.clear();
    xRootRecv.clear();
    xRootSlot.clear();
    xSendSlot.clear();
    xRootChunk = 0;
    xHalo.clear();
    xHaloPoints = 0;
    std::vector<char> need(N, 0);  // tree positions this rank's kernels read
    for (int64_t k = ownBegin; k < ownEnd; ++k) need[k] = 1;
    for (int p : nearPts) need[p] = 1;
    if (sz > 0 && d2 > 0) {  // k_corr: the 3x3 squares around each own target (incl. its own square)
        std::vector<int> iperm(N);
        for (int64_t k = 0; k < N; ++k) iperm[t.perm[k]] = (int)k;
        for (int64_t k = ownBegin; k < ownEnd; ++k) {
            const int sq = t.perm[k] / d2, i = sq / sz, j = sq % sz;
            for (int dr = -1; dr <= 1; ++dr)
                for (int dc = -1; dc <= 1; ++dc) {
                    if (i + dr < 0 || i + dr >= sz || j + dc < 0 || j + dc >= sz) continue;
                    const int64_t q = (int64_t)(sq + dr * sz + dc) * d2;
                    for (int c = 0; c < d2; ++c) need[iperm[q + c]] = 1;
                }
        }
    }
    const bool tiers = upTierTask.size() >= 2;
    if (!tiers) {  // a lone leaf: no up tasks, every point is read by the one apply
        if (ownBegin > 0) xHalo.insert(xHalo.end(), {0, ownBegin});
        if (ownEnd < N) xHalo.insert(xHalo.end(), {ownEnd, N});
        xHaloPoints = N - (ownEnd - ownBegin);
        return;
    }
    const int L0 = tierRootLevel[0];
    const int t0 = upTierTask[0], t1 = upTierTask[1];
    std::vector<int> taskOf(t.nn, -1);  // tier-0 root -> task
    for (int k = t0; k < t1; ++k) taskOf[upTaskRoot[k]] = k;
    std::vector<char> runs(t1 - t0, 0);
    auto markNode = [&](int n) {  // a multipole below L0: the tier-0 task that computes it
        if (t.level[n] <= L0) return;
        while (t.level[n] > L0) n = t.parent[n];
        if (taskOf[n] >= 0) runs[taskOf[n] - t0] = 1;
    };
    for (int n : m2lTgt) {
        for (int64_t k = t.vPtr[n]; k < t.vPtr[n + 1]; ++k)
            if (!t.isEmpty[t.vIdx[k]]) markNode(t.vIdx[k]);
        for (int64_t k = t.xPtr[n]; k < t.xPtr[n + 1]; ++k)
            if (!t.isEmpty[t.xIdx[k]]) markNode(t.xIdx[k]);
    }
    std::vector<char> valid(N, 0);  // input positions the rank's up tasks read
    std::vector<char> covered(N, 0);
    for (int k = t0; k < t1; ++k) {
        const int r = upTaskRoot[k];
        const int64_t b = t.begin[r], e = b + t.count[r];
        for (int64_t p = b; p < e; ++p) {
            covered[p] = 1;
            if (need[p]) runs[k - t0] = 1;
        }
        if (runs[k - t0]) {
            xT0Tasks.push_back(k);
            for (int64_t p = b; p < e; ++p) valid[p] = 1;
        }
    }
    for (int64_t p = 0; p < N; ++p)  // leaves above L0 (P2M in the tiers every rank runs)
        if (!covered[p]) valid[p] = 1;
    for (int64_t p = 0; p < N; ++p)
        if (need[p] && !valid[p]) throw std::logic_error("exchange plan: a read position outside the rank's up tasks");
    for (int64_t p = 0; p < N;) {
        if (!valid[p] || (p >= ownBegin && p < ownEnd)) {
            ++p;
            continue;
        }
        int64_t e = p;
        while (e < N && valid[e] && !(e >= ownBegin && e < ownEnd)) ++e;
        xHalo.push_back(p);
        xHalo.push_back(e);
        xHaloPoints += e - p;
        p = e;
    }
    // the all-gather of the tier-0 roots: slot layout of every rank's contribution
    const std::vector<int64_t> cuts = shard_cuts(t, nranks);
    std::vector<std::vector<int>> owned(nranks);
    for (int k = t0; k < t1; ++k) {
        const int r = upTaskRoot[k];
        const int o = (int)(std::upper_bound(cuts.begin() + 1, cuts.end() - 1, t.begin[r]) - (cuts.begin() + 1));
        owned[o].push_back(r);
    }
    for (auto& v : owned) xRootChunk = std::max<int>(xRootChunk, (int)v.size());
    xRootRecv.assign((size_t)nranks * xRootChunk, -1);
    for (int q = 0; q < nranks; ++q)
        std::copy(owned[q].begin(), owned[q].end(), xRootRecv.begin() + (size_t)q * xRootChunk);
    xRootSend = owned[rank];
    xRootSlot.assign(t.nn, -1);
    for (size_t k = 0; k < xRootRecv.size(); ++k)
        if (xRootRecv[k] >= 0) xRootSlot[xRootRecv[k]] = (int)k;
    xSendSlot.assign(t.nn, -1);
    for (size_t j = 0; j < xRootSend.size(); ++j) xSendSlot[xRootSend[j]] = (int)j;
    for (int r : xRootSend)
        if (!runs[taskOf[r] - t0]) throw std::logic_error("exchange plan: a sent root's task does not run here");
    // ---- the one-collective form: own tier-0 tasks only, the rest comes from the owners
    auto ownerOf = [&](int64_t pos) {
        return (int)(std::upper_bound(cuts.begin() + 1, cuts.end() - 1, pos) - (cuts.begin() + 1));
    };
    bool ok = true;
    for (int r : xRootSend) {
        xOwnT0Tasks.push_back(taskOf[r]);
        ok = ok && t.begin[r] >= ownBegin && t.begin[r] + t.count[r] <= ownEnd;
    }
    std::sort(xOwnT0Tasks.begin(), xOwnT0Tasks.end());
    // the upper multipoles as partial sums: every point under a tier-0 root (no P2M
    // above L0), two levels above the roots, and this rank's roots inside its range
    bool allCovered = true;
    for (int64_t p = 0; p < N && allCovered; ++p) allCovered = covered[p] != 0;
    xUpPartial = xUpPartialIn && ok && nranks > 1 && allCovered && L0 >= 2;
    std::vector<char> needNode(t.nn, 0);
    auto markNeed = [&](int n) {  // a multipole below L0 (at L0: partial sums) in another rank's subtree
        if (t.level[n] >= (xUpPartial ? L0 : L0 + 1) && ownerOf(t.begin[n]) != rank) needNode[n] = 1;
    };
    for (int n : m2lTgt) {
        for (int64_t k = t.vPtr[n]; k < t.vPtr[n + 1]; ++k)
            if (!t.isEmpty[t.vIdx[k]]) markNeed(t.vIdx[k]);
        for (int64_t k = t.xPtr[n]; k < t.xPtr[n + 1]; ++k)
            if (!t.isEmpty[t.xIdx[k]]) markNeed(t.xIdx[k]);
    }
    for (int n = 0; n < t.nn; ++n)
        if (needNode[n]) xNeedNodes.push_back(n);
    for (int64_t p = 0; p < N;) {  // the input this rank reads outside its range: near, stencil, upper-tier P2M
        auto want = [&](int64_t q) { return (need[q] || !covered[q]) && !(q >= ownBegin && q < ownEnd); };
        if (!want(p)) {
            ++p;
            continue;
        }
        int64_t e = p;
        while (e < N && want(e)) ++e;
        xOneHalo.push_back(p);
        xOneHalo.push_back(e);
        xOneHaloPoints += e - p;
        p = e;
    }
    xOneOk = ok && nranks > 1;
    if (xUpPartial) {
        // xUpTop: the topmost level above L0 whose multipoles an M2L reads (V / X
        // sources, or targets with a list: their own multipole feeds the dual products)
        xUpTop = L0;
        for (int n = 0; n < t.nn; ++n) {
            if (t.isEmpty[n]) continue;
            const bool lists = t.vPtr[n + 1] > t.vPtr[n] || t.xPtr[n + 1] > t.xPtr[n];
            if (lists) xUpTop = std::min(xUpTop, t.level[n]);
            for (int64_t k = t.xPtr[n]; k < t.xPtr[n + 1]; ++k) xUpTop = std::min(xUpTop, t.level[t.xIdx[k]]);
        }
        const int La = L0 - 2;
        if (La - xUpTop > kUpChainMax) throw std::logic_error("upper partials: chain deeper than its record");
        auto quadrant = [&](int n) {
            const int p = t.parent[n];
            for (int q = 0; q < 4; ++q)
                if (t.child[p][q] == n) return q;
            throw std::logic_error("upper partials: a node is not its parent's child");
        };
        // tasks in tree order of A; a task's roots by their slot under A
        std::vector<int> tops;
        std::vector<int> taskOfTop(t.nn, -1);
        for (int r : xRootSend) {
            const int A = t.parent[t.parent[r]];
            if (taskOfTop[A] < 0) {
                taskOfTop[A] = (int)tops.size();
                tops.push_back(A);
            }
        }
        std::vector<int> order(tops.size());
        for (size_t i = 0; i < order.size(); ++i) order[i] = (int)i;
        std::sort(order.begin(), order.end(), [&](int a, int b) { return t.begin[tops[a]] < t.begin[tops[b]]; });
        std::vector<std::array<int, kUpTaskInts>> recs(tops.size());
        for (auto& a : recs) a.fill(-1);
        for (int r : xRootSend) {
            const int mid = t.parent[r];
            auto& a = recs[taskOfTop[t.parent[mid]]];
            a[4 * quadrant(mid) + quadrant(r)] = r;
        }
        for (int i : order) {
            auto& a = recs[i];
            const int A = tops[i];
            for (int q1 = 0; q1 < 4; ++q1) {
                const bool has = a[4 * q1] >= 0 || a[4 * q1 + 1] >= 0 || a[4 * q1 + 2] >= 0 || a[4 * q1 + 3] >= 0;
                if (has && L0 - 1 >= xUpTop) {
                    a[16 + q1] = (int)xUpRecNode.size();
                    xUpRecNode.push_back(t.child[A][q1]);
                }
            }
            if (La >= xUpTop) {
                a[20] = (int)xUpRecNode.size();
                xUpRecNode.push_back(A);
            }
            const int nc = std::max(La - xUpTop, 0);
            a[21] = nc;
            int n = A;
            for (int c = 0; c < kUpChainMax; ++c) {
                a[22 + c] = 0;
                if (c >= nc) continue;
                a[22 + c] = quadrant(n);
                n = t.parent[n];
                a[30 + c] = (int)xUpRecNode.size();
                xUpRecNode.push_back(n);
            }
            a[38] = A;
            a[39] = 0;
            xUpTask.insert(xUpTask.end(), a.begin(), a.end());
        }
        // the tails: each own tier-0 task's partial task (its root's grandparent), in
        // xUpTask's order, and how many roots each one waits for
        std::vector<int> pos(tops.size());
        for (size_t k = 0; k < order.size(); ++k) pos[order[k]] = (int)k;
        xUpRoots.assign(tops.size(), 0);
        xT0Part.assign(2 * xOwnT0Tasks.size(), -1);
        for (size_t i = 0; i < xOwnT0Tasks.size(); ++i) {
            const int r = upTaskRoot[xOwnT0Tasks[i]];
            const int pt = pos[taskOfTop[t.parent[t.parent[r]]]];
            int q = 0;
            while (q < 16 && xUpTask[(size_t)pt * kUpTaskInts + q] != r) ++q;
            if (q == 16) throw std::logic_error("upper partials: a root is not in its task");
            xT0Part[2 * i] = 16 * pt + q;
            xT0Part[2 * i + 1] = r;
            ++xUpRoots[pt];
        }
        for (size_t pt = 0; pt < xUpRoots.size(); ++pt) {  // every tail waits for exactly its task's roots
            int slots = 0;
            for (int i = 0; i < 16; ++i) slots += xUpTask[pt * kUpTaskInts + i] >= 0;
            if (slots != xUpRoots[pt]) throw std::logic_error("upper partials: a tail's root count differs from its task");
        }
    }
    nearGrpEarly.clear();
    nearGrpLate.clear();
    for (size_t g = 0; g + 1 < nsPtr.size(); ++g) {
        bool own = true;
        for (int64_t r = nsPtr[g]; r < nsPtr[g + 1] && own; ++r) own = nsPts[r] >= ownBegin && nsPts[r] < ownEnd;
        (own ? nearGrpEarly : nearGrpLate).push_back((int)g);
    }
}

}  // namespace aniso
