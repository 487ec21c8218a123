// capi.cpp -- extern "C" boundary over aniso::Operator.  No exception crosses
// the ABI: every failure becomes a status code + thread-local message.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <new>
#include <stdexcept>
#include <string>

#include "../../include/aniso_mi355x.h"
#include "../../include/aniso_mi355x_dev.h"
#include "aniso_op.hpp"
#include "kernels.hpp"

namespace aniso {
[[noreturn]] void throw_hip(hipError_t e, const char* file, int line);
}  // namespace aniso

struct aniso_op_s {
    uint64_t magic = 0xA2150A2150ULL;
    aniso::Operator op;
    template <class... A>
    explicit aniso_op_s(A... a) : op(a...) {}
};

namespace {
thread_local std::string g_err;

template <class F>
int guarded(F&& f) {
    try {
        g_err.clear();
        f();
        return ANISO_OK;
    } catch (const std::out_of_range& e) {
        g_err = e.what();
        return ANISO_ERR_RANGE;
    } catch (const std::invalid_argument& e) {
        g_err = e.what();
        return ANISO_ERR_INVALID;
    } catch (const std::logic_error& e) {
        g_err = e.what();
        return ANISO_ERR_STATE;
    } catch (const std::bad_alloc&) {
        g_err = "host out of memory";
        return ANISO_ERR_RUNTIME;
    } catch (const std::runtime_error& e) {
        g_err = e.what();
        std::string w = e.what();
        return (w.find("before") != std::string::npos) ? ANISO_ERR_STATE : ANISO_ERR_RUNTIME;
    } catch (...) {
        g_err = "unknown error";
        return ANISO_ERR_RUNTIME;
    }
}

// Every call that may touch the device runs on the handle's device and leaves the
// caller's current device as it found it (a process driving several GPUs).
struct DeviceRestore {
    int prev = -1;
    explicit DeviceRestore(aniso_handle h) {
        if (h && h->magic == 0xA2150A2150ULL && h->op.deviceId() >= 0) (void)hipGetDevice(&prev);
    }
    ~DeviceRestore() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

aniso::Operator& get(aniso_handle h) {
    if (!h || h->magic != 0xA2150A2150ULL) throw std::invalid_argument("invalid aniso handle");
    return h->op;
}

// validates the handle (returns ANISO_ERR_HANDLE from the calling entry point)
#define CHECK_HANDLE(h)                              \
    do {                                             \
        if (!(h) || (h)->magic != 0xA2150A2150ULL) { \
            g_err = "invalid aniso handle";          \
            return ANISO_ERR_HANDLE;                 \
        }                                            \
    } while (0)
// restores the caller's current HIP device when the entry point returns
#define DEVICE_GUARD(h) DeviceRestore device_guard_((h))
// the two above, at the top of every entry point that takes a handle
#define ENTER(h)     \
    CHECK_HANDLE(h); \
    DEVICE_GUARD(h)

#define CHECK_PTR(p)                                                         \
    do {                                                                     \
        if (!(p)) throw std::invalid_argument(std::string(#p) + " is NULL"); \
    } while (0)
}  // namespace

extern "C" {

int aniso_create(int sz, int d, int ks, double g, int ns, int np, int maxLevel, aniso_handle* out) {
    return guarded([&] {
        CHECK_PTR(out);
        *out = nullptr;
        *out = new aniso_op_s(sz, d, ks, g, ns, np, maxLevel);
    });
}

int aniso_destroy(aniso_handle h) {
    ENTER(h);
    return guarded([&] {
        h->magic = 0;
        delete h;
    });
}

int aniso_num_nodes(aniso_handle h, int64_t* n) {
    ENTER(h);
    return guarded([&] {
        CHECK_PTR(n);
        *n = get(h).numNodes();
    });
}

int aniso_num_blocks(aniso_handle h, int* ks) {
    ENTER(h);
    return guarded([&] {
        CHECK_PTR(ks);
        *ks = get(h).ks;
    });
}

int aniso_sync(aniso_handle h) {
    ENTER(h);
    return guarded([&] { get(h).sync(); });
}

int aniso_get_nodes(aniso_handle h, double* xy) {
    ENTER(h);
    return guarded([&] {
        CHECK_PTR(xy);
        get(h).getNodes(xy);
    });
}

int aniso_get_weights(aniso_handle h, double* w) {
    ENTER(h);
    return guarded([&] {
        CHECK_PTR(w);
        auto& op = get(h);
        std::memcpy(w, op.geo.w.data(), op.geo.N * sizeof(double));
    });
}

int aniso_set_coeff(aniso_handle h, const double* ss, const double* st) {
    ENTER(h);
    return guarded([&] {
        CHECK_PTR(ss);
        CHECK_PTR(st);
        get(h).setCoeff(ss, st);
    });
}

int aniso_cache(aniso_handle h, int id) {
    ENTER(h);
    return guarded([&] { get(h).cache(id); });
}

int aniso_mapping(aniso_handle h, const double* charge, int id, double* out) {
    ENTER(h);
    return guarded([&] {
        CHECK_PTR(charge);
        CHECK_PTR(out);
        get(h).mappingHost(charge, id, out);
    });
}

int aniso_mapping_dev(aniso_handle h, const double* charge, int id, double* out, void* stream) {
    ENTER(h);
    return guarded([&] {
        CHECK_PTR(charge);
        CHECK_PTR(out);
        get(h).mappingDev(charge, id, out, (hipStream_t)stream, aniso::kStageAll);
    });
}

int aniso_mapping_stages_dev(aniso_handle h, const double* charge, int id, int mask, double* out, void* stream) {
    ENTER(h);
    return guarded([&] {
        CHECK_PTR(charge);
        CHECK_PTR(out);
        if (mask < 0 || mask > aniso::kStageAll) throw std::invalid_argument("bad stage mask");
        get(h).mappingDev(charge, id, out, (hipStream_t)stream, mask);
    });
}

int aniso_mapping_batched(aniso_handle h, const double* Q, int k, int id, double* Out) {
    ENTER(h);
    return guarded([&] {
        CHECK_PTR(Q);
        CHECK_PTR(Out);
        if (k < 0) throw std::invalid_argument("k must be >= 0");
        auto& op = get(h);
        op.mappingBatchedHost(Q, k, id, Out);
    });
}

int aniso_forward_dev(aniso_handle h, const double* u, double* out, void* stream) {
    ENTER(h);
    return guarded([&] {
        CHECK_PTR(u);
        CHECK_PTR(out);
        auto& op = get(h);
        if (!op.modeCached(0)) throw std::runtime_error("forward operator before cache(0)");
        op.forwardDev(u, out, (hipStream_t)stream);
    });
}

int aniso_mapping_tree_dev(aniso_handle h, const double* q_tree, int id, double* out_slice, void* stream) {
    ENTER(h);
    return guarded([&] {
        CHECK_PTR(q_tree);
        CHECK_PTR(out_slice);
        get(h).mappingTreeDev(q_tree, id, out_slice, (hipStream_t)stream);
    });
}

int aniso_forward_tree_dev(aniso_handle h, const double* x_tree, double* y_slice, void* stream) {
    ENTER(h);
    return guarded([&] {
        CHECK_PTR(x_tree);
        CHECK_PTR(y_slice);
        auto& op = get(h);
        if (!op.modeCached(0)) throw std::runtime_error("forward operator before cache(0)");
        op.forwardTreeDev(x_tree, y_slice, (hipStream_t)stream);
    });
}

int aniso_forward_tree_begin_dev(aniso_handle h, const double* x_tree, double* y_slice, double* roots_send,
                                 void* stream) {
    ENTER(h);
    return guarded([&] {
        CHECK_PTR(x_tree);
        CHECK_PTR(y_slice);
        get(h).forwardTreePhase(1, x_tree, y_slice, roots_send, nullptr, (hipStream_t)stream);
    });
}

int aniso_forward_tree_end_dev(aniso_handle h, const double* x_tree, double* y_slice, const double* roots_recv,
                               void* stream) {
    ENTER(h);
    return guarded([&] {
        CHECK_PTR(x_tree);
        CHECK_PTR(y_slice);
        get(h).forwardTreePhase(2, x_tree, y_slice, nullptr, roots_recv, (hipStream_t)stream);
    });
}

int aniso_forward_f32_dev(aniso_handle h, const float* x, float* y, void* stream) {
    ENTER(h);
    return guarded([&] {
        CHECK_PTR(x);
        CHECK_PTR(y);
        get(h).forwardF32Dev(x, y, (hipStream_t)stream);
    });
}

int aniso_forward16_f64_dev(aniso_handle h, const double* x, double* y, void* stream) {
    ENTER(h);
    return guarded([&] {
        CHECK_PTR(x);
        CHECK_PTR(y);
        get(h).mrhs64Dev(0, true, x, y, (hipStream_t)stream);
    });
}

int aniso_mapping16_f64_dev(aniso_handle h, int id, const double* x, double* y, int mask, void* stream) {
    ENTER(h);
    return guarded([&] {
        CHECK_PTR(x);
        CHECK_PTR(y);
        if (mask < 0 || mask > aniso::kStageAll) throw std::invalid_argument("bad stage mask");
        get(h).mrhs64Dev(id, false, x, y, (hipStream_t)stream, mask);
    });
}

int aniso_forward_f32_stages_dev(aniso_handle h, const float* x, int mask, float* y, void* stream) {
    ENTER(h);
    return guarded([&] {
        CHECK_PTR(x);
        CHECK_PTR(y);
        if (mask < 0 || mask > aniso::kStageAll) throw std::invalid_argument("bad stage mask");
        get(h).forwardF32Dev(x, y, (hipStream_t)stream, mask);
    });
}

int aniso_apply_block_dev(aniso_handle h, int nrhs, const double* x, int64_t ldx, int use_sigma, int nterm,
                          const int* ids, const double* mixes, double* out, int64_t ldo, int tree, void* stream) {
    ENTER(h);
    return guarded([&] {
        CHECK_PTR(x);
        CHECK_PTR(out);
        CHECK_PTR(ids);
        CHECK_PTR(mixes);
        get(h).applyBlockDev(nrhs, x, ldx, tree != 0, use_sigma != 0, nterm, ids, mixes, out, ldo, tree != 0,
                             (hipStream_t)stream);
    });
}

int aniso_block_op_dev(aniso_handle h, int which, const double* x, int64_t ldx, double* out, int64_t ldo, int tree,
                       void* stream) {
    ENTER(h);
    return guarded([&] {
        CHECK_PTR(x);
        CHECK_PTR(out);
        get(h).blockOpDev(which, x, ldx, out, ldo, tree != 0, (hipStream_t)stream);
    });
}

int aniso_block_op_begin_dev(aniso_handle h, int which, const double* x, int64_t ldx, double* out, int64_t ldo,
                             double* roots_send, void* stream) {
    ENTER(h);
    return guarded([&] {
        CHECK_PTR(x);
        CHECK_PTR(out);
        get(h).blockOpDev(which, x, ldx, out, ldo, true, (hipStream_t)stream, NAN, nullptr, 1, roots_send, nullptr);
    });
}

int aniso_block_op_end_dev(aniso_handle h, int which, const double* x, int64_t ldx, double* out, int64_t ldo,
                           const double* roots_recv, void* stream) {
    ENTER(h);
    return guarded([&] {
        CHECK_PTR(x);
        CHECK_PTR(out);
        get(h).blockOpDev(which, x, ldx, out, ldo, true, (hipStream_t)stream, NAN, nullptr, 2, nullptr, roots_recv);
    });
}

int aniso_block_op(aniso_handle h, int which, const double* u, double* out) {
    ENTER(h);
    return guarded([&] {
        CHECK_PTR(u);
        CHECK_PTR(out);
        get(h).blockOpHost(which, u, nullptr, NAN, out);
    });
}

int aniso_apply_block(aniso_handle h, const double* u, const double* sigma_s, double g, double* out) {
    ENTER(h);
    return guarded([&] {
        CHECK_PTR(u);
        CHECK_PTR(sigma_s);
        CHECK_PTR(out);
        if (!(g >= 0.0 && g < 1.0)) throw std::invalid_argument("g must be in [0, 1)");
        get(h).blockOpHost(2, u, sigma_s, g, out);
    });
}

int aniso_block_mixes(int nb, double g, int chi, double* mixes) {
    return guarded([&] {
        CHECK_PTR(mixes);
        const auto m = aniso::Operator::blockMixes(nb, g, chi != 0);
        std::copy(m.begin(), m.end(), mixes);
    });
}

int aniso_gmres(aniso_handle h, const double* q, double* x, int m, int maxit, double tol, double* hist, int maxhist,
                int* iters, double* final_resid) {
    ENTER(h);
    return guarded([&] {
        CHECK_PTR(q);
        CHECK_PTR(x);
        int j = get(h).gmresHost(q, x, m, maxit, tol, hist, hist ? maxhist : 0, final_resid);
        if (iters) *iters = j;
    });
}

int aniso_block_solve(aniso_handle h, const double* rhs, double* x, int restart, double tol, int maxit, double* hist,
                      int maxhist, int* iters, double* relres) {
    ENTER(h);
    return guarded([&] {
        CHECK_PTR(rhs);
        CHECK_PTR(x);
        const int it = get(h).blockSolveHost(rhs, x, restart, tol, maxit, hist, hist ? maxhist : 0, relres);
        if (iters) *iters = it;
    });
}

int aniso_block_solve_dev(aniso_handle h, const double* rhs, double* x, int restart, double tol, int maxit,
                          double* hist, int maxhist, int* iters, double* relres, void* stream) {
    ENTER(h);
    return guarded([&] {
        CHECK_PTR(rhs);
        CHECK_PTR(x);
        auto& op = get(h);
        hipStream_t s = (hipStream_t)stream;
        const int it = op.blockSolveDev(rhs, x, restart, tol, maxit, hist, hist ? maxhist : 0, relres, s);
        if (iters) *iters = it;
    });
}

int aniso_solve16_mixed_dev(aniso_handle h, const double* b, int64_t ldb, double* x, int64_t ldx, int m, double tol,
                            double inner_tol, int max_outer, int max_cycles, int* outer, int* inner, double* relres,
                            void* stream) {
    ENTER(h);
    return guarded([&] {
        CHECK_PTR(b);
        CHECK_PTR(x);
        double rel[16];
        int o = 0;
        const int it = get(h).solve16Mixed(b, ldb, x, ldx, m, tol, inner_tol, max_outer, max_cycles, &o, rel,
                                           (hipStream_t)stream);
        if (outer) *outer = o;
        if (inner) *inner = it;
        if (relres) std::copy(rel, rel + 16, relres);
    });
}

int aniso_set_shard(aniso_handle h, int rank, int nranks) {
    ENTER(h);
    return guarded([&] { get(h).setShard(rank, nranks); });
}

int aniso_shard_cuts(aniso_handle h, int nranks, int64_t* cuts) {
    ENTER(h);
    return guarded([&] {
        CHECK_PTR(cuts);
        const auto c = aniso::shard_cuts(get(h).tree, nranks);
        std::copy(c.begin(), c.end(), cuts);
    });
}

int aniso_set_deterministic(aniso_handle h, int on) {
    ENTER(h);
    return guarded([&] { get(h).setDeterministic(on != 0); });
}

int aniso_shard_exchange(aniso_handle h, int nrhs, int64_t* info) {
    ENTER(h);
    return guarded([&] {
        CHECK_PTR(info);
        if (nrhs < 1 || nrhs > 8) throw std::invalid_argument("nrhs must be in 1..8");
        const auto& p = get(h).plan;
        info[0] = p.xRootChunk;
        info[1] = (int64_t)aniso::kRank * aniso::Operator::rootRhs(nrhs);
        info[2] = (int64_t)p.xHalo.size() / 2;
        info[3] = p.xHaloPoints;
        info[4] = p.tierRootLevel.empty() ? -1 : p.tierRootLevel[0];
        info[5] = (int64_t)p.xT0Tasks.size();
        info[6] = (int64_t)p.xRootSend.size();
        info[7] = p.upTierTask.size() >= 2 ? p.upTierTask[1] - p.upTierTask[0] : 0;
        info[8] = p.nranks;
    });
}

int aniso_shard_exchange_one(aniso_handle h, int64_t* info) {
    ENTER(h);
    return guarded([&] {
        CHECK_PTR(info);
        const auto& p = get(h).plan;
        info[0] = p.xOneOk ? 1 : 0;
        info[1] = (int64_t)p.xOwnT0Tasks.size();
        info[2] = (int64_t)p.xNeedNodes.size();
        info[3] = (int64_t)p.xOneHalo.size() / 2;
        info[4] = p.xOneHaloPoints;
    });
}

int aniso_shard_upper_partials(aniso_handle h, int64_t* info) {
    ENTER(h);
    return guarded([&] {
        CHECK_PTR(info);
        const auto& p = get(h).plan;
        info[0] = p.xUpPartial ? 1 : 0;
        info[1] = (int64_t)(p.xUpTask.size() / aniso::Plan::kUpTaskInts);
        info[2] = (int64_t)p.xUpRecNode.size();
        info[3] = p.xUpTop;
        info[4] = p.tierRootLevel.empty() ? -1 : p.tierRootLevel[0];
        int64_t roots = 0;
        for (size_t t = 0; t < p.xUpTask.size(); t += aniso::Plan::kUpTaskInts)
            for (int i = 0; i < 16; ++i) roots += p.xUpTask[t + i] >= 0;
        info[5] = roots;
    });
}

int aniso_shard_upper_records(aniso_handle h, int* nodes) {
    ENTER(h);
    return guarded([&] {
        CHECK_PTR(nodes);
        const auto& p = get(h).plan;
        std::copy(p.xUpRecNode.begin(), p.xUpRecNode.end(), nodes);
    });
}

int aniso_shard_one_halo(aniso_handle h, int64_t* ranges) {
    ENTER(h);
    return guarded([&] {
        CHECK_PTR(ranges);
        const auto& p = get(h).plan;
        std::copy(p.xOneHalo.begin(), p.xOneHalo.end(), ranges);
    });
}

int aniso_shard_halo(aniso_handle h, int64_t* ranges) {
    ENTER(h);
    return guarded([&] {
        CHECK_PTR(ranges);
        const auto& p = get(h).plan;
        std::copy(p.xHalo.begin(), p.xHalo.end(), ranges);
    });
}

int aniso_shard_roots(aniso_handle h, int* send_nodes, int* recv_nodes, int* t0_roots) {
    ENTER(h);
    return guarded([&] {
        const auto& p = get(h).plan;
        if (send_nodes) std::copy(p.xRootSend.begin(), p.xRootSend.end(), send_nodes);
        if (recv_nodes) std::copy(p.xRootRecv.begin(), p.xRootRecv.end(), recv_nodes);
        if (t0_roots)
            for (int k : p.xT0Tasks) *t0_roots++ = p.upTaskRoot[k];
    });
}

int aniso_get_shard(aniso_handle h, int64_t* b, int64_t* e) {
    ENTER(h);
    return guarded([&] {
        CHECK_PTR(b);
        CHECK_PTR(e);
        get(h).getShard(b, e);
    });
}

int aniso_tree_perm(aniso_handle h, int* perm) {
    ENTER(h);
    return guarded([&] {
        CHECK_PTR(perm);
        auto& t = get(h).tree;
        std::memcpy(perm, t.perm.data(), t.perm.size() * sizeof(int));
    });
}

int aniso_permute_to_tree_dev(aniso_handle h, const double* orig, double* tree, void* stream) {
    ENTER(h);
    return guarded([&] {
        CHECK_PTR(orig);
        CHECK_PTR(tree);
        get(h).permuteToTree(orig, tree, (hipStream_t)stream);
    });
}

int aniso_tree_size(aniso_handle h, int* nnodes, int* max_level) {
    ENTER(h);
    return guarded([&] {
        auto& t = get(h).tree;
        if (nnodes) *nnodes = t.nn;
        if (max_level) *max_level = t.maxLevel;
    });
}

int aniso_tree_nodes(aniso_handle h, int* ints, double* geom) {
    ENTER(h);
    return guarded([&] {
        auto& t = get(h).tree;
        for (int i = 0; i < t.nn; ++i) {
            if (ints) {
                int* o = ints + 11 * (size_t)i;
                o[0] = t.parent[i];
                for (int c = 0; c < 4; ++c) o[1 + c] = t.child[i][c];
                o[5] = t.level[i];
                o[6] = t.slot[i];
                o[7] = t.isLeaf[i];
                o[8] = t.isEmpty[i];
                o[9] = (int)t.count[i];
                o[10] = (int)t.begin[i];
            }
            if (geom) {
                double* g = geom + 4 * (size_t)i;
                g[0] = t.ncx[i];
                g[1] = t.ncy[i];
                g[2] = t.nrx[i];
                g[3] = t.nry[i];
            }
        }
    });
}

int aniso_tree_list(aniso_handle h, int which, int64_t* ptr, int* idx) {
    ENTER(h);
    return guarded([&] {
        auto& t = get(h).tree;
        const std::vector<int64_t>* P[4] = {&t.uPtr, &t.vPtr, &t.wPtr, &t.xPtr};
        const std::vector<int>* I[4] = {&t.uIdx, &t.vIdx, &t.wIdx, &t.xIdx};
        if (which < 0 || which > 3) throw std::invalid_argument("which must be 0..3");
        CHECK_PTR(ptr);
        std::memcpy(ptr, P[which]->data(), P[which]->size() * sizeof(int64_t));
        if (idx) std::memcpy(idx, I[which]->data(), I[which]->size() * sizeof(int));
    });
}

constexpr int kStatsV1 = 26, kStats = 34;  // aniso_stats: the 26 entries its round-4 contract promised

static void stats_fill(aniso::Operator& op, int64_t* s) {
    s[0] = op.nearEntries();
    s[1] = op.m2lEntries();
    s[2] = op.plan.pairsM2L;
    s[3] = (int64_t)op.plan.leaves.size();
    s[4] = (int64_t)op.plan.m2lTgt.size();
    s[5] = op.tree.nn;
    int64_t mx = 0;
    for (int i = 0; i < op.tree.nn; ++i)
        if (op.tree.isLeaf[i]) mx = std::max<int64_t>(mx, op.tree.count[i]);
    s[6] = mx;
    s[7] = op.geo.N;
    s[8] = op.plan.storedNear;
    s[9] = op.plan.storedM2L;
    s[10] = op.plan.m2lCanon;
    s[11] = op.plan.nearPartTotal;
    s[12] = op.harmonicReady() ? 1 : 0;
    s[13] = (int64_t)op.plan.attOwner.size();
    const bool cl = op.harmonicReady() && op.clustersOn();
    s[14] = cl ? (int64_t)op.plan.hmClPtr.size() - 1 : 0;
    s[15] = cl ? op.plan.hmDual : 0;
    s[16] = cl ? (int64_t)op.plan.hmSrc.size() : (int64_t)op.plan.attSrc.size();
    s[17] = op.f32Bytes();  // config 5's fp32 operator caches (0 before its first apply)
    s[18] = cl && op.topFusedOn() ? 1 : 0;
    // the cluster plan itself (block handles; host-side, no GPU needed)
    s[19] = (int64_t)op.plan.hmHaloNode.size();
    s[20] = op.plan.hmMaxLds;
    s[21] = (int64_t)op.plan.hmSrc.size();
    s[22] = op.topRecoveries;
    // the harmonic near field's symmetric U storage (0: directed, Plan::nearSymHsOn)
    s[23] = op.plan.nearSymHsOn ? op.plan.hsStored : 0;
    s[24] = op.plan.nearSymHsOn ? op.plan.hsPartTotal : 0;
    s[25] = op.oneXApplies;  // sharded matvecs through the one-collective exchange
    s[26] = op.mrhsM2LPairs();  // directed M2L pairs of the 16-RHS MFMA operators (0 before their plan)
    s[27] = op.topSteals();     // upper-tier tasks computed by waiting blocks of the fused launch
    s[28] = op.upPartialApplies;  // one-collective matvecs with the upper multipoles as partial sums
    s[29] = op.nearOverlaps() ? 1 : 0;  // the block apply's near field on the side stream (else serial)
    s[30] = op.nearUpTier() ? 1 : 0;  // the one-GPU block apply's bottom up tier inside the near field
    // the staged near field's index streams (bench.py's extended algorithmic bytes): its
    // 16-bit source-row entries (one per leaf and source point), its correction-stencil
    // row entries (9 per target), and the bottom-tier nodes whose multipoles its up tail
    // writes (16 leaves + 4 parents + 1 root per group)
    s[31] = (int64_t)op.plan.nearLoc.size();
    s[32] = (int64_t)op.plan.nearCorrRow.size();
    s[33] = (int64_t)(op.plan.nearUpGrp.size() / aniso::kNearUpInts) * 21;
}

// the fixed-size entry: the first kStatsV1 = 26 entries, as aniso_mi355x_dev.h has
// promised since round 4 (entries 26.. only through aniso_stats_n)
int aniso_stats(aniso_handle h, int64_t* s) {
    ENTER(h);
    return guarded([&] {
        CHECK_PTR(s);
        int64_t all[kStats];
        stats_fill(get(h), all);
        std::copy(all, all + kStatsV1, s);
    });
}

int aniso_stats_n(aniso_handle h, int64_t* s, int cap, int* n) {
    ENTER(h);
    return guarded([&] {
        CHECK_PTR(n);
        if (cap < 0) throw std::invalid_argument("aniso_stats_n: cap must be >= 0");
        if (cap > 0) CHECK_PTR(s);
        int64_t all[kStats];
        stats_fill(get(h), all);
        std::copy(all, all + std::min(cap, kStats), s);
        *n = kStats;
    });
}

int aniso_set_timing(aniso_handle h, int on) {
    ENTER(h);
    return guarded([&] { get(h).setTiming(on); });  // 0 off, 1 every stage, 2 M2L + near only
}

int aniso_stage_times(aniso_handle h, float* t) {
    ENTER(h);
    return guarded([&] {
        CHECK_PTR(t);
        auto s = get(h).stageTimes();
        t[0] = s.exch; t[1] = s.up; t[2] = s.m2l; t[3] = s.gather; t[4] = s.near; t[5] = s.down; t[6] = s.corr;
        t[7] = s.total;
    });
}

int aniso_top_trace(aniso_handle h, int64_t* rec, int64_t cap, int64_t* n) {
    ENTER(h);
    return guarded([&] {
        CHECK_PTR(n);
        if (rec && cap < 0) throw std::invalid_argument("aniso_top_trace: cap must be >= 0");
        const auto t = get(h).topTrace();
        *n = (int64_t)t.size() / 8;
        if (rec) std::copy(t.begin(), t.begin() + std::min<int64_t>(cap, *n) * 8, rec);
    });
}

int aniso_line_integrals(aniso_handle h, const double* seg, int n, double* out) {
    ENTER(h);
    return guarded([&] {
        CHECK_PTR(seg);
        CHECK_PTR(out);
        get(h).lineIntegrals(seg, n, out);
    });
}

int aniso_comm_unique_id(unsigned char* id) {
    return guarded([&] {
        CHECK_PTR(id);
        aniso::rccl_unique_id(id);
    });
}

int aniso_comm_init_rccl(aniso_handle h, const unsigned char* id) {
    ENTER(h);
    return guarded([&] {
        CHECK_PTR(id);
        auto& op = get(h);
        op.commInit(aniso::make_rccl_collectives(id, op.plan.nranks, op.plan.rank));
    });
}

int aniso_comm_init_callbacks(aniso_handle h, const aniso_collectives* c) {
    ENTER(h);
    return guarded([&] {
        CHECK_PTR(c);
        auto& op = get(h);
        op.commInit(aniso::make_callback_collectives(*c, op.plan.nranks, op.plan.rank));
    });
}

int aniso_krylov_dot(aniso_handle h, int64_t n, int nv, const double* V, int64_t ldv, const double* w, double* out,
                     void* stream) {
    ENTER(h);
    return guarded([&] {
        CHECK_PTR(V);
        CHECK_PTR(w);
        CHECK_PTR(out);
        auto& op = get(h);
        op.krylovDot(n, nv, V, ldv, w, out, (hipStream_t)stream);
    });
}

int aniso_krylov_update(aniso_handle h, int64_t n, int nv, const double* V, int64_t ldv, const double* c, double* w,
                        double* out, int dots, void* stream) {
    ENTER(h);
    return guarded([&] {
        CHECK_PTR(V);
        CHECK_PTR(c);
        CHECK_PTR(w);
        CHECK_PTR(out);
        auto& op = get(h);
        op.krylovUpdate(n, nv, V, ldv, c, w, out, dots != 0, (hipStream_t)stream);
    });
}

int aniso_arnoldi_state_size(int m, int64_t* doubles) {
    return guarded([&] {
        CHECK_PTR(doubles);
        if (m < 1) throw std::invalid_argument("arnoldi: restart length m >= 1");
        *doubles = aniso::arn_state_doubles(m);
    });
}

int aniso_arnoldi_begin(aniso_handle h, int64_t n, int m, const double* V, int64_t ldv, double* state,
                        const double* rr, double normb, double* status, void* stream) {
    ENTER(h);
    return guarded([&] {
        CHECK_PTR(state);
        if (!rr) CHECK_PTR(V);
        get(h).arnoldiBegin(n, m, V, ldv, state, rr, normb, status, (hipStream_t)stream);
    });
}

int aniso_arnoldi_step(aniso_handle h, int64_t n, int m, int j, double* V, int64_t ldv, const double* w,
                       double* state, double* status, void* stream) {
    ENTER(h);
    return guarded([&] {
        CHECK_PTR(V);
        CHECK_PTR(w);
        CHECK_PTR(state);
        get(h).arnoldiStep(n, m, j, V, ldv, w, state, status, (hipStream_t)stream);
    });
}

int aniso_arnoldi_project(aniso_handle h, int64_t n, int j, const double* V, int64_t ldv, const double* w,
                          double* out, void* stream) {
    ENTER(h);
    return guarded([&] {
        CHECK_PTR(V);
        CHECK_PTR(w);
        CHECK_PTR(out);
        get(h).arnoldiProject(n, j, V, ldv, w, out, (hipStream_t)stream);
    });
}

int aniso_arnoldi_coef(aniso_handle h, int m, int j, double* state, const double* red, void* stream) {
    ENTER(h);
    return guarded([&] {
        CHECK_PTR(state);
        CHECK_PTR(red);
        get(h).arnoldiCoef(m, j, state, red, (hipStream_t)stream);
    });
}

int aniso_arnoldi_update(aniso_handle h, int64_t n, int m, int j, double* V, int64_t ldv, const double* w,
                         const double* state, double* out, void* stream) {
    ENTER(h);
    return guarded([&] {
        CHECK_PTR(V);
        CHECK_PTR(w);
        CHECK_PTR(state);
        CHECK_PTR(out);
        get(h).arnoldiUpdate(n, m, j, V, ldv, w, state, out, (hipStream_t)stream);
    });
}

int aniso_arnoldi_column(aniso_handle h, int m, int j, double* state, const double* red, double* status,
                         void* stream) {
    ENTER(h);
    return guarded([&] {
        CHECK_PTR(state);
        CHECK_PTR(red);
        get(h).arnoldiColumn(m, j, state, red, status, (hipStream_t)stream);
    });
}

int aniso_arnoldi_solution(aniso_handle h, int64_t n, int m, int used, const double* V, int64_t ldv, double* state,
                           double* x, void* stream) {
    ENTER(h);
    return guarded([&] {
        CHECK_PTR(state);
        if (used > 0) {
            CHECK_PTR(V);
            CHECK_PTR(x);
        }
        get(h).arnoldiSolution(n, m, used, V, ldv, state, x, (hipStream_t)stream);
    });
}

int aniso_mapped_alloc(size_t bytes, void** host, void** dev) {
    return guarded([&] {
        CHECK_PTR(host);
        CHECK_PTR(dev);
        *host = *dev = nullptr;
        if (bytes == 0) throw std::invalid_argument("aniso_mapped_alloc: bytes > 0");
        hipError_t e = hipHostMalloc(host, bytes, hipHostMallocMapped | hipHostMallocCoherent);
        if (e != hipSuccess) aniso::throw_hip(e, __FILE__, __LINE__);
        std::memset(*host, 0, bytes);
        e = hipHostGetDevicePointer(dev, *host, 0);
        if (e != hipSuccess) {
            (void)hipHostFree(*host);
            *host = nullptr;
            aniso::throw_hip(e, __FILE__, __LINE__);
        }
    });
}

int aniso_mapped_free(void* host) {
    return guarded([&] {
        if (!host) return;
        const hipError_t e = hipHostFree(host);
        if (e != hipSuccess) aniso::throw_hip(e, __FILE__, __LINE__);
    });
}

int aniso_comm_init_loopback(aniso_handle h) {
    ENTER(h);
    return guarded([&] {
        auto& op = get(h);
        op.commInit(aniso::make_loopback_collectives(op.plan.nranks, op.plan.rank));
    });
}

int aniso_block_op_sharded_dev(aniso_handle h, int which, double* x, int64_t ldx, double* y, int64_t ldy,
                               void* stream) {
    ENTER(h);
    return guarded([&] {
        CHECK_PTR(x);
        CHECK_PTR(y);
        auto& op = get(h);
        op.blockOpShardedDev(which, x, ldx, y, ldy, (hipStream_t)stream);
    });
}

int aniso_memcpy(void* dst, const void* src, size_t bytes) {
    return guarded([&] {
        if (bytes == 0) return;
        CHECK_PTR(dst);
        CHECK_PTR(src);
        const hipError_t e = hipMemcpy(dst, src, bytes, hipMemcpyDefault);
        if (e != hipSuccess) aniso::throw_hip(e, __FILE__, __LINE__);
    });
}

int aniso_last_error(char* buf, size_t len) {
    if (!buf || !len) return ANISO_ERR_INVALID;
    size_t n = std::min(len - 1, g_err.size());
    std::memcpy(buf, g_err.data(), n);
    buf[n] = 0;
    return ANISO_OK;
}

const char* aniso_version(void) { return "aniso_mi355x 0.1 (gfx950)"; }

}  // extern "C"
