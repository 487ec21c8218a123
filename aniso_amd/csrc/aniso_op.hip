// aniso_op.hip -- host orchestration of the MI355X operator (one per handle).
//
// Lifecycle mirrors the reference's MEX ops (AnisoWrapper.cpp:10-136):
//   Operator()  <- 'new'       geometry + quadtree + lists on the host (no GPU)
//   setCoeff    <- 'setCoeff'  sigma coefficients; uploads geometry/tree to HBM
//   cache(m)    <- 'cache'     device-side build of the merged pair operators
//   mapping*    <- 'mapping'   one apply, all stages on the GPU
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <thread>

#include "aniso_op.hpp"
#include "kernels.hpp"

namespace aniso {

[[noreturn]] void throw_hip(hipError_t e, const char* file, int line) {
    throw std::runtime_error(std::string("HIP error ") + hipGetErrorName(e) + " (" + hipGetErrorString(e) + ") at " +
                             file + ":" + std::to_string(line));
}

#define HIP_CHECK(x)                                         \
    do {                                                     \
        hipError_t e__ = (x);                                \
        if (e__ != hipSuccess) throw_hip(e__, __FILE__, __LINE__); \
    } while (0)

DevBuf::~DevBuf() {
    if (p) (void)hipFree(p);
}

void DevBuf::alloc(size_t nbytes) {
    if (p && bytes == nbytes) return;
    if (p) {
        HIP_CHECK(hipFree(p));
        p = nullptr;
    }
    bytes = nbytes;
    if (nbytes) HIP_CHECK(hipMalloc(&p, nbytes));
}

void DevBuf::upload(const void* host, size_t nbytes) {
    alloc(nbytes);
    if (nbytes) HIP_CHECK(hipMemcpy(p, host, nbytes, hipMemcpyHostToDevice));
}

template <class T>
static void up(DevBuf& b, const std::vector<T>& v) {
    b.upload(v.data(), v.size() * sizeof(T));
}

static int host_threads() {
    unsigned n = std::thread::hardware_concurrency();
    return n ? (int)std::min(n, 16u) : 4;
}

Operator::Operator(int sz, int d, int ks_, double g_, int ns_, int np_, int maxLevel_)
    : ks(ks_), ns(ns_), np(np_), maxLevel(maxLevel_), g(g_) {
    if (ks < 1) throw std::invalid_argument("kernel size must be >= 1");
    if (np != kNP) throw std::invalid_argument("np must be 4 on the MI355X path (rank-16 Chebyshev)");
    if (d < 1 || d > kMaxD) throw std::invalid_argument("quadRule must be in 1..6 on the MI355X path");
    if (maxLevel < 0) throw std::invalid_argument("maxLevel must be >= 0");
    kernelSize = 2 * ks - 1;
    geo.build(sz, d, ns);
    tree.build(geo.px.data(), geo.py.data(), geo.N, np * np, maxLevel, host_threads());
    plan.build(tree, np, 0, 1);
    sigma_s.assign(geo.N, 0.0);
    sigma_t.assign(geo.N, 0.0);
    modes.resize(kernelSize);
}

Operator::~Operator() {
    if (device >= 0) {
        (void)hipSetDevice(device);
        for (auto& set : evPool)
            for (auto& e : set) (void)hipEventDestroy(e);
        if (own) (void)hipStreamDestroy(own);
        if (aux) (void)hipStreamDestroy(aux);
        if (evFork) (void)hipEventDestroy(evFork);
        if (evJoin) (void)hipEventDestroy(evJoin);
    }
}

void Operator::getNodes(double* xy) const {
    for (int64_t i = 0; i < geo.N; ++i) {
        xy[i] = geo.px[i];
        xy[i + geo.N] = geo.py[i];
    }
}

void Operator::setShard(int rank, int nranks) {
    plan.build(tree, np, rank, nranks);
    for (auto& m : modes) {
        m.Knear.alloc(0);
        m.Km2l.alloc(0);
        m.ready = false;
    }
    if (device >= 0) uploadPlan();
}

void Operator::ensureDevice() {
    if (device >= 0) {
        HIP_CHECK(hipSetDevice(device));
        return;
    }
    HIP_CHECK(hipGetDevice(&device));
    HIP_CHECK(hipStreamCreateWithFlags(&own, hipStreamNonBlocking));
    HIP_CHECK(hipStreamCreateWithFlags(&aux, hipStreamNonBlocking));
    HIP_CHECK(hipEventCreateWithFlags(&evFork, hipEventDisableTiming));
    HIP_CHECK(hipEventCreateWithFlags(&evJoin, hipEventDisableTiming));
    if (const char* e = std::getenv("ANISO_OVERLAP")) overlap = e[0] == '1';
    // tree-order coordinates
    std::vector<double> pxT(geo.N), pyT(geo.N);
    for (int64_t k = 0; k < geo.N; ++k) {
        pxT[k] = geo.px[tree.perm[k]];
        pyT[k] = geo.py[tree.perm[k]];
    }
    up(dPxT, pxT);
    up(dPyT, pyT);
    up(dPerm, tree.perm);
    up(dW, geo.w);
    std::vector<double> wT(geo.N);
    for (int64_t k = 0; k < geo.N; ++k) wT[k] = geo.w[tree.perm[k]];
    up(dWT, wT);
    std::vector<int> iperm(geo.N);
    for (int64_t k = 0; k < geo.N; ++k) iperm[tree.perm[k]] = (int)k;
    up(dIperm, iperm);
    up(dNcx, tree.ncx);
    up(dNcy, tree.ncy);
    up(dNrx, tree.nrx);
    up(dNry, tree.nry);
    up(dBegin, tree.begin);
    up(dCount, tree.count);
    up(dParent, tree.parent);
    up(dSlot, tree.slot);
    std::vector<int4> ch(tree.nn);
    for (int i = 0; i < tree.nn; ++i) ch[i] = make_int4(tree.child[i][0], tree.child[i][1], tree.child[i][2], tree.child[i][3]);
    for (auto& c : ch) {  // leaves: point children at self (never dereferenced for non-leaves)
        if (c.x < 0) c = make_int4(0, 0, 0, 0);
    }
    up(dChild, ch);
    // parameter block
    Params P;
    std::memset(&P, 0, sizeof(P));
    P.sz = geo.sz;
    P.d = geo.d;
    P.d2 = geo.d2;
    P.nsq = geo.nsq;
    P.dx = geo.dx;
    for (int i = 0; i < geo.d; ++i) {
        P.gx[i] = geo.gx[i];
        P.gw[i] = geo.gw[i];
    }
    // Chebyshev nodes / polynomials / transfer operators (bbfmm.h:597-693)
    for (int i = 0; i < kNP; ++i) P.cheb[i] = -std::cos((i + 0.5) * M_PI / kNP);
    for (int i = 0; i < kNP; ++i) {
        double T[kNP];
        T[0] = 1.0;
        T[1] = P.cheb[i];
        for (int l = 2; l < kNP; ++l) T[l] = 2.0 * P.cheb[i] * T[l - 1] - T[l - 2];
        for (int l = 0; l < kNP; ++l) P.tnode[i + l * kNP] = T[l];
    }
    double S[2 * kNP][kNP];
    for (int k = 0; k < 2 * kNP; ++k) {
        double s = (k < kNP) ? -0.5 + 0.5 * P.cheb[k] : 0.5 + 0.5 * P.cheb[k - kNP];
        double T[kNP];
        T[0] = 1.0;
        T[1] = s;
        for (int l = 2; l < kNP; ++l) T[l] = 2.0 * s * T[l - 1] - T[l - 2];
        for (int i = 0; i < kNP; ++i) {
            double acc = 0.0;
            for (int l = 0; l < kNP; ++l) acc += T[l] * P.tnode[i + l * kNP];
            S[k][i] = (2.0 * acc - 1.0) * (1.0 / kNP);
        }
    }
    for (int id = 0; id < 4; ++id) {
        int b0 = id & 1, b1 = (id >> 1) & 1;
        for (int i = 0; i < kNP; ++i)
            for (int j = 0; j < kNP; ++j)
                for (int k = 0; k < kNP; ++k)
                    for (int l = 0; l < kNP; ++l)
                        P.R[id][(i * kNP + j) + (k * kNP + l) * kRank] = S[b1 * kNP + i][k] * S[b0 * kNP + j][l];
    }
    const int d2 = geo.d2;
    for (int i = 0; i < d2 * d2; ++i) P.interp[i] = geo.interp[i];
    for (int i = 0; i < d2; ++i) P.sqrtW[i] = geo.sqrtW[i];
    CorrTables ct;
    ct.build(geo, 0);
    for (size_t i = 0; i < ct.legB.size(); ++i) P.legB[i] = ct.legB[i];
    for (int i = 0; i < d2; ++i) P.coefScale[i] = ct.coefScale[i];
    dParams.upload(&P, sizeof(P));
    // work arrays
    dCharge.alloc(geo.N * sizeof(double));
    dOut.alloc(geo.N * sizeof(double));
    dFT.alloc(geo.N * sizeof(double));
    dCT.alloc(geo.N * sizeof(double));
    dTmp.alloc(geo.N * sizeof(double));
    dTmp2.alloc(geo.N * sizeof(double));
    dTmpS.alloc(geo.N * sizeof(double));
    dMult.alloc((size_t)tree.nn * kRank * sizeof(double));
    dLocal.alloc((size_t)tree.nn * kRank * sizeof(double));
    dTotal.alloc((size_t)tree.nn * kRank * sizeof(double));
    HIP_CHECK(hipMemset(dMult.p, 0, dMult.bytes));
    HIP_CHECK(hipMemset(dLocal.p, 0, dLocal.bytes));
    uploadPlan();
}

static std::vector<int4> to_int4(const std::vector<std::array<int, 4>>& v) {
    std::vector<int4> o(v.size());
    for (size_t i = 0; i < v.size(); ++i) o[i] = make_int4(v[i][0], v[i][1], v[i][2], v[i][3]);
    return o;
}

void Operator::uploadPlan() {
    up(dLeaves, plan.leaves);
    up(dNearPtr, plan.nearPtr);
    up(dNearSrc, plan.nearSrc);
    up(dNearKOff, plan.nearKOff);
    up(dM2LTgt, plan.m2lTgt);
    up(dM2LPtr, plan.m2lPtr);
    up(dM2LSrc, plan.m2lSrc);
    std::vector<int> pairTgt(plan.m2lSrc.size());
    for (size_t i = 0; i < plan.m2lTgt.size(); ++i)
        for (int64_t p = plan.m2lPtr[i]; p < plan.m2lPtr[i + 1]; ++p)  // ~target: canonical (column-major) block
            pairTgt[p] = p < plan.m2lPtr[i] + plan.m2lNDir[i] ? plan.m2lTgt[i] : ~plan.m2lTgt[i];
    up(dM2LPairTgt, pairTgt);
    up(dM2LNDir, plan.m2lNDir);
    up(dM2LCanonBase, plan.m2lCanonBase);
    up(dM2LInPtr, plan.m2lInPtr);
    up(dM2LOutSlot, plan.m2lOutSlot);
    dM2LPart.alloc((size_t)std::max(plan.m2lCanon, 1) * kRank * sizeof(double));
    std::vector<int2> ns(plan.nearSym.size());
    for (size_t i = 0; i < ns.size(); ++i) ns[i] = make_int2(plan.nearSym[i][0], plan.nearSym[i][1]);
    up(dNearSym, ns);
    up(dDnLeafNear, plan.dnLeafNear);
    up(dDnDesc, to_int4(plan.dnDesc));
    up(dDnGrpFix, plan.dnGrpFix);
    up(dDnLeafGeom, plan.dnLeafGeom);
    up(dDnChainPtr, plan.dnChainPtr);
    up(dDnChain, plan.dnChain);
    up(dDnNearPtr, plan.dnNearPtr);
    up(dDnNearOff, plan.dnNearOff);
    dNearPart.alloc((size_t)std::max<int64_t>(plan.nearPartTotal, 1) * sizeof(double));
    up(dLeafInfo, to_int4(plan.leafInfo));
    up(dNearPtsPtr, plan.nearPtsPtr);
    up(dNearPts, plan.nearPts);
    up(dUpTaskPtr, plan.upTaskPtr);
    up(dUpGrpPtr, plan.upGrpPtr);
    up(dUpGrp, plan.upGrp);
    up(dUpNode, plan.upNode);
    up(dUpCode, to_int4(plan.upCode));
    up(dUpDesc, to_int4(plan.upDesc));
    up(dUpGrpFix, plan.upGrpFix);
    up(dUpGeom, plan.upGeom);
    up(dUpLeaf, plan.upLeaf);
    up(dDnTaskPtr, plan.dnTaskPtr);
    up(dDnGrpPtr, plan.dnGrpPtr);
    up(dDnGrp, plan.dnGrp);
    up(dDnNode, to_int4(plan.dnNode));
    up(dDnLeafPtr, plan.dnLeafPtr);
    up(dDnLeafSlot, plan.dnLeafSlot);
    up(dDnLeafIdx, plan.dnLeafIdx);
    up(dDnLeafPts, plan.dnLeafPts);
    up(dDnPtsRange, plan.dnPtsRange);
    // a task's expansions live in LDS (<= 4 levels: 85 nodes); a workgroup may use all 160 KiB
    if (up_tier_lds(plan.upMaxTask) > 160 * 1024 || down_tier_lds(plan.dnMaxTask, plan.dnMaxLeaves, plan.dnMaxNear, plan.dnMaxChain) > 160 * 1024)
        throw std::logic_error("up/down pass task exceeds one workgroup's LDS");
    maxNearS = 1;
    for (size_t li = 0; li < plan.leaves.size(); ++li) {
        int64_t S = 0;
        for (int64_t j = plan.nearPtr[li]; j < plan.nearPtr[li + 1]; ++j) S += tree.count[plan.nearSrc[j]];
        maxNearS = std::max<int>(maxNearS, (int)S);
    }
}

// setCoeff (AnisoWrapper.cpp:46-69): sigma copies + interpolation() (KernelFactory.cpp:212-227);
// singPrecompute() lives in Geometry; the device keeps sigma_t's coefficients / legendreNorms.
void Operator::setCoeff(const double* ss, const double* st) {
    ensureDevice();
    std::memcpy(sigma_s.data(), ss, geo.N * sizeof(double));
    std::memcpy(sigma_t.data(), st, geo.N * sizeof(double));
    const int d2 = geo.d2;
    std::vector<double> coef((size_t)geo.nsq * d2);
    std::vector<double> lt(d2);
    for (int i = 0; i < geo.nsq; ++i) {
        for (int j = 0; j < d2; ++j) lt[j] = geo.sqrtW[j] * st[(size_t)i * d2 + j];
        for (int r = 0; r < d2; ++r) {
            double s = 0.0;
            for (int k = 0; k < d2; ++k) s += geo.interp[r + (size_t)k * d2] * lt[k];
            coef[(size_t)i * d2 + r] = s / geo.lnorm[r];
        }
    }
    up(dStCoef, coef);
    up(dSigmaS, sigma_s);
    std::vector<double> sT(geo.N);
    for (int64_t k = 0; k < geo.N; ++k) sT[k] = sigma_s[tree.perm[k]];
    up(dSigmaT, sT);
    for (auto& m : modes) m.ready = false;
    coeffSet = true;
}

// cache(Id) (AnisoWrapper.cpp:72-90): runKernelsCache + runKernelsCacheSing
// (merged operators, built on the GPU), refineAddOnCache + singularAddCache
// (translation-invariant stencil tables, built on the host).
void Operator::cache(int id) {
    if (id < 0 || id >= kernelSize)
        throw std::out_of_range("kernel id " + std::to_string(id) + " out of range [0, " + std::to_string(kernelSize) + ")");
    if (!coeffSet) throw std::runtime_error("cache called before setCoeff");
    ensureDevice();
    ModeCache& mc = modes[id];
    mc.Knear.alloc((size_t)plan.nearKTotal * sizeof(double));
    mc.Km2l.alloc((size_t)plan.storedM2L * 256 * sizeof(double));
    const Params* P = dParams.as<Params>();
    int maxSrc = 1;
    for (size_t li = 0; li < plan.leaves.size(); ++li)
        maxSrc = std::max<int>(maxSrc, (int)(plan.nearPtr[li + 1] - plan.nearPtr[li]));
    launch_cache_m2l(plan.storedM2L,dM2LPairTgt.as<int>(), dM2LSrc.as<int>(), dNcx.as<double>(), dNcy.as<double>(),
                     dNrx.as<double>(), dNry.as<double>(), dStCoef.as<double>(), P, id, mc.Km2l.as<double>(), own);
    launch_cache_near((int)plan.leaves.size(), dLeaves.as<int>(), dNearPtr.as<int64_t>(), dNearSrc.as<int>(),
                      dNearKOff.as<int64_t>(), dBegin.as<int64_t>(), dCount.as<int64_t>(), dPxT.as<double>(),
                      dPyT.as<double>(), dStCoef.as<double>(), P, id, maxSrc, mc.Knear.as<double>(), own);
    CorrTables ct;
    ct.build(geo, id);
    up(mc.C, ct.C);
    up(mc.mu, ct.mu);
    HIP_CHECK(hipStreamSynchronize(own));
    mc.ready = true;
}

void Operator::mappingHost(const double* charge, int id, double* out) {
    if (id < 0 || id >= kernelSize) throw std::out_of_range("kernel id out of range");
    if (!modes[id].ready) throw std::runtime_error("mapping on kernel id " + std::to_string(id) + " before cache(" + std::to_string(id) + ")");
    ensureDevice();
    HIP_CHECK(hipMemcpyAsync(dCharge.p, charge, geo.N * sizeof(double), hipMemcpyHostToDevice, own));
    if (plan.nranks > 1) HIP_CHECK(hipMemsetAsync(dOut.p, 0, dOut.bytes, own));
    mappingDev(dCharge.as<double>(), id, dOut.as<double>(), own, kStageAll);
    HIP_CHECK(hipMemcpyAsync(out, dOut.p, geo.N * sizeof(double), hipMemcpyDeviceToHost, own));
    HIP_CHECK(hipStreamSynchronize(own));
}

// mapping (AnisoWrapper.cpp:92-136) on device pointers, enqueued on stream s.
// Only owned targets of `out` are written when the operator is sharded.
void Operator::mappingDev(const double* charge, int id, double* out, hipStream_t s, int mask) {
    apply(charge, false, nullptr, id, out, false, s, mask);
}

// mapping on a tree-order input (all N) into the owned tree-order slice
// out[k - ownBegin], k in [ownBegin, ownEnd): no permutation gathers, and the
// slices of the shards concatenate to the tree-order output.
void Operator::mappingTreeDev(const double* qTree, int id, double* outSlice, hipStream_t s) {
    apply(qTree, true, nullptr, id, outSlice, true, s, kStageAll);
}

// main.cpp forwardOperator (main.cpp:125-136) in tree order: y = x - K_0(sigma_s x)
// on the owned slice, x tree-ordered (all N).
void Operator::forwardTreeDev(const double* xTree, double* ySlice, hipStream_t s) {
    apply(xTree, true, dSigmaT.as<double>(), 0, dTmpS.as<double>(), true, s, kStageAll);
    launch_sub_slice(plan.ownEnd - plan.ownBegin, xTree + plan.ownBegin, dTmpS.as<double>(), ySlice, s);
}

void Operator::apply(const double* charge, bool treeIn, const double* sigT, int id, double* out, bool treeOut,
                     hipStream_t s, int mask) {
    if (id < 0 || id >= kernelSize) throw std::out_of_range("kernel id out of range");
    if (!modes[id].ready) throw std::runtime_error("mapping on kernel id " + std::to_string(id) + " before cache(" + std::to_string(id) + ")");
    ensureDevice();
    const ModeCache& mc = modes[id];
    const Params* P = dParams.as<Params>();
    const bool tm = timeStages;
    hipEvent_t* ev = nullptr;
    if (tm) {
        if (evUsed == (int)evPool.size()) {
            std::array<hipEvent_t, kStageEvents> set;
            for (auto& e : set) HIP_CHECK(hipEventCreate(&e));
            evPool.push_back(set);
        }
        ev = evPool[evUsed++].data();
        HIP_CHECK(hipEventRecord(ev[0], s));
    }
    const int* operm = treeOut ? nullptr : dPerm.as<int>();
    const int64_t obase = treeOut ? plan.ownBegin : 0;
    // up pass (global, every rank): tiers bottom-up; its P2M also forms the weighted
    // charges fT (tree order) the near field and the corrections read
    if (plan.upTierTask.size() < 2)  // a lone leaf: no up pass
        launch_prepare(geo.N, charge, treeIn ? 1 : 0, dPerm.as<int>(), sigT, dWT.as<double>(), dFT.as<double>(),
                       dCT.as<double>(), s);
    for (size_t k = 0; k + 1 < plan.upTierTask.size(); ++k)
        launch_up_tier(plan.upTierTask[k + 1] - plan.upTierTask[k], plan.upTierTask[k], plan.upMaxTask,
                       dUpDesc.as<int4>(), dUpGrpFix.as<int>(), dUpNode.as<int>(), dUpCode.as<int4>(),
                       dUpGeom.as<double4>(), dUpLeaf.as<int2>(), dPxT.as<double>(), dPyT.as<double>(), charge,
                       treeIn ? 1 : 0, dPerm.as<int>(), sigT, dWT.as<double>(), dFT.as<double>(),
                       dCT.as<double>(), P, dMult.as<double>(), s);
    if (tm) HIP_CHECK(hipEventRecord(ev[1], s));
    // The near field and the corrections need only the weighted charges; with
    // ANISO_OVERLAP=1 they run on the auxiliary stream beside the M2L stream (both
    // write `out`: near stores, corr adds; the down pass adds after the join).
    hipStream_t sn = overlap ? aux : s;
    if (overlap) {
        HIP_CHECK(hipEventRecord(evFork, s));
        HIP_CHECK(hipStreamWaitEvent(aux, evFork, 0));
    }
    // K_{B<-A} = (-1)^m K_{A<-B}^T for the merged kernel; Id = m
    const double sgn = (id % 2 == 0) ? 1.0 : -1.0;
    if (tm) HIP_CHECK(hipEventRecord(ev[6], sn));
    launch_near((int)plan.leaves.size(), dLeafInfo.as<int4>(), dNearPtsPtr.as<int64_t>(), dNearPts.as<int>(),
                dNearKOff.as<int64_t>(), dNearSym.as<int2>(), mc.Knear.as<double>(), dFT.as<double>(), operm, obase,
                maxNearS, mask, sgn, M_1_PI / 2.0, dNearPart.as<double>(), out, sn);
    if (tm) HIP_CHECK(hipEventRecord(ev[7], sn));
    launch_corr(geo.d, plan.ownBegin, plan.ownEnd, dPerm.as<int>(), dIperm.as<int>(), dCT.as<double>(), dFT.as<double>(),
                mc.C.as<double>(),
                mc.mu.as<double>(), P, mask, M_1_PI / 2.0, treeOut, out, sn);
    if (tm) HIP_CHECK(hipEventRecord(ev[8], sn));
    if (overlap) HIP_CHECK(hipEventRecord(evJoin, aux));
    if (tm) HIP_CHECK(hipEventRecord(ev[2], s));
    if (mask & kStageFar)
        launch_m2l((int)plan.m2lTgt.size(), dM2LTgt.as<int>(), dM2LPtr.as<int64_t>(), dM2LNDir.as<int>(),
                   dM2LCanonBase.as<int>(), dM2LOutSlot.as<int>(), dM2LSrc.as<int>(), mc.Km2l.as<double>(),
                   dMult.as<double>(), sgn, dM2LPart.as<double>(), dLocal.as<double>(), s);
    if (tm) HIP_CHECK(hipEventRecord(ev[3], s));
    if ((mask & kStageFar) && plan.m2lCanon > 0)
        launch_m2l_gather((int)plan.m2lTgt.size(), dM2LTgt.as<int>(), dM2LInPtr.as<int>(), dM2LPart.as<double>(),
                          dLocal.as<double>(), s);
    if (tm) HIP_CHECK(hipEventRecord(ev[4], s));
    if (overlap) HIP_CHECK(hipStreamWaitEvent(s, evJoin, 0));
    if (tm) HIP_CHECK(hipEventRecord(ev[9], s));
    // down pass (owned part): tiers top-down; L2L + L2P + gathered transposed near products
    if (mask & (kStageFar | kStageNear))
        launch_down_tier((int)plan.dnDesc.size() / 3, plan.dnMaxTask, plan.dnMaxLeaves, dDnDesc.as<int4>(),
                         dDnGrpFix.as<int>(), dDnNode.as<int4>(), dLocal.as<double>(), P, dDnLeafSlot.as<int>(),
                         dDnLeafPts.as<int>(), dDnLeafNear.as<int2>(), dDnLeafGeom.as<double4>(), dPxT.as<double>(),
                         dPyT.as<double>(), operm, obase, dDnNearOff.as<int>(), plan.dnMaxNear,
                         dNearPart.as<double>(), dDnChain.as<int2>(), plan.dnMaxChain, mask, M_1_PI / 2.0, out, s);
    if (tm) HIP_CHECK(hipEventRecord(ev[5], s));
}

void Operator::setTiming(bool on) {
    timeStages = on;
    if (on) evUsed = 0;
}

StageTimes Operator::stageTimes() {
    StageTimes r;
    if (evUsed == 0) return r;
    HIP_CHECK(hipEventSynchronize(evPool[evUsed - 1][5]));
    auto el = [](hipEvent_t a, hipEvent_t b) {
        float t = 0;
        HIP_CHECK(hipEventElapsedTime(&t, a, b));
        return (double)t;
    };
    double acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int k = 0; k < evUsed; ++k) {
        const auto& e = evPool[k];
        acc[1] += el(e[0], e[1]);  // up, with the weighted charges (acc[0], prep, is fused into it)
        acc[2] += el(e[2], e[3]);  // m2l
        acc[3] += el(e[3], e[4]);  // gather
        acc[4] += el(e[6], e[7]);  // near (auxiliary stream)
        acc[5] += el(e[9], e[5]);  // down (after the join)
        acc[6] += el(e[7], e[8]);  // corr (auxiliary stream)
        acc[7] += el(e[0], e[5]);  // whole apply
    }
    for (double& a : acc) a /= evUsed;
    r.prep = (float)acc[0];
    r.up = (float)acc[1];
    r.m2l = (float)acc[2];
    r.gather = (float)acc[3];
    r.near = (float)acc[4];
    r.down = (float)acc[5];
    r.corr = (float)acc[6];
    r.total = (float)acc[7];
    return r;
}

void Operator::lineIntegrals(const double* seg, int n, double* out) {
    if (!coeffSet) throw std::runtime_error("line integrals before setCoeff");
    if (n < 0) throw std::invalid_argument("n must be >= 0");
    if (n == 0) return;
    ensureDevice();
    DevBuf ds, dout;
    ds.upload(seg, (size_t)n * 4 * sizeof(double));
    dout.alloc((size_t)n * sizeof(double));
    launch_line_integrals(n, ds.as<double>(), dStCoef.as<double>(), dParams.as<Params>(), dout.as<double>(), own);
    HIP_CHECK(hipStreamSynchronize(own));
    HIP_CHECK(hipMemcpy(out, dout.p, (size_t)n * sizeof(double), hipMemcpyDeviceToHost));
}

void Operator::permuteToTree(const double* orig, double* treeOut, hipStream_t s) {
    ensureDevice();
    launch_permute(geo.N, dPerm.as<int>(), orig, treeOut, s);
}

}  // namespace aniso
