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
    // symmetric U storage pays for single right-hand sides; a block handle (ks > 1,
    // the aniso.m operator) reads every near block directed.
    // ANISO_NEAR_SYMMETRIC=0/1 overrides.
    plan.nearSymmetric = ks == 1;
    if (const char* e = std::getenv("ANISO_NEAR_SYMMETRIC")) plan.nearSymmetric = e[0] == '1';
    plan.maxCanon = ks == 1 ? kMaxCanon : kMaxCanonBlock;
    // ANISO_NEAR_HS_SYM=1: the harmonic block apply stores the U pairs between owned
    // leaves once (Plan::nearSymHs; K <= 5: the canonical loop's registers leave K = 8
    // at one wave per SIMD).  Off by default: measured slower
    plan.nearSymHs = false;
    if (const char* e = std::getenv("ANISO_NEAR_HS_SYM")) plan.nearSymHs = ks > 1 && ks <= 5 && e[0] == '1';
    // ANISO_UPPER_PARTIAL=0: a sharded one-collective matvec exchanges the tier-0 roots
    // and runs the upper up tiers on every rank (the round-4 form)
    if (const char* e = std::getenv("ANISO_UPPER_PARTIAL")) plan.xUpPartialIn = std::atoi(e) != 0;
    plan.build(tree, np, 0, 1);
    plan.buildExchange(tree, geo.sz, geo.d2);
    plan.buildTopWait(tree);
    // block handles apply aniso.m's operator through the mode-shared E caches
    // (DESIGN.md §3.9); ANISO_HARMONIC=0 keeps the per-mode operator stream
    useAtt = ks > 1 && !plan.nearSymmetric;
    if (const char* e = std::getenv("ANISO_HARMONIC")) useAtt = useAtt && e[0] != '0';
    if (const char* e = std::getenv("ANISO_OVERLAP")) overlap = std::atoi(e);
    if (const char* e = std::getenv("ANISO_FUSE_SUB")) fuseSub = e[0] != '0';
    if (const char* e = std::getenv("ANISO_TOP_SPIN_LIMIT")) topSpinLimit = (unsigned)std::strtoul(e, nullptr, 10);
    if (const char* e = std::getenv("ANISO_TOP_TRACE")) topTraceOn = std::atoi(e) != 0;
    if (const char* e = std::getenv("ANISO_NEAR_IN_TOP")) nearInTop = std::atoi(e) != 0;
    if (const char* e = std::getenv("ANISO_NEAR_EARLY")) nearEarly = std::atoi(e) != 0;
    if (const char* e = std::getenv("ANISO_ONE_EXCHANGE")) oneXOn = std::atoi(e) != 0;
    if (const char* e = std::getenv("ANISO_SHARD_NEAR_EARLY")) shardNearEarly = std::atoi(e) != 0;
    if (const char* e = std::getenv("ANISO_UP_TAILS")) upTailsOn = std::atoi(e) != 0;
    if (const char* e = std::getenv("ANISO_NEAR_AFTER_PACK")) nearAfterPack = std::atoi(e) != 0;
    if (const char* e = std::getenv("ANISO_SIDE_PRIO")) sidePrio = std::atoi(e);
    if (const char* e = std::getenv("ANISO_DET_PER_TARGET")) detPerTarget = std::atoi(e) != 0;
    if (const char* e = std::getenv("ANISO_NEAR_UP")) nearUpOn = std::atoi(e) != 0;
    if (const char* e = std::getenv("ANISO_NEAR_ORDER")) nearOrderUp = std::strcmp(e, "first") != 0;
    hmRing = hm_ring_depth();
    if (const char* e = std::getenv("ANISO_HM_WPE")) hmWpe = std::atoi(e);
    if (const char* e = std::getenv("ANISO_NEAR_WPE")) nearWpe = std::atoi(e);
    if (const char* e = std::getenv("ANISO_TOP_FUSED")) topFusedMode = std::atoi(e) != 0 ? 1 : 0;
    sigma_s.assign(geo.N, 0.0);
    sigma_t.assign(geo.N, 0.0);
    modes.resize(kernelSize);
}

Operator::~Operator() {
    if (device >= 0) {
        int prev = -1;  // restore the caller's device (the destructor runs from Python __del__)
        (void)hipGetDevice(&prev);
        (void)hipSetDevice(device);
        if (comm) {  // the communicator before the streams its collectives ran on
            (void)hipDeviceSynchronize();
            comm.reset();
        }
        for (auto& e : evPool) (void)hipEventDestroy(e);
        if (evFork) (void)hipEventDestroy(evFork);
        if (evJoin) (void)hipEventDestroy(evJoin);
        if (side) (void)hipStreamDestroy(side);
        if (own) (void)hipStreamDestroy(own);
        if (topErr) (void)hipHostFree(topErr);
        if (prev >= 0) (void)hipSetDevice(prev);
    }
}

void Operator::getNodes(double* xy) const {
    for (int64_t i = 0; i < geo.N; ++i) {
        xy[i] = geo.px[i];
        xy[i + geo.N] = geo.py[i];
    }
}

void Operator::setShard(int rank, int nranks) {
    if (comm) {  // a communicator belongs to one shard layout; drain its collectives first
        if (device >= 0) HIP_CHECK(hipDeviceSynchronize());
        comm.reset();
        oxReady = false;
    }
    plan.build(tree, np, rank, nranks);
    plan.buildExchange(tree, geo.sz, geo.d2);
    plan.buildTopWait(tree);
    pend = Pending();
    for (auto& m : modes) {
        m.Knear.alloc(0);
        m.Km2l.alloc(0);
        m.ready = false;
    }
    f32Ready = false;
    mrhsPlanReady = false;
    m64.clear();
    if (device >= 0) uploadPlan();
}

void Operator::ensureDevice() {
    if (device >= 0) {
        HIP_CHECK(hipSetDevice(device));
        return;
    }
    HIP_CHECK(hipGetDevice(&device));
    HIP_CHECK(hipStreamCreateWithFlags(&own, hipStreamNonBlocking));
    // side stream at normal priority (a high-priority one measured slower, r01f; the
    // lowest priority 11-25 % slower, r04l; a CU-masked one serialised the two streams
    // on a rank of 8: 0.455 against 0.235 ms, r06q).  ANISO_SIDE_PRIO: -1 lowest, 1 highest
    if (sidePrio != 0) {
        int lo = 0, hi = 0;
        HIP_CHECK(hipDeviceGetStreamPriorityRange(&lo, &hi));
        HIP_CHECK(hipStreamCreateWithPriority(&side, hipStreamNonBlocking, sidePrio < 0 ? lo : hi));
    } else {
        HIP_CHECK(hipStreamCreateWithFlags(&side, hipStreamNonBlocking));
    }
    HIP_CHECK(hipEventCreateWithFlags(&evFork, hipEventDisableTiming));
    HIP_CHECK(hipEventCreateWithFlags(&evJoin, hipEventDisableTiming));
    HIP_CHECK(hipHostMalloc((void**)&topErr, sizeof(unsigned), hipHostMallocMapped | hipHostMallocCoherent));
    *(volatile unsigned*)topErr = 0;
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
    {  // per node {cx, cy, rx, ry}: the source box one LDS-DMA lane pair fetches (k_m2l_hcr)
        std::vector<double> g4((size_t)tree.nn * 4);
        for (int i = 0; i < tree.nn; ++i) {
            g4[4 * (size_t)i] = tree.ncx[i];
            g4[4 * (size_t)i + 1] = tree.ncy[i];
            g4[4 * (size_t)i + 2] = tree.nrx[i];
            g4[4 * (size_t)i + 3] = tree.nry[i];
        }
        up(dNodeGeo, g4);
    }
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
    hostP = P;
    // work arrays
    dCharge.alloc(geo.N * sizeof(double));
    dOut.alloc(geo.N * sizeof(double));
    dTmp.alloc(geo.N * sizeof(double));
    dTmp2.alloc(geo.N * sizeof(double));
    dTmpS.alloc(geo.N * sizeof(double));
    ensureWork(1);
    uploadPlan();
}

// Per-right-hand-side work arrays, sized for the largest K used so far:
// fT/cT [N][K], multipoles and locals [node][16][K], M2L and near partials.
void Operator::ensureWork(int K) {
    if (K <= workK) return;
    workK = K;
    dFT.alloc((size_t)geo.N * rhs_stride(K) * sizeof(double));
    dCT.alloc((size_t)geo.N * rhs_stride(K) * sizeof(double));
    dMult.alloc((size_t)tree.nn * kRank * K * sizeof(double));
    dLocal.alloc((size_t)tree.nn * kRank * K * sizeof(double));
    HIP_CHECK(hipMemset(dMult.p, 0, dMult.bytes));
    HIP_CHECK(hipMemset(dLocal.p, 0, dLocal.bytes));
    dM2LPart.alloc((size_t)std::max(plan.m2lCanon, 1) * kRank * K * sizeof(double));
    dNearPart.alloc((size_t)std::max<int64_t>({plan.nearPartTotal, plan.hsPartTotal, 1}) * K * sizeof(double));
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
    if (useAtt) {
        up(dAttPtr, plan.attPtr);
        up(dAttSrc, plan.attSrc);
        up(dAttBlk, plan.attBlk);
        std::vector<int> own(plan.attOwner), oth(plan.attOther);  // stored blocks, then the cluster plan's copies
        own.insert(own.end(), plan.hmCopyOwner.begin(), plan.hmCopyOwner.end());
        oth.insert(oth.end(), plan.hmCopyOther.begin(), plan.hmCopyOther.end());
        up(dAttOwner, own);
        up(dAttOther, oth);
        up(dHmClPtr, plan.hmClPtr);
        up(dHmTgt, plan.hmTgt);
        up(dHmPtr, plan.hmPtr);
        up(dHmSrc, plan.hmSrc);
        up(dHmBlk, plan.hmBlk);
        up(dHmSlot, plan.hmSlot);
        up(dHmNDir, plan.hmNDir);
        up(dHmClWait, plan.hmClWait);
        up(dHmHaloPtr, plan.hmHaloPtr);
        up(dHmHaloPos, plan.hmHaloPos);
        dHmClBound.alloc(0);  // the deterministic sums' bounds follow the plan (detBounds)
        dTopCnt.alloc((kMaxTopTiers + 1) * sizeof(unsigned));
        dTopSteals.alloc(sizeof(unsigned));
        HIP_CHECK(hipMemset(dTopSteals.p, 0, sizeof(unsigned)));
        attReady = false;
    }
    up(dM2LCanonBase, plan.m2lCanonBase);
    up(dM2LInPtr, plan.m2lInPtr);
    up(dM2LOutSlot, plan.m2lOutSlot);
    dM2LPart.alloc((size_t)std::max(plan.m2lCanon, 1) * kRank * workK * sizeof(double));
    std::vector<int2> ns(plan.nearSym.size());
    for (size_t i = 0; i < ns.size(); ++i) ns[i] = make_int2(plan.nearSym[i][0], plan.nearSym[i][1]);
    up(dNearSym, ns);
    up(dDnLeafNear, plan.dnLeafNear);
    up(dDnDesc, to_int4(plan.dnDesc));
    up(dDnGrpFix, plan.dnGrpFix);
    up(dDnLeafGeom, plan.dnLeafGeom);
    up(dDnChainPtr, plan.dnChainPtr);
    up(dDnChain, plan.dnChain);
    up(dDnChainFold, plan.dnChainFold);
    up(dDnNearPtr, plan.dnNearPtr);
    up(dDnNearOff, plan.dnNearOff);
    dNearPart.alloc((size_t)std::max<int64_t>({plan.nearPartTotal, plan.hsPartTotal, 1}) * workK * sizeof(double));
    if (plan.nearSymHsOn) {
        up(dHsPtsPtr, plan.hsPtsPtr);
        up(dHsLoc, plan.hsLoc);
        up(dHsKOff, plan.hsKOff);
        std::vector<int2> hs(plan.hsSym.size());
        for (size_t i = 0; i < hs.size(); ++i) hs[i] = make_int2(plan.hsSym[i][0], plan.hsSym[i][1]);
        up(dHsSym, hs);
        up(dHsSrcPtr, plan.hsSrcPtr);
        up(dHsSrc, plan.hsSrc);
        up(dHsDst, plan.hsDst);
        up(dNearSelfRow, plan.nearSelfRow);
        up(dNearGrpInPtr, plan.nearGrpInPtr);
        up(dNearGrpIn, plan.nearGrpIn);
    }
    up(dLeafInfo, to_int4(plan.leafInfo));
    up(dNearPtsPtr, plan.nearPtsPtr);
    up(dNearPts, plan.nearPts);
    up(dXT0Tasks, plan.xT0Tasks);
    up(dXOwnT0Tasks, plan.xOwnT0Tasks);
    up(dXUpTask, plan.xUpTask);
    up(dXT0Part, plan.xT0Part);
    up(dXUpRoots, plan.xUpRoots);
    dXUpCnt.alloc(std::max<size_t>(plan.xUpRoots.size(), 1) * sizeof(unsigned));
    HIP_CHECK(hipMemset(dXUpCnt.p, 0, dXUpCnt.bytes));  // each tail resets its counter after use
    up(dNearUpGrp, plan.nearUpGrp);
    up(dNearGrpEarly, plan.nearGrpEarly);
    up(dNearGrpLate, plan.nearGrpLate);
    up(dXRootRecv, plan.xRootRecv);
    up(dNsPtr, plan.nsPtr);
    up(dNsPts, plan.nsPts);
    up(dNearLoc, plan.nearLoc);
    up(dNearCorrRow, plan.nearCorrRow);
    up(dXRootSlot, plan.xRootSlot);
    up(dXSendSlot, plan.xSendSlot);
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
    if (up_tier_lds(plan.upMaxTask, 1) > 160 * 1024 ||
        down_tier_lds(plan.dnMaxTask, plan.dnMaxLeaves, plan.dnMaxNear, plan.dnMaxChain, 1) > 160 * 1024)
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
    attReady = false;
    f32Ready = false;  // config 5's fp32 caches are rounded from the mode-0 operators of sigma_t
    m64.clear();       // ... and the fp64 16-RHS caches are the modes' operators
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
    if (id == 0) f32Ready = false;  // rebuilt from the new mode-0 operators at the next fp32 apply
    m64.erase(id);
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
    if (useAtt && !attReady) buildAttCache();
    CorrTables ct;
    ct.build(geo, id);
    up(mc.C, ct.C);
    up(mc.mu, ct.mu);
    mc.hostC = ct.C;
    mc.hostMu = ct.mu;
    HIP_CHECK(hipStreamSynchronize(own));  // folded tables may still be read by queued work
    corrTabs.clear();
    HIP_CHECK(hipStreamSynchronize(own));
    mc.ready = true;
}

// The mode-shared caches: E = e^-tau for every directed M2L pair
// (column-major 16 x 16) and near block (the directed near layout), and sigma_t at
// every point (the mode-0 diagonal).  Built once per setCoeff on a block handle.
void Operator::buildAttCache() {
    const Params* P = dParams.as<Params>();
    const int64_t npairs = (int64_t)(plan.attOwner.size() + plan.hmCopyOwner.size());  // stored blocks + copies
    dAttM2L.alloc((size_t)npairs * 256 * sizeof(double));
    // the near blocks in the layout the harmonic near field reads: directed, or with
    // symmetric U storage its own lists (Plan::buildNearHs)
    const bool hs = plan.nearSymHsOn;
    const std::vector<int64_t>& nptr = hs ? plan.hsSrcPtr : plan.nearPtr;
    dAttNear.alloc((size_t)(hs ? plan.hsKTotal : plan.nearKTotal) * sizeof(double));
    dSigDiag.alloc((size_t)geo.N * sizeof(double));
    int maxSrc = 1;
    for (size_t li = 0; li < plan.leaves.size(); ++li) maxSrc = std::max<int>(maxSrc, (int)(nptr[li + 1] - nptr[li]));
    launch_cache_att_m2l(npairs, dAttOwner.as<int>(), dAttOther.as<int>(), dNcx.as<double>(), dNcy.as<double>(),
                         dNrx.as<double>(), dNry.as<double>(), dStCoef.as<double>(), P, dAttM2L.as<double>(), own);
    launch_cache_near((int)plan.leaves.size(), dLeaves.as<int>(), (hs ? dHsSrcPtr : dNearPtr).as<int64_t>(),
                      (hs ? dHsSrc : dNearSrc).as<int>(), (hs ? dHsKOff : dNearKOff).as<int64_t>(),
                      dBegin.as<int64_t>(), dCount.as<int64_t>(), dPxT.as<double>(), dPyT.as<double>(),
                      dStCoef.as<double>(), P, kAttMode, maxSrc, dAttNear.as<double>(), own);
    launch_sigma_diag(geo.N, dPxT.as<double>(), dPyT.as<double>(), dStCoef.as<double>(), P, dSigDiag.as<double>(),
                      own);
    if (!dAttMax.bytes) dAttMax.alloc(sizeof(double));
    launch_abs_max(npairs * 256, dAttM2L.as<double>(), dAttMax.as<double>(), own);
    HIP_CHECK(hipStreamSynchronize(own));
    attReady = true;
}

// The deterministic sums' geometric bound per cluster (harmonic.hip hc_det_scale):
// 2 x 16 columns x the most pair products one of its LDS slots receives x the largest
// 1 / gap over its pairs (gap: the boxes' separation along the wider axis, a lower
// bound on the distance of any two of their Chebyshev nodes).
void Operator::detBounds() {
    const int ncl = (int)plan.hmClPtr.size() - 1;
    if (ncl <= 0 || dHmClBound.bytes >= (size_t)ncl * sizeof(double)) return;
    std::vector<double> bound(ncl);
    std::vector<int> cnt;
    for (int c = 0; c < ncl; ++c) {
        const int c0 = plan.hmClPtr[c], nt = plan.hmClPtr[c + 1] - c0;
        const int nh = plan.hmHaloPtr.empty() ? 0 : plan.hmHaloPtr[c + 1] - plan.hmHaloPtr[c];
        cnt.assign(nt + nh, 0);
        double ig = 0.0;
        for (int ti = 0; ti < nt; ++ti) {
            const int t = plan.hmTgt[c0 + ti];
            const int64_t p0 = plan.hmPtr[c0 + ti], pd = p0 + plan.hmNDir[c0 + ti], p1 = plan.hmPtr[c0 + ti + 1];
            for (int64_t e = p0; e < p1; ++e) {
                const int n = plan.hmSrc[e];
                const double gx = std::fabs(tree.ncx[t] - tree.ncx[n]) - tree.nrx[t] - tree.nrx[n];
                const double gy = std::fabs(tree.ncy[t] - tree.ncy[n]) - tree.nry[t] - tree.nry[n];
                const double gap = std::max(gx, gy);
                if (!(gap > 0.0)) throw std::logic_error("deterministic M2L: a V-list pair of touching boxes");
                ig = std::max(ig, 1.0 / gap);
                ++cnt[ti];
                if (e >= pd) ++cnt.at(plan.hmSlot[e]);
            }
        }
        const int most = cnt.empty() ? 0 : *std::max_element(cnt.begin(), cnt.end());
        bound[c] = 2.0 * 16.0 * most * ig;
    }
    up(dHmClBound, bound);
}

// Do the terms of a batched apply have aniso.m's harmonic structure (harmonic.hip)?
// Terms must be modes 0, 1, ..., nterm-1 with mix[m][i][b] = sum over j with |j| = b,
// |i + j| = m of w_b; w comes from output row 0 (mix[b][0][b] = hw_b).  Rows that are
// all zero (padded right-hand sides) are masked out.
bool Operator::harmonicWeights(int K, int nterm, const int* ids, const double* mixes, HarmWeights& hw) const {
    if (!useAtt || !attReady || plan.nearPartTotal > 0 || K < 2 || K > kMaxRhs || nterm > 2 * K - 1) return false;
    if (!(K == 2 || K == 4 || K == 5 || K == 8)) return false;
    for (int t = 0; t < nterm; ++t)
        if (ids[t] != t) return false;
    std::memset(&hw, 0, sizeof(hw));
    auto mx = [&](int m, int i, int b) { return m < nterm ? mixes[((size_t)m * K + i) * K + b] : 0.0; };
    double mag = 0.0;
    for (int t = 0; t < nterm * K * K; ++t) mag = std::max(mag, std::fabs(mixes[t]));
    for (int i = 0; i < K; ++i) {
        bool any = false;
        for (int m = 0; m < nterm; ++m)
            for (int b = 0; b < K; ++b) any = any || mx(m, i, b) != 0.0;
        hw.om[i] = any ? 1.0 : 0.0;
    }
    if (hw.om[0] == 0.0) return false;
    for (int b = 0; b < K; ++b) hw.hw[b] = mx(b, 0, b);
    std::vector<double> want((size_t)(2 * K - 1) * K * K, 0.0);
    for (int i = 0; i < K; ++i)
        for (int j = -(K - 1); j <= K - 1; ++j) {
            const int b = std::abs(j), m = std::abs(i + j);
            want[((size_t)m * K + i) * K + b] += b == 0 ? hw.hw[0] : 0.5 * hw.hw[b];
        }
    for (int i = 0; i < K; ++i) {
        if (hw.om[i] == 0.0) continue;
        hw.dw[i] = want[((size_t)0 * K + i) * K + i];
        for (int m = 0; m < 2 * K - 1; ++m)
            for (int b = 0; b < K; ++b)
                if (std::fabs(want[((size_t)m * K + i) * K + b] - mx(m, i, b)) > 1e-13 * mag) return false;
    }
    return true;
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
    checkDeviceErrors();
}

// k right-hand sides of one mode: up to 8 per batched apply (identity mix), or, for
// more than 8 on an unsharded handle, 16 per apply of the fp64 MFMA operator
// (f64op.hip; zero columns pad the last chunk).  That operator keeps its own fp64
// copy of the mode's operators on the directed lists (mrhs64Bytes: about 6 GB per
// mode at 1M points, 24 GB at 4M), freed by setCoeff / cache(id): it is used only
// when that copy fits in the free HBM, else the 8-column batches run.
void Operator::mappingBatchedHost(const double* Q, int k, int id, double* Out) {
    if (k == 0) return;
    ensureDevice();
    const int64_t N = geo.N;
    bool mfma = k > 8 && plan.nranks == 1;
    if (mfma && !m64.count(id) && id >= 0 && id < kernelSize && modes[id].ready) {
        // the plan first (mrhs64Bytes builds and uploads it), then the free HBM it leaves
        const size_t need = mrhs64Bytes() + (size_t)64 * N * sizeof(double);  // + the four 16-column staging buffers
        size_t freeB = 0, totalB = 0;
        HIP_CHECK(hipMemGetInfo(&freeB, &totalB));
        mfma = need + (size_t)(1ull << 30) <= freeB;  // keep a GiB of headroom
    }
    if (mfma) {
        if (id < 0 || id >= kernelSize) throw std::out_of_range("kernel id out of range");
        if (!modes[id].ready)
            throw std::runtime_error("mapping on kernel id " + std::to_string(id) + " before cache(" + std::to_string(id) + ")");
        DevBuf dq, dout, x16, y16;
        dq.alloc((size_t)16 * N * sizeof(double));
        dout.alloc((size_t)16 * N * sizeof(double));
        x16.alloc((size_t)16 * N * sizeof(double));
        y16.alloc((size_t)16 * N * sizeof(double));
        for (int j0 = 0; j0 < k; j0 += 16) {
            const int kc = std::min(16, k - j0);
            HIP_CHECK(hipMemcpyAsync(dq.p, Q + (size_t)j0 * N, (size_t)kc * N * sizeof(double), hipMemcpyHostToDevice,
                                     own));
            launch64_gather16(N, kc, dPerm.as<int>(), dq.as<double>(), x16.as<double>(), own);
            mrhs64Dev(id, false, x16.as<double>(), y16.as<double>(), own);
            launch64_scatter16(N, kc, dPerm.as<int>(), y16.as<double>(), dout.as<double>(), own);
            HIP_CHECK(hipMemcpyAsync(Out + (size_t)j0 * N, dout.p, (size_t)kc * N * sizeof(double),
                                     hipMemcpyDeviceToHost, own));
            HIP_CHECK(hipStreamSynchronize(own));
        }
        checkDeviceErrors();
        return;
    }
    const int kb = std::min(k, 8);
    DevBuf dq, dout;
    dq.alloc((size_t)kb * N * sizeof(double));
    dout.alloc((size_t)kb * N * sizeof(double));
    for (int j0 = 0; j0 < k; j0 += kb) {
        const int nb = std::min(kb, k - j0);
        std::vector<double> eye((size_t)nb * nb, 0.0);
        for (int i = 0; i < nb; ++i) eye[(size_t)i * nb + i] = 1.0;
        HIP_CHECK(hipMemcpyAsync(dq.p, Q + (size_t)j0 * N, (size_t)nb * N * sizeof(double), hipMemcpyHostToDevice, own));
        if (plan.nranks > 1) HIP_CHECK(hipMemsetAsync(dout.p, 0, dout.bytes, own));
        applyBlock(nb, dq.as<double>(), N, false, nullptr, 1, &id, eye.data(), dout.as<double>(), N, false, own,
                   kStageAll);
        HIP_CHECK(hipMemcpyAsync(Out + (size_t)j0 * N, dout.p, (size_t)nb * N * sizeof(double), hipMemcpyDeviceToHost,
                                 own));
        HIP_CHECK(hipStreamSynchronize(own));
        checkDeviceErrors();
    }
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
    forwardTreePhase(0, xTree, ySlice, nullptr, nullptr, s);
}

void Operator::forwardTreePhase(int phase, const double* xTree, double* ySlice, double* rootsSend,
                                const double* rootsRecv, hipStream_t s) {
    if (!modeCached(0)) throw std::runtime_error("forward operator before cache(0)");
    ensureDevice();
    pendingCall(phase, PendingCall{0, 0, xTree, ySlice, dSigmaT.p, geo.N, 0, 0.0});
    const double one = 1.0;
    const int id = 0;
    applyBlock(1, xTree, geo.N, true, dSigmaT.as<double>(), 1, &id, &one, dTmpS.as<double>(), geo.N, true, s,
               kStageAll, phase, rootsSend, rootsRecv);
    if (phase == 1) return;
    const int64_t n = plan.ownEnd - plan.ownBegin;
    launch_sub_slice(n, 1, xTree + plan.ownBegin, n, dTmpS.as<double>(), n, ySlice, n, s);
}

void Operator::apply(const double* charge, bool treeIn, const double* sigT, int id, double* out, bool treeOut,
                     hipStream_t s, int mask) {
    const double one = 1.0;
    applyBlock(1, charge, geo.N, treeIn, sigT, 1, &id, &one, out, geo.N, treeOut, s, mask);
}

void Operator::applyBlockDev(int nrhs, const double* x, int64_t ldx, bool treeIn, bool useSigma, int nterm,
                             const int* ids, const double* mixes, double* out, int64_t ldo, bool treeOut,
                             hipStream_t s, int mask) {
    if (useSigma && !coeffSet) throw std::runtime_error("block apply with sigma_s before setCoeff");
    ensureDevice();
    applyBlock(nrhs, x, ldx, treeIn, useSigma ? dSigmaT.as<double>() : nullptr, nterm, ids, mixes, out, ldo, treeOut,
               s, mask);
}

int Operator::mark(hipStream_t s) {
    if (evUsed == (int)evPool.size()) {
        hipEvent_t e;
        HIP_CHECK(hipEventCreate(&e));
        evPool.push_back(e);
    }
    HIP_CHECK(hipEventRecord(evPool[evUsed], s));
    return evUsed++;
}

// Device table of the mode terms of a batched apply (operator pointers, sign and
// K x K mix per term).  Tables are cached by content: a block operator reuses one
// table every call, so no upload sits on the apply's path.
const ModeArgs* Operator::modeTable(int K, int nterm, const int* ids, const double* mixes) {
    std::vector<ModeArgs> tab(nterm);
    std::memset(tab.data(), 0, tab.size() * sizeof(ModeArgs));
    for (int t = 0; t < nterm; ++t) {
        const ModeCache& mc = modes[ids[t]];
        ModeArgs& m = tab[t];
        m.Km2l = mc.Km2l.as<double>();
        m.Knear = mc.Knear.as<double>();
        m.C = mc.C.as<double>();
        m.mu = mc.mu.as<double>();
        m.sgn = (ids[t] % 2 == 0) ? 1.0 : -1.0;  // K_{B<-A} = (-1)^m K_{A<-B}^T
        for (int i = 0; i < K; ++i)
            for (int b = 0; b < K; ++b) m.mix[i][b] = mixes[((size_t)t * K + i) * K + b];
    }
    std::string key(reinterpret_cast<const char*>(tab.data()), tab.size() * sizeof(ModeArgs));
    auto it = modeTabs.find(key);
    if (it != modeTabs.end()) return it->second.as<ModeArgs>();
    if (modeTabs.size() >= 64) {  // bound the cache; hipFree waits for work that may still read a table
        HIP_CHECK(hipDeviceSynchronize());
        modeTabs.clear();
    }
    DevBuf& buf = modeTabs[key];
    buf.upload(tab.data(), tab.size() * sizeof(ModeArgs));
    return buf.as<ModeArgs>();
}

// The correction tables of a batched apply, folded over its terms on the host:
// Wc[tq][q9][c][i][b] = sum_t mix_t[i][b] C_t[tq][q9][c] and
// Wm[tq][i][b][a][bb] = sum_t mix_t[i][b] mu_t[tq][a][bb] (k_corr).  Cached by
// content, like the mode table.
const CorrFold& Operator::corrTable(int K, int nterm, const int* ids, const double* mixes) {
    std::string key(reinterpret_cast<const char*>(&K), sizeof(int));
    key.append(reinterpret_cast<const char*>(ids), nterm * sizeof(int));
    key.append(reinterpret_cast<const char*>(mixes), (size_t)nterm * K * K * sizeof(double));
    auto it = corrTabs.find(key);
    if (it != corrTabs.end()) return it->second;
    const int d = geo.d, d2 = geo.d2;
    std::vector<double> wc((size_t)d2 * 9 * d2 * K * K, 0.0), wm((size_t)d2 * K * K * d2, 0.0);
    for (int t = 0; t < nterm; ++t) {
        const ModeCache& mc = modes[ids[t]];
        for (int i = 0; i < K; ++i)
            for (int b = 0; b < K; ++b) {
                const double w = mixes[((size_t)t * K + i) * K + b];
                if (w == 0.0) continue;
                for (int tq = 0; tq < d2; ++tq) {
                    for (int q = 0; q < 9 * d2; ++q)  // (q9, c)
                        wc[(((size_t)tq * 9 * d2 + q) * K + i) * K + b] += w * mc.hostC[(size_t)tq * 9 * d2 + q];
                    for (int ab = 0; ab < d * d; ++ab)
                        wm[(((size_t)tq * K + i) * K + b) * d2 + ab] += w * mc.hostMu[(size_t)tq * d * d + ab];
                }
            }
    }
    if (corrTabs.size() >= 64) {  // bound the cache; hipFree waits for work that may still read a table
        HIP_CHECK(hipDeviceSynchronize());
        corrTabs.clear();
    }
    CorrFold& f = corrTabs[key];
    up(f.Wc, wc);
    up(f.Wm, wm);
    return f;
}

// One batched apply: the up pass over the K base vectors, then per term t (mode
// ids[t], mix mixes[t]) the near field, the corrections, the M2L stream and its
// gather, each accumulating; then one down pass.  sigT (sigma_s in tree order, or
// nullptr) multiplies the inputs at their tree positions.
//
// phase 1 / 2 split a sharded apply around the caller's all-gather of the tier-0
// root multipoles: phase 1 runs this rank's tier-0 up tasks only
// (plan.xT0Tasks), packs its roots into rootsSend and starts the near field and
// corrections (they need only the weighted charges of the rank's own and halo
// points); phase 2 scatters rootsRecv, runs the upper tiers (every rank), the M2L
// and the down pass.
void Operator::applyBlock(int K, const double* x, int64_t ldx, bool treeIn, const double* sigT, int nterm,
                          const int* ids, const double* mixes, double* out, int64_t ldo, bool treeOut, hipStream_t s,
                          int mask, int phase, double* rootsSend, const double* rootsRecv) {
    if (K < 1 || K > 8) throw std::invalid_argument("block apply supports 1..8 right-hand sides, got " + std::to_string(K));
    checkDeviceErrors();
    if (nterm < 1) throw std::invalid_argument("block apply needs at least one mode term");
    for (int t = 0; t < nterm; ++t) {
        if (ids[t] < 0 || ids[t] >= kernelSize) throw std::out_of_range("kernel id out of range");
        if (!modes[ids[t]].ready)
            throw std::runtime_error("mapping on kernel id " + std::to_string(ids[t]) + " before cache(" + std::to_string(ids[t]) + ")");
    }
    if (phase != 0 && !treeIn) throw std::invalid_argument("a sharded (two-phase) apply takes tree-order input");
    if (phase == 1 && plan.xRootChunk > 0 && !rootsSend) throw std::invalid_argument("sharded apply: null roots_send");
    if (phase == 2 && plan.xRootChunk > 0 && !rootsRecv) throw std::invalid_argument("sharded apply: null roots_recv");
    if (phase == 2 && !(pend.active && pend.K == rootRhs(K)))
        throw std::logic_error("sharded apply: end without a matching begin");
    ensureDevice();
    const int64_t nOut = treeOut ? plan.ownEnd - plan.ownBegin : geo.N;
    if (ldx < geo.N || ldo < nOut) throw std::invalid_argument("block apply: leading dimension too small");
    if (!rhs_supported(K)) {  // pad with zero right-hand sides to the next compiled count
        const int Kp = rhs_padded(K);
        dPadIn.alloc((size_t)Kp * geo.N * sizeof(double));
        dPadOut.alloc((size_t)Kp * geo.N * sizeof(double));
        if (phase != 2) {  // phase 2 reads what phase 1 staged
            HIP_CHECK(hipMemsetAsync(dPadIn.p, 0, dPadIn.bytes, s));
            HIP_CHECK(hipMemcpy2DAsync(dPadIn.p, geo.N * sizeof(double), x, ldx * sizeof(double),
                                       geo.N * sizeof(double), K, hipMemcpyDeviceToDevice, s));
        }
        std::vector<double> mp((size_t)nterm * Kp * Kp, 0.0);
        for (int t = 0; t < nterm; ++t)
            for (int i = 0; i < K; ++i)
                for (int b = 0; b < K; ++b) mp[((size_t)t * Kp + i) * Kp + b] = mixes[((size_t)t * K + i) * K + b];
        applyBlock(Kp, dPadIn.as<double>(), geo.N, treeIn, sigT, nterm, ids, mp.data(), dPadOut.as<double>(), geo.N,
                   treeOut, s, mask, phase, rootsSend, rootsRecv);
        if (phase != 1)
            HIP_CHECK(hipMemcpy2DAsync(out, ldo * sizeof(double), dPadOut.p, geo.N * sizeof(double),
                                       nOut * sizeof(double), K, hipMemcpyDeviceToDevice, s));
        return;
    }
    ensureWork(K);
    if (up_tier_lds(plan.upMaxTask, K) > 160 * 1024 ||
        down_tier_lds(plan.dnMaxTask, plan.dnMaxLeaves, plan.dnMaxNear, plan.dnMaxChain, K) > 160 * 1024)
        throw std::logic_error("up/down pass task exceeds one workgroup's LDS at " + std::to_string(K) + " right-hand sides");
    const Params* P = dParams.as<Params>();
    const bool tr = timeStages != 0;  // the roofline spans: M2L (stage 2), near field (4)
    const bool tm = timeStages == 1;  // every stage
    auto span = [&](int stage, int a, int b) {
        if (a >= 0 && b >= 0) spans.push_back({stage, a, b});
    };
    const int* operm = treeOut ? nullptr : dPerm.as<int>();
    const int64_t obase = treeOut ? plan.ownBegin : 0;
    const double scale = M_1_PI / 2.0;  // AnisoWrapper.cpp:129-130
    HarmWeights hw;
    const bool harmonic = harmonicWeights(K, nterm, ids, mixes, hw);
    // the harmonic block apply runs its near field + corrections (they write `out`)
    // on a side stream beside the M2L (it writes the locals), forked as soon as the
    // weighted charges are complete: after the last up tier with a P2M leaf
    const ModeArgs* tab = modeTable(K, nterm, ids, mixes);
    const CorrFold& cf = corrTable(K, nterm, ids, mixes);
    const NearCorr nc{dNearCorrRow.as<uint16_t>(), dPerm.as<int>(), dIperm.as<int>(), dCT.as<double>(),
                      cf.Wc.as<double>(), cf.Wm.as<double>(), P};
    const int ntier = (int)plan.upTierTask.size() - 1;  // 0: a lone leaf
    // a sharded one-collective matvec with the upper multipoles as partial sums
    // (blockOpShardedDev, Plan::xUpPartial): phase 1 forms this rank's records, the
    // exchange's unpack sums them, phase 2 runs no up tier
    const bool upPartial = oneXActive && upActive && phase != 0;
    // the upper tiers ride in the M2L launch (k_top_m2l_hc) when every leaf is in the
    // bottom tier: the near field then forks after it
    const bool topFused = harmonic && (mask & kStageFar) && topFusedOn() && !upPartial;
    // ANISO_NEAR_IN_TOP: the near field (+ corrections) as the last blocks of that
    // launch (the one-block M2L form; a shard's phase 1 then leaves it to phase 2)
    const bool ringOn = hmRing > 0 && hm_ring_xl(K, plan.hmMaxLds, hmRing) >= 0;
    // symmetric U storage (Plan::nearSymHsOn): the harmonic near field reads its own
    // column lists and leaves the partner products of other groups to the down pass
    const bool hsSym = harmonic && plan.nearSymHsOn;
    const bool nearFused = topFused && overlapOn() && nearInTop && !ringOn && !hsSym && plan.nearCorrOk &&
                           near_hs_fusable((int)plan.leaves.size(), plan.nearMaxLeaf, plan.nsMax,
                                           dNearLoc.as<uint16_t>(), &nc, mask);
    const bool fork = harmonic && overlapOn() && !nearFused;
    const hipStream_t sn = fork ? side : s;
    // the staged near field with its fused corrections forms its charges from the
    // input itself (NearHsArgs::xin), so it needs nothing from the up pass: it forks
    // at the start of the apply, beside the latency-bound up tiers, and the up pass
    // stores no fT / cT (ANISO_NEAR_EARLY=0: it forks after the up pass and reads them)
    const bool nearIn = harmonic && nearEarly && !nearFused && plan.nearCorrOk && (mask & kStageNear) &&
                        near_hs_fusable((int)plan.leaves.size(), plan.nearMaxLeaf, plan.nsMax,
                                        dNearLoc.as<uint16_t>(), &nc, mask);
    // the one-collective exchange (blockOpShardedDev): phase 1 runs the own tier-0
    // tasks only and leaves the near field to phase 2, after the exchange
    const bool oneX = oneXActive && phase != 0;
    if (oneX && !(harmonic && nearIn))
        throw std::logic_error("one-collective exchange: the apply is not the harmonic one with its near field from the input");
    double* const fTw = nearIn ? nullptr : dFT.as<double>();
    double* const cTw = nearIn ? nullptr : dCT.as<double>();
    // the near field forks after the whole up pass on one GPU: forked after the
    // bottom tier it starved the latency-bound upper tiers the M2L waits on (up pass
    // 0.25 -> 0.14 ms, 644 -> 660 block matvec/s); a sharded apply starts it in
    // phase 1, beside the root exchange (8 shards: 0.317 vs 0.327 ms per rank)
    const int forkTier = phase == 0 && !topFused ? std::max(ntier - 1, 0) : plan.upLastLeafTier;
    // one up tier; a sharded apply's bottom tier runs this rank's tasks only (list)
    // and stores its tier-0 roots into send, its next tier reads the gathered ones
    // the partial tasks of the upper multipoles ride as tails of the own tier-0 launch
    // (blockOpShardedDev decides: upTailActive; they write into the send buffer)
    UpTail tail;
    if (upPartial && upTailActive) {
        tail.partOf = dXT0Part.as<int2>();
        const size_t sb = plan.xUpRoots.size() * 16 * kRank * K * sizeof(double);
        if (dXUpStage.bytes < sb) dXUpStage.alloc(sb);
        tail.stage = dXUpStage.as<double>();
        tail.cnt = dXUpCnt.as<unsigned>();
        tail.nroots = dXUpRoots.as<int>();
        tail.task = dXUpTask.as<int>();
        tail.rec = dXUpRec.as<double>();
        tail.nPeer = (int)oxRootParts;
        tail.peerOff = dOxRootSend.as<int64_t>();
        tail.buf = dOxSendBuf.as<double>();
    }
    auto upTier = [&](int k, const int* list, int ntask, const double* recv, double* send, const UpTail* tl = nullptr) {
        launch_up_tier(K, ntask, plan.upTierTask[k], list, plan.upTierMaxTask[k], dUpDesc.as<int4>(), dUpGrpFix.as<int>(),
                       dUpNode.as<int>(), dUpCode.as<int4>(), dUpGeom.as<double4>(), dUpLeaf.as<int2>(),
                       dPxT.as<double>(), dPyT.as<double>(), x, ldx, treeIn ? 1 : 0, dPerm.as<int>(), sigT,
                       dWT.as<double>(), fTw, cTw, P, dMult.as<double>(),
                       recv ? dXRootSlot.as<int>() : nullptr, recv, send ? dXSendSlot.as<int>() : nullptr, send, s,
                       topFused && k == 0 ? dTopCnt.as<unsigned>() : nullptr, tl);
        if (fork && !nearIn && k == forkTier) HIP_CHECK(hipEventRecord(evFork, s));
    };
    auto tierTasks = [&](int k) { return plan.upTierTask[k + 1] - plan.upTierTask[k]; };
    NearHsArgs nin{};  // nearIn: the input the near field forms its charges from
    if (nearIn) {
        nin.xin = x;
        nin.ldi = ldx;
        nin.treeIn = treeIn ? 1 : 0;
        nin.perm = dPerm.as<int>();
        nin.sigT = sigT;
        nin.wT = dWT.as<double>();
    }
    // the bottom up tier inside the staged near field (one GPU, serial: the near field
    // runs first, so tier 1 -- in the fused launch or its own -- finds the tier-0 roots)
    // (K <= 5: the 4-wave near kernel with the tail spills at K = 8)
    const bool nearUp = phase == 0 && nearIn && !fork && nearUpTier() && ntier >= 1 && !hsSym && K <= 5;
    if (nearUp) {
        nin.upMult = dMult.as<double>();
        nin.upGrp = dNearUpGrp.as<int>();
        nin.upP = P;
        nin.upNcx = dNcx.as<double>();
        nin.upNcy = dNcy.as<double>();
        nin.upNrx = dNrx.as<double>();
        nin.upNry = dNry.as<double>();
        nin.zeroCnt = topFused ? dTopCnt.as<unsigned>() : nullptr;
    }
    if (hsSym) {
        nin.nearSym = dHsSym.as<int2>();
        nin.colDst = dHsDst.as<int>();
        nin.selfRow = dNearSelfRow.as<uint16_t>();
        nin.nearPart = dNearPart.as<double>();
        nin.grpInPtr = dNearGrpInPtr.as<int>();
        nin.grpIn = dNearGrpIn.as<int>();
        nin.grpSlots = plan.nearGrpSlots;
    }
    const int64_t* const hmPtsPtr = (hsSym ? dHsPtsPtr : dNearPtsPtr).as<int64_t>();
    const int64_t* const hmKOff = (hsSym ? dHsKOff : dNearKOff).as<int64_t>();
    const uint16_t* const hmLoc = (hsSym ? dHsLoc : dNearLoc).as<uint16_t>();
    // near field + corrections (they need only fT / cT, or with nearIn the input)
    auto nearStage = [&] {
        if (fork) HIP_CHECK(hipStreamWaitEvent(side, evFork, 0));
        const int en = tr ? mark(sn) : -1;
        bool corrFused = false;
        if (harmonic) {
            // the corrections ride in the staged near kernel (d = 1, its table holds
            // every stencil neighbour; Plan::nearCorrRow)
            corrFused = launch_near_hm(K, (int)plan.leaves.size(), plan.nearMaxLeaf, dLeafInfo.as<int4>(), hmPtsPtr,
                           dNearPts.as<int>(), hmKOff, dAttNear.as<double>(), dPxT.as<double>(), dPyT.as<double>(),
                           dSigDiag.as<double>(), hw, dFT.as<double>(), operm, obase, ldo, mask, scale, out, hmLoc,
                           dNsPtr.as<int64_t>(), dNsPts.as<int>(), plan.nsMax, plan.nearCorrOk ? &nc : nullptr,
                           nearWpe, sn, &nin);
        } else if (plan.nearPartTotal > 0) {
            // symmetric U storage (K = 1 handles): one launch per term; the transposed
            // products go to partials summed over the terms
            for (int t = 0; t < nterm; ++t) {
                const int id = ids[t];
                // K_{B<-A} = (-1)^m K_{A<-B}^T for the merged kernel; Id = m
                const double sgn = (id % 2 == 0) ? 1.0 : -1.0;
                launch_near_sym(K, (int)plan.leaves.size(), dLeafInfo.as<int4>(), dNearPtsPtr.as<int64_t>(),
                                dNearPts.as<int>(), dNearKOff.as<int64_t>(), dNearSym.as<int2>(),
                                modes[id].Knear.as<double>(), dFT.as<double>(), mixes + (size_t)t * K * K, operm,
                                obase, ldo, maxNearS, mask, sgn, scale, t > 0 ? 1 : 0, dNearPart.as<double>(), out, s);
            }
        } else {  // directed storage: all terms in one launch
            launch_near(K, (int)plan.leaves.size(), plan.nearMaxLeaf, dLeafInfo.as<int4>(), dNearPtsPtr.as<int64_t>(),
                        dNearPts.as<int>(), dNearKOff.as<int64_t>(), tab, nterm, dFT.as<double>(), operm, obase, ldo,
                        mask, scale, 0, out, s);
        }
        const int e1 = tr ? mark(sn) : -1;
        span(4, en, e1);
        if (!corrFused)
            launch_corr(K, geo.d, plan.ownBegin, plan.ownEnd, dPerm.as<int>(), dIperm.as<int>(), dCT.as<double>(),
                        dFT.as<double>(), cf.Wc.as<double>(), cf.Wm.as<double>(), P, mask, scale, treeOut, ldo, out, sn);
        const int e2 = tm ? mark(sn) : -1;
        span(6, e1, e2);
        if (fork) HIP_CHECK(hipEventRecord(evJoin, side));
    };
    const bool clustered = harmonic && useClusters;
    const int ncl = (int)plan.hmClPtr.size() - 1;
    HcArgs hca{dHmClPtr.as<int>(), dHmTgt.as<int>(), dHmPtr.as<int64_t>(), dHmNDir.as<int>(), dHmSrc.as<int>(),
                     dHmBlk.as<int>(), dHmSlot.as<int>(), dAttM2L.as<double>(), dNcx.as<double>(), dNcy.as<double>(),
                     dNrx.as<double>(), dNry.as<double>(), P, hw, dMult.as<double>(), dLocal.as<double>(),
                     dNodeGeo.as<double>()};
    hca.wpe = hmWpe;
    const bool halo = !plan.hmHaloNode.empty();
    if (halo) {  // the halo form: partials of the cross-cluster partner products (Plan::hmHaloPtr)
        const size_t hb = plan.hmHaloNode.size() * kRank * K * sizeof(double);
        if (dHmPart.bytes < hb) dHmPart.alloc(hb);
        hca.haloPtr = dHmHaloPtr.as<int>();
        hca.haloPos = dHmHaloPos.as<int>();
        hca.hpart = dHmPart.as<double>();
    }
    if (hmRing > 0) {
        const int xl = hm_ring_xl(K, plan.hmMaxLds, hmRing);
        hca.ring = xl < 0 ? 0 : hmRing;
        hca.ringXL = xl > 0;
    }
    auto m2lClusters = [&](int c0, int c1, hipStream_t st) {
        HcArgs a = hca;
        if (detSums) {  // fixed-point cluster sums: the bounds of this apply's multipoles first
            detBounds();
            const int nn = (int)tree.ncx.size();
            if (dNodeWmax.bytes < (size_t)nn * sizeof(double)) dNodeWmax.alloc((size_t)nn * sizeof(double));
            launch_node_wmax(K, nn, dMult.as<double>(), hw, dNodeWmax.as<double>(), st);
            a.wmax = dNodeWmax.as<double>();
            a.clBound = dHmClBound.as<double>() + c0;
            a.emax = dAttMax.as<double>();
        }
        a.clPtr += c0;
        if (a.haloPtr) a.haloPtr += c0;
        launch_m2l_hc(K, c1 - c0, plan.hmMaxLds, a, st);
    };
    int e0 = -1;
    int eStart = -1;  // the apply's first event: the total span covers every stage
    bool nearDone = false;
    if (phase != 2) {
        // up pass: tiers bottom-up; its P2M also forms the weighted charges fT (tree
        // order) the near field and the corrections read
        e0 = tm ? mark(s) : -1;
        eStart = e0;
        const bool nearEarlyGroups = nearIn && oneX && !plan.nearGrpEarly.empty() && shardNearEarly;
        const bool earlyAfterPack = nearEarlyGroups && phase == 1 && ntier >= 1 && packHook;
        auto nearEarlyStage = [&] {
            // one-collective form: the groups that read only the own range start now,
            // beside the own tier-0 tasks (or after the pack); the rest waits for the
            // exchange (phase 2)
            nin.grpList = dNearGrpEarly.as<int>();
            nin.ngrp = (int)plan.nearGrpEarly.size();
            if (fork) HIP_CHECK(hipEventRecord(evFork, s));
            nearStage();
            if (!fork && tm) e0 = mark(s);
        };
        if (nearEarlyGroups && !earlyAfterPack) nearEarlyStage();
        // the fork point is the start of the apply, but the near field's launch is issued
        // after the bottom up tier's, so the dispatcher tends to hand the up tasks their
        // workgroup slots first (0.6-1.2 % per block matvec on one GPU, 1.6 % on a rank
        // of 8, r04z; ANISO_NEAR_ORDER=first issues it first)
        const bool nearAfterUp = nearIn && !oneX && fork && nearOrderUp && phase == 0 && ntier >= 1;
        if (nearIn && !oneX) {  // the near field first: beside the up pass (fork) or before it (serial)
            if (fork) HIP_CHECK(hipEventRecord(evFork, s));
            if (!nearAfterUp) {
                nearStage();
                nearDone = true;
            }
            if (!fork && tm) e0 = mark(s);  // serial: the up span starts after the near field
        }
        if (ntier < 1) {  // a lone leaf: no up pass
            launch_prepare(K, geo.N, x, ldx, treeIn ? 1 : 0, dPerm.as<int>(), sigT, dWT.as<double>(),
                           dFT.as<double>(), dCT.as<double>(), s);
            if (fork) HIP_CHECK(hipEventRecord(evFork, s));
        }
        if (phase == 1 && ntier >= 1) {
            if (oneX)
                upTier(0, dXOwnT0Tasks.as<int>(), (int)plan.xOwnT0Tasks.size(), nullptr, upPartial ? nullptr : rootsSend,
                       tail.partOf ? &tail : nullptr);
            else upTier(0, dXT0Tasks.as<int>(), (int)plan.xT0Tasks.size(), nullptr, rootsSend);
            if (earlyAfterPack) {  // the pack's partial tasks take their slots before the near groups do
                packHook(s);
                packIssued = true;
                nearEarlyStage();
            }
        }
        for (int k = nearUp ? 1 : 0; k < (topFused ? 1 : ntier) && phase == 0; ++k) {
            upTier(k, nullptr, tierTasks(k), nullptr, nullptr);
            if (k == 0 && nearAfterUp) {
                nearStage();
                nearDone = true;
            }
        }
        if (phase == 1) {
            const int ep = tm ? mark(s) : -1;
            span(1, e0, ep);
            if ((ntier < 1 || forkTier == 0) && !nearFused && !nearDone && !oneX) {
                nearStage();
                nearDone = true;
            }
            pend.active = true;
            pend.nearDone = nearDone;
            pend.K = K;
            pend.e0 = e0;
            pend.eStart = eStart;
            pend.ePack = ep;
            return;
        }
    } else {
        e0 = pend.e0;
        eStart = pend.eStart;
        nearDone = pend.nearDone;
        pend.active = false;
        const int ex = tm ? mark(s) : -1;
        span(0, pend.ePack, ex);  // the caller's root exchange
        if (oneX && !nearDone) {  // the rest of the near field after the one exchange (it filled the input's halo)
            // (ANISO_SHARD_NEAR_EARLY=0: every group here, in one launch)
            nin.grpList = shardNearEarly ? dNearGrpLate.as<int>() : nullptr;
            nin.ngrp = shardNearEarly ? (int)plan.nearGrpLate.size() : 0;
            if (fork) HIP_CHECK(hipEventRecord(evFork, s));
            nearStage();
            nin.grpList = nullptr;
            nin.ngrp = 0;
            nearDone = true;
        }
        if (upPartial) {  // the exchange's unpack summed the upper multipoles
        } else if (topFused) {  // the upper tiers run inside the M2L launch below
        } else if (ntier >= 2) {  // the first upper tier reads the gathered roots (and stores them for the M2L)
            upTier(1, nullptr, tierTasks(1), rootsRecv, nullptr);
            for (int k = 2; k < ntier; ++k) upTier(k, nullptr, tierTasks(k), nullptr, nullptr);
        } else {
            launch_roots_unpack(K, (int)plan.xRootRecv.size(), dXRootRecv.as<int>(), rootsRecv, dMult.as<double>(),
                                s);
        }
        e0 = ex;  // the up span of phase 2: upper tiers
    }
    int ep = tr ? mark(s) : -1;
    span(1, e0, ep);
    if (phase == 2) e0 = pend.e0;
    if (!nearDone && !nearFused) {
        nearStage();
        if (tr && sn == s) ep = mark(s);  // serial (ANISO_OVERLAP=0): the M2L span starts after the near field
    }
    if (mask & kStageFar) {
        if (topFused) {
            // the launch's LDS holds the largest task of tiers >= 1 only (tier 0 runs apart)
            // (sizing it for the 85-node tier-0 tasks too cost 0.3-0.5 %, r04j)
            const UpArgs ua{plan.upMaxTaskFrom(1), dUpDesc.as<int4>(), dUpGrpFix.as<int>(), dUpNode.as<int>(),
                            dUpCode.as<int4>(), dUpGeom.as<double4>(), dUpLeaf.as<int2>(), dPxT.as<double>(),
                            dPyT.as<double>(), x, ldx, treeIn ? 1 : 0, dPerm.as<int>(), sigT, dWT.as<double>(),
                            fTw, cTw, P, dMult.as<double>(),
                            phase == 2 ? dXRootSlot.as<int>() : nullptr};
            TopArgs ta{};
            const int u1 = plan.upTierTask[1];
            ta.nUp = plan.upTierTask[ntier] - u1;
            ta.ntier = ntier;
            for (int k = 1; k <= ntier; ++k) ta.blk0[k] = plan.upTierTask[k] - u1;
            for (int k = 1; k < ntier; ++k) ta.task0[k] = plan.upTierTask[k];
            ta.clWait = dHmClWait.as<int>();
            ta.cnt = dTopCnt.as<unsigned>();
            ta.recv1 = phase == 2 ? rootsRecv : nullptr;
            ta.spinLimit = topSpinLimit;
            ta.steals = dTopSteals.as<unsigned>();
            HIP_CHECK(hipHostGetDevicePointer((void**)&ta.err, topErr, 0));
            const NearHsArgs na{(int)plan.leaves.size(), plan.nsMax, dLeafInfo.as<int4>(), hmPtsPtr, hmLoc,
                          dNsPtr.as<int64_t>(), dNsPts.as<int>(), hmKOff, dAttNear.as<double>(), dPxT.as<double>(),
                          dPyT.as<double>(), dSigDiag.as<double>(), hw, dFT.as<double>(), operm, obase, ldo, mask,
                          scale, out, nc};

            if (topTraceOn) {
                topTraceNear = nearFused ? (na.nl + 15) / 16 : 0;
                topTraceBlocks = ta.nUp + ncl + topTraceNear;
                if (dTopTrace.bytes < (size_t)topTraceBlocks * 4 * sizeof(int64_t))
                    dTopTrace.alloc((size_t)topTraceBlocks * 4 * sizeof(int64_t));
                ta.trace = dTopTrace.as<int64_t>();
            }
            launch_top_m2l_hc(K, ncl, plan.hmMaxLds, ua, ta, hca, nearFused ? &na : nullptr, s);
        } else if (clustered) {
            m2lClusters(0, ncl, s);
        } else if (harmonic) {
            launch_m2l_hm(K, (int)plan.m2lTgt.size(), dM2LTgt.as<int>(), dAttPtr.as<int64_t>(), dAttSrc.as<int>(),
                          dAttBlk.as<int>(), dAttM2L.as<double>(), dNcx.as<double>(), dNcy.as<double>(),
                          dNrx.as<double>(), dNry.as<double>(), P, hw, dMult.as<double>(), dLocal.as<double>(), s);
        } else {
            launch_m2l(K, (int)plan.m2lTgt.size(), dM2LTgt.as<int>(), dM2LPtr.as<int64_t>(), dM2LNDir.as<int>(),
                       dM2LCanonBase.as<int>(), dM2LOutSlot.as<int>(), dM2LSrc.as<int>(), tab, nterm,
                       dMult.as<double>(), plan.m2lMaxCanon, dM2LPart.as<double>(), dLocal.as<double>(), s);
        }
    }
    int e = tr ? mark(s) : -1;
    span(2, ep, e);
    ep = e;
    if (!harmonic && (mask & kStageFar) && plan.m2lCanon > 0) {
        launch_m2l_gather(K, (int)plan.m2lTgt.size(), dM2LTgt.as<int>(), dM2LInPtr.as<int>(), dM2LPart.as<double>(),
                          dLocal.as<double>(), s);
        e = tm ? mark(s) : -1;
        span(3, ep, e);
        ep = e;
    }
    if (fork) HIP_CHECK(hipStreamWaitEvent(s, evJoin, 0));
    // down pass (owned part): L2L + L2P + gathered transposed near products, once
    // for the sum over the terms (both are linear in the locals / partials)
    if (mask & (kStageFar | kStageNear))
        launch_down_tier(K, (int)plan.dnDesc.size() / 3, plan.dnMaxTask, plan.dnMaxLeaves, dDnDesc.as<int4>(),
                         dDnGrpFix.as<int>(), dDnNode.as<int4>(), dLocal.as<double>(), P, dDnLeafSlot.as<int>(),
                         dDnLeafPts.as<int>(), dDnLeafNear.as<int2>(), dDnLeafGeom.as<double4>(), dPxT.as<double>(),
                         dPyT.as<double>(), operm, obase, ldo, dDnNearOff.as<int>(), plan.dnMaxNear,
                         // the near partials: a single-RHS symmetric plan, or the harmonic one's
                         (harmonic ? hsSym : plan.nearPartTotal > 0) ? dNearPart.as<double>() : nullptr,
                         dDnChain.as<int2>(), plan.dnMaxChain, mask, scale, out, subX, subLd,
                         s, halo && clustered ? dHmPart.as<double>() : nullptr, dDnChainFold.as<int>());
    if (tr) {
        const int e2 = tm ? mark(s) : -1;
        span(5, ep, e2);
        span(7, eStart, e2);
        ++applies;
    }
}

int Operator::rootRhs(int nrhs) { return rhs_supported(nrhs) ? nrhs : rhs_padded(nrhs); }

// aniso.m forward / mforward mixes (aniso.m:121-157).  Output block iid takes,
// for every j in [-(nb-1), nb-1], mode m = |iid + j| of input block |j| with
// weight chi_|j| (mforward; 1 for forward).  Per mode m the pairs (iid, b = |j|)
// are j = m - iid and j = -m - iid (one j when m = 0).
std::vector<double> Operator::blockMixes(int nb, double g, bool chi) {
    if (nb < 1) throw std::invalid_argument("block count must be >= 1");
    const int nm = 2 * nb - 1;
    std::vector<double> mix((size_t)nm * nb * nb, 0.0);
    const double gN = std::pow(g, nb);
    for (int iid = 0; iid < nb; ++iid)
        for (int j = -(nb - 1); j <= nb - 1; ++j) {
            const int b = std::abs(j), m = std::abs(iid + j);
            const double w = chi ? (std::pow(g, b) - gN) / (1.0 - gN) : 1.0;
            mix[((size_t)m * nb + iid) * nb + b] += w;
        }
    return mix;
}

void Operator::blockOpDev(int which, const double* x, int64_t ldx, double* out, int64_t ldo, bool treeIo,
                          hipStream_t s, double gval, const double* sigT, int phase, double* rootsSend,
                          const double* rootsRecv) {
    if (which < 0 || which > 2) throw std::invalid_argument("block operator: which must be 0, 1 or 2");
    if (!coeffSet) throw std::runtime_error("block operator before setCoeff");
    ensureDevice();
    const int nb = ks, nm = 2 * ks - 1;
    const auto mix = blockMixes(nb, std::isnan(gval) ? g : gval, which != 0);
    const double* sig = sigT ? sigT : dSigmaT.as<double>();
    pendingCall(phase, PendingCall{1, which, x, out, sig, ldx, ldo, std::isnan(gval) ? g : gval});
    std::vector<int> ids(nm);
    for (int m = 0; m < nm; ++m) ids[m] = m;
    if (which < 2) {
        applyBlock(nb, x, ldx, treeIo, which != 0 ? sig : nullptr, nm, ids.data(), mix.data(), out, ldo, treeIo, s,
                   kStageAll, phase, rootsSend, rootsRecv);
        return;
    }
    // x - mforward(x) on the owned targets (aniso.m:155)
    const int64_t nOut = treeIo ? plan.ownEnd - plan.ownBegin : geo.N;
    if (!treeIo && plan.nranks != 1) throw std::logic_error("block matvec in original order on a sharded handle: use tree order");
    const double* xo = x + (treeIo ? plan.ownBegin : 0);  // x at the output positions
    if (fuseSub && rhs_supported(nb) && !plan.dnDesc.empty()) {
        // the down pass, last writer of every owned point, stores x - (near + corr + far)
        subX = xo;
        subLd = ldx;
        try {
            applyBlock(nb, x, ldx, treeIo, sig, nm, ids.data(), mix.data(), out, ldo, treeIo, s, kStageAll, phase,
                       rootsSend, rootsRecv);
        } catch (...) {
            subX = nullptr;
            throw;
        }
        subX = nullptr;
        return;
    }
    if (phase != 2) dBlk.alloc((size_t)nb * nOut * sizeof(double));
    applyBlock(nb, x, ldx, treeIo, sig, nm, ids.data(), mix.data(), dBlk.as<double>(), nOut, treeIo, s, kStageAll,
               phase, rootsSend, rootsRecv);
    if (phase != 1) launch_sub_slice(nOut, nb, xo, ldx, dBlk.as<double>(), nOut, out, ldo, s);
}

void Operator::blockOpHost(int which, const double* u, const double* sigmaS, double gval, double* out) {
    if (plan.nranks != 1) throw std::logic_error("host block operator on a sharded handle");
    if (!coeffSet) throw std::runtime_error("block operator before setCoeff");
    ensureDevice();
    const int64_t N = geo.N;
    const size_t bytes = (size_t)ks * N * sizeof(double);
    dHostIn.alloc(bytes);
    dHostOut.alloc(bytes);
    HIP_CHECK(hipMemcpyAsync(dHostIn.p, u, bytes, hipMemcpyHostToDevice, own));
    const double* sigT = nullptr;
    if (sigmaS) {
        std::vector<double> sT(N);
        for (int64_t k = 0; k < N; ++k) sT[k] = sigmaS[tree.perm[k]];
        HIP_CHECK(hipStreamSynchronize(own));  // a previous call may still read dSigAlt
        dSigAlt.upload(sT.data(), N * sizeof(double));
        sigT = dSigAlt.as<double>();
    }
    blockOpDev(which, dHostIn.as<double>(), N, dHostOut.as<double>(), N, false, own, gval, sigT);
    HIP_CHECK(hipMemcpyAsync(out, dHostOut.p, bytes, hipMemcpyDeviceToHost, own));
    HIP_CHECK(hipStreamSynchronize(own));
    if (recoverTopTimeout(own)) {  // the fused launch timed out: the same apply on the tier launches
        struct Restore {
            bool& f;
            ~Restore() { f = false; }
        } restore{forceUnfused};
        blockOpDev(which, dHostIn.as<double>(), N, dHostOut.as<double>(), N, false, own, gval, sigT);
        HIP_CHECK(hipMemcpyAsync(out, dHostOut.p, bytes, hipMemcpyDeviceToHost, own));
        HIP_CHECK(hipStreamSynchronize(own));
    }
    checkDeviceErrors();
}

void Operator::setTiming(int level) {
    if (level < 0 || level > 2) throw std::invalid_argument("timing level must be 0, 1 or 2");
    timeStages = level;
    if (level) {
        evUsed = 0;
        spans.clear();
        applies = 0;
        ensureDevice();
        while (evPool.size() < 512) {  // events for ~50 applies created here, not inside a timed region
            hipEvent_t e;
            HIP_CHECK(hipEventCreate(&e));
            evPool.push_back(e);
        }
    }
}

std::vector<int64_t> Operator::topTrace() {
    sync();
    std::vector<int64_t> out;
    if (!topTraceOn || topTraceBlocks == 0) return out;
    std::vector<int64_t> raw((size_t)topTraceBlocks * 4);
    HIP_CHECK(hipMemcpy(raw.data(), dTopTrace.p, raw.size() * sizeof(int64_t), hipMemcpyDeviceToHost));
    const int ntier = (int)plan.upTierTask.size() - 1;
    const int u1 = plan.upTierTask[1], nUp = plan.upTierTask[ntier] - u1;
    out.reserve((size_t)topTraceBlocks * 8);
    for (int b = 0; b < topTraceBlocks; ++b) {
        out.insert(out.end(), raw.begin() + 4 * b, raw.begin() + 4 * b + 4);
        if (b < nUp) {
            int k = 1;
            while (k + 1 < ntier && b >= plan.upTierTask[k + 1] - u1) ++k;
            out.insert(out.end(), {(int64_t)-k, (int64_t)(k - 1), 0, 0});
        } else if (b >= topTraceBlocks - topTraceNear) {  // a near-field group (16 leaves)
            out.insert(out.end(), {(int64_t)-99, 0, 16, 0});
        } else {
            const int c = b - nUp, t0 = plan.hmClPtr[c], t1 = plan.hmClPtr[c + 1];
            out.insert(out.end(), {(int64_t)c, (int64_t)plan.hmClWait[c], (int64_t)(t1 - t0),
                                   (int64_t)(plan.hmPtr[t1] - plan.hmPtr[t0])});
        }
    }
    return out;
}

StageTimes Operator::stageTimes() {
    StageTimes r;
    if (applies == 0 || spans.empty()) return r;
    HIP_CHECK(hipEventSynchronize(evPool[spans.back().b]));
    double acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (const Span& sp : spans) {
        float t = 0;
        HIP_CHECK(hipEventElapsedTime(&t, evPool[sp.a], evPool[sp.b]));
        acc[sp.stage] += t;
    }
    for (double& a : acc) a /= applies;
    r.exch = (float)acc[0];
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

// ---------------------------------------------------------------- fp32 operator
// (f32op.hip).  The plan is the unsharded tree's: every non-empty
// leaf with its directed U then W sources (bbfmm.h:1081-1099), M2M levels bottom-up
// (bbfmm.h:855-859), every non-empty node's V then X pairs (bbfmm.h:1051-1065), L2L
// levels top-down (bbfmm.h:1070-1071).  The caches are the fp64 mode-0 operators
// (k_cache_m2l / k_cache_near on these directed lists) rounded to fp32.
void Operator::buildMrhsPlan() {
    if (plan.nranks != 1) throw std::logic_error("16-right-hand-side operator on a sharded handle");
    if (mrhsPlanReady) return;
    ensureDevice();
    F32Plan& f = f32;
    f = F32Plan();
    const Tree& t = tree;
    std::vector<int> lv;
    for (int i = 0; i < t.nn; ++i)
        if (t.isLeaf[i] && !t.isEmpty[i]) lv.push_back(i);
    std::sort(lv.begin(), lv.end(), [&](int a, int b) { return t.begin[a] < t.begin[b]; });
    f.nearPtr.push_back(0);
    f.srcPtr.push_back(0);
    for (int n : lv) {
        int64_t S = 0;
        const int64_t s0 = (int64_t)f.srcNodes.size();
        for (int64_t k = t.uPtr[n]; k < t.uPtr[n + 1]; ++k)
            if (!t.isEmpty[t.uIdx[k]]) f.srcNodes.push_back(t.uIdx[k]);
        for (int64_t k = t.wPtr[n]; k < t.wPtr[n + 1]; ++k)
            if (!t.isEmpty[t.wIdx[k]]) f.srcNodes.push_back(t.wIdx[k]);
        for (size_t k = s0; k < f.srcNodes.size(); ++k) {
            const int b = f.srcNodes[k];
            for (int64_t q = 0; q < t.count[b]; ++q) f.nearPts.push_back((int)(t.begin[b] + q));
            S += t.count[b];
        }
        f.maxSrc = std::max<int>(f.maxSrc, (int)(f.srcNodes.size() - s0));
        const int64_t Sp = (S + 15) & ~(int64_t)15;
        for (int64_t q = S; q < Sp; ++q) f.nearPts.push_back((int)t.begin[n]);  // zero columns
        const int nT = (int)t.count[n];
        f.leaves.push_back(n);
        f.leafInfo.push_back({n, (int)t.begin[n], nT, (int)Sp});
        f.srcCount.push_back((int)S);
        f.koff.push_back(f.nearTiles);
        f.koffD.push_back(f.nearD);
        f.nearTiles += (int64_t)((nT + 15) / 16) * (Sp / 16) * 64;
        f.nearD += S * ((nT + 3) & ~3);
        f.nearPtr.push_back((int64_t)f.nearPts.size());
        f.srcPtr.push_back((int64_t)f.srcNodes.size());
    }
    const int D = t.maxLevel;
    f.m2m.assign(std::max(D, 1), {});
    f.l2l.assign(D + 1, {});
    for (int i = 0; i < t.nn; ++i) {
        if (t.isEmpty[i] || t.parent[i] < 0) continue;
        if (!t.isLeaf[i]) f.m2m[t.level[i]].push_back(i);
        if (t.level[i] >= 2) f.l2l[t.level[i]].push_back(i);
        f.m2lTgt.push_back(i);
    }
    f.m2lPtr.push_back(0);
    for (int n : f.m2lTgt) {
        for (int64_t k = t.vPtr[n]; k < t.vPtr[n + 1]; ++k)
            if (!t.isEmpty[t.vIdx[k]]) f.m2lSrc.push_back(t.vIdx[k]);
        for (int64_t k = t.xPtr[n]; k < t.xPtr[n + 1]; ++k)
            if (!t.isEmpty[t.xIdx[k]]) f.m2lSrc.push_back(t.xIdx[k]);
        f.m2lPtr.push_back((int64_t)f.m2lSrc.size());
        for (int64_t p = f.m2lPtr[f.m2lPtr.size() - 2]; p < f.m2lPtr.back(); ++p) f.m2lPairTgt.push_back(n);
    }
    // device lists
    up(d32Leaves, f.leaves);
    std::vector<int4> li(f.leafInfo.size());
    for (size_t i = 0; i < li.size(); ++i)
        li[i] = make_int4(f.leafInfo[i][0], f.leafInfo[i][1], f.leafInfo[i][2], f.leafInfo[i][3]);
    up(d32LeafInfo, li);
    up(d32NearPtr, f.nearPtr);
    up(d32NearPts, f.nearPts);
    up(d32Koff, f.koff);
    up(d32Tgt, f.m2lTgt);
    up(d32Ptr, f.m2lPtr);
    up(d32Src, f.m2lSrc);
    up(d32Level, t.level);
    up(d32PairTgt, f.m2lPairTgt);
    up(d32SrcPtr, f.srcPtr);
    up(d32SrcNodes, f.srcNodes);
    up(d32KoffD, f.koffD);
    up(d32SrcCount, f.srcCount);
    d32LevelNodes.clear();
    d32LevelNodes.resize(f.m2m.size() + f.l2l.size());
    for (size_t l = 0; l < f.m2m.size(); ++l) up(d32LevelNodes[l], f.m2m[l]);
    for (size_t l = 0; l < f.l2l.size(); ++l) up(d32LevelNodes[f.m2m.size() + l], f.l2l[l]);
    // transfer operators in A order: Rup = R_q^T (M2M), Rdn = R_q (L2L); fp32 lane l,
    // element e: k = 4 (l >> 4) + e; fp64: k = (l >> 4) + 4 e (each MFMA's own order)
    std::vector<float> rup(4 * 256), rdn(4 * 256);
    std::vector<double> rup64(4 * 256), rdn64(4 * 256);
    for (int q = 0; q < 4; ++q)
        for (int l = 0; l < 64; ++l)
            for (int e = 0; e < 4; ++e) {
                const int i = l & 15, k = 4 * (l >> 4) + e, k64 = (l >> 4) + 4 * e;
                rup[q * 256 + l * 4 + e] = (float)hostP.R[q][k + i * 16];
                rdn[q * 256 + l * 4 + e] = (float)hostP.R[q][i + k * 16];
                rup64[q * 256 + l * 4 + e] = hostP.R[q][k64 + i * 16];
                rdn64[q * 256 + l * 4 + e] = hostP.R[q][i + k64 * 16];
            }
    up(d32Rup, rup);
    up(d32Rdn, rdn);
    up(d64Rup, rup64);
    up(d64Rdn, rdn64);
    mrhsPlanReady = true;
}

// config 5's fp32 caches: the fp64 mode-0 blocks on the directed lists, rounded
void Operator::buildF32() {
    if (!modeCached(0)) throw std::runtime_error("fp32 operator before cache(0)");
    buildMrhsPlan();
    const F32Plan& f = f32;
    const Tree& t = tree;
    d32Mult.alloc((size_t)t.nn * 256 * sizeof(float));
    d32Local.alloc((size_t)t.nn * 256 * sizeof(float));
    d32FT.alloc((size_t)geo.N * 16 * sizeof(float));
    d32CT.alloc((size_t)geo.N * 16 * sizeof(float));
    const Params* P = dParams.as<Params>();
    {
        const int64_t np_ = (int64_t)f.m2lSrc.size();
        DevBuf tmp;
        tmp.alloc((size_t)std::max<int64_t>(np_, 1) * 256 * sizeof(double));
        d32Km2l.alloc((size_t)std::max<int64_t>(np_, 1) * 256 * sizeof(float));
        launch_cache_m2l(np_, d32PairTgt.as<int>(), d32Src.as<int>(), dNcx.as<double>(), dNcy.as<double>(),
                         dNrx.as<double>(), dNry.as<double>(), dStCoef.as<double>(), P, 0, tmp.as<double>(), own);
        launch32_conv_m2l(np_, tmp.as<double>(), d32Km2l.p, own);
        HIP_CHECK(hipStreamSynchronize(own));
    }
    {
        DevBuf tmp;
        tmp.alloc((size_t)std::max<int64_t>(f.nearD, 1) * sizeof(double));
        d32Knear.alloc((size_t)std::max<int64_t>(f.nearTiles, 1) * 4 * sizeof(float));
        launch_cache_near((int)f.leaves.size(), d32Leaves.as<int>(), d32SrcPtr.as<int64_t>(), d32SrcNodes.as<int>(),
                          d32KoffD.as<int64_t>(), dBegin.as<int64_t>(), dCount.as<int64_t>(), dPxT.as<double>(),
                          dPyT.as<double>(), dStCoef.as<double>(), P, 0, f.maxSrc, tmp.as<double>(), own);
        launch32_conv_near((int)f.leaves.size(), d32LeafInfo.as<int4>(), d32KoffD.as<int64_t>(),
                           d32Koff.as<int64_t>(), d32SrcCount.as<int>(), tmp.as<double>(), d32Knear.p, own);
        HIP_CHECK(hipStreamSynchronize(own));
    }
    f32Ready = true;
}

// the fp64 16-RHS caches of mode id (f64op.hip): the mode's blocks on the directed
// lists, the M2L blocks rearranged in place into A order, the near blocks as tiles
// Built into a local cache, entered into m64 only once every allocation and kernel
// has succeeded: a failed build (out of HBM, a fault) leaves no half-built entry for
// the next call to launch on (ANISO_FAULT_INJECT=mrhs64 makes it throw after its
// allocations, for the test of that path).
size_t Operator::mrhs64Bytes() {
    buildMrhsPlan();
    const F32Plan& f = f32;
    size_t b = (size_t)std::max<int64_t>((int64_t)f.m2lSrc.size(), 1) * 256 * sizeof(double);
    b += (size_t)std::max<int64_t>(f.nearTiles, 1) * 4 * sizeof(double);
    b += (size_t)std::max<int64_t>(f.nearD, 1) * sizeof(double);  // the build's temporary
    if (!d64Mult.p) b += 2 * (size_t)tree.nn * 256 * sizeof(double) + 2 * (size_t)geo.N * 16 * sizeof(double);
    return b;
}

void Operator::buildMrhs64(int id) {
    buildMrhsPlan();
    const F32Plan& f = f32;
    const Params* P = dParams.as<Params>();
    d64Mult.alloc((size_t)tree.nn * 256 * sizeof(double));
    d64Local.alloc((size_t)tree.nn * 256 * sizeof(double));
    d64FT.alloc((size_t)geo.N * 16 * sizeof(double));
    d64CT.alloc((size_t)geo.N * 16 * sizeof(double));
    Mrhs64Cache c;
    const int64_t np_ = (int64_t)f.m2lSrc.size();
    c.Km2l.alloc((size_t)std::max<int64_t>(np_, 1) * 256 * sizeof(double));
    launch_cache_m2l(np_, d32PairTgt.as<int>(), d32Src.as<int>(), dNcx.as<double>(), dNcy.as<double>(),
                     dNrx.as<double>(), dNry.as<double>(), dStCoef.as<double>(), P, id, c.Km2l.as<double>(), own);
    launch64_lane_major(np_, c.Km2l.as<double>(), own);
    {
        DevBuf tmp;
        tmp.alloc((size_t)std::max<int64_t>(f.nearD, 1) * sizeof(double));
        c.Knear.alloc((size_t)std::max<int64_t>(f.nearTiles, 1) * 4 * sizeof(double));
        launch_cache_near((int)f.leaves.size(), d32Leaves.as<int>(), d32SrcPtr.as<int64_t>(), d32SrcNodes.as<int>(),
                          d32KoffD.as<int64_t>(), dBegin.as<int64_t>(), dCount.as<int64_t>(), dPxT.as<double>(),
                          dPyT.as<double>(), dStCoef.as<double>(), P, id, f.maxSrc, tmp.as<double>(), own);
        launch64_conv_near((int)f.leaves.size(), d32LeafInfo.as<int4>(), d32KoffD.as<int64_t>(),
                           d32Koff.as<int64_t>(), d32SrcCount.as<int>(), tmp.as<double>(), c.Knear.p, own);
        HIP_CHECK(hipStreamSynchronize(own));
    }
    if (const char* e = std::getenv("ANISO_FAULT_INJECT"))
        if (std::string(e) == "mrhs64") throw std::runtime_error("fp64 16-RHS cache build failed (ANISO_FAULT_INJECT)");
    m64.emplace(id, std::move(c));
}

void Operator::mrhs64Dev(int id, bool forward, const double* X, double* Y, hipStream_t s, int mask) {
    if (plan.nranks != 1) throw std::logic_error("16-right-hand-side operator on a sharded handle");
    if (id < 0 || id >= kernelSize) throw std::out_of_range("kernel id out of range");
    if (forward && id != 0) throw std::invalid_argument("the forward operator is mode 0's (main.cpp:125-136)");
    if (!modes[id].ready)
        throw std::runtime_error("16-RHS fp64 operator on kernel id " + std::to_string(id) + " before cache(" +
                                 std::to_string(id) + ")");
    ensureDevice();
    checkDeviceErrors();
    if (!m64.count(id)) buildMrhs64(id);
    const Mrhs64Cache& c = m64.at(id);
    const Params* P = dParams.as<Params>();
    const F32Plan& f = f32;
    const double scale = M_1_PI / 2.0;  // AnisoWrapper.cpp:129-130
    const bool tm = timeStages;
    const int e0 = tm ? mark(s) : -1;
    launch64_p2m((int)f.leaves.size(), d32Leaves.as<int>(), dBegin.as<int64_t>(), dCount.as<int64_t>(),
                 dNcx.as<double>(), dNcy.as<double>(), dNrx.as<double>(), dNry.as<double>(), dPxT.as<double>(),
                 dPyT.as<double>(), X, forward ? dSigmaT.as<double>() : nullptr, dWT.as<double>(), P, d64Mult.p,
                 d64FT.as<double>(), d64CT.as<double>(), s);
    for (int l = (int)f.m2m.size() - 1; l >= 1; --l)
        launch64_m2m((int)f.m2m[l].size(), d32LevelNodes[l].as<int>(), dChild.as<int4>(), dCount.as<int64_t>(),
                     d64Rup.p, d64Mult.p, s);
    const int e1 = tm ? mark(s) : -1;
    if (tm) spans.push_back({1, e0, e1});
    if (mask & kStageFar) {
        launch64_m2l((int)f.m2lTgt.size(), d32Tgt.as<int>(), d32Ptr.as<int64_t>(), d32Src.as<int>(), c.Km2l.p,
                     d64Mult.p, d64Local.p, s);
        const int e2 = tm ? mark(s) : -1;
        if (tm) spans.push_back({2, e1, e2});
        for (size_t l = 2; l < f.l2l.size(); ++l)
            launch64_l2l((int)f.l2l[l].size(), d32LevelNodes[f.m2m.size() + l].as<int>(), dParent.as<int>(),
                         dSlot.as<int>(), d64Rdn.p, d64Local.p, s);
    }
    const int e3 = tm ? mark(s) : -1;
    launch64_leaf((int)f.leaves.size(), d32LeafInfo.as<int4>(), d32NearPtr.as<int64_t>(), d32NearPts.as<int>(),
                  d32Koff.as<int64_t>(), c.Knear.p, d32Level.as<int>(), dNcx.as<double>(), dNcy.as<double>(),
                  dNrx.as<double>(), dNry.as<double>(), dPxT.as<double>(), dPyT.as<double>(), P, d64Local.p,
                  d64FT.as<double>(), X, scale, (mask & kStageAll) | (forward ? kStageForward : 0), Y, s);
    const int e4 = tm ? mark(s) : -1;
    if (tm) spans.push_back({4, e3, e4});
    // corrections: Y -= scale' corr with scale' = scale (forward: X - K x) or -scale (mapping: K x)
    launch64_corr(geo.d, geo.N, dPerm.as<int>(), dIperm.as<int>(), d64CT.as<double>(), d64FT.as<double>(),
                  modes[id].C.as<double>(), modes[id].mu.as<double>(), P, mask, forward ? scale : -scale, Y, s);
    if (tm) {
        const int e5 = mark(s);
        spans.push_back({6, e4, e5});
        spans.push_back({7, e0, e5});
        ++applies;
    }
}

void Operator::forwardF32Dev(const float* X, float* Y, hipStream_t s, int mask) {
    if (plan.nranks != 1) throw std::logic_error("fp32 operator on a sharded handle");
    if (!f32Ready) buildF32();
    ensureDevice();
    const Params* P = dParams.as<Params>();
    const F32Plan& f = f32;
    const float scale = (float)(M_1_PI / 2.0);  // AnisoWrapper.cpp:129-130
    const bool tm = timeStages;
    const int e0 = tm ? mark(s) : -1;
    launch32_p2m((int)f.leaves.size(), d32Leaves.as<int>(), dBegin.as<int64_t>(), dCount.as<int64_t>(),
                 dNcx.as<double>(), dNcy.as<double>(), dNrx.as<double>(), dNry.as<double>(), dPxT.as<double>(),
                 dPyT.as<double>(), X, dSigmaT.as<double>(), dWT.as<double>(), P, d32Mult.p, d32FT.as<float>(),
                 d32CT.as<float>(), s);
    for (int l = (int)f.m2m.size() - 1; l >= 1; --l)
        launch32_m2m((int)f.m2m[l].size(), d32LevelNodes[l].as<int>(), dChild.as<int4>(), dCount.as<int64_t>(),
                     d32Rup.p, d32Mult.p, s);
    const int e1 = tm ? mark(s) : -1;
    if (tm) spans.push_back({1, e0, e1});
    if (mask & kStageFar) {
        launch32_m2l((int)f.m2lTgt.size(), d32Tgt.as<int>(), d32Ptr.as<int64_t>(), d32Src.as<int>(), d32Km2l.p,
                     d32Mult.p, d32Local.p, s);
        const int e2 = tm ? mark(s) : -1;
        if (tm) spans.push_back({2, e1, e2});
        for (size_t l = 2; l < f.l2l.size(); ++l)
            launch32_l2l((int)f.l2l[l].size(), d32LevelNodes[f.m2m.size() + l].as<int>(), dParent.as<int>(),
                         dSlot.as<int>(), d32Rdn.p, d32Local.p, s);
    }
    const int e3 = tm ? mark(s) : -1;
    launch32_leaf((int)f.leaves.size(), d32LeafInfo.as<int4>(), d32NearPtr.as<int64_t>(), d32NearPts.as<int>(),
                  d32Koff.as<int64_t>(), d32Knear.p, d32Level.as<int>(), dNcx.as<double>(), dNcy.as<double>(),
                  dNrx.as<double>(), dNry.as<double>(), dPxT.as<double>(), dPyT.as<double>(), P, d32Local.p,
                  d32FT.as<float>(), X, scale, mask, Y, s);
    const int e4 = tm ? mark(s) : -1;
    if (tm) spans.push_back({4, e3, e4});
    launch32_corr(geo.d, geo.N, dPerm.as<int>(), dIperm.as<int>(), d32CT.as<float>(), d32FT.as<float>(),
                  modes[0].C.as<double>(), modes[0].mu.as<double>(), P, mask, scale, Y, s);
    if (tm) {
        const int e5 = mark(s);
        spans.push_back({6, e4, e5});
        spans.push_back({7, e0, e5});
        ++applies;
    }
}

// Attach a communicator (every rank together) and build the halo exchange: each rank
// receives, from the owner of each position of its halo (plan.xHalo), that position;
// what it sends to peer p is p's halo inside its own range, so every rank's halo
// ranges are exchanged once (one all-gather of the counts, one of the ranges).
void Operator::commInit(std::unique_ptr<Collectives> c) {
    if (!c) throw std::invalid_argument("null communicator");
    if (c->nranks != plan.nranks || c->rank != plan.rank)
        throw std::logic_error("communicator rank / size (" + std::to_string(c->rank) + " of " +
                               std::to_string(c->nranks) + ") differ from the handle's shard (" +
                               std::to_string(plan.rank) + " of " + std::to_string(plan.nranks) + ")");
    ensureDevice();
    if (comm && device >= 0) HIP_CHECK(hipDeviceSynchronize());  // collectives in flight on the old one
    comm.reset();
    const int P = c->nranks, me = c->rank;
    DevBuf a, b;
    // every rank's lists (one all-gather of the counts, one of the padded lists); a
    // loopback communicator (development: one rank's schedule on one GPU) has no
    // peers, so their lists come from their plans built here
    struct PeerLists {
        std::vector<double> halo, oneHalo, needNodes, ok, upRec;
    };
    std::vector<PeerLists> peerLists;
    if (c->loopback()) {
        peerLists.resize(P);
        for (int r = 0; r < P; ++r) {
            Plan q;  // the same plan inputs (Plan::build keeps these), rank r's shard
            if (r != me) {
                q.nearSymmetric = plan.nearSymmetric;
                q.nearSymHs = plan.nearSymHs;
                q.maxCanon = plan.maxCanon;
                q.xUpPartialIn = plan.xUpPartialIn;
                q.build(tree, np, r, P);
                q.buildExchange(tree, geo.sz, geo.d2);
            }
            const Plan& src = r == me ? plan : q;
            peerLists[r].halo.assign(src.xHalo.begin(), src.xHalo.end());
            peerLists[r].oneHalo.assign(src.xOneHalo.begin(), src.xOneHalo.end());
            peerLists[r].needNodes.assign(src.xNeedNodes.begin(), src.xNeedNodes.end());
            peerLists[r].ok = {(r == me ? oneExchangeLocal() : src.xOneOk) ? 1.0 : 0.0, src.xUpPartial ? 1.0 : 0.0,
                               cachesReady() ? 1.0 : 0.0};
            peerLists[r].upRec.assign(src.xUpRecNode.begin(), src.xUpRecNode.end());
        }
    }
    auto gatherList = [&](std::vector<double> PeerLists::*field, const std::vector<double>& mineV,
                          std::vector<std::vector<double>>& allV) {
        allV.assign(P, {});
        if (!peerLists.empty()) {
            for (int r = 0; r < P; ++r) allV[r] = peerLists[r].*field;
            return;
        }
        double n = (double)mineV.size();
        a.alloc(sizeof(double));
        b.alloc((size_t)P * sizeof(double));
        HIP_CHECK(hipMemcpy(a.p, &n, sizeof(double), hipMemcpyHostToDevice));
        c->allgather(a.as<double>(), b.as<double>(), 1, own);
        HIP_CHECK(hipStreamSynchronize(own));
        std::vector<double> cnt(P);
        HIP_CHECK(hipMemcpy(cnt.data(), b.p, (size_t)P * sizeof(double), hipMemcpyDeviceToHost));
        size_t m = 1;
        for (double x : cnt) m = std::max(m, (size_t)x);
        std::vector<double> pad(m, -1.0);
        std::copy(mineV.begin(), mineV.end(), pad.begin());
        a.alloc(m * sizeof(double));
        b.alloc((size_t)P * m * sizeof(double));
        HIP_CHECK(hipMemcpy(a.p, pad.data(), m * sizeof(double), hipMemcpyHostToDevice));
        c->allgather(a.as<double>(), b.as<double>(), m, own);
        HIP_CHECK(hipStreamSynchronize(own));
        std::vector<double> flat((size_t)P * m);
        HIP_CHECK(hipMemcpy(flat.data(), b.p, flat.size() * sizeof(double), hipMemcpyDeviceToHost));
        for (int r = 0; r < P; ++r)
            allV[r].assign(flat.begin() + (size_t)r * m, flat.begin() + (size_t)r * m + (size_t)cnt[r]);
    };
    std::vector<std::vector<double>> haloAll;
    gatherList(&PeerLists::halo, std::vector<double>(plan.xHalo.begin(), plan.xHalo.end()), haloAll);
    const auto cuts = shard_cuts(tree, P);
    if (cuts[me] != plan.ownBegin || cuts[me + 1] != plan.ownEnd) throw std::logic_error("shard cuts disagree with the plan");
    const int nb = ks;
    auto ranges = [&](int r) {  // rank r's halo ranges
        std::vector<std::pair<int64_t, int64_t>> v;
        for (size_t i = 0; i + 1 < haloAll[r].size(); i += 2) v.push_back({(int64_t)haloAll[r][i], (int64_t)haloAll[r][i + 1]});
        return v;
    };
    auto intersect = [](const std::vector<std::pair<int64_t, int64_t>>& rs, int64_t lo, int64_t hi,
                        std::vector<int64_t>& out) {
        for (const auto& r : rs)
            for (int64_t k = std::max(r.first, lo); k < std::min(r.second, hi); ++k) out.push_back(k);
    };
    std::vector<int64_t> spos, sbase, sstr, rpos, rbase, rstr;
    hxScount.assign(P, 0);
    hxSoff.assign(P, 0);
    hxRcount.assign(P, 0);
    hxRoff.assign(P, 0);
    const auto myHalo = ranges(me);
    for (int p = 0; p < P; ++p) {
        hxSoff[p] = (int64_t)spos.size() * nb;
        hxRoff[p] = (int64_t)rpos.size() * nb;
        if (p == me) continue;
        std::vector<int64_t> sp, rp;
        intersect(ranges(p), plan.ownBegin, plan.ownEnd, sp);  // p's halo inside my range
        intersect(myHalo, cuts[p], cuts[p + 1], rp);           // my halo inside p's range
        for (size_t i = 0; i < sp.size(); ++i) {
            spos.push_back(sp[i]);
            sbase.push_back(hxSoff[p] + (int64_t)i);
            sstr.push_back((int64_t)sp.size());
        }
        for (size_t i = 0; i < rp.size(); ++i) {
            rpos.push_back(rp[i]);
            rbase.push_back(hxRoff[p] + (int64_t)i);
            rstr.push_back((int64_t)rp.size());
        }
        hxScount[p] = (int64_t)sp.size() * nb;
        hxRcount[p] = (int64_t)rp.size() * nb;
    }
    hxNsend = (int64_t)spos.size();
    hxNrecv = (int64_t)rpos.size();
    up(dHxSendPos, spos);
    up(dHxSendBase, sbase);
    up(dHxSendStride, sstr);
    up(dHxRecvPos, rpos);
    up(dHxRecvBase, rbase);
    up(dHxRecvStride, rstr);
    dHxSendBuf.alloc((size_t)std::max<int64_t>(hxNsend * nb, 1) * sizeof(double));
    dHxRecvBuf.alloc((size_t)std::max<int64_t>(hxNrecv * nb, 1) * sizeof(double));
    const int64_t rec = (int64_t)plan.xRootChunk * kRank * rootRhs(nb);
    dXRootsSend.alloc((size_t)std::max<int64_t>(rec, 1) * sizeof(double));
    dXRootsRecv.alloc((size_t)std::max<int64_t>(rec * P, 1) * sizeof(double));
    HIP_CHECK(hipMemset(dXRootsSend.p, 0, dXRootsSend.bytes));
    // ---- the one-collective layout: every rank's needed multipoles (node lists, one
    // all-gather of the counts and one of the lists) and its input ranges (as above)
    oxReady = false;
    std::vector<std::vector<double>> oksAll;
    // every rank's shard- and process-dependent part of the decision (its plan, its
    // staged near field, its knobs): the one-collective form only where all of them
    // hold, so that oxReady, and with it the collectives each matvec issues, is the
    // same on every rank (oneExchangeUsable adds only rank-independent checks)
    // (and whether its plan has the upper multipoles as partial sums: only if every
    // rank's has, since the parts then carry records instead of roots)
    // (and whether it has cached every mode: a sharded matvec on a rank without its
    // caches could only fail on that rank while its peers wait inside the exchange, so
    // comm_init fails on EVERY rank instead, after this gather)
    gatherList(&PeerLists::ok, {oneExchangeLocal() ? 1.0 : 0.0, plan.xUpPartial ? 1.0 : 0.0, cachesReady() ? 1.0 : 0.0},
               oksAll);
    bool allOk = true, allUp = true;
    for (int r = 0; r < P; ++r) {
        const auto& o = oksAll[r];
        if (o.size() < 3 || o[2] < 0.5)
            throw std::logic_error("comm_init: rank " + std::to_string(r) +
                                   " has not cached every mode; every rank caches its modes before comm_init");
        allOk = allOk && o[0] > 0.5;
        allUp = allUp && o[1] > 0.5;
    }
    oxUp = false;
    if (allOk) {  // every rank decides alike: all take part in the same collectives
        std::vector<std::vector<double>> oneAll, nodesAll, upAll;
        gatherList(&PeerLists::oneHalo, std::vector<double>(plan.xOneHalo.begin(), plan.xOneHalo.end()), oneAll);
        gatherList(&PeerLists::needNodes, std::vector<double>(plan.xNeedNodes.begin(), plan.xNeedNodes.end()), nodesAll);
        if (allUp)
            gatherList(&PeerLists::upRec, std::vector<double>(plan.xUpRecNode.begin(), plan.xUpRecNode.end()), upAll);
        const int RK = kRank * rootRhs(nb);
        // the partial-sum records: (node, rank, record, source offset), summed per node in
        // (rank, record) order; this rank's own from its record buffer (~offset)
        struct UpSum {
            int node, rank, j;
            int64_t src;
        };
        std::vector<UpSum> sums;
        const int64_t myRec = allUp ? (int64_t)plan.xUpRecNode.size() * RK : 0;
        if (allUp)
            for (size_t j = 0; j < plan.xUpRecNode.size(); ++j)
                sums.push_back({plan.xUpRecNode[j], me, (int)j, ~((int64_t)j * RK)});
        auto ownerOf = [&](int n) {
            return (int)(std::upper_bound(cuts.begin() + 1, cuts.end() - 1, tree.begin[n]) - (cuts.begin() + 1));
        };
        auto pts = [&](int r, int64_t lo, int64_t hi, std::vector<int64_t>& out) {  // rank r's ranges inside [lo, hi)
            for (size_t i = 0; i + 1 < oneAll[r].size(); i += 2)
                for (int64_t k = std::max((int64_t)oneAll[r][i], lo); k < std::min((int64_t)oneAll[r][i + 1], hi); ++k)
                    out.push_back(k);
        };
        auto nodes = [&](int r, int owner, std::vector<int>& out) {  // rank r's needed nodes owned by `owner`
            for (double v : nodesAll[r])
                if (ownerOf((int)v) == owner) out.push_back((int)v);
        };
        std::vector<int64_t> sp_, sb_, ss_, rp_, rb_, rs_, snb, rnb;
        std::vector<int> sn_, rn_;
        oxScount.assign(P, 0);
        oxSoff.assign(P, 0);
        oxRcount.assign(P, 0);
        oxRoff.assign(P, 0);
        // per peer part: the tier-0 root records (rec doubles, every peer gets this
        // rank's), the input positions (block-major), the multipole rows -- one send
        // and one receive per peer
        std::vector<int64_t> rtS, rtR, rtD;
        int64_t so = 0, ro = 0;
        for (int p = 0; p < P; ++p) {
            oxSoff[p] = so;
            oxRoff[p] = ro;
            if (p == me) continue;
            if (allUp) {  // this rank's records to p; p's records from it
                if (myRec > 0) {
                    rtS.push_back(so);
                    so += myRec;
                }
                for (size_t j = 0; j < upAll[p].size(); ++j)
                    sums.push_back({(int)upAll[p][j], p, (int)j, ro + (int64_t)j * RK});
                ro += (int64_t)upAll[p].size() * RK;
            } else if (rec > 0) {
                rtS.push_back(so);
                rtR.push_back(ro);
                rtD.push_back((int64_t)p * rec);
                so += rec;
                ro += rec;
            }
            std::vector<int64_t> sp, rp;
            std::vector<int> sn, rn;
            pts(p, plan.ownBegin, plan.ownEnd, sp);  // p's positions inside my range
            pts(me, cuts[p], cuts[p + 1], rp);       // mine inside p's range
            nodes(p, me, sn);                        // p's nodes in my subtrees
            nodes(me, p, rn);                        // mine in p's
            for (size_t i = 0; i < sp.size(); ++i) {
                sp_.push_back(sp[i]);
                sb_.push_back(so + (int64_t)i);
                ss_.push_back((int64_t)sp.size());
            }
            for (size_t i = 0; i < rp.size(); ++i) {
                rp_.push_back(rp[i]);
                rb_.push_back(ro + (int64_t)i);
                rs_.push_back((int64_t)rp.size());
            }
            const int64_t sn0 = so + (int64_t)sp.size() * nb, rn0 = ro + (int64_t)rp.size() * nb;
            for (size_t j = 0; j < sn.size(); ++j) {
                sn_.push_back(sn[j]);
                snb.push_back(sn0 + (int64_t)j * RK);
            }
            for (size_t j = 0; j < rn.size(); ++j) {
                rn_.push_back(rn[j]);
                rnb.push_back(rn0 + (int64_t)j * RK);
            }
            so += (int64_t)sp.size() * nb + (int64_t)sn.size() * RK;
            ro += (int64_t)rp.size() * nb + (int64_t)rn.size() * RK;
            oxScount[p] = so - oxSoff[p];
            oxRcount[p] = ro - oxRoff[p];
        }
        if (allUp) {
            std::sort(sums.begin(), sums.end(), [](const UpSum& a, const UpSum& b) {
                return a.node != b.node ? a.node < b.node : a.rank != b.rank ? a.rank < b.rank : a.j < b.j;
            });
            std::vector<int> sNode, sPtr(1, 0);
            std::vector<int64_t> sSrc;
            for (size_t i = 0; i < sums.size(); ++i) {
                if (i == 0 || sums[i].node != sums[i - 1].node) {
                    if (i > 0) sPtr.push_back((int)sSrc.size());
                    sNode.push_back(sums[i].node);
                }
                sSrc.push_back(sums[i].src);
            }
            if (!sums.empty()) sPtr.push_back((int)sSrc.size());
            oxUpSums = (int64_t)sNode.size();
            up(dOxUpSumNode, sNode);
            up(dOxUpSumPtr, sPtr);
            up(dOxUpSumSrc, sSrc);
            dXUpRec.alloc((size_t)std::max<int64_t>(myRec, 1) * sizeof(double));
            oxUp = true;
        }
        oxRootParts = (int64_t)rtS.size();
        up(dOxRootSend, rtS);
        up(dOxRootRecv, rtR);
        up(dOxRootDst, rtD);
        oxNsendPts = (int64_t)sp_.size();
        oxNrecvPts = (int64_t)rp_.size();
        oxNsendNodes = (int64_t)sn_.size();
        oxNrecvNodes = (int64_t)rn_.size();
        if (oxNrecvNodes != (int64_t)plan.xNeedNodes.size())
            throw std::logic_error("one-collective exchange: a needed multipole has no owner");
        up(dOxSendPos, sp_);
        up(dOxSendBase, sb_);
        up(dOxSendStride, ss_);
        up(dOxRecvPos, rp_);
        up(dOxRecvBase, rb_);
        up(dOxRecvStride, rs_);
        up(dOxSendNode, sn_);
        up(dOxSendNodeBase, snb);
        up(dOxRecvNode, rn_);
        up(dOxRecvNodeBase, rnb);
        dOxSendBuf.alloc((size_t)std::max<int64_t>(so, 1) * sizeof(double));
        dOxRecvBuf.alloc((size_t)std::max<int64_t>(ro, 1) * sizeof(double));
        oxReady = true;
    }
    comm = std::move(c);
}

// Can this sharded matvec take the one-collective exchange?  Its phase 1 must leave
// nothing to the halo: the harmonic block apply with the near field formed from the
// input (run in phase 2, after the exchange) and no padded right-hand sides -- exactly
// applyBlock's `harmonic && nearIn` for this call.  The decision must be the same on
// every rank (the ranks issue matching collectives), so it is split: the part that
// depends on a rank's shard or process (oneExchangeLocal) is all-gathered at commInit
// into oxReady; what is left here depends only on the problem (ks, g, which) and on
// the mode caches, which every rank builds alike before a block matvec.
bool Operator::oneExchangeLocal() const {
    if (!plan.xOneOk || !oneXOn || !useAtt || !rhs_supported(ks) || !nearEarly || nearInTop || !plan.nearCorrOk ||
        plan.nearPartTotal > 0)
        return false;
    const NearCorr probe{dNearCorrRow.as<uint16_t>(), nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
    return near_hs_fusable((int)plan.leaves.size(), plan.nearMaxLeaf, plan.nsMax, dNearLoc.as<uint16_t>(), &probe,
                           kStageAll);
}

// every mode cached (and the mode-shared caches built, where the handle uses them):
// what a sharded block matvec needs on every rank
bool Operator::cachesReady() const {
    for (int m = 0; m < kernelSize; ++m)
        if (!modes[m].ready) return false;
    return !useAtt || attReady;
}

bool Operator::oneExchangeUsable(int which) {
    if (!oxReady) return false;
    if (!attReady)  // mode caches differ between ranks would split the decision: refuse before any collective
        throw std::logic_error("sharded block operator before cache(): every rank caches its modes first");
    const int nm = 2 * ks - 1;
    const auto mix = blockMixes(ks, g, which != 0);
    std::vector<int> ids(nm);
    for (int m = 0; m < nm; ++m) ids[m] = m;
    HarmWeights hw;
    return harmonicWeights(ks, nm, ids.data(), mix.data(), hw);
}

void Operator::blockOpShardedDev(int which, double* x, int64_t ldx, double* y, int64_t ldy, hipStream_t s) {
    if (!comm) throw std::logic_error("sharded block operator before aniso_comm_init");
    if (ldx < geo.N || ldy < geo.N) throw std::invalid_argument("sharded block operator: leading dimension below N");
    ensureDevice();
    const int nb = ks;
    double* yo = y + plan.ownBegin;
    const int64_t rec = (int64_t)plan.xRootChunk * kRank * rootRhs(nb);
    if (oneExchangeUsable(which)) {
        // phase 1 (own tier-0 subtrees), then ONE grouped exchange: the roots to every
        // rank, and from each owner the input positions and multipoles this rank reads;
        // then phase 2 (near field, upper tiers + M2L, down pass)
        oneXActive = true;
        upActive = oxUp;
        upTailActive = oxUp && upTailsOn && !plan.xUpRoots.empty();
        packIssued = false;
        if (oxUp && oxRootParts > 63) throw std::logic_error("partial-sum records: more than 63 peer parts");
        try {
            const int RK = kRank * rootRhs(nb);
            // one pack launch (this rank's roots -- or its partial-sum records -- into
            // every peer's part, the input positions and the multipole rows each peer
            // reads), one all-to-all-v, one unpack launch (the peers' roots into the slot
            // layout and the own roots -- or every upper node's records summed -- the
            // input's halo, the multipoles)
            // (built when the pack is enqueued: phase 1 may size the work buffers, dMult)
            OxArgs pk;
            auto packArgs = [&] {
                pk.nRoot = oxRootParts;
                pk.rec = oxUp ? (int64_t)plan.xUpRecNode.size() * RK : rec;
                pk.rootOff = dOxRootSend.as<int64_t>();
                pk.roots = oxUp ? dXUpRec.as<double>() : dXRootsSend.as<double>();
                pk.nPts = oxNsendPts;
                pk.nb = nb;
                pk.pos = dOxSendPos.as<int64_t>();
                pk.base = dOxSendBase.as<int64_t>();
                pk.stride = dOxSendStride.as<int64_t>();
                pk.x = x;
                pk.ldx = ldx;
                pk.nNode = oxNsendNodes;
                pk.len = RK;
                pk.node = dOxSendNode.as<int>();
                pk.nodeBase = dOxSendNodeBase.as<int64_t>();
                pk.mult = dMult.as<double>();
                pk.buf = dOxSendBuf.as<double>();
            };
            auto pack = [&](hipStream_t st) {
                packArgs();
                if (oxUp) {  // the pack launch forms this rank's records (its first workgroups) unless the
                             // bottom tier's tails already did
                    OxArgs pr = pk;
                    pr.nRoot = 0;
                    launch_ox_pack_up(rootRhs(nb), upTailActive ? 0 : (int)(plan.xUpTask.size() / Plan::kUpTaskInts),
                                      dXUpTask.as<int>(), dMult.as<double>(), dParams.as<Params>(),
                                      dXUpRec.as<double>(), (int)oxRootParts, dOxRootSend.as<int64_t>(), pr, st);
                } else {
                    launch_ox(pk, true, st);
                }
            };
            if (nearAfterPack) packHook = pack;
            blockOpDev(which, x, ldx, yo, ldy, true, s, NAN, nullptr, 1, dXRootsSend.as<double>(), nullptr);
            packHook = nullptr;
            if (!packIssued) pack(s);
            comm->alltoallv(dOxSendBuf.as<double>(), oxScount.data(), oxSoff.data(), dOxRecvBuf.as<double>(),
                            oxRcount.data(), oxRoff.data(), s);
            OxArgs uk = pk;
            uk.rootOff = dOxRootRecv.as<int64_t>();
            uk.rootDst = dOxRootDst.as<int64_t>();
            uk.roots = dXRootsRecv.as<double>();
            uk.ownRoots = rec > 0 ? dXRootsSend.as<double>() : nullptr;
            uk.ownDst = (int64_t)plan.rank * rec;
            uk.nPts = oxNrecvPts;
            uk.pos = dOxRecvPos.as<int64_t>();
            uk.base = dOxRecvBase.as<int64_t>();
            uk.stride = dOxRecvStride.as<int64_t>();
            uk.nNode = oxNrecvNodes;
            uk.node = dOxRecvNode.as<int>();
            uk.nodeBase = dOxRecvNodeBase.as<int64_t>();
            uk.buf = dOxRecvBuf.as<double>();
            if (oxUp) {
                uk.nRoot = 0;
                uk.ownRoots = nullptr;
                uk.nSum = oxUpSums;
                uk.sumNode = dOxUpSumNode.as<int>();
                uk.sumPtr = dOxUpSumPtr.as<int>();
                uk.sumSrc = dOxUpSumSrc.as<int64_t>();
                uk.ownRec = dXUpRec.as<double>();
            }
            launch_ox(uk, false, s);
            blockOpDev(which, x, ldx, yo, ldy, true, s, NAN, nullptr, 2, nullptr, dXRootsRecv.as<double>());
        } catch (...) {
            oneXActive = false;
            upActive = false;
            upTailActive = false;
            packHook = nullptr;
            throw;
        }
        oneXActive = false;
        upActive = false;
        upTailActive = false;
        ++oneXApplies;
        if (oxUp) ++upPartialApplies;
        return;
    }
    // the input's halo from its owners
    launch_halo_pack(hxNsend, nb, dHxSendPos.as<int64_t>(), dHxSendBase.as<int64_t>(), dHxSendStride.as<int64_t>(),
                     x, ldx, dHxSendBuf.as<double>(), s);
    comm->alltoallv(dHxSendBuf.as<double>(), hxScount.data(), hxSoff.data(), dHxRecvBuf.as<double>(),
                    hxRcount.data(), hxRoff.data(), s);
    launch_halo_unpack(hxNrecv, nb, dHxRecvPos.as<int64_t>(), dHxRecvBase.as<int64_t>(), dHxRecvStride.as<int64_t>(),
                       dHxRecvBuf.as<double>(), x, ldx, s);
    // phase 1, the tier-0 root all-gather, phase 2 (the owned slice of y)
    blockOpDev(which, x, ldx, yo, ldy, true, s, NAN, nullptr, 1, dXRootsSend.as<double>(), nullptr);
    if (rec > 0) comm->allgather(dXRootsSend.as<double>(), dXRootsRecv.as<double>(), (size_t)rec, s);
    blockOpDev(which, x, ldx, yo, ldy, true, s, NAN, nullptr, 2, nullptr, dXRootsRecv.as<double>());
}

void Operator::checkDeviceErrors() {
    if (!topErr || ownTimeline) return;
    if (*(volatile unsigned*)topErr == 0) return;
    *(volatile unsigned*)topErr = 0;
    throw std::runtime_error(
        "hand-off time-out in the fused top-of-tree M2L launch (k_top_m2l_hc): a cluster gave up waiting for the "
        "upper up tiers, so the output of an apply enqueued earlier on this handle is invalid");
}

bool Operator::recoverTopTimeout(hipStream_t s) {
    if (!topErr || *(volatile unsigned*)topErr == 0) return false;
    HIP_CHECK(hipStreamSynchronize(s));  // every launch that could still raise it has finished
    *(volatile unsigned*)topErr = 0;
    forceUnfused = true;
    ++topRecoveries;
    return true;
}

int64_t Operator::topSteals() {
    if (device < 0 || !dTopSteals.p) return 0;
    HIP_CHECK(hipSetDevice(device));
    unsigned v = 0;
    HIP_CHECK(hipMemcpy(&v, dTopSteals.p, sizeof(unsigned), hipMemcpyDeviceToHost));
    return v;
}

void Operator::sync() {
    if (device < 0) return;
    HIP_CHECK(hipSetDevice(device));
    HIP_CHECK(hipDeviceSynchronize());
    checkDeviceErrors();
}

// The two phases of a sharded apply must come from the same public call: an _end
// that does not repeat its _begin (another operation, block-operator kind, vectors,
// strides or coefficients) would run on the other call's weighted charges.
void Operator::pendingCall(int phase, const PendingCall& c) {
    if (phase == 1) {
        pendCall = c;
    } else if (phase == 2) {
        if (!pend.active || !(pendCall == c))
            throw std::logic_error("sharded apply: end does not match the pending begin (operation, which, x, out, "
                                   "strides and coefficients must repeat)");
    }
}

void Operator::permuteToTree(const double* orig, double* treeOut, hipStream_t s) {
    ensureDevice();
    launch_permute(geo.N, dPerm.as<int>(), orig, treeOut, s);
}

}  // namespace aniso
