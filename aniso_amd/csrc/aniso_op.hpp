// aniso_op.hpp -- the MI355X operator behind the C ABI (one per handle).
//
// Host state (geometry, tree, plan) is built by the constructor without touching
// the GPU; device buffers are created on first use (setCoeff), on the HIP device
// that is current at that moment.
#pragma once

#include <hip/hip_runtime.h>

#include <array>
#include <cmath>
#include <map>
#include <functional>
#include <memory>
#include <string>
#include <vector>

#include "comm.hpp"
#include "host.hpp"
#include "kernels.hpp"

namespace aniso {

int64_t arn_state_doubles(int m);  // the Arnoldi state block of restart length m (arnoldi.hpp)

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    DevBuf() = default;
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
    DevBuf(DevBuf&& o) noexcept : p(o.p), bytes(o.bytes) { o.p = nullptr; o.bytes = 0; }
    ~DevBuf();
    void alloc(size_t nbytes);
    void upload(const void* host, size_t nbytes);
    template <class T>
    T* as() const { return static_cast<T*>(p); }
};

struct ModeCache {
    DevBuf Knear, Km2l, C, mu;
    std::vector<double> hostC, hostMu;  // the correction tables (folded per batched apply)
    bool ready = false;
};

// Correction tables of one batched apply: every term's stencil / singular table
// folded with its mix (launch_corr).
struct CorrFold {
    DevBuf Wc, Wm;
};

struct StageTimes {
    float exch = 0, up = 0, m2l = 0, gather = 0, near = 0, down = 0, corr = 0, total = 0;
};

class Operator {
public:
    Operator(int sz, int d, int ks, double g, int ns, int np, int maxLevel);
    ~Operator();

    // --- the reference's MEX ops (AnisoWrapper.cpp:10-136)
    int64_t numNodes() const { return geo.N; }
    void getNodes(double* xy) const;
    void setCoeff(const double* sigma_s, const double* sigma_t);
    void cache(int id);
    void mappingHost(const double* charge, int id, double* out);
    void mappingBatchedHost(const double* Q, int k, int id, double* Out);  // N x k column-major
    void mappingDev(const double* charge, int id, double* out, hipStream_t s, int stageMask = 0x3f);
    void mappingTreeDev(const double* qTree, int id, double* outSlice, hipStream_t s);
    void forwardTreeDev(const double* xTree, double* ySlice, hipStream_t s);
    // sharded applies in two phases around the caller's all-gather of the tier-0
    // root multipoles: begin runs this rank's tier-0 up tasks (input
    // valid at the own range and plan.xHalo only), packs its roots into rootsSend
    // (plan.xRootChunk x 16 x K doubles, K = rootRhs(nrhs)) and starts the near
    // field (it writes the output); end scatters the gathered roots (nranks
    // chunks), runs the upper tiers, the M2L and the down pass.  The same x and out
    // in both calls, tree order.
    void forwardTreePhase(int phase, const double* xTree, double* ySlice, double* rootsSend, const double* rootsRecv,
                          hipStream_t s);
    static int rootRhs(int nrhs);  // right-hand sides per root record of an nrhs apply (padded count)

    // --- block operator (aniso.m:121-157)
    // out[i] = sum_t sum_b mixes[t][i][b] K_{ids[t]}(sig .* x[b]) for i, b < nrhs <= 8:
    // one up pass over the nrhs base vectors, every mode's operators streamed once
    // for all right-hand sides, one down pass.  x: nrhs vectors of all N points
    // (stride ldx; original or tree order); out: original order (owned targets) or
    // the owned tree-order slice (treeOut), stride ldo.  mixes: nterm x nrhs x nrhs.
    void applyBlockDev(int nrhs, const double* x, int64_t ldx, bool treeIn, bool useSigma, int nterm, const int* ids,
                       const double* mixes, double* out, int64_t ldo, bool treeOut, hipStream_t s,
                       int mask = 15);
    // aniso.m on nb = ks blocks of n = N points: which = 0 forward (the right-hand
    // side, aniso.m:121-136), 1 mforward (aniso.m:138-157), 2 x - mforward(x) (the
    // GMRES matvec, aniso.m:155); tree = tree-order input and owned-slice output.
    // gval / sigT (tree-order sigma_s on the device) override the handle's g and
    // sigma_s when given (NaN / nullptr: the handle's).
    void blockOpDev(int which, const double* x, int64_t ldx, double* out, int64_t ldo, bool tree, hipStream_t s,
                    double gval = NAN, const double* sigT = nullptr, int phase = 0, double* rootsSend = nullptr,
                    const double* rootsRecv = nullptr);
    // host-pointer block operator (aniso.m:121-157): u and out hold nb = ks blocks of
    // N points each (block b at b * N, original order); sigmaS (N, or nullptr: the
    // handle's sigma_s) and gval (NaN: the handle's g) as aniso.m's mforward reads them
    void blockOpHost(int which, const double* u, const double* sigmaS, double gval, double* out);
    // the (2 nb - 1) mode mixes of forward (chi = false) or mforward (chi = true)
    static std::vector<double> blockMixes(int nb, double g, bool chi);

    // --- extensions
    void setShard(int rank, int nranks);
    // the library's own multi-GPU exchange (comm.hpp): attach a
    // communicator of this shard's rank / nranks, then blockOpShardedDev runs the
    // input's halo all-to-all, phase 1, the root all-gather and phase 2 in one call
    void commInit(std::unique_ptr<Collectives> c);
    void blockOpShardedDev(int which, double* x, int64_t ldx, double* y, int64_t ldy, hipStream_t s);
    bool commReady() const { return comm != nullptr; }
    void getShard(int64_t* ownBegin, int64_t* ownEnd) const { *ownBegin = plan.ownBegin; *ownEnd = plan.ownEnd; }
    // sharded apply: writes only owned targets of out (original order), others untouched
    void permuteToTree(const double* orig, double* tree, hipStream_t s);
    void lineIntegrals(const double* seg, int n, double* out);
    // callers of the hot path (main.cpp:125-141)
    void forwardDev(const double* u, double* out, hipStream_t s);
    int gmresHost(const double* q, double* x, int m, int maxit, double tol, double* hist, int maxhist,
                  double* finalResid);
    // aniso.m:159-173: gmres(A, rhs, restart, tol, maxit), A = x - mforward(x), on the
    // ks stacked blocks (original order, block b at b * N); device / host pointers
    int blockSolveDev(const double* rhs, double* x, int restart, double tol, int maxit, double* hist, int maxhist,
                      double* relres, hipStream_t s);
    int solve16Mixed(const double* B, int64_t ldb, double* X, int64_t ldx, int m, double tol, double innerTol,
                     int maxOuter, int maxCycles, int* outer, double* rel, hipStream_t s);
    int blockSolveHost(const double* rhs, double* x, int restart, double tol, int maxit, double* hist, int maxhist,
                       double* relres);
    // config 5's fp32 operator (f32op.hip): Y = X - K_0(sigma_s .* X)
    // for 16 right-hand sides, X and Y point-major (N x 16 floats, tree order), every
    // FMM translation a 16 x 16 x 16 MFMA product on fp32 caches (built from the
    // fp64 mode-0 operators at the first call).  Unsharded handles only.
    void forwardF32Dev(const float* X, float* Y, hipStream_t s, int mask = kStageAll);
    // the fp64 16-right-hand-side operator on MFMA (f64op.hip): Y = K_id X
    // (forward = false) or main.cpp's Y = X - K_0(sigma_s .* X) (forward = true, id 0);
    // X, Y point-major N x 16 doubles in tree order.  The mode's fp64 caches (directed
    // lists, A order) are built from its operators at the first call.  Unsharded only.
    void mrhs64Dev(int id, bool forward, const double* X, double* Y, hipStream_t s, int mask = kStageAll);
    // the block solve's CGS2 sweeps as primitives (aniso_krylov_dot / _update)
    void krylovDot(int64_t n, int nv, const double* V, int64_t ldv, const double* w, double* out, hipStream_t s);
    void krylovUpdate(int64_t n, int nv, const double* V, int64_t ldv, const double* c, double* w, double* out,
                      bool dots, hipStream_t s);
    // DCGS2 Arnoldi primitives on a caller's state block (arnoldi.hpp; aniso_arnoldi_*):
    // begin a cycle (V[0] = the residual; rr: its all-reduced |r|^2, or null: this rank's),
    // one step on one rank, or its parts around a caller's all-reduces (project / update
    // write this rank's row sums; coef / column take the reduced ones), and the cycle's
    // update x += P T R^-1 g
    void arnoldiBegin(int64_t n, int m, const double* V, int64_t ldv, double* st, const double* rr, double normb,
                      double* status, hipStream_t s);
    void arnoldiStep(int64_t n, int m, int j, double* V, int64_t ldv, const double* w, double* st, double* status,
                     hipStream_t s);
    void arnoldiProject(int64_t n, int j, const double* V, int64_t ldv, const double* w, double* out, hipStream_t s);
    void arnoldiCoef(int m, int j, double* st, const double* red, hipStream_t s);
    void arnoldiUpdate(int64_t n, int m, int j, double* V, int64_t ldv, const double* w, const double* st, double* out,
                       hipStream_t s);
    void arnoldiColumn(int m, int j, double* st, const double* red, double* status, hipStream_t s);
    void arnoldiSolution(int64_t n, int m, int used, const double* V, int64_t ldv, double* st, double* x,
                         hipStream_t s);
    // directed M2L pairs of the 16-right-hand-side operators (0 before their plan is built)
    int64_t mrhsM2LPairs() const { return mrhsPlanReady ? (int64_t)f32.m2lSrc.size() : 0; }
    int64_t f32Bytes() const { return f32Ready ? (int64_t)(d32Km2l.bytes + d32Knear.bytes) : 0; }
    hipStream_t stream() const { return own; }
    // raise (ANISO_ERR_RUNTIME) if a fused top-of-tree launch gave up waiting for its
    // producers since the last check: its locals, and so the apply's output, are invalid
    void checkDeviceErrors();
    // recovery from a fused-launch time-out where the library owns the timeline (the
    // host-pointer block operator, the block solve): if the flag is set, drain `s`,
    // clear it, switch the fused launch off for the rest of the call (forceUnfused)
    // and count it; the caller then re-runs the apply on the tier launches
    bool recoverTopTimeout(hipStream_t s);
    int64_t topRecoveries = 0;  // applies re-run after a time-out (aniso_stats)
    int64_t topSteals();        // tier tasks the fused launch's waiting blocks computed themselves (aniso_stats)
    int64_t oneXApplies = 0;    // sharded matvecs through the one-collective exchange (aniso_stats)
    int64_t upPartialApplies = 0;  // ... of them with the upper multipoles as partial sums (aniso_stats)
    bool nearOverlaps() const { return overlapOn(); }  // the block apply's near field on a side stream
    // the one-GPU block apply forms its bottom up tier inside the near field
    bool nearUpTier() const { return nearUpOn && plan.nearUpOk && !overlapOn(); }
    bool forceUnfused = false;
    // set while a call that recovers its own time-outs (the block solve) runs: the
    // entry checks of the applies it enqueues leave the flag to its recovery points
    bool ownTimeline = false;
    // wait for every apply enqueued by this handle (both streams), then check
    void sync();
    // development timeline of the last fused top-of-tree launch (ANISO_TOP_TRACE=1,
    // tools/top_trace.py): per block 8 values {start, waited, end (100 MHz ticks), hw id,
    // kind (-k: up tier k; else the cluster id), wait tier, targets, block reads}
    std::vector<int64_t> topTrace();
    bool harmonicReady() const { return useAtt && attReady; }
    bool clustersOn() const { return useClusters; }
    // the block apply's upper up tiers ride in the clustered M2L launch (k_top_m2l_hc);
    // ANISO_TOP_FUSED=0 runs them as launches of their own before the clusters (a rank
    // of 8: 0.262 against 0.251 ms, same-process A/B r03ls)
    bool topFusedOn() const {
        const int ntier = (int)plan.upTierTask.size() - 1;
        return useClusters && !detSums && topFusedMode != 0 && !forceUnfused && top_fused_enabled() && ntier >= 2 &&
               ntier <= kMaxTopTiers &&
               plan.upLastLeafTier == 0 && plan.hmClWait.size() + 1 == plan.hmClPtr.size();
    }
    // bitwise-reproducible applies: the clustered M2L with its LDS
    // sums in fixed point (integer adds: order-independent) and the upper up tiers as
    // launches of their own; ANISO_DET_PER_TARGET=1 keeps the round-2 form instead (one
    // wave per target, every sum in a fixed order, every block read from both ends)
    void setDeterministic(bool on) {
        detSums = on && !detPerTarget;
        useClusters = !(on && detPerTarget);
    }
    bool deterministicOn() const { return detSums || !useClusters; }
    bool modeCached(int id) const { return id >= 0 && id < kernelSize && modes[id].ready; }
    int kernelSize = 0;
    // stage timing with HIP events recorded in-stream (no host sync per apply);
    // stageTimes() averages every apply recorded since setTiming(level > 0).
    // level 1: every stage; level 2: the M2L and near-field spans only (4 events per
    // block apply instead of 9 -- the timers cost 1.3 % of a block matvec, r04as)
    void setTiming(int level);
    StageTimes stageTimes();
    int timeStages = 0;

    Geometry geo;
    Tree tree;
    Plan plan;
    int ks = 0, ns = 0, np = 0, maxLevel = 0;
    double g = 0;
    bool coeffSet = false;
    std::vector<double> sigma_s, sigma_t;

    // stats
    int64_t nearEntries() const { return plan.pairsNear; }
    int64_t m2lEntries() const { return plan.pairsM2L * 256; }
    int maxNearSources() const { return maxNearS; }

private:
    void apply(const double* charge, bool treeIn, const double* sigT, int id, double* out, bool treeOut, hipStream_t s,
               int mask);
    // phase 0: the whole apply (input valid everywhere, every up task); 1 / 2: the
    // two halves of a sharded apply (forwardTreeBegin / End)
    void applyBlock(int K, const double* x, int64_t ldx, bool treeIn, const double* sigT, int nterm, const int* ids,
                    const double* mixes, double* out, int64_t ldo, bool treeOut, hipStream_t s, int mask,
                    int phase = 0, double* rootsSend = nullptr, const double* rootsRecv = nullptr);
    struct Pending {  // state between the two phases of a sharded apply
        bool active = false, nearDone = false;
        int K = 0, e0 = -1, ePack = -1, eStart = -1;
    } pend;
    // the public call that started a pending sharded apply: its _end must repeat it
    // (operation, which, vectors, strides, sigma_s, g)
    struct PendingCall {
        int kind = -1, which = -1;
        const void *x = nullptr, *out = nullptr, *sig = nullptr;
        int64_t ldx = 0, ldo = 0;
        double g = 0;
        bool operator==(const PendingCall& o) const {
            return kind == o.kind && which == o.which && x == o.x && out == o.out && sig == o.sig && ldx == o.ldx &&
                   ldo == o.ldo && (g == o.g || (std::isnan(g) && std::isnan(o.g)));
        }
    } pendCall;
    void pendingCall(int phase, const PendingCall& c);
    void ensureWork(int K);  // work arrays for K right-hand sides
    const ModeArgs* modeTable(int K, int nterm, const int* ids, const double* mixes);
    // harmonic (mode-shared) block apply, DESIGN.md §3.9: the E caches of every
    // directed M2L pair and near block, built at the first cache() of a block handle
    bool harmonicWeights(int K, int nterm, const int* ids, const double* mixes, HarmWeights& hw) const;
    void buildAttCache();
    bool useAtt = false, attReady = false;
    DevBuf dAttM2L, dAttNear, dSigDiag, dAttPtr, dAttSrc, dAttBlk, dAttOwner, dAttOther;
    DevBuf dAttMax;                // max |E| of dAttM2L (the deterministic sums' bound)
    DevBuf dHmClBound, dNodeWmax;  // the deterministic sums: per cluster, per node
    DevBuf dHmClPtr, dHmTgt, dHmPtr, dHmSrc, dHmBlk, dHmSlot, dHmNDir;  // cluster plan
    DevBuf dHmHaloPtr, dHmHaloPos, dHmPart, dDnChainFold;  // the halo form (Plan::hmHaloPtr)
    DevBuf dHmClWait, dTopCnt;  // fused top-of-tree launch: per-cluster wait tier, per-tier counters
    DevBuf dTopSteals;          // tier tasks computed by waiting blocks of the fused launch (persistent)
    DevBuf dTopTrace;           // ANISO_TOP_TRACE=1: the launch's per-block timeline
    DevBuf dKryPart;            // partial sums of the Krylov primitives
    // config 5's library solve (solve16Mixed): its vectors and fp32 basis, kept between
    // solves (grown, never shrunk: a hipFree synchronises the device)
    DevBuf s16B, s16X, s16R, s16W, s16D, s16Df, s16W32, s16V, s16St, s16Part, s16R0;
    void arnoldiParts(int rows);  // dKryPart for sweeps of `rows` rows
    bool topTraceOn = false;
    int hmRing = 0;  // the cluster M2L's LDS ring depth (ANISO_HM_RING; 0: the one-block-in-flight form)
    int hmWpe = 0;   // ANISO_HM_WPE=3/4/8: the one-block form's occupancy (0: 4 where LDS allows)
    // ANISO_NEAR_WPE: the staged near field capped at 128 VGPRs, 4 waves per SIMD (the default
    // since round 5: 0.312 against 0.329 ms standalone, r05y), or 3 (121 VGPRs, the round-4 form)
    int nearWpe = 4;
    int topFusedMode = 1;  // ANISO_TOP_FUSED=0: the upper up tiers as launches of their own
    // the near field's groups ride at the end of the fused top-of-tree + M2L launch
    // instead of a side-stream launch (ANISO_NEAR_IN_TOP=1; on a shard in phase 2)
    bool nearInTop = false;
    // the staged near field forms its charges from the input and forks at the start
    // of the block apply, beside the up pass (ANISO_NEAR_EARLY=0: after it, from fT)
    bool nearEarly = true;
    bool nearOrderUp = true;  // the near launch issued after the bottom up tier's (ANISO_NEAR_ORDER=first: before)
    // a one-collective sharded matvec starts the near field's own-range groups beside
    // phase 1 (ANISO_SHARD_NEAR_EARLY=0: every group after the exchange)
    bool shardNearEarly = true;
    // the bottom up tier inside the staged near field on one GPU (Plan::nearUpOk, serial
    // schedule; ANISO_NEAR_UP=0: its own launch)
    bool nearUpOn = true;
    DevBuf dNearUpGrp;
    int topTraceBlocks = 0, topTraceNear = 0;
    // the attached communicator and its halo exchange plan (commInit): per element of
    // the send / receive position lists its tree position and its place in the
    // peer-major buffers (base + b * stride for block b); doubles per peer
    std::unique_ptr<Collectives> comm;
    DevBuf dHxSendPos, dHxSendBase, dHxSendStride, dHxRecvPos, dHxRecvBase, dHxRecvStride, dHxSendBuf, dHxRecvBuf;
    DevBuf dXRootsSend, dXRootsRecv;
    std::vector<int64_t> hxScount, hxSoff, hxRcount, hxRoff;
    int64_t hxNsend = 0, hxNrecv = 0;
    // the one-collective exchange (Plan::xOneOk; ANISO_ONE_EXCHANGE=0 keeps the halo
    // all-to-all before phase 1): per peer one buffer part = the tier-0 root records,
    // its input positions (block-major, as the halo exchange), its multipole rows
    // (16 x K each);
    // oneXActive marks the two phases of such a matvec for applyBlock
    DevBuf dOxSendPos, dOxSendBase, dOxSendStride, dOxRecvPos, dOxRecvBase, dOxRecvStride;
    DevBuf dOxSendNode, dOxSendNodeBase, dOxRecvNode, dOxRecvNodeBase, dOxSendBuf, dOxRecvBuf, dXOwnT0Tasks;
    DevBuf dOxRootSend, dOxRootRecv, dOxRootDst;  // the root records' place in each peer part
    DevBuf dNearGrpEarly, dNearGrpLate;           // Plan::nearGrpEarly / nearGrpLate
    int64_t oxRootParts = 0;
    std::vector<int64_t> oxScount, oxSoff, oxRcount, oxRoff;
    int64_t oxNsendPts = 0, oxNrecvPts = 0, oxNsendNodes = 0, oxNrecvNodes = 0;
    bool oxReady = false, oneXActive = false, oneXOn = true;
    // the upper multipoles as partial sums (Plan::xUpPartial on every rank): the parts
    // carry every rank's records instead of the roots; the unpack sums each upper
    // node's records (oxUpSumNode / Ptr / Src: >= 0 an offset into the receive buffer,
    // < 0 ~offset into this rank's own records); upActive marks such a matvec
    bool oxUp = false, upActive = false;
    // the partial tasks as tails of the bottom tier (ANISO_UP_TAILS=1; default: in the
    // pack launch, measured faster on a rank of 8: r06h)
    bool upTailsOn = false, upTailActive = false;
    // the one-collective exchange's pack launch, enqueued by phase 1 right after the own
    // tier-0 launch when the near field's early groups fork after it
    // (ANISO_NEAR_AFTER_PACK=1): packHook set by blockOpShardedDev, packIssued by phase 1
    bool nearAfterPack = false, packIssued = false;
    int sidePrio = 0;  // ANISO_SIDE_PRIO: the side stream's priority (-1 lowest, 0 default, 1 highest)
    std::function<void(hipStream_t)> packHook;
    DevBuf dXT0Part, dXUpRoots, dXUpCnt, dXUpStage;
    DevBuf dXUpTask, dXUpRec, dOxUpSumNode, dOxUpSumPtr, dOxUpSumSrc;
    int64_t oxUpSums = 0;
    bool oneExchangeUsable(int which);
    bool cachesReady() const;
    bool oneExchangeLocal() const;  // this rank's (shard- and process-dependent) part, gathered at commInit
    // sticky time-out flag of the fused launch's in-kernel hand-offs, in host-visible
    // memory (the kernel stores 1 there when a wait gives up; checked at every API
    // entry and by sync(), never read on the device)
    unsigned* topErr = nullptr;
    // ANISO_TOP_SPIN_LIMIT: polls of a tier counter (~1 us each) before a waiting block of
    // the fused launch computes the tier itself (tests: 0 makes every waiter compute)
    unsigned topSpinLimit = 1u << 16;
    bool useClusters = true;
    bool detSums = false;       // the clustered M2L's fixed-point sums (setDeterministic)
    bool detPerTarget = false;  // ANISO_DET_PER_TARGET
    void detBounds();           // dHmClBound from the plan (once)
    std::map<std::string, DevBuf> modeTabs;
    const CorrFold& corrTable(int K, int nterm, const int* ids, const double* mixes);
    std::map<std::string, CorrFold> corrTabs;
    int workK = 0;

    void ensureDevice();
  public:
    int deviceId() const { return device; }
  private:
    void uploadPlan();
    int device = -1;
    hipStream_t own = nullptr;
    // side stream of the harmonic block apply: near field + corrections run beside
    // the M2L (both HBM-bound, neither saturates alone)
    hipStream_t side = nullptr;
    hipEvent_t evFork = nullptr, evJoin = nullptr;
    // x - mforward(x) fused into the down pass (blockOpDev sets subX for one apply)
    bool fuseSub = true;
    const double* subX = nullptr;
    int64_t subLd = 0;
    // the near field beside the up pass and the M2L on a side stream: -1 (default) on a
    // shard only -- one GPU runs them serially, 1.190 against 1.202 ms per block matvec
    // (same-process A/B, r05r; 1.148 against 1.162, r04ar): each kernel alone keeps
    // the load path busy, and the fork and join cost more than the overlap saves; a
    // rank of 8 overlaps (0.208 against 0.229 ms, r04ar).  ANISO_OVERLAP=0/1 forces it.
    int overlap = -1;
    bool overlapOn() const { return overlap < 0 ? plan.nranks > 1 : overlap != 0; }
    // stage timing: events recorded in-stream, (stage, start, end) spans per apply
    std::vector<hipEvent_t> evPool;
    int evUsed = 0;
    struct Span {
        int stage, a, b;
    };
    std::vector<Span> spans;
    int applies = 0;
    int mark(hipStream_t s);
    int maxNearS = 0;
    // geometry / tree on device
    DevBuf dPxT, dPyT, dPerm, dW, dNcx, dNcy, dNrx, dNry, dBegin, dCount, dParent, dSlot, dChild, dIsLeaf, dNodeGeo;
    DevBuf dLeaves, dNearPtr, dNearSrc, dNearKOff, dM2LTgt, dM2LPtr, dM2LSrc, dM2LPairTgt;
    DevBuf dUpTaskPtr, dUpGrpPtr, dUpGrp, dUpNode, dUpCode, dUpDesc, dUpGrpFix, dUpGeom, dUpLeaf;                       // up-pass tiers
    DevBuf dDnTaskPtr, dDnGrpPtr, dDnGrp, dDnNode, dDnLeafPtr, dDnLeafSlot, dDnLeafIdx, dDnLeafPts, dDnPtsRange, dDnDesc, dDnGrpFix, dDnLeafGeom;  // down
    DevBuf dLeafInfo, dNearPtsPtr, dNearPts;
    DevBuf dNsPtr, dNsPts, dNearLoc;  // near field sources staged per workgroup (k_near_hs)
    // the harmonic near field's symmetric U storage (Plan::nearSymHsOn): its column
    // lists, canonical partner blocks and the leaves' first table rows
    DevBuf dHsPtsPtr, dHsLoc, dHsKOff, dHsSym, dHsSrcPtr, dHsSrc, dHsDst, dNearSelfRow;
    DevBuf dNearGrpInPtr, dNearGrpIn;
    DevBuf dNearCorrRow;              // d = 1: the stencil's table rows (corrections fused into k_near_hs)
    DevBuf dXT0Tasks, dXRootRecv, dXRootSlot, dXSendSlot;  // sharded up pass (plan.buildExchange)
    DevBuf dM2LNDir, dM2LCanonBase, dM2LInPtr, dM2LOutSlot, dM2LPart;  // symmetric M2L
    DevBuf dNearSym, dNearPart, dDnLeafNear, dDnNearPtr, dDnNearOff, dDnChainPtr, dDnChain;              // symmetric near field
    DevBuf dParams, dStCoef;
    DevBuf dCharge, dOut, dFT, dCT, dMult, dLocal, dSigmaS, dTmp, dTmp2;
    DevBuf dWT, dSigmaT, dIperm, dTmpS;  // tree-order path
    DevBuf dPadIn, dPadOut, dBlk;       // block operator: padded right-hand sides, x - mforward(x)
    DevBuf dHostIn, dHostOut, dSigAlt;  // host-pointer block operator: staging, sigma_s override
    std::vector<ModeCache> modes;
    Params hostP{};  // the parameter block uploaded to dParams
    // fp32 operator (buildF32): leaves with their directed U/W sources (padded to 16
    // columns), M2M / L2L levels, directed M2L pairs
    void buildF32();
    bool f32Ready = false;
    void buildMrhsPlan();  // the directed lists both 16-RHS operators share (f32 plan below)
    bool mrhsPlanReady = false;
    struct Mrhs64Cache {
        DevBuf Km2l, Knear;
    };
    std::map<int, Mrhs64Cache> m64;  // fp64 16-RHS caches per mode id
    void buildMrhs64(int id);
    size_t mrhs64Bytes();  // HBM a buildMrhs64 would allocate
    DevBuf d64Rup, d64Rdn, d64Mult, d64Local, d64FT, d64CT;
    DevBuf d32PairTgt, d32SrcPtr, d32SrcNodes, d32KoffD, d32SrcCount;  // cache-build inputs of the 16-RHS plan
    struct F32Plan {
        std::vector<int> leaves;
        std::vector<std::array<int, 4>> leafInfo;  // node, begin, count, padded sources
        std::vector<int64_t> nearPtr, koff, koffD, srcPtr;
        std::vector<int> nearPts, srcNodes, srcCount;
        std::vector<std::vector<int>> m2m, l2l;  // per level: M2M bottom-up, L2L top-down
        std::vector<int> m2lTgt, m2lSrc, m2lPairTgt;
        std::vector<int64_t> m2lPtr;
        int64_t nearTiles = 0, nearD = 0;
        int maxSrc = 1;
    } f32;
    DevBuf d32Leaves, d32LeafInfo, d32NearPtr, d32NearPts, d32Koff, d32Tgt, d32Ptr, d32Src;
    DevBuf d32Km2l, d32Knear, d32Rup, d32Rdn, d32Mult, d32Local, d32FT, d32CT, d32Level;
    std::vector<DevBuf> d32LevelNodes;  // m2m levels then l2l levels
};

}  // namespace aniso
