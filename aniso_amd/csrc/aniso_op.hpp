// aniso_op.hpp -- the MI355X operator behind the C ABI (one per handle).
//
// Host state (geometry, tree, plan) is built by the constructor without touching
// the GPU; device buffers are created on first use (setCoeff), on the HIP device
// that is current at that moment.
#pragma once

#include <hip/hip_runtime.h>

#include <array>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "host.hpp"

namespace aniso {

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
    bool ready = false;
};

struct StageTimes {
    float prep = 0, up = 0, m2l = 0, gather = 0, near = 0, down = 0, corr = 0, total = 0;
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
    void mappingDev(const double* charge, int id, double* out, hipStream_t s, int stageMask = 0x3f);
    void mappingTreeDev(const double* qTree, int id, double* outSlice, hipStream_t s);
    void forwardTreeDev(const double* xTree, double* ySlice, hipStream_t s);

    // --- extensions
    void setShard(int rank, int nranks);
    void getShard(int64_t* ownBegin, int64_t* ownEnd) const { *ownBegin = plan.ownBegin; *ownEnd = plan.ownEnd; }
    // sharded apply: writes only owned targets of out (original order), others untouched
    void permuteToTree(const double* orig, double* tree, hipStream_t s);
    void lineIntegrals(const double* seg, int n, double* out);
    // callers of the hot path (main.cpp:125-141)
    void forwardDev(const double* u, double* out, hipStream_t s);
    int gmresHost(const double* q, double* x, int m, int maxit, double tol, double* hist, int maxhist,
                  double* finalResid);
    hipStream_t stream() const { return own; }
    bool modeCached(int id) const { return id >= 0 && id < kernelSize && modes[id].ready; }
    int kernelSize = 0;
    // stage timing with HIP events recorded in-stream (no host sync per apply);
    // stageTimes() averages every apply recorded since setTiming(true)
    void setTiming(bool on);
    StageTimes stageTimes();
    bool timeStages = false;

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

    void ensureDevice();
    void uploadPlan();
    int device = -1;
    hipStream_t own = nullptr;
    hipStream_t aux = nullptr;        // near field + corrections overlap the far field
    hipEvent_t evFork = nullptr, evJoin = nullptr;
    bool overlap = false;  // ANISO_OVERLAP=1: near + corr on the auxiliary stream (no gain measured)
    static constexpr int kStageEvents = 10;
    std::vector<std::array<hipEvent_t, kStageEvents>> evPool;
    int evUsed = 0;
    int maxNearS = 0;
    // geometry / tree on device
    DevBuf dPxT, dPyT, dPerm, dW, dNcx, dNcy, dNrx, dNry, dBegin, dCount, dParent, dSlot, dChild, dIsLeaf;
    DevBuf dLeaves, dNearPtr, dNearSrc, dNearKOff, dM2LTgt, dM2LPtr, dM2LSrc, dM2LPairTgt;
    DevBuf dUpTaskPtr, dUpGrpPtr, dUpGrp, dUpNode, dUpCode, dUpDesc, dUpGrpFix, dUpGeom, dUpLeaf;                       // up-pass tiers
    DevBuf dDnTaskPtr, dDnGrpPtr, dDnGrp, dDnNode, dDnLeafPtr, dDnLeafSlot, dDnLeafIdx, dDnLeafPts, dDnPtsRange, dDnDesc, dDnGrpFix, dDnLeafGeom;  // down
    DevBuf dLeafInfo, dNearPtsPtr, dNearPts;
    DevBuf dM2LNDir, dM2LCanonBase, dM2LInPtr, dM2LOutSlot, dM2LPart;  // symmetric M2L
    DevBuf dNearSym, dNearPart, dDnLeafNear, dDnNearPtr, dDnNearOff, dDnChainPtr, dDnChain;              // symmetric near field
    DevBuf dParams, dStCoef;
    DevBuf dCharge, dOut, dFT, dCT, dMult, dLocal, dTotal, dSigmaS, dTmp, dTmp2;
    DevBuf dWT, dSigmaT, dIperm, dTmpS;  // tree-order path
    std::vector<ModeCache> modes;
};

}  // namespace aniso
