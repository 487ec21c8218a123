// host.hpp -- host-side (C++) state of the MI355X matvec: geometry, quadtree,
// flattened interaction lists and the small translation-invariant tables.
//
// Everything here is built once per geometry (aniso_create) or per mode
// (aniso_cache) and uploaded to HBM; the per-apply work is all on the GPU.
#pragma once

#include <algorithm>
#include <array>
#include <cstdint>
#include <string>
#include <vector>

namespace aniso {

constexpr double kEps = 1e-12;  // bbfmm/utils.h:46
constexpr int kLeafCode = -2147483647 - 1;  // upCode of a leaf (P2M from its points)
constexpr int kTaskLevels = 7;  // levels per up/down task record (tasks span <= 4)
constexpr int kMaxCanon = 32;       // canonical (symmetric) M2L pairs per target (k_m2l's register staging)
constexpr int kMaxCanonBlock = 16;  // the same on block handles (ks > 1; LDS staging at K >= 4)
constexpr int kClusterDepth = 3;   // harmonic M2L clusters: <= 4^3 = 64 targets
constexpr int kMinClusters = 512;  // ... but no fewer workgroups than this (shards of N-GPU runs)

// Geometry::Geometry (Geometry.cpp:10-114) + the singular Duffy rule
// (KernelFactory.cpp:15-16, 863-986).
struct Geometry {
    int sz = 0, d = 0, d2 = 0, ns = 0;
    double dx = 0;
    int nsq = 0;
    int64_t N = 0;
    std::vector<double> px, py, w;            // nodes + weights, square-major order
    std::vector<double> gx, gw;               // 1-D volume rule on [-1,1]
    std::vector<double> qx, qy, qw, sqrtW;    // tensor rule (d2)
    int nref = 0;
    std::vector<double> refx, refy, refw;     // two-level refinement rule (16 d2)
    std::vector<double> interp;               // d2 x d2, col-major
    std::vector<double> nearMap;              // nref x d2, col-major
    std::vector<double> lnorm;                // d2 (norms of the *refinement* matrix: quirk)
    std::vector<double> sgx, sgw;             // singular rule on [0,1] (affine)
    int nsing = 0;                            // 8 ns^2
    std::vector<double> singX, singY, singW;  // d2 x nsing

    void build(int sz_, int d_, int ns_);
};

// bbfmm::tree (bbfmm.h:146-449) flattened: node ids follow the reference's
// assignment order (4 consecutive ids per split, depth-first), points are
// stored in leaf-contiguous tree order (perm), lists as sorted CSR.
struct Tree {
    int nn = 0, maxLevel = 0;
    double cx = 0, cy = 0, rx = 0, ry = 0;
    std::vector<int> parent, level, slot, isLeaf, isEmpty;
    std::vector<std::array<int, 4>> child;
    std::vector<double> ncx, ncy, nrx, nry;
    std::vector<int64_t> begin, count;        // point range in tree order
    std::vector<int> perm;                    // tree position -> original index
    std::vector<int64_t> uPtr, vPtr, wPtr, xPtr;
    std::vector<int> uIdx, vIdx, wIdx, xIdx;

    void build(const double* x, const double* y, int64_t n, int rank, int maxLevelArg, int nthreads);
};

// Per-shard work lists (all of them when nranks == 1).
struct Plan {
    int rank = 0, nranks = 1;
    int64_t ownBegin = 0, ownEnd = 0;          // owned tree-position range
    std::vector<int> leaves;                   // non-empty leaves whose points are owned
    std::vector<int64_t> nearPtr;              // CSR over leaves -> source nodes
    std::vector<int> nearSrc;
    std::vector<int64_t> nearKOff;             // per leaf: offset of its K block (doubles)
    std::vector<std::array<int, 4>> leafInfo;  // per leaf: node, begin, count, S (source points)
    // symmetric storage: M2L targets' stored sources are
    // [m2lNDir directed | canonical]; canonical pair c (= m2lCanonBase + j) sends
    // its transposed product to partial slot m2lOutSlot[c]; slots are contiguous
    // per receiver: [m2lInPtr[k], m2lInPtr[k+1]) for target m2lTgt[k].
    bool symmetric = true;
    // input: symmetric U storage in the near field (worth it for single right-hand
    // sides; block applies read every block directed)
    bool nearSymmetric = true;
    int nearMaxLeaf = 0;  // largest owned target leaf (points)
    // input: canonical M2L pairs kept per target (<= kMaxCanon; block handles use
    // fewer: k_m2l stages their transposed products in LDS)
    int maxCanon = kMaxCanon;
    int m2lMaxCanon = 0;  // largest canonical count of a target
    std::vector<int> m2lNDir, m2lCanonBase, m2lInPtr, m2lOutSlot;
    int m2lCanon = 0;
    int64_t storedM2L = 0, storedNear = 0, nearPartTotal = 0;
    std::vector<std::array<int, 2>> nearSym;   // per leaf: directed source points, partial base
    std::vector<int> nearInPtr, nearInOff;     // per leaf: offsets of the partial blocks addressed to it
    std::vector<int64_t> nearPtsPtr;           // per leaf: its S source points (tree positions)
    std::vector<int> nearPts;
    // near field staged per workgroup (k_near_hs): 16 consecutive
    // leaves (<= 16 points each) share one LDS table of the union of their source
    // points; nearLoc[j] = nearPts[j]'s row in its group's table, nsPtr = CSR of the
    // tables (tree positions).  Empty when the leaves do not fit the scheme.
    std::vector<int64_t> nsPtr;
    std::vector<int> nsPts;
    std::vector<uint16_t> nearLoc;
    int nsMax = 0;  // largest table (points)
    // d = 1: per (leaf, target row) the table rows of the 3x3 stencil's 9 points
    // (0xFFFF outside the grid), so k_near_hs applies the corrections from its table
    std::vector<uint16_t> nearCorrRow;
    bool nearCorrOk = false;
    // input: the staged near field of block handles with symmetric U storage (DESIGN.md
    // §3.11): a U pair of two owned leaves <= 16 points is stored once, by its smaller
    // id, whose lanes apply it both ways from one read.  The partner's product goes to
    // LDS when the partner is in the same 16-leaf group, else to a partial slot the
    // down pass adds (nearInPtr / nearInOff).  Per leaf: hsSym = (directed columns,
    // all columns: the canonical ones, partner by partner, follow the directed ones),
    // per column hsDst = where its partner product goes (>= 0 the partial slot of that
    // point, < 0 ~(its LDS row: group slot x 16 + point); 0 for directed columns), and
    // nearSelfRow = the table row of the leaf's first point.  Built only when every
    // owned leaf fits the staged kernel (nearSymHsOn), else the harmonic near field
    // reads the directed lists.
    bool nearSymHs = false;
    bool nearSymHsOn = false;
    std::vector<int> hsDst;
    std::vector<uint16_t> nearSelfRow;
    // its column lists (beside the directed nearPtsPtr / nearLoc / nearKOff, which the
    // per-mode kernels keep): table rows per column, E offsets, (directed, all)
    // columns per leaf, source nodes per leaf (the att cache build), partial slots
    std::vector<int64_t> hsPtsPtr, hsKOff, hsSrcPtr;
    std::vector<uint16_t> hsLoc;
    std::vector<std::array<int, 2>> hsSym;
    std::vector<int> hsSrc;
    int64_t hsKTotal = 0, hsPartTotal = 0, hsStored = 0;
    // the partner products within a 16-leaf group go to LDS slots (16 rows x K each,
    // one per in-group canonical block, <= kNearGrpSlots per group; the rest to
    // partials): per leaf the slots it receives (CSR, ascending), summed in that
    // fixed order -- no atomics, so the apply stays deterministic
    static constexpr int kNearGrpSlots = 48;
    // the bottom up tier inside the staged near field (one rank): every
    // 16-leaf group is exactly one tier-0 subtree (a root, 4 parents, 16 leaves, all
    // non-empty) -- then per group 25 ints (NearHsArgs::upGrp): per leaf (parent slot
    // << 2 | quadrant), per parent its quadrant, the parents' nodes, the root node
    std::vector<int> nearUpGrp;
    bool nearUpOk = false;
    std::vector<int> nearGrpInPtr, nearGrpIn;
    int nearGrpSlots = 0;
    int64_t nearKTotal = 0;
    std::vector<int> m2lTgt;                   // active target nodes with M2L work
    std::vector<int64_t> m2lPtr;               // CSR over m2lTgt -> source nodes
    std::vector<int> m2lSrc;
    // mode-shared (attenuation) plan of block handles: every V then
    // X source of each m2lTgt with the E block it reads: attBlk >= 0 a stored block
    // read as stored, ~attBlk a stored block read transposed (tau is symmetric: the
    // V pair's block is stored once, by its smaller id, when both ends are targets
    // here).  Stored block k: target attOwner[k], source attOther[k].
    std::vector<int64_t> attPtr;
    std::vector<int> attSrc, attBlk, attOwner, attOther;
    // the same work in clusters: cluster c = the active targets of
    // one level under one ancestor kClusterDepth levels up (<= 4^kClusterDepth
    // nodes), one workgroup each, locals accumulated in LDS.  A V pair with both
    // ends in one cluster is applied from ONE read of its stored block by the
    // smaller id (hmSlot = the partner's slot in the cluster, which also receives the
    // transposed product); the partner skips it.  Other pairs as attSrc / attBlk.
    // per target: [hmNDir directed | in-cluster canonical] entries
    std::vector<int> hmClPtr, hmTgt, hmSrc, hmBlk, hmSlot, hmNDir;
    std::vector<int64_t> hmPtr;
    int hmMaxCl = 0;
    int hmDepth = 0;  // cluster depth chosen (ancestor levels up)
    std::vector<int> hmClWait;  // per cluster: the upper up tier whose multipoles it reads (0: none)
    int64_t hmDual = 0;
    // cross-cluster pairs read by the non-storing end: a directed copy of the stored
    // block (E of the reversed pair), appended after the stored blocks in the cache,
    // so that k_m2l_hc reads every block in the stored orientation (16-B lane loads).
    // Empty in the halo form (below, the default).
    std::vector<int> hmCopyOwner, hmCopyOther;
    // the halo form: a cross-cluster V pair with both ends
    // targets is read ONCE, by the cluster of its smaller id, which adds the partner's
    // product to an LDS slot of its halo (slots nt .. nt + nh - 1 of cluster c, whose
    // nodes are hmHaloNode[hmHaloPtr[c] ..]); at the cluster's end the halo slots go
    // to a partial buffer, and a fold adds each node's partials to its locals (CSR:
    // node hmFoldNode[f] receives halo slots hmFoldIdx[hmFoldPtr[f] .. hmFoldPtr[f+1])).
    // input: ANISO_HM_HALO=0 keeps the directed copies (A/B runs)
    bool hmHalo = true;
    std::vector<int> hmHaloPtr, hmHaloNode, hmFoldPtr, hmFoldNode, hmFoldIdx;
    // the partials are stored receiver-contiguously: halo slot h at position
    // hmHaloPos[h] (its place in hmFoldIdx), so node n's partials are one range,
    // packed per node as (first << 3) | count in hmFoldOf[n] (0: none); the down pass
    // adds them where it loads the locals (dnNode[.][3], dnChainFold)
    std::vector<int> hmHaloPos, hmFoldOf;
    int hmMaxLds = 0;  // largest cluster + halo (LDS slots of 16 x K doubles)
    // tiered up / down passes: tier k has root level
    // tierRootLevel[k] and bottom level tierBottomLevel[k] (k = 0 is the deepest).
    std::vector<int> tierRootLevel, tierBottomLevel;
    // up (global on every rank; tiers bottom-up): task = subtree nodes, deepest
    // level first; upCode per node: child LDS slots, -1 empty, -(id+2) a root of
    // the tier below (read from HBM), kLeafCode for a leaf (P2M)
    std::vector<int> upTierTask, upTaskPtr, upGrpPtr, upGrp, upNode;
    std::vector<std::array<int, 4>> upCode;
    int upMaxTask = 1;
    // per tier: its largest task (a launch sizes its LDS for its own tiers only: the
    // fused top-of-tree launch runs tiers >= 1, 21-node tasks instead of tier 0's 85)
    std::vector<int> upTierMaxTask;
    int upMaxTaskFrom(int k0) const {
        int m = 1;
        for (size_t k = (size_t)k0; k < upTierMaxTask.size(); ++k) m = std::max(m, upTierMaxTask[k]);
        return m;
    }
    int upLastLeafTier = 0;  // last up tier with a P2M leaf: fT / cT are complete after it
    // the same, as records the kernel loads in one round: per task (first node,
    // nodes, first point, levels) + kTaskLevels+1 level starts; per node the box
    // (cx, cy, 1/rx, 1/ry) and the point range relative to the task's first point
    std::vector<std::array<int, 4>> upDesc;
    std::vector<int> upGrpFix;
    std::vector<std::array<double, 4>> upGeom;
    std::vector<std::array<int, 2>> upLeaf;
    // down (owned part): tasks with owned leaves, all tiers in one launch; dnNode =
    // (node, parent code: LDS slot, -1 none/zero, -2 the task root (chain total);
    // child slot (R index), 0); leaves of each task in tree order (L2P + near gather)
    std::vector<int> dnTierTask, dnTaskPtr, dnGrpPtr, dnGrp;
    std::vector<std::array<int, 4>> dnNode;
    std::vector<int> dnLeafPtr, dnLeafSlot, dnLeafIdx, dnLeafPts;  // leaves in tree order; dnLeafPts = begin
    std::vector<std::array<int, 2>> dnPtsRange;                     // per task: owned point range
    std::vector<std::array<int, 2>> dnLeafNear;  // per leaf entry: (first, count) in its task's dnNearOff
    std::vector<int> dnNearPtr, dnNearOff;       // per task: the near partial offsets of its leaves
    int dnMaxNear = 1;
    std::vector<int> dnChainPtr;                 // per task: its root's ancestors below the tree root,
    std::vector<std::array<int, 2>> dnChain;     // top-down (node, child slot): the parent total's L2L chain
    std::vector<int> dnChainFold;                // per chain entry: its node's halo partials (hmFoldOf)
    int dnMaxChain = 1;
    // per task three int4 records (nodes, leaves / owned points, chain / near
    // offsets, levels) + kTaskLevels+1 level starts; per leaf entry its box
    std::vector<std::array<int, 4>> dnDesc;
    std::vector<int> dnGrpFix;
    std::vector<std::array<double, 4>> dnLeafGeom;
    int dnMaxTask = 1, dnMaxLeaves = 1;
    int64_t pairsNear = 0, pairsM2L = 0;       // kernel entries per apply
    // sharded up pass: the rank runs only the tier-0 up tasks it
    // needs -- those holding its own points or anything its M2L, near field or
    // correction stencil reads below the tier-0 root level -- and exchanges the
    // tier-0 root multipoles with every rank (one all-gather; the tiers above run
    // on every rank).  Its input must be valid at its own range and at xHalo.
    std::vector<int> upTaskRoot;      // per up task: its root node
    std::vector<int> xT0Tasks;        // tier-0 tasks run by this rank (ascending)
    std::vector<int> xRootSend;       // tier-0 roots this rank contributes (tree order)
    std::vector<int> xRootRecv;       // nranks x xRootChunk all-gather slots -> node (-1: padding)
    std::vector<int> xRootSlot;       // per node: its all-gather slot (-1: not a tier-0 root)
    std::vector<int> xSendSlot;       // per node: its slot in this rank's send buffer (-1: not sent here)
    int xRootChunk = 0;               // roots per rank in the all-gather (the largest contribution)
    std::vector<int64_t> xHalo;       // [b, e) pairs of tree positions needed outside [ownBegin, ownEnd)
    int64_t xHaloPoints = 0;
    // The one-collective exchange: a rank runs only the
    // tier-0 tasks of its own subtrees (xOwnT0Tasks); after them one grouped
    // send/receive carries the tier-0 roots to every rank together with, from each
    // owner, the multipoles below the root level that this rank's M2L reads
    // (xNeedNodes) and the input at the positions its near field, corrections and
    // upper-tier P2M read outside its range (xOneHalo, [b, e) pairs).  xOneOk: the
    // tree allows it (every own tier-0 subtree inside the own range).
    std::vector<int> xOwnT0Tasks;
    // the staged near field's 16-leaf groups whose source table lies in the own range
    // (they run beside phase 1) and the others (after the exchange)
    std::vector<int> nearGrpEarly, nearGrpLate;
    std::vector<int> xNeedNodes;      // ascending node ids, owned by other ranks
    std::vector<int64_t> xOneHalo;
    int64_t xOneHaloPoints = 0;
    bool xOneOk = false;
    // The upper multipoles as partial sums (the one-collective
    // form over a tree whose points all lie under tier-0 roots).  M2M is linear, so a
    // rank forms its own roots' share of every upper multipole in phase 1: per partial
    // task -- its roots under one node A two levels above them -- the mid level, A,
    // and A's contribution to each ancestor up to xUpTop, the topmost level any M2L
    // reads.  Every rank receives every rank's records and sums each node's in a fixed
    // order (rank, record), so phase 2 runs no up tier and every cluster starts at
    // once; the level-L0 roots an M2L reads travel as multipole rows (xNeedNodes).
    // Task record (kUpTaskInts ints): [0, 16) root at slot 4 q1 + q0 (-1 none), [16, 20)
    // record of mid q1, [20] record of A, [21] chain length, [22, 30) chain quadrants
    // (A's, then its parent's ...), [30, 38) chain records (-1: a level no M2L reads).
    static constexpr int kUpTaskInts = 40;
    static constexpr int kUpChainMax = 8;
    bool xUpPartialIn = true;  // input: ANISO_UPPER_PARTIAL
    bool xUpPartial = false;
    int xUpTop = 0;
    std::vector<int> xUpTask;
    std::vector<int> xUpRecNode;  // per record of this rank: its upper node
    // the partial tasks as tails of the bottom tier: per xOwnT0Tasks entry {16 p + q
    // (its root is slot q of partial task p; -1: none), its root node}, and per partial
    // task its root count
    std::vector<int> xT0Part, xUpRoots;

    void build(const Tree& t, int np, int rank, int nranks);
    // the exchange plan above; sz / d2: the square grid of the correction stencil
    void buildExchange(const Tree& t, int sz, int d2);
    // hmClWait (after build and buildExchange)
    void buildTopWait(const Tree& t);

  private:
    void buildUpTasks(const Tree& t);
    void buildClusters(const Tree& t);
    void buildDownTasks(const Tree& t);
    void buildNearHs(const Tree& t, const std::vector<int>& leafIdx);
    void buildNearUp(const Tree& t);
};

std::vector<int64_t> shard_cuts(const Tree& t, int nranks);

// Small per-mode tables for the correction stencil (nearRemoval + refineAddOn,
// KernelFactory.cpp:445-478, 662-709) and the singular add-on moments
// (KernelFactory.cpp:828-860).  See DESIGN.md "Corrections".
struct CorrTables {
    std::vector<double> C;        // d2 (target) x 9 (3x3 squares) x d2 (source)
    std::vector<double> mu;       // d2 x d x d singular moments
    std::vector<double> legB;     // d x d x d : beta_{n,a} polynomial coefficients in X
    std::vector<double> coefScale;// d2: 1/lnorm
    void build(const Geometry& g, int mode);
};

double legendre_tr1(unsigned l, double x);  // std::tr1::legendre restated
void gauss_rule(int deg, double* x, double* w);

}  // namespace aniso
