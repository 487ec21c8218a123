// kernels.hpp -- device-side parameter block and kernel declarations.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace aniso {

constexpr int kNP = 4;          // Chebyshev order per dimension (np); rank = 16
constexpr int kRank = kNP * kNP;
constexpr int kMaxD = 6;        // quadRule supported on the GPU path

// Small read-only tables shared by all kernels of one operator (lives in HBM,
// served from L1/L2: a few KB).
struct Params {
    int sz, d, d2, nsq;
    double dx;
    double gx[kMaxD], gw[kMaxD];            // volume Gauss rule (line integral)
    double cheb[kNP];                       // -cos((i+1/2) pi / np)
    double tnode[kNP * kNP];                // T_l(c_i) at [i + l*np]
    double R[4][kRank * kRank];             // M2M / L2L transfer, col-major
    double interp[kMaxD * kMaxD * kMaxD * kMaxD];  // d2 x d2 col-major
    double sqrtW[kMaxD * kMaxD];
    double coefScale[kMaxD * kMaxD];        // 1 / legendreNorms
    double legB[kMaxD * kMaxD * kMaxD];     // Taylor-shifted Legendre coefficients
};

constexpr int kMaxRhs = 8;  // right-hand sides of one batched apply

// One mode term of a batched apply (device-side table, one entry per term): the
// mode's cached operators and its K x K mix (rhs i = sum_b mix[i][b] base b).
struct ModeArgs {
    const double* Km2l;   // stored M2L blocks (column-major 16 x 16)
    const double* Knear;  // near-field blocks
    const double* C;      // stencil weights (d2 x 9 x d2)
    const double* mu;     // singular moments
    double sgn;           // (-1)^m: K_{B<-A} = sgn K_{A<-B}^T
    double pad;
    double mix[kMaxRhs][kMaxRhs];
};

// Harmonic weights of a block apply (harmonic.hip): the mixes of
// aniso.m's forward / mforward, out_i = sum_j w_|j| K_|i+j| x_|j|, as hw_b = w_0
// (b = 0) or 2 w_b, dw_i = the mode-0 (diagonal) weight of output i, and om_i = 0
// for an output the mixes leave empty (a padded right-hand side).
struct HarmWeights {
    double hw[kMaxRhs];
    double dw[kMaxRhs];
    double om[kMaxRhs];
};

enum StageMask : int {
    kStageFar = 1,      // M2L + L2L + L2P (both kernels)
    kStageNear = 2,     // U/W near field (both kernels)
    kStageStencil = 4,  // nearRemoval + refineAddOn
    kStageSing = 8,     // singularAddOn
    kStageAll = 15,
    kStageForward = 16,  // 16-RHS fp64 operator (f64op.hip): Y = X - K (sigma_s X) instead of Y = K X
};

constexpr int kTierThreads = 256;  // workgroup of the down pass tasks
// up pass tasks: 256 threads (P2M holds 16 products per lane, ~94 VGPRs = 5 waves
// per SIMD), so four workgroups fit per CU and 1,024 tasks run in one round
constexpr int kUpThreads = 256;

// ---- apply kernels (apply.hip), batched over K right-hand sides.
// K is a runtime argument dispatched to compiled instances (rhs_supported); the
// operator pads other counts with zero right-hand sides (rhs_padded).  Vectors are
// [K][ld] (rhs-major); tree-order work arrays fT/cT are [N][K], expansions
// [node][16][K].  `mix` is a K x K row-major matrix: the kernels of one mode
// apply it to the base inputs on the fly (rhs i = sum_b mix[i][b] base b).
bool rhs_supported(int k);
int rhs_padded(int k);  // smallest supported count >= k, or -1
int rhs_stride(int k);  // row stride (doubles) of the tree-order charge arrays fT / cT
void launch_prepare(int K, int64_t N, const double* xin, int64_t ldi, int treeIn, const int* perm,
                    const double* sigT, const double* wT, double* fT, double* cT, hipStream_t s);
size_t up_tier_lds(int maxTask, int K);
size_t down_tier_lds(int maxTask, int maxLeaves, int maxNear, int maxChain, int K);
// taskList (nullptr: tasks taskBase .. taskBase + ntask - 1): the tasks to run.
// Sharded applies (all may be null): rootSlot / recv -- children that
// are tier-0 roots with a slot are read from the all-gathered records recv (and
// stored to mult for the M2L); sendSlot / send -- a task root with a send slot also
// stores its record into this rank's all-gather buffer.
// The upper multipoles' partial tasks (Plan::xUpTask) as tails of the sharded
// bottom tier: block b's task root (node partOf[b].y) is slot q of
// partial task p (partOf[b].x = 16 p + q; -1: none).  The block copies its root
// multipole write-through into stage[16 p + q]; the last of a partial task's
// nroots[p] roots to finish (an agent-scope counter, cnt[p], reset by that block)
// runs it from the staged roots, storing its records into rec and into each of nPeer
// parts at peerOff (doubles into buf, the exchange's send buffer).
struct UpTail {
    const int2* partOf = nullptr;
    double* stage = nullptr;
    unsigned* cnt = nullptr;
    const int* nroots = nullptr;
    const int* task = nullptr;
    double* rec = nullptr;
    int nPeer = 0;
    const int64_t* peerOff = nullptr;
    double* buf = nullptr;
};
void launch_up_tier(int K, int ntask, int taskBase, const int* taskList, int maxTask, const int4* desc,
                    const int* grpFix, const int* node, const int4* code, const double4* geom, const int2* leafRange,
                    const double* pxT, const double* pyT, const double* xin, int64_t ldi, int treeIn, const int* perm,
                    const double* sigT, const double* wT, double* fT, double* cT, const Params* P, double* mult,
                    const int* rootSlot, const double* recv, const int* sendSlot, double* send, hipStream_t s,
                    unsigned* zeroCnt = nullptr, const UpTail* tail = nullptr);
// config 5's fp32 operator (f32op.hip): node expansions as 64 lanes x float4
// (void* below), vectors point-major N x 16 floats
void launch32_p2m(int nleaf, const int* leaves, const int64_t* begin, const int64_t* count, const double* ncx,
                  const double* ncy, const double* nrx, const double* nry, const double* pxT, const double* pyT,
                  const float* X, const double* sigT, const double* wT, const Params* P, void* mult, float* fT,
                  float* cT, hipStream_t s);
void launch32_m2m(int nn, const int* nodes, const int4* child, const int64_t* count, const void* Rup, void* mult,
                  hipStream_t s);
void launch32_m2l(int ntgt, const int* tgt, const int64_t* ptr, const int* src, const void* K32, const void* mult,
                  void* local, hipStream_t s);
void launch32_l2l(int nn, const int* nodes, const int* parent, const int* slot, const void* Rdn, void* local,
                  hipStream_t s);
void launch32_leaf(int nleaf, const int4* leafInfo, const int64_t* nearPtr, const int* nearPts, const int64_t* koff,
                   const void* Knear, const int* level, const double* ncx, const double* ncy, const double* nrx,
                   const double* nry, const double* pxT, const double* pyT, const Params* P, const void* local,
                   const float* fT, const float* X, float scale, int flags, float* Y, hipStream_t s);
void launch32_corr(int d, int64_t N, const int* perm, const int* iperm, const float* cT, const float* fT,
                   const double* C, const double* mu, const Params* P, int flags, float scale, float* Y,
                   hipStream_t s);
void launch32_conv_m2l(int64_t npairs, const double* Kd, void* K32, hipStream_t s);
void launch32_conv_near(int nl, const int4* info, const int64_t* koffD, const int64_t* koff, const int* srcCount,
                        const double* Kd, void* K32, hipStream_t s);
// the fp64 16-right-hand-side operator on MFMA (f64op.hip): the same plan and
// layouts as the fp32 one, expansions as 64 lanes x 4 doubles
void launch64_p2m(int nleaf, const int* leaves, const int64_t* begin, const int64_t* count, const double* ncx,
                  const double* ncy, const double* nrx, const double* nry, const double* pxT, const double* pyT,
                  const double* X, const double* sigT, const double* wT, const Params* P, void* mult, double* fT,
                  double* cT, hipStream_t s);
void launch64_m2m(int nn, const int* nodes, const int4* child, const int64_t* count, const void* Rup, void* mult,
                  hipStream_t s);
void launch64_m2l(int ntgt, const int* tgt, const int64_t* ptr, const int* src, const void* K64, const void* mult,
                  void* local, hipStream_t s);
void launch64_l2l(int nn, const int* nodes, const int* parent, const int* slot, const void* Rdn, void* local,
                  hipStream_t s);
void launch64_leaf(int nleaf, const int4* leafInfo, const int64_t* nearPtr, const int* nearPts, const int64_t* koff,
                   const void* Knear, const int* level, const double* ncx, const double* ncy, const double* nrx,
                   const double* nry, const double* pxT, const double* pyT, const Params* P, const void* local,
                   const double* fT, const double* X, double scale, int flags, double* Y, hipStream_t s);
void launch64_corr(int d, int64_t N, const int* perm, const int* iperm, const double* cT, const double* fT,
                   const double* C, const double* mu, const Params* P, int flags, double scale, double* Y,
                   hipStream_t s);
void launch64_lane_major(int64_t npairs, double* K, hipStream_t s);
void launch64_conv_near(int nl, const int4* info, const int64_t* koffD, const int64_t* koff, const int* srcCount,
                        const double* Kd, void* K64, hipStream_t s);
void launch64_gather16(int64_t N, int k, const int* perm, const double* Q, double* X16, hipStream_t s);
void launch64_scatter16(int64_t N, int k, const int* perm, const double* Y16, double* Out, hipStream_t s);
// the tier-0 root records of a sharded apply without upper tiers, scattered back
// from the all-gather (mult[nodes[j]] = recv[j] where nodes[j] >= 0)
void launch_roots_unpack(int K, int nslots, const int* nodes, const double* recv, double* mult, hipStream_t s);
// All terms in one launch: local = sum over the terms (stored), transposed
// canonical products summed over the terms into their partial slots (stored).
void launch_m2l(int K, int ntgt, const int* tgt, const int64_t* ptr, const int* nDir, const int* canonBase,
                const int* outSlot, const int* src, const ModeArgs* tab, int nterm, const double* mult, int maxCanon,
                double* partial, double* local, hipStream_t s);
void launch_m2l_gather(int K, int ntgt, const int* tgt, const int* inPtr, const double* partial, double* local,
                       hipStream_t s);
// Output index mode of k_near / k_down_tier / k_corr: operm = perm writes the
// original-order vector out[perm[k]]; operm = nullptr writes the owned tree-order
// slice out[k - obase].  ldo = the stride between right-hand sides of out.
// near field with symmetric U storage (K = 1 handles): partial products to `partial`
void launch_near_sym(int K, int nl, const int4* leafInfo, const int64_t* nearPtsPtr, const int* nearPts,
                     const int64_t* nearKOff, const int2* nearSym, const double* Kop, const double* fT,
                     const double* mix, const int* operm, int64_t obase, int64_t ldo, int maxS, int flags, double sgn,
                     double scale, int accum, double* partial, double* out, hipStream_t s);
// near field with directed storage, all terms in one launch (out stored, or added
// with accum); maxLeaf = the largest target leaf (points)
void launch_near(int K, int nl, int maxLeaf, const int4* leafInfo, const int64_t* nearPtsPtr, const int* nearPts,
                 const int64_t* nearKOff, const ModeArgs* tab, int nterm, const double* fT, const int* operm,
                 int64_t obase, int64_t ldo, int flags, double scale, int accum, double* out, hipStream_t s);
void launch_down_tier(int K, int ntask, int maxTask, int maxLeaves, const int4* desc, const int* grpFix,
                      const int4* dn, const double* local, const Params* P, const int* leafSlot, const int* leafBegin,
                      const int2* leafNear, const double4* leafGeom, const double* pxT, const double* pyT,
                      const int* operm, int64_t obase, int64_t ldo, const int* nearOff, int maxNear,
                      const double* nearPart, const int2* chain, int maxChain, int flags, double scale, double* out,
                      const double* xsub, int64_t ldx,
                      hipStream_t s, const double* hpart = nullptr, const int* chainFold = nullptr);
// corrections of all terms in one launch, added to out: Wc / Wm the terms'
// stencil and singular tables folded with their mixes (Operator::corrTable)
void launch_corr(int K, int d, int64_t b, int64_t e, const int* perm, const int* iperm, const double* cT,
                 const double* fT, const double* Wc, const double* Wm, const Params* P, int flags, double scale,
                 bool treeOut, int64_t ldo, double* out, hipStream_t s);
// harmonic block apply (harmonic.hip): all modes from the mode-shared E caches
void launch_m2l_hm(int K, int ntgt, const int* tgt, const int64_t* ptr, const int* src, const int* blk, const double* E,
                   const double* ncx, const double* ncy, const double* nrx, const double* nry, const Params* P,
                   const HarmWeights& hw, const double* mult, double* local, hipStream_t s);
// the clustered M2L's arguments (harmonic.hip k_m2l_hc, k_top_m2l_hc)
struct HcArgs {
    const int* clPtr;
    const int* tgt;
    const int64_t* ptr;
    const int* ndir;
    const int* src;
    const int* blk;
    const int* slot;
    const double* E;
    const double* ncx;
    const double* ncy;
    const double* nrx;
    const double* nry;
    const Params* P;
    HarmWeights hw;
    const double* mult;
    double* local;
    const double* geo = nullptr;  // per node {cx, cy, rx, ry} (the ring form, k_m2l_hcr)
    int ring = 0;                 // host: the ring form's depth (0: the one-block-in-flight form)
    bool ringXL = false;          // host: the ring form keeps the target multipole in LDS (3 waves / SIMD)
    int wpe = 0;                  // host: the cluster form's occupancy (harmonic.hip hm_form; 0: the default)
    // the halo form (Plan::hmHaloPtr): cluster c's halo slots h = haloPtr[c] ..
    // haloPtr[c+1] - 1 go to partial haloPos[h] of hpart (16 x K doubles each, stored
    // scaled, receiver-contiguous: the down pass adds them to the locals)
    const int* haloPtr = nullptr;
    const int* haloPos = nullptr;
    double* hpart = nullptr;
    // the deterministic sums (k_m2l_hc only): per node the bound W of
    // its weighted multipole (k_node_wmax), per cluster the host's geometric bound, the
    // largest stored E (device scalar).  wmax == nullptr: the ds_add_f64 sums
    const double* wmax = nullptr;
    const double* clBound = nullptr;
    const double* emax = nullptr;
};
// The fused top-of-tree + clustered M2L launch (harmonic.hip k_top_m2l_hc, DESIGN.md
// §3.10): blocks 0 .. nUp - 1 run the up tasks of tiers 1 .. ntier - 1 (tier k's
// tasks wait until tier k - 1 has finished), the other blocks are the clusters, a
// cluster whose sources include upper-tier multipoles waiting for that tier.
constexpr int kMaxTopTiers = 8;
struct UpArgs {  // one up task's inputs (up_task.hpp)
    int maxTask;
    const int4* desc;
    const int* grpFix;
    const int* node;
    const int4* code;
    const double4* geom;
    const int2* leafRange;
    const double* pxT;
    const double* pyT;
    const double* xin;
    int64_t ldi;
    int treeIn;
    const int* perm;
    const double* sigT;
    const double* wT;
    double* fT;
    double* cT;
    const Params* P;
    double* mult;
    const int* rootSlot;
};
struct TopArgs {
    int nUp;                      // up-task blocks
    int ntier;                    // tiers 1 .. ntier - 1 run in the launch
    int blk0[kMaxTopTiers + 1];   // first block of tier k; blk0[ntier] = nUp
    int task0[kMaxTopTiers];      // first task of tier k
    const int* clWait;            // per cluster: the upper tier it waits for (0: none)
    unsigned* cnt;                // finished tasks per tier (zeroed by tier 0)
    const double* recv1;          // sharded phase 2: the gathered tier-0 roots tier 1 reads
    unsigned spinLimit;           // polls of a tier's counter before the waiting block computes the tier itself
                                  // (0: at once -- tests only)
    unsigned* steals;             // persistent count of tier tasks computed by a waiting block (aniso_stats)
    unsigned* err;                // host-visible sticky flag (kept for the ABI; the launch no longer sets it)
    int64_t* trace;               // development (ANISO_TOP_TRACE=1): per block {start, waited, end, hw id}
    int nCl;                      // cluster blocks (set by the launcher); near-field groups follow them
};
// the fused corrections of the staged near field (d = 1; harmonic.hip k_near_hs)
struct NearCorr {  // the fused corrections of k_near_hs (d = 1), or ignored when rows == nullptr
    const uint16_t* rows;
    const int* perm;
    const int* iperm;
    const double* cT;
    const double* Wc;
    const double* Wm;
    const Params* P;
};
// the staged near field's arguments (harmonic.hip k_near_hs, and the last blocks of
// k_top_m2l_hc when the near field rides in that launch): 16 leaves per group
struct NearHsArgs {
    int nl;                  // target leaves
    int nsMax;               // largest source table (rows)
    const int4* leafInfo;
    const int64_t* nearPtsPtr;
    const uint16_t* nearLoc;
    const int64_t* nsPtr;
    const int* nsPts;
    const int64_t* nearKOff;
    const double* E;
    const double* pxT;
    const double* pyT;
    const double* sigDiag;
    HarmWeights hw;
    const double* fT;
    const int* operm;
    int64_t obase;
    int64_t ldo;
    int flags;
    double scale;
    double* out;
    NearCorr nc;
    // charges from the apply's input (xin != nullptr): f = x sigma_s w and c = x
    // sigma_s formed here (as up_task does), so the near field needs nothing from the
    // up pass and can run beside it; else fT / cT (and nc.cT) as the up pass wrote them
    const double* xin = nullptr;
    int64_t ldi = 0;
    int treeIn = 0;
    const int* perm = nullptr;
    const double* sigT = nullptr;
    const double* wT = nullptr;
    // symmetric U storage (Plan::nearSymHsOn; colDst == nullptr: every column
    // directed): per leaf (directed columns, all columns), per column where its
    // partner product goes, the leaf's first table row; partials of other groups
    const int2* nearSym = nullptr;
    const int* colDst = nullptr;
    const uint16_t* selfRow = nullptr;
    double* nearPart = nullptr;
    // the in-group partner products' LDS slots (Plan::nearGrpIn): per leaf the slots
    // it receives, and the most slots of a group (the launch's LDS)
    const int* grpInPtr = nullptr;
    const int* grpIn = nullptr;
    int grpSlots = 0;
    // the 16-leaf groups to run (ngrp of them; nullptr: all, in order): a sharded
    // apply's one-collective form runs the groups that read only the own range before
    // the exchange and the rest after it (Plan::nearGrpEarly / nearGrpLate)
    const int* grpList = nullptr;
    int ngrp = 0;
    // the bottom up tier in the staged near field (one GPU, serial schedule;
    // Plan::nearUpGrp): every 16-leaf group is one tier-0 subtree (its
    // 16 leaves, their 4 parents, the root).  Its lanes form the leaves' P2M from the
    // charges the epilogue loads, the workgroup the subtree's M2M, into upMult (the
    // multipoles of an up tier; the tier launch is skipped).  upGrp: per group
    // kNearUpInts ints -- per leaf (parent slot << 2 | quadrant), per parent its
    // quadrant, the 4 parent nodes, the root node.  zeroCnt: the fused top-of-tree
    // launch's counters, zeroed here instead of by the skipped tier launch.
    double* upMult = nullptr;
    const int* upGrp = nullptr;
    const Params* upP = nullptr;
    const double* upNcx = nullptr;
    const double* upNcy = nullptr;
    const double* upNrx = nullptr;
    const double* upNry = nullptr;
    unsigned* zeroCnt = nullptr;
};
constexpr int kNearUpInts = 25;
// LDS the fused up tail needs in the group's table region (doubles): 256 points x
// (8 Chebyshev weights + K charges), then the 4 parents' 16 x K
inline size_t near_up_lds_doubles(int K) { return (size_t)256 * (8 + K) + 4 * 16 * K; }
bool top_fused_enabled();
// near: the staged near field with its corrections fused (near_hs_fusable) as the
// launch's last blocks, or nullptr (it runs as a launch of its own)
void launch_top_m2l_hc(int K, int ncl, int maxCl, const UpArgs& u, const TopArgs& t, const HcArgs& a,
                       const NearHsArgs* near, hipStream_t s);
// whether launch_near_hm would run the staged near field with fused corrections
bool near_hs_fusable(int nl, int maxLeaf, int nsMax, const uint16_t* nearLoc, const NearCorr* corr, int flags);
void launch_m2l_hc(int K, int ncl, int maxCl, const HcArgs& a, hipStream_t s);
// the deterministic cluster sums' bounds: out[n] = max over node n's 16 columns of
// sum_b |hw_b mult_b|; out[0] = max |x|
void launch_node_wmax(int K, int nnodes, const double* mult, const HarmWeights& hw, double* out, hipStream_t s);
void launch_abs_max(int64_t n, const double* x, double* out, hipStream_t s);

int hm_ring_depth();  // ANISO_HM_RING (read at handle creation): the cluster M2L's LDS ring depth
int hm_ring_xl(int K, int maxCl, int depth);  // its target multipole in LDS / VGPRs / ring off (1, 0, -1)
// returns true when the corrections were fused (the caller skips launch_corr)
bool launch_near_hm(int K, int nl, int maxLeaf, const int4* leafInfo, const int64_t* nearPtsPtr, const int* nearPts,
                    const int64_t* nearKOff, const double* E, const double* pxT, const double* pyT,
                    const double* sigDiag, const HarmWeights& hw, const double* fT, const int* operm, int64_t obase,
                    int64_t ldo, int flags, double scale, double* out, const uint16_t* nearLoc, const int64_t* nsPtr,
                    const int* nsPts, int nsMax, const NearCorr* corr, int wpe, hipStream_t s,
                    const NearHsArgs* in = nullptr);  // in->xin: the staged kernel's charges from the input
void launch_sub_slice(int64_t n, int nrhs, const double* x, int64_t ldx, const double* a, int64_t lda, double* y,
                      int64_t ldy, hipStream_t s);

// ---- cache build and helpers (kernels.hip)
void launch_cache_m2l(int64_t npairs, const int* pairTgt, const int* src, const double* ncx, const double* ncy,
                      const double* nrx, const double* nry, const double* stcoef, const Params* P, int mode,
                      double* K, hipStream_t s);
void launch_cache_near(int nl, const int* leaves, const int64_t* nearPtr, const int* nearSrc, const int64_t* nearKOff,
                       const int64_t* begin, const int64_t* count, const double* pxT, const double* pyT,
                       const double* stcoef, const Params* P, int mode, int maxSrc, double* K, hipStream_t s);
// mode-shared cache: pair_kernel's mode argument kAttMode gives
// e^-tau alone (0 at r = 0); launch_cache_near takes it as well
constexpr int kAttMode = -1;
void launch_cache_att_m2l(int64_t npairs, const int* pairTgt, const int* src, const double* ncx, const double* ncy,
                          const double* nrx, const double* nry, const double* stcoef, const Params* P, double* E,
                          hipStream_t s);
void launch_sigma_diag(int64_t N, const double* pxT, const double* pyT, const double* stcoef, const Params* P,
                       double* out, hipStream_t s);
void launch_permute(int64_t N, const int* perm, const double* orig, double* tree, hipStream_t s);
// halo exchange of an nb-block vector (comm.hpp): element j of a position list goes
// to / comes from buf[base[j] + b * stride[j]] for block b, vector entry x[b * ldx + pos[j]]
void launch_halo_pack(int64_t n, int nb, const int64_t* pos, const int64_t* base, const int64_t* stride,
                      const double* x, int64_t ldx, double* buf, hipStream_t s);
void launch_halo_unpack(int64_t n, int nb, const int64_t* pos, const int64_t* base, const int64_t* stride,
                        const double* buf, double* x, int64_t ldx, hipStream_t s);
// the one-collective exchange's pack (send) or unpack (receive) in one launch: root
// records (nRoot parts of rec doubles at rootOff in buf; unpack: to rootDst in roots,
// and this rank's own record from ownRoots), input positions (pos / base / stride as
// the halo exchange, nb blocks of x), multipole rows (node / nodeBase, len doubles)
struct OxArgs {
    int64_t nRoot = 0, rec = 0;
    const int64_t* rootOff = nullptr;
    const int64_t* rootDst = nullptr;
    double* roots = nullptr;           // pack: this rank's records (read); unpack: the slot layout (written)
    const double* ownRoots = nullptr;  // unpack: this rank's records, copied to its own slot
    int64_t ownDst = 0;
    int64_t nPts = 0;
    int nb = 0;
    const int64_t* pos = nullptr;
    const int64_t* base = nullptr;
    const int64_t* stride = nullptr;
    double* x = nullptr;
    int64_t ldx = 0;
    int64_t nNode = 0;
    int len = 0;
    const int* node = nullptr;
    const int64_t* nodeBase = nullptr;
    double* mult = nullptr;
    double* buf = nullptr;
    // unpack, the upper multipoles as partial sums (Plan::xUpPartial): node sumNode[j]
    // = the sum of its records sumSrc[sumPtr[j] .. sumPtr[j + 1]) in that order (>= 0:
    // offset into buf, < 0: ~offset into ownRec), len doubles each
    int64_t nSum = 0;
    const int* sumNode = nullptr;
    const int* sumPtr = nullptr;
    const int64_t* sumSrc = nullptr;
    const double* ownRec = nullptr;
};
void launch_ox(const OxArgs& a, bool pack, hipStream_t s);
void launch_spin_us(int us, int blocks, hipStream_t s);  // development: a stand-in exchange latency
// the pack launch with the upper multipoles as partial sums (apply.hip k_ox_pack_up):
// one workgroup per task of Plan::xUpTask (kUpTaskInts ints each) stores its records
// into rec and into each of nPeer parts at peerOff (doubles into a.buf), the rest pack
// a's input positions and multipole rows (a.nRoot must be 0)
void launch_ox_pack_up(int K, int ntask, const int* task, const double* mult, const Params* P, double* rec,
                       int nPeer, const int64_t* peerOff, const OxArgs& a, hipStream_t s);


// host-callable device helpers used by tests through the C ABI
void launch_line_integrals(int n, const double* seg, const double* stcoef, const Params* P, double* out,
                           hipStream_t s);

}  // namespace aniso
