/*
 * aniso_mi355x_dev.h -- development and test entries of libaniso_mi355x.so.
 *
 * Not part of the drop-in boundary (aniso_mi355x.h, the MEX plugin's ops and their
 * block / solve / batched / shard extensions): per-stage applies for stage parity,
 * tree / plan introspection, in-stream stage timing, the fused launch's timeline and
 * a loopback communicator for timing one rank's schedule on one GPU.  Same
 * conventions and error codes as aniso_mi355x.h.
 */
#ifndef ANISO_MI355X_DEV_H
#define ANISO_MI355X_DEV_H

#include "aniso_mi355x.h"

#ifdef __cplusplus
extern "C" {
#endif

/* apply restricted to the stages in `mask` (ANISO_STAGE_*), unscaled stages are
 * still multiplied by 1/(2 pi) like the full output; device pointers */
int aniso_mapping_stages_dev(aniso_handle h, const double *charge, int id, int mask, double *out, void *stream);
/* introspection of the exchange plan (each pointer may be NULL): the roots this rank
 * sends (info[6] node ids, send order), the all-gather slot -> node map (info[8] x
 * info[0], -1 = padding), the roots of the tier-0 tasks run here (info[5]) */
int aniso_shard_roots(aniso_handle h, int *send_nodes, int *recv_nodes, int *t0_roots);
/* development: a loopback communicator -- this rank's own part of the all-gather
 * copied into place, nothing sent or received -- to time one rank's schedule of an
 * N-GPU run on one GPU (tools/shard_time.py --native); its results are not the
 * sharded operator's */
int aniso_comm_init_loopback(aniso_handle h);
/* the same restricted to the stages in mask (ANISO_STAGE_*; the identity x is always there) */
int aniso_forward_f32_stages_dev(aniso_handle h, const float *x, int mask, float *y, void *stream);
/* ---- introspection (tests / benchmarks) ---- */
/* the one-collective exchange of aniso_block_op_sharded_dev:
 * info[0..4] = 1 if the shard layout allows it, the rank's own tier-0 tasks, the
 * multipoles below the tier-0 root level it receives, the input ranges and points
 * outside its range it receives (near field, corrections, upper-tier P2M) */
int aniso_shard_exchange_one(aniso_handle h, int64_t *info);
/* its input ranges: 2 x info[3] tree positions [b, e) */
int aniso_shard_one_halo(aniso_handle h, int64_t *ranges);
/* the upper multipoles as partial sums of the one-collective exchange (section 5,
 * round 5; ANISO_UPPER_PARTIAL=0 keeps the root records): info[0..5] = 1 if this
 * rank's plan forms them, its partial tasks, its records (one per upper node share
 * an M2L reads), the topmost level an M2L reads, the tier-0 root level, the roots
 * its tasks cover (= its own tier-0 roots) */
int aniso_shard_upper_partials(aniso_handle h, int64_t *info);
/* the node of each of this rank's records (info[2] ints, record order) */
int aniso_shard_upper_records(aniso_handle h, int *nodes);
int aniso_tree_size(aniso_handle h, int *nnodes, int *max_level);
/* per node ints[11*i ..]: parent, child0..3, level, slot, isLeaf, isEmpty, nSource, begin;
 * geom[4*i ..]: cx, cy, rx, ry */
int aniso_tree_nodes(aniso_handle h, int *ints, double *geom);
/* which: 0=U 1=V 2=W 3=X.  ptr has nnodes+1 entries; idx (may be NULL) ptr[nnodes] */
int aniso_tree_list(aniso_handle h, int which, int64_t *ptr, int *idx);
/* stats[0..25]: near entries, M2L entries, M2L pairs, leaves (owned), targets with
 * M2L work, tree nodes, max leaf size, N, then the symmetric storage actually
 * streamed per apply: stored near entries, stored M2L blocks, canonical M2L
 * pairs (partial slots), near partial entries; then 1 if the block operator runs
 * on the mode-shared (harmonic) caches, their stored M2L block count, the
 * harmonic M2L's clusters (0: per-target waves), its in-cluster pairs (one read
 * for both ends) and the E blocks it reads per block apply; then the bytes of the
 * fp32 operator caches (aniso_forward_f32_dev; 0 until its first call); then 1 if
 * the block operator's upper up tiers run inside the clustered M2L launch
 * (k_top_m2l_hc), else 0; then the cluster plan of a
 * block handle, available before setCoeff: its halo slots (cross-cluster partner
 * products, one read per stored block), the largest cluster + halo (LDS slots) and
 * the E blocks the clusters read per apply; then the applies re-run on the tier
 * launches after a hand-off time-out of the fused launch (the host-pointer block
 * operator and the block solve recover; device-pointer entries report it); then
 * the harmonic near field's symmetric U storage: its stored E entries and partner
 * partial entries (both 0 when it reads every near block directed); then the
 * sharded matvecs run through the one-collective exchange (section 5); then the
 * directed M2L pairs of the 16-right-hand-side MFMA operators (0 before their plan);
 * then the upper-tier tasks that waiting blocks of the fused top-of-tree launch
 * computed themselves after ANISO_TOP_SPIN_LIMIT polls (section 3.10); then the
 * one-collective matvecs that exchanged the upper multipoles as partial sums; then 1
 * if the block apply runs its near field on a side stream beside the up pass and the
 * M2L (a shard, or ANISO_OVERLAP=1), 0 if serially (one GPU's default); then 1 if
 * the serial block apply forms its bottom up tier inside the staged near field
 * (section 3.11; ANISO_NEAR_UP=0 keeps its own launch); then the staged near
 * field's 16-bit source-row entries, its correction-stencil row entries and the
 * bottom-tier nodes its up tail writes (bench.py's extended algorithmic bytes).
 * aniso_stats_n writes the first min(cap, *n) of them and sets *n to their count
 * (34 here); aniso_stats, the fixed-size form, writes the first 26 (stats must hold
 * 26 entries). */
int aniso_stats_n(aniso_handle h, int64_t *stats, int cap, int *n);
int aniso_stats(aniso_handle h, int64_t *stats);
/* per-stage device times (ms), averaged over every apply since aniso_set_timing(h, 1)
 * (HIP events recorded in-stream, 8 floats): exchange (between the two phases of a
 * sharded apply: the caller's root all-gather; 0 otherwise), up (weighted charges +
 * P2M/M2M tiers), m2l, gather (transposed M2L products), near, down (L2L/L2P tiers + transposed
 * near products), corr, total.  A block apply sums each stage over its mode terms.
 * aniso_set_timing(h, 2) records the m2l and near spans only (the others read 0):
 * fewer in-stream events inside a timed region.  Other levels: ANISO_ERR_INVALID. */
int aniso_set_timing(aniso_handle h, int on);
int aniso_stage_times(aniso_handle h, float *t8);
/* development: the per-block timeline of the last fused top-of-tree launch, recorded
 * when the process runs with ANISO_TOP_TRACE=1 (tools/top_trace.py); *n = its blocks,
 * rec (cap >= 0 blocks of 8 int64, may be NULL) = {start, waited, end (100 MHz ticks), hw id,
 * kind (-k: up tier k, else the cluster id), wait tier, targets, block reads} */
int aniso_top_trace(aniso_handle h, int64_t *rec, int64_t cap, int64_t *n);
/* device line integrals tau(a,b) of the current sigma_t for n segments
 * seg[4i..4i+3] = (x0, y0, x1, y1) (KernelFactory.cpp:67-166); host pointers */
int aniso_line_integrals(aniso_handle h, const double *seg, int n, double *out);

#ifdef __cplusplus
}
#endif
#endif
