/* uno_kkt_debug.h -- diagnostics of the MI355X KKT backend (not part of the Uno plugin boundary).
 * With option "stamps" = 1 every factorization records, per front f, eight words
 * out[8f + 0..3] = s_memrealtime (100 MHz) at kernel entry / after assembly / after the pivot loop /
 * after write-out, out[8f+4] = pivot candidates examined, out[8f+5] = pivot steps. */
#ifndef UNO_KKT_DEBUG_H
#define UNO_KKT_DEBUG_H
#include <stdint.h>
#include "uno_kkt.h"
#ifdef __cplusplus
extern "C" {
#endif
/* Host-only symbolic analysis + subtree partition over `world` ranks (no device): per front its owner
 * (rank, or -1 = top front factored by rank 0) and assembly-tree parent.  Returns the number of fronts,
 * -nf if cap is too small, -1 on a bad pattern. */
int64_t uno_kkt_debug_partition(int64_t n, int64_t nnz, const int64_t* row, const int64_t* col, int world,
                                int32_t* owner, int32_t* parent, int64_t cap, int64_t* n_subtrees);
/* The multi-GPU gate of uno_kkt_analyze (host only): 1 if a group of `world` ranks would partition the
 * factorization (at least `world` subtrees and estimated efficiency >= min_efficiency), 0 if it would run
 * replicas; -1 on a bad pattern.  efficiency / n_subtrees (optional) receive the estimate. */
int uno_kkt_debug_partition_gate(int64_t n, int64_t nnz, const int64_t* row, const int64_t* col, int world,
                                 double min_efficiency, double* efficiency, int64_t* n_subtrees);
/* Host-only symbolic analysis: per front its order, fully-summed columns and assembly-tree level. */
int64_t uno_kkt_debug_fronts(int64_t n, int64_t nnz, const int64_t* row, const int64_t* col, int32_t* front_order,
                             int32_t* front_pivots, int32_t* front_level, int64_t cap);
int64_t uno_kkt_debug_stamps(uno_kkt_t handle, uint64_t* out, int64_t cap, int32_t* front_order,
                             int32_t* front_pivots, int32_t* front_level);
/* Option "solve_stamps" = 1: per front 8 words of the last dataflow solve, s_memrealtime (100 MHz) at
 * {start, dependency satisfied, values staged, published} of the forward (0..3) and backward (4..7) pass. */
int64_t uno_kkt_debug_solve_stamps(uno_kkt_t handle, uint64_t* out, int64_t cap);
/* The handle's current front structure (after any delay merges): per front order, pivots and level. */
int64_t uno_kkt_debug_front_info(uno_kkt_t handle, int32_t* front_order, int32_t* front_pivots, int32_t* front_level,
                                 int64_t cap);
/* Equilibration of the last factorization: the scaling s (by original index) and ||A_pre||_inf as the
 * library computed them (waits for the factorization).  Returns 0, or an error code. */
/* option comm_trace = 1: the attached transport's calls in order, 4 int64 per record (op, peer / root, bytes,
 * reduction op; op 0 send, 1 recv, 2 allreduce, 3 broadcast, 4 group_begin, 5 group_end, 6 order: recorded right
 * before every send / recv / collective with peer = 1 when the call is enqueued on the handle's main stream and
 * bytes = the bit mask of side streams holding factor launches not yet joined into it -- 1 / 0 is the stream
 * ordering after every producing launch).  Returns the number of records (-1: no traced transport); at most
 * cap / 4 are copied; clear != 0 starts a new trace. */
int64_t uno_kkt_debug_comm_trace(uno_kkt_t handle, int64_t* out, int64_t cap, int clear);
int uno_kkt_debug_scaling(uno_kkt_t handle, double* scale, double* anorm);
#ifdef __cplusplus
}
#endif
#endif
