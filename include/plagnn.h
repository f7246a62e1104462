/*
 * plagnn.h — C-ABI of the MI355X-native message-passing engine for PLA-GNN.
 *
 * This is the drop-in boundary for the reference's hot path. The reference
 * (quinlanW/PLA-GNN) reaches its message passing only through DGL 0.8.2's
 * Python API; every entry point below replaces one native operation that
 * DGL/torch runs underneath the reference's call sites:
 *
 *   pg_csr_from_coo      <- dgl.graph((start, end), num_nodes=N) + dgl.add_self_loop
 *                           and DGL's lazy COO->CSC (in-CSR) build
 *                           (code/utils.py:44-45, first update_all at code/model.py:20)
 *   pg_csr_transpose     <- DGL's reverse-graph CSR used by GSpMM.backward
 *   pg_spmm_max_fwd      <- update_all(copy_u('h','m'), max('m','neigh')) inside
 *                           SAGEConv(..., 'pool')  (code/model.py:13-15, 20, 22, 24)
 *                           = DGL SpMMCmpCsr<copy_lhs, Max> (argmax recorded)
 *   pg_spmm_max_bwd      <- DGL GSpMM.backward, copy_lhs/max branch:
 *                           dX = zeros; dX.scatter_add_(0, argX, dZ)   (reached from
 *                           train_loss.backward(), code/train.py:204), fused with the
 *                           relu' mask of fc_pool's activation
 *   pg_spmm_max_bwd_scatter  same, in DGL's scatter form (float atomics)
 *   pg_spmm_sum          <- update_all(copy_u / u_mul_e, sum|mean) (SAGEConv 'mean',
 *                           GraphConv, edge_weight=...) and their backward on the
 *                           transposed CSR. Not run by the reference: reference-unpinned.
 *   pg_argpos_to_src     <- DGL's argX (source node id of the max) from our compact
 *                           per-row edge positions
 *   pg_sigmoid_multi_loss<- th.sigmoid (code/model.py:29) + multi_loss
 *                           (code/train.py:89-108) forward and backward
 *   pg_mlp_head          <- liner2 + sigmoid + multi_loss (train and val) + their backward
 *                           down to liner1's activation (code/model.py:28-29), fused
 *   pg_adam_*            <- torch.optim.Adam(model.parameters(), lr) .step()
 *                           (code/train.py:180, 205), torch 1.10 formula
 *   pg_bias_act[_bwd]    <- nn.Linear bias add + F.relu / F.leaky_relu(0.01)
 *                           (code/model.py:21-27), fused
 *   pg_col_sum           <- bias gradients (sum of dY over nodes)
 *   pg_gemm_f32          <- nn.Linear GEMMs (fc_pool / fc_self / fc_neigh / liner1-2),
 *                           f32 in / f32 out with f32 accuracy: aligned operands run as
 *                           three-piece bf16 splits on v_mfma_f32_32x32x16_bf16
 *                           (gemm_x3.hip), the rest on v_mfma_f32_32x32x2_f32 (gemm.hip)
 *   pg_gemm_f32_cat      <- fc_self(h) + fc_neigh(h_neigh) (code/model.py:13-15) as one
 *                           product over two K pieces, and its input gradient
 *   pg_gemm_*_group      <- a step's weight-gradient GEMMs (code/train.py:204), one launch
 *   pg_pad2d_group       <- the drop-in SAGEConv's zero-padded weight images (503 -> 512)
 *   pg_gemm_bf16,        <- the same layers and aggregation in the bf16-storage mode
 *   pg_spmm_max_*_bf16      (BASELINE configs[4]: bf16 storage, f32 accumulate); not run
 *   pg_cast_*               by the reference (fp32 only): reference-unpinned
 *   pg_ecc               <- edge_clustering_coefficients (code/data_preprocess.py:175-214),
 *                           the ECC feature / edge-weight front end
 *   pg_loc_correction,   <- protein_loc_correction / performances_record
 *   pg_loc_performance      (code/train.py:19-86), the per-epoch eval
 *   pg_csr_spmm_f64      <- the centred products of pca() (code/data_preprocess.py:475-487,
 *                           scikit-learn 1.1.1 randomized PCA), the PCA front end
 *   pg_perturb_*         <- construct_gcn_matrix's np.corrcoef (code/data_preprocess.py:
 *                           165-170) + modify_network_topology (217-257), fused: the
 *                           N x N correlation / difference matrices are never stored
 *
 * Conventions
 *   - All buffers are caller-owned. Device entry points take device pointers and
 *     enqueue asynchronously on `stream` (a hipStream_t; NULL = default stream);
 *     they never allocate, copy to host or synchronise, so they can be captured
 *     into a HIP graph. Scratch comes from the caller through (ws, ws_bytes),
 *     sized by the matching *_workspace() query.
 *   - Host entry points (pg_csr_*, pg_schedule_*) take host pointers.
 *   - Dense matrices are row-major with an explicit leading dimension (elements).
 *   - Return 0 on success, a negative PG_ERR_* code for an argument error, or a
 *     positive hipError_t for a launch error. pg_last_error_string() gives a
 *     thread-local message for the last failure. No C++ exception crosses the ABI.
 *   - Entry points suffixed _cpu are the same operations on host pointers (OpenMP)
 *     for tensors the caller keeps on the CPU device (DGL's CPU backend role,
 *     main_normal.py -d cpu). They are never used as a fallback for a GPU call.
 */
#ifndef PLAGNN_H
#define PLAGNN_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* pg_stream_t; /* hipStream_t */

#define PG_OK 0
#define PG_ERR_INVALID (-1)     /* bad argument / shape */
#define PG_ERR_UNSUPPORTED (-2) /* valid but not implemented for these arguments */
#define PG_ERR_WORKSPACE (-3)   /* ws_bytes smaller than the *_workspace() query */
#define PG_ERR_HOST (-4)        /* host-side failure (allocation, ...) */

/* element type of the per-(row, feature) argmax record */
#define PG_ARG_U16 16 /* position of the winning edge inside its row, 0xFFFF = none */
#define PG_ARG_I32 32 /* same, int32, -1 = none (rows with degree >= 65535) */
/* flag OR-ed into arg_kind of pg_spmm_max_fwd[_bf16] / pg_spmm_max_bwd[_bf16] (ABI 6): the
 * forward records "none" where the maximum is 0 (not DGL's argX there: for relu inputs
 * whose gradient the relu' mask removes anyway); the backward then skips those entries
 * as fwd_out would, without reading fwd_out, and takes mask_src (required, X >= 0) as
 * implied. The other record consumers take the plain kind. */
#define PG_ARG_DEAD_NONE 0x100

/* activation codes for pg_bias_act / pg_gemm_f32 epilogues */
/* storage types of pg_gemm_bf16's output */
#define PG_DTYPE_F32 0
#define PG_DTYPE_BF16 1

#define PG_ACT_NONE 0
#define PG_ACT_RELU 1
#define PG_ACT_LEAKY 2 /* F.leaky_relu, negative_slope given separately */

/*
 * A compressed sparse row view of one graph direction plus its launch schedule.
 * For the in-CSR (DGL's CSC): rows = destination nodes, col = source node ids,
 * entries of a row in ascending edge id (the order DGL reduces them in).
 * For its transpose (out-CSR): rows = source nodes, col = destination ids in
 * ascending order, eslot = the in-CSR slot j of the same edge, epos = j - ptr_in[col]
 * (the edge's position inside its in-CSR row, which is what argmax records hold).
 * Work schedule (built by pg_schedule_build): items {row, k0, k1, slot} cover every
 * row; a row longer than `chunk` entries is split into several items that write
 * partial results to `slot`; merges {row, first_slot, n_slots, 0} combine them.
 */
typedef struct pg_csr {
  int64_t n_rows;
  int64_t n_cols;
  int64_t nnz;
  const int32_t* ptr;    /* [n_rows + 1] */
  const int32_t* col;    /* [nnz] */
  const int32_t* eslot;  /* [nnz] or NULL (NULL: slot == k) */
  const int32_t* epos;   /* [nnz] transposed CSR: position inside the in-CSR row; in-CSR
                          * (optional, ABI 10): the transposed index of each slot, used by
                          * pg_spmm_max_bwd[_bf16] to store list descriptors where the pull
                          * reads them in order (NULL: at the slots) */
  const float* ew;       /* edge weights indexed by in-CSR slot, or NULL */
  const int32_t* items;  /* [4 * n_items] */
  int64_t n_items;
  const int32_t* merges; /* [4 * n_merges] */
  int64_t n_merges;
  int64_t n_slots;
  int32_t max_deg;
  int32_t chunk;
} pg_csr_t;

/* ---------------- host: graph construction (code/utils.py:44-45) ---------------- */

/* COO (src[e], dst[e]) -> in-CSR: ptr[n_dst+1], col[nnz] = src, eid[nnz] = edge id.
 * Stable counting sort by dst, so each row lists its edges in ascending edge id. */
int pg_csr_from_coo(const int64_t* src, const int64_t* dst, int64_t nnz, int64_t n_src,
                    int64_t n_dst, int32_t* ptr, int32_t* col, int32_t* eid);

/* Transpose: tptr[n_cols+1], tcol[nnz] = row ids ascending, tslot[nnz] = slot in the
 * input CSR, tpos[nnz] = tslot - ptr[tcol] (may be NULL). */
int pg_csr_transpose(const int32_t* ptr, const int32_t* col, int64_t n_rows, int64_t n_cols,
                     int64_t nnz, int32_t* tptr, int32_t* tcol, int32_t* tslot, int32_t* tpos);

/* Work schedule sizes for rows of `ptr` split at `chunk` entries. */
int pg_schedule_count(const int32_t* ptr, int64_t n_rows, int32_t chunk, int64_t* n_items,
                      int64_t* n_merges, int64_t* n_slots, int32_t* max_deg);
/* Fill items[4*n_items] and merges[4*n_merges] (both longest first). */
int pg_schedule_build(const int32_t* ptr, int64_t n_rows, int32_t chunk, int32_t* items,
                      int32_t* merges);

/* ---------------- device: message passing ---------------- */

/* out[v,f] = max_{k in row v} (ew? ew[k]:1) * X[col[k], f]  (strict >, first wins, start -inf);
 * argpos[v,f] = k - ptr[v] of the winner. Rows with no entries: out = 0, argpos = none.
 * A +-inf result is stored as 0 (DGL's replace_inf_with_zero after a max reduce).
 * Requires X, out 4-byte aligned; the vector path is taken when ldx, ldo, F are
 * multiples of 4 and the base pointers are 16-byte aligned. Rows the schedule splits are
 * combined in piece order (the earliest maximal entry wins); with a 256-byte aligned ws
 * (at least the query's bytes) inside the same launch, else by a second launch. */
size_t pg_spmm_max_fwd_workspace(const pg_csr_t* g, int64_t F, int arg_kind);
int pg_spmm_max_fwd(const pg_csr_t* g, const float* X, int64_t ldx, int64_t F, float* out,
                    int64_t ldo, void* argpos, int64_t lda, int arg_kind, void* ws,
                    size_t ws_bytes, pg_stream_t stream);

/* Deterministic backward (gather over the transposed CSR gt of g; gt->epos required):
 *   dx[u,f] = sum_{(v,j) in gt row u, ascending v} [argpos[v,f] == j - g.ptr[v]] * ew[j] * dout[v,f]
 * then, if mask_src != NULL, dx[u,f] *= (mask_src[u,f] > 0)  (relu' of fc_pool).
 * fwd_out (optional, needs mask_src = the forward's input X): the forward's output. An
 * entry (v, f) with fwd_out[v,f] == 0 is skipped: its winner u has X[u,f] * w == 0, so it
 * is either masked (X[u,f] = 0) or weighted 0 — the result is unchanged. (A +-inf
 * maximum, stored as 0, is skipped too.) The mask is still applied.
 * PG_ARG_DEAD_NONE records (the same skip made by the forward; needs mask_src = X, a relu
 * output, X >= 0): every entry left has X[u,f] * w != 0, hence X[u,f] > 0, so the mask is
 * implied and mask_src is not read (an element no entry reaches is +0 either way). With
 * X < 0 somewhere the result is undefined.
 * Every dx element is written (no zero-fill needed). A source row the schedule of gt
 * splits is summed piece by piece (each piece in ascending v from +0) and the pieces in
 * order from +0, inside the pull's launch for 16-byte rows (F, ldx multiples of 4). */
size_t pg_spmm_max_bwd_workspace(const pg_csr_t* gt, int64_t F);
int pg_spmm_max_bwd(const pg_csr_t* g, const pg_csr_t* gt, const void* argpos, int64_t lda,
                    int arg_kind, const float* dout, int64_t ldd, int64_t F,
                    const float* mask_src, int64_t ldm, const float* fwd_out, int64_t ldf,
                    float* dx, int64_t ldx, void* ws, size_t ws_bytes, pg_stream_t stream);

/* DGL-form backward: dx = 0; dx[src(argpos[v,f]), f] += ew * dout[v,f] with f32
 * atomics (summation order not reproducible). The callee zero-fills dx. */
int pg_spmm_max_bwd_scatter(const pg_csr_t* g, const void* argpos, int64_t lda, int arg_kind,
                            const float* dout, int64_t ldd, int64_t F, float* dx, int64_t ldx,
                            int64_t n_src, pg_stream_t stream);

/* out[r,f] = sum_{k in row r} coef_k * X[col[k], f] with
 *   coef_k = (ew ? ew[eslot ? eslot[k] : k] : 1)
 *   norm_mode 0: plain sum; 1: divide the row sum by the row's entry count (mean);
 *   2: each term divided by the entry count of col[k] in norm_ptr (mean backward).
 * Rows with no entries get 0. */
size_t pg_spmm_sum_workspace(const pg_csr_t* g, int64_t F);
int pg_spmm_sum(const pg_csr_t* g, const float* X, int64_t ldx, int64_t F, int norm_mode,
                const int32_t* norm_ptr, float* out, int64_t ldo, void* ws, size_t ws_bytes,
                pg_stream_t stream);

/* argx[v,f] = col[ptr[v] + argpos[v,f]] (DGL's argX, int64), -1 where none. */
int pg_argpos_to_src(const pg_csr_t* g, const void* argpos, int64_t lda, int arg_kind,
                     int64_t F, int64_t* argx, int64_t ldx, pg_stream_t stream);

/* ---------------- device: dense helpers of the training step ---------------- */

/* y = act(y + bias) in place (bias may be NULL). */
int pg_bias_act(float* y, int64_t ldy, int64_t rows, int64_t cols, const float* bias, int act,
                float slope, pg_stream_t stream);
/* dy = dy * act'(y) in place, from the activation OUTPUT y (relu: y>0; leaky: y>0?1:slope). */
int pg_act_bwd(float* dy, int64_t lddy, const float* y, int64_t ldy, int64_t rows, int64_t cols,
               int act, float slope, pg_stream_t stream);
/* out[c] (+)= sum_r x[r,c]; deterministic (fixed two-level order). */
size_t pg_col_sum_workspace(int64_t rows, int64_t cols);
int pg_col_sum(const float* x, int64_t ldx, int64_t rows, int64_t cols, float* out,
               int accumulate, void* ws, size_t ws_bytes, pg_stream_t stream);

/* Sigmoid + class-weighted BCE of code/train.py:89-108 on the rows in index[]:
 *   prob = sigmoid(z) for all n_rows rows (written if prob != NULL)
 *   loss[0] = sum_c -(1/n) sum_{r in index} (t log(clamp(p,1e-9,10)) w_c
 *                                   + (1-t) log(clamp(1-p,1e-9,10))) / (w_c+1) * 2
 *   dz (if not NULL) = d loss / d z for rows in index, 0 elsewhere (all n_rows rows written).
 * class_w[2c] = (float)w_c and class_w[2c+1] = (float)(w_c + 1), both rounded from the
 * float64 weights of weight_cal (code/train.py:111-126). C <= 64. loss may be NULL. */
/* The model head after liner1, fused (code/model.py:28-29, code/train.py:89-108, 199-207):
 *   z = A4 W2^T + b2;  prob = sigmoid(z);  multi_loss over the rows with row_set 1 (train,
 *   loss2[0], n = n_train) and row_set 2 (val, loss2[1], n = n_val);  dz = d loss2[0] / dz
 *   (0 outside the train rows);  dA4 = (dz W2) * leaky'(A4) with negative slope `slope`.
 * A4 [n][K] and dA4 [n][K] are f32 or bf16 (a_dtype); W2 [C][K], b2 [C] f32; K <= 128,
 * C <= 16. Optional outputs (NULL = skip): prob, dz, dz_bf16 (a bf16 copy of dz, leading
 * dimension lddz), dA4. Scratch: pg_mlp_head_workspace(n, C) bytes. */
size_t pg_mlp_head_workspace(int64_t n, int32_t C);
int pg_mlp_head(const void* A4, int64_t lda, int64_t n, int32_t K, int a_dtype, const float* W2,
                int64_t ldw, const float* b2, int32_t C, const float* labels, int64_t ldl,
                const float* class_w, const int8_t* row_set, int64_t n_train, int64_t n_val,
                float* prob, int64_t ldp, float* dz, int64_t lddz, void* dz_bf16, void* dA4,
                int64_t ldg, float slope, float* loss2, void* ws, size_t ws_bytes,
                pg_stream_t stream);
/* liner1 + the head above + liner1's input gradient in one pass (ABI 12; f32; replaces the
 * fwd.liner1 GEMM, pg_mlp_head and the dgrad.liner1 GEMM of a training step, code/model.py:
 * 26-29 and their backward):
 *   A4 = leaky(H3 W1^T + b1);  then pg_mlp_head's outputs on A4 (prob, dz, dA4, loss2);
 *   dH3 = (dA4 W1) * leaky'(H3)  (liner1's input gradient through the last SAGE layer's
 *   leaky_relu, with negative slope `slope` for both activations).
 * H3 [n][F3], W1 [K1][F3], b1 [K1], A4 [n][K1], dA4 [n][K1], dH3 [n][F3] f32; F3 % 4 == 0,
 * K1 <= 128, C <= 16; H3, W1, W2 16-B aligned with leading dimensions multiples of 4. The two
 * products are computed exactly as pg_gemm_f32's three-piece kernel computes them (same
 * split, same k order and MFMA sequence), so A4 and dH3 equal its results bitwise. prob and
 * dz are optional (NULL). Scratch (256-B aligned): pg_mlp_l1_head_workspace(n, C, F3, K1)
 * bytes; F3 <= 4096. adam_state (optional, NULL = none): the launch also does
 * pg_adam_prepare(adam_state, lr, beta1, beta2)'s work (one per step, before pg_adam_apply),
 * so a training step needs one launch fewer. */
size_t pg_mlp_l1_head_workspace(int64_t n, int32_t C, int32_t F3, int32_t K1);
int pg_mlp_l1_head(const float* H3, int64_t ldh, int64_t n, int32_t F3, const float* W1, int64_t ldw1,
                   const float* b1, int32_t K1, float* A4, int64_t lda4, const float* W2, int64_t ldw,
                   const float* b2, int32_t C, const float* labels, int64_t ldl, const float* class_w,
                   const int8_t* row_set, int64_t n_train, int64_t n_val, float* prob, int64_t ldp,
                   float* dz, int64_t lddz, float* dA4, int64_t ldg, float* dH3, int64_t lddh, float slope,
                   float* loss2, void* ws, size_t ws_bytes, float* adam_state, double lr, double beta1,
                   double beta2, pg_stream_t stream);
/* (ABI 13) W1's three bf16 pieces kept by the caller instead of split in each call:
 * pg_mlp_l1_split writes them (two fragment-native layouts, pg_mlp_l1_pieces_bytes(F3, K1)
 * bytes, 256-B aligned) from W1; pg_mlp_l1_head_ex is pg_mlp_l1_head reading them (W1
 * itself is then not read); pg_adam_apply_l1 is pg_adam_apply over the n flat parameters
 * that also rewrites, for W1 = param + w1_offset ([K1][ldw1] inside the n), the pieces of
 * every element it updates: after it the pieces equal pg_mlp_l1_split of the new W1 bitwise,
 * so a training step needs no split launch. The pieces go stale if W1 is written any other
 * way: split again. Results are bitwise those of pg_mlp_l1_head / pg_adam_apply. */
size_t pg_mlp_l1_pieces_bytes(int32_t F3, int32_t K1);
int pg_mlp_l1_split(const float* W1, int64_t ldw1, int32_t F3, int32_t K1, void* pieces, pg_stream_t stream);
int pg_mlp_l1_head_ex(const float* H3, int64_t ldh, int64_t n, int32_t F3, const float* W1, int64_t ldw1,
                      const float* b1, int32_t K1, float* A4, int64_t lda4, const float* W2, int64_t ldw,
                      const float* b2, int32_t C, const float* labels, int64_t ldl, const float* class_w,
                      const int8_t* row_set, int64_t n_train, int64_t n_val, float* prob, int64_t ldp,
                      float* dz, int64_t lddz, float* dA4, int64_t ldg, float* dH3, int64_t lddh, float slope,
                      float* loss2, void* ws, size_t ws_bytes, float* adam_state, double lr, double beta1,
                      double beta2, const void* w1_pieces, pg_stream_t stream);
int pg_adam_apply_l1(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n,
                     const float* state, double beta1, double beta2, double eps, double weight_decay,
                     int64_t w1_offset, int64_t ldw1, int32_t F3, int32_t K1, void* w1_pieces,
                     pg_stream_t stream);
size_t pg_sigmoid_multi_loss_workspace(int64_t n_index, int32_t C);
int pg_sigmoid_multi_loss(const float* z, int64_t ldz, int64_t n_rows, int32_t C,
                          const float* labels, int64_t ldl, const float* class_w,
                          const int32_t* index, int64_t n_index, float* prob, int64_t ldp,
                          float* loss, float* dz, int64_t lddz, void* ws, size_t ws_bytes,
                          pg_stream_t stream);

/* Adam, torch 1.10 formula (code/train.py:180,205 with the pinned torch 1.10.0):
 *   m = m*b1 + (1-b1)*g;  v = v*b2 + (1-b2)*g*g;
 *   p = p + (-lr/bc1) * (m / (sqrt(v)/sqrt(bc2) + eps)),  bc_i = 1 - b_i^step
 * Hyper-parameters are doubles, as the Python floats torch receives; scalar factors are
 * formed in double and rounded to float once, like torch's scalar arguments.
 * state[0] = step count (float, exact to 2^24), advanced on the device by
 * pg_adam_prepare so a captured graph replays correctly; state[1..3] scratch. */
int pg_adam_prepare(float* state, double lr, double beta1, double beta2, pg_stream_t stream);
int pg_adam_apply(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n,
                  const float* state, double beta1, double beta2, double eps,
                  double weight_decay, pg_stream_t stream);

/* Epilogue of pg_gemm_f32 (NULL = plain C = alpha * op(A) op(B) + beta * C). */
typedef struct pg_gemm_epilogue {
  const float* bias; /* [N] row vector added after alpha*AB + beta*C, or NULL */
  int act;           /* PG_ACT_*: applied to the result, unless dact is given */
  float slope;       /* negative slope of PG_ACT_LEAKY */
  const float* dact; /* if not NULL: multiply the result by act'(dact[m][n]) instead, dact being
                        the activation OUTPUT (relu: dact > 0 ? 1 : 0; leaky: dact > 0 ? 1 : slope)
                        = the fused backward of relu / leaky_relu */
  int64_t lddact;
  float* rowsum;     /* if not NULL: rowsum[m] = sum_k op(A)[m][k] (overwritten). For a weight
                        gradient dY^T X (transa) these are the bias gradients sum_nodes dY. */
} pg_gemm_epilogue_t;

/* C[M,N] = alpha * op(A) * op(B) + beta * C, then the epilogue.
 * op(A) = A (M x K, lda) or A^T when transa (A stored K x M); op(B) = B (K x N) or B^T when
 * transb (B stored N x K). fp32 in, fp32 out, f32 accumulate on the matrix cores:
 *   - 16-B aligned operands whose contiguous extents and leading dimensions are multiples
 *     of 4: every element split into three bf16 pieces a = a_h + a_m + a_l, six piece
 *     products (h.h, h.m, m.h, h.l, l.h, m.m) on v_mfma_f32_32x32x16_bf16. Error per
 *     output <= ~1e-6 of sum_k |a b| (f32 level). Finite operands with |x| < 3.39e38
 *     only: an Inf or NaN operand gives NaN in its outputs (where f32 arithmetic could
 *     give +-Inf), and finite values that round to Inf in bf16 also give NaN.
 *   - otherwise: v_mfma_f32_32x32x2_f32 (f32 products, IEEE non-finite behaviour).
 * When split_k > 1, beta must be 0 or 1 and the epilogue may only carry rowsum (partials
 * are combined in the workspace, in slice order: deterministic). */
/* Recommended split_k for pg_gemm_f32 (long-K products such as weight gradients):
 * about five 64 x 64 workgroups per CU, each slice >= 96 entries of K, at most 256. */
int pg_gemm_f32_split_k(int64_t M, int64_t N, int64_t K);
size_t pg_gemm_f32_workspace(int64_t M, int64_t N, int64_t K, int split_k);
/* Deferred split-K: pg_gemm_f32_partials runs the split product (C = op(A) op(B), rowsum
 * allowed, nothing else) and leaves the partial slabs in ws (layout of pg_gemm_f32:
 * split_used slabs of M x N, then split_used row-sum slices of M); *split_used = the slice
 * count actually run. pg_gemm_splitk_reduce_batch then combines up to 16 such products in
 * one launch, C = alpha * sum_z slab_z (+ beta * C, beta 0 or 1), each exactly as
 * pg_gemm_f32's own combine (bitwise the same result). The ws regions must stay untouched
 * between the two calls. */
typedef struct pg_splitk_job {
  const float* ws;  /* the partials' workspace */
  int split_k;      /* *split_used of the partials call */
  int64_t M, N;
  float alpha, beta;
  float* C;
  int64_t ldc;
  float* rowsum;    /* or NULL (must match the partials call's ep->rowsum != NULL) */
} pg_splitk_job_t;
int pg_gemm_f32_partials(int transa, int transb, int64_t M, int64_t N, int64_t K, const float* A,
                         int64_t lda, const float* B, int64_t ldb, const pg_gemm_epilogue_t* ep,
                         int split_k, void* ws, size_t ws_bytes, int* split_used, pg_stream_t stream);
int pg_gemm_splitk_reduce_batch(const pg_splitk_job_t* jobs, int n_jobs, pg_stream_t stream);
/* Grouped split-K products (a training step's weight gradients, code/model.py:13-17
 * backward: they feed only the optimizer, so all of them can run at the end of the
 * backward): part p computes C_p = op(A_p) op(B_p) (+ C_p when beta_p = 1; beta 0 or 1)
 * and, if rowsum_p, rowsum_p = the row sums of op(A_p), as pg_gemm_f32 with no other
 * epilogue. The parts' tiles times one K-slice count for the whole group run as ONE
 * three-piece launch sized for the chip (so the partial slabs scale with the group's
 * workgroups, not with each product's), then one combine launch; deterministic. Parts
 * that are not all of one (transa, transb), or whose operands the three-piece kernel does
 * not take (16-B alignment, extents multiple of 4), run one after another as pg_gemm_f32.
 * Up to 16 parts. The workspace size depends on the shapes and flags only. */
typedef struct pg_gemm_part {
  int32_t transa, transb;
  int64_t M, N, K;
  const void* A; /* f32 (pg_gemm_f32_group) or bf16 bits (pg_gemm_bf16_group); C is f32 */
  int64_t lda;
  const void* B;
  int64_t ldb;
  float beta;
  float* C;
  int64_t ldc;
  float* rowsum; /* or NULL */
} pg_gemm_part_t;
size_t pg_gemm_f32_group_workspace(const pg_gemm_part_t* parts, int n_parts);
int pg_gemm_f32_group(const pg_gemm_part_t* parts, int n_parts, void* ws, size_t ws_bytes,
                      pg_stream_t stream);
int pg_gemm_f32(int transa, int transb, int64_t M, int64_t N, int64_t K, float alpha,
                const float* A, int64_t lda, const float* B, int64_t ldb, float beta, float* C,
                int64_t ldc, const pg_gemm_epilogue_t* ep, int split_k, void* ws,
                size_t ws_bytes, pg_stream_t stream);
/* pg_gemm_f32 with both operands given as two pieces concatenated along K (ABI 10):
 * C = alpha [A1 | A2] op([B1 ; B2]) + beta C (+ bias, leaky_relu), A1 M x K1, A2 M x K2 (not
 * transposed), op(B1) K1 x N, op(B2) K2 x N: the dgl shim's SAGEConv products
 * [H | M] [Wself | Wneigh]^T and [dY | dP] [Wself ; Wpool] without copying the pieces
 * together (code/model.py:13-15, 20-25). Three-piece kernel only: K1 a multiple of 4, each
 * piece's operands 16-B aligned with leading dimensions and contiguous extents multiples of
 * 4, else PG_ERR_UNSUPPORTED (the caller concatenates instead); ep: bias and act none |
 * leaky only. */
int pg_gemm_f32_cat(int transb, int64_t M, int64_t N, int64_t K1, int64_t K2, float alpha, const float* A1,
                    int64_t lda1, const float* A2, int64_t lda2, const float* B1, int64_t ldb1, const float* B2,
                    int64_t ldb2, float beta, float* C, int64_t ldc, const pg_gemm_epilogue_t* ep,
                    pg_stream_t stream);

/* ---------------- device: bf16 storage mode (f32 accumulate) ---------------- */

/* pg_gemm_f32's contract with bf16 operands (uint16 bits, row-major): op(A), op(B) bf16,
 * products on v_mfma_f32_32x32x16_bf16 with f32 accumulate; C is f32 (c_dtype =
 * PG_DTYPE_F32) or bf16 (PG_DTYPE_BF16, rounded to nearest even). The epilogue's bias and
 * rowsum are f32; C read for beta != 0 is in C's storage type; ep->dact points to bf16
 * values (activation outputs are stored bf16 in this mode).
 * Requirements: 16-B aligned A, B, C; lda, ldb multiples of 8; the contiguous extent of
 * each operand (K for A / B^T, M for A^T, N for B) a multiple of 8; N and ldc multiples of
 * 4; split_k > 1 only with an f32 C. Else PG_ERR_UNSUPPORTED. */
int pg_gemm_bf16_split_k(int64_t M, int64_t N, int64_t K);
size_t pg_gemm_bf16_workspace(int64_t M, int64_t N, int64_t K, int split_k);
/* pg_gemm_f32_group's contract with bf16 operands and f32 C (bf16 weight gradients): parts
 * of one (transa, transb) whose 256 x 256 tiles waste at most 4x their area run as one
 * split-K launch of the two-phase kernel (one K-slice count for the group, chosen so the
 * items fill whole rounds of one workgroup per CU) and one combine; the others (and all of
 * them when the operands break pg_gemm_bf16's layout rules) one after another as
 * pg_gemm_bf16. Up to 16 parts. */
size_t pg_gemm_bf16_group_workspace(const pg_gemm_part_t* parts, int n_parts);
int pg_gemm_bf16_group(const pg_gemm_part_t* parts, int n_parts, void* ws, size_t ws_bytes,
                       pg_stream_t stream);
int pg_gemm_bf16(int transa, int transb, int64_t M, int64_t N, int64_t K, float alpha,
                 const void* A, int64_t lda, const void* B, int64_t ldb, float beta, void* C,
                 int64_t ldc, int c_dtype, const pg_gemm_epilogue_t* ep, int split_k, void* ws,
                 size_t ws_bytes, pg_stream_t stream);
/* pg_spmm_max_fwd / pg_spmm_max_bwd on bf16 features (X, out, dout, mask_src, dx): the
 * max is a selection, so out holds the winning bf16 value exactly (u_mul_e products are
 * rounded to nearest even); the backward accumulates in f32 and rounds dx once. Same
 * workspace queries. The backward needs PG_ARG_U16 records and F <= 1024. */
int pg_spmm_max_fwd_bf16(const pg_csr_t* g, const void* X, int64_t ldx, int64_t F, void* out,
                         int64_t ldo, void* argpos, int64_t lda, int arg_kind, void* ws,
                         size_t ws_bytes, pg_stream_t stream);
int pg_spmm_max_bwd_bf16(const pg_csr_t* g, const pg_csr_t* gt, const void* argpos, int64_t lda,
                         int arg_kind, const void* dout, int64_t ldd, int64_t F,
                         const void* mask_src, int64_t ldm, const void* fwd_out, int64_t ldf,
                         void* dx, int64_t ldx, void* ws, size_t ws_bytes, pg_stream_t stream);
/* dst[i] = bf16(src[map ? map[i] : i]) (map[i] < 0: 0), round to nearest even: the bf16
 * weight copies of the f32 master parameters, in any layout the GEMMs want. */
int pg_cast_f32_bf16(const float* src, const int32_t* map, int64_t n, void* dst, pg_stream_t stream);
int pg_cast_bf16_f32(const void* src, int64_t n, float* dst, pg_stream_t stream);

/* Zero-padded 2-D copies in one launch (ABI 11): for each part, dst[r][c] = src[r][c] for
 * r < rows, c < cols, else 0, over drows x dcols (row-major, leading dimensions lds / ldd).
 * The drop-in SAGEConv's padded weight images (503 -> 512: [Wpool], bpool, [Wself | Wneigh])
 * built from the layer's parameters each forward (code/model.py:13-15). */
#define PG_PAD2D_MAX 8
typedef struct pg_pad2d {
  const float* src;
  int64_t lds, rows, cols;
  float* dst;
  int64_t ldd, drows, dcols;
} pg_pad2d_t;
int pg_pad2d_group(const pg_pad2d_t* parts, int n, pg_stream_t stream);

/* The PCA front end (code/data_preprocess.py:475-487 `pca`, scikit-learn 1.1.1
 * PCA(n_components, random_state=42) on the ECC / GCN*PPI matrices, 528-546): its randomized
 * SVD's products with the centred matrix, float64, as a CSR x dense SpMM with a rank-1 term:
 *   Y[r, :] = sum_{j in row r} val[j] X[col[j], :] - (u ? u[r] : 1) * v[:]   (v NULL: no term)
 * k <= 512 columns. Sum in CSR order (deterministic). */
int pg_csr_spmm_f64(int64_t n_rows, const int32_t* ptr, const int32_t* col, const double* val,
                    const double* X, int64_t ldx, int64_t k, const double* u, const double* v,
                    double* Y, int64_t ldy, pg_stream_t stream);

/* ---------------- host (_cpu): the same operations on host pointers ---------------- */
int pg_spmm_max_fwd_cpu(const pg_csr_t* g, const float* X, int64_t ldx, int64_t F, float* out,
                        int64_t ldo, void* argpos, int64_t lda, int arg_kind);
int pg_spmm_max_bwd_cpu(const pg_csr_t* g, const pg_csr_t* gt, const void* argpos, int64_t lda,
                        int arg_kind, const float* dout, int64_t ldd, int64_t F,
                        const float* mask_src, int64_t ldm, float* dx, int64_t ldx);
int pg_spmm_sum_cpu(const pg_csr_t* g, const float* X, int64_t ldx, int64_t F, int norm_mode,
                    const int32_t* norm_ptr, float* out, int64_t ldo);
int pg_argpos_to_src_cpu(const pg_csr_t* g, const void* argpos, int64_t lda, int arg_kind,
                         int64_t F, int64_t* argx, int64_t ldx);

/* ---------------- device: §8f — edge clustering coefficient ---------------- */

/* code/data_preprocess.py:175-214 edge_clustering_coefficients on a symmetric adjacency
 * in CSR form (sorted, unique column ids per row):
 *   ecc[k] for entry k = (i, j), i != j:
 *     epsilon if min(deg_i, deg_j) - 1 == 0, else |N(i) ∩ N(j)| / (min(deg_i, deg_j) - 1)
 *   deg = row sums of the stored values (NULL: row lengths); diagonal entries get 0.
 * mirror[k] = index of the entry (j, i); order = rows longest first (optional, speed only).
 * n <= 2^22 (the neighbour bitmap of a row lives in LDS). Bit-exact (integer counts, one
 * f64 division). */
int pg_ecc(const int32_t* ptr, const int32_t* col, const int32_t* mirror, const double* deg,
           const int32_t* order, int64_t n, int64_t nnz, double epsilon, double* ecc,
           pg_stream_t stream);

/* ---------------- device: §8f — per-epoch evaluation ---------------- */

/* code/train.py:19-39 protein_loc_correction on proba[n][C] (float32, C <= 64):
 *   new = (p - colmin) / (colmax - colmin); new /= rowsum(new);
 *   pred[r][c] = new > rowmax - (rowmax - rowmin) * (float)alpha ? 1.0 : 0.0  (float64)
 * code/train.py:42-86 performances_record: out3 = {aim, coverage, accuracy}, the row terms
 * summed in row order in float32 and divided by n, as the reference's running scalars.
 * Scratch: pg_loc_eval_workspace(n, C) bytes. */
size_t pg_loc_eval_workspace(int64_t n, int32_t C);
int pg_loc_correction(const float* proba, int64_t ldp, int64_t n, int32_t C, double alpha,
                      double* pred, int64_t ldpred, void* ws, size_t ws_bytes, pg_stream_t stream);
int pg_loc_performance(const float* loc_true, int64_t ldt, const double* loc_pred, int64_t ldp,
                       int64_t n, int32_t C, double* out3, void* ws, size_t ws_bytes,
                       pg_stream_t stream);

/* ---------------- device: §8f — topology perturbation ---------------- */

/* code/data_preprocess.py:165-170 (np.corrcoef of the expression rows, diagonal and NaN
 * set to 0) for the normal and the intervention state, and :217-257
 * modify_network_topology on their difference, without materialising any N x N matrix.
 * xc_*: [n][S] float64 CENTRED expression rows (x - x.mean(axis=1), computed by the
 * caller as numpy does), 2 <= S <= 8; inv_fact = 1 / (S - 1).
 *   pcc(i, j) = clip(((fma-chain dot(xc_i, xc_j)) * inv_fact) / sd_i / sd_j, -1, 1),
 *               0 on the diagonal and where NaN;  sd_i = sqrt(dot(xc_i, xc_i) * inv_fact)
 *   diff(i, j) = pcc_inter(i, j) - pcc_normal(i, j)
 * pg_perturb_prepare: sd_* [n].
 * pg_perturb_sum: *total = sum over all n*n entries of diff (squared = 0) or of
 *   (diff - mean)^2 (squared = 1); compensated f64, deterministic. Scratch:
 *   pg_perturb_workspace(n) bytes. The caller forms mean = total / n^2,
 *   std = sqrt(total_sq / n^2), lo_thr = mean - thr * std, hi_thr = mean + thr * std.
 * pg_perturb_count / pg_perturb_fill: the perturbed adjacency, given the original as CSR
 *   (sorted unique columns per row; val = stored int64 values, NULL = all ones):
 *   v' = 0 if v == 1 and diff < lo_thr;  1 if v == 0 and diff > hi_thr;  v otherwise.
 *   count: non-zeros per row; fill: column ids and values of the non-zeros, row-major,
 *   ascending columns, row i starting at offsets[i]. n <= 1 310 720 (LDS row bitmap). */
size_t pg_perturb_workspace(int64_t n);
int pg_perturb_prepare(const double* xc_normal, const double* xc_inter, int64_t n, int32_t S,
                       double inv_fact, double* sd_normal, double* sd_inter, pg_stream_t stream);
int pg_perturb_sum(const double* xc_normal, const double* xc_inter, const double* sd_normal,
                   const double* sd_inter, int64_t n, int32_t S, double inv_fact, int squared,
                   double mean, double* total, void* ws, size_t ws_bytes, pg_stream_t stream);
int pg_perturb_count(const double* xc_normal, const double* xc_inter, const double* sd_normal,
                     const double* sd_inter, int64_t n, int32_t S, double inv_fact,
                     const int32_t* ptr, const int32_t* col, const int64_t* val, double lo_thr,
                     double hi_thr, int32_t* counts, pg_stream_t stream);
int pg_perturb_fill(const double* xc_normal, const double* xc_inter, const double* sd_normal,
                    const double* sd_inter, int64_t n, int32_t S, double inv_fact,
                    const int32_t* ptr, const int32_t* col, const int64_t* val, double lo_thr,
                    double hi_thr, const int64_t* offsets, int32_t* out_col, int64_t* out_val,
                    pg_stream_t stream);

/* ---------------- misc ---------------- */
const char* pg_last_error_string(void);
int pg_version(void); /* 2: pg_csr_t.einv; 3: pg_spmm_max_bwd fwd_out; 5: no in-kernel split-K
                         (epilogue without splitk_cnt), no grouped SpMM pair; 6: with fwd_out,
                         pg_spmm_max_bwd[_bf16] takes mask_src >= 0 and does not read it;
                         PG_ARG_DEAD_NONE; 7: pg_spmm_max_bwd reads no einv, smaller
                         workspace; 8: pg_csr_t without einv; max backward lists as 8-B
                         records with the edge weight folded in; with fwd_out alone the
                         relu' mask is applied, only PG_ARG_DEAD_NONE implies it;
                         9: pg_gemm_f32_group; 10: the in-CSR's epos = transposed
                         indices (transposed max-backward descriptors), pg_gemm_f32_cat;
                         11: pg_pad2d_group; 12: pg_mlp_l1_head;
                         13: pg_mlp_l1_split, pg_mlp_l1_head_ex, pg_adam_apply_l1 */

#ifdef __cplusplus
}
#endif
#endif /* PLAGNN_H */
