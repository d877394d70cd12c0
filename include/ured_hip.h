/*
 * ured_hip.h — C-ABI of libured_hip.so, the MI355X (gfx950) hot path of the
 * U-RED retrieval-and-deformation training step.
 *
 * Conventions (all entry points):
 *   - plain device pointers + sizes, no torch types; fp32 point sets are
 *     contiguous AoS [.., 3]; indices are int32.
 *   - `stream` is a hipStream_t (0 = null stream); nothing synchronises the
 *     host, nothing allocates: callers pass workspaces where one is needed.
 *   - return 0 on success, otherwise a non-zero code (a hipError_t or
 *     URED_EINVAL); ured_last_error() then holds a thread-local message.
 *     (The reference returns 1/0 after printf and its wrapper ignores it,
 *     chamfer3D.cu:145-151 / dist_chamfer_3D.py:45; our wrapper raises.)
 *
 * Reference interfaces replaced (paths relative to the reference root):
 *   ured_nn_fwd      <- chamfer_3D.forward   chamfer_cuda.cpp:17-19 -> chamfer3D.cu:136-154
 *   ured_nn_bwd      <- chamfer_3D.backward  chamfer_cuda.cpp:22-28 -> chamfer3D.cu:176-195
 *     (both under Density_aware_Chamfer_Distance/utils_v2/metrics/CD/chamfer3D/)
 *   ured_nn_seg_fwd  <- the per-sample loops of loss/chamfer_loss.py:13-30
 *                       (Shape_Measure ChamferLoss calls) and
 *                       loss/basic_loss.py:249-265 (pytorch3d knn_points K=1),
 *                       batched into one ragged launch.
 *   ured_nn_fwd_ws / ured_nn_seg_fwd_ws <- the same two, both directions in one pass
 *   ured_get_shape_fwd/bwd <- get_shape's torch.bmm (dataset/dataset_utils.py:691-726)
 *   ured_emd_fwd / ured_emd_bwd <- emd.forward / emd.backward (utils_v2/metrics/EMD/emd.cpp:14-24)
 *   ured_nn_seg_bwd  <- autograd of the above (NmDistanceGradKernel semantics,
 *                       chamfer3D.cu:155-174, made deterministic).
 *   ured_node_gemm / ured_node_bn_fwd / ured_node_bn_bwd <- the graph-node Conv1d / BatchNorm1d
 *                       layers of DeformNet_MatchingNet (network/deformation_net.py:61,90,
 *                       attention_graph/attention_gnn.py:20-54, attention_utils.py:62-86).
 */
#ifndef URED_HIP_H
#define URED_HIP_H

#ifdef __cplusplus
extern "C" {
#endif

#define URED_OK 0
#define URED_EINVAL 1001

/* Library identification: returns URED_ABI_VERSION. */
#define URED_ABI_VERSION 9   /* 9: ured_attn_fwd_sets / ured_attn_bwd_sets, ured_get_shape_src_fwd / _bwd; 8: ured_nn_bwd_set; 7: ured_copy_batch; 6: ured_part_rows_bwd_add; 5: node BN SyncBN fields (stats_out/stats_in, sums_out/sums_in); ured_bn_stats et al. */
int ured_abi_version(void);
/* Thread-local message for the last failing call on this thread ("" if none). */
const char* ured_last_error(void);

/* ---------------- nearest neighbour (chamfer) ---------------- */

/* Dense NN, both directions (reference chamfer_3D.forward).
 * xyz1 [b,n,3], xyz2 [b,m,3] ->
 *   dist1[b,n] = min_k |xyz2[k]-xyz1[j]|^2, idx1[b,n] its argmin (lowest index on ties)
 *   dist2[b,m], idx2[b,m] vice versa.
 * Distance formula (bit-exact contract): d = fmaf(dz,dz, fmaf(dy,dy, dx*dx)), dx = q2.x - q1.x.
 * dirs: bit 0 -> compute (dist1, idx1); bit 1 -> compute (dist2, idx2). */
int ured_nn_fwd(const float* xyz1, const float* xyz2, int b, int n, int m, int dirs,
                float* dist1, int* idx1, float* dist2, int* idx2, void* stream);

/* Dense NN backward (reference chamfer_3D.backward): accumulates
 *   gxyz1[j] += 2 gd1[j] (p1_j - p2_idx1[j]) - sum_{k: idx2[k]=j} 2 gd2[k] (p2_k - p1_j)
 * and symmetrically into gxyz2. Deterministic (gather form, k ascending), no atomics.
 * gd1/gd2 may be NULL (treated as zero). */
int ured_nn_bwd(const float* xyz1, const float* xyz2, int b, int n, int m,
                const float* gd1, const float* gd2, const int* idx1, const int* idx2,
                float* gxyz1, float* gxyz2, void* stream);
/* The same gradient WRITTEN instead of accumulated (every element of gxyz1 / gxyz2 is set, so
 * the caller needs no zero fill; n, m > 0). The autograd Function behind chamfer_3DDist uses it;
 * ured_nn_bwd keeps the reference's accumulate-into-caller-zeroed-buffers contract. */
int ured_nn_bwd_set(const float* xyz1, const float* xyz2, int b, int n, int m,
                    const float* gd1, const float* gd2, const int* idx1, const int* idx2,
                    float* gxyz1, float* gxyz2, void* stream);

/* Ragged NN over segment pairs. segs is a DEVICE int32 array [nseg][4] =
 * {a_off, a_len, b_off, b_len} in points of the two buffers a [*,3] and b [*,3].
 * Within one call, a-ranges must be pairwise disjoint and so must b-ranges.
 * For every pair: dist_a[a_off+i], idx_a[a_off+i] = NN of a-point i among the
 * pair's b-points (idx relative to b_off); and vice versa into dist_b/idx_b.
 * Points not covered by any pair are left untouched. max_a_len / max_b_len are
 * host-side upper bounds of a_len / b_len (they size the grid; no host sync).
 * A pair with an empty other side writes dist 0, idx 0. */
int ured_nn_seg_fwd(const float* a, const float* b, const int* segs, int nseg,
                    int max_a_len, int max_b_len, int dirs,
                    float* dist_a, int* idx_a, float* dist_b, int* idx_b, void* stream);

/* Fused forward (both directions from ONE evaluation of every pair distance; same results,
 * bit for bit, as ured_nn_fwd / ured_nn_seg_fwd with dirs = 3). The caller passes a device
 * workspace of ured_nn_fwd_workspace(...) bytes (no initialisation needed; contents are
 * scratch). a_total / b_total = number of points in the a / b buffers (dense: b*n, b*m).
 * ured_nn_fwd_workspace returns 0 when the fused path does not apply (dirs != 3, empty
 * sizes); the _ws entry points then (or with workspace == NULL) run the two-pass kernel. */
#include <stddef.h>
size_t ured_nn_fwd_workspace(int nseg, int max_a_len, int max_b_len, int a_total, int b_total, int dirs);
int ured_nn_fwd_ws(const float* xyz1, const float* xyz2, int b, int n, int m, int dirs,
                   float* dist1, int* idx1, float* dist2, int* idx2, void* workspace, size_t ws_bytes,
                   void* stream);
int ured_nn_seg_fwd_ws(const float* a, const float* b, const int* segs, int nseg,
                       int max_a_len, int max_b_len, int dirs, int a_total, int b_total,
                       float* dist_a, int* idx_a, float* dist_b, int* idx_b,
                       void* workspace, size_t ws_bytes, void* stream);

/* get_shape (dataset/dataset_utils.py:691-726): out[j, r] = sum_k A[j, r, k] p[j, k] for every
 * part slot j (A [nparts, rows, 6] contiguous, 8-byte aligned; p [nparts, 6] = weight*param +
 * default); the backward gives grad_p[j, k] = sum_r A[j, r, k] grad_out[j, r] (deterministic). */
int ured_get_shape_fwd(const float* A, const float* p, int nparts, int rows, float* out, void* stream);
int ured_get_shape_bwd(const float* A, const float* grad_out, int nparts, int rows, float* grad_p, void* stream);
/* The training step's form (engine/train.py:222-223: get_source_info + get_shape): part slot j reads
 * mats + src_j * rows * 6, src_j = labels[j] (int64; + nsrc when negative, python indexing), so no
 * gathered copy of the source matrices; p[j] = weight * param[j] + dflt[j] (dflt may be NULL) is
 * formed in-kernel with get_shape's separate mul and add; the backward writes
 * grad_param = weight * sum_r A grad_out. */
int ured_get_shape_src_fwd(const float* mats, const long long* labels, int nsrc, const float* param,
                           const float* dflt, float weight, int nparts, int rows, float* out, void* stream);
int ured_get_shape_src_bwd(const float* mats, const long long* labels, int nsrc, const float* grad_out, float weight,
                           int nparts, int rows, float* grad_param, void* stream);

/* Per-part axis-aligned boxes (compute_aabbox, dataset/dataset_utils.py:77-85, as used by
 * get_part, engine/train.py:119-128): x [R,3] points sorted by segment, off int32 [G+1] row
 * offsets -> out [G,6] = (center, half extent) of each segment; empty segments give zeros. */
int ured_seg_aabb(const float* x, const int* off, int G, float* out, void* stream);

/* Backward of get_part's per-point regrouping (engine/train.py:103-136: the points of every
 * sample sorted by part label, and the per-part sums of their features): for R = B*N rows of C
 * floats, out[b*N + i] = d_sorted[s] + d_sums[gid[s]] with s = b*N + inv[b, i] (the row's
 * position after the sort, inv int64 [B, N]; gid int32 [R] the part slot of each sorted row).
 * Either gradient may be NULL (zero). One pass: replaces an index_select, a gather and an add. */
int ured_part_rows_bwd(const float* d_sorted, const float* d_sums, const long long* inv, const int* gid, int B, int N,
                       int C, float* out, void* stream);
/* The same plus `add` [R,C] (may be NULL, or `out` itself: in-place accumulation): out = (d_sorted
 * + d_sums) + add, where add is another consumer's gradient of the same per-point features (the
 * reconstruction decoder's input gradient, engine/train.py:240,250): the sum autograd would form
 * in a separate pass (ABI 6). */
int ured_part_rows_bwd_add(const float* d_sorted, const float* d_sums, const long long* inv, const int* gid, int B,
                           int N, int C, const float* add, float* out, void* stream);

/* ---------------- EMD (auction algorithm) ---------------- */
/* Approximate EMD matching of xyz1 [b,n,3] to xyz2 [b,n,3] (reference emd.forward,
 * utils_v2/metrics/EMD/emd.cpp:14-19 -> emd_cuda.cu:183-256): `iters` auction rounds with
 * parameter eps; assignment[b,n] = matched xyz2 index, dist[b,n] = squared distance to it.
 * Deterministic (highest increment wins an object, ties to the lowest bidder index; scan ties to
 * the lowest object index). Workspace: ured_emd_workspace(b, n) bytes, no initialisation. */
size_t ured_emd_workspace(int b, int n);
int ured_emd_fwd(const float* xyz1, const float* xyz2, int b, int n, float eps, int iters,
                 float* dist, int* assignment, void* workspace, size_t ws_bytes, void* stream);
/* gradxyz1 += 2 graddist (xyz1 - xyz2[assignment]) (reference emd.backward, emd_cuda.cu:283-304;
 * xyz2 gets no gradient, as in emd_module.py:76-80). */
int ured_emd_bwd(const float* xyz1, const float* xyz2, int b, int n, const float* graddist, const int* assignment,
                 float* gradxyz1, void* stream);

/* Backward of ured_nn_seg_fwd: accumulates into ga (a-points) and gb (b-points)
 * exactly the per-pair formula of ured_nn_bwd. gd_a / gd_b may be NULL; gb may be NULL when
 * the b points need no gradient (only the a side is computed). */
int ured_nn_seg_bwd(const float* a, const float* b, const int* segs, int nseg,
                    int max_a_len, int max_b_len,
                    const float* gd_a, const float* gd_b, const int* idx_a, const int* idx_b,
                    float* ga, float* gb, void* stream);


/* Density-aware chamfer reduction of dense NN outputs (replaces the torch tail of
 * calc_dcd, Density_aware_Chamfer_Distance/utils_v2/model_utils.py:13-51, and the
 * cd_p / cd_t of calc_cd, :53-70; the NN itself is ured_nn_fwd with xyz1 = gt,
 * xyz2 = x, as calc_cd calls cham_loss(gt, output)).
 * dist1/idx1 [b,n1]: gt -> x; dist2/idx2 [b,n2]: x -> gt. Per item:
 *   w1 = frac_21 / (count_x(idx1)^n_lambda + 1e-6),  loss1 = mean(1 - exp(-alpha d1) w1)
 *   w2 = frac_12 / (count_gt(idx2)^n_lambda + 1e-6), loss2 = mean(1 - exp(-alpha d2) w2)
 *   loss = (loss1 + loss2)/2, cd_p = (mean sqrt d1 + mean sqrt d2)/2, cd_t = mean d1 + mean d2.
 * Forward only (no autograd), deterministic. n1 + n2 <= 16384. */
int ured_dcd(const float* dist1, const int* idx1, const float* dist2, const int* idx2, int b, int n1, int n2,
             float alpha, int n_lambda, float frac_12, float frac_21, float* loss, float* cd_p, float* cd_t,
             void* stream);

/* ---------------- per-point MLP (1x1 conv) on fp32 MFMA ---------------- *
 * Replaces the Conv1d(k=1)+BatchNorm1d+ReLU chains of TargetEncoder
 * (network/simple_encoder.py:52-107) and re_residual_net / FeedForwardNet_norm
 * (network/deformation_net.py:96-107, attention_graph/attention_utils.py:62-86),
 * forward and backward, with activations stored point-major [M][C].
 *
 * ured_gemm computes C[M][N] = sum_k A'[m][k] B'[k][n] on v_mfma_f32_32x32x2_f32
 * (exact fp32 fma chains), 128x128x32 tiles, where
 *   A'[m][k] = a_kmajor ? A[k*lda+m] : (k < k1 ? pro(A[m*lda+k]) : A2[m*lda2+k-k1])
 *   B'[k][n] = b_kmajor ? pro_b(B[k*ldb+n]) : B[n*ldb+k]
 *   pro(x)   = PRO_ENC: max(x*s[c]+t[c],0)   (Conv->BN->ReLU; c = channel = contiguous index)
 *              PRO_RES: max(x,0)*s[c]+t[c]   (Conv->ReLU->BN)
 * and an epilogue:
 *   EPI_STORE : C = acc (+bias[n])
 *   EPI_FWD   : Y = acc + bias[n] + rowbias[grp(m)][n] stored to C; per-128-row block
 *               column partials {mean, M2} of p (p = Y, or relu(Y) if stat_relu) into
 *               stat_ws[2][N][blk] (one column's block partials contiguous); if pool_ws: per block column {max,argmax,min,argmin}
 *               of Y into pool_ws[blk][4][N] (group_rows multiple of 128)
 *   EPI_BNBWD : dh = acc (+ pool_grad[g][n] where pool_idx[g][n] == m) (+ gadd[m][n]); with
 *               the previous layer's (Y, mean, invstd, scale, shift): ENC g = dh*(Y*scale+shift > 0),
 *               xhat = (Y-mean)*invstd; RES g = dh, xhat = (relu(Y)-mean)*invstd; BN g = dh,
 *               xhat = (Y-mean)*invstd. K = 0 is allowed (acc = 0: a pooled / extra gradient only);
 *               stores g to C and block column partials {sum g, sum g*xhat} to bwd_ws
 *   EPI_SPLITK: partial sums of the k-range of blockIdx.z stored to C + z*M*ldc
 */
#define URED_PRO_NONE 0
#define URED_PRO_ENC 1
#define URED_PRO_RES 2
#define URED_EPI_STORE 0
#define URED_EPI_FWD 1
#define URED_EPI_BNBWD 2
#define URED_EPI_SPLITK 3
/* EPI_BNBWD activation order of the layer whose output is being differentiated (bwd_res field) */
#define URED_ACT_ENC 0   /* Conv -> BN -> ReLU */
#define URED_ACT_RES 1   /* Conv -> ReLU -> BN */
#define URED_ACT_BN 2    /* Conv -> BN (no activation; PointNet's conv3, pointnet_utils.py:126) */

typedef struct UredGemmDesc {
    int M, N, K;
    int a_kmajor, b_kmajor, pro_a, pro_b, epi;
    const float* A; int lda;
    const float* A2; int lda2; int k1;         /* k >= k1 read from A2 (row-major A only); k1 = K if unused */
    const float* B; int ldb;
    const float* pro_s; const float* pro_t;     /* prologue per-channel affine */
    float* C; int ldc;
    const float* bias;                          /* [N] or NULL */
    const float* rowbias; int ldr;              /* [G][ldr] or NULL */
    const int* gidx; int group_rows;            /* row -> group: gidx[m] or m / group_rows */
    int stat_relu;
    float* stat_ws;                             /* [2][N][ceil(M/128)] */
    float* pool_ws;                             /* [ceil(M/128)][4][N] or NULL */
    const float* Yp; int ldy;                   /* EPI_BNBWD: previous layer's raw output */
    const float* bn_mean; const float* bn_invstd; const float* bn_scale; const float* bn_shift;
    int bwd_res;                                /* URED_ACT_ENC / URED_ACT_RES / URED_ACT_BN */
    const int* pool_idx; const float* pool_grad; int pool_group_rows;
    float* bwd_ws;                              /* [2][N][ceil(M/128)] */
    int splits;                                 /* EPI_SPLITK: gridDim.z (k-range per split = ceil(K/splits/32)*32) */
    const float* gadd; int ldg;                 /* EPI_BNBWD: optional extra gradient, dh += gadd[m*ldg+n] */
} UredGemmDesc;

int ured_gemm(const UredGemmDesc* d, void* stream);

/* Optimizer tail of the training step (reference engine/train.py:331-346: clip_grad_norm_(5.0)
 * per module, then torch.optim.Adam with L2 weight decay, train_utils/optimizer_dm.py:68-104)
 * over flat buffers param/grad/exp_avg/exp_avg_sq. Chunk c covers [chunk_beg[c], chunk_end[c])
 * (16-B aligned, lengths multiples of 4) of parameter chunk_param[c] in module segment
 * chunk_seg[c]; segment s owns chunks [seg_chunk0[s], seg_chunk0[s+1]). Only the chunks of the
 * parameters that take this step are listed (those with a gradient: torch's clip_grad_norm_
 * and Adam skip the others). max_norm > 0: per-segment L2 norm (fp64 chunk partials in
 * `partial`, fixed order) -> coef[s] = min(max_norm / (norm + 1e-6), 1), gradient scaled in
 * place; max_norm <= 0: no clipping. param_step[active_params[i]] (device, one step count per
 * parameter as in torch's Adam) is incremented for i < n_active, then every listed element takes
 * one Adam step with *lr (device) and its parameter's bias corrections. Deterministic. */
int ured_adam_clip_step(float* param, float* grad, float* exp_avg, float* exp_avg_sq,
                        const long long* chunk_beg, const long long* chunk_end, const int* chunk_seg,
                        const int* chunk_param, int nchunks, const int* seg_chunk0, int nseg, float max_norm,
                        const float* lr, float* param_step, const int* active_params, int n_active,
                        double beta1, double beta2, double eps, double weight_decay, double* partial, float* coef,
                        void* stream);

/* Weight gradient of an edge layer (min(Cout, Kin) <= 4, the other <= 256):
 * out[co*ldo + ki] (+)= sum_m dY[m*ldd + co] * pro(X[m*ldx + ki]), deterministic (row-block
 * partials in ws, then a fixed-order tree per output). ws holds URED_SKINNY_WS_BLOCKS*Cout*Kin
 * floats. Replaces the MFMA wgrad for the 3-channel layers (a 128x128 tile would be mostly padding). */
#define URED_SKINNY_WS_BLOCKS 256
int ured_wgrad_skinny(const float* dY, int ldd, const float* X, int ldx, int Cout, int Kin, int M, int pro,
                      const float* pro_s, const float* pro_t, float* out, int ldo, int accumulate, float* ws,
                      void* stream);

/* Sum split-K partials: out[m][n] = (accumulate ? out : 0) + sum_z ws[z][m][n] (+ bias[n] if non-NULL);
 * fixed combine order (deterministic). */
int ured_splitk_reduce(const float* ws, int splits, int M, int N, float* out, int ldo, int accumulate,
                       const float* bias, void* stream);

/* BN forward finalize over the per-block partials of EPI_FWD (M rows, blocks of 128):
 * fp64 Chan merge -> mean, invstd = 1/sqrt(var_biased+eps), scale = gamma*invstd,
 * shift = beta - mean*scale; running stats (if non-NULL) updated in place with
 * momentum and the unbiased variance (torch.nn.BatchNorm1d semantics).
 * Row multiplicities (unique-row training): if group_w is non-NULL, each stored row of
 * group g = row / group_rows (group_rows a multiple of 128) stands for group_w[g] identical
 * rows of the batch; statistics are those of the expanded batch (count sum_g w_g*rows_g).
 * The same (group_w, group_rows) pair goes to the two backward calls below.
 * num_batches_tracked (nullable, int64 on the device) is incremented by one (the module's
 * counter update of a training-mode forward, folded into this launch). */
int ured_bn_fwd_finalize(const float* stat_ws, int M, int N, const float* gamma, const float* beta,
                         float eps, float momentum, float* running_mean, float* running_var,
                         float* mean, float* invstd, float* scale, float* shift,
                         const float* group_w, int group_rows, long long* num_batches_tracked, void* stream);

/* BN backward finalize over EPI_BNBWD partials: dbeta = sum g, dgamma = sum g*xhat
 * (fp64, fixed order; written, or added if accumulate) and the coefficients of
 * dY = coef_a*g + coef_b*(p - mean) + coef_c (see ured_bn_bwd_apply). */
int ured_bn_bwd_finalize(const float* bwd_ws, int M, int N, const float* gamma, const float* invstd,
                         float* dgamma, float* dbeta, int accumulate,
                         float* coef_a, float* coef_b, float* coef_c,
                         const float* group_w, int group_rows, void* stream);

/* ---- SyncBN (optional, cfg["sync_bn"]; csrc/syncbn.hip): the two finalizes above split
 * around a cross-rank exchange of fp64 per-column statistics, torch SyncBatchNorm semantics.
 * ured_bn_stats: the Chan merge of ured_bn_fwd_finalize stopped before normalising:
 *   out [3][N] = (weighted count, mean, M2) of this rank's rows.
 * ured_bn_finalize_stats: ured_bn_fwd_finalize's outputs from merged stats [3][N].
 * ured_bn_bwd_sums: out [3][N] = (sum g, sum g*xhat, weighted count) of this rank.
 * ured_bn_bwd_finalize_sums: dbeta / dgamma from `local` (written or added), the
 *   ured_bn_bwd_apply coefficients from `global` (the all-reduced sums and count). */
int ured_bn_stats(const float* stat_ws, int M, int N, const float* group_w, int group_rows, double* out,
                  void* stream);
int ured_bn_finalize_stats(const double* stats, int N, const float* gamma, const float* beta, float eps,
                           float momentum, float* running_mean, float* running_var, float* mean, float* invstd,
                           float* scale, float* shift, long long* num_batches_tracked, void* stream);
int ured_bn_bwd_sums(const float* bwd_ws, int M, int N, const float* group_w, int group_rows, double* out,
                     void* stream);
int ured_bn_bwd_finalize_sums(const double* local, const double* global, int N, const float* gamma,
                              const float* invstd, float* dgamma, float* dbeta, int accumulate, float* coef_a,
                              float* coef_b, float* coef_c, void* stream);

/* dY[m][n] = coef_a*g + coef_b*(p-mean) + coef_c with p = Y (ENC) or relu(Y) (RES, then
 * times (Y > 0)). Also writes per-128-row column partial sums of dY to colsum_ws[blk][N].
 * With group_w, G holds the multiplicity-summed gradient of each stored row and the
 * mean terms are scaled by the row's weight: dY = coef_a*g + w*(coef_b*(p-mean) + coef_c). */
int ured_bn_bwd_apply(const float* G, const float* Y, int M, int N, int ld, int res,
                      const float* mean, const float* coef_a, const float* coef_b, const float* coef_c,
                      float* dY, float* colsum_ws, const float* group_w, int group_rows, void* stream);

/* Max-pool finalize (TargetEncoder max_pool1d over each group of group_rows points of
 * relu(scale*Y+shift), simple_encoder.py:105; relu = 0: of scale*Y+shift, PointNet's
 * torch.max over bn3(conv3(x)), pointnet_utils.py:126-127): pooled[g][n] and the winning
 * row index argidx[g][n] (lowest row on ties). */
int ured_pool_finalize(const float* pool_ws, int M, int N, int group_rows, const float* scale,
                       const float* shift, int relu, float* pooled, int* argidx, void* stream);

/* Same result as EPI_FWD pooling + ured_pool_finalize for any group size (a direct scan of Y [M][N]). */
int ured_pool_rows(const float* Y, int M, int N, int group_rows, const float* scale, const float* shift,
                   int relu, float* pooled, int* argidx, void* stream);

/* out[m][n] = act(Y[m*ldy+n]*scale[n] + shift[n]), act = relu (relu != 0) or identity: a
 * BatchNorm(+ReLU) output materialised (PointNet pointfeat, pointnet_utils.py:120,124). */
int ured_bn_act(const float* Y, int M, int N, int ldy, const float* scale, const float* shift, int relu,
                float* out, int ldo, void* stream);

/* out[g][n] = sum_{m in [off[g], off[g+1])} X[m*ldx+n] (rows ascending); off == NULL means
 * fixed groups of group_rows rows. G groups. */
int ured_group_colsum(const float* X, int ldx, int N, const int* off, int group_rows, int G,
                      float* out, int ldo, void* stream);
/* As ured_group_colsum, with each group's rows cut into `splits` equal ranges summed by
 * separate workgroups into ws [G][splits][N], then the partials summed in split order
 * (deterministic; for few, long groups). splits == 1: ws may be NULL. */
int ured_group_colsum_split(const float* X, int ldx, int N, const int* off, int group_rows, int G, int splits,
                            float* ws, float* out, int ldo, void* stream);

/* ---------------- graph attention (DeformNet_MatchingNet) ---------------- */

/* Multi-head softmax attention over graph nodes, node-major layout
 * (replaces attention_graph/attention.py:8-19 as called by attention_gnn.py:20-32).
 * Row r of sample b: q + (b*n + r)*ldq, k/v + (b*m + r)*ld{k,v}; head h occupies columns
 * [h*d, (h+1)*d) (the reference's view(B, H, d, nodes) channel split).
 *   weights[b][h][i][j] = softmax_j(scale * <q_bi^h, k_bj^h>),  out_bi^h = sum_j weights * v_bj^h
 * weights [B*H*n*m] is written by the forward and read by the backward, which overwrites
 * dq [B,n,*], dk/dv [B,m,*] (may be column slices of one buffer). Limits: n, m <= 32,
 * d <= 128, and the (n, m, d) LDS image within 64 KB. */
#define URED_ATTN_MAX_NODES 32
#define URED_ATTN_MAX_HEAD_DIM 128
int ured_attn_fwd(const float* q, int ldq, const float* k, int ldk, const float* v, int ldv,
                  int B, int H, int n, int m, int d, float scale, float* out, int ldo, float* weights,
                  void* stream);
int ured_attn_bwd(const float* q, int ldq, const float* k, int ldk, const float* v, int ldv, const float* weights,
                  const float* dout, int lddo, int B, int H, int n, int m, int d, float scale,
                  float* dq, int lddq, float* dk, int lddk, float* dv, int lddv, void* stream);

/* Up to URED_ATTN_MAX_SETS independent attention calls (e.g. the two node sets of one
 * DescriptorsSelfAttention layer, attention_gnn.py:120-127: desc0 and desc1 through the same module)
 * in ONE launch; each set is exactly the call above with its own fields (fwd: out / ldo / weights,
 * bwd: weights / dout / dq / dk / dv), so the results are those of separate calls, bitwise. */
#define URED_ATTN_MAX_SETS 2
typedef struct {
    const float* q; int ldq;
    const float* k; int ldk;
    const float* v; int ldv;
    int B, H, n, m, d;
    float scale;
    float* out; int ldo;            /* forward output */
    float* weights;                 /* [B*H*n*m]: written by the forward, read by the backward */
    const float* dout; int lddo;    /* backward only */
    float* dq; int lddq;
    float* dk; int lddk;
    float* dv; int lddv;
} UredAttnSet;
int ured_attn_fwd_sets(int nsets, const UredAttnSet* sets, void* stream);
int ured_attn_bwd_sets(int nsets, const UredAttnSet* sets, void* stream);

/* ---------------- graph-node layers (DeformNet_MatchingNet, node.hip) ----------------
 * Replace the node-level Conv1d(k=1) layers (in_proj_q/k/v, out_proj, the FeedForwardNet_norm
 * convs and param_decoder: network/deformation_net.py:61,90, attention_graph/attention_gnn.py:
 * 20-32,50-54, attention_graph/attention_utils.py:62-86), forward and both backward GEMMs,
 * and the BatchNorm1d of FeedForwardNet_norm (Conv -> ReLU -> BN).
 *
 * ured_node_gemm: C[m][n] (+)= epi( sum_k A(m,k) B(k,n) ), M rows of graph nodes (small), with
 *   A(m,k) = A [m*sam + k*sak]           for k <  k1
 *          = A2[m*sam2 + (k-k1)*sak2]    for k >= k1   (cat([x, message]) along K, read in place)
 *   B(k,n) = B [k*sbk + n*sbn]           for n <  n1 (W^T: sbk = 1, sbn = ldW; W: sbk = ldW, sbn = 1)
 *          = B2[k*sbk2 + (n-n1)*sbn2]    for n >= n1 when B2 != NULL (wgrad of cat([x, message]))
 *   v = sum + bias[n] + rowbias[(m/rdiv)*ldrb + n]; relu_out: v = max(v, 0);
 *   gate: v = gate[m*ldgate+n] > 0 ? v : 0; v += R[m*ldR+n] for n < R_ncols;
 *   accumulate: C += v, else C = v.
 * k1 >= K or k1 % 16 == 0. Nullable: A2, B2, bias, rowbias, gate, R. Deterministic (fixed split
 * and summation order).
 * kind URED_NODE_COLSUM (a bias gradient riding in the same batched launch): C[n] (+)= sum over
 * m < M of A[m*sam + n*sak], n < N (B, K unused). */
#define URED_NODE_GEMM 0
#define URED_NODE_COLSUM 1
typedef struct {
    int M, N, K;
    const float* A; long long sam, sak;
    const float* A2; long long sam2, sak2; int k1;
    const float* B; long long sbk, sbn;
    const float* B2; long long sbk2, sbn2; int n1;
    float* C; long long ldc; int accumulate;
    const float* bias;
    const float* rowbias; long long ldrb; int rdiv;
    int relu_out;
    const float* gate; long long ldgate;
    const float* R; long long ldR; int R_ncols;
    int kind;
} UredNodeGemmDesc;
int ured_node_gemm(const UredNodeGemmDesc* d, void* stream);
/* Up to URED_NODE_MAX_JOBS independent node GEMMs in one launch (no ordering between them). */
#define URED_NODE_MAX_JOBS 6
int ured_node_gemm_batch(const UredNodeGemmDesc* const* d, int n, void* stream);

/* BatchNorm1d over node sets: rows [off[s], off[s+1]) are one call of the module (the two node
 * sets of a self-attention layer share it: the reference calls it once per set, in order).
 * x = relu_in ? max(Y, 0) : Y. training: per-set batch mean / biased variance (fp64 sums),
 * running stats updated per set in order (unbiased variance, momentum), num_batches_tracked
 * (nullable) += nsets; eval: running stats. Writes mean/invstd [nsets][N] and
 * act[m*ld_act+n] = (x - mean) * invstd * gamma + beta.
 * SyncBN (training only): stats_out non-NULL -> ONLY write each set's local fp64 (count, mean,
 * M2) to stats_out [nsets][3][N] and return (nothing else is written); stats_in non-NULL -> use
 * those (cross-rank merged) per-set statistics instead of this call's rows (running stats
 * updated with the merged count's unbiased variance). */
#define URED_NODE_MAX_SETS 4
typedef struct {
    int N, nsets, off[URED_NODE_MAX_SETS + 1];
    const float* Y; long long ldy; int relu_in, training;
    const float* gamma; const float* beta;
    float* running_mean; float* running_var; long long* num_batches_tracked;
    float momentum, eps;
    float* mean; float* invstd;
    float* act; long long ld_act;
    double* stats_out; const double* stats_in;
} UredNodeBNDesc;
int ured_node_bn_fwd(const UredNodeBNDesc* d, void* stream);

/* Backward of ured_node_bn_fwd: G = d loss / d act -> dY (through the ReLU when relu_in),
 * dgamma / dbeta summed over the sets (written, or added if accumulate).
 * SyncBN: sums_out non-NULL -> ONLY write each set's local fp64 (sum g, sum g*xhat, count) to
 * sums_out [nsets][3][N] and return; sums_in non-NULL -> the input gradient uses those
 * (cross-rank summed) sums and counts, dgamma / dbeta stay this rank's local sums. */
typedef struct {
    int N, nsets, off[URED_NODE_MAX_SETS + 1];
    const float* G; long long ldg;
    const float* Y; long long ldy; int relu_in, training;
    const float* gamma; const float* mean; const float* invstd;
    float* dY; long long lddy;
    float* dgamma; float* dbeta; int accumulate;
    double* sums_out; const double* sums_in;
} UredNodeBNBwdDesc;
int ured_node_bn_bwd(const UredNodeBNBwdDesc* d, void* stream);


/* get_part's per-sample bookkeeping (engine/train.py:103-136, compute_aabbox dataset_utils.py:77-85)
 * in one launch (csrc/parts.hip): labels int64 [B,N] (part ids in [0,P)), x [B,N,3] ->
 * x_sorted [B,N,3] (points stably sorted by label), perm / inv_perm int64 [B,N], gid int32 [B*N]
 * (part slot b*P + rank of each sorted point), off int32 [B*P+1] (row offsets of the slots),
 * counts int64 [B,P], k int64 [B], mask float [B,P], rank_of_label int64 [B,P] (cumsum(present)-1),
 * present uint8 [B,P], aabb [B,P,6] by slot and param_def [B,P,6] by label value ((center,
 * half extent), 0 for absent labels). Replaces the per-part Python loop / torch.unique. */
int ured_build_parts(const long long* labels, const float* x, int B, int N, int P, float* x_sorted,
                     long long* perm, long long* inv_perm, int* gid, int* off, long long* counts,
                     long long* k, float* mask, long long* rank_of_label, unsigned char* present,
                     float* aabb, float* param_def, void* stream);

/* Several device-to-device copies in one launch (csrc/copy.hip): the HIP-graph step refreshes its
 * static input batch before each replay (engine/graph.py) with this instead of one blit per
 * tensor. dst[i][0, bytes[i]) = src[i][0, bytes[i]); regions must not overlap; 16-B moves where
 * both addresses and the size allow, else 4-B or 1-B moves for that item. */
#define URED_COPY_MAX 16
typedef struct { void* dst; const void* src; long long bytes; } UredCopyItem;
int ured_copy_batch(const UredCopyItem* items, int n, void* stream);

/* ---------------- loss head (csrc/loss.hip) ---------------- */
/* compute_cm_loss of the deformed shape `out` [B,S,3] and of its mirror image (x -> -x,
 * get_symmetric) against the same target x [B,N,3] (engine/train.py:288,302 ->
 * loss/chamfer_loss.py:13-30, the Shape_Measure ChamferLoss calls per sample and per part):
 *   prep   : A = [out; mirror(out)] [2B,S,3], X2 = [x; x], XS2 = [x_sorted; x_sorted] [2B,N,3] and
 *            the segment tables of ured_nn_seg_fwd: full family int32 [2B,4] (a = the first
 *            k_b*NP points of half-sample s, b = its x) and part family [2B*P,4] (chunk i < k_b of
 *            NP points vs the points of part i: off int32 [B*P+1] / counts int64 [B,P] of
 *            x_sorted, k int64 [B] parts per sample);
 *   reduce : the four scalars [full, part, mirror full, mirror part] from the two families' NN
 *            distances (dist_a_* [2B*S], dist_b_* [2B*N]); CD = mean(cost1) + mean(cost2), part
 *            CD = mean over the sample's parts, both averaged over B. ws: 3*2B*(P+1) floats;
 *            counter: a device uint that is 0 before the launch (it is left at 0);
 *   grad   : d terms g4 [4] -> the per-distance upstream weights of ured_nn_seg_bwd (gid int32
 *            [B*N]: part slot of each sorted row) and ga [2B*S*3] zeroed for its accumulation;
 *   fold   : grad_out [B,S,3] = ga[:B] + mirror(ga[B:]).
 * Replace the per-sample / per-part Python loops, means and masks of the reference (and their
 * autograd) with 4 + 3 launches around the two NN launches. */
int ured_cd_pair_prep(const float* out, const float* x, const float* x_sorted, const long long* k,
                      const long long* counts, const int* off, int B, int S, int N, int P, int NP, float* A,
                      float* X2, float* XS2, int* segs_full, int* segs_part, void* stream);
int ured_cd_pair_reduce(const float* dist_a_full, const float* dist_b_full, const float* dist_a_part,
                        const float* dist_b_part, const long long* k, const long long* counts, const int* off,
                        int B, int S, int N, int P, int NP, float* ws, unsigned* counter, float* terms, void* stream);
int ured_cd_pair_grad(const float* g4, const long long* k, const long long* counts, const int* gid, int B, int S,
                      int N, int P, int NP, float* gd_a_full, float* gd_b_full, float* gd_a_part, float* gd_b_part,
                      float* ga, void* stream);
int ured_cd_pair_fold(const float* ga, int B, int S, float* grad_out, void* stream);

/* residual_retrieval_loss (loss/basic_loss.py:249-265: x -> out nearest neighbour knn [B,N]
 * relative to the sample's rows, terms mean_n sum|x + res - out[nn]| and mean_n sum|res|),
 * compute_pc_consistency(rec, x) and compute_pc_consistency_weighted(recon_src, src_points, mask)
 * (loss/basic_consistency_loss.py:4-22), the last over the U distinct source parts of the batch
 * (recu / ptsu [U,NP,3]; slot r of the R = B*P part slots holds part inv[r], weight mask[r]).
 * Forward -> terms [4]; backward: upstream g4 [4] -> dres, drec [B,N,3], drecu [U,NP,3]. */
typedef struct {
    int B, N, S, U, NP, R;
    const float* x; const float* out; const int* knn; const float* res; const float* rec;
    const float* recu; const float* ptsu; const long long* inv; const float* mask;
} UredPointLossDesc;
int ured_point_losses_fwd(const UredPointLossDesc* d, float* ws, unsigned* counter, float* terms, void* stream);
int ured_point_losses_bwd(const UredPointLossDesc* d, const float* g4, float* dres, float* drec, float* drecu,
                          void* stream);

/* compute_contrast_loss_loss (loss/contrast_loss.py:61-102): t [n,C] target part features,
 * s_all [n_all,C] source codes of every rank (this rank's rows start at s_off), src_labels int64
 * [n] (-1: row ignored, else its label is s_off + i); loss = CE(scale * norm(t) norm(s_all)^T).
 * Forward writes inv norms [n + n_all], lse [n], ws [2n] and loss [1]; backward (g: d loss)
 * writes dt [n,C] and, when ds is not NULL, ds [n,C] for this rank's rows. */
int ured_contrast_fwd(const float* t, const float* s_all, const long long* src_labels, int n, int n_all, int C,
                      int s_off, float scale, float* inv, float* lse, float* ws, unsigned* counter, float* loss,
                      void* stream);
int ured_contrast_bwd(const float* t, const float* s_all, const long long* src_labels, int n, int n_all, int C,
                      int s_off, float scale, const float* inv, const float* lse, const float* g, float* dt, float* ds,
                      void* stream);

/* loss_all = sum_i weights[i] * *terms[i] in order (engine/train.py:278-335), one thread; the
 * backward writes gterms[i] = weights[i] * g. */
#define URED_ASSEMBLE_MAX 16
int ured_loss_assemble(int K, const float* const* terms, const float* weights, float* out, void* stream);
int ured_loss_assemble_bwd(int K, const float* weights, const float* g, float* gterms, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* URED_HIP_H */
