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
 *   ured_nn_seg_bwd  <- autograd of the above (NmDistanceGradKernel semantics,
 *                       chamfer3D.cu:155-174, made deterministic).
 */
#ifndef URED_HIP_H
#define URED_HIP_H

#ifdef __cplusplus
extern "C" {
#endif

#define URED_OK 0
#define URED_EINVAL 1001

/* Library identification: returns URED_ABI_VERSION. */
#define URED_ABI_VERSION 1
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

/* Backward of ured_nn_seg_fwd: accumulates into ga (a-points) and gb (b-points)
 * exactly the per-pair formula of ured_nn_bwd. gd_a / gd_b may be NULL. */
int ured_nn_seg_bwd(const float* a, const float* b, const int* segs, int nseg,
                    int max_a_len, int max_b_len,
                    const float* gd_a, const float* gd_b, const int* idx_a, const int* idx_b,
                    float* ga, float* gb, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* URED_HIP_H */
