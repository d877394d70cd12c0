// loss.hip — the U-RED step's loss head on MI355X (gfx950): the bookkeeping around the
// nearest-neighbour kernels and the small losses, as a handful of launches instead of the
// ~150 tiny torch kernels (means, masks, concatenations, normalisations, cross-entropy, their
// autograd nodes) the composed ops cost.
//
//   ured_cd_pair_prep / _reduce / _grad / _fold
//       compute_cm_loss of the deformed shape AND of its mirror image against the same target
//       (engine/train.py:288,302; loss/chamfer_loss.py:13-30): the two full families
//       out[b, :k_b*1024] <-> x[b] and the two part families out[b, i*1024:(i+1)*1024] <->
//       points of part i of x[b], as 2B + 2BP segments of two ragged NN launches (nn.hip); the
//       reductions to the four loss scalars; the per-point upstream weights of the backward and
//       the fold of the mirror half's gradient.
//   ured_point_losses_fwd / _bwd
//       residual_retrieval_loss (loss/basic_loss.py:249-265), compute_pc_consistency and
//       compute_pc_consistency_weighted (loss/basic_consistency_loss.py:4-22) — the last one on
//       the distinct source parts of a unique-source batch with slot multiplicities.
//   ured_contrast_norms / _fwd / _bwd
//       compute_contrast_loss_loss (loss/contrast_loss.py:61-102): L2 normalisation, the
//       logits (1/0.07) t s^T, cross-entropy with ignore_index -1, and their backward.
//   ured_loss_assemble / _bwd
//       loss_all = sum_i w_i term_i in the order of engine/train.py:278-335, and its backward
//       (the per-term upstream gradients every backward above reads from device memory).
//
// Reductions are deterministic: fixed per-thread strides, fixed-shape LDS trees, and the
// final combine done by the LAST workgroup to finish (an integer arrival counter; partials
// stored and read back write-through, see last_arrival), in a fixed order, in fp64. The counter is reset by that
// workgroup, so a launch leaves it at 0 for the next one (and for HIP-graph replays).
#include <hip/hip_runtime.h>
#define URED_DBG_FILE 3
#include "ured_common.h"
#include "../../include/ured_hip.h"

namespace {

constexpr int LT = 256;          // threads per workgroup of the reduction kernels

template <typename T>
__device__ __forceinline__ T block_sum(T v, T* sh) {
    const int t = threadIdx.x;
    sh[t] = v;
    __syncthreads();
    for (int o = LT / 2; o > 0; o >>= 1) {
        if (t < o) sh[t] += sh[t + o];
        __syncthreads();
    }
    const T r = sh[0];
    __syncthreads();
    return r;
}

__device__ __forceinline__ float block_max(float v, float* sh) {
    const int t = threadIdx.x;
    sh[t] = v;
    __syncthreads();
    for (int o = LT / 2; o > 0; o >>= 1) {
        if (t < o) sh[t] = fmaxf(sh[t], sh[t + o]);
        __syncthreads();
    }
    const float r = sh[0];
    __syncthreads();
    return r;
}

// Arrival of this workgroup's partials; true in the last workgroup to arrive, which may then
// read every workgroup's partials. The hand-off (MI355X_MICROARCH.md, inter-workgroup
// visibility, first row of the sc1 table): partials are stored write-through (st_agent: global
// store sc1), every storing wave waits for its stores (vmcnt(0)) before the workgroup barrier,
// ONE lane adds to the agent-scope counter, and the workgroup whose add returned the last
// count reads the partials with sc1 loads (ld_agent) — no cache-flushing fences (__threadfence
// costs ~3.5 us here). That workgroup resets the counter for the next launch / graph replay.
__device__ __forceinline__ bool last_arrival(unsigned* counter, unsigned nblocks) {
    __shared__ bool last;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned prev = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last = prev == nblocks - 1;
        if (last) __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    return last;
}

__device__ __forceinline__ float ld_agent(const float* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void st_agent(float* p, float v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---------------------------------------------------------------------------------------
// chamfer pair (full + part families of out and of its mirror image)
// ---------------------------------------------------------------------------------------
struct CdShape {
    int B, S, N, P, NP;
};

// A = [out; mirror(out)] (2B x S points), X2 = [x; x], XS2 = [x_sorted; x_sorted] (2B x N);
// the segment tables: full (2B rows) and part (2B*P rows) of (a_off, a_len, b_off, b_len).
__global__ __launch_bounds__(LT) void cd_pair_prep_kernel(CdShape sh, const float* __restrict__ out,
        const float* __restrict__ x, const float* __restrict__ xs, const long long* __restrict__ k,
        const long long* __restrict__ counts, const int* __restrict__ off, float* __restrict__ A,
        float* __restrict__ X2, float* __restrict__ XS2, int* __restrict__ segf, int* __restrict__ segp) {
    const long long t = (long long)blockIdx.x * LT + threadIdx.x;
    const long long BS = (long long)sh.B * sh.S, BN = (long long)sh.B * sh.N;
    if (t < 2 * BS) {
        const long long src = t < BS ? t : t - BS;
        const float sx = out[3 * src], sy = out[3 * src + 1], sz = out[3 * src + 2];
        A[3 * t] = t < BS ? sx : -sx;
        A[3 * t + 1] = sy;
        A[3 * t + 2] = sz;
    }
    if (t < 2 * BN) {
        const long long src = t < BN ? t : t - BN;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            X2[3 * t + c] = x[3 * src + c];
            XS2[3 * t + c] = xs[3 * src + c];
        }
    }
    if (t < 2 * sh.B * (sh.P + 1)) {
        const int s = (int)(t / (sh.P + 1)), i = (int)(t % (sh.P + 1));
        const int h = s / sh.B, b = s % sh.B;
        const int kb = (int)k[b];
        URED_DBG_CHECK(kb >= 0 && kb <= sh.P);
        if (i == sh.P) {
            int4 q = make_int4(s * sh.S, kb * sh.NP, s * sh.N, sh.N);
            reinterpret_cast<int4*>(segf)[s] = q;
        } else {
            const bool v = i < kb;
            // off: the part's first row in the [B * N] sorted rows (b * N + start, csrc/parts.hip)
            URED_DBG_CHECK(!v || (off[b * sh.P + i] >= b * sh.N && counts[(size_t)b * sh.P + i] >= 0 &&
                                  off[b * sh.P + i] + counts[(size_t)b * sh.P + i] <= (long long)(b + 1) * sh.N));
            int4 q = make_int4(s * sh.S + i * sh.NP, v ? sh.NP : 0, off[b * sh.P + i] + h * (int)BN,
                               v ? (int)counts[(size_t)b * sh.P + i] : 0);
            reinterpret_cast<int4*>(segp)[s * sh.P + i] = q;
        }
    }
}

// Partials per workgroup (i, s): i < P -> part slot i of half-sample s: the full family's
// a-side sum over the slot's chunk, the part family's a-side sum and b-side sum; i == P -> the
// full family's b-side sum over x. The last workgroup combines (fp64, fixed order):
//   full_s = sum_a / (k_b NP) + sum_b / N,  part_s = (1/k_b) sum_{i<k_b} (a_i / NP + b_i / cnt_i)
//   terms  = [mean_b full (h=0), mean_b part (h=0), mean_b full (h=1), mean_b part (h=1)].
constexpr int CD_MAX_UNITS = 2 * 128 * 33;    // 2B (P+1) partial units staged in LDS (B <= 128, P <= 32)

__global__ __launch_bounds__(LT) void cd_pair_reduce_kernel(CdShape sh, const float* __restrict__ daf,
        const float* __restrict__ dbf, const float* __restrict__ dap, const float* __restrict__ dbp,
        const long long* __restrict__ k, const long long* __restrict__ counts, const int* __restrict__ off,
        float* __restrict__ part, unsigned* counter, float* __restrict__ terms) {
    __shared__ float shf[LT];
    __shared__ double shd[LT];
    extern __shared__ float stage[];           // last workgroup: 3 * 2B(P+1) partials
    const int i = blockIdx.x, s = blockIdx.y;
    const int h = s / sh.B, b = s % sh.B;
    const int kb = (int)k[b];
    const int t = threadIdx.x;
    float q0 = 0.f, q1 = 0.f, q2 = 0.f;
    if (i < sh.P) {
        if (i < kb) {
            const long long a0 = (long long)s * sh.S + (long long)i * sh.NP;
            float s0 = 0.f, s1 = 0.f;
            for (int p = t; p < sh.NP; p += LT) { s0 += daf[a0 + p]; s1 += dap[a0 + p]; }
            const int cnt = (int)counts[(size_t)b * sh.P + i];
            URED_DBG_CHECK(kb <= sh.P && cnt >= 0 && off[b * sh.P + i] >= b * sh.N &&
                           off[b * sh.P + i] + cnt <= (b + 1) * sh.N);
            const long long b0 = (long long)off[b * sh.P + i] + (long long)h * sh.B * sh.N;
            float s2 = 0.f;
            for (int j = t; j < cnt; j += LT) s2 += dbp[b0 + j];
            q0 = block_sum(s0, shf); q1 = block_sum(s1, shf); q2 = block_sum(s2, shf);
        }
    } else {
        const long long b0 = (long long)s * sh.N;
        float s0 = 0.f;
        for (int j = t; j < sh.N; j += LT) s0 += dbf[b0 + j];
        q0 = block_sum(s0, shf);
    }
    const int slot = s * (sh.P + 1) + i;
    if (t == 0) { st_agent(part + 3 * slot, q0); st_agent(part + 3 * slot + 1, q1); st_agent(part + 3 * slot + 2, q2); }
    if (!last_arrival(counter, gridDim.x * gridDim.y)) return;
    const int units = 2 * sh.B * (sh.P + 1);
    for (int q = t; q < 3 * units; q += LT) stage[q] = ld_agent(part + q);   // independent loads
    __syncthreads();
    // combine: one thread per half-sample, then the batch means
    double fs = 0.0, ps = 0.0;
    int hh = 0;
    if (t < 2 * sh.B) {
        const int ss = t, bb = ss % sh.B;
        hh = ss / sh.B;
        const int kk = (int)k[bb];
        double sa = 0.0, sp = 0.0;
        for (int ii = 0; ii < kk; ++ii) {
            const int sl = ss * (sh.P + 1) + ii;
            sa += (double)stage[3 * sl];
            const double cnt = (double)counts[(size_t)bb * sh.P + ii];
            sp += (double)stage[3 * sl + 1] / sh.NP + (cnt > 0 ? (double)stage[3 * sl + 2] / cnt : 0.0);
        }
        const double sbf = (double)stage[3 * (ss * (sh.P + 1) + sh.P)];
        fs = kk > 0 ? sa / ((double)kk * sh.NP) + sbf / sh.N : __builtin_nan("");
        ps = kk > 0 ? sp / kk : __builtin_nan("");
    }
    const double f0 = block_sum(t < 2 * sh.B && hh == 0 ? fs : 0.0, shd);
    const double p0 = block_sum(t < 2 * sh.B && hh == 0 ? ps : 0.0, shd);
    const double f1 = block_sum(t < 2 * sh.B && hh == 1 ? fs : 0.0, shd);
    const double p1 = block_sum(t < 2 * sh.B && hh == 1 ? ps : 0.0, shd);
    if (t == 0) {
        terms[0] = (float)(f0 / sh.B); terms[1] = (float)(p0 / sh.B);
        terms[2] = (float)(f1 / sh.B); terms[3] = (float)(p1 / sh.B);
    }
}

// Upstream weights of every NN distance (d loss / d dist) and ga = 0:
//   full a: g_full[h] / (B k_b NP) on the sample's first k_b*NP points, 0 after;
//   full b: g_full[h] / (B N);   part a: g_part[h] / (B k_b NP) on valid chunks;
//   part b: g_part[h] / (B k_b cnt_{b,i}) on the points of part i (gid: slot of each sorted row).
__global__ __launch_bounds__(LT) void cd_pair_grad_kernel(CdShape sh, const float* __restrict__ g4,
        const long long* __restrict__ k, const long long* __restrict__ counts, const int* __restrict__ gid,
        float* __restrict__ gaf, float* __restrict__ gbf, float* __restrict__ gap, float* __restrict__ gbp,
        float* __restrict__ ga) {
    const long long t = (long long)blockIdx.x * LT + threadIdx.x;
    const long long BS = (long long)sh.B * sh.S, BN = (long long)sh.B * sh.N;
    if (t < 2 * BS) {
        const int s = (int)(t / sh.S), p = (int)(t % sh.S);
        const int h = s / sh.B, b = s % sh.B;
        const int kb = (int)k[b];
        const bool v = kb > 0 && p < kb * sh.NP;
        const float den = (float)sh.B * (float)(kb > 0 ? kb : 1) * (float)sh.NP;
        gaf[t] = v ? g4[2 * h] / den : 0.f;
        gap[t] = v ? g4[2 * h + 1] / den : 0.f;
        ga[3 * t] = 0.f; ga[3 * t + 1] = 0.f; ga[3 * t + 2] = 0.f;
    }
    if (t < 2 * BN) {
        const int h = (int)(t / BN);
        const long long r = t - h * BN;
        const int b = (int)(r / sh.N);
        gbf[t] = g4[2 * h] / ((float)sh.B * (float)sh.N);
        const int slot = gid[r], i = slot % sh.P;
        URED_DBG_CHECK(slot >= 0);
        const int kb = (int)k[b];
        const long long cnt = counts[(size_t)b * sh.P + i];
        gbp[t] = (i < kb && cnt > 0) ? g4[2 * h + 1] / ((float)sh.B * (float)kb * (float)cnt) : 0.f;
    }
}

// g_out[b, p] = ga[b, p] + mirror(ga[B + b, p])  (the mirror image's gradient folded back)
__global__ __launch_bounds__(LT) void cd_pair_fold_kernel(long long BS, const float* __restrict__ ga,
                                                          float* __restrict__ g) {
    const long long t = (long long)blockIdx.x * LT + threadIdx.x;
    if (t >= BS) return;
    const float* u = ga + 3 * t;
    const float* m = ga + 3 * (t + BS);
    g[3 * t] = u[0] - m[0];
    g[3 * t + 1] = u[1] + m[1];
    g[3 * t + 2] = u[2] + m[2];
}

// ---------------------------------------------------------------------------------------
// residual + reconstruction losses
// ---------------------------------------------------------------------------------------
struct PointLossArgs {
    int B, N, S, U, NP, R;                   // R = slots (B * P)
    const float* x;                          // [B, N, 3]
    const float* out;                        // [B, S, 3] deformed shape (no gradient)
    const int* knn;                          // [B, N] x -> out NN index within the sample's rows
    const float* res;                        // [B, N, 3] residuals
    const float* rec;                        // [B, N, 3] recon_decoder_full output
    const float* recu;                       // [U, NP, 3] recon_decoder_src output per distinct part
    const float* ptsu;                       // [U, NP, 3] the distinct parts' points
    const long long* inv;                    // [R] distinct part of each slot
    const float* mask;                       // [R] part-slot mask
    float* part;                             // partials workspace
    unsigned* counter;
    float* terms;                            // [4]: res L1, res reg, recon full, recon src
    const float* g4;                         // backward: upstream gradients of the 4 terms
    float* dres; float* drec; float* drecu;  // backward outputs
};

constexpr int PL_CHUNK = 256;                // points per workgroup of the B*N part

__device__ __forceinline__ float slot_weight(const PointLossArgs& a, int u, float* shf, float* msum) {
    // w_u = sum of the mask over the slots that hold distinct part u; *msum = sum of the mask
    float w = 0.f, m = 0.f;
    for (int r = threadIdx.x; r < a.R; r += LT) {
        const float mk = a.mask[r];
        m += mk;
        w += a.inv[r] == u ? mk : 0.f;
    }
    *msum = block_sum(m, shf);
    return block_sum(w, shf);
}

__global__ __launch_bounds__(LT) void point_losses_fwd_kernel(PointLossArgs a) {
    __shared__ float shf[LT];
    __shared__ double shd[LT];
    const int nb1 = (a.B * a.N + PL_CHUNK - 1) / PL_CHUNK;
    const int blk = blockIdx.x, t = threadIdx.x;
    float q0 = 0.f, q1 = 0.f, q2 = 0.f;
    if (blk < nb1) {
        float l1 = 0.f, l2 = 0.f, l3 = 0.f;
        const long long e0 = (long long)blk * PL_CHUNK, e1 = min((long long)a.B * a.N, e0 + PL_CHUNK);
        for (long long e = e0 + t; e < e1; e += LT) {
            const int b = (int)(e / a.N);
            URED_DBG_CHECK((unsigned)a.knn[e] < (unsigned)a.S);
            const float* nn = a.out + 3 * ((long long)b * a.S + a.knn[e]);
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                const float xv = a.x[3 * e + c], r = a.res[3 * e + c];
                l1 += fabsf(xv + r - nn[c]);
                l2 += fabsf(r);
                const float d = a.rec[3 * e + c] - xv;
                l3 += d * d;
            }
        }
        q0 = block_sum(l1, shf); q1 = block_sum(l2, shf); q2 = block_sum(l3, shf);
    } else {
        const int u = blk - nb1;
        float l = 0.f;
        const long long base = (long long)u * a.NP * 3;
        for (int e = t; e < a.NP * 3; e += LT) {
            const float d = a.recu[base + e] - a.ptsu[base + e];
            l += d * d;
        }
        float msum;
        const float w = slot_weight(a, u, shf, &msum);
        q0 = block_sum(l, shf) * w;      // w_u * sum over the part's points
        q1 = msum;
    }
    if (t == 0) { st_agent(a.part + 3 * blk, q0); st_agent(a.part + 3 * blk + 1, q1); st_agent(a.part + 3 * blk + 2, q2); }
    if (!last_arrival(a.counter, gridDim.x)) return;
    double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
    for (int q = t; q < nb1; q += LT) {
        s0 += ld_agent(a.part + 3 * q); s1 += ld_agent(a.part + 3 * q + 1); s2 += ld_agent(a.part + 3 * q + 2);
    }
    for (int q = nb1 + t; q < nb1 + a.U; q += LT) s3 += ld_agent(a.part + 3 * q);
    s0 = block_sum(s0, shd); s1 = block_sum(s1, shd); s2 = block_sum(s2, shd); s3 = block_sum(s3, shd);
    if (t == 0) {
        const double M = (double)a.B * a.N;
        const double msum = a.U > 0 ? (double)ld_agent(a.part + 3 * nb1 + 1) : 0.0;
        a.terms[0] = (float)(s0 / M);
        a.terms[1] = (float)(s1 / M);
        a.terms[2] = (float)(s2 / M);
        a.terms[3] = (float)(s3 / a.NP / msum);
    }
}

__device__ __forceinline__ float sgnf(float v) { return v > 0.f ? 1.f : (v < 0.f ? -1.f : 0.f); }

__global__ __launch_bounds__(LT) void point_losses_bwd_kernel(PointLossArgs a) {
    __shared__ float shf[LT];
    const long long BN = (long long)a.B * a.N;
    const int nb1 = (int)((BN + LT - 1) / LT);
    const int blk = blockIdx.x, t = threadIdx.x;
    if (blk < nb1) {
        const long long e = (long long)blk * LT + t;
        if (e >= BN) return;
        const float M = (float)BN;
        const float g0 = a.g4[0] / M, g1 = a.g4[1] / M, g2 = 2.f * a.g4[2] / M;
        const int b = (int)(e / a.N);
        const float* nn = a.out + 3 * ((long long)b * a.S + a.knn[e]);
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const float xv = a.x[3 * e + c], r = a.res[3 * e + c];
            a.dres[3 * e + c] = g0 * sgnf(xv + r - nn[c]) + g1 * sgnf(r);
            a.drec[3 * e + c] = g2 * (a.rec[3 * e + c] - xv);
        }
        return;
    }
    // distinct source parts: one workgroup per (part, chunk of LT*4 floats)
    const int per = (a.NP * 3 + 4 * LT - 1) / (4 * LT);
    const int u = (blk - nb1) / per, ch = (blk - nb1) % per;
    float msum;
    const float w = slot_weight(a, u, shf, &msum);
    const float gs = 2.f * a.g4[3] * w / ((float)a.NP * msum);
    const long long base = (long long)u * a.NP * 3;
    for (int e = ch * 4 * LT + t; e < min(a.NP * 3, (ch + 1) * 4 * LT); e += LT)
        a.drecu[base + e] = gs * (a.recu[base + e] - a.ptsu[base + e]);
}

// ---------------------------------------------------------------------------------------
// contrastive loss (InfoNCE with ignore_index -1)
// ---------------------------------------------------------------------------------------
struct ContrastArgs {
    int n, n_all, C, s_off;                  // rows of t, rows of s_all, width, this rank's first s row
    float scale;                             // exp(logit scale)
    const float* t;                          // [n, C] target part features
    const float* s;                          // [n_all, C] source codes (all ranks)
    const long long* src_labels;             // [n]: -1 -> ignored row, else label = s_off + i
    float* inv;                              // [n + n_all] 1 / max(|row|, 1e-12)
    float* lse;                              // [n] log-sum-exp of each logits row
    float* part;                             // [n] per-row loss
    unsigned* counter;
    float* loss;                             // [1]
    const float* g;                          // backward: upstream gradient of the loss
    float* dt; float* ds;                    // backward outputs ([n, C]; ds: this rank's rows only, or NULL)
};

constexpr int CT_MAXN = 4096;                // logits row held in LDS

__global__ __launch_bounds__(LT) void contrast_norms_kernel(ContrastArgs a) {
    __shared__ float shf[LT];
    const int r = blockIdx.x;
    const float* row = r < a.n ? a.t + (size_t)r * a.C : a.s + (size_t)(r - a.n) * a.C;
    float q = 0.f;
    for (int c = threadIdx.x; c < a.C; c += LT) q += row[c] * row[c];
    q = block_sum(q, shf);
    if (threadIdx.x == 0) a.inv[r] = 1.f / fmaxf(sqrtf(q), 1e-12f);
}

// dot(v (LDS), row (global)) by ONE thread: float4 loads (C % 4 == 0, 16-B aligned rows), four
// independent accumulators so that several loads are in flight per lane
__device__ __forceinline__ float row_dot(const float* v, const float* row, int C) {
    const float4* r4 = reinterpret_cast<const float4*>(row);
    const float4* v4 = reinterpret_cast<const float4*>(v);
    float d0 = 0.f, d1 = 0.f, d2 = 0.f, d3 = 0.f;
    const int C4 = C >> 2;
#pragma unroll 4
    for (int q = 0; q < C4; ++q) {
        const float4 a = r4[q], b = v4[q];
        d0 += a.x * b.x; d1 += a.y * b.y; d2 += a.z * b.z; d3 += a.w * b.w;
    }
    return (d0 + d1) + (d2 + d3);
}

// logits of t row i against every s row into lg[] (LDS): scale * (t_i . s_j) * inv_t * inv_s
// (thread j takes row j: 256 rows in flight per workgroup)
__device__ __forceinline__ void logits_row(const ContrastArgs& a, int i, float* trow, float* lg) {
    for (int c = threadIdx.x; c < a.C; c += LT) trow[c] = a.t[(size_t)i * a.C + c];
    __syncthreads();
    const float it = a.inv[i] * a.scale;
    for (int j = threadIdx.x; j < a.n_all; j += LT)
        lg[j] = row_dot(trow, a.s + (size_t)j * a.C, a.C) * it * a.inv[a.n + j];
    __syncthreads();
}

__global__ __launch_bounds__(LT) void contrast_fwd_kernel(ContrastArgs a) {
    extern __shared__ float lds[];           // [C] t row, [n_all] logits
    __shared__ float shf[LT];
    __shared__ double shd[LT];
    float* trow = lds;
    float* lg = lds + a.C;
    const int i = blockIdx.x, t = threadIdx.x;
    logits_row(a, i, trow, lg);
    float m = -__builtin_inff();
    for (int j = t; j < a.n_all; j += LT) m = fmaxf(m, lg[j]);
    m = block_max(m, shf);
    float se = 0.f;
    for (int j = t; j < a.n_all; j += LT) se += expf(lg[j] - m);
    se = block_sum(se, shf);
    const bool valid = a.src_labels[i] != -1;
    URED_DBG_CHECK(!valid || (a.s_off + i >= 0 && a.s_off + i < a.n_all));   // the label's logit (LDS)
    if (t == 0) {
        const float l = m + logf(se);
        a.lse[i] = l;
        st_agent(a.part + 2 * i, valid ? l - lg[a.s_off + i] : 0.f);
        st_agent(a.part + 2 * i + 1, valid ? 1.f : 0.f);
    }
    if (!last_arrival(a.counter, gridDim.x)) return;
    double s0 = 0.0, s1 = 0.0;
    for (int q = t; q < a.n; q += LT) { s0 += ld_agent(a.part + 2 * q); s1 += ld_agent(a.part + 2 * q + 1); }
    s0 = block_sum(s0, shd);
    s1 = block_sum(s1, shd);
    if (t == 0) a.loss[0] = (float)(s0 / s1);     // mean over the rows that are not ignored (0/0 -> nan)
}

// normalize backward of one row: d x = (dxh - xh (xh . dxh)) * inv  (|x| > eps), dxh * inv otherwise
__device__ __forceinline__ void normalize_bwd(const ContrastArgs& a, const float* x, float inv, float* dxh,
                                              float* out, float* shf) {
    float p = 0.f;
    for (int c = threadIdx.x; c < a.C; c += LT) p += x[c] * inv * dxh[c];
    p = block_sum(p, shf);
    const bool clamped = inv >= 1e12f;
    for (int c = threadIdx.x; c < a.C; c += LT)
        out[c] = clamped ? dxh[c] * inv : (dxh[c] - x[c] * inv * p) * inv;
}

// workgroups [0, n): t rows; [n, n + n_local): this rank's s rows (when ds != NULL)
__global__ __launch_bounds__(LT) void contrast_bwd_kernel(ContrastArgs a) {
    extern __shared__ float lds[];           // [C] row, [C] d row, [max(n, n_all)] dlogits
    __shared__ float shf[LT];
    __shared__ double shd[LT];
    float* row = lds;
    float* drow = lds + a.C;
    float* dl = lds + 2 * a.C;
    const int t = threadIdx.x;
    // number of valid rows (the CE mean's denominator)
    float nv = 0.f;
    for (int q = t; q < a.n; q += LT) nv += a.src_labels[q] != -1 ? 1.f : 0.f;
    nv = block_sum(nv, shf);
    const float gsc = a.g[0] / nv;
    if ((int)blockIdx.x < a.n) {
        const int i = blockIdx.x;
        logits_row(a, i, row, dl);           // row = t_i, dl = logits
        const bool valid = a.src_labels[i] != -1;
        const float l = a.lse[i];
        for (int j = t; j < a.n_all; j += LT)
            dl[j] = valid ? gsc * (expf(dl[j] - l) - (j == a.s_off + i ? 1.f : 0.f)) * a.scale * a.inv[a.n + j] : 0.f;
        __syncthreads();
        // d t_hat_i = sum_j dl_j * s_j   (dl already carries scale * inv_s_j)
        for (int c = t; c < a.C; c += LT) {
            float acc = 0.f;
            for (int j = 0; j < a.n_all; ++j) acc += dl[j] * a.s[(size_t)j * a.C + c];
            drow[c] = acc;
        }
        __syncthreads();
        normalize_bwd(a, row, a.inv[i], drow, a.dt + (size_t)i * a.C, shf);
        return;
    }
    const int jl = blockIdx.x - a.n, j = a.s_off + jl;
    for (int c = t; c < a.C; c += LT) row[c] = a.s[(size_t)j * a.C + c];
    __syncthreads();
    const float isj = a.inv[a.n + j];
    // column j of the logits and its gradient, for every t row i
    for (int i = t; i < a.n; i += LT) {
        const float lg = row_dot(row, a.t + (size_t)i * a.C, a.C) * a.inv[i] * a.scale * isj;
        const bool valid = a.src_labels[i] != -1;
        dl[i] = valid ? gsc * (expf(lg - a.lse[i]) - (j == a.s_off + i ? 1.f : 0.f)) * a.scale * a.inv[i] : 0.f;
    }
    __syncthreads();
    for (int c = t; c < a.C; c += LT) {
        float acc = 0.f;
        for (int i = 0; i < a.n; ++i) acc += dl[i] * a.t[(size_t)i * a.C + c];
        drow[c] = acc;
    }
    __syncthreads();
    normalize_bwd(a, row, isj, drow, a.ds + (size_t)jl * a.C, shf);
    (void)shd;
}

// ---------------------------------------------------------------------------------------
// loss assembly
// ---------------------------------------------------------------------------------------
struct AssembleArgs {
    int K;
    const float* term[URED_ASSEMBLE_MAX];
    float w[URED_ASSEMBLE_MAX];
    float* out;                               // forward: loss_all
    const float* g;                           // backward: upstream gradient of loss_all
    float* gterms;                            // backward: [K] = w_i * g
};

__global__ void assemble_fwd_kernel(AssembleArgs a) {
    if (threadIdx.x != 0) return;
    float s = 0.f;                            // engine/train.py:278-335: loss_all = 0.0; loss_all += t_i * w_i
    for (int i = 0; i < a.K; ++i) s = s + *a.term[i] * a.w[i];
    a.out[0] = s;
}

__global__ void assemble_bwd_kernel(AssembleArgs a) {
    const int i = threadIdx.x;
    if (i < a.K) a.gterms[i] = a.w[i] * a.g[0];
}

}  // namespace

extern "C" {

int ured_cd_pair_prep(const float* out, const float* x, const float* x_sorted, const long long* k,
                      const long long* counts, const int* off, int B, int S, int N, int P, int NP, float* A,
                      float* X2, float* XS2, int* segs_full, int* segs_part, void* stream) {
    ured::clear_error();
    URED_REQUIRE(B > 0 && S > 0 && N > 0 && P > 0 && NP > 0 && S >= P * NP, "ured_cd_pair_prep: bad sizes");
    URED_REQUIRE(out && x && x_sorted && k && counts && off && A && X2 && XS2 && segs_full && segs_part,
                 "ured_cd_pair_prep: null pointer");
    const long long tot = 2LL * B * S > 2LL * B * N ? 2LL * B * S : 2LL * B * N;
    hipLaunchKernelGGL(cd_pair_prep_kernel, dim3((unsigned)((tot + LT - 1) / LT)), dim3(LT), 0, (hipStream_t)stream,
                       CdShape{B, S, N, P, NP}, out, x, x_sorted, k, counts, off, A, X2, XS2, segs_full, segs_part);
    return ured::launch_status("ured_cd_pair_prep");
}

int ured_cd_pair_reduce(const float* dist_a_full, const float* dist_b_full, const float* dist_a_part,
                        const float* dist_b_part, const long long* k, const long long* counts, const int* off,
                        int B, int S, int N, int P, int NP, float* ws, unsigned* counter, float* terms, void* stream) {
    ured::clear_error();
    URED_REQUIRE(B > 0 && 2 * B <= LT && S > 0 && N > 0 && P > 0 && NP > 0 && 2 * B * (P + 1) <= CD_MAX_UNITS,
                 "ured_cd_pair_reduce: bad sizes");
    URED_REQUIRE(dist_a_full && dist_b_full && dist_a_part && dist_b_part && k && counts && off && ws && counter && terms,
                 "ured_cd_pair_reduce: null pointer");
    hipLaunchKernelGGL(cd_pair_reduce_kernel, dim3(P + 1, 2 * B), dim3(LT), (size_t)3 * 2 * B * (P + 1) * sizeof(float),
                       (hipStream_t)stream,
                       CdShape{B, S, N, P, NP}, dist_a_full, dist_b_full, dist_a_part, dist_b_part, k, counts, off, ws,
                       counter, terms);
    return ured::launch_status("ured_cd_pair_reduce");
}

int ured_cd_pair_grad(const float* g4, const long long* k, const long long* counts, const int* gid, int B, int S,
                      int N, int P, int NP, float* gd_a_full, float* gd_b_full, float* gd_a_part, float* gd_b_part,
                      float* ga, void* stream) {
    ured::clear_error();
    URED_REQUIRE(B > 0 && S > 0 && N > 0 && P > 0 && NP > 0, "ured_cd_pair_grad: bad sizes");
    URED_REQUIRE(g4 && k && counts && gid && gd_a_full && gd_b_full && gd_a_part && gd_b_part && ga,
                 "ured_cd_pair_grad: null pointer");
    const long long tot = 2LL * B * S > 2LL * B * N ? 2LL * B * S : 2LL * B * N;
    hipLaunchKernelGGL(cd_pair_grad_kernel, dim3((unsigned)((tot + LT - 1) / LT)), dim3(LT), 0, (hipStream_t)stream,
                       CdShape{B, S, N, P, NP}, g4, k, counts, gid, gd_a_full, gd_b_full, gd_a_part, gd_b_part, ga);
    return ured::launch_status("ured_cd_pair_grad");
}

int ured_cd_pair_fold(const float* ga, int B, int S, float* grad_out, void* stream) {
    ured::clear_error();
    URED_REQUIRE(B > 0 && S > 0 && ga && grad_out, "ured_cd_pair_fold: bad arguments");
    const long long BS = (long long)B * S;
    hipLaunchKernelGGL(cd_pair_fold_kernel, dim3((unsigned)((BS + LT - 1) / LT)), dim3(LT), 0, (hipStream_t)stream,
                       BS, ga, grad_out);
    return ured::launch_status("ured_cd_pair_fold");
}

static int point_losses_check(const UredPointLossDesc* d) {
    URED_REQUIRE(d->B > 0 && d->N > 0 && d->S > 0 && d->U >= 0 && d->NP > 0 && d->R >= 0,
                 "ured_point_losses: bad sizes");
    URED_REQUIRE(d->x && d->out && d->knn && d->res && d->rec, "ured_point_losses: null pointer");
    URED_REQUIRE(d->U == 0 || (d->recu && d->ptsu && d->inv && d->mask && d->R > 0), "ured_point_losses: null part pointer");
    return 0;
}

static PointLossArgs point_args(const UredPointLossDesc* d) {
    PointLossArgs a{};
    a.B = d->B; a.N = d->N; a.S = d->S; a.U = d->U; a.NP = d->NP; a.R = d->R;
    a.x = d->x; a.out = d->out; a.knn = d->knn; a.res = d->res; a.rec = d->rec; a.recu = d->recu; a.ptsu = d->ptsu;
    a.inv = d->inv; a.mask = d->mask;
    return a;
}

int ured_point_losses_fwd(const UredPointLossDesc* d, float* ws, unsigned* counter, float* terms, void* stream) {
    ured::clear_error();
    if (int rc = point_losses_check(d)) return rc;
    URED_REQUIRE(ws && counter && terms, "ured_point_losses_fwd: null pointer");
    PointLossArgs a = point_args(d);
    a.part = ws; a.counter = counter; a.terms = terms;
    const int nb1 = (d->B * d->N + PL_CHUNK - 1) / PL_CHUNK;
    hipLaunchKernelGGL(point_losses_fwd_kernel, dim3(nb1 + d->U), dim3(LT), 0, (hipStream_t)stream, a);
    return ured::launch_status("ured_point_losses_fwd");
}

int ured_point_losses_bwd(const UredPointLossDesc* d, const float* g4, float* dres, float* drec, float* drecu,
                          void* stream) {
    ured::clear_error();
    if (int rc = point_losses_check(d)) return rc;
    URED_REQUIRE(g4 && dres && drec && (d->U == 0 || drecu), "ured_point_losses_bwd: null pointer");
    PointLossArgs a = point_args(d);
    a.g4 = g4; a.dres = dres; a.drec = drec; a.drecu = drecu;
    const long long BN = (long long)d->B * d->N;
    const int nb1 = (int)((BN + LT - 1) / LT);
    const int per = (d->NP * 3 + 4 * LT - 1) / (4 * LT);
    hipLaunchKernelGGL(point_losses_bwd_kernel, dim3(nb1 + d->U * per), dim3(LT), 0, (hipStream_t)stream, a);
    return ured::launch_status("ured_point_losses_bwd");
}

static ContrastArgs contrast_args(int n, int n_all, int C, int s_off, float scale, const float* t, const float* s,
                                  const long long* src_labels, float* inv, float* lse) {
    ContrastArgs a{};
    a.n = n; a.n_all = n_all; a.C = C; a.s_off = s_off; a.scale = scale;
    a.t = t; a.s = s; a.src_labels = src_labels; a.inv = inv; a.lse = lse;
    return a;
}

int ured_contrast_fwd(const float* t, const float* s_all, const long long* src_labels, int n, int n_all, int C,
                      int s_off, float scale, float* inv, float* lse, float* ws, unsigned* counter, float* loss,
                      void* stream) {
    ured::clear_error();
    URED_REQUIRE(n > 0 && n_all >= n && C > 0 && s_off >= 0 && s_off + n <= n_all && n_all <= CT_MAXN,
                 "ured_contrast_fwd: bad sizes (n %d, n_all %d, C %d, s_off %d)", n, n_all, C, s_off);
    URED_REQUIRE(t && s_all && src_labels && inv && lse && ws && counter && loss, "ured_contrast_fwd: null pointer");
    URED_REQUIRE(C % 4 == 0 && (((uintptr_t)t | (uintptr_t)s_all) & 15) == 0,
                 "ured_contrast_fwd: C %% 4 == 0 and 16-byte aligned rows required", C);
    ContrastArgs a = contrast_args(n, n_all, C, s_off, scale, t, s_all, src_labels, inv, lse);
    a.part = ws; a.counter = counter; a.loss = loss;
    hipLaunchKernelGGL(contrast_norms_kernel, dim3(n + n_all), dim3(LT), 0, (hipStream_t)stream, a);
    const size_t lds = (size_t)(C + n_all) * sizeof(float);
    hipLaunchKernelGGL(contrast_fwd_kernel, dim3(n), dim3(LT), lds, (hipStream_t)stream, a);
    return ured::launch_status("ured_contrast_fwd");
}

int ured_contrast_bwd(const float* t, const float* s_all, const long long* src_labels, int n, int n_all, int C,
                      int s_off, float scale, const float* inv, const float* lse, const float* g, float* dt, float* ds,
                      void* stream) {
    ured::clear_error();
    URED_REQUIRE(n > 0 && n_all >= n && C > 0 && s_off >= 0 && s_off + n <= n_all && n_all <= CT_MAXN,
                 "ured_contrast_bwd: bad sizes");
    URED_REQUIRE(t && s_all && src_labels && inv && lse && g && dt, "ured_contrast_bwd: null pointer");
    ContrastArgs a = contrast_args(n, n_all, C, s_off, scale, t, s_all, src_labels, const_cast<float*>(inv),
                                   const_cast<float*>(lse));
    a.g = g; a.dt = dt; a.ds = ds;
    const size_t lds = (size_t)(2 * C + (n > n_all ? n : n_all)) * sizeof(float);
    hipLaunchKernelGGL(contrast_bwd_kernel, dim3(n + (ds ? n : 0)), dim3(LT), lds, (hipStream_t)stream, a);
    return ured::launch_status("ured_contrast_bwd");
}

int ured_loss_assemble(int K, const float* const* terms, const float* weights, float* out, void* stream) {
    ured::clear_error();
    URED_REQUIRE(K > 0 && K <= URED_ASSEMBLE_MAX && terms && weights && out, "ured_loss_assemble: bad arguments");
    AssembleArgs a{};
    a.K = K;
    for (int i = 0; i < K; ++i) {
        URED_REQUIRE(terms[i], "ured_loss_assemble: null term %d", i);
        a.term[i] = terms[i]; a.w[i] = weights[i];
    }
    a.out = out;
    hipLaunchKernelGGL(assemble_fwd_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, a);
    return ured::launch_status("ured_loss_assemble");
}

int ured_loss_assemble_bwd(int K, const float* weights, const float* g, float* gterms, void* stream) {
    ured::clear_error();
    URED_REQUIRE(K > 0 && K <= URED_ASSEMBLE_MAX && weights && g && gterms, "ured_loss_assemble_bwd: bad arguments");
    AssembleArgs a{};
    a.K = K;
    for (int i = 0; i < K; ++i) a.w[i] = weights[i];
    a.g = g; a.gterms = gterms;
    hipLaunchKernelGGL(assemble_bwd_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, a);
    return ured::launch_status("ured_loss_assemble_bwd");
}

}  // extern "C"

URED_DBG_ACCESSOR(ured_dbg_loss)
