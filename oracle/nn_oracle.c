/*
 * nn_oracle.c — TEST INFRASTRUCTURE ONLY (the parity checker, never shipped,
 * never on the product path). Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load it.
 *
 * Plain-C restatement of the reference nearest-neighbour (chamfer) kernels:
 *   forward  : Density_aware_Chamfer_Distance/utils_v2/metrics/CD/chamfer3D/chamfer3D.cu:12-134
 *              (NmDistanceKernel: per query the min over refs of the squared
 *              distance, strict '<' scan in increasing ref index -> lowest
 *              index wins ties, :36-69 and :126)
 *   backward : chamfer3D.cu:155-174 (NmDistanceGradKernel: g = 2*grad_dist,
 *              grad_q += g*(q-r), grad_r[idx] -= g*(q-r)); the reference
 *              accumulates with atomicAdd in arbitrary order, this restatement
 *              fixes the order (own term first, then ref-side terms in
 *              ascending query index) — the same order the HIP kernel uses.
 * Distance formula contract: d = fmaf(dz,dz, fmaf(dy,dy, dx*dx)), dx = r.x - q.x
 * (compile with -ffp-contract=off so nothing else is fused).
 *
 * Parity pin: tests/test_oracle_golden.py checks this file against golden
 * vectors produced by the reference's own chamfer_python.distChamfer
 * (…/utils_v2/metrics/CD/chamfer_python.py:18-39), the oracle its unit test
 * uses (ChamferDistancePytorch/unit_test.py:14-35).
 */
#include <math.h>
#include <stddef.h>
#include <stdint.h>

static inline float sqd(const float* q, const float* r) {
    float dx = r[0] - q[0], dy = r[1] - q[1], dz = r[2] - q[2];
    return fmaf(dz, dz, fmaf(dy, dy, dx * dx));
}

/* one direction: queries q[nq], refs r[nr] */
void oracle_nn_dir(const float* q, int nq, const float* r, int nr, float* dist, int* idx) {
    for (int j = 0; j < nq; ++j) {
        if (nr <= 0) { dist[j] = 0.f; idx[j] = 0; continue; }
        float best = 0.f; int bi = 0;
        for (int k = 0; k < nr; ++k) {
            float d = sqd(q + 3 * (size_t)j, r + 3 * (size_t)k);
            if (k == 0 || d < best) { best = d; bi = k; }
        }
        dist[j] = best; idx[j] = bi;
    }
}

void oracle_nn_fwd(const float* xyz1, const float* xyz2, int b, int n, int m,
                   float* dist1, int* idx1, float* dist2, int* idx2) {
    for (int i = 0; i < b; ++i) {
        oracle_nn_dir(xyz1 + (size_t)i * n * 3, n, xyz2 + (size_t)i * m * 3, m, dist1 + (size_t)i * n, idx1 + (size_t)i * n);
        oracle_nn_dir(xyz2 + (size_t)i * m * 3, m, xyz1 + (size_t)i * n * 3, n, dist2 + (size_t)i * m, idx2 + (size_t)i * m);
    }
}

/* gradient for the query side of one direction pair (p: own points, o: other points) */
static void grad_side(const float* p, int np_, const float* o, int no,
                      const float* gd_p, const int* idx_p, const float* gd_o, const int* idx_o,
                      float* gp) {
    for (int j = 0; j < np_; ++j) {
        float ax = 0.f, ay = 0.f, az = 0.f;
        const float* pj = p + 3 * (size_t)j;
        if (no > 0 && gd_p) {
            const float* r = o + 3 * (size_t)idx_p[j];
            float g = gd_p[j] * 2.f;
            ax = g * (pj[0] - r[0]); ay = g * (pj[1] - r[1]); az = g * (pj[2] - r[2]);
        }
        if (gd_o) {
            for (int k = 0; k < no; ++k) {
                if (idx_o[k] != j) continue;
                const float* ok = o + 3 * (size_t)k;
                float g = gd_o[k] * 2.f;
                ax = ax - g * (ok[0] - pj[0]);
                ay = ay - g * (ok[1] - pj[1]);
                az = az - g * (ok[2] - pj[2]);
            }
        }
        gp[3 * (size_t)j + 0] += ax; gp[3 * (size_t)j + 1] += ay; gp[3 * (size_t)j + 2] += az;
    }
}

void oracle_nn_bwd(const float* xyz1, const float* xyz2, int b, int n, int m,
                   const float* gd1, const float* gd2, const int* idx1, const int* idx2,
                   float* g1, float* g2) {
    for (int i = 0; i < b; ++i) {
        const float* p1 = xyz1 + (size_t)i * n * 3; const float* p2 = xyz2 + (size_t)i * m * 3;
        grad_side(p1, n, p2, m, gd1 ? gd1 + (size_t)i * n : 0, idx1 + (size_t)i * n,
                  gd2 ? gd2 + (size_t)i * m : 0, idx2 + (size_t)i * m, g1 + (size_t)i * n * 3);
        grad_side(p2, m, p1, n, gd2 ? gd2 + (size_t)i * m : 0, idx2 + (size_t)i * m,
                  gd1 ? gd1 + (size_t)i * n : 0, idx1 + (size_t)i * n, g2 + (size_t)i * m * 3);
    }
}

/* ragged: segs[nseg][4] = a_off, a_len, b_off, b_len (host memory here) */
void oracle_nn_seg_fwd(const float* a, const float* b, const int* segs, int nseg, int dirs,
                       float* dist_a, int* idx_a, float* dist_b, int* idx_b) {
    for (int s = 0; s < nseg; ++s) {
        int ao = segs[4 * s], al = segs[4 * s + 1], bo = segs[4 * s + 2], bl = segs[4 * s + 3];
        if (dirs & 1) oracle_nn_dir(a + 3 * (size_t)ao, al, b + 3 * (size_t)bo, bl, dist_a + ao, idx_a + ao);
        if (dirs & 2) oracle_nn_dir(b + 3 * (size_t)bo, bl, a + 3 * (size_t)ao, al, dist_b + bo, idx_b + bo);
    }
}

void oracle_nn_seg_bwd(const float* a, const float* b, const int* segs, int nseg,
                       const float* gd_a, const float* gd_b, const int* idx_a, const int* idx_b,
                       float* ga, float* gb) {
    for (int s = 0; s < nseg; ++s) {
        int ao = segs[4 * s], al = segs[4 * s + 1], bo = segs[4 * s + 2], bl = segs[4 * s + 3];
        grad_side(a + 3 * (size_t)ao, al, b + 3 * (size_t)bo, bl, gd_a ? gd_a + ao : 0, idx_a + ao,
                  gd_b ? gd_b + bo : 0, idx_b + bo, ga + 3 * (size_t)ao);
        grad_side(b + 3 * (size_t)bo, bl, a + 3 * (size_t)ao, al, gd_b ? gd_b + bo : 0, idx_b + bo,
                  gd_a ? gd_a + ao : 0, idx_a + ao, gb + 3 * (size_t)bo);
    }
}
