/* TEST INFRASTRUCTURE ONLY — the parity checker for csrc/emd.hip, never the product path.
 *
 * Plain-C restatement of the reference auction EMD,
 *   Density_aware_Chamfer_Distance/utils_v2/metrics/EMD/emd_cuda.cu:
 *     Bid      :89-181  value = 3.0 - sqrtf(|x2 - x1|^2) - price (double-promoted, :145),
 *                       strict '>' best / better scan (:146-153), increment best - better + eps (:178)
 *     GetMax /
 *     Assign   :183-222 object -> highest increment; previous owner evicted unless last round;
 *                       last round: every bidder takes its bid
 *     CalcDist :224-233
 *   with the deterministic tie rules of emd.hip (the reference decides by racing atomics):
 *   scan ties -> lowest object index; equal increments on one object -> lowest bidder index.
 * Built with -ffp-contract=off; fmaf() spells the contract's fused distance explicitly. */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

static float sqd(float x1, float y1, float z1, float x2, float y2, float z2) {
    float dx = x2 - x1, dy = y2 - y1, dz = z2 - z1;
    return fmaf(dz, dz, fmaf(dy, dy, dx * dx));
}

static uint32_t fbits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

void oracle_emd_fwd(const float* xyz1, const float* xyz2, int b, int n, float eps, int iters,
                    float* dist, int* assignment) {
    float* price = (float*)malloc(sizeof(float) * n);
    float* inc = (float*)malloc(sizeof(float) * n);
    int* inv = (int*)malloc(sizeof(int) * n);
    int* bid = (int*)malloc(sizeof(int) * n);
    int* bidding = (int*)malloc(sizeof(int) * n);
    uint64_t* key = (uint64_t*)malloc(sizeof(uint64_t) * n);
    for (int bb = 0; bb < b; ++bb) {
        const float* p1 = xyz1 + (size_t)bb * n * 3;
        const float* p2 = xyz2 + (size_t)bb * n * 3;
        int* as = assignment + (size_t)bb * n;
        for (int i = 0; i < n; ++i) { price[i] = 0.f; inv[i] = -1; as[i] = -1; key[i] = 0; bid[i] = -1; }
        for (int it = 0; it < iters; ++it) {
            const int last = it == iters - 1;
            for (int i = 0; i < n; ++i) {
                bidding[i] = as[i] == -1;
                if (!bidding[i]) continue;
                float best = -1e9f, better = -1e9f;
                int bi = -1;
                for (int k = 0; k < n; ++k) {
                    float dd = sqd(p1[3 * i], p1[3 * i + 1], p1[3 * i + 2], p2[3 * k], p2[3 * k + 1], p2[3 * k + 2]);
                    float d = (float)((3.0 - (double)sqrtf(dd)) - (double)price[k]);
                    if (d > best) { better = best; best = d; bi = k; }
                    else if (d > better) better = d;
                }
                bid[i] = bi;
                if (bi < 0) { bidding[i] = 0; continue; }
                inc[i] = best - better + eps;
                uint64_t kk = ((uint64_t)fbits(inc[i]) << 32) | (uint64_t)(0xFFFFFFFFu - (uint32_t)i);
                if (kk > key[bi]) key[bi] = kk;
            }
            for (int i = 0; i < n; ++i) {
                if (!bidding[i]) continue;
                int j = bid[i];
                int won = last || (0xFFFFFFFFu - (uint32_t)(key[j] & 0xFFFFFFFFu)) == (uint32_t)i;
                if (!won) continue;
                if (!last && inv[j] != -1) as[inv[j]] = -1;
                inv[j] = i;
                as[i] = j;
                price[j] += inc[i];
            }
            if (!last)
                for (int i = 0; i < n; ++i) if (bidding[i]) key[bid[i]] = 0;
        }
        for (int i = 0; i < n; ++i) {
            int k = as[i] < 0 ? 0 : as[i];
            dist[(size_t)bb * n + i] = sqd(p2[3 * k], p2[3 * k + 1], p2[3 * k + 2], p1[3 * i], p1[3 * i + 1], p1[3 * i + 2]);
        }
    }
    free(price); free(inc); free(inv); free(bid); free(bidding); free(key);
}
