"""Synthetic U-RED batches and source-part database (numpy, PCG64-seeded).

The reference ships no data and reads absolute /mnt/d paths plus per-part
pickles inside every step (engine/global_variables.py:13-37,
dataset/dataset_utils.py:1101-1143). Benchmarks and parity tests therefore use
this generator, which produces exactly the arrays the reference's train loop
holds after get_labels / get_source_info / get_source_points
(engine/train.py:196-210), following SURVEY.md §8(d):

  target cloud x[b]   N points uniform in the unit ball, normalize_pts'ed
                      (engine/geometry_utils.py:88-94)
  part labels         k_b parts as y-quantile slabs, labels 0..k_b-1
  semantics           per part uniform in [0, 42) (the label_to_idx range)
  source DB           per part 1024 points uniform in a random AABB; points_mat
                      A = [I3 | diag(q)], q = (p - c)/s (engine/run_preprocessing.py:118-165
                      with R = I); default_param = [c, s]
  pseudo-labels       a source index per valid part slot, -1 for padding; -1
                      resolves to the last source (Python negative indexing,
                      dataset/dataset_utils.py:800-805)
"""
import numpy as np

NUM_SEM = 42
NP_PER_PART = 1024


def normalize_pts(p):
    out = np.asarray(p, np.float32).copy()
    out -= out.mean(axis=0)
    out /= np.sqrt(np.max(np.sum(out ** 2, axis=1)))
    return out


def make_source_db(num_sources, seed=1, np_per_part=NP_PER_PART):
    rng = np.random.Generator(np.random.PCG64(seed))
    c = rng.uniform(-0.5, 0.5, size=(num_sources, 3)).astype(np.float32)
    s = rng.uniform(0.05, 0.5, size=(num_sources, 3)).astype(np.float32)
    q = rng.uniform(-1.0, 1.0, size=(num_sources, np_per_part, 3)).astype(np.float32)
    pts = (c[:, None, :] + q * s[:, None, :]).astype(np.float32)
    # A per point: rows (x,y,z), cols [t_x t_y t_z s_x s_y s_z]: p = t + diag(q) s
    A = np.zeros((num_sources, np_per_part, 3, 6), np.float32)
    for r in range(3):
        A[:, :, r, r] = 1.0
        A[:, :, r, 3 + r] = q[:, :, r]
    mats = A.reshape(num_sources, np_per_part * 3, 6)
    default_param = np.concatenate([c, s], axis=1).astype(np.float32)
    sem = rng.integers(0, NUM_SEM, size=num_sources).astype(np.int64)
    return {"src_points": pts, "src_mats": mats, "src_default_param": default_param, "src_sem": sem}


def make_source_meshes(db, seed=2, vmin=100, vmax=600):
    """Mesh side of the source DB (vertices / vertices_mat of run_preprocessing.py:852-862):
    per source V_s vertices uniform in its AABB and vertices_mat rows [I3 | diag(q)] as for the
    points. Stacked flat: vmats [sum 3V_s, 6] float32, voff int64 [NS+1] row offsets."""
    rng = np.random.Generator(np.random.PCG64(seed))
    c, s = db["src_default_param"][:, :3], db["src_default_param"][:, 3:]
    mats, verts, off = [], [], [0]
    for i in range(c.shape[0]):
        V = int(rng.integers(vmin, vmax + 1))
        q = rng.uniform(-1.0, 1.0, size=(V, 3)).astype(np.float32)
        verts.append((c[i] + q * s[i]).astype(np.float32))
        A = np.zeros((V, 3, 6), np.float32)
        for r in range(3):
            A[:, r, r] = 1.0
            A[:, r, 3 + r] = q[:, r]
        mats.append(A.reshape(3 * V, 6))
        off.append(off[-1] + 3 * V)
    return {"vertices": verts, "vmats": np.concatenate(mats), "voff": np.asarray(off, np.int64)}


def make_batch(batch_size, num_points, num_sources, max_parts=16, parts=4, seed=0, invalid_frac=0.0):
    """One synthetic batch. `parts` is an int (k_b for every sample) or a list per sample."""
    rng = np.random.Generator(np.random.PCG64(seed))
    B, N = batch_size, num_points
    ks = [parts] * B if np.isscalar(parts) else list(parts)
    assert len(ks) == B and all(1 <= k <= max_parts for k in ks) and all(k <= N for k in ks)
    x = np.zeros((B, N, 3), np.float32)
    labels = np.zeros((B, N), np.int64)
    tgt_sem = np.zeros((B, N), np.int64)
    src_labels = np.full((B, max_parts), -1, np.int64)
    for b in range(B):
        d = rng.standard_normal((N, 3))
        d /= np.linalg.norm(d, axis=1, keepdims=True)
        r = rng.uniform(0, 1, size=(N, 1)) ** (1.0 / 3.0)
        x[b] = normalize_pts(d * r)
        rank = np.empty(N, np.int64)
        rank[np.argsort(x[b, :, 1], kind="stable")] = np.arange(N)
        labels[b] = (rank * ks[b]) // N
        psem = rng.integers(0, NUM_SEM, size=ks[b])
        tgt_sem[b] = psem[labels[b]]
        src = rng.integers(0, num_sources, size=ks[b])
        if invalid_frac > 0:
            src[rng.uniform(size=ks[b]) < invalid_frac] = -1
        src_labels[b, :ks[b]] = src
    src_index = np.where(src_labels < 0, num_sources - 1, src_labels)
    return {"x": x, "labels": labels, "tgt_sem": tgt_sem, "src_labels": src_labels,
            "src_index": src_index, "parts": np.asarray(ks, np.int64)}


def make_targets_from_sources(src_points, src_sem, num_targets, num_points, parts=4, seed=0):
    """Targets assembled from source parts (the PartNet situation the pseudo-labels assume: a
    target part resembles some source part): target j takes k_j distinct random sources, part i
    is num_points / k_j points drawn (with replacement) from source s_i's cloud at its own place,
    with that source's semantics; the cloud is shuffled and normalize_pts'ed. The nearest source of
    each part by calc_dcd is then its own source, so a batch encodes as many distinct source parts
    as make_batch's uniformly drawn labels do. Returns make_batch's fields plus "src_true"."""
    rng = np.random.Generator(np.random.PCG64(seed))
    src_points = np.asarray(src_points, np.float32)
    src_sem = np.asarray(src_sem, np.int64)
    NS, NPP = src_points.shape[:2]
    T, N = num_targets, num_points
    ks = [parts] * T if np.isscalar(parts) else list(parts)
    x = np.zeros((T, N, 3), np.float32)
    labels = np.zeros((T, N), np.int64)
    tgt_sem = np.zeros((T, N), np.int64)
    src_true = np.full((T, max(ks)), -1, np.int64)
    for j in range(T):
        k = ks[j]
        srcs = rng.choice(NS, size=k, replace=False)
        sizes = np.full(k, N // k)
        sizes[:N % k] += 1
        lab = np.repeat(np.arange(k), sizes)
        pts = np.concatenate([src_points[s][rng.integers(0, NPP, size=n)] for s, n in zip(srcs, sizes)])
        order = rng.permutation(N)
        x[j] = normalize_pts(pts[order])
        labels[j] = lab[order]
        tgt_sem[j] = src_sem[srcs][labels[j]]
        src_true[j, :k] = srcs
    return {"x": x, "labels": labels, "tgt_sem": tgt_sem, "parts": np.asarray(ks, np.int64), "src_true": src_true}

