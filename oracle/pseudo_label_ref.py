"""TEST INFRASTRUCTURE ONLY (the checker, never the product path).

CPU restatement of the reference's pseudo-label selection, line by line:
  read_pickle_topk   dataset/dataset_utils.py:1043-1051 (torch.topk(cd_m, 10, largest=False))
  check_similarity   dataset/dataset_utils.py:1070-1075 (np.argpartition(dist, cl_k)[:cl_k])
  mask_label         dataset/dataset_utils.py:1077-1086
  get_labels         dataset/dataset_utils.py:1101-1143 (label part: dist < alpha, then the
                     semantic match, fallbacks; masked parts -> -1)
Rows come as arrays instead of pickle paths; semantic labels as integer ids.
"""
import numpy as np
import torch


def read_topk(cd_m_row, k=10):
    dist, indices = torch.topk(torch.tensor(np.asarray(cd_m_row, np.float64)), k, largest=False)
    return dist.tolist(), indices.tolist()


def check_similarity(label1, label2, dist_src, cl_k):
    topk_indices1 = np.argpartition(dist_src[label1], cl_k)[:cl_k]
    topk_indices2 = np.argpartition(dist_src[label2], cl_k)[:cl_k]
    return label1 in topk_indices2 and label2 in topk_indices1


def mask_label(label_list, dist_src, cl_k):
    n = len(label_list)
    bool_matrix = np.full((n, n), False)
    for i in range(n):
        for j in range(i + 1, n):
            bool_matrix[i, j] = check_similarity(label_list[i], label_list[j], dist_src, cl_k)
    return bool_matrix.sum(0)


def get_labels(part_rows, cd_m, part_sem, sources_sem, dist_src, alpha, cl_k, max_parts):
    """part_rows: per sample, the table rows of its parts (in part order)."""
    out = np.full((len(part_rows), max_parts), -1, np.int64)
    for j, rows in enumerate(part_rows):
        label_now = []
        for r in rows:
            obj_sem = int(part_sem[r])
            dist, indices = read_topk(cd_m[r])
            part_obj_sem = [int(sources_sem[x]) for x in indices]
            indices_dist = [indices[k] for k in range(len(indices)) if dist[k] < alpha]
            indices_sem = [indices_dist[i] for i in range(len(indices_dist)) if part_obj_sem[i] == obj_sem]
            if indices_sem:
                label_now.append(indices_sem[0])
            elif indices_dist:
                label_now.append(indices_dist[0])
            else:
                label_now.append(indices[0])
        label_mask = mask_label(label_now, dist_src, cl_k)
        label_now = [label_now[i] if not label_mask[i] else -1 for i in range(len(label_now))]
        out[j, :len(label_now)] = np.stack(label_now)
    return out
