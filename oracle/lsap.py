"""CPU restatement of scipy.optimize.linear_sum_assignment (scipy 1.15.3,
scipy/optimize/_lsap.py -> rectangular_lsap.cpp: Crouse's shortest augmenting path, 2016) —
TEST INFRASTRUCTURE ONLY (the checker of the HIP matcher kernel, never the product path).

The reference calls it from the HF Mask2Former Hungarian matcher
(transformers 5.15 modeling_mask2former.py:474, ``linear_sum_assignment(cost_matrix.cpu())``),
once per image and per decoder output in every training step.  Pinned against
scipy itself on random and tie-heavy integer cost matrices (tests/test_oracle_lsap.py): the
discrete tie-breaking (reverse-ordered ``remaining`` list, swap-with-last removal, "prefer a free
column on equal cost") decides which optimum is returned, so it is restated exactly.
"""
import math

import numpy as np


def _augmenting_path(nc, cost, u, v, path, row4col, spc, i, SR, SC, remaining):
    min_val = 0.0
    num_remaining = nc
    for it in range(nc):
        remaining[it] = nc - it - 1
    SR[:] = False
    SC[:] = False
    spc[:] = math.inf
    sink = -1
    while sink == -1:
        index = -1
        lowest = math.inf
        SR[i] = True
        for it in range(num_remaining):
            j = remaining[it]
            r = min_val + cost[i, j] - u[i] - v[j]
            if r < spc[j]:
                path[j] = i
                spc[j] = r
            if spc[j] < lowest or (spc[j] == lowest and row4col[j] == -1):
                lowest = spc[j]
                index = it
        min_val = lowest
        if min_val == math.inf:
            return -1, min_val
        j = remaining[index]
        if row4col[j] == -1:
            sink = j
        else:
            i = row4col[j]
        SC[j] = True
        num_remaining -= 1
        remaining[index] = remaining[num_remaining]
    return sink, min_val


def linear_sum_assignment(cost):
    """Same contract as scipy's (minimisation): returns (row_ind, col_ind) int64 arrays."""
    cost = np.asarray(cost, dtype=np.float64)
    nr, nc = cost.shape
    if nr == 0 or nc == 0:
        return np.zeros(0, np.int64), np.zeros(0, np.int64)
    transpose = nc < nr
    if transpose:
        cost = cost.T.copy()
        nr, nc = nc, nr
    if np.isnan(cost).any() or (cost == -np.inf).any():
        raise ValueError("matrix contains invalid numeric entries")
    u = np.zeros(nr)
    v = np.zeros(nc)
    spc = np.empty(nc)
    path = np.full(nc, -1, np.int64)
    col4row = np.full(nr, -1, np.int64)
    row4col = np.full(nc, -1, np.int64)
    SR = np.zeros(nr, bool)
    SC = np.zeros(nc, bool)
    remaining = np.zeros(nc, np.int64)
    for cur in range(nr):
        sink, min_val = _augmenting_path(nc, cost, u, v, path, row4col, spc, cur, SR, SC, remaining)
        if sink < 0:
            raise ValueError("cost matrix is infeasible")
        u[cur] += min_val
        for i in range(nr):
            if SR[i] and i != cur:
                u[i] += min_val - spc[col4row[i]]
        for j in range(nc):
            if SC[j]:
                v[j] -= min_val - spc[j]
        j = sink
        while True:
            i = path[j]
            row4col[j] = i
            col4row[i], j = j, col4row[i]
            if i == cur:
                break
    if transpose:
        order = np.argsort(col4row, kind="stable")
        return col4row[order].astype(np.int64), order.astype(np.int64)
    return np.arange(nr, dtype=np.int64), col4row.astype(np.int64)
