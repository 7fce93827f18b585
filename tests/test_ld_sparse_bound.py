"""The sparse-missing LD prefilter's bound (vcfxg_ld_fast.hip ld_sparse_prefilter), restated in
numpy and checked against the exact pair sums of computeRsqSIMD (VCFX_ld_calculator.cpp:352-393):
no pair whose exact r^2 reaches the threshold may fall outside it.  Host-only (the kernel's own
parity is tests/test_gpu_ld.py); the cases stress the bound where it is loosest -- rare variants
whose carriers are the other variant's missing samples, and blocks with the largest missing
counts the sparse groups allow (15)."""
import numpy as np
import pytest


def exact_r2(xi, xj):
    """computeRsqSIMD's r^2 over the samples valid in both (missing = -1); 0 on a zero variance"""
    ok = (xi >= 0) & (xj >= 0)
    n = int(ok.sum())
    a, b = xi[ok].astype(np.int64), xj[ok].astype(np.int64)
    sx, sy, sxy, sxx, syy = a.sum(), b.sum(), (a * b).sum(), (a * a).sum(), (b * b).sum()
    c = n * sxy - sx * sy
    vx, vy = n * sxx - sx * sx, n * syy - sy * sy
    if n < 2 or vx <= 0 or vy <= 0:
        return 0.0
    return c * c / (vx * vy)


def bound_candidates(X, rows, cols, tm):
    """the prefilter's decision for every (row, col) pair of one block (exact arithmetic)"""
    ns = X.shape[1]
    miss = X < 0
    x0 = np.where(miss, 0, X).astype(np.int64)
    m = miss.sum(1)
    N, S, Q = ns - m, x0.sum(1), (x0 * x0).sum(1)
    xs = np.where(Q != S, 2, 1)
    V = N * Q - S * S
    MI, MJ = m[rows].max(), m[cols].max()
    am_r = np.minimum(MJ * xs[rows], S[rows])
    am_c = np.minimum(MI * xs[cols], S[cols])
    AI, AJ = am_r.max(), am_c.max()
    vmin_r = V[rows] - N[rows] * np.minimum(MJ * xs[rows] ** 2, Q[rows]) - MJ * Q[rows]
    vmin_c = V[cols] - N[cols] * np.minimum(MI * xs[cols] ** 2, Q[cols]) - MI * Q[cols]
    sxy = x0[rows] @ x0[cols].T  # missing coded 0: the sum over the common samples
    c0 = N[rows][:, None] * sxy - np.outer(S[rows], S[cols])
    lhs = np.abs(c0) + MJ * sxy + (AJ * (S[rows] + am_r))[:, None] + (AI * S[cols])[None, :]
    live_r, live_c = V[rows] > 0, V[cols] > 0
    rhs2 = tm * np.outer(np.maximum(vmin_r, 0), np.maximum(vmin_c, 0)).astype(np.float64)
    cand = lhs.astype(np.float64) ** 2 >= rhs2
    return cand & live_r[:, None] & live_c[None, :]


def make_block(rng, nvar, ns, mrate, rare, adversarial):
    p = rng.uniform(0.001, 0.02, nvar) if rare else rng.uniform(0.05, 0.5, nvar)
    base = rng.binomial(2, p[:1], ns)  # one haplotype-ish source: many pairs in high LD
    X = np.empty((nvar, ns), np.int64)
    for v in range(nvar):
        X[v] = np.where(rng.random(ns) < 0.8, base, rng.binomial(2, p[v], ns))
    k = rng.poisson(mrate * ns, nvar).clip(0, 15)
    for v in range(nvar):
        if adversarial and v % 2:
            carriers = np.flatnonzero(X[v - 1] > 0)[: k[v]]  # miss exactly the other's carriers
            X[v, carriers] = -1
        else:
            X[v, rng.choice(ns, k[v], replace=False)] = -1
    return X


@pytest.mark.parametrize("rare,adversarial,mrate", [(False, False, 0.001), (True, False, 0.004),
                                                     (True, True, 0.006), (False, True, 0.006)])
def test_prefilter_keeps_every_passing_pair(rare, adversarial, mrate):
    rng = np.random.default_rng(7 + rare + 2 * adversarial)
    ns, nvar = 600, 48
    for tm in (0.2, 0.5, 0.8):
        X = make_block(rng, nvar, ns, mrate, rare, adversarial)
        rows, cols = np.arange(nvar // 2), np.arange(nvar // 2, nvar)
        cand = bound_candidates(X, rows, cols, tm)
        for a, i in enumerate(rows):
            for b, j in enumerate(cols):
                if exact_r2(X[i], X[j]) >= tm:
                    assert cand[a, b], (i, j, exact_r2(X[i], X[j]), tm)
