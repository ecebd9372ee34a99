"""Host model of k_pose's MAD medians (gf-pl-slam_amd/csrc/k_pose.hip, wave_select /
stdv_mad_regs): the k-th smallest key is built from the top, two bits per pass, as the largest P
with #{x < P} <= k (read out early once one key is left in the window), over the unsigned bit patterns of non-negative doubles (then of floats).  This
restates the kernel's loop in numpy and checks it against the sort the reference takes the
element from (vector_stdv_mad, src/auxiliar.cpp:521-537: std::sort, then [n / 2]) on ties,
zeros, subnormals, huge values and +inf.  The GPU path itself is compared with the oracle by
the -m gpu pose tests (tests/test_gpu_parity.py)."""
import numpy as np


def wave_select(keys, k, bits):
    """The kernel's selection over unsigned keys (all-ones padding never counts): two bits per
    pass — the largest of the three thresholds P | j 2^b with #{x < T} <= k, the same choice as
    two single-bit steps since the counts are monotone in T — and the early read-out once the
    window [P, P + 2^b) between the counts lo <= k < hi holds a single key."""
    keys = np.asarray(keys, dtype=np.uint64)
    valid = keys[keys != np.uint64(~np.uint64(0))] if bits == 64 else keys[keys != np.uint64(0xFFFFFFFF)]
    n = len(valid)
    P, lo, hi = 0, 0, n
    for b in range(bits - 2, -1, -2):
        c = [int(np.count_nonzero(valid < np.uint64(P | (j << b)))) for j in (1, 2, 3)]
        if c[2] <= k:
            P, lo = P | (3 << b), c[2]
        elif c[1] <= k:
            P, lo, hi = P | (2 << b), c[1], c[2]
        elif c[0] <= k:
            P, lo, hi = P | (1 << b), c[0], c[1]
        else:
            hi = c[0]
        assert lo <= k < hi
        if hi - lo == 1 and b > 0:
            inside = valid[(valid >= np.uint64(P)) & (valid - np.uint64(P) < np.uint64(1 << b))]
            assert len(inside) == 1
            return int(inside[0])
    return P


def stdv_mad_model(r):
    n = len(r)
    if n == 0:
        return 0.0
    k64 = r.astype(np.float64).view(np.uint64)
    median = np.uint64(wave_select(k64, n // 2, 64)).view(np.float64)
    dev = np.abs((r - median).astype(np.float32))            # (double)fabsf((float)(x - median))
    k32 = dev.view(np.uint32).astype(np.uint64)
    mad = np.float64(np.uint32(wave_select(k32, n // 2, 32)).view(np.float32))
    return 1.4826 * mad


def stdv_mad_reference(r):
    n = len(r)
    if n == 0:
        return 0.0
    s = np.sort(r.astype(np.float64))
    median = s[n // 2]
    dev = np.sort(np.abs((s - median).astype(np.float32)).astype(np.float64))
    return 1.4826 * dev[n // 2]


def test_select_equals_sorted_order_statistic():
    rng = np.random.default_rng(7)
    for trial in range(300):
        n = int(rng.integers(1, 513))
        kind = trial % 5
        if kind == 0:
            x = rng.random(n) * 10.0
        elif kind == 1:                                   # heavy ties
            x = rng.integers(0, 4, n).astype(np.float64) * 0.25
        elif kind == 2:                                   # zeros, subnormals, huge
            x = rng.choice([0.0, 5e-324, 1e-310, 1.0, 1e300, np.inf], n)
        elif kind == 3:                                   # residual-like: sqrt(.) * sqrt(sigma2)
            x = np.sqrt(rng.random(n) * 4.0) * np.sqrt(1.44 ** rng.integers(0, 4, n))
        else:
            x = np.exp(rng.normal(0.0, 20.0, n))
        for k in (0, n // 2, n - 1):
            got = np.uint64(wave_select(x.view(np.uint64), k, 64)).view(np.float64)
            assert got == np.sort(x)[k]


def test_mad_model_equals_reference_mad():
    rng = np.random.default_rng(11)
    for trial in range(200):
        n = int(rng.integers(1, 513))
        x = np.sqrt(rng.random(n) * rng.choice([1e-6, 1.0, 1e4])) * 1.2
        if trial % 3 == 0:
            x[rng.integers(0, n, n // 3)] = x[0]          # duplicates of one residual
        assert stdv_mad_model(x) == stdv_mad_reference(x)


def test_mad_model_empty_is_zero():
    assert stdv_mad_model(np.zeros(0)) == 0.0


def test_select_edge_sets():
    for vals in ([0.0], [0.0, 0.0], [5.0] * 7, [0.0, 1e-300, 1e300], [1.0, 2.0], [np.inf, 1.0, np.inf]):
        x = np.asarray(vals, dtype=np.float64)
        for k in range(len(vals)):
            got = np.uint64(wave_select(x.view(np.uint64), k, 64)).view(np.float64)
            assert got == np.sort(x)[k]
