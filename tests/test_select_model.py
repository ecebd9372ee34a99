"""Host model of k_pose's MAD medians (gf-pl-slam_amd/csrc/k_pose.hip, wave_select /
stdv_mad_regs): the k-th smallest key is built bit by bit from the top as the largest P with
#{x < P} <= k, over the unsigned bit patterns of non-negative doubles (then of floats).  This
restates the kernel's loop in numpy and checks it against the sort the reference takes the
element from (vector_stdv_mad, src/auxiliar.cpp:521-537: std::sort, then [n / 2]) on ties,
zeros, subnormals, huge values and +inf.  The GPU path itself is compared with the oracle by
the -m gpu pose tests (tests/test_gpu_parity.py)."""
import numpy as np


def wave_select(keys, k, bits):
    """The kernel's bit-greedy selection over unsigned keys (all-ones padding never wins)."""
    P = 0
    for b in range(bits - 1, -1, -1):
        T = P | (1 << b)
        if int(np.count_nonzero(keys < np.uint64(T))) <= k:
            P = T
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
